#!/bin/bash
# FA kernel tests + FA timing on the training shapes.
set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -q -k "flash or attention or determin" --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/fa_t.log 2>&1
rc=$?; tail -3 gpurun_out/fa_t.log; [ $rc -eq 0 ] || { grep -E "Error|assert|error|mismatch" gpurun_out/fa_t.log | head -20; exit $rc; }
timeout -k 10 200 python -u scripts/fa_bench2.py 16,1024,32,32,128 4,4096,32,32,128 2,4096,8,1,128 2,2048,32,2,128 2>&1 | grep -v amdgpu.ids
