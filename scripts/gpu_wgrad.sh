#!/bin/bash
# wgrad kernel: numerics tests, isolated TF/s vs hipBLASLt, ablations.
set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -q -k "wgrad" --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/wg_t.log 2>&1
rc=$?; tail -3 gpurun_out/wg_t.log; [ $rc -eq 0 ] || { grep -E "Error|assert|error" gpurun_out/wg_t.log | head -20; exit $rc; }
timeout -k 10 300 python -u scripts/wgrad_bench.py gpurun_out/wg_bench.json 2>&1 | grep -v amdgpu.ids && \
timeout -k 10 200 python -u scripts/wgrad_bench.py --ablation 2>&1 | grep -v amdgpu.ids
