#!/bin/bash
# FA numerics, timing (new defaults), then PMC summary at the 7B shape.
set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -x -q -k flash --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/fa_tests.log 2>&1
rc=$?; tail -2 gpurun_out/fa_tests.log; [ $rc -eq 0 ] || { grep -E "Error|assert|mismatch|max" gpurun_out/fa_tests.log | head -30; exit $rc; }
timeout -k 10 200 python scripts/fa_bench2.py > gpurun_out/fa_bench_new.log 2>&1 || { tail -20 gpurun_out/fa_bench_new.log; exit 1; }
grep variant gpurun_out/fa_bench_new.log
bash scripts/gpu_pmc_fa2.sh 2>&1 | tail -6
