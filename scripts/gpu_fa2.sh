#!/bin/bash
# FA numerics (GPU tests, new kernels are the defaults) then old-vs-new timing.
set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -x -q -k flash --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/fa_tests.log 2>&1
rc=$?; tail -3 gpurun_out/fa_tests.log; [ $rc -eq 0 ] || { grep -E "Error|assert|mismatch|max" gpurun_out/fa_tests.log | head -30; exit $rc; }
EMA_FA_FWD=1 EMA_FA_DKDV=1 EMA_FA_DQ=1 timeout -k 10 200 python scripts/fa_bench2.py > gpurun_out/fa_bench_old.log 2>&1 || { tail -20 gpurun_out/fa_bench_old.log; exit 1; }
grep variant gpurun_out/fa_bench_old.log
EMA_FA_DKDV=1 timeout -k 10 200 python scripts/fa_bench2.py > gpurun_out/fa_bench_dq.log 2>&1 || { tail -20 gpurun_out/fa_bench_dq.log; exit 1; }
grep variant gpurun_out/fa_bench_dq.log
timeout -k 10 200 python scripts/fa_bench2.py > gpurun_out/fa_bench_new.log 2>&1 || { tail -20 gpurun_out/fa_bench_new.log; exit 1; }
grep variant gpurun_out/fa_bench_new.log
