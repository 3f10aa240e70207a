#!/bin/bash
# FA forward variants: numerics (GPU tests) then timing per variant.
set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -x -q -k flash --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/fa_tests.log 2>&1
rc=$?; tail -3 gpurun_out/fa_tests.log; [ $rc -eq 0 ] || { tail -40 gpurun_out/fa_tests.log; exit $rc; }
for v in 1 4 8; do
  EMA_FA_FWD=$v timeout -k 10 200 python scripts/fa_bench2.py > gpurun_out/fa_bench_v$v.log 2>&1 || { tail -20 gpurun_out/fa_bench_v$v.log; exit 1; }
  cat gpurun_out/fa_bench_v$v.log | grep variant
done
