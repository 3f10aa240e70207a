#!/bin/bash
# A/B: 8-wave (one block per CU) vs 4-wave (two blocks per CU) FA forward / dQ blocks.
set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
EMA_FA_WAVES=4 timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -q -k "flash or rope or deterministic" \
  --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/fa_tests_w4.log 2>&1
rc=$?; echo "fa tests w4 rc=$rc"; tail -2 gpurun_out/fa_tests_w4.log
[ $rc -eq 0 ] || { grep -E "Error|assert|FAILED" gpurun_out/fa_tests_w4.log | head -20; exit $rc; }
for w in 8 4; do
  EMA_FA_WAVES=$w timeout -k 10 200 python scripts/fa_bench2.py 16,1024,32,32,128 4,4096,32,32,128 8,2048,32,2,64 2,4096,8,1,128 4,4096,4,4,128 > gpurun_out/fa_bench_w$w.log 2>&1 || { tail -20 gpurun_out/fa_bench_w$w.log; exit 1; }
  echo "waves $w"; grep shape gpurun_out/fa_bench_w$w.log
done
