#!/bin/bash
# Persistent dK/dV kernel: FA GPU tests (persistent and one-item-per-block grids), timing A/B.
set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
for gmode in p full; do
  EMA_FA_DKDV_GRID=$gmode timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -q -k "flash or deterministic" \
    --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/fa_tests_$gmode.log 2>&1
  rc=$?; echo "fa tests grid=$gmode rc=$rc"; tail -2 gpurun_out/fa_tests_$gmode.log
  [ $rc -eq 0 ] || { grep -E "Error|assert|FAILED" gpurun_out/fa_tests_$gmode.log | head -20; exit $rc; }
done
for gmode in p full; do
  EMA_FA_DKDV_GRID=$gmode timeout -k 10 200 python scripts/fa_bench2.py 16,1024,32,32,128 4,4096,32,32,128 8,2048,32,2,64 2,4096,8,1,128 4,4096,4,4,128 > gpurun_out/fa_bench_$gmode.log 2>&1 || { tail -20 gpurun_out/fa_bench_$gmode.log; exit 1; }
  echo "grid $gmode"; grep shape gpurun_out/fa_bench_$gmode.log
done
