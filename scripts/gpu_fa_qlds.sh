#!/bin/bash
# FA forward Q via LDS-DMA (default) vs per-lane loads: tests + timing.
set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -q -k "flash or rope or deterministic" \
  --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/fa_tests.log 2>&1
rc=$?; echo "fa tests rc=$rc"; tail -2 gpurun_out/fa_tests.log
[ $rc -eq 0 ] || { grep -E "Error|assert|FAILED" gpurun_out/fa_tests.log | head -20; exit $rc; }
for q in 1 0; do
  EMA_FA_QLDS=$q timeout -k 10 200 python scripts/fa_bench2.py 16,1024,32,32,128 4,4096,32,32,128 8,2048,32,2,64 2,4096,8,1,128 4,4096,4,4,128 > gpurun_out/fa_bench_q$q.log 2>&1 || { tail -20 gpurun_out/fa_bench_q$q.log; exit 1; }
  echo "qlds $q"; grep shape gpurun_out/fa_bench_q$q.log
done
