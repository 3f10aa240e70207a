#!/bin/bash
# Skinny GEMM: tests, micro bench, serving A/B.
set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_gpu_e2e.py -m gpu -x -q -k "skinny or kv_cached or decode" \
  --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/sk_tests.log 2>&1
rc=$?; echo "skinny tests rc=$rc"; tail -2 gpurun_out/sk_tests.log
[ $rc -eq 0 ] || { grep -E "Error|assert|FAILED" gpurun_out/sk_tests.log | head -20; exit $rc; }
timeout -k 10 200 python scripts/skinny_bench.py > gpurun_out/skinny_bench.log 2>&1 || { tail -20 gpurun_out/skinny_bench.log; exit 1; }
grep "M=" gpurun_out/skinny_bench.log
for sk in 1 0; do
  EMA_SKINNY_GEMM=$sk timeout -k 10 600 python scripts/serve_bench.py --batches 1,8,16 > gpurun_out/serve_$sk.log 2>&1 || { tail -20 gpurun_out/serve_$sk.log; exit 1; }
  echo "skinny=$sk"; grep batch gpurun_out/serve_$sk.log
done
