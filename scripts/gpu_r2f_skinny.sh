#!/bin/bash
# 8-wave skinny GEMM A/B (EMA_SKINNY_WAVES=4 vs 8), serving eager/graph, decode-step profile.
set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_gpu_e2e.py -m gpu -x -q -k "skinny or decode or graph" \
  --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/sk_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/sk_tests.log
[ $rc -eq 0 ] || { grep -E "Error|assert|FAILED" gpurun_out/sk_tests.log | head -20; exit $rc; }
for wv in 4 8; do
  EMA_SKINNY_WAVES=$wv timeout -k 10 200 python scripts/skinny_bench.py > gpurun_out/skinny_w$wv.log 2>&1 || { tail -20 gpurun_out/skinny_w$wv.log; exit 1; }
  echo "waves=$wv"; grep "M=" gpurun_out/skinny_w$wv.log
done
for g in "" "--graph"; do
  timeout -k 10 300 python -u scripts/serve_bench.py $g > gpurun_out/serve_r2f$g.log 2>&1 || { tail -20 gpurun_out/serve_r2f$g.log; exit 1; }
  grep '^{' gpurun_out/serve_r2f$g.log
done
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/profdec -o s -- python scripts/serve_bench.py --batches 8 --gen 32 --graph > gpurun_out/profdec.log 2>&1; echo "prof rc=$?"
