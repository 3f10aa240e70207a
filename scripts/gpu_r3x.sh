#!/bin/bash
# Fused decode MLP kernel: tests, then graph-decode serving A/B (fused vs three launches).
set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 240 python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -v --timeout 120 \
  --timeout-method thread -p no:cacheprovider -k "decode_mlp or skinny" > gpurun_out/r3x_tests.log 2>&1
rc=$?; tail -14 gpurun_out/r3x_tests.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  for f in 1 0; do
    echo "fused=$f round $r"
    EMA_DECODE_MLP=$f timeout -k 10 200 python -u scripts/serve_bench.py --batches 1,8 --graph \
      > gpurun_out/r3x_serve_${f}_${r}.log 2>&1 || { tail -20 gpurun_out/r3x_serve_${f}_${r}.log; exit 1; }
    grep decode_tokens gpurun_out/r3x_serve_${f}_${r}.log
  done
done
