#!/bin/bash
# Same-box A/B of the GLU half-block last round (EMA_SKINNY_HALVES=1 default vs 0): graph decode.
set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 200 python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -q --timeout 120 \
  --timeout-method thread -p no:cacheprovider -k "skinny_fused_glu or decode_mlp" > gpurun_out/r3ab_tests.log 2>&1
rc=$?; tail -1 gpurun_out/r3ab_tests.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  for h in 1 0; do
    echo "halves=$h round $r"
    EMA_SKINNY_HALVES=$h timeout -k 10 200 python -u scripts/serve_bench.py --batches 1,8 --graph \
      > gpurun_out/r3ab_${h}_${r}.log 2>&1 || { tail -20 gpurun_out/r3ab_${h}_${r}.log; exit 1; }
    grep decode_tokens gpurun_out/r3ab_${h}_${r}.log
  done
done
