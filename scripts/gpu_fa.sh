#!/bin/bash
# FlashAttention numerics + backward occupancy variants at the Llama-2-7B shape.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests/test_kernels_gpu.py -q -x -k "flash" > gpurun_out/fa_tests.log 2>&1 || { echo tests failed; tail -40 gpurun_out/fa_tests.log; exit 1; }
tail -2 gpurun_out/fa_tests.log
for occ in ${OCCS:-11}; do
  echo "occ $occ"
  EMA_FA_BWD_OCC=$occ timeout -k 10 120 python scripts/fa_bench.py > gpurun_out/fa_bench_$occ.log 2>&1 || { echo bench failed; tail -20 gpurun_out/fa_bench_$occ.log; exit 1; }
  tail -2 gpurun_out/fa_bench_$occ.log
done
