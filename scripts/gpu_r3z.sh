#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 240 python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -v --timeout 120 \
  --timeout-method thread -p no:cacheprovider -k "rope or ring or decode_mlp" > gpurun_out/r3z.log 2>&1
rc=$?; tail -12 gpurun_out/r3z.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u scripts/cp_pair_bench.py > gpurun_out/r3z_cp_bench.log 2>&1
rc=$?; cat gpurun_out/r3z_cp_bench.log | tail -5; exit $rc
