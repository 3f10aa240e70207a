#!/bin/bash
# Round 3s: persistent skinny ring depth 16 vs 8 (EMA_SKINNY_PU): tests, kernel bench, graph decode.
set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
EMA_SKINNY_PU=16 timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider \
  tests/test_kernels_gpu.py -m gpu -k "skinny" > gpurun_out/r3s_tests.log 2>&1 || { tail -40 gpurun_out/r3s_tests.log; exit 1; }
tail -1 gpurun_out/r3s_tests.log
for pu in 16 8; do
  EMA_SKINNY_PU=$pu timeout -k 10 200 python -u scripts/skinny_bench.py > gpurun_out/r3s_skinny_pu$pu.log 2>&1 || { tail -20 gpurun_out/r3s_skinny_pu$pu.log; exit 1; }
  echo "pu=$pu"; grep -E "^M=(1|8) N=(12288|4096|22016|32000) K=4096" gpurun_out/r3s_skinny_pu$pu.log
done
for r in 1 2; do for pu in 16 8; do
  EMA_SKINNY_PU=$pu timeout -k 10 300 python -u scripts/serve_bench.py --batches 1,8 --graph > gpurun_out/r3s_serve_pu$pu.log 2>&1 || { tail -30 gpurun_out/r3s_serve_pu$pu.log; exit 1; }
  echo "pu=$pu round $r"; grep '^{"batch' gpurun_out/r3s_serve_pu$pu.log | cut -c1-140
done; done
