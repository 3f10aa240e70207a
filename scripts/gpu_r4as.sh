#!/bin/bash
# Round 4as: persistent skinny ring 16 deep for two un-normed row blocks (b > 16 decode).
set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider \
  tests/test_kernels_gpu.py -m gpu -k "skinny" > gpurun_out/r4as_tests.log 2>&1 || { tail -40 gpurun_out/r4as_tests.log; exit 1; }
tail -1 gpurun_out/r4as_tests.log
timeout -k 10 240 python -u scripts/skinny_mb_bench.py --rows 24,32 > gpurun_out/r4as_skinny.txt 2>&1 || { tail -30 gpurun_out/r4as_skinny.txt; exit 1; }
grep "M=" gpurun_out/r4as_skinny.txt
timeout -k 10 400 python -u scripts/serve_bench.py --batches 24,32 --graph > gpurun_out/r4as_serve_graph.log 2>&1 || { tail -30 gpurun_out/r4as_serve_graph.log; exit 1; }
grep '^{"batch' gpurun_out/r4as_serve_graph.log
