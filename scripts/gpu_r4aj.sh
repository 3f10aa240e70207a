#!/bin/bash
# Round 4aj: 17-32-row decode with the norm split out of the projections:
# skinny / decode tests, skinny bench at 16-32 rows, graphed serving 1-32.
set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider \
  tests/test_kernels_gpu.py tests/test_gpu_e2e.py -m gpu -k "skinny or decode or graph or greedy" \
  > gpurun_out/r4aj_tests.log 2>&1 || { tail -40 gpurun_out/r4aj_tests.log; exit 1; }
tail -1 gpurun_out/r4aj_tests.log
timeout -k 10 240 python -u scripts/skinny_mb_bench.py > gpurun_out/r4aj_skinny_mb.txt 2>&1 || { tail -30 gpurun_out/r4aj_skinny_mb.txt; exit 1; }
grep "M=" gpurun_out/r4aj_skinny_mb.txt
timeout -k 10 400 python -u scripts/serve_bench.py --batches 1,8,16,24,32 --graph > gpurun_out/r4aj_serve_graph.log 2>&1 || { tail -30 gpurun_out/r4aj_serve_graph.log; exit 1; }
grep '^{"batch' gpurun_out/r4aj_serve_graph.log
