#!/bin/bash
# Round 4al: per-block skinny ring 16 deep for one row block: fc2 bench, serving.
set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 240 python -u scripts/skinny_mb_bench.py --rows 1,8,16 > gpurun_out/r4al_skinny.txt 2>&1 || { tail -30 gpurun_out/r4al_skinny.txt; exit 1; }
grep "M=" gpurun_out/r4al_skinny.txt
timeout -k 10 400 python -u scripts/serve_bench.py --batches 1,8,16 --graph > gpurun_out/r4al_serve_graph.log 2>&1 || { tail -30 gpurun_out/r4al_serve_graph.log; exit 1; }
grep '^{"batch' gpurun_out/r4al_serve_graph.log
