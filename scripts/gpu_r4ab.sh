#!/bin/bash
# Round 4ab: SP MLP pipeline with planned (uneven) pieces: piece-cost bench on one GPU.
set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u scripts/sp_overlap_bench.py --json gpurun_out/r4ab_sp_pieces.json > gpurun_out/r4ab_sp_pieces.txt 2>&1 || { tail -30 gpurun_out/r4ab_sp_pieces.txt; exit 1; }
cat gpurun_out/r4ab_sp_pieces.txt
