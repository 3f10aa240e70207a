#!/bin/bash
# Round 4ai: fused skinny GEMMs at 16 / 24 / 32 rows vs hipBLASLt.
set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 240 python -u scripts/skinny_mb_bench.py > gpurun_out/r4ai_skinny_mb.txt 2>&1 || { tail -30 gpurun_out/r4ai_skinny_mb.txt; exit 1; }
cat gpurun_out/r4ai_skinny_mb.txt
