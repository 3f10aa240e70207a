#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
EMA_FA_STAMPS=1 timeout -k 10 120 python scripts/fa_bench.py > gpurun_out/fa_stamps.log 2>&1 || { echo failed; tail -20 gpurun_out/fa_stamps.log; exit 1; }
grep stamps gpurun_out/fa_stamps.log | tail -2
