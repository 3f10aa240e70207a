#!/bin/bash
# Round 4ad: the other BASELINE proxies on the round-4 tree (70B TP8 full recompute / memory-budget, Falcon-40B TP4 PP2).
set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
for px in llama70b-tp8 llama70b-tp8-budget falcon40b-tp4-pp2; do
timeout -k 10 600 python -u bench.py --proxy $px --steps 3 --warmup 1 > gpurun_out/r4ad_px_$px.log 2>&1 || { tail -20 gpurun_out/r4ad_px_$px.log; exit 1; }
tail -1 gpurun_out/r4ad_px_$px.log | cut -c1-400
done
