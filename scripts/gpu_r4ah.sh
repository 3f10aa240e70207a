#!/bin/bash
# Round 4ah: kernel profile of graphed decode at 16 and 32 sequences.
set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1
for b in 16 32; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r4ah_b$b -o prof -- \
    python3 -u scripts/serve_bench.py --batches $b --graph --gen 64 > gpurun_out/r4ah_b$b.log 2>&1 \
    || { tail -30 gpurun_out/r4ah_b$b.log; exit 1; }
  grep '^{"batch' gpurun_out/r4ah_b$b.log
done
find gpurun_out/r4ah_b16 gpurun_out/r4ah_b32 -name "*kernel_stats.csv" | head
