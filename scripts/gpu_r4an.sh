#!/bin/bash
# Round 4an: kernel profile of the 7B training step on the final tree.
set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r4an -o prof -- \
  python3 -u bench.py --steps 2 --warmup 1 > gpurun_out/r4an_bench.log 2>&1 || { tail -30 gpurun_out/r4an_bench.log; exit 1; }
tail -1 gpurun_out/r4an_bench.log | cut -c1-300
find gpurun_out/r4an -name "*kernel_stats.csv" | head -3
