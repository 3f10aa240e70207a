#!/bin/bash
# Round 3k: FA forward per-workgroup stamps; batch-32 decode after moving
# small-M inference MLPs off the NT kernel.
set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 200 python -u scripts/fa_stamps.py --json gpurun_out/r3k_fa_stamps.json > gpurun_out/r3k_fa_stamps.log 2>&1 || { tail -20 gpurun_out/r3k_fa_stamps.log; exit 1; }
grep '^{' gpurun_out/r3k_fa_stamps.log
timeout -k 10 300 python -u scripts/serve_bench.py --batches 32 --graph > gpurun_out/r3k_serve_b32.log 2>&1 || { tail -30 gpurun_out/r3k_serve_b32.log; exit 1; }
grep '^{"batch' gpurun_out/r3k_serve_b32.log
