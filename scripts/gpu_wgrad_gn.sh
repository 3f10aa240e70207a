#!/bin/bash
# wgrad tile-grouping sweep on the 7B shapes (isolated).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
for GN in 8 4 16 2 -4 -8; do
  echo "GN=$GN"; EMA_WGRAD_GN=$GN timeout -k 10 200 python -u scripts/wgrad_bench.py 2>&1 | grep -E "^(qkv|dense|fc1|fc2|lm_head)" | sed 's/, "hipblaslt_default_tflops".*//' || exit 1
done
