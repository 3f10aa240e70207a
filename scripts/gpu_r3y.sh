#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 120 python -u scripts/decode_mlp_bench.py 2>&1 | tee gpurun_out/r3y.log
