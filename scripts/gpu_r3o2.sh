#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 120 python -u scripts/decode_debug.py 2>&1 | grep -v amdgpu.ids
