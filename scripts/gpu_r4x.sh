#!/bin/bash
# Round 4x: GPU end-to-end tests after the PP-aware graphed decode forward.
set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_e2e.py -m gpu > gpurun_out/r4x_e2e.log 2>&1 || { tail -40 gpurun_out/r4x_e2e.log; exit 1; }
tail -1 gpurun_out/r4x_e2e.log
