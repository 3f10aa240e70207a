#!/bin/bash
# Round 4am: one-shot xGMI all-reduce + all-gather tests (ranks sharing the GPU).
set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest -x -v -s --timeout 280 --timeout-method thread -p no:cacheprovider \
  tests/test_xgmi_gpu.py tests/test_gpu_e2e.py -k "xgmi" -m gpu > gpurun_out/r4am_xgmi.log 2>&1 || { tail -60 gpurun_out/r4am_xgmi.log; exit 1; }
grep -E "xgmi one-shot|PASSED|passed" gpurun_out/r4am_xgmi.log
