#!/bin/bash
# Round 4ag: one-shot xGMI all-reduce (2 / 4 ranks sharing the GPU), then the
# 17-32-row skinny kernels: tests, serving at 1-32 sequences.
set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest -x -v -s --timeout 280 --timeout-method thread -p no:cacheprovider \
  tests/test_xgmi_gpu.py tests/test_gpu_e2e.py -k "xgmi" -m gpu > gpurun_out/r4ag_xgmi.log 2>&1 || { tail -60 gpurun_out/r4ag_xgmi.log; exit 1; }
tail -3 gpurun_out/r4ag_xgmi.log
bash scripts/gpu_r4af.sh
