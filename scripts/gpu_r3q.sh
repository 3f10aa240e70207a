#!/bin/bash
# Round 3q: fused decode layer at TP=2 (gloo on one GPU) and the decode / graph regressions.
set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 500 python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_e2e.py -m gpu -k "decode or graph or generation" > gpurun_out/r3q_tests.log 2>&1 || { tail -60 gpurun_out/r3q_tests.log; exit 1; }
grep -E "PASSED|FAILED" gpurun_out/r3q_tests.log | cut -c1-120; tail -1 gpurun_out/r3q_tests.log
