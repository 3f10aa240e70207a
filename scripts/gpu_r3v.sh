#!/bin/bash
# Round 3v: ring attention (context parallelism) with the HIP FA kernels.
set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread -p no:cacheprovider \
  tests/test_kernels_gpu.py -m gpu -k "ring_attention" > gpurun_out/r3v_tests.log 2>&1 || { tail -40 gpurun_out/r3v_tests.log; exit 1; }
grep -E "PASSED|FAILED" gpurun_out/r3v_tests.log | cut -c1-120; tail -1 gpurun_out/r3v_tests.log
