#!/bin/bash
# Ring / context-parallel kernel tests on the GPU.
set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -v --timeout 120 \
  --timeout-method thread -p no:cacheprovider -k "ring" > gpurun_out/r3w.log 2>&1
rc=$?; tail -15 gpurun_out/r3w.log; exit $rc
