#!/bin/bash
# Selected GPU tests (pattern in $K), verbose, time-limited.
set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v -s --timeout 200 --timeout-method thread -p no:cacheprovider -k "$1" > gpurun_out/quick.log 2>&1
rc=$?; grep -E "PASSED|FAILED|Error|passed|failed" gpurun_out/quick.log | tail -25; exit $rc
