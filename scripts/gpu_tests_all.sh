#!/bin/bash
# Full GPU test suite + smoke.
set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread \
  -p no:cacheprovider > gpurun_out/gputests.log 2>&1
rc=$?; echo "gpu tests rc=$rc"; tail -2 gpurun_out/gputests.log
[ $rc -eq 0 ] || { grep -E "Error|assert|FAILED" gpurun_out/gputests.log | head -20; exit $rc; }
timeout -k 10 300 python __graft_entry__.py smoke > gpurun_out/smoke.log 2>&1 || { tail -30 gpurun_out/smoke.log; exit 1; }
grep smoke gpurun_out/smoke.log
