#!/bin/bash
# Round-end check of the final tree: full GPU tests, smoke, default bench.
set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/gputests.log 2>&1
rc=$?; echo "gpu tests rc=$rc"; tail -1 gpurun_out/gputests.log
[ $rc -eq 0 ] || { grep -E "Error|assert|FAILED" gpurun_out/gputests.log | head -30; exit $rc; }
timeout -k 10 300 python __graft_entry__.py smoke > gpurun_out/smoke.log 2>&1 || { tail -20 gpurun_out/smoke.log; exit 1; }
grep smoke gpurun_out/smoke.log
timeout -k 10 600 python bench.py > gpurun_out/b7_final.log 2>&1 || { tail -20 gpurun_out/b7_final.log; exit 1; }
tail -1 gpurun_out/b7_final.log | cut -c1-700
