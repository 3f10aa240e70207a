#!/bin/bash
# Full GPU test suite + smoke + serving eager/graph.
set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/gputests.log 2>&1
rc=$?; echo "gpu tests rc=$rc"; tail -2 gpurun_out/gputests.log
[ $rc -eq 0 ] || { grep -E "Error|assert|FAILED" gpurun_out/gputests.log | head -30; exit $rc; }
timeout -k 10 300 python __graft_entry__.py smoke > gpurun_out/smoke.log 2>&1 || { tail -20 gpurun_out/smoke.log; exit 1; }
tail -2 gpurun_out/smoke.log
for g in "" "--graph"; do
  timeout -k 10 300 python -u scripts/serve_bench.py $g > gpurun_out/serve_r2f$g.log 2>&1 || { tail -20 gpurun_out/serve_r2f$g.log; exit 1; }
  grep '^{' gpurun_out/serve_r2f$g.log
done
