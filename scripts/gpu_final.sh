#!/bin/bash
# Round-end check: full GPU suite, smoke, 1-GPU headline bench.
set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread \
  -p no:cacheprovider > gpurun_out/final_gputests.log 2>&1
rc=$?; echo "gpu tests rc=$rc"; tail -2 gpurun_out/final_gputests.log
[ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" gpurun_out/final_gputests.log | head -20; exit $rc; }
timeout -k 10 300 python __graft_entry__.py smoke > gpurun_out/final_smoke.log 2>&1 || { tail -30 gpurun_out/final_smoke.log; exit 1; }
grep smoke gpurun_out/final_smoke.log
timeout -k 10 400 python -u bench.py --steps 8 --warmup 2 > gpurun_out/final_bench.log 2>&1 || { tail -20 gpurun_out/final_bench.log; exit 1; }
tail -1 gpurun_out/final_bench.log
