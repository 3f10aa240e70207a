#!/bin/bash
# Round 4at: full GPU suite, smoke, 7B bench (+ kernel profile), serving.
set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 1000 python -u -m pytest -x -q --timeout 280 --timeout-method thread -p no:cacheprovider \
  tests -m gpu > gpurun_out/r4at_tests.log 2>&1 || { tail -40 gpurun_out/r4at_tests.log; exit 1; }
tail -1 gpurun_out/r4at_tests.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r4at_smoke.log 2>&1 || { tail -20 gpurun_out/r4at_smoke.log; exit 1; }
tail -2 gpurun_out/r4at_smoke.log
timeout -k 10 500 python -u bench.py --steps 8 --warmup 2 > gpurun_out/r4at_bench.log 2>&1 || { tail -20 gpurun_out/r4at_bench.log; exit 1; }
tail -1 gpurun_out/r4at_bench.log | cut -c1-600
