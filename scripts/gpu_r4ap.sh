#!/bin/bash
# Round 4ap: rmsnorm forward with the weight loads issued beside x for <= 64 rows:
# norm tests, graphed serving.
set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider \
  tests/test_kernels_gpu.py tests/test_gpu_e2e.py -m gpu -k "norm or decode" \
  > gpurun_out/r4ap_tests.log 2>&1 || { tail -40 gpurun_out/r4ap_tests.log; exit 1; }
tail -1 gpurun_out/r4ap_tests.log
timeout -k 10 400 python -u scripts/serve_bench.py --batches 1,16,24,32 --graph > gpurun_out/r4ap_serve_graph.log 2>&1 || { tail -30 gpurun_out/r4ap_serve_graph.log; exit 1; }
grep '^{"batch' gpurun_out/r4ap_serve_graph.log
