#!/bin/bash
# r2f: wgrad SCHED 3 + hipGraph decode: tests, serving (eager vs graph), 7B bench.
set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_gpu_e2e.py -m gpu -x -v -k "wgrad or decode or graph or linear or deterministic" \
  --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/r2f_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/r2f_tests.log
[ $rc -eq 0 ] || { grep -E "Error|assert|FAILED" gpurun_out/r2f_tests.log | head -30; exit $rc; }
timeout -k 10 300 python -u scripts/serve_bench.py --graph > gpurun_out/serve_graph.log 2>&1 || { tail -30 gpurun_out/serve_graph.log; exit 1; }
grep '^{' gpurun_out/serve_graph.log
timeout -k 10 300 python -u scripts/serve_bench.py > gpurun_out/serve_eager.log 2>&1 || { tail -30 gpurun_out/serve_eager.log; exit 1; }
grep '^{' gpurun_out/serve_eager.log
timeout -k 10 600 python bench.py > gpurun_out/b7_default.log 2>&1 || { tail -20 gpurun_out/b7_default.log; exit 1; }
tail -1 gpurun_out/b7_default.log | cut -c1-600
