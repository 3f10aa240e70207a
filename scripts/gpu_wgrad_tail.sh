#!/bin/bash
# wgrad tail split-K: tests, isolated fc1/fc2/qkv timing, 7B bench.
set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_gpu_e2e.py -m gpu -x -q -k "wgrad or linear or deterministic or e2e" \
  --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/wg_tests.log 2>&1
rc=$?; echo "wgrad tests rc=$rc"; tail -2 gpurun_out/wg_tests.log
[ $rc -eq 0 ] || { grep -E "Error|assert|FAILED" gpurun_out/wg_tests.log | head -20; exit $rc; }
timeout -k 10 300 python scripts/wgrad_shapes.py 22016x4096 12288x4096 4096x11008 4096x4096 32000x4096 > gpurun_out/wg_shapes.log 2>&1 || { tail -20 gpurun_out/wg_shapes.log; exit 1; }
cat gpurun_out/wg_shapes.log
timeout -k 10 700 python bench.py > gpurun_out/b7_default.log 2>&1 || { tail -20 gpurun_out/b7_default.log; exit 1; }
tail -1 gpurun_out/b7_default.log | cut -c1-400
