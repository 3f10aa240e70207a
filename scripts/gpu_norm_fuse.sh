#!/bin/bash
# Norm weight-grad fusion into main_grad: norm/e2e GPU tests, 7B bench, TP8-proxy bench.
set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_gpu_e2e.py -m gpu -x -q -k "norm or e2e or llama or falcon" \
  --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/norm_tests.log 2>&1
rc=$?; echo "norm tests rc=$rc"; tail -2 gpurun_out/norm_tests.log
[ $rc -eq 0 ] || { grep -E "Error|assert|FAILED" gpurun_out/norm_tests.log | head -20; exit $rc; }
timeout -k 10 600 python bench.py --proxy llama7b-tp8 --steps 4 --warmup 2 > gpurun_out/px_l7tp8.log 2>&1 || { tail -20 gpurun_out/px_l7tp8.log; exit 1; }
tail -1 gpurun_out/px_l7tp8.log
timeout -k 10 600 python bench.py > gpurun_out/b7_s1k.log 2>&1 || { tail -20 gpurun_out/b7_s1k.log; exit 1; }
tail -1 gpurun_out/b7_s1k.log
