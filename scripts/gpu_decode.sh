#!/bin/bash
# Decode attention kernel: GPU tests + timing vs the FA forward kernel.
set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_inference.py -m gpu -x -q -k "decode or kvcache or flash or inference" \
  --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/dec_tests.log 2>&1
rc=$?; echo "decode tests rc=$rc"; tail -2 gpurun_out/dec_tests.log
[ $rc -eq 0 ] || { grep -E "Error|assert|FAILED" gpurun_out/dec_tests.log | head -20; exit $rc; }
timeout -k 10 200 python scripts/decode_bench.py > gpurun_out/decode_bench.log 2>&1 || { tail -20 gpurun_out/decode_bench.log; exit 1; }
cat gpurun_out/decode_bench.log
