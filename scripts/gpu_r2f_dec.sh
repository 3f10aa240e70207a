#!/bin/bash
# decode kernel with RH = heads per KV group (MHA: 1): tests, decode bench, serving eager/graph.
set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_gpu_e2e.py -m gpu -x -q -k "decode or graph or kv_cached" \
  --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/dec_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/dec_tests.log
[ $rc -eq 0 ] || { grep -E "Error|assert|FAILED" gpurun_out/dec_tests.log | head -20; exit $rc; }
timeout -k 10 200 python scripts/decode_bench.py > gpurun_out/decode_bench.log 2>&1 || { tail -20 gpurun_out/decode_bench.log; exit 1; }
grep "b=" gpurun_out/decode_bench.log
for g in "" "--graph"; do
  timeout -k 10 300 python -u scripts/serve_bench.py $g > gpurun_out/serve_r2f$g.log 2>&1 || { tail -20 gpurun_out/serve_r2f$g.log; exit 1; }
  grep '^{' gpurun_out/serve_r2f$g.log
done
