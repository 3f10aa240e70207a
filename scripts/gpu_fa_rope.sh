#!/bin/bash
# FA with fused RoPE: FA/rope GPU tests, FA timing, 7B bench.
set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -q -k "flash or rope or deterministic" \
  --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/fa_tests.log 2>&1
rc=$?; echo "fa tests rc=$rc"; tail -2 gpurun_out/fa_tests.log
[ $rc -eq 0 ] || { grep -E "Error|assert|FAILED" gpurun_out/fa_tests.log | head -20; exit $rc; }
timeout -k 10 200 python scripts/fa_bench2.py > gpurun_out/fa_bench.log 2>&1 || { tail -20 gpurun_out/fa_bench.log; exit 1; }
grep shape gpurun_out/fa_bench.log
timeout -k 10 600 python bench.py --steps 8 --warmup 3 > gpurun_out/bench_7b.log 2>&1 || { tail -30 gpurun_out/bench_7b.log; exit 1; }
tail -1 gpurun_out/bench_7b.log
