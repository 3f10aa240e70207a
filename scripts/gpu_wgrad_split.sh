#!/bin/bash
# Split-K wgrad: wgrad/linear GPU tests, then same-box proxy A/B (new floor 32 tiles vs old 256).
set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_gpu_e2e.py -m gpu -x -q -k "wgrad or linear or deterministic or e2e or llama" \
  --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/wg_tests.log 2>&1
rc=$?; echo "wgrad tests rc=$rc"; tail -2 gpurun_out/wg_tests.log
[ $rc -eq 0 ] || { grep -E "Error|assert|FAILED" gpurun_out/wg_tests.log | head -20; exit $rc; }
for px in llama7b-tp8 llama70b-tp8; do
for mt in 32 256; do
  EMA_WGRAD_MIN_TILES=$mt timeout -k 10 600 python bench.py --proxy $px --steps 3 --warmup 1 > gpurun_out/px_${px}_$mt.log 2>&1 || { tail -20 gpurun_out/px_${px}_$mt.log; exit 1; }
  echo "$px min_tiles=$mt $(tail -1 gpurun_out/px_${px}_$mt.log | python3 -c 'import json,sys; r=json.loads(sys.stdin.read()); print(r["value"], r["ms_per_step"], r["mfu"])')"
done
done
