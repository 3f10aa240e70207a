#!/bin/bash
# wgrad SCHED 5 (3 + 1 DMA split) vs SCHED 3 (2 + 2): wgrad tests, then the 7B bench twice on one box.
set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_gpu_e2e.py -m gpu -x -q -k "wgrad or linear or deterministic or e2e" \
  --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/wg_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -1 gpurun_out/wg_tests.log
[ $rc -eq 0 ] || { grep -E "Error|assert|FAILED" gpurun_out/wg_tests.log | head -20; exit $rc; }
for v in 3 5 3 5; do
  EMA_WGRAD_SCHED=$v timeout -k 10 600 python bench.py --steps 6 --warmup 2 > gpurun_out/ab_s$v.log 2>&1 || { tail -20 gpurun_out/ab_s$v.log; exit 1; }
  echo "sched=$v $(tail -1 gpurun_out/ab_s$v.log | python3 -c 'import json,sys; d=json.load(sys.stdin); print(d["value"], d["mfu"])')"
done
