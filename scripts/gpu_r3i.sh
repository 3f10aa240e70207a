#!/bin/bash
# Round 3i: persistent skinny GEMM (X / RMSNorm in registers, ring across
# block seams): tests, A/B vs the per-block kernel, fused / unfused graph
# decode; then the simulated-TP proxies (scripts/gpu_r3h.sh).
set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider \
  tests/test_kernels_gpu.py tests/test_gpu_e2e.py -m gpu -k "skinny or decode or graph or kvcache" \
  > gpurun_out/r3i_tests.log 2>&1 || { tail -40 gpurun_out/r3i_tests.log; exit 1; }
tail -1 gpurun_out/r3i_tests.log
for ps in 1 0; do
  EMA_SKINNY_PERSIST=$ps timeout -k 10 200 python -u scripts/skinny_bench.py > gpurun_out/r3i_skinny_p$ps.log 2>&1 || { tail -20 gpurun_out/r3i_skinny_p$ps.log; exit 1; }
  echo "persist=$ps"; cat gpurun_out/r3i_skinny_p$ps.log
done
timeout -k 10 400 python -u scripts/serve_bench.py --batches 1,8,16 --graph > gpurun_out/r3i_serve_fused_graph.log 2>&1 || { tail -30 gpurun_out/r3i_serve_fused_graph.log; exit 1; }
grep '^{"batch' gpurun_out/r3i_serve_fused_graph.log
EMA_DECODE_FUSED=0 timeout -k 10 400 python -u scripts/serve_bench.py --batches 1,8,16 --graph > gpurun_out/r3i_serve_unfused_graph.log 2>&1 || { tail -30 gpurun_out/r3i_serve_unfused_graph.log; exit 1; }
grep '^{"batch' gpurun_out/r3i_serve_unfused_graph.log
bash scripts/gpu_r3h.sh
