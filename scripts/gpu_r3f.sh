#!/bin/bash
# Round 3f (re-entry check): full GPU suite + smoke, 1-GPU bench, fused graph decode serving.
set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
bash scripts/gpu_tests_all.sh || exit 1
timeout -k 10 400 python -u bench.py --steps 8 --warmup 3 > gpurun_out/r3f_bench.log 2>&1 || { tail -20 gpurun_out/r3f_bench.log; exit 1; }
tail -1 gpurun_out/r3f_bench.log | cut -c1-600
timeout -k 10 400 python -u scripts/serve_bench.py --batches 1,8,16 --graph > gpurun_out/r3f_serve_fused_graph.log 2>&1 || { tail -30 gpurun_out/r3f_serve_fused_graph.log; exit 1; }
grep batch gpurun_out/r3f_serve_fused_graph.log
EMA_DECODE_FUSED=0 timeout -k 10 400 python -u scripts/serve_bench.py --batches 1,8,16 --graph > gpurun_out/r3f_serve_unfused_graph.log 2>&1 || { tail -30 gpurun_out/r3f_serve_unfused_graph.log; exit 1; }
grep batch gpurun_out/r3f_serve_unfused_graph.log
