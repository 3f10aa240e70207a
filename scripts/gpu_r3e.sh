#!/bin/bash
# Round 3e: fused decode (skinny GEMM with norm / RoPE / cache / GLU / residual
# fused) vs unfused, hipGraph and eager, batch 1 / 8 / 16; kernel stats of the
# fused batch-8 graph decode.
set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u scripts/serve_bench.py --batches 1,8,16 --graph > gpurun_out/r3e_serve_fused_graph.log 2>&1 || { tail -30 gpurun_out/r3e_serve_fused_graph.log; exit 1; }
grep batch gpurun_out/r3e_serve_fused_graph.log
EMA_DECODE_FUSED=0 timeout -k 10 400 python -u scripts/serve_bench.py --batches 1,8,16 --graph > gpurun_out/r3e_serve_unfused_graph.log 2>&1 || { tail -30 gpurun_out/r3e_serve_unfused_graph.log; exit 1; }
grep batch gpurun_out/r3e_serve_unfused_graph.log
timeout -k 10 400 python -u scripts/serve_bench.py --batches 1,8 > gpurun_out/r3e_serve_fused_eager.log 2>&1 || { tail -30 gpurun_out/r3e_serve_fused_eager.log; exit 1; }
grep batch gpurun_out/r3e_serve_fused_eager.log
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r3e_prof -o s -- python3 scripts/serve_bench.py --batches 8 --graph --gen 32 > gpurun_out/r3e_prof.log 2>&1 || { tail -20 gpurun_out/r3e_prof.log; exit 1; }
f=$(find gpurun_out/r3e_prof -name '*kernel_stats.csv' | head -1) && python3 scripts/summarize_prof.py "$f" gpurun_out/r3e_decode_b8_kernels.txt 'Llama-2-7B fused decode, batch 8, hipGraph' && head -25 gpurun_out/r3e_decode_b8_kernels.txt
