#!/bin/bash
# Round 3u: Llama-2-7B step kernel stats with the unfused MLP (EMA_FUSED_MLP=0) for
# an in-model comparison against profiles/r3j_llama7b_1gpu_step_kernels.txt.
set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
EMA_FUSED_MLP=0 timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r3u_step -o s -- python3 bench.py --steps 2 --warmup 1 > gpurun_out/r3u_step.log 2>&1 || { tail -20 gpurun_out/r3u_step.log; exit 1; }
f=$(find gpurun_out/r3u_step -name '*kernel_stats.csv' | head -1) && python3 scripts/summarize_prof.py "$f" gpurun_out/r3u_step_kernels.txt 'Llama-2-7B 1 GPU training, EMA_FUSED_MLP=0 (hipBLASLt + GLU kernels), bench.py --steps 2 --warmup 1 (3 steps traced)' && head -16 gpurun_out/r3u_step_kernels.txt
rm -f gpurun_out/r3u_step/*kernel_trace.csv
