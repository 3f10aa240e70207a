#!/bin/bash
# Round 3t: kernel stats of the Llama-2-7B TP8+SP per-rank proxy step (seq 4096).
set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r3t_px -o s -- python3 bench.py --proxy llama7b-tp8 --steps 2 --warmup 1 > gpurun_out/r3t_px.log 2>&1 || { tail -20 gpurun_out/r3t_px.log; exit 1; }
tail -1 gpurun_out/r3t_px.log | cut -c1-300
f=$(find gpurun_out/r3t_px -name '*kernel_stats.csv' | head -1) && python3 scripts/summarize_prof.py "$f" gpurun_out/r3t_px_l7tp8_kernels.txt 'Llama-2-7B TP8+SP per-rank proxy, seq 4096, mbs 4 x 4 (3 steps traced)' && head -28 gpurun_out/r3t_px_l7tp8_kernels.txt
