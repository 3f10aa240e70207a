#!/bin/bash
# Round 4v: b1 decode kernel profile after the X-first skinny prologue; 7B bench repeat (box variance check).
set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r4v_prof_b1 -o s -- python3 scripts/serve_bench.py --batches 1 --graph --gen 64 > gpurun_out/r4v_prof_b1.log 2>&1 || { tail -20 gpurun_out/r4v_prof_b1.log; exit 1; }
f=$(find gpurun_out/r4v_prof_b1 -name '*kernel_stats.csv' | head -1) && python3 scripts/summarize_prof.py "$f" gpurun_out/r4v_decode_b1_kernels.txt "Llama-2-7B graph decode batch 1 (prompt 128, 64 generated): X-first skinny prologue" && head -10 gpurun_out/r4v_decode_b1_kernels.txt
timeout -k 10 500 python -u bench.py --steps 8 --warmup 2 > gpurun_out/r4v_bench.log 2>&1 || { tail -20 gpurun_out/r4v_bench.log; exit 1; }
tail -1 gpurun_out/r4v_bench.log | cut -c1-400
