#!/bin/bash
# Round 4ae: 7B at seq 4096 (mbs 4 x 8) on the round-4 tree.
set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u bench.py --seq_len 4096 --micro_batch 4 --num_micro 8 --steps 5 --warmup 2 > gpurun_out/r4ae_bench_s4k.log 2>&1 || { tail -20 gpurun_out/r4ae_bench_s4k.log; exit 1; }
tail -1 gpurun_out/r4ae_bench_s4k.log | cut -c1-400
