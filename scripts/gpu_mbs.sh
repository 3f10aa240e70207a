#!/bin/bash
# micro-batch shape sweep at fixed per-GPU global batch (32 x 1024 tokens)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
for cfg in "16 2" "4 8" "32 1"; do
  set -- $cfg
  timeout -k 10 400 python bench.py --steps 5 --warmup 2 --micro_batch $1 --num_micro $2 > gpurun_out/bench_mbs$1.log 2>&1 || { echo "mbs $1 failed"; tail -5 gpurun_out/bench_mbs$1.log; exit 1; }
  tail -1 gpurun_out/bench_mbs$1.log
done
