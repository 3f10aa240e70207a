#!/bin/bash
# 7B headline: per-GPU batch 16 x 8 (default, gbs 1024 at 8 GPUs) vs 16 x 2.
set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 600 python bench.py > gpurun_out/b7_default.log 2>&1 || { tail -20 gpurun_out/b7_default.log; exit 1; }
tail -1 gpurun_out/b7_default.log
timeout -k 10 600 python bench.py --num_micro 2 --steps 8 --warmup 3 > gpurun_out/b7_nm2.log 2>&1 || { tail -20 gpurun_out/b7_nm2.log; exit 1; }
tail -1 gpurun_out/b7_nm2.log
