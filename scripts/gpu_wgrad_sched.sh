#!/bin/bash
# wgrad DMA-placement variants (SCHED 2 production, 3 split, 4 spread): numerics + fc1/qkv/fc2 TF/s.
set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 200 python -u scripts/wgrad_bench.py --ablation 50 70 80 > gpurun_out/wg_sched_fc1.log 2>&1 || { tail -20 gpurun_out/wg_sched_fc1.log; exit 1; }
cat gpurun_out/wg_sched_fc1.log
WG_SHAPE=12288,4096 timeout -k 10 200 python -u scripts/wgrad_bench.py --ablation 50 70 80 > gpurun_out/wg_sched_qkv.log 2>&1 || { tail -20 gpurun_out/wg_sched_qkv.log; exit 1; }
cat gpurun_out/wg_sched_qkv.log
WG_SHAPE=4096,11008 timeout -k 10 200 python -u scripts/wgrad_bench.py --ablation 50 70 80 > gpurun_out/wg_sched_fc2.log 2>&1 || { tail -20 gpurun_out/wg_sched_fc2.log; exit 1; }
cat gpurun_out/wg_sched_fc2.log
