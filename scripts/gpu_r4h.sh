#!/bin/bash
# Round 4h: piece-row interleaving across waves; tile-grouping sweep (EMA_GEMM_GM).
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u scripts/gemm_ablation.py 16384 4096 11008 16384 4096 4096 2>&1 | tee gpurun_out/r4h_gemm_ablation.txt || exit 1
for gm in 4 16 -4 -16 2 -2; do
  echo "EMA_GEMM_GM=$gm"
  EMA_GEMM_GM=$gm timeout -k 10 120 python -u scripts/gemm_ablation.py 16384 4096 11008 16384 4096 4096 2>&1 | tee -a gpurun_out/r4h_gm_sweep.txt || exit 1
done
