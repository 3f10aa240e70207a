#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u scripts/gemm_ablation.py 16384 4096 11008 16384 4096 4096 16384 11008 4096 2>&1 | tee gpurun_out/r4k_gemm_ablation.txt || exit 1
