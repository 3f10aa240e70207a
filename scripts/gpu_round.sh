#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python scripts/gemm_bench.py --out gpurun_out/gemm_default.json > gpurun_out/gemm_default.log 2>&1 || { echo gemm failed; tail -20 gpurun_out/gemm_default.log; exit 1; }
cat gpurun_out/gemm_default.log
PYTORCH_TUNABLEOP_ENABLED=1 PYTORCH_TUNABLEOP_TUNING=1 PYTORCH_TUNABLEOP_FILENAME=gpurun_out/tunableop_results%d.csv timeout -k 10 600 python scripts/gemm_bench.py --out gpurun_out/gemm_tunable.json > gpurun_out/gemm_tunable.log 2>&1 || { echo tunable failed; tail -20 gpurun_out/gemm_tunable.log; exit 1; }
cat gpurun_out/gemm_tunable.log
STEPS=6 bash scripts/gpu_bench.sh
