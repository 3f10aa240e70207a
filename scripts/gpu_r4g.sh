#!/bin/bash
# Round 4g: NT DMA spreading schedules + GLU/DGLU persistent epilogues.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gemm_gpu.py > gpurun_out/r4g_gemm_tests.log 2>&1 || { tail -30 gpurun_out/r4g_gemm_tests.log; exit 1; }
tail -2 gpurun_out/r4g_gemm_tests.log
timeout -k 10 300 python -u scripts/gemm_ablation.py 16384 4096 11008 16384 4096 4096 16384 11008 4096 2>&1 | tee gpurun_out/r4g_gemm_ablation.txt || exit 1
timeout -k 10 300 python -u scripts/gemm_nt_bench.py --variants 5,6 2>&1 | tee gpurun_out/r4g_gemm_nt_bench.txt || exit 1
