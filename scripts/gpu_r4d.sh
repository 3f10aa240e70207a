#!/bin/bash
# Round 4d: NT GEMM ablation modes, SP piece-major overlap cost, 7B bench.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u scripts/gemm_ablation.py 2>&1 | tee gpurun_out/r4d_gemm_ablation.txt || exit 1
timeout -k 10 200 python -u scripts/sp_overlap_bench.py --json gpurun_out/r4d_sp_pieces.json 2>&1 | tee gpurun_out/r4d_sp_pieces.txt || exit 1
timeout -k 10 500 python -u bench.py --steps 6 --warmup 2 > gpurun_out/r4d_bench.log 2>&1 || { tail -20 gpurun_out/r4d_bench.log; exit 1; }
tail -1 gpurun_out/r4d_bench.log | cut -c1-600
