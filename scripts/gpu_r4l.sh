#!/bin/bash
# Round 4l: production one-slot schedule: GEMM tests, NT bench (variants 5/6), 7B bench.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gemm_gpu.py > gpurun_out/r4l_gemm_tests.log 2>&1 || { tail -30 gpurun_out/r4l_gemm_tests.log; exit 1; }
tail -2 gpurun_out/r4l_gemm_tests.log
timeout -k 10 300 python -u scripts/gemm_nt_bench.py --variants 5,6 2>&1 | tee gpurun_out/r4l_gemm_nt_bench.txt || exit 1
timeout -k 10 500 python -u bench.py --steps 6 --warmup 2 > gpurun_out/r4l_bench.log 2>&1 || { tail -20 gpurun_out/r4l_bench.log; exit 1; }
tail -1 gpurun_out/r4l_bench.log | cut -c1-400
EMA_GEMM_NT=6 timeout -k 10 500 python -u bench.py --steps 6 --warmup 2 > gpurun_out/r4l_bench_v6.log 2>&1 || { tail -20 gpurun_out/r4l_bench_v6.log; exit 1; }
tail -1 gpurun_out/r4l_bench_v6.log | cut -c1-400
