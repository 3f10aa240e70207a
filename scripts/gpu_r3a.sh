#!/bin/bash
# Round 3: NT GEMM numerics (both variants, row maps, fused MLP) + A/B vs hipBLASLt
# on the 7B shapes + the 7B step with and without the fused MLP.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gemm_gpu.py > gpurun_out/r3a_gemm_tests.log 2>&1 || { tail -30 gpurun_out/r3a_gemm_tests.log; exit 1; }
tail -2 gpurun_out/r3a_gemm_tests.log
timeout -k 10 300 python -u scripts/gemm_nt_bench.py --json gpurun_out/r3a_gemm_nt_bench.json 2>&1 | tee gpurun_out/r3a_gemm_nt_bench.txt || exit 1
timeout -k 10 400 python -u bench.py --steps 6 --warmup 2 > gpurun_out/r3a_bench_fused.log 2>&1 || { tail -20 gpurun_out/r3a_bench_fused.log; exit 1; }
tail -1 gpurun_out/r3a_bench_fused.log
EMA_FUSED_MLP=0 timeout -k 10 400 python -u bench.py --steps 6 --warmup 2 > gpurun_out/r3a_bench_unfused.log 2>&1 || { tail -20 gpurun_out/r3a_bench_unfused.log; exit 1; }
tail -1 gpurun_out/r3a_bench_unfused.log
