#!/bin/bash
# Round 4: NT GEMM early-refill schedule (variant 5) numerics + A/B vs variant 4 and hipBLASLt.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gemm_gpu.py > gpurun_out/r4a_gemm_tests.log 2>&1 || { tail -30 gpurun_out/r4a_gemm_tests.log; exit 1; }
tail -2 gpurun_out/r4a_gemm_tests.log
timeout -k 10 300 python -u scripts/gemm_nt_bench.py --variants 5,6 --json gpurun_out/r4a_gemm_nt_bench.json 2>&1 | tee gpurun_out/r4a_gemm_nt_bench.txt || exit 1
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k wgrad > gpurun_out/r4a_wgrad_tests.log 2>&1 || { tail -30 gpurun_out/r4a_wgrad_tests.log; exit 1; }
tail -2 gpurun_out/r4a_wgrad_tests.log
timeout -k 10 300 python -u scripts/wgrad_bench.py --variants 2>&1 | tee gpurun_out/r4a_wgrad_variants.txt || exit 1
