#!/bin/bash
# TN operand-layout study on one MI355X: transpose kernel + TN linear numerics,
# hipBLASLt layout sweep at the bench's token count, then full-step A/B.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
    tests/test_kernels_gpu.py -k "transpose or tn_layouts or linear_wgrad or extension" \
    > gpurun_out/tn_tests.log 2>&1 &&
timeout -k 10 300 python -u scripts/gemm_bench.py --M 16384 --out gpurun_out/gemm_layouts_m16k.json \
    > gpurun_out/gemm_layouts.log 2>&1 &&
timeout -k 10 420 python -u bench.py --steps 6 --warmup 2 > gpurun_out/bench_dgradwt.log 2>&1 &&
EMA_WGRAD_TN=1 timeout -k 10 420 python -u bench.py --steps 6 --warmup 2 \
    > gpurun_out/bench_wgradtn.log 2>&1 &&
EMA_DGRAD_WT=0 timeout -k 10 420 python -u bench.py --steps 6 --warmup 2 \
    > gpurun_out/bench_baseline.log 2>&1
