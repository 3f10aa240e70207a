#!/bin/bash
# Round 4j: wgrad 4-wave persistent with spread DMA vs 8-wave ping-pong vs hipBLASLt.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k wgrad > gpurun_out/r4j_wgrad_tests.log 2>&1 || { tail -30 gpurun_out/r4j_wgrad_tests.log; exit 1; }
tail -2 gpurun_out/r4j_wgrad_tests.log
timeout -k 10 300 python -u scripts/wgrad_bench.py --variants 2>&1 | tee gpurun_out/r4j_wgrad_variants.txt || exit 1
