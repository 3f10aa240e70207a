#!/bin/bash
# Round 4e: NT GEMM DMA-cost ablation (register loads / half DMA), FA backward
# VALU cuts + fused ring-attention merge: numerics + timing.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u scripts/gemm_ablation.py 16384 4096 11008 16384 4096 4096 2>&1 | tee gpurun_out/r4e_gemm_ablation.txt || exit 1
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py tests/test_doc_mask.py tests/test_context_parallel.py -k "flash or attention or doc or ring" > gpurun_out/r4e_fa_tests.log 2>&1 || { tail -30 gpurun_out/r4e_fa_tests.log; exit 1; }
tail -2 gpurun_out/r4e_fa_tests.log
timeout -k 10 300 python -u scripts/fa_bench2.py 2>&1 | tee gpurun_out/r4e_fa_bench.txt || exit 1
timeout -k 10 300 python -u scripts/cp_pair_bench.py 2>&1 | tee gpurun_out/r4e_cp_pair_bench.txt || exit 1
