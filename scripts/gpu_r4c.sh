#!/bin/bash
# Round 4c: FA forward VALU cuts (mask, packed softmax, permlane reductions):
# FA numerics tests + timing on the training shapes.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py tests/test_doc_mask.py -k "flash or attention or doc" > gpurun_out/r4c_fa_tests.log 2>&1 || { tail -30 gpurun_out/r4c_fa_tests.log; exit 1; }
tail -2 gpurun_out/r4c_fa_tests.log
timeout -k 10 300 python -u scripts/fa_bench2.py 2>&1 | tee gpurun_out/r4c_fa_bench.txt || exit 1
