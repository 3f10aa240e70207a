#!/bin/bash
# GLU half-block tail (skinny_pgemm_k): skinny / decode tests, rope / ring tests, serving A/B vs
# the previous commit's .so is not possible in one tree, so: serving + kernel bench now; CP pair bench.
set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -v --timeout 120 \
  --timeout-method thread -p no:cacheprovider -k "skinny or decode or rope or ring" > gpurun_out/r3aa_tests.log 2>&1
rc=$?; tail -4 gpurun_out/r3aa_tests.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" gpurun_out/r3aa_tests.log | head; exit $rc; }
timeout -k 10 200 python -u scripts/serve_bench.py --batches 1,8,16,32 --graph > gpurun_out/r3aa_serve.log 2>&1 \
  || { tail -20 gpurun_out/r3aa_serve.log; exit 1; }
grep decode_tokens gpurun_out/r3aa_serve.log
timeout -k 10 120 python -u scripts/skinny_bench.py > gpurun_out/r3aa_skinny.log 2>&1 || { tail -5 gpurun_out/r3aa_skinny.log; exit 1; }
grep "N=22016" gpurun_out/r3aa_skinny.log
timeout -k 10 300 python -u scripts/cp_pair_bench.py > gpurun_out/r3aa_cp_bench.log 2>&1
rc=$?; tail -3 gpurun_out/r3aa_cp_bench.log; exit $rc
