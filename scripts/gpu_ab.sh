#!/bin/bash
# Kernel tests, then the 7B bench: tuned hipBLASLt solutions vs heuristic ones.
set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_kernels_gpu.py -q -m gpu -p no:cacheprovider > gpurun_out/kernels.log 2>&1
rc=$?; echo "kernel tests rc=$rc"; tail -3 gpurun_out/kernels.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python bench.py --steps 6 --warmup 2 > gpurun_out/bench_tuned.log 2>&1 || { tail -30 gpurun_out/bench_tuned.log; exit 1; }
tail -1 gpurun_out/bench_tuned.log
EMA_GEMM_TUNE=0 timeout -k 10 900 python bench.py --steps 6 --warmup 2 > gpurun_out/bench_untuned.log 2>&1 || { tail -30 gpurun_out/bench_untuned.log; exit 1; }
tail -1 gpurun_out/bench_untuned.log
cp ~/.cache/epfl_megatron_amd/gemm_tune.json gpurun_out/gemm_tune_cache.json || true
