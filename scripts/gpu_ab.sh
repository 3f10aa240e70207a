#!/bin/bash
# Kernel tests, then the 7B bench with the hand-written wgrad vs hipBLASLt.
set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_kernels_gpu.py -q -m gpu -p no:cacheprovider > gpurun_out/kernels.log 2>&1
rc=$?; echo "kernel tests rc=$rc"; tail -3 gpurun_out/kernels.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python bench.py --steps 6 --warmup 2 > gpurun_out/bench_hip.log 2>&1 || { tail -30 gpurun_out/bench_hip.log; exit 1; }
tail -1 gpurun_out/bench_hip.log
EMA_WGRAD=hipblaslt timeout -k 10 900 python bench.py --steps 6 --warmup 2 > gpurun_out/bench_lt.log 2>&1 || { tail -30 gpurun_out/bench_lt.log; exit 1; }
tail -1 gpurun_out/bench_lt.log
