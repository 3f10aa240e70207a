#!/bin/bash
# Late-round GPU check: all GPU tests, the 1-GPU bench (headline config) and a
# seq-4096 Llama-2-7B run for the long-context comparison in BASELINE.md.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests -q -x -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { echo "gpu tests failed"; tail -40 gpurun_out/gpu_tests.log; exit 1; }
tail -1 gpurun_out/gpu_tests.log
timeout -k 10 420 python -u bench.py --steps 6 --warmup 2 > gpurun_out/bench_7b.log 2>&1 || { echo "7b bench failed"; tail -30 gpurun_out/bench_7b.log; exit 1; }
tail -1 gpurun_out/bench_7b.log
timeout -k 10 420 python -u bench.py --steps 4 --warmup 2 --seq_len 4096 --micro_batch 4 --num_micro 2 > gpurun_out/bench_7b_s4096.log 2>&1 || { echo "s4096 bench failed"; tail -30 gpurun_out/bench_7b_s4096.log; exit 1; }
tail -1 gpurun_out/bench_7b_s4096.log
