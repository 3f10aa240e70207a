#!/bin/bash
# Round 4w: same-box A/B of side-stream weight-gradient GEMMs (EMA_WGRAD_STREAM) in the 7B step;
# the decode kpw threshold; training-path GPU tests with the side stream.
set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 500 python -u bench.py --steps 8 --warmup 2 > gpurun_out/r4w_bench_a.log 2>&1 || { tail -20 gpurun_out/r4w_bench_a.log; exit 1; }
tail -1 gpurun_out/r4w_bench_a.log | cut -c1-300
EMA_WGRAD_STREAM=1 timeout -k 10 500 python -u bench.py --steps 8 --warmup 2 > gpurun_out/r4w_bench_b.log 2>&1 || { tail -20 gpurun_out/r4w_bench_b.log; exit 1; }
tail -1 gpurun_out/r4w_bench_b.log | cut -c1-300
timeout -k 10 500 python -u bench.py --steps 8 --warmup 2 > gpurun_out/r4w_bench_a2.log 2>&1 || { tail -20 gpurun_out/r4w_bench_a2.log; exit 1; }
tail -1 gpurun_out/r4w_bench_a2.log | cut -c1-300
EMA_WGRAD_STREAM=1 timeout -k 10 500 python -u bench.py --steps 8 --warmup 2 > gpurun_out/r4w_bench_b2.log 2>&1 || { tail -20 gpurun_out/r4w_bench_b2.log; exit 1; }
tail -1 gpurun_out/r4w_bench_b2.log | cut -c1-300
EMA_WGRAD_STREAM=1 timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_e2e.py -m gpu > gpurun_out/r4w_e2e_side.log 2>&1 || { tail -30 gpurun_out/r4w_e2e_side.log; exit 1; }
tail -1 gpurun_out/r4w_e2e_side.log
timeout -k 10 200 python -u scripts/decode_kpw_bench.py > gpurun_out/r4w_kpw.txt 2>&1 || { tail -30 gpurun_out/r4w_kpw.txt; exit 1; }
head -2 gpurun_out/r4w_kpw.txt
