#!/bin/bash
# Round-2 GPU check: e2e numerics + sync-free step, kernel tests, smoke,
# 1-GPU Llama-2-7B bench, FA forward variants.  Each GPU step is time-limited;
# a kernel-test failure stops the run.
set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_e2e.py -m gpu -v -s --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/gpu_e2e.log 2>&1
echo "e2e rc=$?"; grep -E "gpu \[|cpu \[|passed|failed|RuntimeError" gpurun_out/gpu_e2e.log | tail -8
timeout -k 10 900 python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread \
  -p no:cacheprovider > gpurun_out/gputests.log 2>&1
rc=$?; echo "kernel tests rc=$rc"; tail -3 gpurun_out/gputests.log
[ $rc -eq 0 ] || { grep -E "Error|assert" gpurun_out/gputests.log | head -20; exit $rc; }
timeout -k 10 300 python __graft_entry__.py smoke > gpurun_out/smoke.log 2>&1 || { tail -30 gpurun_out/smoke.log; exit 1; }
grep smoke gpurun_out/smoke.log
timeout -k 10 900 python bench.py --steps 8 --warmup 3 > gpurun_out/bench_7b.log 2>&1 || { tail -30 gpurun_out/bench_7b.log; exit 1; }
tail -1 gpurun_out/bench_7b.log
timeout -k 10 200 python scripts/fa_bench2.py > gpurun_out/fa_bench.log 2>&1 || { tail -20 gpurun_out/fa_bench.log; exit 1; }
grep shape gpurun_out/fa_bench.log
