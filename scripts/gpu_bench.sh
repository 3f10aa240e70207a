#!/bin/bash
# Kernel tests + smoke + Llama-2-7B bench + rocprofv3 kernel profile (gpurun).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
STEPS=${STEPS:-6}
timeout -k 10 600 python -m pytest tests/test_kernels_gpu.py -q -m gpu -p no:cacheprovider > gpurun_out/kernels.log 2>&1
echo "kernel tests rc=$?"; tail -3 gpurun_out/kernels.log
timeout -k 10 600 python bench.py --model tiny --steps 3 --warmup 1 > gpurun_out/bench_tiny.log 2>&1 || { echo "tiny bench failed"; tail -30 gpurun_out/bench_tiny.log; exit 1; }
tail -1 gpurun_out/bench_tiny.log
timeout -k 10 1200 python bench.py --steps $STEPS --warmup 2 "$@" > gpurun_out/bench_7b.log 2>&1 || { echo "7b bench failed"; tail -30 gpurun_out/bench_7b.log; exit 1; }
tail -1 gpurun_out/bench_7b.log
if [ "${PROFILE:-1}" = "1" ]; then
  cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT}"
  timeout -k 10 900 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o bench --output-format csv -- python bench.py --steps 2 --warmup 1 "$@" > gpurun_out/prof.log 2>&1
  echo "rocprof rc=$?"
fi
