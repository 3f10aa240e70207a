#!/bin/bash
# All GPU tests + Llama-2-7B bench + rocprofv3 kernel profile summary.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 900 python -m pytest tests -q -x -m gpu -p no:cacheprovider > gpurun_out/gpu_tests.log 2>&1 || { echo "gpu tests failed"; tail -40 gpurun_out/gpu_tests.log; exit 1; }
tail -1 gpurun_out/gpu_tests.log
timeout -k 10 600 python bench.py --steps ${STEPS:-6} --warmup 2 > gpurun_out/bench_7b.log 2>&1 || { echo "7b bench failed"; tail -30 gpurun_out/bench_7b.log; exit 1; }
tail -1 gpurun_out/bench_7b.log
if [ "${PROFILE:-1}" = "1" ]; then
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o bench --output-format csv -- python3 bench.py --steps 2 --warmup 1 > gpurun_out/prof.log 2>&1 || { echo "prof failed"; tail -20 gpurun_out/prof.log; exit 1; }
  f=$(find gpurun_out/prof -name "*kernel_stats.csv" | head -1)
  python scripts/summarize_prof.py "$f" gpurun_out/prof_summary.csv "${PROF_TITLE:-rocprofv3 --kernel-trace --stats: Llama-2-7B bf16, 1x MI355X, seq 1024, mbs 16, 2 microbatches/step, bench.py --steps 2 --warmup 1}"
  head -22 gpurun_out/prof_summary.csv | cut -c1-150
fi
