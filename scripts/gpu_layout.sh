#!/bin/bash
# GEMM layout study (incl. token-contiguous wgrad) + current bench + kernel profile.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python scripts/gemm_bench.py --out gpurun_out/gemm_layouts2.json > gpurun_out/gemm_layouts2.log 2>&1 || { echo gemm failed; tail -20 gpurun_out/gemm_layouts2.log; exit 1; }
cat gpurun_out/gemm_layouts2.log
timeout -k 10 400 python bench.py --steps 6 --warmup 2 > gpurun_out/bench.log 2>&1 || { echo bench failed; tail -30 gpurun_out/bench.log; exit 1; }
tail -1 gpurun_out/bench.log
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 > gpurun_out/prof.log 2>&1 || { echo prof failed; tail -30 gpurun_out/prof.log; exit 1; }
f=$(find gpurun_out/prof -name "*kernel_stats.csv" | head -1); python scripts/summarize_prof.py "$f" gpurun_out/prof_summary.csv "rocprofv3 kernel stats, bench.py --steps 2 --warmup 1"; head -30 gpurun_out/prof_summary.csv
