#!/bin/bash
# FA numerics + timing + dkdv stamps (diagnostic) + per-kernel stats
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -m pytest tests/test_kernels_gpu.py -q -x -k "flash" > gpurun_out/fa_tests.log 2>&1 || { echo tests failed; tail -40 gpurun_out/fa_tests.log; exit 1; }
tail -1 gpurun_out/fa_tests.log
timeout -k 10 120 python scripts/fa_bench.py 2>&1 | tail -2
EMA_FA_STAMPS=1 timeout -k 10 120 python scripts/fa_bench.py > gpurun_out/fa_stamps.log 2>&1 || { echo stamps failed; tail -20 gpurun_out/fa_stamps.log; exit 1; }
grep stamps gpurun_out/fa_stamps.log | tail -1
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/faq -o f --output-format csv -- python3 scripts/fa_bench.py > gpurun_out/faq.log 2>&1 || { echo prof failed; exit 1; }
f=$(find gpurun_out/faq -name "*kernel_stats.csv" | head -1); grep fa_ "$f" | cut -d, -f1,4 | cut -c1-40,80-
