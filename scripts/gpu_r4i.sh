#!/bin/bash
# Round 4i: full GPU suite, 7B bench, kernel stats of the current step.
set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider \
  tests -m gpu > gpurun_out/r4i_tests.log 2>&1 || { tail -40 gpurun_out/r4i_tests.log; exit 1; }
tail -1 gpurun_out/r4i_tests.log
timeout -k 10 500 python -u bench.py --steps 8 --warmup 2 > gpurun_out/r4i_bench.log 2>&1 || { tail -20 gpurun_out/r4i_bench.log; exit 1; }
tail -1 gpurun_out/r4i_bench.log | cut -c1-500
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r4i_step -o s -- python3 bench.py --steps 2 --warmup 1 > gpurun_out/r4i_step.log 2>&1 || { tail -20 gpurun_out/r4i_step.log; exit 1; }
f=$(find gpurun_out/r4i_step -name '*kernel_stats.csv' | head -1) && python3 scripts/summarize_prof.py "$f" gpurun_out/r4i_step_kernels.txt 'Llama-2-7B 1 GPU training, bench.py --steps 2 --warmup 1 (3 steps traced), round-4 default path' && head -24 gpurun_out/r4i_step_kernels.txt
