#!/bin/bash
# Round 3j: persistent skinny without the final-block over-fetch (tests, A/B,
# graph decode incl. the LM head on the skinny kernel), FA short-sequence
# diagnosis, kernel stats of the current Llama-2-7B training step.
set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider \
  tests/test_kernels_gpu.py tests/test_gpu_e2e.py -m gpu -k "skinny or decode or graph or kvcache" \
  > gpurun_out/r3j_tests.log 2>&1 || { tail -40 gpurun_out/r3j_tests.log; exit 1; }
tail -1 gpurun_out/r3j_tests.log
timeout -k 10 200 python -u scripts/skinny_bench.py > gpurun_out/r3j_skinny.log 2>&1 || { tail -20 gpurun_out/r3j_skinny.log; exit 1; }
grep "^M=" gpurun_out/r3j_skinny.log
timeout -k 10 400 python -u scripts/serve_bench.py --batches 1,8,16,32 --graph > gpurun_out/r3j_serve_graph.log 2>&1 || { tail -30 gpurun_out/r3j_serve_graph.log; exit 1; }
grep '^{"batch' gpurun_out/r3j_serve_graph.log
timeout -k 10 300 python -u scripts/fa_diag.py --json gpurun_out/r3j_fa_diag.json > gpurun_out/r3j_fa_diag.log 2>&1 || { tail -20 gpurun_out/r3j_fa_diag.log; exit 1; }
cat gpurun_out/r3j_fa_diag.log | grep -v amdgpu.ids
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r3j_step -o s -- python3 bench.py --steps 2 --warmup 1 > gpurun_out/r3j_step.log 2>&1 || { tail -20 gpurun_out/r3j_step.log; exit 1; }
f=$(find gpurun_out/r3j_step -name '*kernel_stats.csv' | head -1) && python3 scripts/summarize_prof.py "$f" gpurun_out/r3j_step_kernels.txt 'Llama-2-7B 1 GPU training, bench.py --steps 2 --warmup 1 (3 steps traced), round-3 default path' && head -30 gpurun_out/r3j_step_kernels.txt
