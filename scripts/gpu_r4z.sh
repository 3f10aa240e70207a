#!/bin/bash
# Round 4z: greedy tail at 1024 threads: tests, serving, b1 profile.
set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider \
  tests/test_kernels_gpu.py tests/test_gpu_e2e.py -m gpu -k "greedy_tail or decode or graph or skinny" \
  > gpurun_out/r4z_tests.log 2>&1 || { tail -40 gpurun_out/r4z_tests.log; exit 1; }
tail -1 gpurun_out/r4z_tests.log
timeout -k 10 400 python -u scripts/serve_bench.py --batches 1,8,16,32 --graph > gpurun_out/r4z_serve_graph.log 2>&1 || { tail -30 gpurun_out/r4z_serve_graph.log; exit 1; }
grep '^{"batch' gpurun_out/r4z_serve_graph.log
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r4z_prof_b1 -o s -- python3 scripts/serve_bench.py --batches 1 --graph --gen 64 > gpurun_out/r4z_prof_b1.log 2>&1 || { tail -20 gpurun_out/r4z_prof_b1.log; exit 1; }
f=$(find gpurun_out/r4z_prof_b1 -name '*kernel_stats.csv' | head -1) && python3 scripts/summarize_prof.py "$f" gpurun_out/r4z_decode_b1_kernels.txt "Llama-2-7B graph decode batch 1 (prompt 128, 64 generated): fused greedy tail" && head -20 gpurun_out/r4z_decode_b1_kernels.txt
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r4z_prof_b1_g32 -o s -- python3 scripts/serve_bench.py --batches 1 --graph --gen 32 > gpurun_out/r4z_prof_b1_g32.log 2>&1 || { tail -20 gpurun_out/r4z_prof_b1_g32.log; exit 1; }
f=$(find gpurun_out/r4z_prof_b1_g32 -name '*kernel_stats.csv' | head -1) && python3 scripts/summarize_prof.py "$f" gpurun_out/r4z_decode_b1_g32_kernels.txt "b1 graph decode, 32 generated (fill / copy counts vs 64)" && grep -i "fill\|copyBuffer\|greedy" gpurun_out/r4z_decode_b1_g32_kernels.txt
