#!/bin/bash
# Round 3o: decode attention with every load issued up front and single-chunk direct output.
set -o pipefail
timeout -k 10 120 python -u scripts/decode_debug.py 2>&1 | grep -v amdgpu.ids || exit 1
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider \
  tests/test_kernels_gpu.py tests/test_gpu_e2e.py -m gpu -k "decode or graph or kvcache or skinny or generat" \
  > gpurun_out/r3o_tests.log 2>&1 || { tail -40 gpurun_out/r3o_tests.log; exit 1; }
tail -1 gpurun_out/r3o_tests.log
timeout -k 10 400 python -u scripts/serve_bench.py --batches 1,8,16,32 --graph > gpurun_out/r3o_serve_graph.log 2>&1 || { tail -30 gpurun_out/r3o_serve_graph.log; exit 1; }
grep '^{"batch' gpurun_out/r3o_serve_graph.log
timeout -k 10 400 python -u scripts/serve_bench.py --batches 1,8 > gpurun_out/r3o_serve_eager.log 2>&1 || { tail -30 gpurun_out/r3o_serve_eager.log; exit 1; }
grep '^{"batch' gpurun_out/r3o_serve_eager.log
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r3o_prof_b1 -o s -- python3 scripts/serve_bench.py --batches 1 --graph --gen 64 > gpurun_out/r3o_prof_b1.log 2>&1 || { tail -20 gpurun_out/r3o_prof_b1.log; exit 1; }
f=$(find gpurun_out/r3o_prof_b1 -name '*kernel_stats.csv' | head -1) && python3 scripts/summarize_prof.py "$f" gpurun_out/r3o_decode_b1_kernels.txt "Llama-2-7B graph decode batch 1 (prompt 128, 64 generated), decode attention loads up front" && head -12 gpurun_out/r3o_decode_b1_kernels.txt
