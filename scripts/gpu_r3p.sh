#!/bin/bash
# Round 3p: decode attention (loads up front, single-chunk direct output) + batched RoPE
# tables in the FA dQ / dK epilogues: debug check, tests, serving, training bench, decode profile.
set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 120 python -u scripts/decode_debug.py > gpurun_out/r3p_decode_debug.log 2>&1 || { tail -20 gpurun_out/r3p_decode_debug.log; exit 1; }
grep "bad" gpurun_out/r3p_decode_debug.log
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider \
  tests/test_kernels_gpu.py tests/test_gpu_e2e.py -m gpu -k "decode or graph or kvcache or skinny or generat or flash or rope or deterministic or document" \
  > gpurun_out/r3p_tests.log 2>&1 || { tail -40 gpurun_out/r3p_tests.log; exit 1; }
tail -1 gpurun_out/r3p_tests.log
timeout -k 10 400 python -u scripts/serve_bench.py --batches 1,8,16,32 --graph > gpurun_out/r3p_serve_graph.log 2>&1 || { tail -30 gpurun_out/r3p_serve_graph.log; exit 1; }
grep '^{"batch' gpurun_out/r3p_serve_graph.log
timeout -k 10 400 python -u bench.py --steps 6 --warmup 2 > gpurun_out/r3p_bench.log 2>&1 || { tail -20 gpurun_out/r3p_bench.log; exit 1; }
tail -1 gpurun_out/r3p_bench.log | cut -c1-420
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r3p_prof_b1 -o s -- python3 scripts/serve_bench.py --batches 1 --graph --gen 64 > gpurun_out/r3p_prof_b1.log 2>&1 || { tail -20 gpurun_out/r3p_prof_b1.log; exit 1; }
f=$(find gpurun_out/r3p_prof_b1 -name '*kernel_stats.csv' | head -1) && python3 scripts/summarize_prof.py "$f" gpurun_out/r3p_decode_b1_kernels.txt "Llama-2-7B graph decode batch 1 (prompt 128, 64 generated), decode attention with loads up front" && head -12 gpurun_out/r3p_decode_b1_kernels.txt
