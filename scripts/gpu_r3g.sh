#!/bin/bash
# Round 3g: document-masked FA + FA regression tests, skinny GEMM register ring
# (tests + fused / unfused graph decode), FA timing after the doc-mask change.
set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider \
  tests/test_kernels_gpu.py tests/test_gpu_e2e.py -m gpu -k "flash or skinny or decode or graph or rope or deterministic" \
  > gpurun_out/r3g_tests.log 2>&1 || { tail -40 gpurun_out/r3g_tests.log; exit 1; }
tail -2 gpurun_out/r3g_tests.log
timeout -k 10 300 python scripts/fa_bench2.py 16,1024,32,32,128 4,4096,32,32,128 8,2048,32,2,64 > gpurun_out/r3g_fa_bench.log 2>&1 || { tail -20 gpurun_out/r3g_fa_bench.log; exit 1; }
grep shape gpurun_out/r3g_fa_bench.log
timeout -k 10 400 python -u scripts/serve_bench.py --batches 1,8,16 --graph > gpurun_out/r3g_serve_fused_graph.log 2>&1 || { tail -30 gpurun_out/r3g_serve_fused_graph.log; exit 1; }
grep '^{"batch' gpurun_out/r3g_serve_fused_graph.log
EMA_DECODE_FUSED=0 timeout -k 10 400 python -u scripts/serve_bench.py --batches 1,8,16 --graph > gpurun_out/r3g_serve_unfused_graph.log 2>&1 || { tail -30 gpurun_out/r3g_serve_unfused_graph.log; exit 1; }
grep '^{"batch' gpurun_out/r3g_serve_unfused_graph.log
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r3g_prof -o s -- python3 scripts/serve_bench.py --batches 8 --graph --gen 32 > gpurun_out/r3g_prof.log 2>&1 || { tail -20 gpurun_out/r3g_prof.log; exit 1; }
f=$(find gpurun_out/r3g_prof -name '*kernel_stats.csv' | head -1) && python3 scripts/summarize_prof.py "$f" gpurun_out/r3g_decode_b8_kernels.txt 'Llama-2-7B fused decode, batch 8, hipGraph, skinny ring' && head -16 gpurun_out/r3g_decode_b8_kernels.txt
