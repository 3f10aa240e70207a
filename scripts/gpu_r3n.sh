#!/bin/bash
# Round 3n: FA tests after the RoPE-table batching; graph-decode kernel stats at batch 1 and 8.
set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider \
  tests/test_kernels_gpu.py tests/test_gpu_e2e.py -m gpu -k "flash or rope or deterministic or document" \
  > gpurun_out/r3n_tests.log 2>&1 || { tail -40 gpurun_out/r3n_tests.log; exit 1; }
tail -1 gpurun_out/r3n_tests.log
timeout -k 10 300 python scripts/fa_bench2.py 16,1024,32,32,128 > gpurun_out/r3n_fa.log 2>&1 && grep shape gpurun_out/r3n_fa.log
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for b in 1 8; do
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r3n_prof_b$b -o s -- python3 scripts/serve_bench.py --batches $b --graph --gen 64 > gpurun_out/r3n_prof_b$b.log 2>&1 || { tail -20 gpurun_out/r3n_prof_b$b.log; exit 1; }
f=$(find gpurun_out/r3n_prof_b$b -name '*kernel_stats.csv' | head -1) && python3 scripts/summarize_prof.py "$f" gpurun_out/r3n_decode_b${b}_kernels.txt "Llama-2-7B graph decode batch $b (prompt 128, 64 generated), fused layer + persistent skinny" && head -14 gpurun_out/r3n_decode_b${b}_kernels.txt
done
