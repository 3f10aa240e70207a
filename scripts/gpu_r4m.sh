#!/bin/bash
# Round 4m: decode weight-stream layout experiment + current serving baseline.
set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 120 ./scripts/gemv_layout_bench > gpurun_out/r4m_gemv_layout.txt 2>&1 || { cat gpurun_out/r4m_gemv_layout.txt; exit 1; }
cat gpurun_out/r4m_gemv_layout.txt
timeout -k 10 400 python -u scripts/serve_bench.py --batches 1,8 --graph > gpurun_out/r4m_serve_graph.log 2>&1 || { tail -30 gpurun_out/r4m_serve_graph.log; exit 1; }
grep '^{"batch' gpurun_out/r4m_serve_graph.log
