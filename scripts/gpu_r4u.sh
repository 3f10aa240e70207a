#!/bin/bash
# Round 4u: CP document-mask pair kernels vs the CPU path, one pair at a time.
set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u scripts/cp_doc_debug.py > gpurun_out/r4u_cp_doc_debug.txt 2>&1 || { cat gpurun_out/r4u_cp_doc_debug.txt; exit 1; }
cat gpurun_out/r4u_cp_doc_debug.txt
