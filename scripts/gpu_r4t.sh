#!/bin/bash
# Round 4t: full GPU suite (incl. CP document-mask ring kernels), smoke, 7B bench, serving, decode kpw.
set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u scripts/cp_doc_debug.py > gpurun_out/r4t_cp_doc_debug.txt 2>&1 || { cat gpurun_out/r4t_cp_doc_debug.txt; exit 1; }
grep "fwd" gpurun_out/r4t_cp_doc_debug.txt
timeout -k 10 900 python -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider \
  tests -m gpu > gpurun_out/r4t_tests.log 2>&1 || { tail -40 gpurun_out/r4t_tests.log; exit 1; }
tail -1 gpurun_out/r4t_tests.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r4t_smoke.log 2>&1 || { tail -20 gpurun_out/r4t_smoke.log; exit 1; }
tail -2 gpurun_out/r4t_smoke.log
timeout -k 10 500 python -u bench.py --steps 8 --warmup 2 > gpurun_out/r4t_bench.log 2>&1 || { tail -20 gpurun_out/r4t_bench.log; exit 1; }
tail -1 gpurun_out/r4t_bench.log | cut -c1-500
timeout -k 10 400 python -u scripts/serve_bench.py --batches 1,8,16 --graph > gpurun_out/r4t_serve_graph.log 2>&1 || { tail -30 gpurun_out/r4t_serve_graph.log; exit 1; }
grep '^{"batch' gpurun_out/r4t_serve_graph.log
timeout -k 10 200 python -u scripts/decode_kpw_bench.py > gpurun_out/r4t_kpw.txt 2>&1 || { tail -30 gpurun_out/r4t_kpw.txt; exit 1; }
cat gpurun_out/r4t_kpw.txt
