#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
for a in 0 1; do
  EMA_FA_ABLATE=$a timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/faabl_$a -o f --output-format csv -- python3 scripts/fa_bench.py > gpurun_out/faabl_$a.log 2>&1 || { echo prof failed; tail -20 gpurun_out/faabl_$a.log; exit 1; }
  f=$(find gpurun_out/faabl_$a -name "*kernel_stats.csv" | head -1)
  echo "== ablate $a"; grep fa_ "$f" | cut -d, -f1,4 | cut -c1-40,80-
done
