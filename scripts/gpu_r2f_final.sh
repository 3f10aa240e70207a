#!/bin/bash
# Evidence after the wgrad DMA split + hipGraph decode: 7B headline (default
# bench), seq 4096, TP-rank proxies, serving, rocprofv3 step kernel stats.
set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
run() {  # name, timeout, args...
  local n=$1 t=$2; shift 2
  timeout -k 10 $t python bench.py "$@" > gpurun_out/$n.log 2>&1 || { echo "$n failed"; tail -20 gpurun_out/$n.log; exit 1; }
  tail -1 gpurun_out/$n.log
}
run b7_default 700
run b7_s4k 700 --steps 6 --warmup 2 --seq_len 4096 --micro_batch 4 --num_micro 8
run px_l7tp8 600 --proxy llama7b-tp8 --steps 4 --warmup 2
run px_l70tp8 900 --proxy llama70b-tp8 --steps 3 --warmup 1
run px_f40 900 --proxy falcon40b-tp4-pp2 --steps 3 --warmup 1
timeout -k 10 600 python scripts/serve_bench.py --batches 1,8,32 --graph > gpurun_out/serve.log 2>&1 || { tail -20 gpurun_out/serve.log; exit 1; }
grep batch gpurun_out/serve.log
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof7b -o s -- python3 bench.py --steps 1 --warmup 1 > gpurun_out/prof7b.log 2>&1; echo "prof rc=$?"
