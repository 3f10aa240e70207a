#!/bin/bash
# Round 3h: simulated-TP per-rank proxies of the three multi-GPU BASELINE configs
# (SP row sharding, TP comm accounting, memory-model recompute for 70B).
set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
for px in llama7b-tp8 llama70b-tp8 falcon40b-tp4-pp2; do
  timeout -k 10 500 python -u bench.py --proxy $px --steps 3 --warmup 1 > gpurun_out/r3h_px_$px.log 2>&1 || { tail -30 gpurun_out/r3h_px_$px.log; exit 1; }
  tail -1 gpurun_out/r3h_px_$px.log > gpurun_out/r3h_px_$px.json
  python3 -c "import json,sys; r=json.load(open('gpurun_out/r3h_px_$px.json')); print('$px', r['value'], 'tok/s', 'mfu', r['mfu'], 'mem', r['max_mem_gb'], r['config']['parallelism'], {k: v for k, v in r.items() if k.startswith('proxy_') and not isinstance(v, (dict, list))})"
done
