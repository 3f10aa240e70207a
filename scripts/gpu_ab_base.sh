#!/bin/bash
# Same-box A/B of the Llama-2-7B training bench: ab_base/ (a build of an earlier
# revision, see its git rev in the profile) vs the current tree, alternating.
set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
for r in 1 2; do
  for v in base new; do
    if [ $v = base ]; then d=ab_base; else d=.; fi
    timeout -k 10 400 python -u $d/bench.py --steps 6 --warmup 2 > gpurun_out/ab_$v$r.log 2>&1 || { tail -20 gpurun_out/ab_$v$r.log; exit 1; }
    echo "$v $r: $(tail -1 gpurun_out/ab_$v$r.log | python3 -c 'import json,sys; r=json.loads(sys.stdin.read()); print(r["value"], "tok/s", r["ms_per_step"], "ms")')"
  done
done
