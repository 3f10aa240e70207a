#!/bin/bash
# In-model A/B of the wgrad backend on the 7B bench (same box, back to back), then a
# kernel-stats profile of the step with the hand-written kernel.
set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
for W in hip hipblaslt hip; do
  EMA_WGRAD=$W timeout -k 10 600 python bench.py --steps 6 --warmup 2 > gpurun_out/ab_$W.log 2>&1 || { tail -20 gpurun_out/ab_$W.log; exit 1; }
  echo "EMA_WGRAD=$W $(tail -1 gpurun_out/ab_$W.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["mfu"], d["final_loss"])')"
done
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
EMA_WGRAD=hip timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof7b_wg -o s -- python3 bench.py --steps 2 --warmup 1 > gpurun_out/prof7b_wg.log 2>&1; echo "prof rc=$?"
