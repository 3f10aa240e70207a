#!/bin/bash
# Same-box A/B: norm weight grads fused into main_grad (1) vs autograd bf16 grads (0).
set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
for rep in 1 2; do
for f in 1 0; do
  EMA_NORM_MAIN_GRAD=$f timeout -k 10 600 python bench.py --proxy llama7b-tp8 --steps 4 --warmup 2 > gpurun_out/px_$f.log 2>&1 || { tail -20 gpurun_out/px_$f.log; exit 1; }
  echo "fuse=$f $(tail -1 gpurun_out/px_$f.log | python3 -c 'import json,sys; r=json.loads(sys.stdin.read()); print(r["value"], r["ms_per_step"])')"
done
done
for f in 1 0; do
  EMA_NORM_MAIN_GRAD=$f timeout -k 10 600 python bench.py --num_micro 2 --steps 8 --warmup 3 > gpurun_out/b7_$f.log 2>&1 || { tail -20 gpurun_out/b7_$f.log; exit 1; }
  echo "7B fuse=$f $(tail -1 gpurun_out/b7_$f.log | python3 -c 'import json,sys; r=json.loads(sys.stdin.read()); print(r["value"], r["ms_per_step"])')"
done
