#!/bin/bash
# Round 4ac: TP8 proxy (one TP rank of Llama-2-7B TP8 + SP, seq 4096) with planned vs even SP MLP pieces, same box.
set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
for i in 1 2; do
timeout -k 10 400 python -u bench.py --proxy llama7b-tp8 --steps 6 --warmup 2 > gpurun_out/r4ac_px_planned_$i.log 2>&1 || { tail -20 gpurun_out/r4ac_px_planned_$i.log; exit 1; }
tail -1 gpurun_out/r4ac_px_planned_$i.log | cut -c1-330
EMA_SP_MLP_PIECES=1024,1024 timeout -k 10 400 python -u bench.py --proxy llama7b-tp8 --steps 6 --warmup 2 > gpurun_out/r4ac_px_even_$i.log 2>&1 || { tail -20 gpurun_out/r4ac_px_even_$i.log; exit 1; }
tail -1 gpurun_out/r4ac_px_even_$i.log | cut -c1-330
done
