#!/bin/bash
# Round-2 (session 2) health check on a fresh box: GPU tests, smoke, 1-GPU bench,
# then an RCCL rehearsal (2 ranks sharing cuda:0) of the collectives and the
# DP + dist-opt bench path.  Every GPU step is time-limited; failures stop the run.
set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
  -p no:cacheprovider > gpurun_out/gputests.log 2>&1
rc=$?; echo "gpu tests rc=$rc"; tail -3 gpurun_out/gputests.log
[ $rc -eq 0 ] || { grep -E "Error|assert|FAILED" gpurun_out/gputests.log | head -20; exit $rc; }
timeout -k 10 300 python __graft_entry__.py smoke > gpurun_out/smoke.log 2>&1 || { tail -30 gpurun_out/smoke.log; exit 1; }
grep smoke gpurun_out/smoke.log
timeout -k 10 600 python bench.py --steps 8 --warmup 3 > gpurun_out/bench_7b.log 2>&1 || { tail -30 gpurun_out/bench_7b.log; exit 1; }
tail -1 gpurun_out/bench_7b.log
timeout -k 10 120 python scripts/rccl_probe.py 2 > gpurun_out/rccl_probe.log 2>&1
rc=$?; echo "rccl probe rc=$rc"; tail -5 gpurun_out/rccl_probe.log
[ $rc -eq 0 ] || exit 0
timeout -k 10 300 python bench.py --gpus 2 --model tiny --seq_len 256 --micro_batch 4 --num_micro 2 \
  --steps 4 --warmup 2 > gpurun_out/bench_tiny_g2.log 2>&1
echo "tiny g2 rc=$?"; tail -2 gpurun_out/bench_tiny_g2.log
