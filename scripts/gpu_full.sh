#!/bin/bash
# Whole GPU suite (one pytest process), smoke, then the round evidence benches + step profile.
set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/gpu_all.log 2>&1
rc=$?; echo "gpu tests rc=$rc"; tail -3 gpurun_out/gpu_all.log
[ $rc -eq 0 ] || { grep -E "Error|assert|FAILED" gpurun_out/gpu_all.log | head -20; exit $rc; }
timeout -k 10 300 python __graft_entry__.py smoke > gpurun_out/smoke.log 2>&1 || { tail -30 gpurun_out/smoke.log; exit 1; }
tail -2 gpurun_out/smoke.log
bash scripts/gpu_r2_evidence.sh
