#!/bin/bash
# Serving benchmark (KV-cached decode) + kernel stats of the decode loop.
set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 600 python scripts/serve_bench.py --batches 1,8,32 > gpurun_out/serve.log 2>&1 || { tail -30 gpurun_out/serve.log; exit 1; }
grep batch gpurun_out/serve.log
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/profserve -o s -- python3 scripts/serve_bench.py --batches 8 > gpurun_out/profserve.log 2>&1; echo "prof rc=$?"
