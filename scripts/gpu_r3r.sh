#!/bin/bash
# Round 3r: software-pipelined FA forward (EMA_FA_PIPE=1): tests + same-box A/B.
set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
EMA_FA_PIPE=1 EMA_FA_WAVES=8 timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider \
  tests/test_kernels_gpu.py -m gpu -k "flash_attention" > gpurun_out/r3r_tests.log 2>&1 || { tail -40 gpurun_out/r3r_tests.log; exit 1; }
tail -1 gpurun_out/r3r_tests.log
for r in 1 2; do for pp in 1 0; do
  EMA_FA_PIPE=$pp timeout -k 10 300 python scripts/fa_bench2.py 16,1024,32,32,128 4,4096,32,32,128 2,4096,8,1,128 > gpurun_out/r3r_fa_p$pp.log 2>&1 || { tail -20 gpurun_out/r3r_fa_p$pp.log; exit 1; }
  echo "pipe=$pp round $r"; grep shape gpurun_out/r3r_fa_p$pp.log
done; done
