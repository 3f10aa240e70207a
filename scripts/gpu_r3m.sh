#!/bin/bash
# Round 3m: staggered FA forward (waves 4-7 one barrier behind): tests, A/B vs lockstep.
set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider \
  tests/test_kernels_gpu.py tests/test_gpu_e2e.py -m gpu -k "flash or rope or deterministic or document" \
  > gpurun_out/r3m_tests.log 2>&1 || { tail -40 gpurun_out/r3m_tests.log; exit 1; }
tail -1 gpurun_out/r3m_tests.log
for r in 1 2; do for st in 1 0; do
  EMA_FA_STAGGER=$st timeout -k 10 300 python scripts/fa_bench2.py 16,1024,32,32,128 4,4096,32,32,128 2,4096,8,1,128 > gpurun_out/r3m_fa_s$st.log 2>&1 || { tail -20 gpurun_out/r3m_fa_s$st.log; exit 1; }
  echo "stagger=$st round $r"; grep shape gpurun_out/r3m_fa_s$st.log
done; done
timeout -k 10 300 python -u scripts/fa_diag.py > gpurun_out/r3m_fa_diag.log 2>&1 || { tail -20 gpurun_out/r3m_fa_diag.log; exit 1; }
grep "^b=" gpurun_out/r3m_fa_diag.log
