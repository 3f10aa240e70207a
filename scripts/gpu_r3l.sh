#!/bin/bash
# Round 3l: persistent FA forward (K/V ring across block seams, next-block Q
# loads after the last QK^T, deferred O stores): FA tests, A/B, stamps.
set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider \
  tests/test_kernels_gpu.py tests/test_gpu_e2e.py -m gpu -k "flash or rope or deterministic or document" \
  > gpurun_out/r3l_tests.log 2>&1 || { tail -40 gpurun_out/r3l_tests.log; exit 1; }
tail -1 gpurun_out/r3l_tests.log
EMA_FA_PERSIST=0 timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider \
  tests/test_kernels_gpu.py -m gpu -k "flash_attention" > gpurun_out/r3l_tests_np.log 2>&1 || { tail -40 gpurun_out/r3l_tests_np.log; exit 1; }
tail -1 gpurun_out/r3l_tests_np.log
for r in 1 2; do for ps in 1 0; do
  EMA_FA_PERSIST=$ps timeout -k 10 300 python scripts/fa_bench2.py 16,1024,32,32,128 4,4096,32,32,128 8,2048,32,2,64 2,4096,8,1,128 > gpurun_out/r3l_fa_p$ps.log 2>&1 || { tail -20 gpurun_out/r3l_fa_p$ps.log; exit 1; }
  echo "persist=$ps round $r"; grep shape gpurun_out/r3l_fa_p$ps.log
done; done
timeout -k 10 200 python -u scripts/fa_stamps.py --json gpurun_out/r3l_fa_stamps.json > gpurun_out/r3l_fa_stamps.log 2>&1 || { tail -20 gpurun_out/r3l_fa_stamps.log; exit 1; }
grep '^{' gpurun_out/r3l_fa_stamps.log
timeout -k 10 300 python -u scripts/fa_diag.py > gpurun_out/r3l_fa_diag.log 2>&1 || { tail -20 gpurun_out/r3l_fa_diag.log; exit 1; }
grep "^b=" gpurun_out/r3l_fa_diag.log
