#!/bin/bash
# FA kernel change check: FA/rope GPU tests, FA timing, 7B bench at seq 4096.
set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_gpu_e2e.py -m gpu -x -q -k "flash or rope or deterministic or e2e or llama or falcon" \
  --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/fa_tests.log 2>&1
rc=$?; echo "fa tests rc=$rc"; tail -2 gpurun_out/fa_tests.log
[ $rc -eq 0 ] || { grep -E "Error|assert|FAILED" gpurun_out/fa_tests.log | head -20; exit $rc; }
timeout -k 10 200 python scripts/fa_bench2.py 16,1024,32,32,128 4,4096,32,32,128 8,2048,32,2,64 2,4096,8,1,128 4,4096,4,4,128 > gpurun_out/fa_bench.log 2>&1 || { tail -20 gpurun_out/fa_bench.log; exit 1; }
grep shape gpurun_out/fa_bench.log
timeout -k 10 600 python bench.py --steps 6 --warmup 2 --seq_len 4096 --micro_batch 4 --num_micro 8 > gpurun_out/b7_s4k.log 2>&1 || { tail -30 gpurun_out/b7_s4k.log; exit 1; }
tail -1 gpurun_out/b7_s4k.log
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/profpx -o s -- python3 bench.py --proxy llama7b-tp8 --steps 2 --warmup 1 > gpurun_out/profpx.log 2>&1; echo "prof rc=$?"
