#!/bin/bash
# Round 4j: wgrad 4-wave persistent with spread DMA vs 8-wave ping-pong vs hipBLASLt.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k wgrad > gpurun_out/r4j_wgrad_tests.log 2>&1 || { tail -30 gpurun_out/r4j_wgrad_tests.log; exit 1; }
tail -2 gpurun_out/r4j_wgrad_tests.log
timeout -k 10 300 python -u scripts/wgrad_bench.py --variants 2>&1 | tee gpurun_out/r4j_wgrad_variants.txt || exit 1
for mb in "16 8" "32 4"; do
  set -- $mb
  timeout -k 10 500 python -u bench.py --steps 6 --warmup 2 --micro_batch $1 --num_micro $2 > gpurun_out/r4j_bench_mbs$1.log 2>&1 || { tail -20 gpurun_out/r4j_bench_mbs$1.log; exit 1; }
  tail -1 gpurun_out/r4j_bench_mbs$1.log | python3 -c "import json,sys; r=json.loads(sys.stdin.read()); print('mbs', r['config']['micro_batch'], 'x', r['config']['num_micro_batches'], r['value'], 'tok/s', r['ms_per_step'], 'ms', 'mem', r['max_mem_gb'])"
done
