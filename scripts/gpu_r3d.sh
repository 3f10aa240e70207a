#!/bin/bash
# Round 3d: fused MLP with hipBLASLt plain GEMMs vs unfused (A/B, alternating),
# SP piece-GEMM overhead, PMC: NT GEMM vs hipBLASLt (fc2 fwd shape) and FA fwd (s=1k).
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py tests/test_gpu_e2e.py -k "wgrad or skinny or decode or graph" > gpurun_out/r3d_wgrad_tests.log 2>&1 || { tail -30 gpurun_out/r3d_wgrad_tests.log; exit 1; }
tail -2 gpurun_out/r3d_wgrad_tests.log
for i in 1 2; do
timeout -k 10 400 python -u bench.py --steps 6 --warmup 2 > gpurun_out/r3d_bench_fused$i.log 2>&1 || { tail -20 gpurun_out/r3d_bench_fused$i.log; exit 1; }
tail -1 gpurun_out/r3d_bench_fused$i.log | cut -c1-400
EMA_FUSED_MLP=0 timeout -k 10 400 python -u bench.py --steps 6 --warmup 2 > gpurun_out/r3d_bench_unfused$i.log 2>&1 || { tail -20 gpurun_out/r3d_bench_unfused$i.log; exit 1; }
tail -1 gpurun_out/r3d_bench_unfused$i.log | cut -c1-400
done
timeout -k 10 200 python -u scripts/sp_overlap_bench.py --json gpurun_out/r3d_sp_pieces.json > gpurun_out/r3d_sp_pieces.txt 2>&1 || { tail -20 gpurun_out/r3d_sp_pieces.txt; exit 1; }
cat gpurun_out/r3d_sp_pieces.txt
bash scripts/gpu_r3b.sh > gpurun_out/r3d_pmc_gemm.txt 2>&1 || { tail -20 gpurun_out/r3d_pmc_gemm.txt; exit 1; }
cat gpurun_out/r3d_pmc_gemm.txt
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -s KILL 120 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/pmfa_t -o w -- python3 scripts/fa_once.py > gpurun_out/pmfa_t.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS --kernel-trace --output-format csv -d gpurun_out/pmfa_1 -o w -- python3 scripts/fa_once.py > gpurun_out/pmfa_1.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc SQ_WAIT_INST_LDS SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_SALU SQ_ACTIVE_INST_LDS --kernel-trace --output-format csv -d gpurun_out/pmfa_2 -o w -- python3 scripts/fa_once.py > gpurun_out/pmfa_2.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d gpurun_out/pmfa_3 -o w -- python3 scripts/fa_once.py > gpurun_out/pmfa_3.log 2>&1 || exit 1
python3 scripts/summarize_fa_pmc.py gpurun_out/pmfa_t gpurun_out/pmfa_1 gpurun_out/pmfa_2 gpurun_out/pmfa_3
python3 - <<'PY'
import csv, glob, collections
c = collections.defaultdict(lambda: collections.defaultdict(float))
for f in glob.glob("gpurun_out/pmfa_3/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        c[r["Kernel_Name"]][r["Counter_Name"]] += float(r["Counter_Value"])
for k, cc in c.items():
    h, m = cc["TCC_HIT_sum"], cc["TCC_MISS_sum"]
    print(f"{k[:70]:70s} L2 hit {100*h/max(h+m,1):.1f}%  misses {m:.3e} (x128B = {m*128/1e6:.0f} MB over 5 calls)")
PY
