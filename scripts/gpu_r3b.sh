#!/bin/bash
# PMC passes: hipBLASLt vs the two NT GEMM variants on the fc2 forward shape.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
S="16384 4096 11008"
timeout -s KILL 120 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/pmcnt_t -o w -- python3 scripts/gemm_nt_once.py $S > gpurun_out/pmcnt_t.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS --kernel-trace --output-format csv -d gpurun_out/pmcnt_1 -o w -- python3 scripts/gemm_nt_once.py $S > gpurun_out/pmcnt_1.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc SQ_WAIT_INST_LDS SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_SALU SQ_ACTIVE_INST_LDS --kernel-trace --output-format csv -d gpurun_out/pmcnt_2 -o w -- python3 scripts/gemm_nt_once.py $S > gpurun_out/pmcnt_2.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d gpurun_out/pmcnt_3 -o w -- python3 scripts/gemm_nt_once.py $S > gpurun_out/pmcnt_3.log 2>&1 || exit 1
python3 scripts/summarize_fa_pmc.py gpurun_out/pmcnt_t gpurun_out/pmcnt_1 gpurun_out/pmcnt_2 gpurun_out/pmcnt_3
python3 - <<'PY'
import csv, glob, collections
c = collections.defaultdict(lambda: collections.defaultdict(float))
t = collections.defaultdict(float); n = collections.defaultdict(int)
for f in glob.glob("gpurun_out/pmcnt_3/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        c[r["Kernel_Name"]][r["Counter_Name"]] += float(r["Counter_Value"])
for f in glob.glob("gpurun_out/pmcnt_t/**/*kernel_trace.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        t[r["Kernel_Name"]] += float(r["End_Timestamp"]) - float(r["Start_Timestamp"]); n[r["Kernel_Name"]] += 1
for k, cc in c.items():
    h, m = cc["TCC_HIT_sum"], cc["TCC_MISS_sum"]
    clk = cc["GRBM_GUI_ACTIVE"] / 8 / max(t.get(k, 0), 1) if t.get(k) else float("nan")
    print(f"{k[:70]:70s} L2 hit {100*h/max(h+m,1):.1f}%  clock~{clk:.2f} GHz (GUI_ACTIVE/8 / traced ns)")
PY
