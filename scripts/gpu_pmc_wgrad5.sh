#!/bin/bash
# PMC passes over the wgrad kernel (fc1 shape), full and no-load ablation.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
for MODE in 50; do
timeout -s KILL 120 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/pmcwg${MODE}_t -o w -- python3 scripts/wgrad_once.py 22016 4096 $MODE > gpurun_out/pmcwg_t.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS --kernel-trace --output-format csv -d gpurun_out/pmcwg${MODE}_1 -o w -- python3 scripts/wgrad_once.py 22016 4096 $MODE > gpurun_out/pmcwg_1.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc SQ_WAIT_INST_LDS SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_SALU SQ_ACTIVE_INST_LDS --kernel-trace --output-format csv -d gpurun_out/pmcwg${MODE}_2 -o w -- python3 scripts/wgrad_once.py 22016 4096 $MODE > gpurun_out/pmcwg_2.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d gpurun_out/pmcwg${MODE}_3 -o w -- python3 scripts/wgrad_once.py 22016 4096 $MODE > gpurun_out/pmcwg_3.log 2>&1 || exit 1
echo "mode $MODE"; python3 scripts/summarize_fa_pmc.py gpurun_out/pmcwg${MODE}_t gpurun_out/pmcwg${MODE}_1 gpurun_out/pmcwg${MODE}_2
python3 - $MODE <<'PY'
import csv, glob, sys, collections
c = collections.defaultdict(float)
for f in glob.glob(f"gpurun_out/pmcwg{sys.argv[1]}_3/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "wgrad" in r["Kernel_Name"]:
            c[r["Counter_Name"]] += float(r["Counter_Value"])
h, m = c["TCC_HIT_sum"], c["TCC_MISS_sum"]
print(f"L2 hit {100*h/max(h+m,1):.1f}%  misses {m:.3g}  read_req {c['TCP_TCC_READ_REQ_sum']:.3g}")
PY
done
