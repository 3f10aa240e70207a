#!/bin/bash
# Kernel tests, norm timing, and LDS-conflict PMC pass over the norm kernels.
set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/kt.log 2>&1
rc=$?; tail -2 gpurun_out/kt.log; [ $rc -eq 0 ] || { grep -E "Error|assert" gpurun_out/kt.log | head; exit $rc; }
timeout -k 10 120 python scripts/norm_bench.py > gpurun_out/norm.log 2>&1 && cat gpurun_out/norm.log
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_WAVES SQ_WAVE_CYCLES --kernel-trace --output-format csv -d gpurun_out/pmcnorm -o n -- python3 scripts/norm_bench.py > gpurun_out/pmcnorm.log 2>&1; echo "pmc rc=$?"
python3 - <<'PY'
import csv, glob, collections
c = collections.defaultdict(lambda: collections.defaultdict(float))
for f in glob.glob("gpurun_out/pmcnorm/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        c[r["Kernel_Name"]][r["Counter_Name"]] += float(r["Counter_Value"])
for k, v in c.items():
    if "norm" in k:
        print(k[:70], "lds conflicts/inst = %.3f" % (v["SQ_LDS_BANK_CONFLICT"] / max(v["SQ_INSTS_LDS"], 1)))
PY
