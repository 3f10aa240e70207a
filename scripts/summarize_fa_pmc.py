"""Per-kernel summary of rocprofv3 counter passes (FA kernels).

    python scripts/summarize_fa_pmc.py TRACE_DIR PMC_DIR [PMC_DIR ...]

Per kernel: calls, mean time, MFMA busy % (SQ_VALU_MFMA_BUSY_CYCLES over
GRBM_GUI_ACTIVE/8 x 256 CUs x 4 SIMDs), and the wave-cycle split
(SQ_WAIT_ANY parked, SQ_WAIT_INST_ANY issue-stalled, SQ_ACTIVE_INST_ANY issuing;
quad-cycle units, ratios only), LDS bank-conflict cycles per LDS instruction.
"""
import csv
import glob
import os
import sys
from collections import defaultdict


def main():
    tdir, pdirs = sys.argv[1], sys.argv[2:]
    t, n = defaultdict(float), defaultdict(int)
    for f in glob.glob(os.path.join(tdir, "**", "*kernel_trace.csv"), recursive=True):
        for row in csv.DictReader(open(f)):
            k = row["Kernel_Name"]
            t[k] += float(row["End_Timestamp"]) - float(row["Start_Timestamp"])
            n[k] += 1
    c = defaultdict(lambda: defaultdict(float))
    for d in pdirs:
        for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            for row in csv.DictReader(open(f)):
                c[row["Kernel_Name"]][row["Counter_Name"]] += float(row["Counter_Value"])
    print(f"{'kernel':60s} calls   us/call  mfma%  wait%  stall%  issue%  ldsconf/inst  valu/mfma")
    for k in sorted(t, key=lambda k: -t[k]):
        if n[k] == 0:
            continue
        cc = c.get(k, {})
        busy = cc.get("GRBM_GUI_ACTIVE", 0) / 8 * 256 * 4
        mf = 100 * cc.get("SQ_VALU_MFMA_BUSY_CYCLES", 0) / busy if busy else float("nan")
        tot = cc.get("SQ_WAIT_ANY", 0) + cc.get("SQ_WAIT_INST_ANY", 0) + cc.get("SQ_ACTIVE_INST_ANY", 0)
        w = [100 * cc.get(x, 0) / tot if tot else float("nan")
             for x in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY")]
        lds = cc.get("SQ_INSTS_LDS", 0)
        conf = cc.get("SQ_LDS_BANK_CONFLICT", 0) / lds if lds else float("nan")
        vm = cc.get("SQ_INSTS_VALU", 0) / max(cc.get("SQ_INSTS_MFMA", 0), 1)
        print(f"{k[:60]:60s} {n[k]:5d} {t[k] / n[k] / 1e3:9.1f} {mf:6.1f} {w[0]:6.1f} {w[1]:7.1f} "
              f"{w[2]:7.1f} {conf:12.3f} {vm:9.2f}")


if __name__ == "__main__":
    main()
