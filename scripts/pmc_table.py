"""Per-kernel averages of every rocprofv3 --pmc counter (one pass per dir).

    python scripts/pmc_table.py DIR [DIR ...]

Prints, per kernel (name truncated), the dispatch count and each counter's
mean per dispatch, then derived ratios where the counters are present:
  busy   = SQ_BUSY_CYCLES / GRBM_GUI_ACTIVE
  wait%  = SQ_WAIT_ANY / SQ_WAVE_CYCLES, stall% = SQ_WAIT_INST_ANY / SQ_WAVE_CYCLES,
  active% = SQ_ACTIVE_INST_ANY / SQ_WAVE_CYCLES (these three partition wave time),
  mfma%  = SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 x 1024 SIMDs),
  conf   = SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE, L2hit = TCC_HIT / (HIT + MISS),
  us     = mean dispatch duration (Start/End_Timestamp), GHz = GRBM_GUI_ACTIVE / 8 XCDs / us.
"""
import csv
import glob
import os
import sys
from collections import defaultdict


def main():
    vals = defaultdict(lambda: defaultdict(list))
    durs = defaultdict(list)
    for d in sys.argv[1:]:
        for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            per = defaultdict(float)  # (kernel, dispatch, counter) -> summed over dimensions
            span = {}
            with open(f) as fh:
                for row in csv.DictReader(fh):
                    key = (row["Kernel_Name"][:60], row.get("Dispatch_Id", "0"))
                    per[key + (row["Counter_Name"],)] += float(row["Counter_Value"])
                    if row.get("Start_Timestamp") and row.get("End_Timestamp"):
                        span[key] = int(row["End_Timestamp"]) - int(row["Start_Timestamp"])
            for (k, _, c), v in per.items():
                vals[k][c].append(v)
            for (k, _), ns in span.items():
                durs[k].append(ns)
    for k, cs in vals.items():
        mean = {c: sum(v) / len(v) for c, v in cs.items()}
        n = max(len(v) for v in cs.values())
        print(f"{k}  (dispatches {n})")
        print("   " + "  ".join(f"{c}={mean[c]:.4g}" for c in sorted(mean)))
        d = []
        g = mean.get("GRBM_GUI_ACTIVE")
        wc = mean.get("SQ_WAVE_CYCLES")
        if g and "SQ_BUSY_CYCLES" in mean:
            d.append(f"busy={mean['SQ_BUSY_CYCLES'] / g:.3f}")
        if wc:
            for c, lab in (("SQ_WAIT_ANY", "wait"), ("SQ_WAIT_INST_ANY", "stall"),
                           ("SQ_ACTIVE_INST_ANY", "active"), ("SQ_WAIT_INST_LDS", "ldsstall")):
                if c in mean:
                    d.append(f"{lab}%={100 * mean[c] / wc:.1f}")
        if g and "SQ_VALU_MFMA_BUSY_CYCLES" in mean:
            d.append(f"mfma%={100 * mean['SQ_VALU_MFMA_BUSY_CYCLES'] / (g / 8 * 1024):.1f}")
        if "SQ_LDS_IDX_ACTIVE" in mean and mean["SQ_LDS_IDX_ACTIVE"]:
            d.append(f"conf={mean.get('SQ_LDS_BANK_CONFLICT', 0) / mean['SQ_LDS_IDX_ACTIVE']:.3f}")
        if "TCC_HIT_sum" in mean:
            h, m = mean["TCC_HIT_sum"], mean.get("TCC_MISS_sum", 0)
            d.append(f"L2hit={100 * h / max(h + m, 1):.1f}%")
        if durs.get(k):
            us = sum(durs[k]) / len(durs[k]) / 1e3
            d.append(f"us={us:.1f}")
            if g:
                d.append(f"GHz={g / 8 / (us * 1e3):.2f}")
        if d:
            print("   -> " + "  ".join(d))


if __name__ == "__main__":
    main()
