"""Per-kernel PMC summary of rocprofv3 --pmc passes (each DIR one pass with
--kernel-trace): mean us/call, clock (GRBM_GUI_ACTIVE / 8 XCDs / duration),
MFMA busy % of SIMD-cycles, wait share, LDS conflicts, L2 hit rate.

    python scripts/summarize_ablation_pmc.py DIR [DIR ...]"""
import csv
import glob
import os
import sys
from collections import defaultdict

cnt = defaultdict(lambda: defaultdict(float))
dur = defaultdict(lambda: defaultdict(float))
calls = defaultdict(int)
for d in sys.argv[1:]:
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        seen = set()
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"][:60]
            cnt[k][r["Counter_Name"]] += float(r["Counter_Value"])
            did = (r.get("Dispatch_Id"), k)
            if did not in seen:
                seen.add(did)
                dur[k][d] += float(r.get("End_Timestamp", 0) or 0) - float(r.get("Start_Timestamp", 0) or 0)
                if d == sys.argv[1]:
                    calls[k] += 1
print(f"{'kernel':60s} {'calls':>5s} {'us/call':>8s} {'GHz':>5s} {'mfma%':>6s} {'wait%':>6s} "
      f"{'ldswait%':>8s} {'ldsconf':>7s} {'L2hit%':>6s}")
for k, c in cnt.items():
    n = max(calls[k], 1)
    t1 = dur[k].get(sys.argv[1], 0.0)
    gui = c.get("GRBM_GUI_ACTIVE", 0.0)
    ghz = gui / 8 / t1 if t1 else 0.0
    simd_cycles = gui / 8 * 256 * 4
    mfma = 100 * c.get("SQ_VALU_MFMA_BUSY_CYCLES", 0.0) / simd_cycles if simd_cycles else 0.0
    wc = c.get("SQ_WAVE_CYCLES", 0.0)
    wait = 100 * c.get("SQ_WAIT_ANY", 0.0) / wc if wc else 0.0
    lw = 100 * c.get("SQ_WAIT_INST_LDS", 0.0) / wc if wc else 0.0
    lds = c.get("SQ_INSTS_LDS", 0.0)
    conf = c.get("SQ_LDS_BANK_CONFLICT", 0.0) / lds if lds else 0.0
    h, m = c.get("TCC_HIT_sum", 0.0), c.get("TCC_MISS_sum", 0.0)
    l2 = 100 * h / (h + m) if h + m else 0.0
    print(f"{k:60s} {n:5d} {t1 / n / 1e3:8.1f} {ghz:5.2f} {mfma:6.1f} {wait:6.1f} {lw:8.1f} "
          f"{conf:7.3f} {l2:6.1f}")
