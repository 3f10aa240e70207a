"""Aggregate rocprofv3 --pmc counter CSVs per kernel and derive utilisation.

    python scripts/summarize_pmc.py OUT.csv DIR [DIR ...]

Columns: kernel, dispatches, total GPU time (ms, from the kernel trace), and
derived metrics: MFMA busy % = SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 XCDs
x 256 CUs x 4 SIMDs) — GRBM_GUI_ACTIVE is summed over the 8 XCDs and the MFMA
busy counter over every SIMD (checked: ~2.1 GRBM cycles/ns per XCD), LDS bank-conflict cycles per LDS instruction, HBM
bytes (FETCH_SIZE + WRITE_SIZE, KiB counters) and achieved GB/s.
"""
import csv
import glob
import os
import sys
from collections import defaultdict


def _short(name, n=90):
    return name.replace(",", ";")[:n]


def main():
    out, dirs = sys.argv[1], sys.argv[2:]
    counters = defaultdict(lambda: defaultdict(float))
    time_ns, calls = defaultdict(float), defaultdict(int)
    seen = set()  # a counter collected in several passes is taken from the first one
    for d in dirs:
        here = set()
        for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            with open(f) as fh:
                for row in csv.DictReader(fh):
                    if row["Counter_Name"] in seen:
                        continue
                    here.add(row["Counter_Name"])
                    counters[row["Kernel_Name"]][row["Counter_Name"]] += float(row["Counter_Value"])
        seen |= here
        if d.endswith("_sq"):
            for f in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
                with open(f) as fh:
                    for row in csv.DictReader(fh):
                        k = row["Kernel_Name"]
                        time_ns[k] += float(row["End_Timestamp"]) - float(row["Start_Timestamp"])
                        calls[k] += 1
    total = sum(time_ns.values()) or 1.0
    rows = []
    for k, c in counters.items():
        t = time_ns.get(k, 0.0)
        busy = c.get("GRBM_GUI_ACTIVE", 0.0) / 8 * 256 * 4
        mfma = c.get("SQ_VALU_MFMA_BUSY_CYCLES", 0.0)
        lds = c.get("SQ_INSTS_LDS", 0.0)
        hbm = (c.get("FETCH_SIZE", 0.0) + c.get("WRITE_SIZE", 0.0)) * 1024.0
        rows.append([_short(k), calls.get(k, 0), round(t / 1e6, 3), round(100 * t / total, 2),
                     round(100 * mfma / busy, 1) if busy else "",
                     round(c.get("SQ_LDS_BANK_CONFLICT", 0.0) / lds, 3) if lds else "",
                     round(hbm / 1e9, 3), round(hbm / t, 1) if t else ""])
    rows.sort(key=lambda r: -r[2])
    with open(out, "w", newline="") as fh:
        fh.write("# rocprofv3 --pmc over bench.py --steps 1 --warmup 1 (Llama-2-7B, mbs 16 x 2, seq 1024)\n")
        w = csv.writer(fh)
        w.writerow(["kernel", "calls", "ms", "pct_time", "mfma_busy_pct", "lds_conflict_per_lds_inst",
                    "hbm_GB", "hbm_GBps"])
        w.writerows(rows)


if __name__ == "__main__":
    main()
