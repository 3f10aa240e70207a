"""Condense a rocprofv3 kernel_stats.csv into a short, committed summary."""
import csv
import sys


def main(src, dst, title):
    rows = list(csv.DictReader(open(src)))
    tot = sum(float(r["TotalDurationNs"]) for r in rows)
    rows.sort(key=lambda r: -float(r["TotalDurationNs"]))
    with open(dst, "w") as f:
        f.write(f"# {title}\n# total kernel time {tot / 1e6:.1f} ms\n")
        f.write("ms_total,pct,calls,avg_us,kernel\n")
        for r in rows[:40]:
            t = float(r["TotalDurationNs"])
            f.write(f"{t / 1e6:.1f},{100 * t / tot:.2f},{r['Calls']},"
                    f"{float(r['AverageNs']) / 1e3:.1f},{r['Name'][:160].replace(',', ';')}\n")


if __name__ == "__main__":
    main(*sys.argv[1:4])
