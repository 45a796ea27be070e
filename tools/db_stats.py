#!/usr/bin/env python3
"""Per-kernel stats (calls, average / min / max duration in us, total share)
from a rocprofv3 results database (rocpd sqlite; what --stats prints, for runs
whose output is the .db), optionally written as CSV.

  python tools/db_stats.py gpurun_out/prof_b/b_results.db [out.csv]
"""
import csv
import sqlite3
import sys


def stats(db):
    c = sqlite3.connect(db)
    rows = c.execute(
        "select s.kernel_name, d.end - d.start from rocpd_kernel_dispatch d "
        "join rocpd_info_kernel_symbol s on d.kernel_id = s.id").fetchall()
    agg = {}
    for name, dur in rows:
        agg.setdefault(name, []).append(dur)
    tot = sum(sum(v) for v in agg.values()) or 1
    out = []
    for name, v in sorted(agg.items(), key=lambda kv: -sum(kv[1])):
        out.append((name, len(v), sum(v) / len(v) / 1e3, min(v) / 1e3, max(v) / 1e3, 100.0 * sum(v) / tot))
    return out


def main():
    res = stats(sys.argv[1])
    if len(sys.argv) > 2:
        with open(sys.argv[2], "w", newline="") as f:
            w = csv.writer(f)
            w.writerow(["Name", "Calls", "AverageNs", "MinNs", "MaxNs", "Percentage"])
            for n, k, a, lo, hi, p in res:
                w.writerow([n, k, round(a * 1e3, 1), round(lo * 1e3, 1), round(hi * 1e3, 1), round(p, 3)])
    for n, k, a, lo, hi, p in res[:25]:
        print(f"{p:6.2f}%  {k:7d}  avg {a:9.2f} us  min {lo:8.2f}  max {hi:8.2f}  {n[:110]}")


if __name__ == "__main__":
    main()
