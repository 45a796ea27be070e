#!/usr/bin/env python3
"""Summarise gpurun_out/pmc: mean kernel duration + per-dispatch counter means."""
import csv
import glob
import os
import sys
from collections import defaultdict

root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmc"
stats = glob.glob(os.path.join(root, "trace", "**", "*kernel_stats.csv"), recursive=True)
for f in stats:
    print("== kernel stats", f)
    for r in csv.DictReader(open(f)):
        print(f"  {r['Name'][:60]:60s} calls={r['Calls']:>5s} avg_us={float(r['AverageNs'])/1e3:9.2f} {float(r['Percentage']):6.2f}%")
agg = defaultdict(lambda: defaultdict(list))
for f in glob.glob(os.path.join(root, "p*", "**", "*counter_collection.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        agg[r["Kernel_Name"][:50]][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, d in agg.items():
    print("==", k)
    for c, v in sorted(d.items()):
        print(f"  {c:28s} {sum(v)/len(v):16.1f}  (n={len(v)})")
