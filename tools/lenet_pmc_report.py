#!/usr/bin/env python3
"""Per-kernel summary of a rocprofv3 --pmc counter collection of the LeNet
probe (tools/round_session.sh lpmc step): mean counter values per dispatch,
and for the psvi kernels the MFMA busy share (SQ_VALU_MFMA_BUSY_CYCLES /
(GRBM_GUI_ACTIVE / 8 x CUs x 4 SIMDs): rocprofv3 sums GRBM_GUI_ACTIVE over the
8 XCDs, MI355X_MICROARCH.md) and VALU / LDS instructions per MFMA.

  python tools/lenet_pmc_report.py <lenet_counter_collection.csv> [--cus 256]
"""
import argparse
import collections
import csv
import re


def short(name):
    name = name.replace("(anonymous namespace)::", "").replace("void ", "")
    return re.sub(r"\(.*", "", name)[:60]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("--cus", type=int, default=256)
    a = ap.parse_args()
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    disp = collections.defaultdict(set)
    for r in csv.DictReader(open(a.csv)):
        k = short(r["Kernel_Name"])
        acc[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
        disp[k].add(r["Dispatch_Id"])
    for k in sorted(acc, key=lambda k: -sum(acc[k].get("GRBM_GUI_ACTIVE", [0]))):
        c = {n: sum(v) / len(v) for n, v in acc[k].items()}
        line = f"{k:60s} dispatches={len(disp[k]):4d}"
        for n in sorted(c):
            line += f" {n}={c[n]:.4g}"
        busy, gui = c.get("SQ_VALU_MFMA_BUSY_CYCLES"), c.get("GRBM_GUI_ACTIVE")
        if busy and gui:
            line += f"  mfma_busy={busy / (gui / 8 * a.cus * 4):.3f}"
        if c.get("SQ_INSTS_MFMA"):
            line += (f"  valu/mfma={c.get('SQ_INSTS_VALU', 0) / c['SQ_INSTS_MFMA']:.2f}"
                     f" lds/mfma={c.get('SQ_INSTS_LDS', 0) / c['SQ_INSTS_MFMA']:.2f}")
        print(line)


if __name__ == "__main__":
    main()
