#!/usr/bin/env python3
"""Timeline of one psvi_inner_loop call from a rocprofv3 kernel trace.

  rocprofv3 --kernel-trace --output-format csv -d OUT -o run -- python3 bench.py ...
  python3 tools/trace_timeline.py OUT/.../run_kernel_trace.csv [--after fill] [--n 80]

Prints, for the kernels following the last torch elementwise kernel (the
bench's params / Adam-state reset before its timed call), each kernel's start
relative to the first, its duration and the idle gap before it, so a call's
fixed cost (first sample, conversions, the last step) and any ramp over its
first steps can be read off per kernel."""
import argparse
import csv
import glob
import os


def load(path):
    if os.path.isdir(path):
        path = glob.glob(os.path.join(path, "**", "*kernel_trace.csv"), recursive=True)[0]
    rows = list(csv.DictReader(open(path)))
    ks = []
    for r in rows:
        ks.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"],
                   r.get("Queue_Id", "")))
    ks.sort()
    return ks


def short(name):
    n = name.split("(")[0]
    if n.startswith("void "):
        n = n[5:]
    return n[:70]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--after", default="elementwise",
                    help="start after the last kernel whose name contains this, before --before")
    ap.add_argument("--before", default="psvi::net_kernel",
                    help="... and which precedes the first of a run of --min-run of these")
    ap.add_argument("--n", type=int, default=90)
    ap.add_argument("--skip", type=int, default=0, help="use the (skip+1)-th marker from the end")
    args = ap.parse_args()
    ks = load(args.trace)
    marks = [i for i, k in enumerate(ks) if args.after in k[2]]
    if not marks:
        raise SystemExit(f"no kernel named *{args.after}*")
    i0 = marks[-1 - args.skip] + 1
    t0 = ks[i0][0]
    prev_end = ks[i0 - 1][1]
    tot = {}
    for k in ks[i0:i0 + args.n]:
        s, e, n, q = k
        print(f"{(s - t0) / 1e3:9.2f} us  dur {(e - s) / 1e3:8.2f}  gap {(s - prev_end) / 1e3:7.2f}  "
              f"q{q:>2} {short(n)}")
        prev_end = max(prev_end, e)
        tot[short(n)] = tot.get(short(n), 0) + (e - s)
    print("--- summed durations (us)")
    for n, d in sorted(tot.items(), key=lambda x: -x[1]):
        print(f"{d / 1e3:10.2f}  {n}")


if __name__ == "__main__":
    main()
