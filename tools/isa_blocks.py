#!/usr/bin/env python3
"""Instruction mix of one kernel in a hipcc --save-temps .s file: per basic
block (label) counts of MFMA, other VALU, SALU, LDS, global/buffer memory and
waitcnt instructions; blocks ending in a backward branch are marked LOOP.

  python tools/isa_blocks.py build/asm/kernels_mvn-hip-amdgcn-amd-amdhsa-gfx950.s <kernel substring> [min_insts]
"""
import re
import sys


def classify(op):
    if op.startswith("v_mfma"):
        return "mfma"
    if op.startswith(("v_", )):
        return "valu"
    if op.startswith("s_waitcnt"):
        return "wait"
    if op.startswith("s_"):
        return "salu"
    if op.startswith("ds_"):
        return "lds"
    if op.startswith(("global_", "buffer_", "flat_", "scratch_")):
        return "vmem"
    return "other"


def main():
    path, sub = sys.argv[1], sys.argv[2]
    mn = int(sys.argv[3]) if len(sys.argv) > 3 else 20
    lines = open(path).read().split("\n")
    start = None
    for i, l in enumerate(lines):
        if re.match(r"^_Z\S*:", l) and sub in l:
            start = i
            break
    if start is None:
        sys.exit("kernel not found")
    name = lines[start][:-1]
    blocks, cur, order = {}, "entry", ["entry"]
    blocks[cur] = {"n": 0}
    tot = {}
    for l in lines[start + 1:]:
        if l.startswith("\t.size") or re.match(r"^\s*s_endpgm", l) and False:
            break
        m = re.match(r"^(\.LBB\S+):", l)
        if m:
            cur = m.group(1)
            blocks[cur] = {"n": 0}
            order.append(cur)
            continue
        t = l.strip()
        if not t or t.startswith((";", ".")):
            continue
        op = t.split()[0]
        c = classify(op)
        b = blocks[cur]
        b[c] = b.get(c, 0) + 1
        b["n"] += 1
        tot[c] = tot.get(c, 0) + 1
        if op.startswith("s_cbranch") or op == "s_branch":
            tgt = t.split()[-1]
            if tgt in blocks and tgt != cur or tgt == cur:
                b["loop"] = tgt
        if op == "s_endpgm":
            pass
    print(name)
    print("total", tot)
    for k in order:
        b = blocks[k]
        if b["n"] < mn:
            continue
        loop = f" LOOP->{b['loop']}" if "loop" in b else ""
        desc = " ".join(f"{c}={b.get(c, 0)}" for c in ("mfma", "valu", "salu", "lds", "vmem", "wait"))
        print(f"{k:14s} n={b['n']:5d} {desc}{loop}")


if __name__ == "__main__":
    main()
