#!/usr/bin/env python3
"""Run pytest with libpsvi_hip debug switches set for the whole process (A/B of
a kernel variant under an existing test):
  python3 tools/ab_pytest.py KEY=VALUE[,KEY=VALUE...] -- <pytest args>"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "blackbox-coresets-vi_amd"))


def main():
    spec, rest = sys.argv[1], sys.argv[sys.argv.index("--") + 1:]
    from psvi.runtime import _lib
    lib = _lib.load()
    for kv in spec.split(","):
        if kv:
            k, v = kv.split("=")
            if lib.psvi_debug_set(int(k), int(v)):
                raise SystemExit(f"psvi_debug_set({k}, {v}) failed")
    import pytest
    raise SystemExit(pytest.main(rest))


if __name__ == "__main__":
    main()
