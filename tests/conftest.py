import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "blackbox-coresets-vi_amd")
for p in (PKG, os.path.join(ROOT, "oracle"), ROOT):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device)")


def pytest_collection_modifyitems(config, items):
    try:
        import torch
        have_gpu = torch.cuda.is_available()
    except Exception:  # pragma: no cover
        have_gpu = False
    if have_gpu:
        return
    skip = pytest.mark.skip(reason="no HIP device")
    for it in items:
        if "gpu" in it.keywords:
            it.add_marker(skip)


def pytest_sessionstart(session):
    """PSVI_DEBUG_SET="key=value,...": psvi_debug_set before any test (A/B
    runs of the suite on an alternative kernel path, e.g. 16=1 for the VALU
    LeNet conv towers); unset in normal runs."""
    spec = os.environ.get("PSVI_DEBUG_SET", "")
    if not spec:
        return
    from psvi.runtime import _lib

    lib = _lib.load()
    for kv in spec.split(","):
        k, v = (int(x) for x in kv.split("="))
        if lib.psvi_debug_set(k, v):
            raise RuntimeError(f"psvi_debug_set({k}, {v}) failed")
