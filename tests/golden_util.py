"""Fixture loading + comparison helpers shared by the parity tests."""
import glob
import json
import os

import numpy as np

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def fixture_names(prefix="g"):
    """Inner-loop fixtures (tools/gen_golden.py) start with "g", outer-objective
    fixtures (tools/gen_golden_outer.py) with "o"."""
    return sorted(os.path.basename(f)[:-4]
                  for f in glob.glob(os.path.join(GOLDEN, prefix + "*.npz")))


def load_fixture(name):
    d = np.load(os.path.join(GOLDEN, name + ".npz"))
    cfg = json.loads(str(d["config"]))
    if "layers" in cfg:
        cfg["layers"] = [tuple(x) for x in cfg["layers"]]
    out = {k: d[k] for k in d.files if k != "config"}
    out["cfg"] = cfg
    return out


def family_of(cfg):
    return {"mf": "meanfield", "mvn": "fullcov", "lenet": "lenet"}[cfg["family"]]


LENET_PLAN_LAYERS = [(25, 6), (150, 16), (400, 120), (120, 84), (84, 10)]


def plan_layers(cfg):
    """The InnerLoopPlan layer table of a fixture (LeNet fixtures list only
    their VILinear layers in cfg["layers"])."""
    return LENET_PLAN_LAYERS if cfg["family"] == "lenet" else cfg["layers"]


def adam_kind(cfg):
    return "higher" if cfg["adam"] == "higher" else "hypergrad"


def rel(a, b):
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    return float(np.abs(a - b).max() / max(np.abs(b).max(), 1e-30))


def l2rel(a, b):
    a = np.asarray(a, np.float64).ravel()
    b = np.asarray(b, np.float64).ravel()
    return float(np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-30))


def assert_grad_close(g, gref, l2tol=1e-4, rtol=1e-3, atol_frac=1e-4, what="grad",
                      ref_fp32=None):
    """north-star tolerance: gradient within 1e-4 relative (l2), and every
    element within rtol plus atol_frac of the largest gradient entry -- or, where
    the reference's own fp32 gradient (ref_fp32) deviates more from the fp64
    oracle (sums of cancelling terms), within four times that deviation."""
    g = np.asarray(g, np.float64)
    gref = np.asarray(gref, np.float64)
    e = l2rel(g, gref)
    assert e <= l2tol, f"{what}: l2-relative error {e:.3e} > {l2tol:.0e}"
    tol = rtol * np.abs(gref) + atol_frac * np.abs(gref).max()
    if ref_fp32 is not None:
        tol = np.maximum(tol, 4.0 * np.abs(np.asarray(ref_fp32, np.float64) - gref))
    bad = np.abs(g - gref) > tol
    assert not bad.any(), (f"{what}: {int(bad.sum())} elements out of tolerance, "
                           f"worst idx {int(np.argmax(np.abs(g - gref)))}")
