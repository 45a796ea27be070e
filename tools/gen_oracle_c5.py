#!/usr/bin/env python3
"""Oracle outputs for the C5 (make_lenet, S = 256, M = 500) parity case.

Test infrastructure: runs the fp64 oracle (oracle/psvi_oracle.py) on one rank's
share of a world-8 sample split -- 32 of the 256 samples against all 500
pseudo-images (and a 64-row data batch for the outer objective) -- and writes
the expected values to tests/golden/c5_lenet_rank.npz.  The inputs are NOT
stored: tests/golden_util.py c5_lenet_case() regenerates them from the seed.
The oracle takes minutes at this size, so its results are committed; the GPU
test (tests/test_hip_lenet_c5.py) compares the HIP path against them.

    python tools/gen_oracle_c5.py
"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, os.path.join(ROOT, "tests"))

import psvi_oracle as O  # noqa: E402
from golden_util import C5, GOLDEN, c5_lenet_case  # noqa: E402


def main():
    c = c5_lenet_case()
    S = c["s_cnt"]
    out = {}
    t0 = time.time()
    # inner objective: sum over the rank's samples of sum_m w_m NLL_sm, + KL
    val, g = O.lenet_elbo_grad(c["params"], c["u"], c["z"], c["w"], c["eps_loc"], S)
    out.update(inner_value=np.float64(val), inner_grad=g.astype(np.float32))
    print(f"inner {time.time() - t0:.1f}s", flush=True)
    # outer objective, the two passes of the sample-sharded form
    X = np.concatenate([c["u"], c["xb"]])
    zz = np.concatenate([c["z"], c["yb"]])
    ww = np.concatenate([c["w"], np.full(C5["Nx"], C5["N"] / C5["Nx"], np.float32)])
    terms, go, gu, gw = O.lenet_outer_coef_grad(c["params"], X, zz, ww, C5["M"], c["eps_loc"],
                                                S, c["cp"], c["cd"], c["ck"])
    out.update(outer_terms=terms, outer_grad=go.astype(np.float32),
               outer_grad_u=gu.astype(np.float32), outer_grad_w=gw)
    print(f"outer {time.time() - t0:.1f}s", flush=True)
    # Hessian-vector product with its mixed products (KL Hessian included)
    _, _, hv, du, dw = O.lenet_inner_hvp(c["params"], c["u"], c["z"], c["w"], c["eps_loc"], S,
                                         c["vec"])
    out.update(hvp=hv.astype(np.float32), hvp_du=du.astype(np.float32), hvp_dw=dw)
    print(f"hvp {time.time() - t0:.1f}s", flush=True)
    cfg = dict(C5, generator="tools/gen_oracle_c5.py", oracle="oracle/psvi_oracle.py fp64")
    np.savez_compressed(os.path.join(GOLDEN, "c5_lenet_rank.npz"), config=json.dumps(cfg), **out)


if __name__ == "__main__":
    main()
