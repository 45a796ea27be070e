"""The drop-in boundary on CPU: libpsvi_hip.so loads, exports every function
include/psvi_hip.h declares (and the ctypes binding covers exactly those),
and the host-side plan logic (geometry, shards, error convention) behaves --
no kernel launches here."""
import ctypes
import os
import re

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "psvi_hip.h")
# the library's diagnostics (not the drop-in interface): exported for tools
DIAG = os.path.join(ROOT, "blackbox-coresets-vi_amd", "csrc", "psvi_diag.h")


def header_functions(path=HEADER):
    text = open(path).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"^\s*(?:const\s+)?\w+\**\s+\**(psvi_\w+)\s*\(", text, re.M)))


def test_header_declares_the_api():
    fns = header_functions()
    for need in ("psvi_plan_create", "psvi_inner_step", "psvi_elbo_grad", "psvi_last_error",
                 "psvi_mvn_phase_sample", "psvi_mvn_phase_net", "psvi_mvn_phase_update",
                 "psvi_mf_phase_accumulate", "psvi_mf_phase_update", "psvi_randn"):
        assert need in fns


def test_library_exports_every_declared_symbol():
    from psvi.runtime import _lib

    lib = _lib.load()
    missing = [f for f in header_functions() + header_functions(DIAG) if not hasattr(lib, f)]
    assert not missing, missing
    # the Python binding declares a signature for each of them, and nothing else
    assert sorted(_lib.SIGNATURES) == sorted(header_functions() + header_functions(DIAG))
    # the diagnostics stay out of the public header
    assert not any(f.startswith("psvi_debug") for f in header_functions())
    assert "PSVI_DBG_" not in open(HEADER).read()


def test_symbols_are_c_abi_unmangled():
    from psvi.runtime import _lib

    so = ctypes.CDLL(_lib.LIB_PATH)
    for f in header_functions():
        getattr(so, f)  # dlsym by the plain C name


def test_version_and_error_convention():
    from psvi.runtime import _lib

    lib = _lib.load()
    assert b"gfx950" in lib.psvi_version()
    d = _lib.NetDesc()
    d.n_layers = 0
    h = ctypes.c_void_p()
    rc = lib.psvi_plan_create(_lib.FAMILY_FULLCOV, ctypes.byref(d), 1, 0, ctypes.byref(h))
    assert rc < 0 and not h.value  # invalid descriptor: negative code, no handle
    assert lib.psvi_last_error()  # and a message
    rc = lib.psvi_plan_create(_lib.FAMILY_FULLCOV, None, 1, 0, ctypes.byref(h))
    assert rc < 0


@pytest.mark.parametrize("world", [1, 2, 3, 8])
def test_plan_geometry_fullcov_c3(world):
    from psvi.runtime import InnerLoopPlan

    layers = [(64, 40), (40, 40), (40, 2)]
    S = 128 * world
    plans = [InnerLoopPlan("fullcov", layers, S, 100, world=world, rank=r) for r in range(world)]
    p0 = plans[0]
    assert p0.param_count == 4_730_326 and p0.eps_count == S * 4322
    infos = [p0.shard_info(r) for r in range(world)]
    # samples: contiguous blocks covering [0, S)
    assert infos[0]["s_offset"] == 0
    assert sum(i["s_count"] for i in infos) == S
    for a, b in zip(infos, infos[1:]):
        assert b["s_offset"] == a["s_offset"] + a["s_count"]
    # rows: runs of whole 64-row bands; every layer's rows covered exactly
    # once; each rank's x-shard columns consecutive, layer-major, rows
    # ascending; the 64 x 64 tile counts balanced to within one small band
    ns = [din * dout + dout for din, dout in layers]
    owner = [np.full(n, -1) for n in ns]
    tiles = []
    for r, i in enumerate(infos):
        col, t = 0, 0
        prev = (-1, -1)
        for (l, lo, cnt, c) in i["runs"]:
            assert c == col and (l, lo) > prev
            assert lo % 64 == 0 and (cnt % 64 == 0 or lo + cnt == ns[l])
            assert (owner[l][lo:lo + cnt] == -1).all()
            owner[l][lo:lo + cnt] = r
            t += sum(b + 1 for b in range(lo // 64, (lo + cnt - 1) // 64 + 1))
            col += cnt
            prev = (l, lo + cnt)
        assert col == i["rows"] == sum(i["row_cnt"])
        for l in range(len(layers)):
            rl = [x for x in i["runs"] if x[0] == l]
            assert i["row_lo"][l] == (rl[0][1] if len(rl) == 1 else (0 if not rl else -1))
        tiles.append(t)
    assert all((o >= 0).all() for o in owner)
    if world == 1:
        assert [x[:3] for x in infos[0]["runs"]] == [(l, 0, n) for l, n in enumerate(ns)]
    else:
        assert max(tiles) - min(tiles) <= 3, tiles
    for r, p in enumerate(plans):
        me = p.shard_info(r)
        assert p.s_local == me["s_count"] and p.xshard_count == S * me["rows"]
        assert p.xrecv_count == sum(me["s_count"] * q["rows"] for q in infos)


def test_plan_geometry_meanfield():
    from psvi.runtime import InnerLoopPlan

    p = InnerLoopPlan("meanfield", [(2, 100), (100, 4)], 32, 50)
    assert p.param_count == 1408 and p.eps_count == 32 * 704
    assert p.acc_count == 2 * 704
    with pytest.raises(ValueError):
        InnerLoopPlan("meanfield", [(2, 100), (99, 4)], 32, 50)  # does not chain


@pytest.mark.parametrize("world", [1, 2, 8])
def test_plan_geometry_lenet_c5(world):
    """make_lenet at C5 (S=256, M=500): 123,412 parameters, one shared sample
    in the last layer (850 eps), samples sharded like the mean-field family."""
    from psvi.runtime import InnerLoopPlan

    LEN = [(25, 6), (150, 16), (400, 120), (120, 84), (84, 10)]
    ps = [InnerLoopPlan("lenet", LEN, 256, 500, world=world, rank=r) for r in range(world)]
    for r, p in enumerate(ps):
        assert p.param_count == 123_412 and p.eps_count == 256 * 60_856 + 850
        assert p.acc_count == 2 * 61_706 and p.in_features == 784
        assert p.s_offset == sum(q.s_local for q in ps[:r])
    assert sum(p.s_local for p in ps) == 256
    with pytest.raises(ValueError):
        InnerLoopPlan("lenet", LEN[:-1], 256, 500)


def test_plan_rejects_oversized_layer():
    from psvi.runtime import InnerLoopPlan, PsviError

    with pytest.raises(PsviError):
        InnerLoopPlan("fullcov", [(4096, 4096)], 8, 8)
