"""The drop-in boundary on CPU: libpsvi_hip.so loads, exports every function
include/psvi_hip.h declares (and the ctypes binding covers exactly those),
and the host-side plan logic (geometry, shards, error convention) behaves --
no kernel launches here."""
import ctypes
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "psvi_hip.h")


def header_functions():
    text = open(HEADER).read()
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
    missing = [f for f in header_functions() if not hasattr(lib, f)]
    assert not missing, missing
    # the Python binding declares a signature for each of them, and nothing else
    assert sorted(_lib.SIGNATURES) == header_functions()


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
    # rows: every layer's rows partitioned in order; nnz roughly balanced
    for l, (din, dout) in enumerate(layers):
        n = din * dout + dout
        lo = [i["row_lo"][l] for i in infos]
        cnt = [i["row_cnt"][l] for i in infos]
        assert lo[0] == 0 and sum(cnt) == n
        for r in range(1, world):
            assert lo[r] == lo[r - 1] + cnt[r - 1]
    if world > 1:
        nnz = [sum(sum(rr for rr in range(i["row_lo"][l], i["row_lo"][l] + i["row_cnt"][l]))
                   for l in range(3)) for i in infos]
        assert max(nnz) < 1.25 * (sum(nnz) / world)
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
