"""ctypes binding of libpsvi_hip.so (C ABI: include/psvi_hip.h).

The library is built in-tree (``make -C blackbox-coresets-vi_amd``) and loaded
from this directory.  There is no fallback: if the shared object is missing or
fails to load, every entry point raises, so a GPU run can never silently route
around the HIP kernels.
"""
import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "libpsvi_hip.so")

MAX_LAYERS = 8
FAMILY_MEANFIELD = 0
FAMILY_FULLCOV = 1
FAMILY_LENET = 2
LOOP_KEEP = 1    # psvi_inner_loop_ex flags
LOOP_RESUME = 2
ADAM_HIGHER = 0
ADAM_HYPERGRAD = 1
ADAM_TORCH = 2

Q_PARAM_COUNT = 1
Q_EPS_COUNT = 2
Q_WS_BYTES = 3
Q_S_LOCAL = 4
Q_S_OFFSET = 5
Q_ACC_COUNT = 6
Q_ROWS_LOCAL = 7
Q_XSHARD_COUNT = 8
Q_XRECV_COUNT = 9
Q_LOOP_WS_BYTES = 10
Q_TILED_FLOATS = 11
Q_OUTER_WS_BYTES = 12
Q_HVP_WS_BYTES = 13
Q_EVAL_WS_BYTES = 14
Q_NET_PART_OK = 15

ERRORS = {-1: "PSVI_EINVAL", -2: "PSVI_ENOSPC", -3: "PSVI_EUNSUP", -4: "PSVI_ESTATE"}


class NetDesc(ctypes.Structure):
    _fields_ = [
        ("n_layers", ctypes.c_int32),
        ("dims", ctypes.c_int32 * (MAX_LAYERS + 1)),
        ("S", ctypes.c_int32),
        ("M", ctypes.c_int32),
        ("prior_sd", ctypes.c_float),
    ]


class AdamHP(ctypes.Structure):
    _fields_ = [
        ("lr", ctypes.c_float),
        ("beta1", ctypes.c_float),
        ("beta2", ctypes.c_float),
        ("eps", ctypes.c_float),
        ("step", ctypes.c_int32),
        ("kind", ctypes.c_int32),
    ]


# name -> (restype, argtypes)
_P = ctypes.c_void_p
_I32 = ctypes.c_int32
_I64 = ctypes.c_int64
_U64 = ctypes.c_uint64
_SZ = ctypes.c_size_t
SIGNATURES = {
    "psvi_plan_create": (_I32, [_I32, ctypes.POINTER(NetDesc), _I32, _I32, ctypes.POINTER(_P)]),
    "psvi_plan_destroy": (_I32, [_P]),
    "psvi_plan_query": (_I32, [_P, _I32, ctypes.POINTER(_I64)]),
    "psvi_plan_shard_info": (_I32, [_P, _I32, ctypes.POINTER(_I64)]),
    "psvi_plan_shard_runs": (_I32, [_P, _I32, _P, _I32, ctypes.POINTER(_I32)]),
    "psvi_inner_step": (_I32, [_P, _P, _P, _P, _P, _P, _P, _P, ctypes.POINTER(AdamHP), _P, _P,
                               _SZ, _P]),
    "psvi_elbo_grad": (_I32, [_P, _P, _P, _P, _P, _P, _I32, _P, _P, _P, _SZ, _P]),
    "psvi_mf_phase_accumulate": (_I32, [_P, _P, _P, _P, _P, _P, _P, _P, _P]),
    "psvi_mf_phase_update": (_I32, [_P, _P, _P, _P, _P, ctypes.POINTER(AdamHP), _P, _P, _I32,
                                    _P]),
    "psvi_mvn_phase_sample": (_I32, [_P, _P, _P, _P, _P]),
    "psvi_mvn_phase_net": (_I32, [_P, _P, _P, _P, _P, _P, _P, _P]),
    "psvi_mvn_phase_net_draw": (_I32, [_P, _P, _P, _P, _P, _P, _P, _P, _I64, _U64, _U64, _P]),
    "psvi_mvn_phase_net_part": (_I32, [_P, _P, _P, _P, _P, _P, _P, _I32, _I32, _P, _I64, _U64, _U64,
                                       _I32, _I32, _P]),
    "psvi_mvn_phase_update": (_I32, [_P, _P, _P, _P, _P, _P, ctypes.POINTER(AdamHP), _P, _P,
                                     _I32, _P]),
    "psvi_mvn_phase_update_sample": (_I32, [_P, _P, _P, _P, _P, _P, ctypes.POINTER(AdamHP), _P,
                                            _I32, _P, _P, _P]),
    "psvi_mvn_tiled_convert": (_I32, [_P, _P, _P, _P, _P, _I32, _P]),
    "psvi_mvn_phase_update_tiled": (_I32, [_P, _P, _P, _P, _P, _P, _P, ctypes.POINTER(AdamHP), _P,
                                           _I32, _P, _P, _P]),
    "psvi_inner_loop": (_I32, [_P, _P, _P, _P, _P, _U64, _U64, _I32, _P, _P, _P,
                               ctypes.POINTER(AdamHP), _P, _P, _SZ, _P]),
    "psvi_inner_loop_ex": (_I32, [_P, _P, _P, _P, _P, _U64, _U64, _I32, _P, _P, _P,
                                  ctypes.POINTER(AdamHP), _P, _P, _SZ, _I32, _P]),
    "psvi_outer_elbo_grad": (_I32, [_P, _I32, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P,
                                    _SZ, _P]),
    "psvi_outer_ablated_elbo_grad": (_I32, [_P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _SZ, _P]),
    "psvi_outer_elbo_grad_coef": (_I32, [_P, _I32, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P,
                                         _SZ, _P]),
    "psvi_evaluate": (_I32, [_P, _I32, _P, _P, _P, _P, _P, _I32, _P, _P, _P, _SZ, _P]),
    "psvi_hvp": (_I32, [_P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _SZ, _P]),
    "psvi_hvp_partial": (_I32, [_P, _P, _P, _P, _P, _P, _P, _I32, _P, _P, _P, _P, _SZ, _P]),
    "psvi_adam_adjoint": (_I32, [_I64, _P, _P, _P, _P, _P, _P, _P, ctypes.POINTER(AdamHP),
                                 _P]),
    "psvi_randn": (_I32, [_P, _I64, _U64, _U64, _P]),
    "psvi_nonfinite": (_I32, [_P, _I64, _I32, _P, _P]),
    "psvi_adam_update": (_I32, [_I64, _P, _P, _P, _P, ctypes.POINTER(AdamHP), _P]),
    "psvi_cg_ws_bytes": (ctypes.c_size_t, []),
    "psvi_cg_scale": (_I32, [_I64, _P, ctypes.c_double, _P, _P]),
    "psvi_cg_pap": (_I32, [_I64, _P, _P, ctypes.c_double, _P, _P, _P, ctypes.c_size_t, _P]),
    "psvi_cg_residual": (_I32, [_I64, _P, _P, ctypes.c_double, _P, _P, ctypes.c_double, _P,
                                ctypes.c_size_t, _P]),
    "psvi_cg_update": (_I32, [_I64, _P, _P, _P, _P, _P, _P]),
    "psvi_debug_set": (_I32, [_I32, _I32]),
    "psvi_debug_set_ptr": (_I32, [_I32, _P]),
    "psvi_debug_loop_timing": (_I32, [_P]),
    "psvi_last_error": (ctypes.c_char_p, []),
    "psvi_version": (ctypes.c_char_p, []),
}

_lib = None
_load_error = None


class PsviError(RuntimeError):
    pass


def load():
    """Load (once) and return the bound library; raises if it is unavailable."""
    global _lib, _load_error
    if _lib is not None:
        return _lib
    if _load_error is not None:
        raise PsviError(_load_error)
    if not os.path.exists(LIB_PATH):
        _load_error = (f"HIP library not built: {LIB_PATH} is missing "
                       "(run `make -C blackbox-coresets-vi_amd` or __graft_entry__.build())")
        raise PsviError(_load_error)
    try:
        lib = ctypes.CDLL(LIB_PATH)
    except OSError as e:  # pragma: no cover - depends on the ROCm runtime
        _load_error = f"failed to load {LIB_PATH}: {e}"
        raise PsviError(_load_error)
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _lib = lib
    return lib


def check(rc, what):
    if rc != 0:
        msg = load().psvi_last_error().decode(errors="replace")
        kind = ERRORS.get(rc, f"hipError {rc}")
        raise PsviError(f"{what} failed ({kind}): {msg}")
