"""ctypes binding of libalbedo_als.so (include/albedo_als.h).

The library is built in-tree (`albedo_amd/libalbedo_als.so`, see `__graft_entry__.build`).  There is
no CPU fallback: when the library or a gfx950 device is missing, engine calls raise.

If the same process uses PyTorch, import torch BEFORE albedo_amd: torch ships its own HIP runtime
(soname libamdhip64.so.7) and loading it after ours would put two HIP runtimes in one process.
"""
from __future__ import annotations

import ctypes as C
import os
import sys

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("ALBEDO_ALS_LIB", os.path.join(_HERE, "libalbedo_als.so"))

ALS_OK = 0
ALS_E_INVALID_ARGUMENT = 1
ALS_E_NOT_POSITIVE_DEFINITE = 2
ALS_E_STATE = 3
ALS_E_HIP = 4
ALS_E_RCCL = 5
ALS_E_OUT_OF_MEMORY = 6
ALS_E_NO_DEVICE = 7
ALS_E_UNSUPPORTED = 8
ALS_USER, ALS_ITEM = 0, 1
ALS_T_COUNT = 8
T_NAMES = ["gram", "eig", "rotate", "comm", "solve_light", "solve_heavy", "half_total", "_"]


class als_params(C.Structure):
    _fields_ = [
        ("rank", C.c_int32),
        ("max_iter", C.c_int32),
        ("implicit_prefs", C.c_int32),
        ("nonnegative", C.c_int32),
        ("num_user_blocks", C.c_int32),
        ("num_item_blocks", C.c_int32),
        ("reg_param", C.c_double),
        ("alpha", C.c_double),
        ("seed", C.c_int64),
        ("device", C.c_int32),
        ("light_max_degree", C.c_int32),
    ]


class ALSError(RuntimeError):
    """Base class; `code` is the ALS_E_* value."""

    def __init__(self, code, msg):
        super().__init__(msg)
        self.code = code


class IllegalArgumentException(ALSError, ValueError):
    """Spark's IllegalArgumentException (ParamValidators, empty ratings, dppsv not-PD)."""


class IllegalStateException(ALSError):
    pass


ALLREDUCE_FN = C.CFUNCTYPE(C.c_int, C.c_void_p, C.POINTER(C.c_double), C.c_int64)
ALLGATHER_FN = C.CFUNCTYPE(C.c_int, C.c_void_p, C.POINTER(C.c_float), C.c_int64)

# (name, restype, argtypes) — every entry point of include/albedo_als.h
P = C.c_void_p
I32P = C.POINTER(C.c_int32)
I64P = C.POINTER(C.c_int64)
F32P = C.POINTER(C.c_float)
F64P = C.POINTER(C.c_double)
SIGNATURES = [
    ("als_params_default", C.c_int, [C.POINTER(als_params)]),
    ("als_create", C.c_int, [C.POINTER(als_params), C.POINTER(P)]),
    ("als_destroy", None, [P]),
    ("als_set_params", C.c_int, [P, C.POINTER(als_params)]),
    ("als_fork", C.c_int, [P, C.POINTER(als_params), C.POINTER(P)]),
    ("als_last_error", C.c_char_p, []),
    ("als_abi_version", C.c_int, []),
    ("als_device_count", C.c_int, [C.POINTER(C.c_int)]),
    ("als_comm_unique_id", C.c_int, [P]),
    ("als_comm_init", C.c_int, [P, C.c_int32, C.c_int32, P]),
    ("als_set_ratings", C.c_int, [P, C.c_int64, I32P, I32P, F32P]),
    ("als_set_ratings_device", C.c_int, [P, C.c_int64, P, P, P]),
    ("als_num_rows", C.c_int64, [P, C.c_int]),
    ("als_num_ratings", C.c_int64, [P]),
    ("als_rank", C.c_int, [P]),
    ("als_get_ids", C.c_int, [P, C.c_int, I32P]),
    ("als_set_initial_factors", C.c_int, [P, C.c_int, C.c_int64, I32P, F32P]),
    ("als_init_factors", C.c_int, [P]),
    ("als_init_factors_random", C.c_int, [P, C.c_uint64]),
    ("als_get_factors", C.c_int, [P, C.c_int, I32P, F32P]),
    ("als_fit", C.c_int, [P]),
    ("als_run_sweeps", C.c_int, [P, C.c_int32]),
    ("als_half_sweep", C.c_int, [P, C.c_int]),
    ("als_get_gram", C.c_int, [P, C.c_int, F64P]),
    ("als_get_degrees", C.c_int, [P, C.c_int, I64P]),
    ("als_get_row_ratings", C.c_int, [P, C.c_int, C.c_int32, C.c_int64, I32P, F32P, I64P]),
    ("als_model_create", C.c_int, [C.c_int32, C.c_int64, I32P, F32P, C.c_int64, I32P, F32P, C.c_int32, C.POINTER(P)]),
    ("als_recommend", C.c_int, [P, C.c_int, C.c_int32, I32P, C.c_int64, I32P, I32P, F32P]),
    ("als_predict", C.c_int, [P, C.c_int64, I32P, I32P, F32P]),
    ("als_evaluate_ndcg", C.c_int, [P, C.c_int32, C.c_int64, I32P, I32P, I64P, F64P, I64P, I32P, F64P, C.c_int64]),
    ("als_last_timings", C.c_int, [P, C.c_int, F64P, C.c_int]),
    ("als_path_stats", C.c_int, [P, C.c_int, I64P]),
    ("als_solver_stats", C.c_int, [P, C.c_int, I64P]),
    ("als_topk_stats", C.c_int, [P, I64P]),
    ("als_topk_timing", C.c_int, [P, F64P]),
    ("als_get_basis", C.c_int, [P, C.c_int, F64P]),
    ("als_topk_last_rescan", C.c_int, [P, I32P, C.c_int64, I64P]),
    ("als_synchronize", C.c_int, [P]),
    ("als_synth_generate", C.c_int, [C.c_int32, C.c_uint64, C.c_int32, C.c_int64, C.c_int64, I64P, F64P, I32P,
                                     I32P, I32P, F32P, I64P]),
    ("als_set_ratings_synthetic", C.c_int, [P, C.c_uint64, C.c_int32, C.c_int64, C.c_int64, I64P, F64P, I32P]),
    ("als_comm_init_host", C.c_int, [P, C.c_int32, C.c_int32, ALLREDUCE_FN, ALLGATHER_FN, P]),
    ("als_host_eigh", C.c_int, [C.c_int32, F64P, F64P, F64P]),
    ("als_device_eigh", C.c_int, [C.c_int32, C.c_int32, F64P, F64P, F64P, F64P, I32P]),
    ("als_host_spark_side_seeds", C.c_int, [C.c_int64, I64P, I64P]),
    ("als_host_spark_init", C.c_int, [I32P, C.c_int64, C.c_int32, C.c_int64, C.c_int32, F32P]),
    ("als_host_plan_shards", C.c_int, [I64P, C.c_int64, C.c_int32, I64P]),
]

_lib = None


def load():
    """Load (once) and return the ctypes library; raises ImportError when it is missing."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise ImportError(
            f"{LIB_PATH} not found: build it with `python -c 'import __graft_entry__ as g; g.build()'` "
            "(the ALS engine has no CPU fallback)")
    lib = C.CDLL(LIB_PATH, mode=C.RTLD_GLOBAL)
    for name, res, args in SIGNATURES:
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _lib = lib
    return lib


def check(rc):
    if rc == ALS_OK:
        return
    msg = load().als_last_error().decode("utf-8", "replace")
    if rc in (ALS_E_INVALID_ARGUMENT, ALS_E_NOT_POSITIVE_DEFINITE):
        raise IllegalArgumentException(rc, msg)
    if rc == ALS_E_STATE:
        raise IllegalStateException(rc, msg)
    raise ALSError(rc, msg)


def ptr(a, ctype):
    return a.ctypes.data_as(C.POINTER(ctype))


def device_count() -> int:
    n = C.c_int(0)
    check(load().als_device_count(C.byref(n)))
    return n.value

