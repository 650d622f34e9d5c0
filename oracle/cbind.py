"""ctypes binding of oracle/c/liboracle_als.so — TEST INFRASTRUCTURE / CPU BASELINE ONLY."""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

_PATH = os.path.join(os.path.dirname(os.path.abspath(__file__)), "c", "liboracle_als.so")
_lib = None


def load():
    global _lib
    if _lib is None:
        _lib = C.CDLL(_PATH)
        P = C.c_void_p
        _lib.oracle_half_sweep.restype = C.c_int
        _lib.oracle_half_sweep.argtypes = [C.c_int64, P, P, P, C.c_int64, P, C.c_int, C.c_int, C.c_double,
                                           C.c_double, P, C.c_int64, P, C.c_int]
        _lib.oracle_solve_rows.restype = C.c_int
        _lib.oracle_solve_rows.argtypes = [C.c_int64, P, P, P, P, C.c_int, C.c_int, C.c_double, C.c_double, P, P,
                                           C.c_int64, P, C.c_int]
        _lib.oracle_solve_rows_nnls.restype = C.c_int
        _lib.oracle_solve_rows_nnls.argtypes = [C.c_int64, P, P, P, P, C.c_int, C.c_int, C.c_double, C.c_double, P,
                                                P, C.c_int64, P, P, C.c_int]
        _lib.oracle_nnls_dense.restype = C.c_int
        _lib.oracle_nnls_dense.argtypes = [C.c_int, P, P, P]
        _lib.oracle_gram.restype = C.c_int
        _lib.oracle_gram.argtypes = [C.c_int64, C.c_int, P, P, C.c_int]
        _lib.oracle_max_threads.restype = C.c_int
        _lib.oracle_recommend.restype = C.c_int
        _lib.oracle_recommend.argtypes = [C.c_int64, P, C.c_int64, P, P, C.c_int, C.c_int, P, P, C.c_int]
    return _lib


def _p(a):
    return a.ctypes.data_as(C.c_void_p) if a is not None else None


def half_sweep(Ysrc, ptr, col, val, *, reg, alpha, implicit=True, rows=None, threads=None):
    lib = load()
    Ysrc = np.ascontiguousarray(Ysrc, dtype=np.float32)
    ptr = np.ascontiguousarray(ptr, dtype=np.int64)
    col = np.ascontiguousarray(col, dtype=np.int32)
    val = np.ascontiguousarray(val, dtype=np.float32)
    n_dst = len(ptr) - 1
    k = Ysrc.shape[1]
    X = np.zeros((n_dst, k), dtype=np.float32)
    rws = None if rows is None else np.ascontiguousarray(rows, dtype=np.int32)
    nt = threads or lib.oracle_max_threads()
    rc = lib.oracle_half_sweep(n_dst, _p(ptr), _p(col), _p(val), Ysrc.shape[0], _p(Ysrc), k, int(implicit),
                               float(alpha), float(reg), _p(rws), 0 if rws is None else len(rws), _p(X), nt)
    if rc != 0:
        raise ValueError(f"oracle half-sweep: row {rc - 1} not positive definite (rc={rc})")
    return X


def gram(Y, threads=None):
    lib = load()
    Y = np.ascontiguousarray(Y, dtype=np.float32)
    k = Y.shape[1]
    G = np.zeros((k, k), dtype=np.float64)
    lib.oracle_gram(Y.shape[0], k, _p(Y), _p(G), threads or lib.oracle_max_threads())
    return G


def solve_rows(Ysrc, G, ptr, col, val, *, reg, alpha, implicit=True, threads=None):
    """Solve every row of the given CSR against src factors Ysrc with a precomputed Gram G."""
    lib = load()
    Ysrc = np.ascontiguousarray(Ysrc, dtype=np.float32)
    G = np.ascontiguousarray(G, dtype=np.float64)
    ptr = np.ascontiguousarray(ptr, dtype=np.int64)
    col = np.ascontiguousarray(col, dtype=np.int32)
    val = np.ascontiguousarray(val, dtype=np.float32)
    n_dst = len(ptr) - 1
    k = Ysrc.shape[1]
    X = np.zeros((n_dst, k), dtype=np.float32)
    rc = lib.oracle_solve_rows(n_dst, _p(ptr), _p(col), _p(val), _p(Ysrc), k, int(implicit), float(alpha),
                               float(reg), _p(G), None, 0, _p(X), threads or lib.oracle_max_threads())
    if rc != 0:
        raise ValueError(f"oracle solve_rows: row {rc - 1} not positive definite (rc={rc})")
    return X


def solve_rows_nnls(Ysrc, G, ptr, col, val, *, reg, alpha, implicit=True, threads=None):
    """solve_rows with Spark's NNLSSolver (setNonnegative(true)): (X [n_dst, k], NNLS iterations per row)."""
    lib = load()
    Ysrc = np.ascontiguousarray(Ysrc, dtype=np.float32)
    G = np.ascontiguousarray(G, dtype=np.float64)
    ptr = np.ascontiguousarray(ptr, dtype=np.int64)
    col = np.ascontiguousarray(col, dtype=np.int32)
    val = np.ascontiguousarray(val, dtype=np.float32)
    n_dst = len(ptr) - 1
    k = Ysrc.shape[1]
    X = np.zeros((n_dst, k), dtype=np.float32)
    it = np.zeros(n_dst, dtype=np.int32)
    lib.oracle_solve_rows_nnls(n_dst, _p(ptr), _p(col), _p(val), _p(Ysrc), k, int(implicit), float(alpha),
                               float(reg), _p(G), None, 0, _p(X), _p(it), threads or lib.oracle_max_threads())
    return X, it


def nnls_dense(A, b):
    """NNLS.solve (fp64, oracle/c/als_cpu.c) on one system A x = b, A with λn on its diagonal:
    (x as float32 -- NNLSSolver's cast --, iterations)."""
    lib = load()
    A = np.ascontiguousarray(A, dtype=np.float64)
    b = np.ascontiguousarray(b, dtype=np.float64)
    x = np.zeros(len(b))
    it = lib.oracle_nnls_dense(len(b), _p(A), _p(b), _p(x))
    if it < 0:
        raise MemoryError("oracle_nnls_dense")
    return x.astype(np.float32), it


def recommend(src_f, dst_ids, dst_f, num, threads=None):
    """oracle/spark_als.py:recommend_for_all in C/OpenMP (F2J sdot, (score desc, id asc) top-num):
    (ids[n_src, num], scores[n_src, num]), -1 / NaN padded."""
    lib = load()
    dst_ids = np.asarray(dst_ids, dtype=np.int32)
    order = np.argsort(dst_ids, kind="stable")
    ids_sorted = np.ascontiguousarray(dst_ids[order])
    dst_f = np.ascontiguousarray(np.asarray(dst_f, dtype=np.float32)[order])
    src_f = np.ascontiguousarray(src_f, dtype=np.float32)
    n_src, k = src_f.shape
    out_i = np.empty((n_src, num), np.int32)
    out_s = np.empty((n_src, num), np.float32)
    rc = lib.oracle_recommend(n_src, _p(src_f), len(ids_sorted), _p(ids_sorted), _p(dst_f), k, num, _p(out_i),
                              _p(out_s), threads or lib.oracle_max_threads())
    if rc != 0:
        raise ValueError(f"oracle_recommend failed (rc={rc}): duplicate dst ids?")
    return out_i, out_s
