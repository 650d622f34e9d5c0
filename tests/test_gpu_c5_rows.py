"""BASELINE config 5 at full size (5M users x 500K repos, 100M stars, rank 256, nonnegative):
sampled rows against the fp64 oracle of Spark's NNLSSolver (mllib NNLS.scala restated in
oracle/spark_als.py), on the engine's own inputs (ratings from als_get_row_ratings, src factors from
als_get_factors, G = their fp64 Gram): the user half of the first sweep, then both halves of the
third sweep (the state the c5 bench times: 1 warmup + 2 timed sweeps) -- 50 repo rows including the
three >1M-star repos (split-K partials + the NNLS PRE kernel) and 100 user rows over the lockstep,
per-row light and per-row heavy paths.  The converged rows are solved by the C restatement of
NNLS.solve (oracle/c/als_cpu.c, equal to the numpy one: tests/test_oracle.py), since a rank-256 repo
row takes up to 5,120 iterations.

Both NNLS kernels are covered: rows of degree <= 6 run 16 per workgroup in lockstep
(nnls_batch.hip), the rest one workgroup per row.  Tolerance: max|x - x64| / max|x64| <= 1e-3
per row (NNLS rows, as tests/test_gpu_parity.py), plus the QP objective of the engine's x within
1e-6 (relative) of the oracle's.
"""
import ctypes as C
import json
import os

import numpy as np
import pytest

from oracle import spark_als as O

pytestmark = pytest.mark.gpu

OUT = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "gpurun_out")


def test_c5_nnls_rows_match_oracle(gpu_lib):
    from albedo_amd import _lib as L
    from albedo_amd.synthetic import CONFIGS, popularity_table, user_degrees
    lib = gpu_lib
    spec = CONFIGS["c5"]
    k = 256
    p = L.als_params()
    L.check(lib.als_params_default(C.byref(p)))
    p.rank, p.implicit_prefs, p.reg_param, p.alpha, p.seed, p.nonnegative = k, 1, 0.5, 40.0, 42, 1
    h = C.c_void_p()
    L.check(lib.als_create(C.byref(p), C.byref(h)))
    try:
        deg = user_degrees(spec)
        prefix = np.ascontiguousarray(np.r_[0, np.cumsum(deg)].astype(np.int64))
        cw, perm = popularity_table(spec)
        L.check(lib.als_set_ratings_synthetic(h, spec.seed, spec.rounds, spec.n_users, spec.n_items,
                                              L.ptr(prefix, C.c_int64), L.ptr(np.ascontiguousarray(cw), C.c_double),
                                              L.ptr(np.ascontiguousarray(perm), C.c_int32)))
        L.check(lib.als_init_factors_random(h, 42))
        L.check(lib.als_half_sweep(h, 1))
        L.check(lib.als_half_sweep(h, 0))
        st = np.zeros(4, np.int64)
        L.check(lib.als_path_stats(h, 0, L.ptr(st, C.c_int64)))
        ni, nu = lib.als_num_rows(h, 1), lib.als_num_rows(h, 0)
        iid = np.empty(ni, np.int32)
        V = np.empty((ni, k), np.float32)
        L.check(lib.als_get_factors(h, 1, L.ptr(iid, C.c_int32), L.ptr(V, C.c_float)))
        uid = np.empty(nu, np.int32)
        U = np.empty((nu, k), np.float32)
        L.check(lib.als_get_factors(h, 0, L.ptr(uid, C.c_int32), L.ptr(U, C.c_float)))
        dg = np.empty(nu, np.int64)
        L.check(lib.als_get_degrees(h, 0, L.ptr(dg, C.c_int64)))
        G = O.gram(V)
        rng = np.random.default_rng(5)
        report = {"paths": st.tolist()}
        worst = {}
        for name, lo, hi, n in (("lockstep", 1, 6, 12), ("light", 7, 64, 8), ("heavy", 65, 10 ** 9, 4)):
            cand = np.flatnonzero((dg >= lo) & (dg <= hi))
            rows = rng.choice(cand, n, replace=False)
            errs, gaps = [], []
            for r in rows:
                cap = int(dg[r])
                src = np.empty(cap, np.int32)
                rt = np.empty(cap, np.float32)
                no = C.c_int64()
                L.check(lib.als_get_row_ratings(h, 0, int(uid[r]), cap, L.ptr(src, C.c_int32), L.ptr(rt, C.c_float),
                                                C.byref(no)))
                Y = V[np.searchsorted(iid, src)]
                A, b, npos = O.normal_equation(Y, np.array([0, cap]), np.arange(cap), rt, 0, True, 40.0, G)
                x_ref = O.nnls_solve(A, b, 0.5 * npos).astype(np.float64)
                x = U[r].astype(np.float64)
                errs.append(float(np.max(np.abs(x - x_ref)) / max(np.max(np.abs(x_ref)), 1e-30)))
                A2 = A + 0.5 * npos * np.eye(k)
                f = lambda v: 0.5 * v @ A2 @ v - b @ v  # noqa: E731
                gaps.append(float((f(x) - f(x_ref)) / max(abs(f(x_ref)), 1e-30)))
            report[name] = {"rows": int(n), "max_rel": max(errs), "objective_gap": [min(gaps), max(gaps)],
                            "ref_zero_frac": None}
            worst[name] = max(errs)
        assert st[0] > 4_000_000  # the lockstep kernel took the low-degree rows
        # ---- sweeps 2 and 3: the converged state of the bench -----------------------------------
        L.check(lib.als_run_sweeps(h, 1))
        L.check(lib.als_get_factors(h, 0, L.ptr(uid, C.c_int32), L.ptr(U, C.c_float)))
        L.check(lib.als_half_sweep(h, 1))
        L.check(lib.als_get_factors(h, 1, L.ptr(iid, C.c_int32), L.ptr(V, C.c_float)))
        ig = np.empty(ni, np.int64)
        L.check(lib.als_get_degrees(h, 1, L.ptr(ig, C.c_int64)))
        top = np.argsort(-ig, kind="stable")[:3]
        assert ig[top[2]] > 1_000_000
        rng = np.random.default_rng(6)
        item_rows = np.r_[top, rng.choice(np.flatnonzero(ig > 8192), 7, replace=False),
                          rng.choice(np.flatnonzero(ig <= 8192), 40, replace=False)]
        report["sweep3_item"] = _check_converged(lib, L, h, 1, iid, V, uid, U, ig, item_rows, k)
        del U
        U = np.empty((nu, k), np.float32)
        L.check(lib.als_half_sweep(h, 0))
        L.check(lib.als_get_factors(h, 0, L.ptr(uid, C.c_int32), L.ptr(U, C.c_float)))
        user_rows = np.r_[rng.choice(np.flatnonzero(dg <= 6), 40, replace=False),
                          rng.choice(np.flatnonzero((dg > 6) & (dg <= 64)), 40, replace=False),
                          rng.choice(np.flatnonzero(dg > 64), 20, replace=False)]
        report["sweep3_user"] = _check_converged(lib, L, h, 0, uid, U, iid, V, dg, user_rows, k)
        os.makedirs(OUT, exist_ok=True)
        with open(os.path.join(OUT, "c5_nnls_rows.json"), "w") as fh:
            json.dump(report, fh)
        print(json.dumps(report))
        for name, e in worst.items():
            assert e <= 1e-3, (name, report)
        for name in ("sweep3_item", "sweep3_user"):
            assert report[name]["max_rel"] <= 1e-3, (name, report[name])
            assert report[name]["objective_gap_max"] <= 1e-6, (name, report[name])
    finally:
        lib.als_destroy(h)


def _check_converged(lib, L, h, side, dst_ids, X, src_ids, Y, deg, rows, k, chunk=1 << 18):
    """Rows `rows` (positions) of `side`, solved into X from src factors Y, against NNLS.solve on
    Spark's normal equation built in fp64 from the engine's own CSR (chunked: a 1.9M-star row)."""
    from oracle import cbind
    G = np.zeros((k, k))
    for r0 in range(0, Y.shape[0], 1 << 20):
        Yc = Y[r0:r0 + (1 << 20)].astype(np.float64)
        G += Yc.T @ Yc
    errs, gaps, iters = [], [], []
    no = C.c_int64()
    for r in rows:
        cap = int(deg[r])
        src = np.empty(cap, np.int32)
        rt = np.empty(cap, np.float32)
        L.check(lib.als_get_row_ratings(h, side, int(dst_ids[r]), cap, L.ptr(src, C.c_int32), L.ptr(rt, C.c_float),
                                        C.byref(no)))
        pos = np.searchsorted(src_ids, src)
        A = G.copy()
        b = np.zeros(k)
        for p0 in range(0, cap, chunk):
            Yr = Y[pos[p0:p0 + chunk]].astype(np.float64)
            r64 = rt[p0:p0 + chunk].astype(np.float64)
            cvec = 40.0 * np.abs(r64)
            A += (Yr.T * cvec) @ Yr
            b += Yr.T @ np.where(r64 > 0, 1.0 + cvec, 0.0)
        A += 0.5 * float(np.sum(rt > 0)) * np.eye(k)
        x_ref, it = cbind.nnls_dense(A, b)
        x_ref = x_ref.astype(np.float64)
        x = X[r].astype(np.float64)
        errs.append(float(np.max(np.abs(x - x_ref)) / max(np.max(np.abs(x_ref)), 1e-30)))
        f = lambda v: 0.5 * v @ A @ v - b @ v  # noqa: E731
        gaps.append(float((f(x) - f(x_ref)) / max(abs(f(x_ref)), 1e-30)))
        iters.append(int(it))
    return {"rows": int(len(rows)), "max_rel": max(errs), "objective_gap_max": max(gaps),
            "objective_gap_min": min(gaps), "max_degree": int(deg[rows].max()), "oracle_iters_max": max(iters),
            "oracle_iters_mean": float(np.mean(iters))}
