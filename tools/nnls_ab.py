"""A/B of the lockstep NNLS kernel at BASELINE c5 (diagnostic, not a test).

usage: python tools/nnls_ab.py run <0|1> <out.npz>     one process per mode (ALBEDO_NNLS_BATCH)
       python tools/nnls_ab.py cmp <a.npz> <b.npz>
run: random init, item half, user half (the mode's kernels), item half again; prints the NNLS
iteration statistics of each half and saves every 16th user row's factors with its degree.
"""
import ctypes as C
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def run(mode, out):
    os.environ["ALBEDO_NNLS_BATCH"] = mode[0]
    from albedo_amd import _lib as L
    from albedo_amd.synthetic import CONFIGS, popularity_table, user_degrees
    lib = L.load()
    spec = CONFIGS["c5"]
    p = L.als_params()
    L.check(lib.als_params_default(C.byref(p)))
    p.rank, p.implicit_prefs, p.reg_param, p.alpha, p.seed, p.nonnegative = 256, 1, 0.5, 40.0, 42, 1
    h = C.c_void_p()
    L.check(lib.als_create(C.byref(p), C.byref(h)))
    deg = user_degrees(spec)
    prefix = np.ascontiguousarray(np.r_[0, np.cumsum(deg)].astype(np.int64))
    cw, perm = popularity_table(spec)
    L.check(lib.als_set_ratings_synthetic(h, spec.seed, spec.rounds, spec.n_users, spec.n_items,
                                          L.ptr(prefix, C.c_int64), L.ptr(np.ascontiguousarray(cw), C.c_double),
                                          L.ptr(np.ascontiguousarray(perm), C.c_int32)))
    L.check(lib.als_init_factors_random(h, 42))
    res = {}
    for name, side in (("item1", 1), ("user", 0), ("user_again", 0), ("item2", 1)):
        t = time.time()
        L.check(lib.als_half_sweep(h, side))
        L.check(lib.als_synchronize(h))
        sv = np.zeros(4, np.int64)
        L.check(lib.als_solver_stats(h, side, L.ptr(sv, C.c_int64)))
        ps = np.zeros(4, np.int64)
        L.check(lib.als_path_stats(h, side, L.ptr(ps, C.c_int64)))
        tt = np.zeros(L.ALS_T_COUNT)
        L.check(lib.als_last_timings(h, side, L.ptr(tt, C.c_double), L.ALS_T_COUNT))
        res[name] = {"mean_iter": float(sv[0]) / max(int(sv[2]), 1), "max_iter": int(sv[1]), "paths": ps.tolist(),
                     "light_ms": tt[4], "heavy_ms": tt[5], "wall_s": time.time() - t}
        if name in ("user", "user_again"):
            n = lib.als_num_rows(h, 0)
            ids = np.empty(n, np.int32)
            f = np.empty((n, 256), np.float32)
            L.check(lib.als_get_factors(h, 0, L.ptr(ids, C.c_int32), L.ptr(f, C.c_float)))
            dg = np.empty(n, np.int64)
            L.check(lib.als_get_degrees(h, 0, L.ptr(dg, C.c_int64)))
            sel = np.arange(0, n, 16)
            if name == "user":  # objective check of a few rows against the QP optimum (scipy nnls)
                from scipy.optimize import nnls
                ni = lib.als_num_rows(h, 1)
                iid = np.empty(ni, np.int32)
                V = np.empty((ni, 256), np.float32)
                L.check(lib.als_get_factors(h, 1, L.ptr(iid, C.c_int32), L.ptr(V, C.c_float)))
                G = V.astype(np.float64).T @ V.astype(np.float64)
                pos = {int(x): i for i, x in enumerate(iid)} if False else None
                order = np.argsort(iid)
                gaps = {}
                for lo, hi in ((1, 6), (7, 24)):
                    rows = sel[(dg[sel] >= lo) & (dg[sel] <= hi)][:25]
                    g = []
                    for r in rows:
                        cap = int(dg[r])
                        src = np.empty(cap, np.int32)
                        rt = np.empty(cap, np.float32)
                        no = C.c_int64()
                        L.check(lib.als_get_row_ratings(h, 0, int(ids[r]), cap, L.ptr(src, C.c_int32),
                                                        L.ptr(rt, C.c_float), C.byref(no)))
                        Y = V[order[np.searchsorted(iid[order], src)]].astype(np.float64)
                        c = 40.0 * np.abs(rt.astype(np.float64))
                        A = G + (Y.T * c) @ Y + 0.5 * np.sum(rt > 0) * np.eye(256)
                        b = Y.T @ (1.0 + c)
                        Lc = np.linalg.cholesky(A)
                        xs, _ = nnls(Lc.T, np.linalg.solve(Lc, b), maxiter=5000)
                        fobj = lambda x: 0.5 * x @ A @ x - b @ x
                        x = f[r].astype(np.float64)
                        g.append((fobj(x) - fobj(xs)) / abs(fobj(xs)))
                    gaps[f"{lo}-{hi}"] = [float(np.median(g)), float(np.max(g))]
                res["objective_gap_median_max"] = gaps
            np.savez(out if name == "user" else out.replace(".npz", "_again.npz"), ids=ids[sel], f=f[sel], deg=dg[sel])
            del f
    print(json.dumps({"mode": mode, **res}))


def cmp(a, b):
    A, B = np.load(a), np.load(b)
    assert np.array_equal(A["ids"], B["ids"])
    fa, fb, d = A["f"].astype(np.float64), B["f"].astype(np.float64), A["deg"]
    num = np.max(np.abs(fa - fb), axis=1)
    den = np.maximum(np.max(np.abs(fb), axis=1), 1e-30)
    rel = num / den
    for lo, hi in ((1, 6), (7, 24), (25, 10 ** 9)):
        m = (d >= lo) & (d <= hi)
        if m.any():
            q = np.quantile(rel[m], [0.5, 0.9, 0.99, 1.0])
            print(f"deg {lo}-{hi}: rows {m.sum()} rel q50/q90/q99/max {q}; zeros a {np.mean(fa[m] == 0):.3f} b {np.mean(fb[m] == 0):.3f}"
                  f"; |x| mean a {np.abs(fa[m]).mean():.3e} b {np.abs(fb[m]).mean():.3e}")
        if m.any():
            print(f"   exactly equal rows: {np.mean(num[m] == 0):.4f}")
    w = np.argsort(rel)[-5:]
    for i in w:
        print("worst", int(A["ids"][i]), int(d[i]), float(rel[i]), float(num[i]), float(den[i]))


if __name__ == "__main__":
    if sys.argv[1] == "run":
        run(sys.argv[2], sys.argv[3])
    else:
        cmp(sys.argv[2], sys.argv[3])
