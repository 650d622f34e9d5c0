"""Diagnostic (GPU box): a synthetic config's fit half-sweep by half-sweep (bench.py's setup), with
the device eigensolver's sweep count, the bases' orthogonality and the rotated Gram's off-diagonal
mass after every half; on a failing half the src Gram and both bases (before and after) go to an
npz for offline analysis.

    python tools/debug_eig.py [--config c4] [--sweeps 25] [--out gpurun_out/debug_eig.npz]
"""
import argparse
import ctypes as C
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c4")
    ap.add_argument("--sweeps", type=int, default=25)
    ap.add_argument("--out", default="gpurun_out/debug_eig.npz")
    args = ap.parse_args()
    from albedo_amd import _lib as L
    from albedo_amd.synthetic import CONFIGS, popularity_table, user_degrees
    sys.path.insert(0, ROOT)
    from bench import CONFIG_RANK
    lib = L.load()
    spec = CONFIGS[args.config]
    k = CONFIG_RANK[args.config]
    p = L.als_params()
    L.check(lib.als_params_default(C.byref(p)))
    p.rank, p.implicit_prefs, p.reg_param, p.alpha, p.seed = k, 1, 0.5, 40.0, 42
    h = C.c_void_p()
    L.check(lib.als_create(C.byref(p), C.byref(h)))
    deg = user_degrees(spec)
    prefix = np.ascontiguousarray(np.r_[0, np.cumsum(deg)].astype(np.int64))
    cw, perm = popularity_table(spec)
    L.check(lib.als_set_ratings_synthetic(h, spec.seed, spec.rounds, spec.n_users, spec.n_items,
                                          L.ptr(prefix, C.c_int64), L.ptr(np.ascontiguousarray(cw), C.c_double),
                                          L.ptr(np.ascontiguousarray(perm), C.c_int32)))
    L.check(lib.als_init_factors_random(h, 42))

    def basis(side):
        b = np.zeros((k, k))
        L.check(lib.als_get_basis(h, side, L.ptr(b, C.c_double)))
        return b

    def gram(side):
        g = np.zeros((k, k))
        L.check(lib.als_get_gram(h, side, L.ptr(g, C.c_double)))
        return g

    for half in range(2 * args.sweeps):
        t = 1 - (half % 2)  # item half first
        s = 1 - t
        Bs0, Bt0 = basis(s), basis(t)
        rc = lib.als_half_sweep(h, t)
        msg = lib.als_last_error().decode() if rc else ""
        sv = np.zeros(4, np.int64)
        L.check(lib.als_solver_stats(h, t, L.ptr(sv, C.c_int64)))
        Bt1 = basis(t)
        G = gram(s)  # original-basis YᵀY of this half's src side
        P = Bs0.T @ Bt1  # the eigenvectors the device produced (src-basis coordinates)
        Gb = Bs0.T @ G @ Bs0
        R = P.T @ Gb @ P
        off = np.linalg.norm(R - np.diag(np.diag(R))) / np.linalg.norm(np.diag(R))
        w = np.linalg.eigvalsh(G)
        print(f"half {half} dst {t}: rc {rc} jacobi sweeps {int(sv[0])}  |BsᵀBs-I| {np.abs(Bs0.T @ Bs0 - np.eye(k)).max():.2e} "
              f"|PᵀP-I| {np.abs(P.T @ P - np.eye(k)).max():.2e}  off(PᵀGP) {off:.2e}  eig [{w.min():.4g}, {w.max():.4g}] "
              f"warm |off| {np.linalg.norm((Bs0.T @ Bt0).T @ Gb @ (Bs0.T @ Bt0) - np.diag(np.diag((Bs0.T @ Bt0).T @ Gb @ (Bs0.T @ Bt0)))) / np.linalg.norm(np.diag(R)):.2e}"
              + (f"  FAILED: {msg}" if rc else ""), flush=True)
        if rc:
            os.makedirs(os.path.dirname(os.path.abspath(args.out)), exist_ok=True)
            np.savez(args.out, G=G, Bs0=Bs0, Bt0=Bt0, Bt1=Bt1, half=half)
            return 1
    return 0


if __name__ == "__main__":
    sys.exit(main())
