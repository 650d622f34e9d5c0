"""numpy restatement of eig.hip's device eigensolver (cyclic parallel Jacobi, round-robin pairs,
stopping rule JAC_TOL / rounding floor), for offline analysis of dumped systems (tools/debug_eig.py)
and CPU tests of the algorithm.  Same rotations and order; the 2x2 block products are numpy
matrix products, so roundings differ from the device in the last bits.
"""
import numpy as np

JAC_TOL = 1e-28
JAC_MAX_SWEEPS = 30


def rr_pair(r, i, n):
    m = n - 1
    if i == 0:
        a, b = r % m, m
    else:
        a, b = (r + i) % m, (r - i + m) % m
    return (a, b) if a < b else (b, a)


def jacobi(M, VT=None, tol=JAC_TOL, max_sweeps=JAC_MAX_SWEEPS, trace=None):
    """M (k x k symmetric) -> (w, VT, sweeps) with VT·M_in·VTᵀ ≈ diag(w) (VT starts from the given
    rows, e.g. Wᵀ of a warm start, and accumulates the rotations)."""
    M = np.array(M, np.float64)
    k = M.shape[0]
    VT = np.eye(k) if VT is None else np.array(VT, np.float64)
    n = k + (k & 1)
    npairs = n // 2
    prev = np.inf
    sweep = 0
    for sweep in range(max_sweeps):
        d = np.diag(M)
        dia = float(np.sum(d * d))
        off = float(np.sum((M - np.diag(d)) ** 2))  # the off-diagonal entries themselves (no cancellation)
        if trace is not None:
            trace.append(off / dia if dia > 0 else 0.0)
        done = not (off > tol * dia) or (not (off > 1e-20 * dia) and not (off < 0.5 * prev))
        prev = off
        if done:
            break
        for r in range(n - 1):
            J = np.eye(k)
            for i in range(npairs):
                p, q = rr_pair(r, i, n)
                if q >= k:
                    continue
                apq = M[p, q]
                c, s = 1.0, 0.0
                if apq != 0.0:
                    with np.errstate(over="ignore"):
                        th = (M[q, q] - M[p, p]) / (2.0 * apq)
                        t = (1.0 if th >= 0.0 else -1.0) / (abs(th) + np.sqrt(th * th + 1.0))
                    c = 1.0 / np.sqrt(t * t + 1.0)
                    s = t * c
                J[p, p] = c
                J[q, q] = c
                J[p, q] = s
                J[q, p] = -s
            M = J.T @ M @ J
            VT = J.T @ VT
    return np.diag(M).copy(), VT, sweep
