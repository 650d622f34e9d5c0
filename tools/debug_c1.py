"""Diagnostic (GPU box): the albedo-protocol stand-in of tests/test_gpu_heavy_tail.py
(3000 x 800, 40k stars, rank 50) half-sweep by half-sweep through the C ABI.  After every half the
device factors are compared with the fp64 oracle half-sweep from the device's own src factors, and
the Gram's device eigensolve with numpy's; the first failing half prints the engine's message.

    python tools/debug_c1.py [--halves 52]
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
    ap.add_argument("--halves", type=int, default=52)
    ap.add_argument("--rank", type=int, default=50)
    args = ap.parse_args()
    from albedo_amd import _lib as L
    from albedo_amd import builder
    from oracle import spark_als as O
    from tests.test_gpu_parity import Ctx
    lib = L.load()
    k = args.rank
    stars = builder.load_raw_starring(3000, 800, 40000, 42)
    B = O.make_blocks(stars["user_id"], stars["repo_id"], stars["starring"].astype(np.float32))
    su, si = O.spark_side_seeds(42)
    c = Ctx(lib, k)
    c.ratings(stars["user_id"], stars["repo_id"], stars["starring"].astype(np.float32))
    c.inject(0, B.user_ids, O.spark_initialize(B.user_ids, k, su))
    c.inject(1, B.item_ids, O.spark_initialize(B.item_ids, k, si))
    for h in range(args.halves):
        side = 1 - (h % 2)  # item half first
        _, src = c.factors(1 - side)
        try:
            c.half(side)
        except Exception as e:  # noqa: BLE001
            print(f"half {h} (dst side {side}) FAILED: {e}", flush=True)
            G = src.astype(np.float64).T @ src.astype(np.float64)
            w = np.linalg.eigvalsh(G)
            print("  src Gram eig min/max", w.min(), w.max(), "finite src", bool(np.isfinite(src).all()),
                  "max |src|", float(np.abs(src).max()), flush=True)
            gw = np.zeros(k)
            gv = np.zeros((k, k))
            sw = np.zeros(1, np.int32)
            w0 = np.eye(k)
            L.check(lib.als_device_eigh(0, k, L.ptr(np.ascontiguousarray(G), C.c_double),
                                        L.ptr(w0, C.c_double), L.ptr(gw, C.c_double), L.ptr(gv, C.c_double),
                                        L.ptr(sw, C.c_int32)))
            print("  device eig (cold) vs numpy: max |dw| / max w", float(np.abs(np.sort(gw) - w).max() / w.max()),
                  "sweeps", int(sw[0]), flush=True)
            return 1
        ptr, col, val = (B.i_ptr, B.i_col, B.i_val) if side == 1 else (B.u_ptr, B.u_col, B.u_val)
        ref = O.half_sweep(src, ptr, col, val, reg=0.5, alpha=40.0)
        _, got = c.factors(side)
        num = np.max(np.abs(got.astype(np.float64) - ref), axis=1)
        den = np.maximum(np.max(np.abs(ref), axis=1), 1e-30)
        worst = int(np.argmax(num / den))
        print(f"half {h} side {side}: row rel {float((num / den).max()):.3e} (row {worst}, degree "
              f"{int(ptr[worst + 1] - ptr[worst])}), finite {bool(np.isfinite(got).all())}", flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
