"""Regenerate the committed golden fixtures from the CPU oracle (oracle/spark_als.py).

The reference (Spark MLlib 2.2.0 via albedo) has no tests or fixtures of its own and cannot run
here, so these vectors are produced by the oracle restatement; they pin the
oracle against regressions and give the GPU tests fixed inputs/outputs.
Run: python tests/golden/make_golden.py
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from albedo_amd.synthetic import SynthSpec, generate  # noqa: E402
from oracle import spark_als as O  # noqa: E402

OUT = os.path.dirname(os.path.abspath(__file__))


def init(n, k, seed):
    rng = np.random.default_rng(seed)
    f = rng.standard_normal((n, k)).astype(np.float32)
    return (f / np.linalg.norm(f, axis=1, keepdims=True)).astype(np.float32)


def f1_half_sweep():
    d = generate(SynthSpec(2000, 500, 20000, seed=11))
    B = O.make_blocks(d["user"], d["item"], d["rating"])
    out = {"user": d["user"], "item": d["item"], "rating": d["rating"]}
    for k in (8, 16):
        U0 = init(len(B.user_ids), k, 100 + k)
        V = O.half_sweep(U0, B.i_ptr, B.i_col, B.i_val, reg=0.5, alpha=40.0, implicit=True)
        out[f"U0_k{k}"] = U0
        out[f"V_k{k}"] = V
        out[f"G_k{k}"] = O.gram(U0)
    np.savez_compressed(os.path.join(OUT, "f1_half_sweep.npz"), **out)


def f2_three_sweeps():
    d = generate(SynthSpec(1500, 400, 15000, seed=12))
    B = O.make_blocks(d["user"], d["item"], d["rating"])
    k = 16
    U0, V0 = init(len(B.user_ids), k, 1), init(len(B.item_ids), k, 2)
    U, V = O.fit(B, rank=k, max_iter=3, reg=0.5, alpha=40.0, implicit=True, init_user=U0, init_item=V0)
    np.savez_compressed(os.path.join(OUT, "f2_three_sweeps.npz"), user=d["user"], item=d["item"],
                        rating=d["rating"], U0=U0, V0=V0, U=U, V=V)


def f3_explicit():
    rng = np.random.default_rng(13)
    d = generate(SynthSpec(800, 300, 8000, seed=13))
    r = rng.integers(1, 6, size=d["user"].size).astype(np.float32)
    B = O.make_blocks(d["user"], d["item"], r)
    k = 10
    U0, V0 = init(len(B.user_ids), k, 3), init(len(B.item_ids), k, 4)
    U, V = O.fit(B, rank=k, max_iter=2, reg=0.1, alpha=1.0, implicit=False, init_user=U0, init_item=V0)
    np.savez_compressed(os.path.join(OUT, "f3_explicit.npz"), user=d["user"], item=d["item"], rating=r,
                        U0=U0, V0=V0, U=U, V=V)


def f4_topk_ties():
    rng = np.random.default_rng(14)
    k = 12
    nu, ni = 300, 900
    uf = rng.standard_normal((nu, k)).astype(np.float32)
    itf = rng.standard_normal((ni, k)).astype(np.float32)
    itf[1::7] = itf[0::7][: len(itf[1::7])]          # duplicate item rows -> exact score ties
    itf[5] = itf[600]
    uid = rng.permutation(10 * nu)[:nu].astype(np.int32) - 50
    iid = rng.permutation(10 * ni)[:ni].astype(np.int32) - 100
    ids30, sc30 = O.recommend_for_all(uid, uf, iid, itf, 30)
    ids60, sc60 = O.recommend_for_all(uid, uf, iid, itf, 60)
    np.savez_compressed(os.path.join(OUT, "f4_topk_ties.npz"), uid=uid, uf=uf, iid=iid, itf=itf,
                        ids30=ids30, sc30=sc30, ids60=ids60, sc60=sc60)


def f6_zero_and_negative():
    d = generate(SynthSpec(600, 200, 5000, seed=15))
    rng = np.random.default_rng(15)
    r = d["rating"].copy()
    users = np.unique(d["user"])
    zero_users = users[:20]
    r[np.isin(d["user"], zero_users)] = 0.0            # rows with no positive rating (λ·n = 0)
    neg = rng.random(r.size) < 0.05
    r[neg] = -1.0                                      # negative ratings: c = α|r|, preference 0
    B = O.make_blocks(d["user"], d["item"], r)
    k = 8
    V0 = init(len(B.item_ids), k, 5)
    U = O.half_sweep(V0, B.u_ptr, B.u_col, B.u_val, reg=0.5, alpha=40.0, implicit=True)
    np.savez_compressed(os.path.join(OUT, "f6_zero_negative.npz"), user=d["user"], item=d["item"], rating=r,
                        V0=V0, U=U)


def f7_heavy_row():
    rng = np.random.default_rng(16)
    n_items = 12000
    heavy = np.full(11000, 7, dtype=np.int32)         # one user starring 11000 repos
    hi = rng.permutation(n_items)[:11000].astype(np.int32)
    d = generate(SynthSpec(500, n_items, 6000, seed=16))
    user = np.concatenate([d["user"], heavy])
    item = np.concatenate([d["item"], hi])
    key = user.astype(np.int64) * (1 << 31) + item
    _, uniq = np.unique(key, return_index=True)
    user, item = user[np.sort(uniq)], item[np.sort(uniq)]
    r = np.ones(user.size, dtype=np.float32)
    B = O.make_blocks(user, item, r)
    k = 16
    V0 = init(len(B.item_ids), k, 6)
    U = O.half_sweep(V0, B.u_ptr, B.u_col, B.u_val, reg=0.5, alpha=40.0, implicit=True)
    np.savez_compressed(os.path.join(OUT, "f7_heavy_row.npz"), user=user, item=item, rating=r, V0=V0, U=U)


def f5_nnls():
    d = generate(SynthSpec(700, 220, 7000, seed=17))
    B = O.make_blocks(d["user"], d["item"], d["rating"])
    k = 16
    U0 = np.abs(init(len(B.user_ids), k, 7))
    V0 = np.abs(init(len(B.item_ids), k, 8))
    V1 = O.half_sweep(U0, B.i_ptr, B.i_col, B.i_val, reg=0.5, alpha=40.0, implicit=True, nonnegative=True)
    U, V = O.fit(B, rank=k, max_iter=2, reg=0.5, alpha=40.0, implicit=True, nonnegative=True,
                 init_user=U0, init_item=V0)
    np.savez_compressed(os.path.join(OUT, "f5_nnls.npz"), user=d["user"], item=d["item"], rating=d["rating"],
                        U0=U0, V0=V0, V1=V1, U=U, V=V)


if __name__ == "__main__":
    f5_nnls()
    f1_half_sweep()
    f2_three_sweeps()
    f3_explicit()
    f4_topk_ties()
    f6_zero_and_negative()
    f7_heavy_row()
    for f in sorted(os.listdir(OUT)):
        if f.endswith(".npz"):
            print(f, os.path.getsize(os.path.join(OUT, f)))
