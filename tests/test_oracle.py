"""CPU oracle checks: known answers from Spark's own test suites, LAPACK, scipy, the C restatement
and the committed golden fixtures (the oracle is test infrastructure; see oracle/__init__.py)."""
import os

import numpy as np
import pytest
import scipy.optimize

from oracle import cbind
from oracle import spark_als as O
from tests.conftest import GOLDEN


def test_ndcg_known_answers():
    # mllib RankingMetricsSuite (Spark 2.2.0): the three-user fixture and its published values
    pairs = [([1, 6, 2, 7, 8, 3, 9, 10, 4, 5], [1, 2, 3, 4, 5]),
             ([4, 1, 5, 6, 2, 7, 3, 8, 9, 10], [1, 2, 3]),
             ([1, 2, 3, 4, 5], [])]
    assert O.ndcg_at(pairs, 3) == pytest.approx(1.0 / 3, abs=1e-8)
    assert O.ndcg_at(pairs, 5) == pytest.approx(0.328788, abs=1e-6)
    assert O.ndcg_at(pairs, 10) == pytest.approx(0.487913, abs=1e-6)
    assert O.ndcg_at(pairs, 15) == pytest.approx(0.487913, abs=1e-6)
    with pytest.raises(ValueError):
        O.ndcg_at(pairs, 0)


def test_product_ndcg_matches_oracle():
    from albedo_amd import evaluation as E
    rng = np.random.default_rng(0)
    pairs = [(list(rng.permutation(50)[:30]), list(rng.permutation(50)[: rng.integers(0, 40)])) for _ in range(40)]
    for k in (1, 5, 30):
        assert E.ndcg_at(pairs, k) == pytest.approx(O.ndcg_at(pairs, k), abs=1e-12)


def test_cholesky_is_lapack_dppsv():
    rng = np.random.default_rng(1)
    for k in (1, 8, 50):
        M = rng.standard_normal((k + 3, k))
        A = M.T @ M
        b = rng.standard_normal(k)
        x = O.cholesky_solve(A, b, 0.3)
        ref = np.linalg.solve(A + 0.3 * np.eye(k), b)
        assert np.allclose(x, ref.astype(np.float32), rtol=1e-5, atol=1e-6)
    with pytest.raises(O.NotPositiveDefinite):
        O.cholesky_solve(np.zeros((4, 4)), np.ones(4), 0.0)


def test_nnls_reaches_scipy_optimum():
    rng = np.random.default_rng(2)
    for n in (4, 16, 32):
        M = rng.standard_normal((3 * n, n))
        y = rng.standard_normal(3 * n)
        A, b = M.T @ M, M.T @ y
        x = O.nnls(A, b)
        ref, _ = scipy.optimize.nnls(M, y)
        assert np.all(x >= 0)
        assert np.allclose(x, ref, rtol=1e-6, atol=1e-6)


def test_f2j_sdot_is_sequential_float32():
    rng = np.random.default_rng(3)
    x = rng.standard_normal((5, 23)).astype(np.float32)
    y = rng.standard_normal((5, 23)).astype(np.float32)
    got = O.f2j_sdot(x, y)
    for r in range(5):
        acc = np.float32(0)
        for i in range(23):
            acc = np.float32(acc + np.float32(x[r, i] * y[r, i]))
        assert got[r] == acc


def test_bounded_priority_queue_matches_sorted_topk():
    rng = np.random.default_rng(4)
    scores = rng.integers(0, 20, size=200).astype(np.float32)  # many ties
    ids = np.arange(200)
    q = O.BoundedPriorityQueue(10, key=lambda e: e[1])
    for i in ids:  # ascending id order: first seen = lower id
        q.add((int(i), float(scores[i])))
    kept = sorted(q.items(), key=lambda e: (-e[1], e[0]))
    order = np.lexsort((ids, -scores))[:10]
    assert [e[0] for e in kept] == list(order)


def test_numpy_oracle_matches_c_oracle():
    from albedo_amd.synthetic import SynthSpec, generate
    d = generate(SynthSpec(300, 120, 3000, seed=5))
    B = O.make_blocks(d["user"], d["item"], d["rating"])
    rng = np.random.default_rng(5)
    for implicit in (True, False):
        Y = rng.standard_normal((len(B.user_ids), 12)).astype(np.float32)
        a = O.half_sweep(Y, B.i_ptr, B.i_col, B.i_val, reg=0.5, alpha=40.0, implicit=implicit)
        b = cbind.half_sweep(Y, B.i_ptr, B.i_col, B.i_val, reg=0.5, alpha=40.0, implicit=implicit)
        assert np.allclose(a, b, rtol=1e-6, atol=1e-7)
    assert np.allclose(cbind.gram(Y), O.gram(Y), rtol=1e-12)


def _load(name):
    return np.load(os.path.join(GOLDEN, name))


def test_oracle_reproduces_golden_f1_f2():
    f = _load("f1_half_sweep.npz")
    B = O.make_blocks(f["user"], f["item"], f["rating"])
    for k in (8, 16):
        V = O.half_sweep(f[f"U0_k{k}"], B.i_ptr, B.i_col, B.i_val, reg=0.5, alpha=40.0)
        assert np.array_equal(V, f[f"V_k{k}"])
    f = _load("f2_three_sweeps.npz")
    B = O.make_blocks(f["user"], f["item"], f["rating"])
    U, V = O.fit(B, rank=16, max_iter=3, reg=0.5, alpha=40.0, init_user=f["U0"], init_item=f["V0"])
    assert np.array_equal(U, f["U"]) and np.array_equal(V, f["V"])


def test_oracle_reproduces_golden_topk():
    f = _load("f4_topk_ties.npz")
    ids, sc = O.recommend_for_all(f["uid"], f["uf"], f["iid"], f["itf"], 30)
    assert np.array_equal(ids, f["ids30"]) and np.array_equal(sc, f["sc30"])


def test_into_user_items_rank_keeps_ties():
    from albedo_amd import evaluation as E
    user = np.array([1, 1, 1, 1, 2, 2])
    item = np.array([10, 11, 12, 13, 20, 21])
    key = np.array([5.0, 7.0, 7.0, 1.0, 3.0, 3.0])
    a = O.into_user_items(user, item, key, 1)
    b = E.into_user_items(user, item, key, 1)
    assert a == b == {1: [11, 12], 2: [20, 21]}


def test_synthetic_generator_shape():
    from albedo_amd.synthetic import SynthSpec, generate, user_degrees
    spec = SynthSpec(2000, 400, 30000, seed=9)
    d = generate(spec)
    key = d["user"].astype(np.int64) * (1 << 31) + d["item"]
    assert np.unique(key).size == key.size  # unique (user, repo) pairs, like app/models.py:166-167
    assert user_degrees(spec).sum() == spec.nnz
    assert key.size >= 0.99 * spec.nnz
    assert np.all(d["rating"] == 1.0)


def test_c_topk_oracle_matches_numpy_oracle_and_golden():
    """The C/OpenMP scorer (full-size parity checks) equals the numpy restatement bit for bit:
    golden F4 (engineered ties), a catalogue that is not a multiple of the 64-row block, duplicate
    rows (equal scores, id tie-break), k above the catalogue size."""
    f = _load("f4_topk_ties.npz")
    for num in (30, 60):
        ids, sc = cbind.recommend(f["uf"], f["iid"], f["itf"], num)
        assert np.array_equal(ids, f[f"ids{num}"]) and np.array_equal(sc.view(np.uint32), f[f"sc{num}"].view(np.uint32))
    rng = np.random.default_rng(3)
    n_i, k = 1000, 37
    iid = rng.permutation(np.arange(n_i, dtype=np.int32) * 7 - 300)
    itf = (rng.standard_normal((n_i, k)) * rng.lognormal(0, 1, (n_i, 1))).astype(np.float32)
    itf[500:540] = itf[:40]
    uf = rng.standard_normal((45, k)).astype(np.float32)
    for num in (1, 30, 64):
        a = O.recommend_for_all(np.arange(45), uf, iid, itf, num)
        b = cbind.recommend(uf, iid, itf, num, threads=3)
        assert np.array_equal(a[0], b[0]) and np.array_equal(a[1].view(np.uint32), b[1].view(np.uint32))
    a = O.recommend_for_all(np.arange(5), uf[:5], iid[:20], itf[:20], 30)
    b = cbind.recommend(uf[:5], iid[:20], itf[:20], 30)
    assert np.array_equal(a[0], b[0]) and np.array_equal(a[1][:, :20], b[1][:, :20]) and np.all(np.isnan(b[1][:, 20:]))


def test_c_nnls_matches_numpy_nnls_on_f5():
    """The C/OpenMP NNLSSolver restatement (oracle/c/als_cpu.c, the c5 bench's cpu_baseline) equals the
    numpy restatement of NNLS.scala (oracle/spark_als.py:nnls) on the F5 golden rows: the committed
    item half-sweep V1 from U0, and the user half-sweep from V1, row by row."""
    f = _load("f5_nnls.npz")
    B = O.make_blocks(f["user"], f["item"], f["rating"])
    U0 = f["U0"].astype(np.float32)
    V, it = cbind.solve_rows_nnls(U0, O.gram(U0), B.i_ptr, B.i_col, B.i_val, reg=0.5, alpha=40.0, threads=4)
    assert np.all(V >= 0) and np.all(it > 0)
    assert np.allclose(V, f["V1"], rtol=1e-6, atol=1e-7)
    U, _ = cbind.solve_rows_nnls(V, O.gram(V), B.u_ptr, B.u_col, B.u_val, reg=0.5, alpha=40.0, threads=3)
    U_ref = O.half_sweep(V, B.u_ptr, B.u_col, B.u_val, reg=0.5, alpha=40.0, nonnegative=True)
    assert np.allclose(U, U_ref, rtol=1e-6, atol=1e-7)
    assert np.mean((U == 0) == (U_ref == 0)) == 1.0
