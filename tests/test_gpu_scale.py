"""Full-size parity at the BASELINE configs the bench measures:

  c2   1M users x 200k repos, 50M stars, rank 64: sampled rows of one sweep against the fp64 solve
  c3   c2 after 10 sweeps from Spark-style init + recommendForAllUsers(30) over all 1M users
       (ALSRecommender.scala:43-58, BoundedPriorityQueue.scala:45-53): ids and F2J score bits of 2,000
       sampled users AND of every user the certification sent to the exact rescan, against the
       C/OpenMP F2J oracle; NDCG@30 of the albedo protocol (ALSRecommenderBuilder.scala:77-104)
       identical to the oracle lists' within 1e-3
  c4   20M x 4M, 1B stars, rank 128: sampled rows (the 10^6-star repos included) of one sweep, then the
       same top-30 check on converged factors (20 sweeps: the state the driver's bench scores)

One engine context per config is shared by that config's tests (module fixtures; the ingest is the
slow part), so the tests of a config run in file order.
"""
import ctypes as C

import numpy as np
import pytest

from oracle import cbind
from oracle import spark_als as O
from tests.test_gpu_parity import Ctx, _check_rows_fp64, _gram_fp64

pytestmark = pytest.mark.gpu


def _ingest(gpu_lib, name, rank):
    from albedo_amd import _lib as L
    from albedo_amd.synthetic import CONFIGS, popularity_table, user_degrees
    spec = CONFIGS[name]
    c = Ctx(gpu_lib, rank)
    deg = user_degrees(spec)
    prefix = np.ascontiguousarray(np.r_[0, np.cumsum(deg)].astype(np.int64))
    del deg
    cw, perm = popularity_table(spec)
    L.check(gpu_lib.als_set_ratings_synthetic(c.h, spec.seed, spec.rounds, spec.n_users, spec.n_items,
                                              L.ptr(prefix, C.c_int64), L.ptr(np.ascontiguousarray(cw), C.c_double),
                                              L.ptr(np.ascontiguousarray(perm), C.c_int32)))
    assert gpu_lib.als_num_ratings(c.h) > 0.99 * spec.nnz
    L.check(gpu_lib.als_init_factors(c.h))
    return c


@pytest.fixture(scope="module")
def c2_ctx(gpu_lib):
    c = _ingest(gpu_lib, "c2", 64)
    yield c
    del c


@pytest.fixture(scope="module")
def c4_ctx(gpu_lib):
    c = _ingest(gpu_lib, "c4", 128)
    yield c
    del c


def _sweeps(c, n):
    c.L.check(c.lib.als_run_sweeps(c.h, n))


def _topk_all_and_check(gpu_lib, c, k, n_sample, max_rescan, seed, albedo_protocol=False):
    """recommendForAllUsers(k) on the engine; the sampled users and the exact-rescan users equal the
    oracle bit for bit.  Returns (rescan count, checked rows, scan stats)."""
    from albedo_amd import _lib as L
    n_u = gpu_lib.als_num_rows(c.h, 0)
    st0 = np.zeros(4, np.int64)
    L.check(gpu_lib.als_topk_stats(c.h, L.ptr(st0, C.c_int64)))
    ids = np.empty((n_u, k), np.int32)
    sc = np.empty((n_u, k), np.float32)
    L.check(gpu_lib.als_recommend(c.h, 0, k, None, n_u, None, L.ptr(ids, C.c_int32), L.ptr(sc, C.c_float)))
    st1 = np.zeros(4, np.int64)
    L.check(gpu_lib.als_topk_stats(c.h, L.ptr(st1, C.c_int64)))
    n_res = np.zeros(1, np.int64)
    L.check(gpu_lib.als_topk_last_rescan(c.h, None, 0, L.ptr(n_res, C.c_int64)))
    resc = np.empty(max(int(n_res[0]), 1), np.int32)
    L.check(gpu_lib.als_topk_last_rescan(c.h, L.ptr(resc, C.c_int32), resc.size, L.ptr(n_res, C.c_int64)))
    resc = resc[:int(n_res[0])]
    assert st1[1] - st0[1] == resc.size
    uids, U = c.factors(0)
    iids, V = c.factors(1)
    rng = np.random.default_rng(seed)
    rows = np.sort(rng.choice(n_u, n_sample, replace=False))
    rrows = np.searchsorted(uids, resc)
    assert np.array_equal(uids[rrows], resc)
    if rrows.size > max_rescan:
        rrows = np.sort(rng.choice(rrows, max_rescan, replace=False))
    rows = np.union1d(rows, rrows)
    ref_ids, ref_sc = cbind.recommend(U[rows], iids, V, k)
    bad = np.nonzero(np.any(ids[rows] != ref_ids, axis=1) | np.any(sc[rows].view(np.uint32) != ref_sc.view(np.uint32), axis=1))[0]
    assert bad.size == 0, (f"{bad.size} of {rows.size} rows differ from the oracle, e.g. user {uids[rows[bad[0]]]}: "
                           f"{ids[rows[bad[0]]][:5]} vs {ref_ids[bad[0]][:5]}")
    out = dict(rescan=int(resc.size), checked=int(rows.size), scanned_frac=float(st1[2] - st0[2]) / max(1, int(st1[3] - st0[3])))
    if albedo_protocol:
        # ALSRecommenderBuilder.scala:65-104: 250 test users + 1, predicted = top-k by score, actual =
        # the user's k most recent stars (synthetic per-star timestamps: a hash of the pair)
        from albedo_amd import evaluation as E
        test = np.sort(rng.choice(n_u, 251, replace=False))
        n_row = np.empty(1, np.int64)
        users, items = [], []
        for r in test:
            uid = int(uids[r])
            L.check(gpu_lib.als_get_row_ratings(c.h, 0, uid, 0, None, None, L.ptr(n_row, C.c_int64)))
            src = np.empty(max(int(n_row[0]), 1), np.int32)
            L.check(gpu_lib.als_get_row_ratings(c.h, 0, uid, src.size, L.ptr(src, C.c_int32), None,
                                                L.ptr(n_row, C.c_int64)))
            users.append(np.full(int(n_row[0]), uid, np.int32))
            items.append(src[:int(n_row[0])])
        users, items = np.concatenate(users), np.concatenate(items)
        ts = ((users.astype(np.uint64) * np.uint64(0x9E3779B1) + items.astype(np.uint64) * np.uint64(0x85EBCA77))
              % np.uint64(300_000_000)).astype(np.int64)
        actual = E.into_user_items(users, items, ts, k)
        o_ids, _ = cbind.recommend(U[test], iids, V, k)
        pred_gpu = {int(uids[r]): [int(x) for x in ids[r] if x >= 0] for r in test}
        pred_ref = {int(uids[r]): [int(x) for x in o_ids[n] if x >= 0] for n, r in enumerate(test)}
        n_gpu = E.RankingEvaluator(actual, "NDCG@k", k).evaluate(pred_gpu)
        n_ref = O.evaluate_ndcg(pred_ref, actual, k)
        assert abs(n_gpu - n_ref) <= 1e-3
        out["ndcg"] = (n_gpu, n_ref)
    return out


@pytest.mark.timeout(400)
def test_c2_scale_rows_match_fp64_solve(gpu_lib, c2_ctx):
    """Full-size property at BASELINE config 2 (1M x 200k, 50M nnz, rank 64): after an item and a
    user half-sweep from Spark-style init, sampled rows of every degree bucket -- and the 10 most
    starred repos (the power-law tail, 10^5 stars) -- equal the fp64 solution of Spark's normal
    equation built on the host from the engine's own inputs."""
    from albedo_amd import _lib as L
    c = c2_ctx
    uids, U0 = c.factors(0)
    c.half(1)
    iids, V = c.factors(1)
    deg = np.empty(iids.size, np.int64)
    L.check(gpu_lib.als_get_degrees(c.h, 1, L.ptr(deg, C.c_int64)))
    top = iids[np.argsort(-deg, kind="stable")[:10]]
    assert deg.max() > 100_000  # the tail this arm is about
    rng = np.random.default_rng(1)
    _check_rows_fp64(gpu_lib, c, 1, np.r_[top, rng.choice(iids, 100, replace=False)], iids, V, uids, U0, 64)
    c.half(0)
    st = c.stats(0)
    assert st[0] > 0 and st[2] > 0  # both solve paths ran
    _, U = c.factors(0)
    rng = np.random.default_rng(0)
    _check_rows_fp64(gpu_lib, c, 0, uids[rng.choice(len(uids), 200, replace=False)], uids, U, iids, V, 64)


@pytest.mark.timeout(400)
def test_c2_two_contexts_bit_identical(gpu_lib):
    """Run-to-run identity at BASELINE config 2 (1M users x 200k repos, 50M stars, rank 64): two
    contexts ingest the same synthetic ratings and run the same item and user half-sweeps side by
    side; every factor is bit-identical.  (r05: the paired light16 rows -- 600K users of degree <= 8
    here -- gave ~150 rows 5-55 % off in one context or the other, a different set each run; see
    tools/determinism.py.)"""
    a = _ingest(gpu_lib, "c2", 64)
    b = _ingest(gpu_lib, "c2", 64)
    for side in (1, 0, 1, 0):
        a.half(side)
        b.half(side)
        fa, fb = a.factors(side)[1], b.factors(side)[1]
        bad = np.nonzero(np.any(fa.view(np.uint32) != fb.view(np.uint32), axis=1))[0]
        assert bad.size == 0, f"side {side}: {bad.size} rows differ between two identical runs, e.g. row {bad[0]}"


@pytest.mark.timeout(400)
def test_c3_topk_all_users_after_10_sweeps(gpu_lib, c2_ctx):
    """BASELINE config 3: the c2 fit at 10 sweeps (this module's previous test ran the first), then
    recommendForAllUsers(30) over all 1M users: 2,000 sampled users plus every exact-rescan user are
    bit-exact against the oracle, and the albedo-protocol NDCG@30 matches."""
    c = c2_ctx
    _sweeps(c, 9)
    r = _topk_all_and_check(gpu_lib, c, 30, 2000, 10 ** 6, seed=3, albedo_protocol=True)
    print("c3 top-30:", r)


def _recommend_all(gpu_lib, c, k):
    from albedo_amd import _lib as L
    n_u = gpu_lib.als_num_rows(c.h, 0)
    ids = np.empty((n_u, k), np.int32)
    sc = np.empty((n_u, k), np.float32)
    L.check(gpu_lib.als_recommend(c.h, 0, k, None, n_u, None, L.ptr(ids, C.c_int32), L.ptr(sc, C.c_float)))
    n_res = np.zeros(1, np.int64)
    L.check(gpu_lib.als_topk_last_rescan(c.h, None, 0, L.ptr(n_res, C.c_int64)))
    resc = np.empty(max(int(n_res[0]), 1), np.int32)
    L.check(gpu_lib.als_topk_last_rescan(c.h, L.ptr(resc, C.c_int32), resc.size, L.ptr(n_res, C.c_int64)))
    return ids, sc, np.sort(resc[:int(n_res[0])])


@pytest.mark.timeout(400)
def test_c3_topk_passes_and_ranges_identical(gpu_lib, c2_ctx, monkeypatch):
    """recommendForAllUsers(30) over the 1M c3 users in one pass (the default: one scan launch, the
    results finished and copied out in ranges) and in passes of 300K rows (ALBEDO_TOPK_PASS; four
    passes, each finished in four 64K-row ranges plus a remainder): the same lists and the same score
    bits (which rows need the exact rescan may differ: a row's scan workgroup, and so the chunks it is
    scored against, depends on the pass it sorts in)."""
    c = c2_ctx
    ids1, sc1, r1 = _recommend_all(gpu_lib, c, 30)
    monkeypatch.setenv("ALBEDO_TOPK_PASS", "300000")
    ids2, sc2, r2 = _recommend_all(gpu_lib, c, 30)
    assert np.array_equal(ids1, ids2)
    assert np.array_equal(sc1.view(np.uint32), sc2.view(np.uint32))
    print("c3 rescans: one pass", r1.size, "300K-row passes", r2.size)


@pytest.mark.timeout(600)
def test_c4_scale_rows_match_fp64_solve(gpu_lib, c4_ctx):
    """Full-size property at BASELINE config 4 (20M x 4M, 1B stars, rank 128; the bench workload):
    after an item and a user half-sweep from Spark-style init, the three most starred repos
    (10^6+ stars: split-K builds), random repo and user rows equal the fp64 solution of Spark's
    normal equation built on the host from the engine's own CSR (the Gram of the 20M user rows
    accumulated in fp64 over row chunks)."""
    from albedo_amd import _lib as L
    c = c4_ctx
    uids, U0 = c.factors(0)
    c.half(1)
    iids, V = c.factors(1)
    ideg = np.empty(iids.size, np.int64)
    L.check(gpu_lib.als_get_degrees(c.h, 1, L.ptr(ideg, C.c_int64)))
    top = iids[np.argsort(-ideg, kind="stable")[:3]]
    assert ideg.max() > 1_000_000
    rng = np.random.default_rng(4)
    _check_rows_fp64(gpu_lib, c, 1, np.r_[top, rng.choice(iids, 30, replace=False)], iids, V, uids, U0, 128,
                     gram=_gram_fp64(U0))
    del U0
    c.half(0)
    _, U = c.factors(0)
    _check_rows_fp64(gpu_lib, c, 0, uids[rng.choice(len(uids), 100, replace=False)], uids, U, iids, V, 128)


@pytest.mark.timeout(900)
def test_c4_topk_converged_factors(gpu_lib, c4_ctx):
    """On factors after 20 sweeps (the driver's bench scores top-k after 25): the 20th sweep's item
    half -- the three most starred repos (10^6+ stars, split-K), 20 rows of degree 65-128 (the rows
    nearest the light limit on the wave kernel) and 30 random repos -- and 200 user rows of its user
    half equal the fp64 solve of Spark's normal equation built from the engine's own CSR and src
    factors; then top-30 over all 20M users, 2,000 sampled users plus 2,000 of the exact-rescan users
    (all of them when fewer) bit-exact against the oracle."""
    from albedo_amd import _lib as L
    c = c4_ctx
    _sweeps(c, 18)
    uids, U19 = c.factors(0)
    c.half(1)
    iids, V = c.factors(1)
    ideg = np.empty(iids.size, np.int64)
    L.check(gpu_lib.als_get_degrees(c.h, 1, L.ptr(ideg, C.c_int64)))
    rng = np.random.default_rng(19)
    top = iids[np.argsort(-ideg, kind="stable")[:3]]
    mid = rng.choice(iids[(ideg > 64) & (ideg <= 128)], 20, replace=False)
    worst = _check_rows_fp64(gpu_lib, c, 1, np.r_[top, mid, rng.choice(iids, 30, replace=False)], iids, V, uids, U19,
                             128)
    print(f"c4 sweep-20 item rows: worst rel err {worst:.2e}")
    del U19
    c.half(0)
    uids, U = c.factors(0)
    rng = np.random.default_rng(20)
    worst = _check_rows_fp64(gpu_lib, c, 0, uids[rng.choice(len(uids), 200, replace=False)], uids, U, iids, V, 128)
    print(f"c4 sweep-20 user rows: worst rel err {worst:.2e}")
    del U, V
    r = _topk_all_and_check(gpu_lib, c, 30, 2000, 2000, seed=4)
    print("c4 top-30:", r)
