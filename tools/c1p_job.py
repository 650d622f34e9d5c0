"""The albedo job (ALSRecommenderBuilder.scala:40-105) end to end at the c1' stand-in scale, timed
per stage, with a sampled parity check.  GPU box only; writes one JSON record.

    python tools/c1p_job.py [--out gpurun_out/c1p_job.json] [--dir /tmp/albedo_c1p]

c1' = SURVEY.md §8(d): 1M users x 200k repos, 50M stars, rank 50, maxIter 26, alpha 40, regParam 0.5,
seed 42 (the albedo.sql dump is not available offline).  Stages:
  create   the parquet Starring dataset (the JDBC read's stand-in, DatasetUtils.scala:111-123):
           device generator -> (user_id, repo_id, starred_at, starring = 1.0) -> parquet parts
  read     loadRawStarringDS = read_starring of the parquet directory (DatasetUtils.scala:36-50)
  ingest   ALS.fit's host -> device copy, id remap and both CSR orientations (als_set_ratings)
  fit      26 sweeps (als_fit)
  save     write().overwrite().save (ModelUtils.scala:7-20, Spark ML layout)
  load     ALSModel.load of that directory
  topk     ALSRecommender.recommendForUsers of 250 sampled test users + the fixed user (:65-84)
  ndcg     intoUserActualItems(30) + RankingEvaluator NDCG@30 (:92-104), on the device
Parity (not timed): the reloaded factors are bit-identical to the fitted ones; 200 user rows of the
last sweep equal the fp64 solve of Spark's normal equation from the item factors and the parquet
rows; the 251 top-30 lists are bit-identical to the oracle scorer (oracle/c, F2J order); NDCG@30
equals the oracle evaluator's.
"""
from __future__ import annotations

import argparse
import ctypes as C
import json
import os
import shutil
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def create(path, spec, workers=16):
    from albedo_amd import _lib as L
    from albedo_amd import persistence
    from albedo_amd.synthetic import popularity_table, user_degrees
    lib = L.load()
    deg = user_degrees(spec)
    prefix = np.ascontiguousarray(np.r_[0, np.cumsum(deg)].astype(np.int64))
    cw, perm = popularity_table(spec)
    n = int(prefix[-1])
    u = np.empty(n, np.int32)
    it = np.empty(n, np.int32)
    r = np.empty(n, np.float32)
    nout = np.zeros(1, np.int64)
    L.check(lib.als_synth_generate(0, spec.seed, spec.rounds, spec.n_users, spec.n_items, L.ptr(prefix, C.c_int64),
                                   L.ptr(np.ascontiguousarray(cw), C.c_double),
                                   L.ptr(np.ascontiguousarray(perm), C.c_int32), L.ptr(u, C.c_int32),
                                   L.ptr(it, C.c_int32), L.ptr(r, C.c_float), L.ptr(nout, C.c_int64)))
    m = int(nout[0])
    u, it = u[:m], it[:m]
    # per-star timestamps: a hash of the pair (deterministic, ties within a user are possible)
    ts = ((u.astype(np.uint64) * np.uint64(0x9E3779B1) + it.astype(np.uint64) * np.uint64(0x85EBCA77))
          % np.uint64(300_000_000)).astype(np.int64) + 1_300_000_000
    def progress(done, total):
        if done % 16 == 0 or done == total:
            print(f"  parquet parts written {done}/{total}", flush=True)

    persistence.write_starring(path, {"user_id": u, "repo_id": it, "starred_at": ts.astype("datetime64[s]"),
                                      "starring": np.ones(m, np.float64)}, rows_per_part=1 << 22,
                               workers=workers, progress=progress)
    return m


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default="gpurun_out/c1p_job.json")
    ap.add_argument("--dir", default="/tmp/albedo_c1p")
    ap.add_argument("--config", default="c1p")
    ap.add_argument("--max-iter", type=int, default=26)
    ap.add_argument("--rank", type=int, default=50)
    ap.add_argument("--ingest-only", action="store_true",
                    help="stop after create / read / ingest (the c4 leg: --config c4 --rank 128 --ingest-only)")
    args = ap.parse_args()
    from albedo_amd import ALS, ALSModel, persistence
    from albedo_amd.builder import sample_test_users
    from albedo_amd.recommenders import ALSRecommender
    from albedo_amd.synthetic import CONFIGS
    from oracle import cbind
    from oracle import spark_als as O

    spec = CONFIGS[args.config]
    T = {}
    rec = {"config": args.config, "users": spec.n_users, "repos": spec.n_items, "rank": args.rank,
           "max_iter": args.max_iter, "alpha": 40.0, "reg_param": 0.5, "seed": 42}
    shutil.rmtree(args.dir, ignore_errors=True)
    os.makedirs(args.dir)
    spath = os.path.join(args.dir, "rawStarringDF.parquet")
    mpath = os.path.join(args.dir, "alsModel.parquet")
    t = time.perf_counter()
    rec["stars"] = create(spath, spec)
    T["create"] = time.perf_counter() - t
    print("created", rec["stars"], "stars", flush=True)

    t = time.perf_counter()
    stars = persistence.read_starring(spath)
    T["read"] = time.perf_counter() - t
    if args.ingest_only:
        args.max_iter = 0
    als = (ALS().setImplicitPrefs(True).setRank(args.rank).setRegParam(0.5).setAlpha(40).setMaxIter(args.max_iter)
           .setSeed(42).setColdStartStrategy("drop").setUserCol("user_id").setItemCol("repo_id")
           .setRatingCol("starring"))
    t = time.perf_counter()
    model = als.fit(stars)
    wall = time.perf_counter() - t
    T["fit"] = model.fit_seconds
    T["ingest"] = wall - model.fit_seconds
    print(f"fit {model.fit_seconds:.2f} s ({args.max_iter} sweeps), ingest {T['ingest']:.2f} s", flush=True)
    if args.ingest_only:
        rec["seconds"] = T
        rec["note"] = ("read = read_starring of the parquet directory (parts decoded in parallel into preallocated "
                       "columns); ingest = ALS.fit wall time minus als_fit (host checks + H2D + device id remap + "
                       "both CSR orientations + the rank layout); maxIter 0")
        os.makedirs(os.path.dirname(os.path.abspath(args.out)), exist_ok=True)
        with open(args.out, "w") as fh:
            json.dump(rec, fh, indent=1)
        print(json.dumps(rec), flush=True)
        shutil.rmtree(args.dir, ignore_errors=True)
        return 0
    t = time.perf_counter()
    model.write().overwrite().save(mpath)
    T["save"] = time.perf_counter() - t
    t = time.perf_counter()
    loaded = ALSModel.load(mpath)
    T["load"] = time.perf_counter() - t
    uids, U = model.user_factors_np()
    iids, V = model.item_factors_np()
    lu, lU = loaded.user_factors_np()
    li, lV = loaded.item_factors_np()
    rec["reload_bit_identical"] = bool(np.array_equal(uids, lu) and np.array_equal(iids, li)
                                       and np.array_equal(U.view(np.uint32), lU.view(np.uint32))
                                       and np.array_equal(V.view(np.uint32), lV.view(np.uint32)))

    test_users = sample_test_users(stars, 42)
    t = time.perf_counter()
    recs = ALSRecommender(model=loaded).setUserCol("user_id").setItemCol("repo_id").setTopK(30).recommendForUsers(
        {"user_id": test_users})
    T["topk"] = time.perf_counter() - t
    sel = np.isin(stars["user_id"], test_users)
    su, si, st = stars["user_id"][sel], stars["repo_id"][sel], stars["starred_at"][sel].astype(np.int64)
    t = time.perf_counter()
    ndcg = loaded.evaluate_ndcg(su, si, st, k=30)
    T["ndcg"] = time.perf_counter() - t
    rec["ndcg30"] = ndcg
    rec["seconds"] = T
    rec["job_seconds"] = sum(T[k] for k in ("read", "ingest", "fit", "save", "load", "topk", "ndcg"))
    print(json.dumps(rec), flush=True)

    # ---- parity (not timed) ------------------------------------------------------------------
    par = {}
    # 200 user rows of the last (user) half-sweep vs the fp64 solve from the item factors
    rng = np.random.default_rng(5)
    order = np.argsort(stars["user_id"], kind="stable")
    us, ist, rs = stars["user_id"][order], stars["repo_id"][order], stars["starring"][order]
    starts = np.searchsorted(us, uids)
    ends = np.searchsorted(us, uids, side="right")
    G = V.astype(np.float64).T @ V.astype(np.float64)
    worst = 0.0
    for r in rng.choice(uids.size, 200, replace=False):
        items = ist[starts[r]:ends[r]]
        rat = rs[starts[r]:ends[r]].astype(np.float64)
        Yr = V[np.searchsorted(iids, items)].astype(np.float64)
        c = 40.0 * np.abs(rat)
        A = G + (Yr.T * c) @ Yr + 0.5 * np.sum(rat > 0) * np.eye(args.rank)
        b = Yr.T @ np.where(rat > 0, 1.0 + c, 0.0)
        x = np.linalg.solve(A, b)
        worst = max(worst, float(np.max(np.abs(U[r] - x)) / np.max(np.abs(x))))
    par["user_rows_200_worst_rel"] = worst
    par["user_rows_ok"] = worst < 1e-4
    # the 251 lists vs the oracle scorer
    rows = np.searchsorted(uids, test_users)
    ref_ids, ref_sc = cbind.recommend(U[rows], iids, V, 30)
    got = {int(u): g for u, g in recs.groupby("user_id")}
    ok = 0
    for n, u in enumerate(test_users):
        g = got[int(u)]
        if (np.array_equal(g["repo_id"].to_numpy(), ref_ids[n][ref_ids[n] >= 0])
                and np.array_equal(g["score"].to_numpy(np.float32).view(np.uint32),
                                   ref_sc[n][ref_ids[n] >= 0].view(np.uint32))):
            ok += 1
    par["topk_lists_bit_exact"] = f"{ok}/{test_users.size}"
    actual = O.into_user_items(su, si, st, 30)
    pred = {int(u): [int(x) for x in ref_ids[n] if x >= 0] for n, u in enumerate(test_users)}
    par["ndcg30_oracle"] = O.evaluate_ndcg(pred, actual, 30)
    par["ndcg30_abs_diff"] = abs(par["ndcg30_oracle"] - ndcg)
    rec["parity"] = par
    print(json.dumps(par), flush=True)
    os.makedirs(os.path.dirname(os.path.abspath(args.out)), exist_ok=True)
    with open(args.out, "w") as fh:
        json.dump(rec, fh, indent=1)
    shutil.rmtree(args.dir, ignore_errors=True)
    return 0 if (par["user_rows_ok"] and ok == test_users.size and rec["reload_bit_identical"]
                 and par["ndcg30_abs_diff"] <= 1e-3) else 1


if __name__ == "__main__":
    sys.exit(main())
