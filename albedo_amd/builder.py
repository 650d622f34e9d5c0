"""ALSRecommenderBuilder.main (ALSRecommenderBuilder.scala:13-108) on the MI355X engine.

    python -m albedo_amd.builder [--users U --repos I --stars N --rank 50 --max-iter 26]

Same protocol as the reference job:
  1. load the starring rows (user_id, repo_id, starred_at, starring = 1.0)   (:40, DatasetUtils:111-123)
  2. loadOrCreateModel(ALSModel, dataDir/today/alsModel.parquet, fit)        (:44-59, ModelUtils:7-20)
     with ALS(implicitPrefs, rank 50, regParam 0.5, alpha 40, maxIter 26, seed 42,
     coldStartStrategy "drop", user_id / repo_id / starring)
  3. randomSplit(0.9, 0.1); sample 250 distinct test users + one fixed user    (:65-71)
  4. ALSRecommender(user_id, repo_id, topK 30).recommendForUsers               (:75-84)
  5. NDCG@30 of intoUserPredictedItems(score desc) against
     loadUserActualItemsDF(30) = intoUserActualItems(starred_at desc)          (:92-104)

Differences, all forced by the environment: the MySQL dump (README.md:29) is not available
offline, so step 1's loadOrCreateDataFrame creates the parquet cache from the seeded synthetic
GitHub-like star matrix (albedo_amd.synthetic) with per-star timestamps instead
of the JDBC read (an existing rawStarringDF.parquet -- e.g. one exported from the real dump -- is
read as is); the reference's split and sample are unseeded
(`randomSplit` without a seed, `scala.util.Random.shuffle`), here they take `--seed`; the fixed
user 652070 is used when present, else the highest user id of the test split.
"""
from __future__ import annotations

import argparse
import os
import time

import numpy as np

from . import persistence, settings
from .als import ALS, ALSModel
from .evaluation import RankingEvaluator, into_user_items
from .recommenders import ALSRecommender
from .synthetic import SynthSpec, generate

FIXED_USER = 652070  # ALSRecommenderBuilder.scala:68


def load_or_create_model(model_cls, path, create_model_func):
    """ModelUtils.loadOrCreateModel (ModelUtils.scala:7-20): load the model at `path`; when the path
    does not exist, create it and write().overwrite().save(path).  Other load errors propagate."""
    if not os.path.exists(path):
        model = create_model_func()
        model.write().overwrite().save(path)
        return model
    return model_cls.load(path)


def synthetic_starring(users=20000, repos=4000, stars=400000, seed=42):
    """Stand-in for the JDBC read of app_repostarring (DatasetUtils.scala:116-118): dict of columns
    user_id, repo_id, starred_at (datetime64[s]), starring (= 1.0, :118)."""
    d = generate(SynthSpec(users, repos, stars, seed=seed), with_timestamps=True)
    return {"user_id": d["user"], "repo_id": d["item"], "starred_at": d["ts"].astype("datetime64[s]"),
            "starring": d["rating"].astype(np.float64)}


SYNTH_SIDECAR = "_albedo_synth.json"  # Hadoop-hidden: parquet readers skip it


def load_raw_starring(users=20000, repos=4000, stars=400000, seed=42, path=None):
    """DatasetUtils.loadRawStarringDS (:111-123): loadOrCreateDataFrame(dataDir/today/
    rawStarringDF.parquet, <read app_repostarring + starring = 1.0>) -- the parquet data is read
    when present, else the synthetic stand-in is written there first.  `path=False` skips the
    cache (pure in-memory).

    Like the reference's date-keyed cache, an existing dataset wins over the requested sizes.  The
    synthetic spec is kept beside the parquet parts (`_albedo_synth.json`, hidden from readers), and
    a cache hit whose spec differs from the request -- or a dataset this code did not write -- is
    reported on stderr with the row count actually used."""
    if path is False:
        return synthetic_starring(users, repos, stars, seed)
    import json
    import sys
    path = path or settings.raw_starring_path()
    spec = {"users": int(users), "repos": int(repos), "stars": int(stars), "seed": int(seed)}
    created = []

    def create():
        created.append(True)
        return synthetic_starring(users, repos, stars, seed)

    df = persistence.load_or_create_dataframe(path, create)
    side = os.path.join(path, SYNTH_SIDECAR)
    if created:
        if os.path.isdir(path):
            with open(side, "w") as fh:
                json.dump(spec, fh)
        return df
    cached = None
    if os.path.exists(side):
        with open(side) as fh:
            cached = json.load(fh)
    if cached != spec:
        what = f"synthetic spec {cached}" if cached else "a dataset not written by this builder"
        print(f"[albedo] {path}: using the existing starring data ({df['user_id'].size} rows, {what}) instead of "
              f"the requested {spec}; delete the directory to regenerate", file=sys.stderr)
    return df


def sample_test_users(stars, seed, n=250):
    """:65-71 — randomSplit(Array(0.9, 0.1)) then 250 shuffled distinct users of the test part,
    plus the fixed user."""
    rng = np.random.default_rng(seed)
    test = rng.random(stars["user_id"].size) >= 0.9
    users = np.unique(stars["user_id"][test])
    picked = rng.permutation(users)[:n].tolist()
    fixed = FIXED_USER if FIXED_USER in set(stars["user_id"].tolist()) else int(users.max())
    return np.asarray(picked + [fixed], dtype=np.int32)


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__.splitlines()[0])
    ap.add_argument("--users", type=int, default=20000)
    ap.add_argument("--repos", type=int, default=4000)
    ap.add_argument("--stars", type=int, default=400000)
    ap.add_argument("--rank", type=int, default=50)
    ap.add_argument("--max-iter", type=int, default=26)
    ap.add_argument("--top-k", type=int, default=30)
    ap.add_argument("--seed", type=int, default=42)
    ap.add_argument("--model-path", default=None)
    ap.add_argument("--starring-path", default=None,
                    help="parquet directory of Starring rows (default dataDir/today/rawStarringDF.parquet)")
    args = ap.parse_args(argv)

    stars = load_raw_starring(args.users, args.repos, args.stars, args.seed, path=args.starring_path)
    path = args.model_path or settings.als_model_path()

    def fit():
        als = (ALS().setImplicitPrefs(True).setRank(args.rank).setRegParam(0.5).setAlpha(40)
               .setMaxIter(args.max_iter).setSeed(42).setColdStartStrategy("drop")
               .setUserCol("user_id").setItemCol("repo_id").setRatingCol("starring"))
        return als.fit(stars)

    t0 = time.perf_counter()
    model = load_or_create_model(ALSModel, path, fit)
    fit_s = time.perf_counter() - t0
    print(model.explainParams())

    test_users = sample_test_users(stars, args.seed)
    recommender = ALSRecommender(model=model).setUserCol("user_id").setItemCol("repo_id").setTopK(args.top_k)
    recs = recommender.recommendForUsers({"user_id": test_users})
    print(recs[recs["user_id"] == test_users[-1]].to_string(index=False))

    actual = into_user_items(stars["user_id"], stars["repo_id"], stars["starred_at"], args.top_k)
    predicted = into_user_items(recs["user_id"].to_numpy(), recs["repo_id"].to_numpy(), recs["score"].to_numpy(),
                                args.top_k)
    evaluator = (RankingEvaluator(actual).setMetricName("NDCG@k").setK(args.top_k)
                 .setUserCol("user_id").setItemsCol("items"))
    metric = evaluator.evaluate(predicted)
    print(f"{evaluator.getFormattedMetricName()} = {metric}")
    print(f"(fit or load: {fit_s:.2f} s, {len(test_users)} test users, model at {path})")
    return metric


if __name__ == "__main__":
    main()
