"""albedo's job layer above the ALS boundary: Recommender / ALSRecommender
(recommenders/Recommender.scala, ALSRecommender.scala), loadOrCreateModel (ModelUtils.scala:7-20),
RankingEvaluator params (RankingEvaluator.scala:21-49) and the ALSRecommenderBuilder protocol
(ALSRecommenderBuilder.scala:13-108).  CPU tests cover the host logic; the gpu-marked ones run the
device top-k through ALSRecommender and the whole builder against the oracle."""
import os

import numpy as np
import pytest


def test_recommender_params_and_schema_check():
    from albedo_amd import ALSRecommender, IllegalArgumentException
    r = ALSRecommender()
    assert (r.getUserCol(), r.getItemCol(), r.getScoreCol(), r.getSourceCol(), r.getTopK()) == \
        ("user", "item", "score", "source", 15)
    assert r.source == "als" and r.uid.startswith("alsRecommender_")
    r.setUserCol("user_id").setItemCol("repo_id").setTopK(30)
    assert (r.getUserCol(), r.getTopK()) == ("user_id", 30)
    r.transformSchema({"user_id": np.array([1, 2], dtype=np.int32)})
    with pytest.raises(IllegalArgumentException,
                       match="Column user_id must be of type IntegerType but was actually LongType"):
        r.transformSchema({"user_id": np.array([1, 2], dtype=np.int64)})
    with pytest.raises(IllegalArgumentException, match="StringType"):
        r.transformSchema({"user_id": np.array(["a"], dtype=object)})
    with pytest.raises(IllegalArgumentException, match="does not exist"):
        r.transformSchema({"user": np.array([1], dtype=np.int32)})


def test_load_or_create_model_creates_once_then_loads(tmp_path):
    from albedo_amd.builder import load_or_create_model
    calls = []

    class FakeModel:
        def __init__(self, tag):
            self.tag = tag

        def write(self):
            model = self

            class W:
                def overwrite(self):
                    return self

                def save(self, path):
                    os.makedirs(path)
                    open(os.path.join(path, "tag"), "w").write(model.tag)
            return W()

        @classmethod
        def load(cls, path):
            return cls("loaded:" + open(os.path.join(path, "tag")).read())

    path = str(tmp_path / "20261016" / "alsModel.parquet")
    m1 = load_or_create_model(FakeModel, path, lambda: calls.append(1) or FakeModel("fit"))
    assert m1.tag == "fit" and calls == [1]
    m2 = load_or_create_model(FakeModel, path, lambda: calls.append(2) or FakeModel("fit2"))
    assert m2.tag == "loaded:fit" and calls == [1]


def test_ranking_evaluator_params():
    from albedo_amd import RankingEvaluator
    ev = RankingEvaluator({1: [1, 2, 3]}).setMetricName("NDCG@k").setK(30).setUserCol("user_id").setItemsCol("items")
    assert ev.getFormattedMetricName() == "NDCG@30" and ev.getK() == 30 and ev.isLargerBetter()
    assert ev.evaluate({1: [1, 2, 3]}) == pytest.approx(1.0)
    with pytest.raises(ValueError):
        ev.setMetricName("AUC")


def test_settings_paths(monkeypatch):
    from albedo_amd import settings
    monkeypatch.setenv("ALBEDO_DATA_DIR", "/data/albedo")
    p = settings.als_model_path()
    assert p.startswith("/data/albedo/") and p.endswith("/alsModel.parquet") and len(p.split("/")[-2]) == 8


def test_builder_input_contract_and_user_sample():
    from albedo_amd.builder import load_raw_starring, sample_test_users
    stars = load_raw_starring(2000, 400, 20000, seed=5)
    assert set(stars) == {"user_id", "repo_id", "starred_at", "starring"}
    assert np.all(stars["starring"] == 1.0)
    key = stars["user_id"].astype(np.int64) * 2**32 + stars["repo_id"]
    assert np.unique(key).size == key.size  # unique (user, repo), app/models.py:166-167
    a = sample_test_users(stars, 7)
    b = sample_test_users(stars, 7)
    assert np.array_equal(a, b) and a.size == 251 and np.unique(a[:-1]).size == 250
    assert a[-1] in set(stars["user_id"].tolist())


@pytest.mark.gpu
def test_als_recommender_matches_oracle_topk(gpu_lib):
    from albedo_amd import ALS, ALSRecommender
    from albedo_amd.synthetic import SynthSpec, generate
    from oracle import spark_als as O
    d = generate(SynthSpec(3000, 700, 40000, seed=11))
    model = ALS(rank=24, maxIter=3, regParam=0.5, alpha=40.0, implicitPrefs=True, seed=42).fit(d)
    uids, uf = model.user_factors_np()
    iids, itf = model.item_factors_np()
    rng = np.random.default_rng(0)
    users = np.r_[rng.choice(uids, 300, replace=False), np.array([-5, 2**31 - 1])].astype(np.int32)
    rec = ALSRecommender(model=model).setTopK(30)
    out = rec.recommendForUsers({"user": users})
    assert list(out.columns) == ["user", "item", "score", "source"] and set(out["source"]) == {"als"}
    known = np.intersect1d(users, uids)
    assert set(out["user"].unique()) == set(known.tolist())  # unknown users drop out (inner join)
    rows = np.searchsorted(uids, known)
    oid, osc = O.recommend_for_all(known, uf[rows], iids, itf, 30)
    for n, u in enumerate(known):
        g = out[out["user"] == u]
        assert np.array_equal(g["item"].to_numpy(), oid[n]), f"user {u}"
        assert np.array_equal(g["score"].to_numpy().view(np.uint32), osc[n].astype(np.float32).view(np.uint32))


@pytest.mark.gpu
def test_builder_ndcg_matches_oracle_and_reloads(gpu_lib, tmp_path, capsys):
    from albedo_amd import ALSModel
    from albedo_amd import builder
    from albedo_amd.evaluation import into_user_items, ndcg_at
    from oracle import spark_als as O
    path = str(tmp_path / "alsModel.parquet")
    argv = ["--users", "4000", "--repos", "800", "--stars", "50000", "--rank", "16", "--max-iter", "3",
            "--model-path", path]
    ndcg = builder.main(argv)
    assert os.path.isdir(os.path.join(path, "userFactors"))
    # the same protocol recomputed on the oracle side from the persisted factors
    model = ALSModel.load(path)
    uids, uf = model.user_factors_np()
    iids, itf = model.item_factors_np()
    stars = builder.load_raw_starring(4000, 800, 50000, 42)
    users = np.intersect1d(builder.sample_test_users(stars, 42), uids)
    oid, osc = O.recommend_for_all(users, uf[np.searchsorted(uids, users)], iids, itf, 30)
    pred = {int(u): oid[n][oid[n] >= 0].tolist() for n, u in enumerate(users)}
    actual = into_user_items(stars["user_id"], stars["repo_id"], stars["starred_at"], 30)
    ref = ndcg_at([(pred[u][:30], actual[u][:30]) for u in pred if u in actual], 30)
    assert ndcg == pytest.approx(ref, abs=1e-12)
    assert 0.0 < ndcg < 1.0
    # second run: loadOrCreateModel finds today's model and does not refit
    assert builder.main(argv) == pytest.approx(ndcg, abs=1e-12)
    assert "NDCG@30 = " in capsys.readouterr().out
