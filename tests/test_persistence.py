"""Spark-layout persistence (albedo_amd/persistence.py), CPU only.

ALSModel directories as Spark 2.2's ALSModelWriter lays them out (ModelUtils.scala:7-20 writes them,
ALSRecommender.scala:16-19 and LogisticRegressionRanker.scala:167-168 read them back), and the
Starring parquet cache of DatasetUtils.loadOrCreateDataFrame / loadRawStarringDS
(DatasetUtils.scala:36-50,111-123).
"""
import json
import os
import re

import numpy as np
import pytest

from albedo_amd import persistence as P


def test_factors_multi_part_roundtrip_spark_names(tmp_path):
    rng = np.random.default_rng(0)
    ids = rng.permutation(np.arange(1000, dtype=np.int32) * 7 - 3000)
    f = rng.standard_normal((1000, 13)).astype(np.float32)
    d = str(tmp_path / "userFactors")
    n = P.write_factors(d, ids, f, rows_per_part=300)
    assert n == 4
    names = sorted(os.listdir(d))
    assert names[0] == "_SUCCESS"
    assert all(re.fullmatch(r"part-\d{5}-[0-9a-f-]{36}-c000\.snappy\.parquet", x) for x in names[1:])
    ids2, f2 = P.read_factors(d, 13)
    assert np.array_equal(ids2, ids) and np.array_equal(f2.view(np.uint32), f.view(np.uint32))


def test_factor_schema_is_spark_array_of_float(tmp_path):
    import pyarrow.parquet as pq
    d = str(tmp_path / "itemFactors")
    P.write_factors(d, np.arange(5, dtype=np.int32), np.ones((5, 3), np.float32))
    part = [x for x in os.listdir(d) if x.startswith("part-")][0]
    sch = pq.read_schema(os.path.join(d, part))
    assert str(sch.field("id").type) == "int32" and not sch.field("id").nullable
    assert str(sch.field("features").type) == "list<element: float not null>"


def test_reader_takes_spark_written_directories(tmp_path):
    """A directory as Spark leaves it: several parts whose names sort out of row order, a legacy
    list layout (element named "array"), checksum / hidden files -- read in part-name order."""
    import pyarrow as pa
    import pyarrow.parquet as pq
    d = tmp_path / "userFactors"
    d.mkdir()
    legacy = pa.list_(pa.field("array", pa.float32()))
    rows = {"part-00001-x-c000.snappy.parquet": (np.array([5, 6], np.int32), [[1.0, 2.0], [3.0, 4.0]]),
            "part-00000-x-c000.snappy.parquet": (np.array([9], np.int32), [[7.0, 8.0]])}
    for name, (ids, feats) in rows.items():
        t = pa.table({"id": pa.array(ids), "features": pa.array(feats, type=legacy)})
        pq.write_table(t, str(d / name))
    (d / "_SUCCESS").write_text("")
    (d / ".part-00000-x-c000.snappy.parquet.crc").write_bytes(b"\0")
    ids, f = P.read_factors(str(d), 2)
    assert ids.tolist() == [9, 5, 6]
    assert f.tolist() == [[7.0, 8.0], [1.0, 2.0], [3.0, 4.0]]
    with pytest.raises(ValueError, match="rank 3"):
        P.read_factors(str(d), 3)


def test_model_metadata_layout(tmp_path):
    path = str(tmp_path / "alsModel.parquet")
    uid = P.random_uid("als")
    assert re.fullmatch(r"als_[0-9a-f]{12}", uid)
    pm = {"userCol": "user_id", "itemCol": "repo_id", "predictionCol": "prediction", "coldStartStrategy": "drop"}
    user = (np.array([3, 1], np.int32), np.zeros((2, 4), np.float32))
    item = (np.array([2], np.int32), np.ones((1, 4), np.float32))
    P.save_als_model(path, uid, pm, 4, user, item, overwrite=False)
    with open(os.path.join(path, "metadata", "part-00000")) as fh:
        meta = json.loads(fh.readline())
    assert meta["class"] == "org.apache.spark.ml.recommendation.ALSModel"
    assert meta["uid"] == uid and meta["rank"] == 4 and meta["paramMap"] == pm and meta["sparkVersion"] == "2.2.0"
    assert os.path.exists(os.path.join(path, "metadata", "_SUCCESS"))
    with pytest.raises(IOError, match="already exists"):
        P.save_als_model(path, uid, pm, 4, user, item, overwrite=False)
    P.save_als_model(path, uid, pm, 4, user, item, overwrite=True)
    meta2, (ui, uf), (ii, itf) = P.load_als_model(path)
    assert meta2["uid"] == uid and ui.tolist() == [3, 1] and itf.tolist() == [[1.0] * 4]
    with pytest.raises(ValueError, match="Expected class name"):
        P.read_metadata(path, "org.apache.spark.ml.recommendation.ALS")
    with pytest.raises(FileNotFoundError):
        P.load_als_model(str(tmp_path / "missing"))


def test_starring_cache_load_or_create(tmp_path):
    """loadOrCreateDataFrame: the first call creates and writes the parquet cache, the second
    reads it (the create function is not called again); timestamps survive as INT96."""
    import pyarrow.parquet as pq
    path = str(tmp_path / "rawStarringDF.parquet")
    calls = []

    def create():
        calls.append(1)
        return {"user_id": np.array([1, 1, 2], np.int32), "repo_id": np.array([10, 11, 10], np.int32),
                "starred_at": np.array([1500000000, 1500000100, 1400000000], "datetime64[s]"),
                "starring": np.ones(3)}

    a = P.load_or_create_dataframe(path, create)
    b = P.load_or_create_dataframe(path, create)
    assert calls == [1]
    assert b["user_id"].tolist() == [1, 1, 2] and b["repo_id"].tolist() == [10, 11, 10]
    assert np.array_equal(b["starred_at"], a["starred_at"].astype("datetime64[us]"))
    assert b["starring"].dtype == np.float64 and np.all(b["starring"] == 1.0)
    part = [x for x in os.listdir(path) if x.startswith("part-")][0]
    meta = pq.ParquetFile(os.path.join(path, part)).metadata
    assert meta.schema.column(2).physical_type == "INT96"


def test_builder_reads_starring_cache(tmp_path):
    from albedo_amd import builder
    from albedo_amd.evaluation import into_user_items
    path = str(tmp_path / "stars.parquet")
    s1 = builder.load_raw_starring(500, 100, 3000, seed=3, path=path)
    s2 = builder.load_raw_starring(1, 1, 1, seed=0, path=path)  # cache hit: the arguments no longer matter
    assert np.array_equal(s1["user_id"], s2["user_id"]) and s2["user_id"].size > 2900
    act1 = into_user_items(s1["user_id"], s1["repo_id"], s1["starred_at"], 30)
    act2 = into_user_items(s2["user_id"], s2["repo_id"], s2["starred_at"], 30)
    assert act1 == act2


def test_existing_starring_dir_is_read_never_replaced(tmp_path, capsys):
    """an existing --starring-path is data, not a cache miss.  A pandas/pyarrow
    export (`<uuid>-0.parquet`) is read as is; a directory without parquet files raises and keeps
    its contents; only a path that does not exist is created (DatasetUtils.scala:36-50)."""
    import pyarrow as pa
    import pyarrow.parquet as pq
    from albedo_amd import builder
    d = tmp_path / "export"
    d.mkdir()
    t = pa.table({"user_id": pa.array([7, 8], pa.int32()), "repo_id": pa.array([1, 2], pa.int32()),
                  "starred_at": pa.array(np.array([1500000000, 1500000001], "datetime64[s]").astype("datetime64[us]")),
                  "starring": pa.array([1.0, 1.0])})
    pq.write_table(t, str(d / "1f2e3d4c-0.parquet"))
    (d / "_SUCCESS").write_text("")
    got = P.load_or_create_dataframe(str(d), lambda: pytest.fail("existing data must not be recreated"))
    assert got["user_id"].tolist() == [7, 8]
    s = builder.load_raw_starring(100, 10, 500, seed=1, path=str(d))
    assert s["user_id"].tolist() == [7, 8]
    assert "not written by this builder" in capsys.readouterr().err
    bad = tmp_path / "notes"
    bad.mkdir()
    (bad / "README.txt").write_text("keep me")
    with pytest.raises(ValueError):
        P.load_or_create_dataframe(str(bad), lambda: pytest.fail("must not create over an existing directory"))
    assert (bad / "README.txt").read_text() == "keep me"


def test_builder_cache_reports_spec_mismatch(tmp_path, capsys):
    from albedo_amd import builder
    path = str(tmp_path / "stars.parquet")
    builder.load_raw_starring(300, 60, 2000, seed=3, path=path)
    assert capsys.readouterr().err == ""
    builder.load_raw_starring(300, 60, 2000, seed=3, path=path)
    assert capsys.readouterr().err == ""
    builder.load_raw_starring(400, 60, 2000, seed=3, path=path)
    assert "using the existing starring data" in capsys.readouterr().err


def test_starring_parallel_parts_match_serial(tmp_path):
    """read_starring decodes uniform parts in parallel straight into preallocated columns and
    write_starring encodes parts on a thread pool: the result equals the serial write / per-part
    read + concatenation, in part order."""
    import pyarrow.parquet as pq
    rng = np.random.default_rng(7)
    n = 10_000
    stars = {"user_id": rng.integers(0, 500, n).astype(np.int32), "repo_id": rng.integers(0, 90, n).astype(np.int32),
             "starred_at": (1_400_000_000 + rng.integers(0, 10**6, n)).astype("datetime64[s]"),
             "starring": np.ones(n)}
    a, b = str(tmp_path / "a"), str(tmp_path / "b")
    seen = []
    P.write_starring(a, stars, rows_per_part=777, workers=4, progress=lambda d, t: seen.append((d, t)))
    P.write_starring(b, stars, rows_per_part=777)
    assert seen[-1] == (13, 13)
    ra, rb = P.read_starring(a), P.read_starring(b)
    for c in P.STARRING_COLUMNS:
        assert np.array_equal(ra[c], rb[c]) and np.array_equal(ra[c], np.asarray(stars[c]).astype(ra[c].dtype))
    # a part with another schema (int64 ids) falls back to the per-part read + numpy promotion
    t = pq.read_table(os.path.join(a, sorted(f for f in os.listdir(a) if f.endswith(".parquet"))[0]))
    import pyarrow as pa
    t2 = t.set_column(0, "user_id", pa.array(t.column("user_id").to_numpy().astype(np.int64)))
    pq.write_table(t2, os.path.join(a, "part-99999-x-c000.snappy.parquet"), use_deprecated_int96_timestamps=True)
    rc = P.read_starring(a)
    assert rc["user_id"].dtype == np.int64 and rc["user_id"].size == n + t.num_rows
    assert np.array_equal(rc["user_id"][:n], stars["user_id"])
