"""Spark-layout persistence of the hot path's inputs and outputs (vectorised pyarrow, no per-row
Python objects).

* ALSModel (Spark 2.2 `ALSModel.ALSModelWriter` / `ALSModelReader`, used by
  `ModelUtils.scala:7-20` and read back by `ALSRecommender.scala:16-19` and
  `LogisticRegressionRanker.scala:167-168`):

      <path>/metadata/part-00000      one JSON line: class, timestamp, sparkVersion, uid,
                                      paramMap (the model's params: userCol, itemCol,
                                      predictionCol, coldStartStrategy), rank
      <path>/metadata/_SUCCESS
      <path>/userFactors/part-NNNNN-<uuid>-c000.snappy.parquet   id: int (non-null),
      <path>/itemFactors/part-NNNNN-<uuid>-c000.snappy.parquet   features: array<float>
      <path>/{userFactors,itemFactors}/_SUCCESS

  Spark writes one part per partition of the factor DataFrame; the reader takes every `part-*`
  parquet file of the directory (Hadoop hidden files `_*` / `.*` skipped), in name order.
* Starring input (`DatasetUtils.loadOrCreateDataFrame` / `loadRawStarringDS`,
  `DatasetUtils.scala:36-50,111-123`): a parquet directory of (user_id int, repo_id int,
  starred_at timestamp, starring double) rows, INT96 timestamps like Spark 2.2's default writer.
"""
from __future__ import annotations

import glob
import json
import os
import shutil
import time
import uuid

import numpy as np

ALS_MODEL_CLASS = "org.apache.spark.ml.recommendation.ALSModel"
SPARK_VERSION = "2.2.0"


def random_uid(prefix: str) -> str:
    """Spark Identifiable.randomUID: prefix + "_" + the last 12 hex digits of a random UUID."""
    return f"{prefix}_{uuid.uuid4().hex[-12:]}"


def _parts(dirpath: str):
    names = [n for n in os.listdir(dirpath) if not n.startswith(("_", "."))] if os.path.isdir(dirpath) else []
    return [os.path.join(dirpath, n) for n in sorted(names) if n.startswith("part-") and ".parquet" in n]


def _finish(dirpath: str):
    open(os.path.join(dirpath, "_SUCCESS"), "w").close()


# ---- metadata (DefaultParamsWriter.saveMetadata / DefaultParamsReader.loadMetadata) --------------

def write_metadata(path: str, cls: str, uid: str, param_map: dict, extra: dict | None = None) -> None:
    meta = {"class": cls, "timestamp": int(time.time() * 1000), "sparkVersion": SPARK_VERSION, "uid": uid,
            "paramMap": param_map}
    meta.update(extra or {})
    d = os.path.join(path, "metadata")
    os.makedirs(d, exist_ok=True)
    with open(os.path.join(d, "part-00000"), "w") as fh:
        fh.write(json.dumps(meta, separators=(",", ":")) + "\n")
    _finish(d)


def read_metadata(path: str, expected_class: str | None = None) -> dict:
    d = os.path.join(path, "metadata")
    files = [f for f in sorted(glob.glob(os.path.join(d, "part-*"))) if not f.endswith(".crc")]
    if not files:
        raise FileNotFoundError(f"Input path does not exist: {d}")
    with open(files[0]) as fh:
        meta = json.loads(fh.readline())
    if expected_class and meta.get("class") != expected_class:
        raise ValueError(f"Error loading metadata: Expected class name {expected_class} but found class name "
                         f"{meta.get('class')}")
    return meta


# ---- factor DataFrames (id: int, features: array<float>) ---------------------------------------

def factor_schema():
    import pyarrow as pa
    return pa.schema([pa.field("id", pa.int32(), nullable=False),
                      pa.field("features", pa.list_(pa.field("element", pa.float32(), nullable=False)))])


def write_factors(dirpath: str, ids: np.ndarray, feats: np.ndarray, rows_per_part: int = 1 << 20) -> int:
    """One `part-NNNNN-<uuid>-c000.snappy.parquet` per `rows_per_part` rows; returns the part count."""
    import pyarrow as pa
    import pyarrow.parquet as pq
    os.makedirs(dirpath, exist_ok=True)
    ids = np.ascontiguousarray(ids, dtype=np.int32)
    feats = np.ascontiguousarray(feats, dtype=np.float32)
    n, k = feats.shape
    job = uuid.uuid4()
    nparts = max(1, -(-n // rows_per_part))
    for p in range(nparts):
        lo, hi = p * rows_per_part, min(n, (p + 1) * rows_per_part)
        m = hi - lo
        offsets = pa.array(np.arange(0, (m + 1) * k, k, dtype=np.int32))
        values = pa.array(feats[lo:hi].reshape(-1))
        col = pa.ListArray.from_arrays(offsets, values, type=factor_schema().field("features").type)
        table = pa.Table.from_arrays([pa.array(ids[lo:hi]), col], schema=factor_schema())
        pq.write_table(table, os.path.join(dirpath, f"part-{p:05d}-{job}-c000.snappy.parquet"), compression="snappy")
    _finish(dirpath)
    return nparts


def read_factors(dirpath: str, rank: int):
    """(ids int32 [n], features float32 [n, rank]) of every part, in part-name order."""
    import pyarrow.parquet as pq
    parts = _parts(dirpath)
    if not parts:
        if not os.path.isdir(dirpath):
            raise FileNotFoundError(f"Input path does not exist: {dirpath}")
        return np.empty(0, np.int32), np.empty((0, rank), np.float32)
    ids, feats = [], []
    for f in parts:
        t = pq.read_table(f, columns=["id", "features"])
        col = t.column("features").combine_chunks()
        n = len(col)
        if col.null_count:
            raise ValueError(f"{f}: null factor rows")
        offs = np.asarray(col.offsets)
        if not np.array_equal(np.diff(offs), np.full(n, rank, offs.dtype)):
            raise ValueError(f"{f}: factor rows are not all of rank {rank}")
        vals = np.asarray(col.values.to_numpy(zero_copy_only=False), dtype=np.float32)
        feats.append(vals[offs[0]:offs[0] + n * rank].reshape(n, rank))
        ids.append(np.asarray(t.column("id").to_numpy(), dtype=np.int32))
    return np.concatenate(ids), np.concatenate(feats)


def save_als_model(path: str, uid: str, param_map: dict, rank: int, user, item, overwrite: bool,
                   rows_per_part: int = 1 << 20) -> None:
    """ALSModelWriter.saveImpl: metadata (+ "rank"), userFactors/, itemFactors/."""
    if os.path.exists(path):
        if not overwrite:
            raise IOError(f"Path {path} already exists. To overwrite it, please use write.overwrite().save(path) "
                          "for Scala and use write().overwrite().save(path) for Java and Python.")
        shutil.rmtree(path)
    write_metadata(path, ALS_MODEL_CLASS, uid, param_map, {"rank": int(rank)})
    write_factors(os.path.join(path, "userFactors"), *user, rows_per_part=rows_per_part)
    write_factors(os.path.join(path, "itemFactors"), *item, rows_per_part=rows_per_part)


def load_als_model(path: str):
    """ALSModelReader.load: (metadata, (user ids, factors), (item ids, factors))."""
    meta = read_metadata(path, ALS_MODEL_CLASS)
    rank = int(meta["rank"])
    return meta, read_factors(os.path.join(path, "userFactors"), rank), read_factors(os.path.join(path, "itemFactors"),
                                                                                     rank)


# ---- starring input (DatasetUtils.scala:36-50, 111-123) ------------------------------------------

STARRING_COLUMNS = ("user_id", "repo_id", "starred_at", "starring")


def write_starring(path: str, stars: dict, rows_per_part: int = 1 << 24, workers: int = 1, progress=None) -> None:
    """`df.write.mode("overwrite").parquet(path)` of a Starring dataset (INT96 timestamps).  `workers`
    parts are encoded at once (pyarrow releases the GIL); `progress(done, total)` after each part."""
    import pyarrow as pa
    import pyarrow.parquet as pq
    if os.path.exists(path):
        shutil.rmtree(path)
    os.makedirs(path)
    ts = np.asarray(stars["starred_at"])
    if ts.dtype.kind != "M":
        ts = ts.astype("datetime64[s]")
    schema = pa.schema([pa.field("user_id", pa.int32()), pa.field("repo_id", pa.int32()),
                        pa.field("starred_at", pa.timestamp("us")), pa.field("starring", pa.float64(), nullable=False)])
    n = len(stars["user_id"])
    job = uuid.uuid4()
    nparts = max(1, -(-n // rows_per_part))

    def part(p):
        lo, hi = p * rows_per_part, min(n, (p + 1) * rows_per_part)
        t = pa.Table.from_arrays([pa.array(np.asarray(stars["user_id"][lo:hi], np.int32)),
                                  pa.array(np.asarray(stars["repo_id"][lo:hi], np.int32)),
                                  pa.array(ts[lo:hi].astype("datetime64[us]")),
                                  pa.array(np.asarray(stars["starring"][lo:hi], np.float64))], schema=schema)
        pq.write_table(t, os.path.join(path, f"part-{p:05d}-{job}-c000.snappy.parquet"), compression="snappy",
                       use_deprecated_int96_timestamps=True)

    if workers <= 1:
        for p in range(nparts):
            part(p)
            if progress:
                progress(p + 1, nparts)
    else:
        from concurrent.futures import ThreadPoolExecutor
        with ThreadPoolExecutor(max_workers=workers) as ex:
            for i, _ in enumerate(ex.map(part, range(nparts))):
                if progress:
                    progress(i + 1, nparts)
    _finish(path)


def _data_files(path: str):
    """Parquet data files of a dataset directory, as Spark's reader lists them: every non-hidden
    file (Hadoop hidden = `_*` / `.*`) ending in `.parquet`, in name order -- Spark's
    `part-NNNNN-<uuid>-c000.snappy.parquet` as well as a pandas/pyarrow export (`<uuid>-0.parquet`)."""
    names = sorted(n for n in os.listdir(path) if not n.startswith(("_", ".")))
    files = [os.path.join(path, n) for n in names if n.endswith(".parquet") and os.path.isfile(os.path.join(path, n))]
    if not files and any(os.path.isdir(os.path.join(path, n)) for n in names):
        raise ValueError(f"{path}: partitioned parquet directories (column=value/ subdirectories) are not supported; "
                         "write the starring rows as one flat parquet directory")
    return files


def read_starring(path: str, columns=STARRING_COLUMNS) -> dict:
    """`spark.read.parquet(path)` of a Starring dataset: dict of numpy columns (timestamps as
    datetime64[us]).  A missing path raises FileNotFoundError ("Path does not exist"); an existing
    directory without parquet data files raises ValueError (nothing is ever deleted here)."""
    import pyarrow.parquet as pq
    if not os.path.exists(path):
        raise FileNotFoundError(f"Path does not exist: {path}")
    parts = _data_files(path) if os.path.isdir(path) else [path]
    if not parts:
        raise ValueError(f"Unable to infer schema for Parquet: {path} holds no parquet data files")
    # Parts with one schema and no nulls (what Spark's writer and write_starring produce): row counts
    # from the footers -> one output array per column, each part decoded by a pool thread straight
    # into its slice (pyarrow releases the GIL; no concatenation copy).  Anything else takes the
    # per-part read + np.concatenate (numpy's promotion of mixed types, NaN for nulls).
    from concurrent.futures import ThreadPoolExecutor
    files = [pq.ParquetFile(f) for f in parts]
    schemas = [pf.schema_arrow for pf in files]
    uniform = all(s.field(c).type == schemas[0].field(c).type for s in schemas for c in columns)
    if uniform and len(parts) > 1:
        counts = [pf.metadata.num_rows for pf in files]
        offs = np.r_[0, np.cumsum(counts)].astype(np.int64)
        out = {}
        for c in columns:
            dt = schemas[0].field(c).type.to_pandas_dtype()
            out[c] = np.empty(int(offs[-1]), "datetime64[us]" if np.dtype(dt).kind == "M" else dt)

        def part(i):
            t = pq.read_table(parts[i], columns=list(columns))
            if t.num_rows != counts[i] or any(t.column(c).null_count for c in columns):
                return False
            for c in columns:
                a = t.column(c).to_numpy()
                out[c][offs[i]:offs[i + 1]] = a.astype("datetime64[us]") if a.dtype.kind == "M" else a
            return True

        with ThreadPoolExecutor(max_workers=max(1, min(16, len(parts), os.cpu_count() or 1))) as ex:
            if all(ex.map(part, range(len(parts)))):
                return out
    cols = {c: [] for c in columns}
    for f in parts:
        t = pq.read_table(f, columns=list(columns))
        for c in columns:
            a = t.column(c).to_numpy()
            cols[c].append(a.astype("datetime64[us]") if a.dtype.kind == "M" else a)
    return {c: np.concatenate(v) for c, v in cols.items()}


def load_or_create_dataframe(path: str, create_fn) -> dict:
    """DatasetUtils.loadOrCreateDataFrame (DatasetUtils.scala:36-50): read the parquet data at
    `path`; only when the path does not exist ("Path does not exist") create the data, write it there
    and return it.  Any other read error of an existing path propagates: a user's directory is never
    replaced."""
    if os.path.exists(path):
        return read_starring(path)
    df = create_fn()
    write_starring(path, df)
    return df
