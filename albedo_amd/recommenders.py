"""albedo's `Recommender` / `ALSRecommender` transformers over the MI355X engine.

* `Recommender` mirrors `recommenders/Recommender.scala:9-68`: params userCol ("user"), itemCol
  ("item"), scoreCol ("score"), sourceCol ("source"), topK (15); `transformSchema` requires the
  user column to be IntegerType (:46-56, same message); `transform` = `recommendForUsers` (:58-60).
* `ALSRecommender` mirrors `recommenders/ALSRecommender.scala:10-65`: the model is
  `ALSModel.load(dataDir/today/alsModel.parquet)` (:16-19) unless one is handed in; the requested
  users are inner-joined with the model's user factors (:33-34, unknown users drop out); every
  user is scored against every item with F2J `sdot` and kept in a `BoundedPriorityQueue(topK)`
  (:43-61, BoundedPriorityQueue.scala:30-53).  Output rows (userCol, itemCol, scoreCol,
  sourceCol = "als") (:63-65).

The reference emits up to topK rows per (user, 4096-item block) and leaves the global cut to the
evaluator's window `rank() <= k` (RankingEvaluator.scala:131-139); here the device returns the
global top-K directly (`als_recommend`: exact F2J scores, ties broken by item id ascending, which
is the first-seen order of the reference's heap over ascending-id blocks).  After
`intoUserPredictedItems(..., k = topK)` both give the same lists, except that `rank()` would also
keep extra items tied with the K-th score, which the reference's heap itself drops (it keeps
first-seen on ties) unless they sit in different item blocks.
"""
from __future__ import annotations

import uuid

import numpy as np

from . import _lib
from ._lib import IllegalArgumentException
from .als import ALSModel, _checked_cast
from . import settings

_SPARK_TYPES = {"i4": "IntegerType", "i8": "LongType", "i2": "ShortType", "i1": "ByteType",
                "f4": "FloatType", "f8": "DoubleType", "b1": "BooleanType"}


def spark_type_name(values) -> str:
    """Spark SQL type name of a column held as a numpy/pandas array."""
    dt = np.asarray(values).dtype
    key = f"{dt.kind}{dt.itemsize}"
    if dt.kind in "OUS":
        return "StringType"
    return _SPARK_TYPES.get(key, str(dt))


class Recommender:
    """recommenders/Recommender.scala:9-68 (abstract ml.Transformer)."""

    _defaults = dict(userCol="user", itemCol="item", scoreCol="score", sourceCol="source", topK=15)
    _uid_prefix = "recommender"
    source = None

    def __init__(self, uid=None):
        self.uid = uid or f"{self._uid_prefix}_{uuid.uuid4().hex[:12]}"  # Identifiable.randomUID
        self._p = dict(self._defaults)

    def _set(self, k, v):
        self._p[k] = v
        return self

    def setUserCol(self, v): return self._set("userCol", v)
    def getUserCol(self): return self._p["userCol"]
    def setItemCol(self, v): return self._set("itemCol", v)
    def getItemCol(self): return self._p["itemCol"]
    def setScoreCol(self, v): return self._set("scoreCol", v)
    def getScoreCol(self): return self._p["scoreCol"]
    def setSourceCol(self, v): return self._set("sourceCol", v)
    def getSourceCol(self): return self._p["sourceCol"]
    def setTopK(self, v): return self._set("topK", int(v))
    def getTopK(self): return self._p["topK"]

    def transformSchema(self, df):
        """Recommender.scala:46-56: the user column must be IntegerType."""
        col = self._p["userCol"]
        try:
            values = df[col]
        except (KeyError, IndexError, TypeError):
            raise IllegalArgumentException(_lib.ALS_E_INVALID_ARGUMENT, f"Field \"{col}\" does not exist.") from None
        actual = spark_type_name(values)
        if actual != "IntegerType":
            raise IllegalArgumentException(
                _lib.ALS_E_INVALID_ARGUMENT,
                f"requirement failed: Column {col} must be of type IntegerType but was actually {actual}.")
        return df

    def transform(self, userDF):
        return self.recommendForUsers(userDF)

    def recommendForUsers(self, userDF):
        raise NotImplementedError


class ALSRecommender(Recommender):
    """recommenders/ALSRecommender.scala:10-65 on the device top-k (MFMA pre-selection + exact F2J
    rescoring, `als_recommend`)."""

    source = "als"
    _uid_prefix = "alsRecommender"

    def __init__(self, uid=None, model: ALSModel | None = None, modelPath: str | None = None):
        super().__init__(uid)
        self._model = model
        self._model_path = modelPath

    @property
    def alsModel(self) -> ALSModel:
        """ALSRecommender.scala:16-19: ALSModel.load(dataDir/today/alsModel.parquet)."""
        if self._model is None:
            self._model = ALSModel.load(self._model_path or settings.als_model_path())
        return self._model

    def recommend_arrays(self, users):
        """(user ids, item ids, scores) as flat arrays: the rows recommendForUsers emits."""
        model = self.alsModel
        uids, _ = model.user_factors_np()
        # activeUsers ⋈ userFactors on id (ALSRecommender.scala:33-34): unknown users drop out
        active = np.intersect1d(_checked_cast(users, self._p["userCol"]), uids)
        num = int(self._p["topK"])
        if active.size == 0 or num <= 0:
            return np.empty(0, np.int32), np.empty(0, np.int32), np.empty(0, np.float32)
        src, ids, sc = model.recommend_np(num, subset=active)
        keep = ids >= 0
        return np.repeat(src, keep.sum(axis=1)), ids[keep], sc[keep]

    def recommendForUsers(self, userDF):
        import pandas as pd
        self.transformSchema(userDF)
        u, i, s = self.recommend_arrays(np.asarray(userDF[self._p["userCol"]]))
        return pd.DataFrame({self._p["userCol"]: u, self._p["itemCol"]: i, self._p["scoreCol"]: s,
                             self._p["sourceCol"]: self.source})
