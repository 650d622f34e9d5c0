"""RankingEvaluator (albedo evaluators/RankingEvaluator.scala:14-143) on numpy.

* intoUserActualItems / intoUserPredictedItems (:121-139): rank() over (user ORDER BY key DESC)
  <= k, then collect_list.  Spark's collect_list order after groupBy is unspecified, so the list
  order is made deterministic as (key desc, item asc); rank() keeps ties (lists may exceed k).
* evaluate (:83-103): inner join on user, slice both lists to k, mllib RankingMetrics.ndcgAt(k) /
  precisionAt(k) / meanAveragePrecision.
"""
from __future__ import annotations

import math

import numpy as np


def into_user_items(user, item, key, k):
    user = np.asarray(user)
    item = np.asarray(item)
    key = np.asarray(key)
    if key.dtype.kind == "M":  # timestamps (starred_at read from parquet)
        key = key.astype("datetime64[us]").astype(np.int64)
    key = key.astype(np.float64)
    order = np.lexsort((item, -key, user))
    u, it, ky = user[order], item[order], key[order]
    if u.size == 0:
        return {}
    starts = np.flatnonzero(np.r_[True, u[1:] != u[:-1]])
    ends = np.r_[starts[1:], u.size]
    out = {}
    for s, e in zip(starts, ends):
        ks = ky[s:e]
        ranks = 1 + np.searchsorted(-ks, -ks, side="left")  # rank(): 1 + #strictly greater
        out[int(u[s])] = it[s:e][ranks <= k].tolist()
    return out


def ndcg_at(pairs, k):
    """mllib RankingMetrics.ndcgAt: mean over users; empty label set contributes 0."""
    if k <= 0:
        raise ValueError("ranking position k should be positive")
    vals = []
    for pred, lab in pairs:
        lab_set = set(int(x) for x in lab)
        if not lab_set:
            vals.append(0.0)
            continue
        n = min(max(len(pred), len(lab_set)), k)
        dcg = max_dcg = 0.0
        for i in range(n):
            gain = 1.0 / math.log(i + 2)
            if i < len(pred) and int(pred[i]) in lab_set:
                dcg += gain
            if i < len(lab_set):
                max_dcg += gain
        vals.append(dcg / max_dcg)
    return float(np.mean(vals)) if vals else float("nan")


def precision_at(pairs, k):
    vals = []
    for pred, lab in pairs:
        lab_set = set(int(x) for x in lab)
        if not lab_set:
            vals.append(0.0)
            continue
        n = min(len(pred), k)
        vals.append(sum(1 for i in range(n) if int(pred[i]) in lab_set) / k)
    return float(np.mean(vals)) if vals else float("nan")


def mean_average_precision(pairs):
    vals = []
    for pred, lab in pairs:
        lab_set = set(int(x) for x in lab)
        if not lab_set:
            vals.append(0.0)
            continue
        hits, prec = 0, 0.0
        for i, p in enumerate(pred):
            if int(p) in lab_set:
                hits += 1
                prec += hits / (i + 1.0)
        vals.append(prec / len(lab_set))
    return float(np.mean(vals)) if vals else float("nan")


class RankingEvaluator:
    """RankingEvaluator.scala:14-108.  The per-user item lists are dicts {user: [items]} (the output
    of `into_user_items`), standing in for the (userCol, itemsCol) DataFrames."""

    _METRICS = ("NDCG@k", "Precision@k", "MAP")

    def __init__(self, user_actual_items: dict, metric_name="NDCG@k", k=15):
        self.actual = user_actual_items
        self.metric_name = metric_name
        self.k = k
        self.user_col = "user"
        self.items_col = "items"

    # Spark-style params (:21-49)
    def setMetricName(self, v):
        if v not in self._METRICS:
            raise ValueError(f"unsupported metric {v}; supports {', '.join(self._METRICS)}")
        self.metric_name = v
        return self

    def getMetricName(self):
        return self.metric_name

    def setK(self, v):
        self.k = int(v)
        return self

    def getK(self):
        return self.k

    def setUserCol(self, v):
        self.user_col = v
        return self

    def getUserCol(self):
        return self.user_col

    def setItemsCol(self, v):
        self.items_col = v
        return self

    def getItemsCol(self):
        return self.items_col

    def isLargerBetter(self):
        return True

    def getFormattedMetricName(self):
        return self.metric_name.replace("@k", f"@{self.k}")

    formatted_metric_name = getFormattedMetricName

    def evaluate(self, user_predicted_items: dict) -> float:
        pairs = [(user_predicted_items[u][: self.k], self.actual[u][: self.k])
                 for u in user_predicted_items if u in self.actual]
        if self.metric_name == "NDCG@k":
            return ndcg_at(pairs, self.k)
        if self.metric_name == "Precision@k":
            return precision_at(pairs, self.k)
        if self.metric_name == "MAP":
            return mean_average_precision(pairs)
        raise ValueError(self.metric_name)
