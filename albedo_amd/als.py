"""Spark-shaped `ALS` estimator and `ALSModel` over libalbedo_als.so.

Mirrors the surface albedo's jobs use:
  * ALSRecommenderBuilder.scala:46-58 / Playground.scala:54-65 / train_als.py:55-61:
      ALS().setImplicitPrefs(True).setRank(50).setRegParam(0.5).setAlpha(40).setMaxIter(26)
           .setSeed(42).setColdStartStrategy("drop").setUserCol(..).setItemCol(..)
           .setRatingCol(..).fit(dataset)
  * ALSRecommender.scala:16-19,33-36 reads model.userFactors / model.itemFactors / model.rank
  * ALSRecommender.scala:28-65 (+ BoundedPriorityQueue.scala:30-53) is recommendForUserSubset
  * LogisticRegressionRanker.scala:167-174,229 uses model.transform (coldStartStrategy drop)
  * ModelUtils.scala:7-20 persists with model.write.overwrite().save(path) / ALSModel.load(path)
Parameter names, defaults and validation messages follow Spark 2.2.0's ALSParams.  Datasets are
pandas DataFrames or dicts of arrays (there is no JVM here); outputs are pandas DataFrames.
All compute runs on the MI355X through the C ABI; there is no CPU fallback.
"""
from __future__ import annotations

import ctypes as C
import time

import numpy as np

from . import _lib
from ._lib import IllegalArgumentException, check, load, ptr

SPARK_DEFAULT_SEED = 1994790107  # "org.apache.spark.ml.recommendation.ALS".hashCode (ALS setDefault(seed))


def _column(dataset, name):
    if dataset is None:
        raise IllegalArgumentException(_lib.ALS_E_INVALID_ARGUMENT, "dataset is None")
    try:
        col = dataset[name]
    except (KeyError, IndexError, TypeError):
        raise IllegalArgumentException(_lib.ALS_E_INVALID_ARGUMENT, f"Field \"{name}\" does not exist.") from None
    return np.asarray(col)


def _checked_cast(values, col):
    """ALS.checkedCast: ids must be numeric and within Int range (Spark 2.2.0 error messages)."""
    v = np.asarray(values)
    if v.dtype.kind not in "iuf":
        raise IllegalArgumentException(_lib.ALS_E_INVALID_ARGUMENT,
                                       f"ALS only supports values in Integer range for column {col}. "
                                       f"Column {col} was not numeric.")
    if v.size == 0:
        return v.astype(np.int32)
    if v.dtype.kind == "f":
        bad = (v != np.floor(v)) | (v < -2**31) | (v > 2**31 - 1) | ~np.isfinite(v)
    else:
        bad = (v < -2**31) | (v > 2**31 - 1)
    if np.any(bad):
        x = v[np.argmax(bad)]
        raise IllegalArgumentException(_lib.ALS_E_INVALID_ARGUMENT,
                                       f"ALS only supports values in Integer range and without fractional part "
                                       f"for columns {col}. Value {x} was either out of Integer range or "
                                       f"contained a fractional part that could not be converted.")
    return v.astype(np.int32)


class _Params:
    _defaults = dict(rank=10, maxIter=10, regParam=0.1, numUserBlocks=10, numItemBlocks=10,
                     implicitPrefs=False, alpha=1.0, userCol="user", itemCol="item",
                     ratingCol="rating", predictionCol="prediction", seed=SPARK_DEFAULT_SEED,
                     nonnegative=False, checkpointInterval=10, coldStartStrategy="nan",
                     intermediateStorageLevel="MEMORY_AND_DISK", finalStorageLevel="MEMORY_AND_DISK",
                     device=-1, lightMaxDegree=-1)
    _doc = dict(rank="rank of the factorization", maxIter="max number of iterations (>= 0)",
                regParam="regularization parameter (>= 0)", alpha="alpha for implicit preference",
                implicitPrefs="whether to use implicit preference", nonnegative="whether to use nonnegative constraint for least squares",
                coldStartStrategy="strategy for dealing with unknown or new users/items at prediction time: nan, drop",
                seed="random seed", numUserBlocks="number of user blocks", numItemBlocks="number of item blocks",
                userCol="column name for user ids", itemCol="column name for item ids",
                ratingCol="column name for ratings", predictionCol="prediction column name",
                checkpointInterval="checkpoint interval (kept for API parity; factors stay resident in HBM)",
                intermediateStorageLevel="kept for API parity", finalStorageLevel="kept for API parity",
                device="HIP device ordinal (-1 = current)",
                lightMaxDegree="rows with <= this many ratings use the push-through solve (-1 default, 0 off)")

    _uid_prefix = "als"

    def __init__(self, uid=None, **kw):
        from .persistence import random_uid
        self.uid = uid or random_uid(self._uid_prefix)  # Identifiable.randomUID("als")
        self._p = dict(self._defaults)
        for k, v in kw.items():
            self._set(k, v)

    def _set(self, k, v):
        if k not in self._defaults:
            raise IllegalArgumentException(_lib.ALS_E_INVALID_ARGUMENT, f"unknown param {k}")
        if k == "coldStartStrategy":
            v = str(v).lower()
            if v not in ("nan", "drop"):
                raise IllegalArgumentException(_lib.ALS_E_INVALID_ARGUMENT,
                                               f"als parameter coldStartStrategy given invalid value {v}.")
        if k == "checkpointInterval" and not (v == -1 or v >= 1):
            raise IllegalArgumentException(_lib.ALS_E_INVALID_ARGUMENT,
                                           f"als parameter checkpointInterval given invalid value {v}.")
        self._p[k] = v
        return self

    def explainParams(self) -> str:
        lines = []
        for k in self._defaults:
            cur = self._p[k]
            dft = self._defaults[k]
            extra = f"(default: {dft}" + (f", current: {cur})" if cur != dft else ")")
            lines.append(f"{k}: {self._doc.get(k, '')} {extra}")
        return "\n".join(lines)


def _make_accessors(cls):
    for k in _Params._defaults:
        cap = k[0].upper() + k[1:]
        setattr(cls, "set" + cap, (lambda key: lambda self, v: self._set(key, v))(k))
        setattr(cls, "get" + cap, (lambda key: lambda self: self._p[key])(k))
    return cls


@_make_accessors
class ALS(_Params):
    """Spark ml.recommendation.ALS (estimator)."""

    def _c_params(self, pm=None):
        v = dict(self._p)
        if pm:
            v.update(pm)
        p = _lib.als_params()
        check(load().als_params_default(C.byref(p)))
        p.rank = int(v["rank"])
        p.max_iter = int(v["maxIter"])
        p.implicit_prefs = 1 if v["implicitPrefs"] else 0
        p.nonnegative = 1 if v["nonnegative"] else 0
        p.num_user_blocks = int(v["numUserBlocks"])
        p.num_item_blocks = int(v["numItemBlocks"])
        p.reg_param = float(v["regParam"])
        p.alpha = float(v["alpha"])
        p.seed = int(v["seed"])
        p.device = int(v["device"])
        p.light_max_degree = int(v["lightMaxDegree"])
        return p

    def _context(self, pm=None):
        lib = load()
        p = self._c_params(pm)
        h = C.c_void_p()
        check(lib.als_create(C.byref(p), C.byref(h)))
        return h

    def _param_map(self, pm):
        """Validate a ParamMap (dict of param name -> value) like Params.copy(extra)."""
        probe = ALS(uid=self.uid, **self._p)
        for k, v in pm.items():
            probe._set(k, v)
        return dict(probe._p)

    def _ratings(self, dataset, cols):
        user = _checked_cast(_column(dataset, cols["userCol"]), cols["userCol"])
        item = _checked_cast(_column(dataset, cols["itemCol"]), cols["itemCol"])
        rating = np.ascontiguousarray(_column(dataset, cols["ratingCol"]), dtype=np.float32)
        if user.size == 0:
            raise IllegalArgumentException(_lib.ALS_E_INVALID_ARGUMENT,
                                           "No ratings available from the input dataset.")
        return np.ascontiguousarray(user), np.ascontiguousarray(item), rating

    def fit(self, dataset, params=None, initialUserFactors=None, initialItemFactors=None, parallelism=8):
        """ALS.fit (Spark Estimator.fit(dataset[, paramMap | paramMaps])).

        `params` = one ParamMap (dict) -> one ALSModel fitted with those overrides; a list of ParamMaps
        -> a list of ALSModels (the CV grid of ALSRecommenderCV.scala:67-90) that share ONE ingest
        (id remap, both CSR orientations, shards) on the device: between fits only the
        rank-dependent buffers are rebuilt (als_set_params).  The column names must agree across the
        maps.  `initial*Factors` = (ids, factors[n, rank]) injects the start point (parity path, one
        map only); without it the Spark-style XORShiftRandom initialisation is used.  `parallelism`
        (the name of Spark 2.3's CrossValidator knob) caps the maps of a list fitted at once."""
        if isinstance(params, (list, tuple)):
            return self._fit_many(dataset, [self._param_map(pm) for pm in params], max_concurrent=parallelism)
        pm = self._param_map(params or {})
        user, item, rating = self._ratings(dataset, pm)
        lib = load()
        h = self._context(pm)
        try:
            check(lib.als_set_ratings(h, user.size, ptr(user, C.c_int32), ptr(item, C.c_int32),
                                      ptr(rating, C.c_float)))
            for side, init in ((_lib.ALS_USER, initialUserFactors), (_lib.ALS_ITEM, initialItemFactors)):
                if init is not None:
                    ids = np.ascontiguousarray(init[0], dtype=np.int32)
                    f = np.ascontiguousarray(init[1], dtype=np.float32)
                    check(lib.als_set_initial_factors(h, side, ids.size, ptr(ids, C.c_int32), ptr(f, C.c_float)))
            t0 = time.perf_counter()
            check(lib.als_fit(h))
            fit_s = time.perf_counter() - t0
        except Exception:
            lib.als_destroy(h)
            raise
        model = ALSModel(h, pm, uid=self.uid)
        model.fit_seconds = fit_s
        return model

    def _fit_many(self, dataset, maps, max_concurrent=8):
        """The CV grid (ALSRecommenderCV.scala:67-90): one ingest; the maps of one rank are fitted
        CONCURRENTLY, each on an als_fork of the ingest context (own factors and streams, shared CSR)
        driven by its own host thread; every model is bit-identical to its standalone fit.

        Each fork holds its own factor, rotation and split-K buffers, so at most `max_concurrent`
        forks exist at once and fewer when the device runs out of memory: a fork or a fit that fails
        with ALS_E_OUT_OF_MEMORY ends the batch, and its map runs again in a smaller batch (alone, if
        need be: the sequential path)."""
        if not maps:
            return []
        from concurrent.futures import ThreadPoolExecutor
        cols = ("userCol", "itemCol", "ratingCol")
        if any(m[c] != maps[0][c] for m in maps for c in cols):
            raise IllegalArgumentException(_lib.ALS_E_INVALID_ARGUMENT,
                                           "a shared-ingest multi-fit needs the same columns in every ParamMap")
        user, item, rating = self._ratings(dataset, maps[0])
        lib = load()
        h = self._context(maps[0])
        models = [None] * len(maps)

        def run(fh):
            t0 = time.perf_counter()
            check(lib.als_fit(fh))
            return time.perf_counter() - t0

        def oom(e):
            return isinstance(e, _lib.ALSError) and e.code == _lib.ALS_E_OUT_OF_MEMORY

        try:
            for pm in maps:  # validate every map before the ingest (no fit runs on a bad grid)
                check(lib.als_set_params(h, C.byref(self._c_params(pm))))
            check(lib.als_set_ratings(h, user.size, ptr(user, C.c_int32), ptr(item, C.c_int32),
                                      ptr(rating, C.c_float)))
            groups = {}
            for i, pm in enumerate(maps):  # forks share the layout of one (rank, nonnegative, light limit)
                key = (int(pm["rank"]), bool(pm["nonnegative"]), int(pm["lightMaxDegree"]))
                groups.setdefault(key, []).append(i)
            for idx in groups.values():
                check(lib.als_set_params(h, C.byref(self._c_params(maps[idx[0]]))))
                todo = list(idx)
                cap = max(1, int(max_concurrent))
                while todo:
                    forks = []
                    try:
                        for i in todo[:cap]:
                            fh = C.c_void_p()
                            try:
                                check(lib.als_fork(h, C.byref(self._c_params(maps[i])), C.byref(fh)))
                            except _lib.ALSError as e:
                                if not (oom(e) and forks):
                                    raise
                                break  # fit the forks that fit in memory first
                            forks.append((i, fh))
                        with ThreadPoolExecutor(max_workers=len(forks)) as ex:
                            futs = [ex.submit(run, fh) for _, fh in forks]
                        done, failed = [], []
                        for (i, fh), fu in zip(forks, futs):
                            e = fu.exception()
                            if e is None:
                                models[i] = self._snapshot(fh, maps[i], fu.result())
                                done.append(i)
                            elif oom(e) and len(forks) > 1:
                                failed.append(i)
                            else:
                                raise e
                        cap = len(forks) if not failed else max(1, len(forks) // 2)
                        todo = [i for i in todo if i not in done]
                    finally:
                        for _, fh in forks:
                            lib.als_destroy(fh)
        finally:
            lib.als_destroy(h)
        return models

    def _snapshot(self, h, pm, fit_s):
        """A model-only context holding the fitted factors of context h (its ingest can then go)."""
        lib = load()
        k = int(pm["rank"])
        f = {}
        for side in (_lib.ALS_USER, _lib.ALS_ITEM):
            n = lib.als_num_rows(h, side)
            ids = np.empty(n, dtype=np.int32)
            fac = np.empty((n, k), dtype=np.float32)
            check(lib.als_get_factors(h, side, ptr(ids, C.c_int32), ptr(fac, C.c_float)))
            f[side] = (ids, fac)
        mh = C.c_void_p()
        (ui, uf), (ii, itf) = f[_lib.ALS_USER], f[_lib.ALS_ITEM]
        check(lib.als_model_create(k, ui.size, ptr(ui, C.c_int32), ptr(uf, C.c_float), ii.size,
                                   ptr(ii, C.c_int32), ptr(itf, C.c_float), int(pm["device"]), C.byref(mh)))
        m = ALSModel(mh, pm, uid=self.uid)
        m._cache.update(f)
        m.fit_seconds = fit_s
        return m


@_make_accessors
class ALSModel(_Params):
    """Spark ml.recommendation.ALSModel over an engine context holding both factor matrices."""

    def __init__(self, handle, params, uid=None):
        super().__init__(uid=uid)
        self._p.update(params)
        self._h = handle
        self._cache = {}

    def __del__(self):
        h = getattr(self, "_h", None)
        if h:
            try:
                load().als_destroy(h)
            except Exception:
                pass
            self._h = None

    @property
    def rank(self) -> int:
        return int(load().als_rank(self._h))

    def _factors(self, side):
        if side not in self._cache:
            lib = load()
            n = lib.als_num_rows(self._h, side)
            ids = np.empty(n, dtype=np.int32)
            f = np.empty((n, self.rank), dtype=np.float32)
            check(lib.als_get_factors(self._h, side, ptr(ids, C.c_int32), ptr(f, C.c_float)))
            self._cache[side] = (ids, f)
        return self._cache[side]

    def user_factors_np(self):
        return self._factors(_lib.ALS_USER)

    def item_factors_np(self):
        return self._factors(_lib.ALS_ITEM)

    @staticmethod
    def _frame(ids, f):
        import pandas as pd
        return pd.DataFrame({"id": ids, "features": list(f)})

    @property
    def userFactors(self):
        return self._frame(*self.user_factors_np())

    @property
    def itemFactors(self):
        return self._frame(*self.item_factors_np())

    # ---- ALSModel.transform ---------------------------------------------------------------------
    def transform(self, dataset):
        import pandas as pd
        user = _checked_cast(_column(dataset, self._p["userCol"]), self._p["userCol"])
        item = _checked_cast(_column(dataset, self._p["itemCol"]), self._p["itemCol"])
        out = np.empty(user.size, dtype=np.float32)
        check(load().als_predict(self._h, user.size, ptr(np.ascontiguousarray(user), C.c_int32),
                                 ptr(np.ascontiguousarray(item), C.c_int32), ptr(out, C.c_float)))
        df = pd.DataFrame(dataset).copy() if not isinstance(dataset, pd.DataFrame) else dataset.copy()
        df[self._p["predictionCol"]] = out
        if self._p["coldStartStrategy"] == "drop":
            df = df[~np.isnan(out)]
        return df

    # ---- recommendForAll* / recommendFor*Subset ------------------------------------------------
    def _recommend(self, side, num, subset=None):
        lib = load()
        if subset is not None:
            col = self._p["userCol"] if side == _lib.ALS_USER else self._p["itemCol"]
            # checkedCast like fit/transform: out-of-Int-range or fractional ids raise, never wrap
            sub = np.ascontiguousarray(np.unique(_checked_cast(subset, col)))
            nq = sub.size
        else:
            sub = None
            nq = lib.als_num_rows(self._h, side)
        src = np.empty(nq, dtype=np.int32)
        ids = np.empty((nq, num), dtype=np.int32)
        sc = np.empty((nq, num), dtype=np.float32)
        check(lib.als_recommend(self._h, side, int(num), ptr(sub, C.c_int32) if sub is not None else None,
                                nq, ptr(src, C.c_int32), ptr(ids, C.c_int32), ptr(sc, C.c_float)))
        return src, ids, sc

    def recommend_np(self, num, subset=None, side=_lib.ALS_USER):
        """(src ids, dst ids [n, num], scores [n, num]) sorted (score desc, id asc); -1/NaN padding."""
        return self._recommend(side, num, subset)

    def _rec_frame(self, src, ids, sc, src_col, dst_col):
        import pandas as pd
        recs = []
        for r in range(len(src)):
            m = ids[r] >= 0
            recs.append([(int(i), float(s)) for i, s in zip(ids[r][m], sc[r][m])])
        keep = [i for i in range(len(src)) if recs[i]]
        return pd.DataFrame({src_col: src[keep], "recommendations": [recs[i] for i in keep]})

    def recommendForAllUsers(self, numItems):
        return self._rec_frame(*self._recommend(_lib.ALS_USER, numItems), self._p["userCol"], self._p["itemCol"])

    def recommendForAllItems(self, numUsers):
        return self._rec_frame(*self._recommend(_lib.ALS_ITEM, numUsers), self._p["itemCol"], self._p["userCol"])

    def recommendForUserSubset(self, dataset, numItems):
        users = _column(dataset, self._p["userCol"])
        return self._rec_frame(*self._recommend(_lib.ALS_USER, numItems, users), self._p["userCol"],
                               self._p["itemCol"])

    def recommendForItemSubset(self, dataset, numUsers):
        items = _column(dataset, self._p["itemCol"])
        return self._rec_frame(*self._recommend(_lib.ALS_ITEM, numUsers, items), self._p["itemCol"],
                               self._p["userCol"])

    # ---- RankingEvaluator on the device (RankingEvaluator.scala:83-139) ----------------------------
    def evaluate_ndcg(self, users, items, keys, k=30, per_user=False):
        """NDCG@k of this model's top-k recommendations against intoUserActualItems(users, items,
        keys desc, k), computed on the device (als_evaluate_ndcg): the albedo protocol of
        ALSRecommenderBuilder.scala:92-104 without the lists leaving HBM.  Returns the mean, or
        (mean, user ids, per-user values) with per_user=True."""
        lib = load()
        u = np.ascontiguousarray(_checked_cast(users, self._p["userCol"]))
        it = np.ascontiguousarray(_checked_cast(items, self._p["itemCol"]))
        ky = np.asarray(keys)
        if ky.dtype.kind == "M":  # starred_at timestamps
            ky = ky.astype("datetime64[us]").astype(np.int64)
        ky = np.ascontiguousarray(ky, dtype=np.int64)
        if not (u.size == it.size == ky.size):
            raise ValueError("users, items and keys must have the same length")
        mean = C.c_double()
        nu = C.c_int64()
        cap = int(np.unique(u).size) if per_user else 0
        uo = np.empty(max(cap, 1), np.int32)
        vo = np.empty(max(cap, 1), np.float64)
        check(lib.als_evaluate_ndcg(self._h, int(k), u.size, ptr(u, C.c_int32), ptr(it, C.c_int32),
                                    ptr(ky, C.c_int64), C.byref(mean), C.byref(nu),
                                    ptr(uo, C.c_int32) if per_user else None,
                                    ptr(vo, C.c_double) if per_user else None, cap))
        if per_user:
            return mean.value, uo[:nu.value], vo[:nu.value]
        return mean.value

    # ---- persistence (Spark 2.2 ALSModelWriter / ALSModelReader layout: albedo_amd/persistence.py) ----
    MODEL_PARAMS = ("userCol", "itemCol", "predictionCol", "coldStartStrategy")  # ALSModelParams

    def save(self, path, overwrite=False, rows_per_part=1 << 20):
        from . import persistence
        persistence.save_als_model(path, self.uid, {k: self._p[k] for k in self.MODEL_PARAMS}, self.rank,
                                   self.user_factors_np(), self.item_factors_np(), overwrite, rows_per_part)

    def write(self):
        model = self

        class _Writer:
            _ow = False

            def overwrite(self):
                self._ow = True
                return self

            def save(self, path):
                model.save(path, overwrite=self._ow)

        return _Writer()

    @classmethod
    def load(cls, path, device=-1):
        from . import persistence
        meta, (uid, uf), (iid, itf) = persistence.load_als_model(path)
        rank = int(meta["rank"])
        h = C.c_void_p()
        check(load().als_model_create(rank, uid.size, ptr(uid, C.c_int32), ptr(uf, C.c_float), iid.size,
                                      ptr(iid, C.c_int32), ptr(itf, C.c_float), int(device), C.byref(h)))
        params = dict(_Params._defaults)
        params.update({k: v for k, v in meta.get("paramMap", {}).items() if k in _Params._defaults})
        params["rank"] = rank
        model = cls(h, params, uid=meta.get("uid"))
        return model
