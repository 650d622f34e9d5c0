"""fp64 CPU restatement of Spark MLlib 2.2.0 ALS (+ albedo's scorer/evaluator) — TEST ORACLE ONLY.

See oracle/__init__.py for the import rule and the pinning status ("ALS loop parity unpinned
against Spark; dppsv / ndcgAt / NNLS optimum pinned").  Spark sources are not in the container;
upstream functions are cited by their path in apache/spark@v2.2.0 together with the albedo call
site that reaches them.
"""
from __future__ import annotations

import math
import struct
from dataclasses import dataclass

import numpy as np
import scipy.linalg.lapack as lapack

# --------------------------------------------------------------------------------------------
# Data blocks (Spark `ALS.partitionRatings` / `makeBlocks` / `InBlock` CSR; reached from
# `ALSRecommenderBuilder.scala:58` -> ALS.fit -> ALS.train).  We keep one block per side: the
# block split only changes fp64 summation order, not the math.
# --------------------------------------------------------------------------------------------


@dataclass
class Blocks:
    user_ids: np.ndarray  # ascending unique raw ids (int32)
    item_ids: np.ndarray
    # user-major CSR (dst = users, src = items) and item-major CSR (dst = items, src = users)
    u_ptr: np.ndarray
    u_col: np.ndarray
    u_val: np.ndarray
    i_ptr: np.ndarray
    i_col: np.ndarray
    i_val: np.ndarray


def make_blocks(user, item, rating) -> Blocks:
    user = np.asarray(user, dtype=np.int32)
    item = np.asarray(item, dtype=np.int32)
    rating = np.asarray(rating, dtype=np.float32)  # ALS.fit casts the rating column to Float
    if user.size == 0:
        raise ValueError("No ratings available from the input")
    uids, ud = np.unique(user, return_inverse=True)
    iids, idn = np.unique(item, return_inverse=True)

    def csr(dst, src, n_dst):
        order = np.lexsort((src, dst))
        ptr = np.zeros(n_dst + 1, dtype=np.int64)
        np.add.at(ptr, dst + 1, 1)
        return np.cumsum(ptr), src[order].astype(np.int32), rating[order]

    u_ptr, u_col, u_val = csr(ud, idn, len(uids))
    i_ptr, i_col, i_val = csr(idn, ud, len(iids))
    return Blocks(uids.astype(np.int32), iids.astype(np.int32), u_ptr, u_col, u_val, i_ptr, i_col, i_val)


# --------------------------------------------------------------------------------------------
# Spark-compatible initialisation, best effort (unverifiable offline).
# upstream: ml/recommendation/ALS.scala `initialize`, util/random/XORShiftRandom.scala,
# scala.util.hashing.MurmurHash3.bytesHash / byteswap64, java.util.Random.nextGaussian.
# --------------------------------------------------------------------------------------------

_M32 = 0xFFFFFFFF
_M64 = 0xFFFFFFFFFFFFFFFF


def _rotl32(x, r):
    return ((x << r) | (x >> (32 - r))) & _M32


def _mix_last(h, k):
    k = (k * 0xCC9E2D51) & _M32
    k = _rotl32(k, 15)
    k = (k * 0x1B873593) & _M32
    return h ^ k


def _mix(h, k):
    h = _mix_last(h, k)
    h = _rotl32(h, 13)
    return (h * 5 + 0xE6546B64) & _M32


def _avalanche(h):
    h ^= h >> 16
    h = (h * 0x85EBCA6B) & _M32
    h ^= h >> 13
    h = (h * 0xC2B2AE35) & _M32
    h ^= h >> 16
    return h


def murmur3_bytes_hash(data: bytes, seed: int = 0x3C074A61) -> int:
    h = seed & _M32
    n = len(data)
    i = 0
    while n - i >= 4:
        k = data[i] | (data[i + 1] << 8) | (data[i + 2] << 16) | (data[i + 3] << 24)
        h = _mix(h, k)
        i += 4
    rem = n - i
    k = 0
    if rem == 3:
        k ^= data[i + 2] << 16
    if rem >= 2:
        k ^= data[i + 1] << 8
    if rem >= 1:
        k ^= data[i]
        h = _mix_last(h, k)
    return _avalanche(h ^ n)


def _to_signed32(x):
    x &= _M32
    return x - (1 << 32) if x & 0x80000000 else x


def _to_signed64(x):
    x &= _M64
    return x - (1 << 64) if x & (1 << 63) else x


def hash_seed(seed: int) -> int:
    # ByteBuffer.allocate(java.lang.Long.SIZE = 64 bytes).putLong(seed): big-endian + 56 zeros
    data = struct.pack(">q", _to_signed64(seed)) + bytes(56)
    low = murmur3_bytes_hash(data)
    high = murmur3_bytes_hash(data, low)
    return ((high << 32) | low) & _M64


def byteswap64(v: int) -> int:
    hc = (v * 0x9E3775CD9E3775CD) & _M64
    hc = int.from_bytes(hc.to_bytes(8, "little"), "big")
    return (hc * 0x9E3775CD9E3775CD) & _M64


class XORShiftRandom:
    def __init__(self, init: int):
        self.seed = hash_seed(init)
        self._have_next = False
        self._next_gauss = 0.0

    def next(self, bits: int) -> int:
        s = self.seed
        s ^= (s << 21) & _M64
        s ^= s >> 35
        s ^= (s << 4) & _M64
        self.seed = s
        return _to_signed32(s & ((1 << bits) - 1))

    def next_long(self) -> int:
        return _to_signed64((self.next(32) << 32) + self.next(32))

    def next_double(self) -> float:
        return ((self.next(26) << 27) + self.next(27)) * (1.0 / (1 << 53))

    def next_gaussian(self) -> float:
        if self._have_next:
            self._have_next = False
            return self._next_gauss
        while True:
            v1 = 2 * self.next_double() - 1
            v2 = 2 * self.next_double() - 1
            s = v1 * v1 + v2 * v2
            if s < 1 and s != 0:
                break
        mul = math.sqrt(-2 * math.log(s) / s)
        self._next_gauss = v2 * mul
        self._have_next = True
        return v1 * mul


def f2j_snrm2(x: np.ndarray) -> np.float32:
    """netlib BLAS snrm2.f (scaled sum of squares), float32 arithmetic."""
    f = np.float32
    scale, ssq = f(0.0), f(1.0)
    for v in x.astype(np.float32):
        if v != 0:
            a = f(abs(v))
            if scale < a:
                q = f(scale / a)
                ssq = f(f(1.0) + f(ssq * f(q * q)))
                scale = a
            else:
                q = f(a / scale)
                ssq = f(ssq + f(q * q))
    return f(scale * f(np.sqrt(ssq)))


def spark_side_seeds(seed: int):
    g = XORShiftRandom(seed)
    return g.next_long(), g.next_long()  # (user side, item side)


def spark_initialize(ids_sorted: np.ndarray, rank: int, side_seed: int, num_blocks: int = 10):
    """ALS.initialize: per block b, XORShiftRandom(byteswap64(seed ^ b)) over the block's ascending ids."""
    ids_sorted = np.asarray(ids_sorted, dtype=np.int64)
    out = np.zeros((len(ids_sorted), rank), dtype=np.float32)
    blk = ((ids_sorted % num_blocks) + num_blocks) % num_blocks
    for b in range(num_blocks):
        rows = np.nonzero(blk == b)[0]
        if len(rows) == 0:
            continue
        rnd = XORShiftRandom(_to_signed64(byteswap64((side_seed ^ b) & _M64)))
        for r in rows:
            v = np.array([np.float32(rnd.next_gaussian()) for _ in range(rank)], dtype=np.float32)
            nrm = f2j_snrm2(v)
            out[r] = v * np.float32(np.float32(1.0) / nrm)
    return out


# --------------------------------------------------------------------------------------------
# The solve (ml/recommendation/ALS.scala: computeYtY, NormalEquation, CholeskySolver,
# NNLSSolver; mllib/optimization/NNLS.scala; mllib/linalg/CholeskyDecomposition.scala).
# --------------------------------------------------------------------------------------------


class NotPositiveDefinite(ValueError):
    pass


def gram(Y: np.ndarray) -> np.ndarray:
    """computeYtY: Σ_rows y yᵀ in fp64 from fp32 factors."""
    Y64 = np.asarray(Y, dtype=np.float64)
    return Y64.T @ Y64


def pack_upper(A: np.ndarray) -> np.ndarray:
    """Column-major packed upper triangle (LAPACK 'U' / Spark NormalEquation.ata layout)."""
    return np.ascontiguousarray(A.T[np.tril_indices(A.shape[0])])


def cholesky_solve(A: np.ndarray, b: np.ndarray, lam: float) -> np.ndarray:
    """CholeskySolver.solve: ata[diag] += lambda; LAPACK dppsv('U'); cast to Float."""
    k = A.shape[0]
    A = A + lam * np.eye(k)
    x, info = lapack.dppsv(k, pack_upper(A), np.asarray(b, dtype=np.float64).reshape(k, 1))
    if info > 0:
        raise NotPositiveDefinite(
            f"LAPACK.dppsv returned {info} because A is not positive definite. Is A derived from "
            "a singular matrix (e.g. collinear column values)?")
    if info < 0:
        raise RuntimeError(f"LAPACK.dppsv returned {info}")
    return x[:, 0].astype(np.float32)


def nnls(ata: np.ndarray, atb: np.ndarray) -> np.ndarray:
    """mllib/optimization/NNLS.scala `solve`: projected gradient with CG acceleration (fp64)."""
    n = len(atb)
    x = np.zeros(n)
    last_dir = np.zeros(n)
    last_norm = 0.0
    iter_max = max(400, 20 * n)
    last_wall = 0
    iterno = 0

    def steplen(d, res):
        top = float(d @ res)
        scratch = ata @ d
        return top / (float(scratch @ d) + 1e-20)

    def stop(step, ndir, nx):
        return (math.isnan(step) or step < 1e-7 or step > 1e40 or ndir < 1e-12 * nx or ndir < 1e-32)

    while iterno < iter_max:
        res = ata @ x - atb
        grad = res.copy()
        grad[(grad > 0.0) & (x == 0.0)] = 0.0
        ngrad = float(grad @ grad)
        d = grad.copy()
        step = steplen(grad, res)
        nx = float(x @ x)
        if iterno > last_wall + 1:
            alpha = ngrad / last_norm
            d = d + alpha * last_dir
            dstep = steplen(d, res)
            ndir = float(d @ d)
            if stop(dstep, ndir, nx):
                d = grad.copy()
                ndir = float(d @ d)
            else:
                step = dstep
        else:
            ndir = float(d @ d)
        if stop(step, ndir, nx):
            return x.copy()
        for i in range(n):
            if step * d[i] > x[i]:
                step = x[i] / d[i]
        for i in range(n):
            if step * d[i] > x[i] * (1 - 1e-14):
                x[i] = 0.0
                last_wall = iterno
            else:
                x[i] -= step * d[i]
        iterno += 1
        last_dir = d.copy()
        last_norm = ngrad
    return x.copy()


def nnls_solve(A: np.ndarray, b: np.ndarray, lam: float) -> np.ndarray:
    """NNLSSolver.solve: fillAtA (full symmetric + lambda on the diagonal), NNLS, cast to Float."""
    A = A + lam * np.eye(A.shape[0])
    return nnls(A, np.asarray(b, dtype=np.float64)).astype(np.float32)


def normal_equation(Ysrc, ptr, col, val, j, implicit, alpha, G):
    """computeFactors inner loop for dst row j: returns (A, b, numExplicits) in fp64."""
    p0, p1 = int(ptr[j]), int(ptr[j + 1])
    Yj = np.asarray(Ysrc[col[p0:p1]], dtype=np.float64)
    r = np.asarray(val[p0:p1], dtype=np.float64)
    if implicit:
        c1 = alpha * np.abs(r)
        pos = r > 0.0
        A = G + (Yj.T * c1) @ Yj
        b = Yj.T @ np.where(pos, 1.0 + c1, 0.0)
        n = int(pos.sum())
    else:
        A = Yj.T @ Yj
        b = Yj.T @ r
        n = p1 - p0
    return A, b, n


def half_sweep(Ysrc, ptr, col, val, *, reg, alpha, implicit=True, nonnegative=False, return_ne=False):
    """One computeFactors call: every dst row solved from the current src factors."""
    n_dst = len(ptr) - 1
    k = Ysrc.shape[1]
    G = gram(Ysrc) if implicit else None
    X = np.zeros((n_dst, k), dtype=np.float32)
    nes = []
    for j in range(n_dst):
        A, b, n = normal_equation(Ysrc, ptr, col, val, j, implicit, alpha, G)
        lam = reg * n
        X[j] = nnls_solve(A, b, lam) if nonnegative else cholesky_solve(A, b, lam)
        if return_ne:
            nes.append((A, b, n))
    return (X, nes) if return_ne else X


def fit(blocks: Blocks, *, rank, max_iter, reg, alpha, implicit=True, nonnegative=False,
        init_user=None, init_item=None, seed=42, num_blocks=10):
    """ALS.train outer loop: per iteration item half-sweep (from users) then user half-sweep."""
    if init_user is None or init_item is None:
        su, si = spark_side_seeds(seed)
        init_user = spark_initialize(blocks.user_ids, rank, su, num_blocks) if init_user is None else init_user
        init_item = spark_initialize(blocks.item_ids, rank, si, num_blocks) if init_item is None else init_item
    U = np.asarray(init_user, dtype=np.float32).copy()
    V = np.asarray(init_item, dtype=np.float32).copy()
    kw = dict(reg=reg, alpha=alpha, implicit=implicit, nonnegative=nonnegative)
    for _ in range(max_iter):
        V = half_sweep(U, blocks.i_ptr, blocks.i_col, blocks.i_val, **kw)
        U = half_sweep(V, blocks.u_ptr, blocks.u_col, blocks.u_val, **kw)
    return U, V


# --------------------------------------------------------------------------------------------
# Scoring / top-k (albedo ALSRecommender.scala:28-65, BoundedPriorityQueue.scala:30-53; Spark
# ALSModel.recommendForAll + TopByKeyAggregator) and ALSModel.transform's per-pair sdot.
# --------------------------------------------------------------------------------------------


def f2j_sdot(X: np.ndarray, Y: np.ndarray) -> np.ndarray:
    """netlib sdot.f as translated by F2J (ALSRecommender.scala:51): float32, no FMA.

    Head of n mod 5 products summed left to right, then groups of five added left to right:
    stemp = ((((stemp + x_i y_i) + x_{i+1} y_{i+1}) + ...).  Broadcasts X[..., k] against Y[..., k].
    """
    X = np.asarray(X, dtype=np.float32)
    Y = np.asarray(Y, dtype=np.float32)
    n = X.shape[-1]
    acc = np.zeros(np.broadcast_shapes(X.shape[:-1], Y.shape[:-1]), dtype=np.float32)
    for i in range(n):  # the 5-way unroll is left-to-right too, so the order is plain sequential
        acc = (acc + (X[..., i] * Y[..., i])).astype(np.float32)
    return acc


class BoundedPriorityQueue:
    """BoundedPriorityQueue.scala:16-53: keeps the top maxSize; replaces the head (the lowest)
    only when the new element is strictly greater, so ties keep the first-seen element."""

    def __init__(self, max_size, key):
        import heapq
        self._h = []
        self._heapq = heapq
        self._n = max_size
        self._key = key
        self._seq = 0

    def add(self, elem):
        k = self._key(elem)
        if len(self._h) < self._n:
            # heap of (key, -insertion seq): among equal keys the LATEST inserted is the head,
            # java.util.PriorityQueue leaves the order of equal keys unspecified; only the
            # strictly-greater replacement rule is observable in the kept set.
            self._heapq.heappush(self._h, (k, self._seq, elem))
        elif self._h and k > self._h[0][0]:
            self._heapq.heapreplace(self._h, (k, self._seq, elem))
        self._seq += 1

    def items(self):
        return [e for _, _, e in self._h]


def recommend_for_all(src_ids, src_f, dst_ids, dst_f, num):
    """Top-`num` dst per src by F2J sdot score, tie-break (score desc, dst id asc).

    Equals BoundedPriorityQueue over dst rows visited in ascending id order (first seen = lower id
    wins the boundary tie) followed by TopByKeyAggregator's descending sort.
    Returns (ids[n_src, num], scores[n_src, num]); rows shorter than num are padded with -1/NaN.
    """
    dst_ids = np.asarray(dst_ids)
    order = np.argsort(dst_ids, kind="stable")
    dst_ids = dst_ids[order]
    dst_f = np.asarray(dst_f, dtype=np.float32)[order]
    n_src = len(src_ids)
    m = min(num, len(dst_ids))
    out_ids = np.full((n_src, num), -1, dtype=np.int32)
    out_sc = np.full((n_src, num), np.nan, dtype=np.float32)
    chunk = max(1, (1 << 24) // max(1, len(dst_ids)))
    for s0 in range(0, n_src, chunk):
        S = f2j_sdot(np.asarray(src_f[s0:s0 + chunk], dtype=np.float32)[:, None, :], dst_f[None, :, :])
        for r in range(S.shape[0]):
            sc = S[r]
            idx = np.lexsort((dst_ids, -sc.astype(np.float64)))[:m]
            out_ids[s0 + r, :m] = dst_ids[idx]
            out_sc[s0 + r, :m] = sc[idx]
    return out_ids, out_sc


# --------------------------------------------------------------------------------------------
# Evaluation (RankingEvaluator.scala:83-139 -> mllib/evaluation/RankingMetrics.scala ndcgAt)
# --------------------------------------------------------------------------------------------


def ndcg_at(pairs, k: int) -> float:
    if k <= 0:
        raise ValueError("ranking position k should be positive")
    vals = []
    for pred, lab in pairs:
        lab_set = set(int(x) for x in lab)
        if lab_set:
            n = min(max(len(pred), len(lab_set)), k)
            max_dcg = dcg = 0.0
            for i in range(n):
                gain = 1.0 / math.log(i + 2)
                if i < len(pred) and int(pred[i]) in lab_set:
                    dcg += gain
                if i < len(lab_set):
                    max_dcg += gain
            vals.append(dcg / max_dcg)
        else:
            vals.append(0.0)
    return float(np.mean(vals)) if vals else float("nan")


def into_user_items(user, item, order_key, k):
    """intoUserActualItems / intoUserPredictedItems: rank() over (user ORDER BY key desc) <= k,
    collect_list; the list order is made deterministic as (key desc, item asc)."""
    user = np.asarray(user)
    item = np.asarray(item)
    key = np.asarray(order_key, dtype=np.float64)
    order = np.lexsort((item, -key, user))
    out = {}
    u_s, i_s, k_s = user[order], item[order], key[order]
    start = 0
    n = len(u_s)
    while start < n:
        end = start
        while end < n and u_s[end] == u_s[start]:
            end += 1
        keys = k_s[start:end]
        # rank() = 1 + number of strictly greater keys in the partition (ties share a rank)
        ranks = 1 + np.searchsorted(-keys, -keys, side="left")
        out[int(u_s[start])] = [int(x) for x in i_s[start:end][ranks <= k]]
        start = end
    return out


def evaluate_ndcg(predicted: dict, actual: dict, k: int) -> float:
    """RankingEvaluator.evaluate: inner join on user, slice both lists to k, ndcgAt(k)."""
    pairs = [(predicted[u][:k], actual[u][:k]) for u in predicted if u in actual]
    return ndcg_at(pairs, k)
