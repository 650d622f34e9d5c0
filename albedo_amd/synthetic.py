"""Seeded synthetic GitHub-like star matrices (the workloads of BASELINE.json configs).

The reference trains on the `app_repostarring` table (`DatasetUtils.scala:111-123`): one row per
(user_id, repo_id) pair, unique (`app/models.py:166-167`), `starring = 1.0` for every row
(`DatasetUtils.scala:118`).  That dump is not available offline, so every config is
a synthetic stand-in with the shape SURVEY.md §8(d) fixes:

* repo popularity  w_j ∝ (j+1)^-s  over a seeded shuffle of repo positions (optionally a "head":
  fixed draw probabilities for the top ranks, config c5's >1M-star repos);
* user degree      P(d) ∝ d^-1.8 on [1, min(dmax, I)], rescaled to exactly N nonzeros;
* per-user draws without replacement (duplicates are re-drawn, `rounds` times at most);
* sparse Int ids through an odd-multiplier bijection of [0, 2^31) so the engine's id remap is
  exercised; rating ≡ 1.0f.

Every random draw is a pure function of (seed, stream, index) through splitmix64, so the device
generator in `libalbedo_als.so` (`als_synth_generate` / `als_set_ratings_synthetic`) reproduces this host generator exactly:
the host computes the per-user degree array and the cumulative popularity table (sequential
numpy, small) and the device does the per-nonzero sampling and de-duplication.
"""
from __future__ import annotations

import dataclasses

import numpy as np

MASK64 = np.uint64(0xFFFFFFFFFFFFFFFF)
GOLD = np.uint64(0x9E3779B97F4A7C15)
M1 = np.uint64(0xBF58476D1CE4E5B9)
M2 = np.uint64(0x94D049BB133111EB)
STREAM_MUL = np.uint64(0xD1B54A32D192ED03)

USER_ID_MUL, USER_ID_ADD = 0x9E3779B1, 0x2545F491
ITEM_ID_MUL, ITEM_ID_ADD = 0x85EBCA77, 0x1B873593


def splitmix64(x: np.ndarray) -> np.ndarray:
    with np.errstate(over="ignore"):
        z = (np.asarray(x, dtype=np.uint64) + GOLD) & MASK64
        z = ((z ^ (z >> np.uint64(30))) * M1) & MASK64
        z = ((z ^ (z >> np.uint64(27))) * M2) & MASK64
        return z ^ (z >> np.uint64(31))


def stream_key(seed: int, stream: int) -> np.uint64:
    with np.errstate(over="ignore"):
        s = np.uint64(seed & 0xFFFFFFFFFFFFFFFF) ^ (np.uint64(stream) * STREAM_MUL)
    return splitmix64(np.array([s], dtype=np.uint64))[0]


def uniform(seed: int, stream: int, idx: np.ndarray) -> np.ndarray:
    """U[0,1) doubles, one per index: (splitmix64(key + idx) >> 11) * 2^-53."""
    key = stream_key(seed, stream)
    with np.errstate(over="ignore"):
        z = splitmix64((np.asarray(idx, dtype=np.uint64) + key) & MASK64)
    return (z >> np.uint64(11)).astype(np.float64) * (1.0 / 9007199254740992.0)


def user_ids(n: int) -> np.ndarray:
    i = np.arange(n, dtype=np.int64)
    return ((i * USER_ID_MUL + USER_ID_ADD) & 0x7FFFFFFF).astype(np.int32)


def item_ids(n: int) -> np.ndarray:
    i = np.arange(n, dtype=np.int64)
    return ((i * ITEM_ID_MUL + ITEM_ID_ADD) & 0x7FFFFFFF).astype(np.int32)


@dataclasses.dataclass(frozen=True)
class SynthSpec:
    n_users: int
    n_items: int
    nnz: int
    zipf_s: float = 0.7
    degree_exp: float = 1.8
    dmax: int = 20000
    seed: int = 42
    rounds: int = 8
    head: tuple = ()  # draw probabilities of the top popularity ranks (the rest: Zipf body)

    def degree_cap(self) -> int:
        # keep every user at most half the catalogue so draws without replacement converge
        return max(1, min(self.dmax, self.n_items // 2 if self.n_items > 1 else 1))


CONFIGS = {
    # BASELINE.json configs, shapes from SURVEY.md §8(d)
    "c1p": SynthSpec(1_000_000, 200_000, 50_000_000, zipf_s=0.7),
    "c2": SynthSpec(1_000_000, 200_000, 50_000_000, zipf_s=0.7),
    "c4": SynthSpec(20_000_000, 4_000_000, 1_000_000_000, zipf_s=0.8),
    # config 5 asks for "extreme degree skew (top repos >1M stars)": a Zipf(0.9) body alone tops
    # out at ~0.79M stars (most users star 1-2 repos, so a repo's reach saturates), so the three
    # most popular repos take 12 % / 9 % / 7 % of the draws: ~1.7M / 1.4M / 1.2M stars
    "c5": SynthSpec(5_000_000, 500_000, 100_000_000, zipf_s=0.9, head=(0.12, 0.09, 0.07)),
}


def user_degrees(spec: SynthSpec) -> np.ndarray:
    """Per-user degree: continuous Pareto(0.8) inverse-CDF on [1, cap], rescaled to sum to nnz."""
    U, N = spec.n_users, spec.nnz
    cap = spec.degree_cap()
    if N > U * cap:
        raise ValueError("nnz exceeds users x per-user cap")
    a = spec.degree_exp - 1.0
    u = uniform(spec.seed, 1, np.arange(U))
    tail = 1.0 - float(cap) ** (-a)
    d_raw = (1.0 - u * tail) ** (-1.0 / a)
    scaled = d_raw * (N / float(np.sum(d_raw)))
    d = np.clip(np.floor(scaled), 1, cap).astype(np.int64)
    # hand out (or take back) the remainder deterministically: by fractional part, then index
    frac = scaled - np.floor(scaled)
    rem = N - int(d.sum())
    order = np.lexsort((np.arange(U), -frac))
    while rem != 0:
        if rem > 0:
            room = order[d[order] < cap]
            take = room[:rem]
            d[take] += 1
            rem -= len(take)
        else:
            spare = order[::-1][d[order[::-1]] > 1]
            take = spare[: -rem]
            d[take] -= 1
            rem += len(take)
    return d


def popularity_table(spec: SynthSpec):
    """(cumulative weights over popularity rank, rank -> repo position permutation)."""
    I = spec.n_items
    w = (np.arange(1, I + 1, dtype=np.float64)) ** (-spec.zipf_s)
    if spec.head:
        h = np.asarray(spec.head, dtype=np.float64)
        w *= (1.0 - h.sum()) / w.sum()
        w[: h.size] += h
    cw = np.cumsum(w)
    perm = np.random.Generator(np.random.PCG64(spec.seed)).permutation(I).astype(np.int32)
    return cw, perm


def sample_items(spec: SynthSpec, cw: np.ndarray, perm: np.ndarray, slots: np.ndarray, attempt: int):
    u = uniform(spec.seed, 2 + attempt, slots)
    j = np.searchsorted(cw, u * cw[-1], side="right")
    j = np.minimum(j, len(cw) - 1)
    return perm[j]


def generate(spec: SynthSpec, with_timestamps: bool = False):
    """Return dict(user, item, rating[, ts]) as COO in slot order (grouped by user)."""
    U, I, N = spec.n_users, spec.n_items, spec.nnz
    deg = user_degrees(spec)
    cw, perm = popularity_table(spec)
    rows = np.repeat(np.arange(U, dtype=np.int64), deg)
    slots = np.arange(N, dtype=np.int64)
    item = sample_items(spec, cw, perm, slots, 0).astype(np.int64)
    alive = np.ones(N, dtype=bool)
    for attempt in range(1, spec.rounds + 1):
        key = rows * I + item
        order = np.lexsort((slots, key))  # by key, then slot: the first slot of a pair keeps it
        ks = key[order]
        dup_sorted = np.zeros(N, dtype=bool)
        dup_sorted[1:] = ks[1:] == ks[:-1]
        dup = np.zeros(N, dtype=bool)
        dup[order] = dup_sorted
        if not dup.any():
            break
        redo = slots[dup]
        item[redo] = sample_items(spec, cw, perm, redo, attempt)
    else:
        key = rows * I + item
        order = np.lexsort((slots, key))
        ks = key[order]
        dup_sorted = np.zeros(N, dtype=bool)
        dup_sorted[1:] = ks[1:] == ks[:-1]
        alive[order[dup_sorted]] = False
    out = {
        "user": user_ids(U)[rows[alive]],
        "item": item_ids(I)[item[alive]],
        "rating": np.ones(int(alive.sum()), dtype=np.float32),
    }
    if with_timestamps:
        out["ts"] = (uniform(spec.seed, 99, slots[alive]) * 3.0e8).astype(np.int64) + 1_300_000_000
    return out
