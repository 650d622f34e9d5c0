"""World-size-2 runs of the sharded path (one process per rank, gloo between them)."""
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

from oracle import spark_als as O
from tests.conftest import ROOT


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _launch(mode, out, world=2, timeout=300, env_extra=None, k=16):
    port = _free_port()
    procs = []
    for r in range(world):
        env = dict(os.environ, RANK=str(r), WORLD_SIZE=str(world), LOCAL_RANK="0", MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port), **(env_extra or {}))
        procs.append(subprocess.Popen([sys.executable, os.path.join(ROOT, "tests", "mp_worker.py"), mode, out, str(k)],
                                      env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT))
    outs = []
    for p in procs:
        try:
            o, _ = p.communicate(timeout=timeout)
        except subprocess.TimeoutExpired:
            for q in procs:
                q.kill()
            raise
        outs.append(o.decode(errors="replace"))
    for p, o in zip(procs, outs):
        assert p.returncode == 0, o[-3000:]
    return np.load(out)


def _problem(k=16):
    from albedo_amd.synthetic import SynthSpec, generate
    d = generate(SynthSpec(1200, 400, 16000, seed=41))
    B = O.make_blocks(d["user"], d["item"], d["rating"])
    rng = np.random.default_rng(3)
    U0 = rng.standard_normal((len(B.user_ids), k)).astype(np.float32)
    V0 = rng.standard_normal((len(B.item_ids), k)).astype(np.float32)
    return B, U0, V0


def _fit_ref(B, U0, V0, k, max_iter, nonneg):
    """O.fit (Spark order: item half, then user half); the NNLS halves through the C restatement of
    NNLSSolver (oracle/c/als_cpu.c, equal to oracle/spark_als.py:nnls: tests/test_oracle.py) so that
    rank 256 stays within seconds."""
    if not nonneg:
        return O.fit(B, rank=k, max_iter=max_iter, reg=0.5, alpha=40.0, init_user=U0, init_item=V0)
    from oracle import cbind
    U, V = U0, V0
    for _ in range(max_iter):
        V, _ = cbind.solve_rows_nnls(U, O.gram(U), B.i_ptr, B.i_col, B.i_val, reg=0.5, alpha=40.0)
        U, _ = cbind.solve_rows_nnls(V, O.gram(V), B.u_ptr, B.u_col, B.u_val, reg=0.5, alpha=40.0)
    return U, V


@pytest.mark.parametrize("world", [2, 3])
def test_sharded_layout_cpu(tmp_path, world):
    """Shard planner + padded all-gather layout reproduce the single-process half-sweep (world 3:
    uneven shards, padded rows in the gathered layout)."""
    res = _launch("cpu", str(tmp_path / "cpu.npz"), world=world)
    B, U0, _ = _problem()
    V = O.half_sweep(U0, B.i_ptr, B.i_col, B.i_val, reg=0.5, alpha=40.0)
    assert np.allclose(res["V"], V, rtol=1e-5, atol=1e-6)


@pytest.mark.gpu
@pytest.mark.parametrize("world,nonneg,split,k", [(2, False, 0, 16), (3, False, 0, 16), (3, True, 0, 16),
                                                  (2, False, 128, 16), (3, False, 128, 16), (3, True, 128, 16),
                                                  (2, False, 128, 128), (3, False, 128, 128), (3, True, 128, 256)])
def test_sharded_fit_gpu_matches_single(gpu_lib, tmp_path, world, nonneg, split, k):
    """Ranks sharing the box's GPU run the engine's sharded fit (device remap into the chunk-major
    gathered layout, the solve in row chunks whose factors are gathered on a second stream, host
    transport for the Gram all-reduce and the all-gathers); factors match the single-process oracle.
    nonneg: the NNLS half-sweeps (lockstep + per-row kernels) with the blocking chunk gathers.
    split: ALBEDO_SPLIT_CHUNK=128 sends every row above 128 ratings (the popular repos) through the
    split-K partial + reduce path inside the solve chunks of each rank.  k = 128 runs the c4 bench's
    kernels sharded: the bf16 rotation of the whole gathered src with the fused pre-split into a
    buffer of prows() + 1 rows, light16 (pairs and singles), light D = 32 / 64, the wave kernel and
    split-K partials; k = 256 the NNLS kernels at the c5 rank.  Then recommendForAllUsers(10) with the
    users sharded across the ranks: every rank returns every list, bit-exact against the oracle scorer
    on the fitted factors."""
    env = {"ALBEDO_SPLIT_CHUNK": str(split)} if split else None
    out = str(tmp_path / "gpu.npz")
    res = _launch("gpunn" if nonneg else "gpu", out, world=world, env_extra=env, k=k)
    B, U0, V0 = _problem(k)
    if split:
        assert np.max(np.diff(B.i_ptr)) > 2 * split  # rows that really take the split-K path
    if k == 128:  # every light bucket and the wave kernel have rows
        deg = np.r_[np.diff(B.i_ptr), np.diff(B.u_ptr)]
        assert all(np.any((deg > lo) & (deg <= hi)) for lo, hi in ((0, 8), (8, 16), (16, 32), (32, 64), (64, 128)))
    U, V = _fit_ref(B, U0, V0, k, 3, nonneg)
    rel = lambda a, b: np.max(np.abs(a - b)) / np.max(np.abs(b))
    assert rel(res["U"], U) < 1e-3 and rel(res["V"], V) < 1e-3
    ref_ids, ref_sc = O.recommend_for_all(B.user_ids, res["U"], B.item_ids, res["V"], 10)
    assert np.array_equal(res["topk_ids"], ref_ids)
    assert np.array_equal(res["topk_sc"].view(np.uint32), ref_sc.view(np.uint32))
    for r in range(1, world):
        assert np.array_equal(np.load(out + f".rank{r}.npy"), ref_ids)


@pytest.mark.gpu
def test_sharded_sweep_gpu_c4_shaped(gpu_lib, tmp_path):
    """A c4-shaped problem (60K users x 12K repos, 2M stars, rank 128) on 2 ranks sharing the GPU: each
    rank's shard crosses all 4 solve chunks with light (light16 on the user side, D = 32 / 64) and
    wave-kernel rows in every chunk, and split-K repos (> 8192 stars) at the default chunk, so the chunked solve and its gathers
    run with a realistic degree mix.  One sweep (item half from U0, user half from the engine's items)
    against the C fp64 restatement of Spark's normal-equation solve, row by row."""
    import ctypes as C
    from albedo_amd import _lib as L
    from albedo_amd.synthetic import SynthSpec, generate
    from oracle import cbind
    k, world = 128, 2
    d = generate(SynthSpec(60000, 12000, 2_000_000, zipf_s=0.8, seed=43))
    B = O.make_blocks(d["user"], d["item"], d["rating"])
    # the engine's own shard plan: every (rank, chunk) of both sides holds light and heavy rows
    for ptr in (B.i_ptr, B.u_ptr):
        n = len(ptr) - 1
        starts = np.empty(world + 1, np.int64)
        L.check(gpu_lib.als_host_plan_shards(L.ptr(np.ascontiguousarray(ptr), C.c_int64), n, world,
                                             L.ptr(starts, C.c_int64)))
        deg = np.diff(ptr)
        chpad = -(-int(np.max(np.diff(starts))) // 4)
        for r in range(world):
            for q in range(4):
                lo = starts[r] + q * chpad
                dq = deg[lo:min(starts[r + 1], lo + chpad)]
                assert np.any(dq <= 64) and np.any(dq > 64), (r, q)
    assert np.max(np.diff(B.i_ptr)) > 8192  # split-K rows
    rng = np.random.default_rng(3)
    U0 = rng.standard_normal((len(B.user_ids), k)).astype(np.float32)
    res = _launch("gpubig", str(tmp_path / "big.npz"), world=world, k=k, timeout=600)
    V_ref = cbind.half_sweep(U0, B.i_ptr, B.i_col, B.i_val, reg=0.5, alpha=40.0)
    U_ref = cbind.half_sweep(res["V"], B.u_ptr, B.u_col, B.u_val, reg=0.5, alpha=40.0)
    for got, ref in ((res["V"], V_ref), (res["U"], U_ref)):
        err = np.linalg.norm(got - ref, axis=1) / np.maximum(np.linalg.norm(ref, axis=1), 1e-30)
        assert np.max(err) < 1e-4, np.max(err)
