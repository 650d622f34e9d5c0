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


def _launch(mode, out, world=2, timeout=300, env_extra=None):
    port = _free_port()
    procs = []
    for r in range(world):
        env = dict(os.environ, RANK=str(r), WORLD_SIZE=str(world), LOCAL_RANK="0", MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port), **(env_extra or {}))
        procs.append(subprocess.Popen([sys.executable, os.path.join(ROOT, "tests", "mp_worker.py"), mode, out],
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


def _problem():
    from albedo_amd.synthetic import SynthSpec, generate
    d = generate(SynthSpec(1200, 400, 16000, seed=41))
    B = O.make_blocks(d["user"], d["item"], d["rating"])
    rng = np.random.default_rng(3)
    U0 = rng.standard_normal((len(B.user_ids), 16)).astype(np.float32)
    V0 = rng.standard_normal((len(B.item_ids), 16)).astype(np.float32)
    return B, U0, V0


@pytest.mark.parametrize("world", [2, 3])
def test_sharded_layout_cpu(tmp_path, world):
    """Shard planner + padded all-gather layout reproduce the single-process half-sweep (world 3:
    uneven shards, padded rows in the gathered layout)."""
    res = _launch("cpu", str(tmp_path / "cpu.npz"), world=world)
    B, U0, _ = _problem()
    V = O.half_sweep(U0, B.i_ptr, B.i_col, B.i_val, reg=0.5, alpha=40.0)
    assert np.allclose(res["V"], V, rtol=1e-5, atol=1e-6)


@pytest.mark.gpu
@pytest.mark.parametrize("world,nonneg,split", [(2, False, 0), (3, False, 0), (3, True, 0), (2, False, 128),
                                                (3, False, 128), (3, True, 128)])
def test_sharded_fit_gpu_matches_single(gpu_lib, tmp_path, world, nonneg, split):
    """Ranks sharing the box's GPU run the engine's sharded fit (device remap into the chunk-major
    gathered layout, the solve in row chunks whose factors are gathered on a second stream, host
    transport for the Gram all-reduce and the all-gathers); factors match the single-process oracle.
    nonneg: the NNLS half-sweeps (lockstep + per-row kernels) with the blocking chunk gathers.
    split: ALBEDO_SPLIT_CHUNK=128 sends every row above 128 ratings (the popular repos) through the
    split-K partial + reduce path inside the solve chunks of each rank.  Then recommendForAllUsers(10)
    with the users sharded across the ranks: every rank returns every list, bit-exact against the
    oracle scorer on the fitted factors."""
    env = {"ALBEDO_SPLIT_CHUNK": str(split)} if split else None
    out = str(tmp_path / "gpu.npz")
    res = _launch("gpunn" if nonneg else "gpu", out, world=world, env_extra=env)
    B, U0, V0 = _problem()
    if split:
        assert np.max(np.diff(B.i_ptr)) > 2 * split  # rows that really take the split-K path
    U, V = O.fit(B, rank=16, max_iter=3, reg=0.5, alpha=40.0, init_user=U0, init_item=V0, nonnegative=nonneg)
    rel = lambda a, b: np.max(np.abs(a - b)) / np.max(np.abs(b))
    assert rel(res["U"], U) < 1e-3 and rel(res["V"], V) < 1e-3
    ref_ids, ref_sc = O.recommend_for_all(B.user_ids, res["U"], B.item_ids, res["V"], 10)
    assert np.array_equal(res["topk_ids"], ref_ids)
    assert np.array_equal(res["topk_sc"].view(np.uint32), ref_sc.view(np.uint32))
    for r in range(1, world):
        assert np.array_equal(np.load(out + f".rank{r}.npy"), ref_ids)
