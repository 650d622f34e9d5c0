"""Worker for the multi-rank tests: one process = one rank; ranks exchange through gloo.

GPU mode: every rank owns an engine context on device 0 (one GPU box) and the engine's host
transport (als_comm_init_host) carries the Gram all-reduce and the factor-shard all-gather over
gloo — the same sharded half-sweep code the RCCL transport runs on a multi-GPU node.
CPU mode: the engine's shard planner + padded gather layout, with the C oracle solving each
rank's rows (no GPU).
"""
import ctypes as C
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    import torch.distributed as dist
    mode, out = sys.argv[1], sys.argv[2]
    k = int(sys.argv[3]) if len(sys.argv) > 3 else 16
    dist.init_process_group("gloo", init_method="env://")
    rank, world = dist.get_rank(), dist.get_world_size()
    from albedo_amd import _lib as L
    from albedo_amd.synthetic import SynthSpec, generate
    from oracle import spark_als as O
    lib = L.load()
    big = mode == "gpubig"
    # gpubig: a c4-shaped problem large enough that every rank's shard has light and heavy rows in each
    # of its 4 solve chunks (and split-K rows at the default 8192-rating chunk); one sweep
    d = generate(SynthSpec(60000, 12000, 2_000_000, zipf_s=0.8, seed=43) if big else SynthSpec(1200, 400, 16000, seed=41))
    B = O.make_blocks(d["user"], d["item"], d["rating"])
    rng = np.random.default_rng(3)
    U0 = rng.standard_normal((len(B.user_ids), k)).astype(np.float32)
    V0 = rng.standard_normal((len(B.item_ids), k)).astype(np.float32)
    if mode in ("gpu", "gpunn", "gpubig"):
        def allreduce(_u, buf, n):
            t = torch.from_numpy(np.ctypeslib.as_array(buf, shape=(n,)))
            dist.all_reduce(t)
            return 0

        def allgather(_u, buf, n):
            a = np.ctypeslib.as_array(buf, shape=(world * n,))
            parts = [torch.empty(n, dtype=torch.float32) for _ in range(world)]
            dist.all_gather(parts, torch.from_numpy(a[rank * n:(rank + 1) * n].copy()))
            for r in range(world):
                a[r * n:(r + 1) * n] = parts[r].numpy()
            return 0

        ar, ag = L.ALLREDUCE_FN(allreduce), L.ALLGATHER_FN(allgather)
        if os.environ.get("ALBEDO_TEST_POLLUTE"):  # tools/repro_mrbig.py: leave NaN-filled freed memory
            junk = torch.full((int(os.environ["ALBEDO_TEST_POLLUTE"]) << 28,), float("nan"), device="cuda")
            torch.cuda.synchronize()
            del junk
            torch.cuda.empty_cache()
        p = L.als_params()
        L.check(lib.als_params_default(C.byref(p)))
        p.rank, p.implicit_prefs, p.reg_param, p.alpha, p.max_iter = k, 1, 0.5, 40.0, 1 if big else 3
        p.nonnegative = 1 if mode == "gpunn" else 0
        h = C.c_void_p()
        L.check(lib.als_create(C.byref(p), C.byref(h)))
        L.check(lib.als_comm_init_host(h, rank, world, ar, ag, None))
        u, i, r = (np.ascontiguousarray(d[x]) for x in ("user", "item", "rating"))
        L.check(lib.als_set_ratings(h, u.size, L.ptr(u, C.c_int32), L.ptr(i, C.c_int32), L.ptr(r, C.c_float)))
        for side, ids, f in ((0, B.user_ids, U0), (1, B.item_ids, V0)):
            ids = np.ascontiguousarray(ids)
            L.check(lib.als_set_initial_factors(h, side, ids.size, L.ptr(ids, C.c_int32), L.ptr(f, C.c_float)))
        L.check(lib.als_fit(h))
        res = {}
        for side, name in ((0, "U"), (1, "V")):
            n = lib.als_num_rows(h, side)
            f = np.empty((n, k), np.float32)
            L.check(lib.als_get_factors(h, side, None, L.ptr(f, C.c_float)))
            res[name] = f
        if big:
            if rank == 0:
                np.savez(out, **res)
            lib.als_destroy(h)
            dist.barrier()
            dist.destroy_process_group()
            return
        # recommendForAllUsers(10), users sharded across the ranks, lists all-gathered
        n_u = lib.als_num_rows(h, 0)
        ids = np.empty((n_u, 10), np.int32)
        sc = np.empty((n_u, 10), np.float32)
        L.check(lib.als_recommend(h, 0, 10, None, n_u, None, L.ptr(ids, C.c_int32), L.ptr(sc, C.c_float)))
        st = np.zeros(4, np.int64)
        L.check(lib.als_topk_stats(h, L.ptr(st, C.c_int64)))
        assert 0 < st[0] < n_u, f"rank {rank} scored {st[0]} of {n_u} users: not sharded"
        res["topk_ids"], res["topk_sc"] = ids, sc
        if rank != 0:  # every rank holds every list
            np.save(out + f".rank{rank}.npy", ids)
        res["split_rows"] = np.array([lib.als_num_rows(h, 1)])
        lib.als_destroy(h)
    else:
        from oracle import cbind
        res = {}
        U = U0
        for side, (ptr, col, val, n_dst, Ysrc) in (("V", (B.i_ptr, B.i_col, B.i_val, len(B.item_ids), U0)),):
            starts = np.empty(world + 1, np.int64)
            L.check(lib.als_host_plan_shards(L.ptr(np.ascontiguousarray(ptr), C.c_int64), n_dst, world,
                                             L.ptr(starts, C.c_int64)))
            maxrows = int(np.max(np.diff(starts)))
            lo, hi = starts[rank], starts[rank + 1]
            G = cbind.gram(Ysrc)
            p_loc = ptr[lo:hi + 1] - ptr[lo]
            X = cbind.solve_rows(Ysrc, G, p_loc, col[ptr[lo]:ptr[hi]], val[ptr[lo]:ptr[hi]], reg=0.5, alpha=40.0)
            block = np.zeros((maxrows, k), np.float32)
            block[: hi - lo] = X
            parts = [torch.empty(maxrows * k) for _ in range(world)]
            dist.all_gather(parts, torch.from_numpy(block.reshape(-1)))
            full = np.concatenate([parts[r].numpy().reshape(maxrows, k)[: starts[r + 1] - starts[r]]
                                   for r in range(world)])
            res[side] = full
    if rank == 0:
        np.savez(out, **res)
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
