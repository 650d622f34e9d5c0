"""Benchmark: implicit-ALS interactions/sec per sweep (BASELINE.json metric) on MI355X.

  python bench.py [--gpus N] [--steps K] [--warmup W] [--config c4|c2]
  (N > 1: python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N)

A step = one full ALS sweep (item half-sweep + user half-sweep: Gram, eigendecomposition,
rotation, RCCL all-reduce/all-gather, light + heavy per-row solves) over the whole synthetic star
matrix, inputs resident in HBM.  Default workload = BASELINE config 4 (20M users x 4M repos,
1B stars, rank 128: the config the metric is quoted on; it fits one 288 GB MI355X) row-sharded
across ranks (strong scaling: the total work is fixed).  Rank 0 prints ONE JSON line.

roofline: the dominant per-row solve kernel's algorithmic bytes per launch (SURVEY.md §8(d):
  nnz·(4 col + 4 val) + (rows+1)·8 + nnz·4k gathered rows + rows·4k written) / its average
  HIP-event duration on the engine's stream, against 8 TB/s HBM.
cpu_baseline: the fp64 C/OpenMP restatement of Spark's half-sweep (oracle/c, "port") timed on a
  degree-stratified row sample of the same workload on every core this process may use (affinity /
  cgroup quota; nproc and the CPU model are reported), each stratum extrapolated to one sweep.
"""
from __future__ import annotations

import argparse
import ctypes as C
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

CONFIG_RANK = {"c2": 64, "c4": 128, "c1p": 50, "c5": 256}
NONNEGATIVE = {"c5"}  # BASELINE config 5: rank 256, nonnegative=true (NNLS), extreme repo skew
METRIC = "implicit-ALS interactions/sec per sweep at rank 128 (1/8 GPU); top-30 recs users/sec"
MFMA_F16_TFLOPS = 2500.0  # dense fp16 MFMA peak, MI355X (MI355X_MICROARCH.md: ~2.5 PF dense)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--config", default="c4", choices=sorted(CONFIG_RANK))
    ap.add_argument("--topk-users", type=int, default=-1,
                    help="users scored by the top-30 run (recommendForAllUsers); -1 = every user, 0 = skip")
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--light", type=int, default=-1)
    return ap.parse_args()


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if world > 1:
        import torch  # noqa: F401  (import before the engine: one HIP runtime per process)
        import torch.distributed as dist
        dist.init_process_group("gloo", init_method="env://")
    from albedo_amd import _lib as L
    from albedo_amd.synthetic import CONFIGS, popularity_table, user_degrees

    lib = L.load()
    spec = CONFIGS[args.config]
    k = CONFIG_RANK[args.config]
    p = L.als_params()
    L.check(lib.als_params_default(C.byref(p)))
    p.rank, p.implicit_prefs, p.reg_param, p.alpha, p.seed = k, 1, 0.5, 40.0, 42
    p.nonnegative = 1 if args.config in NONNEGATIVE else 0
    p.device = local
    p.light_max_degree = args.light
    h = C.c_void_p()
    L.check(lib.als_create(C.byref(p), C.byref(h)))
    if world > 1:
        uid = (C.c_char * 128)()
        if rank == 0:
            L.check(lib.als_comm_unique_id(uid))
        obj = [bytes(uid)]
        dist.broadcast_object_list(obj, src=0)
        uid = (C.c_char * 128).from_buffer_copy(obj[0])
        L.check(lib.als_comm_init(h, rank, world, uid))

    t0 = time.perf_counter()
    deg = user_degrees(spec)
    prefix = np.ascontiguousarray(np.r_[0, np.cumsum(deg)].astype(np.int64))
    cw, perm = popularity_table(spec)
    L.check(lib.als_set_ratings_synthetic(h, spec.seed, spec.rounds, spec.n_users, spec.n_items,
                                          L.ptr(prefix, C.c_int64), L.ptr(np.ascontiguousarray(cw), C.c_double),
                                          L.ptr(np.ascontiguousarray(perm), C.c_int32)))
    L.check(lib.als_init_factors_random(h, 42))
    setup_s = time.perf_counter() - t0
    nnz = lib.als_num_ratings(h)
    n_users, n_items = lib.als_num_rows(h, 0), lib.als_num_rows(h, 1)
    top_deg = {}
    for side, name in ((0, "users"), (1, "repos")):
        dg = np.empty(lib.als_num_rows(h, side), np.int64)
        L.check(lib.als_get_degrees(h, side, L.ptr(dg, C.c_int64)))
        top_deg[name] = np.sort(dg[dg >= 0])[::-1][:5].tolist()

    def barrier():
        L.check(lib.als_synchronize(h))
        if dist is not None:
            dist.barrier()

    for _ in range(args.warmup):
        L.check(lib.als_run_sweeps(h, 1))
    # per-stage device times accumulated over the timed sweeps
    stage = {side: np.zeros(L.ALS_T_COUNT) for side in (0, 1)}
    stats = {side: np.zeros(4, np.int64) for side in (0, 1)}
    barrier()
    t_start = time.perf_counter()
    for _ in range(args.steps):
        L.check(lib.als_half_sweep(h, 1))
        tt = np.zeros(L.ALS_T_COUNT)
        L.check(lib.als_last_timings(h, 1, L.ptr(tt, C.c_double), L.ALS_T_COUNT))
        stage[1] += tt
        L.check(lib.als_half_sweep(h, 0))
        L.check(lib.als_last_timings(h, 0, L.ptr(tt, C.c_double), L.ALS_T_COUNT))
        stage[0] += tt
    barrier()
    elapsed = time.perf_counter() - t_start
    nnls_iters, eig_sweeps = {}, {}
    for side in (0, 1):
        L.check(lib.als_path_stats(h, side, L.ptr(stats[side], C.c_int64)))
        if args.config not in NONNEGATIVE:
            sv = np.zeros(4, np.int64)
            L.check(lib.als_solver_stats(h, side, L.ptr(sv, C.c_int64)))
            eig_sweeps["user" if side == 0 else "item"] = int(sv[0])
        if args.config in NONNEGATIVE:
            sv = np.zeros(4, np.int64)
            L.check(lib.als_solver_stats(h, side, L.ptr(sv, C.c_int64)))
            nb = int(stats[side][0])
            nnls_iters["user" if side == 0 else "item"] = {
                "mean": float(sv[0]) / max(int(sv[2]), 1), "max": int(sv[1]), "rows": int(sv[2]),
                "lockstep_rows": nb, "lockstep_mean": float(sv[3]) / max(nb, 1),
                "per_row_kernel_mean": float(sv[0] - sv[3]) / max(int(sv[2]) - nb, 1)}
    if dist is not None:
        import torch
        t = torch.tensor([elapsed], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    ms_per_step = 1000.0 * elapsed / args.steps
    value = nnz * args.steps / elapsed

    # ---- roofline of the dominant solve kernel (per launch, this rank's shard) -------------------
    def solve_bytes(side, which):  # which: 0 light, 1 heavy
        rows, nz = stats[side][2 * which], stats[side][2 * which + 1]
        return nz * 8 + (rows + 1) * 8 + nz * 4 * k + rows * 4 * k, rows, nz

    kern = {}
    for which, (name, ti, launches) in enumerate((("solve_light", L.T_NAMES.index("solve_light"), 3),
                                                  ("solve_heavy", L.T_NAMES.index("solve_heavy"), 1))):
        tot_ms = stage[0][ti] + stage[1][ti]
        b = solve_bytes(0, which)[0] + solve_bytes(1, which)[0]
        kern[name] = dict(ms=tot_ms / args.steps, bytes_per_sweep=b)
    if args.config in NONNEGATIVE:  # light timer: the lockstep NNLS kernel; heavy: the per-row one
        kern["nnls_batch"] = kern.pop("solve_light")
        kern["solve_nnls"] = kern.pop("solve_heavy")
    elif world > 1:  # chunked solve (factor gathers behind it): one timer covers every solve kernel
        li, he = kern.pop("solve_light"), kern.pop("solve_heavy")
        kern["solve_heavy"] = dict(ms=li["ms"] + he["ms"], bytes_per_sweep=li["bytes_per_sweep"] + he["bytes_per_sweep"])
    dom = max(kern, key=lambda n: kern[n]["ms"])
    d = kern[dom]
    achieved = d["bytes_per_sweep"] / (d["ms"] / 1000.0) / 1e9 if d["ms"] > 0 else 0.0
    peak = 8000.0
    # HBM bytes of the same kernel from the committed PMC passes of this config (tools/prof.sh ->
    # tools/traffic.py; rocprof cannot run inside the timed bench): GB per sweep, like bytes_per_sweep
    # The heavy timer covers every kernel of the explicit path: split-K partials + reduce, the wave
    # kernel, the workgroup kernel (and, with nonnegative, the NNLS kernels)
    timer_kernels = {"solve_light": ("solve_light", "solve_light16"),
                     "solve_heavy": ("solve_wave", "solve_heavy", "wave_partial", "heavy_partial", "heavy_reduce"),
                     "nnls_batch": ("nnls_batch",),
                     "solve_nnls": ("solve_nnls", "solve_nnls_row", "heavy_partial", "heavy_reduce")}[dom]
    traffic = None
    tpath = os.path.join(ROOT, "profiles", f"pmc_traffic_{args.config}.json")
    if os.path.exists(tpath) and world == 1:
        tj = json.load(open(tpath))
        found = [tj[n]["hbm_gb_per_sweep"] for n in timer_kernels if n in tj]
        if found:
            traffic = float(sum(found))

    # NNLS configs: the solve is iteration-latency bound (Spark's projected-gradient loop, hundreds of
    # dependent iterations per row), so the roofline that means something is per row-iteration: the
    # CU cycles one row-iteration takes (solve time x CUs x clock / row-iterations, the iteration
    # counts of the last sweep) against the k^2 FMAs of its one product A.v at the CU's packed-fp32
    # rate (512 FMA per cycle: 4 SIMDs x 64 lanes x v_pk_fma_f32)
    latency_roofline = None
    if args.config in NONNEGATIVE and nnls_iters:
        n_cu, ghz = 256, 2.4
        floor = k * k / 512.0
        per = {}
        lock_it = sum(nnls_iters[sd]["lockstep_mean"] * nnls_iters[sd]["lockstep_rows"] for sd in nnls_iters)
        row_it = sum(nnls_iters[sd]["per_row_kernel_mean"] * (nnls_iters[sd]["rows"] - nnls_iters[sd]["lockstep_rows"])
                     for sd in nnls_iters)
        for name, ms, its in (("nnls_batch (lockstep)", kern["nnls_batch"]["ms"], lock_it),
                              ("solve_nnls (per row)", kern["solve_nnls"]["ms"], row_it)):
            if its > 0 and ms > 0:
                cyc = ms / 1000.0 * n_cu * ghz * 1e9 / its
                per[name] = {"cycles_per_row_iteration": cyc, "floor_cycles": floor, "frac": floor / cyc,
                             "row_iterations": its, "ms_per_sweep": ms}
        latency_roofline = {"bound": "latency (dependent iterations)", "unit": "CU cycles per row-iteration",
                            "clock_ghz_assumed": ghz, "kernels": per}

    # Gram / rotation matrix-core evidence: MFMA busy of the shipped kernels from the committed SQ
    # counter passes of this config (tools/prof.sh -> tools/sqsum.py; PMC cannot run inside the bench)
    mfma_evidence = None
    def latest(stem):  # the newest round's committed profile of this config
        for tag in ("r06", "r05", "r04"):
            path = os.path.join(ROOT, "profiles", f"{tag}_{args.config}_{stem}.json")
            if os.path.exists(path):
                return path
        return None
    spath = latest("sq_counters")
    if spath:
        sj = json.load(open(spath))
        mfma_evidence = {"source": os.path.relpath(spath, ROOT)}
        # the top-k scan's counters from the all-users profile when there is one (the sweep profile
        # scores a 16K-user sample)
        tkp = latest("topk_sq_counters")
        if tkp:
            sj = {k: v for k, v in sj.items() if not k.startswith("topk_scan_kernel")}
            sj.update({k: v for k, v in json.load(open(tkp)).items() if k.startswith("topk_scan_kernel")})
            mfma_evidence["source_topk"] = os.path.relpath(tkp, ROOT)
        for key, v in sj.items():
            name = key.split("<")[0]
            if name in ("gram_bf_kernel", "gram_partial_kernel", "rotate_bf_kernel", "rotate_kernel",
                        "solve_wave_kernel", "topk_scan_kernel") and isinstance(v, dict) and "mfma_busy" in v:
                mfma_evidence[key] = {"mfma_busy": v["mfma_busy"], "lds_conflict": v.get("lds_conflict")}

    # ---- top-30 users/s (secondary metric; a bounded user subset) ------------------------------
    # world > 1: every rank calls als_recommend (the users are sharded across the ranks, each scores
    # its slice against the replicated dst factors, the lists are all-gathered); timed between
    # barriers, max over ranks
    topk_ups = topk_info = None
    if args.topk_users != 0:
        ids = np.empty(n_users, np.int32)
        L.check(lib.als_get_ids(h, 0, L.ptr(ids, C.c_int32)))
        every = args.topk_users < 0 or args.topk_users >= n_users
        sub = ids if every else np.ascontiguousarray(
            ids[np.linspace(0, n_users - 1, args.topk_users).astype(np.int64)])
        out_i = np.empty((sub.size, 30), np.int32)
        out_s = np.empty((sub.size, 30), np.float32)
        out_i[:] = 0  # touch the pages before the timed call
        out_s[:] = 0
        L.check(lib.als_recommend(h, 0, 30, L.ptr(sub[:1024], C.c_int32), min(1024, sub.size), None,
                                  L.ptr(out_i, C.c_int32), L.ptr(out_s, C.c_float)))  # warm
        st0 = np.zeros(4, np.int64)
        L.check(lib.als_topk_stats(h, L.ptr(st0, C.c_int64)))
        tm0 = np.zeros(5, np.float64)
        L.check(lib.als_topk_timing(h, L.ptr(tm0, C.c_double)))
        barrier()
        t1 = time.perf_counter()
        # every user: recommendForAllUsers (subset = NULL); else ALSModel.recommendForUserSubset
        L.check(lib.als_recommend(h, 0, 30, None if every else L.ptr(sub, C.c_int32), sub.size, None,
                                  L.ptr(out_i, C.c_int32), L.ptr(out_s, C.c_float)))
        barrier()
        topk_s = time.perf_counter() - t1
        if dist is not None:
            import torch
            t = torch.tensor([topk_s], dtype=torch.float64)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            topk_s = float(t.item())
        topk_ups = sub.size / topk_s
        st1 = np.zeros(4, np.int64)
        L.check(lib.als_topk_stats(h, L.ptr(st1, C.c_int64)))
        dst = st1 - st0
        tm1 = np.zeros(5, np.float64)
        L.check(lib.als_topk_timing(h, L.ptr(tm1, C.c_double)))
        tm = tm1 - tm0
        scan_tflops = tm[4] / max(tm[1], 1e-9) / 1e9  # flops / ms -> TFLOP/s
        topk_info = {"users": int(sub.size), "all_users": bool(every), "seconds": topk_s,
                     "sweeps_before_topk": args.warmup + args.steps, "exact_rescan_rows": int(dst[1]),
                     "dst_chunks_scanned_frac": float(dst[2]) / max(1, int(dst[3])),
                     "device_ms": {"order_mask": tm[0], "scan": tm[1], "select": tm[2], "exact": tm[3]},
                     # the dominant kernel (the fp16 MFMA scan): scanned flops / its time vs the dense
                     # fp16 MFMA peak (this rank's share; HIP events on the engine stream)
                     "roofline": {"bound": "mfma", "achieved": scan_tflops, "peak": MFMA_F16_TFLOPS,
                                  "unit": "TFLOP/s", "frac": scan_tflops / MFMA_F16_TFLOPS,
                                  "scan_tflop": tm[4] / 1e12, "kernel": "topk_scan"},
                     "note": "wall time of als_recommend(k=30) on the user subset: dst norm sort + fp16 pack, "
                             "MFMA scan with norm-order early exit, exact F2J rescoring, D2H of the lists"}

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu:
        if args.config in NONNEGATIVE:
            cpu = cpu_baseline_nnls(lib, L, h, k, nnz, n_users, n_items, args.cpu_seconds)
        else:
            cpu = cpu_baseline(lib, L, h, k, nnz, n_users, n_items, args.cpu_seconds)

    if rank == 0:
        line = {
            "metric": METRIC, "value": value, "unit": "interactions/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": ms_per_step,
            "higher_is_better": True, "scaling": "strong", "vs_baseline": None,
            "dtype": "fp32 (split-fp16x3 MFMA build, fp32 accumulate; fp64 Gram/eigenbasis"
                     + ("; fp64 NNLS vectors)" if args.config in NONNEGATIVE else ")"),
            "data": "synthetic (seeded power-law star matrix, rating=1.0; SURVEY.md §8(d))",
            "config": {"workload": f"BASELINE {args.config}: {n_users} users x {n_items} repos, {nnz} stars, "
                                   f"rank {k}, implicit alpha 40 regParam 0.5, one sweep = item + user half",
                       "rank": k, "nnz": int(nnz), "parallelism": f"row-shard x{world} (RCCL)",
                       "nonnegative": args.config in NONNEGATIVE, "top5_degrees": top_deg},
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": peak, "unit": "GB/s",
                         "frac": achieved / peak, "traffic": traffic, "kernel": dom,
                         "traffic_kernels": list(timer_kernels),
                         "traffic_unit": "GB per sweep (PMC, profiles/pmc_traffic_<config>.json)",
                         "algorithmic_gb_per_sweep": d["bytes_per_sweep"] / 1e9,
                         "kernel_ms_per_sweep": d["ms"]},
            "cpu_baseline": cpu,
            "mfma_busy_profiled": mfma_evidence,
            "latency_roofline": latency_roofline,
            "topk30_users_per_s": topk_ups,
            "topk30": topk_info,
            "stages_ms_per_sweep": {f"{'user' if s == 0 else 'item'}_{n}": round((stage[s][i] / args.steps), 3)
                                    for s in (0, 1) for i, n in enumerate(L.T_NAMES[:7])},
            "paths": {"user": stats[0].tolist(), "item": stats[1].tolist()},
            "nnls_iterations_last_sweep": nnls_iters or None,
            "eig_jacobi_sweeps_last_sweep": eig_sweeps or None,
            "setup_s": setup_s,
        }
        print(json.dumps(line), flush=True)
    lib.als_destroy(h)
    if dist is not None:
        dist.destroy_process_group()


def host_cpu_info():
    """Cores this process may use (affinity, cgroup quota), the machine's nproc and CPU model."""
    nproc = os.cpu_count() or 1
    try:
        aff = len(os.sched_getaffinity(0))
    except AttributeError:
        aff = nproc
    quota = None
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            quota = max(1, int(int(q) / int(per)))
    except (OSError, ValueError):
        pass
    model = "unknown"
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    usable = min(aff, quota) if quota else aff
    return dict(nproc=nproc, affinity=aff, cgroup_quota=quota, model=model, usable=usable)


# degree strata of the CPU sample (per-star cost differs between a 2-star and a 10^5-star row)
STRATA = (1, 17, 33, 65, 257, 1025, 4097, 16385, 65537)


def cpu_baseline(lib, L, h, k, nnz, n_users, n_items, budget_s):
    """fp64 C/OpenMP restatement (oracle/c) timed on a degree-stratified sample of this workload's
    rows, on every core this process may use; each stratum is extrapolated by its own star count."""
    from oracle import cbind
    info = host_cpu_info()
    threads = info["usable"]
    res = {}
    t_sweep = 0.0
    for dst, n_dst, n_src in ((0, n_users, n_items), (1, n_items, n_users)):
        src = 1 - dst
        sids = np.empty(n_src, np.int32)
        sf = np.empty((n_src, k), np.float32)
        L.check(lib.als_get_factors(h, src, L.ptr(sids, C.c_int32), L.ptr(sf, C.c_float)))
        t0 = time.perf_counter()
        G = cbind.gram(sf, threads=threads)
        g_s = time.perf_counter() - t0
        dids = np.empty(n_dst, np.int32)
        L.check(lib.als_get_ids(h, dst, L.ptr(dids, C.c_int32)))
        deg = np.empty(n_dst, np.int64)
        L.check(lib.als_get_degrees(h, dst, L.ptr(deg, C.c_int64)))
        rng = np.random.default_rng(7 + dst)
        edges = list(STRATA) + [int(deg.max()) + 1]
        n_b = sum(1 for a, b in zip(edges[:-1], edges[1:]) if np.any((deg >= a) & (deg < b)))
        per_star = None  # seconds per star of the last measured stratum (for strata past the cap)
        strata = []
        t_side = g_s
        n_row = np.empty(1, np.int64)
        for a, b in zip(edges[:-1], edges[1:]):
            rows = np.nonzero((deg >= a) & (deg < b))[0]
            if rows.size == 0:
                continue
            stars = int(deg[rows].sum())
            if a >= STRATA[-1] and per_star is not None:
                # single rows of 10^5+ stars would run on one core for minutes: the build is one dspr
                # per star in every stratum, so the per-star cost of the 16K-65K stratum is used
                strata.append(dict(lo=a, rows=int(rows.size), stars=stars, sampled_rows=0, sampled_stars=0,
                                   s=per_star * stars, extrapolated_from_lower=True))
                t_side += per_star * stars
                continue
            order = rng.permutation(rows)
            done, t_rows, total = 0, 0.0, 0
            chunk = max(2 * threads, 64)
            while done < order.size and (t_rows < budget_s / (2 * n_b) or done == 0):
                sel = order[done:done + chunk]
                done += sel.size
                ptr, cols, vals = [0], [], []
                for r in sel:
                    m = int(deg[r])
                    bi, bv = np.empty(max(m, 1), np.int32), np.empty(max(m, 1), np.float32)
                    L.check(lib.als_get_row_ratings(h, dst, int(dids[r]), m, L.ptr(bi, C.c_int32),
                                                    L.ptr(bv, C.c_float), L.ptr(n_row, C.c_int64)))
                    cols.append(np.searchsorted(sids, bi[:m]).astype(np.int32))
                    vals.append(bv[:m])
                    ptr.append(ptr[-1] + m)
                ptr_a = np.asarray(ptr, np.int64)
                t1 = time.perf_counter()
                cbind.solve_rows(sf, G, ptr_a, np.concatenate(cols), np.concatenate(vals), reg=0.5, alpha=40.0,
                                 implicit=True, threads=threads)
                t_rows += time.perf_counter() - t1
                total += int(ptr_a[-1])
                chunk = min(chunk * 2, 8192)
            per_star = t_rows / max(total, 1)
            est = t_rows * stars / max(total, 1)
            strata.append(dict(lo=a, rows=int(rows.size), stars=stars, sampled_rows=int(done), sampled_stars=total,
                               s=est))
            t_side += est
        res[dst] = dict(gram_s=g_s, strata=strata, side_s=t_side)
        t_sweep += t_side
        del sf
    sampled = sum(st["sampled_stars"] for d in res for st in res[d]["strata"])
    return {"value": nnz / t_sweep, "unit": "interactions/s", "cores": threads, "kind": "port",
            "host": {k2: info[k2] for k2 in ("nproc", "affinity", "cgroup_quota", "model")},
            "sweep_s_extrapolated": t_sweep,
            "strata": {("user" if d == 0 else "item"): res[d]["strata"] for d in res},
            "sample": (f"fp64 C/OpenMP restatement of Spark's half-sweep (oracle/c/als_cpu.c, {threads} threads): "
                       f"full Gram of each src side + a degree-stratified row sample ({sampled} stars, strata "
                       f"{list(STRATA)}) solved, each stratum extrapolated by its own star count to one sweep")}


def cpu_baseline_nnls(lib, L, h, k, nnz, n_users, n_items, budget_s):
    """NNLS configs: the fp64 C/OpenMP restatement of Spark's NNLSSolver (oracle/c/als_cpu.c
    oracle_solve_rows_nnls: the normal equation as Spark builds it, fillAtA, NNLS.scala's projected
    gradient with CG acceleration; equal to oracle/spark_als.py:nnls on the F5 rows, tests/test_oracle.py)
    on every core this process may use, over a degree-stratified row sample.  A row's cost is its
    iteration count times a k x k product, not its star count, so each stratum is extrapolated by its
    row count.  The Gram of each src side by the C/OpenMP restatement."""
    from oracle import cbind
    info = host_cpu_info()
    threads = info["usable"]
    res, t_sweep = {}, 0.0
    for dst, n_dst, n_src in ((0, n_users, n_items), (1, n_items, n_users)):
        src = 1 - dst
        sids = np.empty(n_src, np.int32)
        sf = np.empty((n_src, k), np.float32)
        L.check(lib.als_get_factors(h, src, L.ptr(sids, C.c_int32), L.ptr(sf, C.c_float)))
        t0 = time.perf_counter()
        G = cbind.gram(sf, threads=threads)
        g_s = time.perf_counter() - t0
        dids = np.empty(n_dst, np.int32)
        L.check(lib.als_get_ids(h, dst, L.ptr(dids, C.c_int32)))
        deg = np.empty(n_dst, np.int64)
        L.check(lib.als_get_degrees(h, dst, L.ptr(deg, C.c_int64)))
        rng = np.random.default_rng(11 + dst)
        edges = list(STRATA) + [int(deg.max()) + 1]
        n_b = sum(1 for a, b in zip(edges[:-1], edges[1:]) if np.any((deg >= a) & (deg < b)))
        strata, t_side = [], g_s
        n_row = np.empty(1, np.int64)
        for a, b in zip(edges[:-1], edges[1:]):
            rows = np.nonzero((deg >= a) & (deg < b))[0]
            if rows.size == 0:
                continue
            order = rng.permutation(rows)
            done, t_rows, iters = 0, 0.0, 0
            chunk = max(threads, 16)
            while done < order.size and (t_rows < budget_s / (2 * n_b) or done == 0):
                sel = order[done:done + chunk]
                done += sel.size
                ptr, cols, vals = [0], [], []
                for r in sel:
                    m = int(deg[r])
                    bi, bv = np.empty(max(m, 1), np.int32), np.empty(max(m, 1), np.float32)
                    L.check(lib.als_get_row_ratings(h, dst, int(dids[r]), m, L.ptr(bi, C.c_int32),
                                                    L.ptr(bv, C.c_float), L.ptr(n_row, C.c_int64)))
                    cols.append(np.searchsorted(sids, bi[:m]).astype(np.int32))
                    vals.append(bv[:m])
                    ptr.append(ptr[-1] + m)
                t1 = time.perf_counter()
                _, it = cbind.solve_rows_nnls(sf, G, np.asarray(ptr, np.int64), np.concatenate(cols),
                                              np.concatenate(vals), reg=0.5, alpha=40.0, threads=threads)
                t_rows += time.perf_counter() - t1
                iters += int(it.sum())
                chunk = min(chunk * 2, 4096)
            est = t_rows * rows.size / done
            strata.append(dict(lo=a, rows=int(rows.size), sampled_rows=int(done), mean_iters=iters / done, s=est))
            t_side += est
        res[dst] = dict(gram_s=g_s, strata=strata, side_s=t_side)
        t_sweep += t_side
        del sf
    sampled = sum(st["sampled_rows"] for d in res for st in res[d]["strata"])
    return {"value": nnz / t_sweep, "unit": "interactions/s", "cores": threads, "kind": "port",
            "host": {k2: info[k2] for k2 in ("nproc", "affinity", "cgroup_quota", "model")},
            "sweep_s_extrapolated": t_sweep,
            "strata": {("user" if d == 0 else "item"): res[d]["strata"] for d in res},
            "sample": (f"fp64 C/OpenMP restatement of Spark's NNLSSolver (oracle/c/als_cpu.c oracle_solve_rows_nnls, "
                       f"{threads} threads) on {sampled} degree-stratified rows (strata {list(STRATA)}), each stratum "
                       f"extrapolated by its row count; the Gram by the C/OpenMP restatement")}


if __name__ == "__main__":
    main()
