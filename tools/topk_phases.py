"""Probe (not a test): shader-clock phase breakdown of topk_scan_kernel on the bench's top-k state.

  python tools/topk_phases.py --lib tools/ab/topkph.so [--config c4] [--sweeps 25]

The library must be built with -DALBEDO_TOPK_PHASES (topk.hip: per-wave s_memtime accumulators per
phase, summed over waves; the stamps themselves cost ~10 % of the scan's cycles).  Ingests the
synthetic config, runs the sweeps of the default bench (5 warmup + 20 timed = 25), then
recommendForAllUsers(30) over every user and prints the per-phase cycles as JSON.
"""
import argparse
import ctypes as C
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
PH = ["dma_wait_barrier", "bound_test", "mfma_and_tile_checks", "appends", "compaction", "mask_walk",
      "compaction_vmem_drain", "unused"]
CNT = ["chunk_iterations", "chunks_scored", "tiles_with_hits", "compaction_events", "rows_compacted", "-", "-", "-"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--lib", required=True)
    ap.add_argument("--config", default="c4")
    ap.add_argument("--sweeps", type=int, default=25)
    ap.add_argument("--out", default=None)
    args = ap.parse_args()
    from albedo_amd import _lib as L
    L.LIB_PATH = os.path.abspath(args.lib)
    lib = L.load()
    lib.als_debug_topk_phases.restype = C.c_int
    lib.als_debug_topk_phases.argtypes = [C.POINTER(C.c_ulonglong), C.c_int]
    from albedo_amd.synthetic import CONFIGS, popularity_table, user_degrees
    spec = CONFIGS[args.config]
    k = {"c2": 64, "c4": 128}[args.config]
    p = L.als_params()
    L.check(lib.als_params_default(C.byref(p)))
    p.rank, p.implicit_prefs, p.reg_param, p.alpha, p.seed = k, 1, 0.5, 40.0, 42
    h = C.c_void_p()
    L.check(lib.als_create(C.byref(p), C.byref(h)))
    deg = user_degrees(spec)
    prefix = np.ascontiguousarray(np.r_[0, np.cumsum(deg)].astype(np.int64))
    cw, perm = popularity_table(spec)
    L.check(lib.als_set_ratings_synthetic(h, spec.seed, spec.rounds, spec.n_users, spec.n_items,
                                          L.ptr(prefix, C.c_int64), L.ptr(np.ascontiguousarray(cw), C.c_double),
                                          L.ptr(np.ascontiguousarray(perm), C.c_int32)))
    L.check(lib.als_init_factors_random(h, 42))
    for s in range(args.sweeps):
        L.check(lib.als_run_sweeps(h, 1))
        print(f"sweep {s + 1}", flush=True)
    n_u = lib.als_num_rows(h, 0)
    ids = np.empty((n_u, 30), np.int32)
    sc = np.empty((n_u, 30), np.float32)
    buf = (C.c_ulonglong * 16)()
    lib.als_debug_topk_phases(buf, 1)
    t0 = time.perf_counter()
    L.check(lib.als_recommend(h, 0, 30, None, n_u, None, L.ptr(ids, C.c_int32), L.ptr(sc, C.c_float)))
    wall = time.perf_counter() - t0
    lib.als_debug_topk_phases(buf, 0)
    tm = np.zeros(5)
    L.check(lib.als_topk_timing(h, L.ptr(tm, C.c_double)))
    v = list(buf)
    tot = sum(v[:8])
    out = {"wall_s": wall, "topk_ms": tm[:4].tolist(), "users": int(n_u),
           "phase_cycles_sum_over_waves": {PH[i]: v[i] for i in range(8)},
           "phase_frac": {PH[i]: v[i] / max(tot, 1) for i in range(8)},
           "counts": {CNT[i]: v[8 + i] for i in range(5)}}
    print(json.dumps(out, indent=1))
    if args.out:
        with open(args.out, "w") as f:
            json.dump(out, f, indent=1)
    lib.als_destroy(h)


if __name__ == "__main__":
    main()
