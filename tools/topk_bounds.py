"""Top-k pruning analysis on trained factors (GPU box; torch for the reference scores).

Fits a BASELINE config with the engine for --sweeps sweeps, pulls the original-basis factors, and
for a random sample of users measures how much of the dst side each candidate bound would have to
score, against the sample's exact 64th-best (and 30th-best) scores:

  norm     the scan's current bound: dst rows by descending norm, stop once ||s||*||t_head|| <= tau
  split_m  s.t <= s_P.t_P + ||s_perp||*||t_perp|| with P = the leading m eigen-directions of the dst
           Gram (item level: the ideal fraction for that bound)
  chunked  the same bound per chunk of CH rows with a chunk order by ||t_perp|| (per-chunk skip)
  ball     s.t <= s.c + ||s||*r per norm-ordered chunk (c = chunk mean, r = max ||t - c||)

  python tools/topk_bounds.py --config c4 --sweeps 25 --sample 16384 --out gpurun_out/bounds_c4.json
"""
from __future__ import annotations

import argparse
import ctypes as C
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def log(*a):
    print(f"[{time.strftime('%H:%M:%S')}]", *a, flush=True)


def fit_factors(config, sweeps):
    from albedo_amd import _lib as L
    from albedo_amd.synthetic import CONFIGS, popularity_table, user_degrees
    import bench
    lib = L.load()
    spec = CONFIGS[config]
    k = bench.CONFIG_RANK[config]
    p = L.als_params()
    L.check(lib.als_params_default(C.byref(p)))
    p.rank, p.implicit_prefs, p.reg_param, p.alpha, p.seed = k, 1, 0.5, 40.0, 42
    p.device = 0
    h = C.c_void_p()
    L.check(lib.als_create(C.byref(p), C.byref(h)))
    deg = user_degrees(spec)
    prefix = np.ascontiguousarray(np.r_[0, np.cumsum(deg)].astype(np.int64))
    cw, perm = popularity_table(spec)
    L.check(lib.als_set_ratings_synthetic(h, spec.seed, spec.rounds, spec.n_users, spec.n_items,
                                          L.ptr(prefix, C.c_int64), L.ptr(np.ascontiguousarray(cw), C.c_double),
                                          L.ptr(np.ascontiguousarray(perm), C.c_int32)))
    L.check(lib.als_init_factors_random(h, 42))
    log("ingest done")
    L.check(lib.als_run_sweeps(h, sweeps))
    L.check(lib.als_synchronize(h))
    log(f"{sweeps} sweeps done")
    out = []
    for side in (0, 1):
        n = lib.als_num_rows(h, side)
        f = np.empty((n, k), np.float32)
        L.check(lib.als_get_factors(h, side, None, L.ptr(f, C.c_float)))
        out.append(f)
    deg_u = np.empty(out[0].shape[0], np.int64)
    L.check(lib.als_get_degrees(h, 0, L.ptr(deg_u, C.c_int64)))
    lib.als_destroy(h)
    return out[0], out[1], deg_u, k


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c4")
    ap.add_argument("--sweeps", type=int, default=25)
    ap.add_argument("--sample", type=int, default=16384)
    ap.add_argument("--out", default="gpurun_out/bounds.json")
    ap.add_argument("--fake", action="store_true")
    ap.add_argument("--npz", default=None, help="analyse saved factors (U, V, udeg) on the CPU")
    args = ap.parse_args()
    if args.npz:
        z = np.load(args.npz)
        U, V, deg_u = z["U"], z["V"], z["udeg"]
        k = U.shape[1]
        dev = torch.device("cpu")
    elif args.fake:  # CPU dry run of the analysis on random factors
        rng0 = np.random.default_rng(0)
        k = 64
        U = rng0.standard_normal((20000, k)).astype(np.float32)
        V = (rng0.standard_normal((5000, k)) * rng0.lognormal(0, 1, (5000, 1))).astype(np.float32)
        deg_u = rng0.integers(1, 100, 20000)
        dev = torch.device("cpu")
    else:
        torch.cuda.init()
        U, V, deg_u, k = fit_factors(args.config, args.sweeps)
        dev = torch.device("cuda:0")
    CH = {64: 128, 128: 64, 256: 32}[{50: 64, 64: 64, 128: 128, 256: 256}[k]]
    rng = np.random.default_rng(5)
    sel = np.sort(rng.choice(U.shape[0], args.sample, replace=False))
    T = torch.from_numpy(V).to(dev)
    S = torch.from_numpy(U[sel]).to(dev)
    n, m_s = T.shape[0], S.shape[0]
    res = {"config": args.config, "sweeps": args.sweeps, "sample": m_s, "n_dst": n, "rank": k, "CH": CH}
    # exact top-64 per sampled user (fp32)
    best = torch.full((m_s, 64), -float("inf"), device=dev)
    B = 65536
    for j0 in range(0, n, B):
        sc = S @ T[j0:j0 + B].T
        best = torch.topk(torch.cat([best, sc], 1), 64, dim=1).values
    tau64, tau30 = best[:, 63], best[:, 29]
    log("exact top-64 done")
    snorm = S.norm(dim=1)
    tnorm = T.norm(dim=1)
    order = torch.argsort(tnorm, descending=True)
    Ts = T[order]
    tns = tnorm[order]
    nch = (n + CH - 1) // CH
    head = tns[::CH][:nch]
    res["tnorm_quantiles"] = torch.quantile(tnorm[:1_000_000].double(), torch.tensor([0.5, 0.9, 0.99, 0.999, 1.0], dtype=torch.float64, device=dev)).tolist()
    res["snorm_quantiles"] = torch.quantile(snorm.double(), torch.tensor([0.1, 0.5, 0.9, 0.99, 1.0], dtype=torch.float64, device=dev)).tolist()
    res["tau64_over_snorm_tmax_quantiles"] = torch.quantile((tau64 / (snorm * tnorm.max())).double(), torch.tensor([0.1, 0.5, 0.9], dtype=torch.float64, device=dev)).tolist()
    # --- norm order (current scan): depth = chunks whose head still passes ---
    for name, tau in (("tau64", tau64), ("tau30", tau30)):
        need = (snorm[:, None] * head[None, :]) > tau[:, None]
        depth = need.sum(1).double()
        res[f"norm_{name}_chunk_frac_mean"] = float(depth.mean() / nch)
        res[f"norm_{name}_chunk_frac_q"] = torch.quantile(depth / nch, torch.tensor([0.1, 0.5, 0.9, 0.99], dtype=torch.float64, device=dev)).tolist()
    # per degree class of the sampled users
    dsel = torch.from_numpy(deg_u[sel]).to(dev)
    need = (snorm[:, None] * head[None, :]) > tau64[:, None]
    depth = need.sum(1).double() / nch
    res["norm_tau64_by_degree"] = {}
    for lo, hi in ((1, 2), (2, 5), (5, 17), (17, 65), (65, 257), (257, 10 ** 9)):
        msk = (dsel >= lo) & (dsel < hi)
        if int(msk.sum()) > 0:
            res["norm_tau64_by_degree"][f"{lo}-{hi - 1}"] = [int(msk.sum()), float(depth[msk].mean())]
    log("norm bound done", res["norm_tau64_chunk_frac_mean"])
    # --- eigenbasis of the dst Gram and of the src Gram ---
    Gt = (T.double().T @ T.double())
    wt, Vt = torch.linalg.eigh(Gt)
    wt, Vt = wt.flip(0), Vt.flip(1)
    Us = torch.from_numpy(U).to(dev)
    Gs = torch.zeros(k, k, dtype=torch.float64, device=dev)
    for i0 in range(0, Us.shape[0], 1 << 21):
        x = Us[i0:i0 + (1 << 21)].double()
        Gs += x.T @ x
    del Us
    ws, Vs = torch.linalg.eigh(Gs)
    ws, Vs = ws.flip(0), Vs.flip(1)
    res["dst_gram_energy_cum"] = (wt.cumsum(0) / wt.sum())[[0, 1, 3, 7, 15, 31, 63]].tolist()
    res["src_gram_energy_cum"] = (ws.cumsum(0) / ws.sum())[[0, 1, 3, 7, 15, 31, 63]].tolist()
    # --- split bound, item level and chunked ---
    for bname, Vb in (("dstbasis", Vt), ("srcbasis", Vs)):
        Tr = (T.double() @ Vb).float()
        Sr = (S.double() @ Vb).float()
        for m in (1, 2, 4, 8, 16, 32):
            tP, sP = Tr[:, :m], Sr[:, :m]
            tperp = (tnorm.square() - tP.square().sum(1)).clamp_min(0).sqrt()
            sperp = (snorm.square() - sP.square().sum(1)).clamp_min(0).sqrt()
            cnt = torch.zeros(m_s, dtype=torch.float64, device=dev)
            for j0 in range(0, n, B):
                b = sP @ tP[j0:j0 + B].T + sperp[:, None] * tperp[None, j0:j0 + B]
                cnt += (b > tau64[:, None]).sum(1).double()
            res[f"split_{bname}_m{m}_item_frac"] = float(cnt.mean() / n)
            # chunked: dst rows by descending ||t_perp||, per-chunk box over the m leading coords
            o2 = torch.argsort(tperp, descending=True)
            tp2, tq2 = tP[o2], tperp[o2]
            pad = nch * CH - n
            if pad:
                tp2 = torch.cat([tp2, tp2[-1:].expand(pad, m)])
                tq2 = torch.cat([tq2, tq2[-1:].expand(pad)])
            hi = tp2.view(nch, CH, m).amax(1)
            lo = tp2.view(nch, CH, m).amin(1)
            rq = tq2.view(nch, CH).amax(1)
            mid, half = (hi + lo) / 2, (hi - lo) / 2
            bc = sP @ mid.T + sP.abs() @ half.T + sperp[:, None] * rq[None, :]
            res[f"split_{bname}_m{m}_chunk_frac"] = float((bc > tau64[:, None]).double().mean())
            log(bname, m, res[f"split_{bname}_m{m}_item_frac"], res[f"split_{bname}_m{m}_chunk_frac"])
    # --- ball bound on norm-ordered chunks ---
    pad = nch * CH - n
    Tp = torch.cat([Ts, Ts[-1:].expand(pad, k)]) if pad else Ts
    cen = Tp.view(nch, CH, k).mean(1)
    rad = (Tp.view(nch, CH, k) - cen[:, None, :]).norm(dim=2).amax(1)
    bb = S @ cen.T + snorm[:, None] * rad[None, :]
    res["ball_normorder_chunk_frac"] = float((bb > tau64[:, None]).double().mean())
    res["ball_radius_over_head_median"] = float((rad / head).median())
    # box bound (all k coordinates) on norm-ordered chunks
    hi = Tp.view(nch, CH, k).amax(1)
    lo = Tp.view(nch, CH, k).amin(1)
    bx = S @ ((hi + lo) / 2).T + S.abs() @ ((hi - lo) / 2).T
    res["box_normorder_chunk_frac"] = float((bx > tau64[:, None]).double().mean())
    log("ball/box done")
    # group effect: sampled users sorted by the current key (tau64/||s|| as a proxy), groups of 64
    need = (snorm[:, None] * head[None, :]) > tau64[:, None]
    depth = need.sum(1)
    for gsz in (16, 64, 512):
        o = torch.argsort(tau64 / snorm)
        dg = depth[o][: (m_s // gsz) * gsz].view(-1, gsz).amax(1).double()
        res[f"norm_group{gsz}_sorted_by_tau_over_snorm_frac"] = float(dg.mean() / nch)
    os.makedirs(os.path.dirname(args.out) or ".", exist_ok=True)
    json.dump(res, open(args.out, "w"), indent=1)
    log(json.dumps(res))


if __name__ == "__main__":
    main()
