"""Diagnostic (not a test): heavy-path per-row error of one item half-sweep, determinism over reruns."""
import sys, os
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", ".."))
import numpy as np
from tests.test_gpu_parity import Ctx
from albedo_amd import _lib as L
from oracle import spark_als as O
from albedo_amd.synthetic import SynthSpec, generate
if os.environ.get("ALBEDO_LIB"): L.LIB_PATH = os.environ["ALBEDO_LIB"]
lib = L.load()
for k in (50, 128):
    d = generate(SynthSpec(1500, 600, 30000, seed=20 + k))
    B = O.make_blocks(d["user"], d["item"], d["rating"])
    rng = np.random.default_rng(k)
    U0 = rng.standard_normal((len(B.user_ids), k)).astype(np.float32)
    U0 /= np.linalg.norm(U0, axis=1, keepdims=True)
    V_ref = O.half_sweep(U0, B.i_ptr, B.i_col, B.i_val, reg=0.5, alpha=40.0)
    outs = []
    for rep in range(3):
        c = Ctx(lib, k, light=0)
        c.ratings(d["user"], d["item"], d["rating"])
        c.inject(0, B.user_ids, U0)
        c.inject(1, B.item_ids, np.zeros((len(B.item_ids), k), np.float32))
        c.half(1)
        outs.append(c.factors(1)[1])
    c.half(0)
    U_ref = O.half_sweep(outs[-1], B.u_ptr, B.u_col, B.u_val, reg=0.5, alpha=40.0)
    U = c.factors(0)[1]
    eu = np.max(np.abs(U - U_ref), 1) / np.max(np.abs(U_ref), 1)
    du = np.diff(B.u_ptr)
    top = np.argsort(eu)[-6:]
    print(f"k={k} user half: max {eu.max():.2e} median {np.median(eu):.2e} worst deg {du[top].tolist()} err {[f'{x:.1e}' for x in eu[top]]}")
    deg = np.diff(B.i_ptr)
    for rep, V in enumerate(outs):
        e = np.max(np.abs(V - V_ref), 1) / np.max(np.abs(V_ref), 1)
        top = np.argsort(e)[-6:]
        same = np.array_equal(V, outs[0])
        ndiff = int(np.sum(np.any(V != outs[0], axis=1)))
        print(f"k={k} rep={rep} same_as_rep0={same} rows_differ={ndiff} max {e.max():.2e} median {np.median(e):.2e} "
              f"worst rows {top.tolist()} deg {deg[top].tolist()} err {[f'{x:.1e}' for x in e[top]]}", flush=True)
