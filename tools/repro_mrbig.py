"""Determinism probe for the 2-rank shared-GPU c4-shaped sweep (tests/test_multi_rank.py
test_sharded_sweep_gpu_c4_shaped): runs the tests' gpubig worker N times and compares the factors
bit for bit across runs (odd runs first fill and free 16 GiB of device memory with NaN per rank), printing the rows that differ with their degree.  No oracle involved.

usage: python tools/repro_mrbig.py N OUTDIR
"""
import os
import socket
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def run_once(out, world=2, k=128, extra=None):
    port = free_port()
    procs = []
    for r in range(world):
        env = dict(os.environ, RANK=str(r), WORLD_SIZE=str(world), LOCAL_RANK="0", MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port), **(extra or {}))
        procs.append(subprocess.Popen([sys.executable, os.path.join(ROOT, "tests", "mp_worker.py"), "gpubig", out, str(k)],
                                      env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT))
    for p in procs:
        o, _ = p.communicate(timeout=300)
        if p.returncode != 0:
            print(o.decode(errors="replace")[-3000:])
            raise SystemExit(p.returncode)
    return np.load(out)


def main():
    n, outdir = int(sys.argv[1]), sys.argv[2]
    os.makedirs(outdir, exist_ok=True)
    from albedo_amd.synthetic import SynthSpec, generate
    d = generate(SynthSpec(60000, 12000, 2_000_000, zipf_s=0.8, seed=43))
    uid, udeg = np.unique(d["user"], return_counts=True)
    iid, ideg = np.unique(d["item"], return_counts=True)
    first = None
    for t in range(n):
        res = run_once(os.path.join(outdir, f"run{t}.npz"), extra={"ALBEDO_TEST_POLLUTE": "16"} if t % 2 else None)
        if first is None:
            first = {k: res[k].copy() for k in ("U", "V")}
            print(f"run {t}: reference", flush=True)
            continue
        for name, deg in (("V", ideg), ("U", udeg)):
            a, b = first[name], res[name]
            rows = np.nonzero(np.any(a.view(np.uint32) != b.view(np.uint32), axis=1))[0]
            rel = np.linalg.norm(a - b, axis=1) / np.maximum(np.linalg.norm(a, axis=1), 1e-30)
            print(f"run {t} {name}: {rows.size} rows differ, max rel {rel.max():.3g}", flush=True)
            for r in rows[np.argsort(-rel[rows])][:10]:
                print(f"   row {r} deg {deg[r]} rel {rel[r]:.3g}", flush=True)


if __name__ == "__main__":
    main()
