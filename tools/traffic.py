"""HBM traffic of the solve kernels from rocprofv3 PMC passes (FETCH_SIZE, WRITE_SIZE) of one sweep.

usage: python tools/traffic.py <prof dir with pmc_fetch/ and pmc_write/> <config> <out json>

FETCH_SIZE / WRITE_SIZE are kilobytes (rocprofiler-sdk counter_defs.yaml).  On gfx950 FETCH_SIZE
reports half the bytes of a wide coalesced streaming read (16 B per lane; MI355X_MICROARCH.md, HBM
section): the gathers here are float4 per lane over whole factor rows, so the fetch count is
doubled.  WRITE_SIZE is exact for 16-B-per-lane stores.  Values are per sweep (the bench command
runs exactly one sweep: --steps 1 --warmup 0), summed over the kernel's launches in that sweep.
"""
import collections
import csv
import glob
import json
import re
import sys


def per_kernel(path, counter):
    tot = collections.defaultdict(float)
    nd = collections.defaultdict(set)
    for f in glob.glob(f"{path}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] != counter:
                continue
            k = r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0]
            k = k.replace("void ", "").replace("albedo::", "")
            m = re.search(r"([a-z][a-z0-9_]*)_kernel", k)  # also mangled names (anonymous-namespace kernels)
            base = m.group(1) if m else k.split("<")[0]
            tot[base] += float(r["Counter_Value"])
            nd[base].add(r["Dispatch_Id"])
    return tot, {k: len(v) for k, v in nd.items()}


def main():
    root, cfg, out = sys.argv[1], sys.argv[2], sys.argv[3]
    fetch, nf = per_kernel(f"{root}/pmc_fetch", "FETCH_SIZE")
    write, nw = per_kernel(f"{root}/pmc_write", "WRITE_SIZE")
    res = {"_source": f"rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE (separate runs) of `bench.py --config {cfg} "
                      "--steps 1 --warmup 0 --no-cpu --topk-users 0`; FETCH_SIZE x2 (gfx950 wide-read correction); "
                      "GB (1e9 B) per sweep, summed over the kernel's launches"}
    for k in sorted(set(fetch) | set(write)):
        if not k.startswith(("solve_", "gram", "rotate", "topk", "heavy_", "wave_", "presplit", "colmax", "nnls_")):
            continue
        f_gb = 2.0 * fetch.get(k, 0.0) * 1024 / 1e9
        w_gb = write.get(k, 0.0) * 1024 / 1e9
        res[k] = {"hbm_gb_per_sweep": f_gb + w_gb, "fetch_gb": f_gb, "write_gb": w_gb, "launches": nf.get(k, 0)}
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
