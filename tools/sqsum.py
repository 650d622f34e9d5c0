"""Per-kernel SQ counter summary of tools/prof.sh's two SQ passes (sq1/, sq2/) as JSON.

usage: python tools/sqsum.py <prof dir> <out json>

Counters are summed over a kernel's dispatches in each pass.  Derived (MI355X_MICROARCH.md, PMC
units): SQ_WAVE_CYCLES / SQ_WAIT_* / SQ_ACTIVE_INST_* count quad-cycles; SQ_VALU_MFMA_BUSY_CYCLES
counts cycles summed over SIMDs; GRBM_GUI_ACTIVE is summed over the 8 XCDs, so GRBM / 8 is the
kernel's cycle count at the live (DVFS) clock.  mfma_busy = MFMA busy cycles / (cycles x 1024 SIMDs).
"""
import collections
import csv
import glob
import json
import sys


def demangle(name):
    if not name.startswith("_Z"):
        return name
    import shutil
    import subprocess
    tool = shutil.which("c++filt") or "/opt/rocm/lib/llvm/bin/llvm-cxxfilt"
    try:
        return subprocess.run([tool, name], capture_output=True, text=True).stdout.strip() or name
    except OSError:
        return name


def short(name):
    k = demangle(name)
    if k.startswith("_Z"):  # c++filt cannot read some (bf16 / fp16 parameter) manglings: name<int arg>
        import re
        i, last = 3 if k.startswith("_ZN") else 2, None  # <length><identifier> components
        while i < len(k) and k[i].isdigit():
            j = i
            while k[j].isdigit():
                j += 1
            n = int(k[i:j])
            last, i = k[j:j + n], j + n
        m = re.match(r"ILi(\d+)E", k[i:])
        if last:
            return last + (f"<{m.group(1)}>" if m else "")
    k = k.replace("(anonymous namespace)::", "").split("(")[0].replace("void ", "").replace("albedo::", "")
    return k.replace(" ", "")


def load(path):
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    disp = collections.defaultdict(set)
    dur = collections.defaultdict(dict)
    for f in glob.glob(f"{path}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            k = short(r["Kernel_Name"])
            agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
            disp[k].add(r["Dispatch_Id"])
            dur[k][r["Dispatch_Id"]] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9
            agg[k]["_vgpr"] = float(r["VGPR_Count"]) + float(r.get("Accum_VGPR_Count", 0) or 0)
            agg[k]["_lds"] = float(r["LDS_Block_Size"])
    return agg, {k: len(v) for k, v in disp.items()}, {k: sum(v.values()) for k, v in dur.items()}


def main():
    root, out = sys.argv[1], sys.argv[2]
    p1, n1, d1 = load(f"{root}/sq1")
    p2, n2, d2 = load(f"{root}/sq2")
    res = {"_source": f"rocprofv3 --pmc SQ passes of tools/prof.sh ({root}); sums over dispatches per pass",
           "_derived": "mfma_busy = SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE/8 x 1024 SIMDs); wait/active "
                       "fractions of SQ_WAVE_CYCLES; lds_conflict = SQ_LDS_BANK_CONFLICT / SQ_ACTIVE_INST_LDS"}
    for k in sorted(set(p1) | set(p2)):
        a, b = p1.get(k, {}), p2.get(k, {})
        e = {"dispatches": n1.get(k, n2.get(k)), "seconds_pass1": d1.get(k), "seconds_pass2": d2.get(k),
             "vgpr": a.get("_vgpr", b.get("_vgpr")), "lds_bytes": a.get("_lds", b.get("_lds"))}
        e.update({c: v for c, v in a.items() if not c.startswith("_")})
        e.update({c: v for c, v in b.items() if not c.startswith("_")})
        # GRBM_GUI_ACTIVE from whichever pass collected it (prof.sh: pass 2; pmc_topk4.sh: pass 1)
        gp = b if "GRBM_GUI_ACTIVE" in b else a
        cyc = gp.get("GRBM_GUI_ACTIVE", 0.0) / 8.0
        if cyc and "SQ_VALU_MFMA_BUSY_CYCLES" in a:
            e["mfma_busy"] = a["SQ_VALU_MFMA_BUSY_CYCLES"] / (cyc * 1024)
        dur = (d2 if gp is b else d1).get(k)
        if cyc and dur:
            e["clock_ghz"] = cyc / dur * 1e-9
        w = a.get("SQ_WAVE_CYCLES")
        if w:
            for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY"):
                if c in a:
                    e[c.lower().replace("sq_", "") + "_frac"] = a[c] / w
        if b.get("SQ_ACTIVE_INST_LDS"):
            e["lds_conflict"] = b.get("SQ_LDS_BANK_CONFLICT", 0.0) / b["SQ_ACTIVE_INST_LDS"]
        res[k] = e
    json.dump(res, open(out, "w"), indent=1)


if __name__ == "__main__":
    main()
