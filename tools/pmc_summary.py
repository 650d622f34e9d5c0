"""Summarise rocprofv3 PMC csv passes: per kernel, sum of each counter and per-dispatch averages."""
import collections
import csv
import glob
import sys

root = sys.argv[1]
agg = collections.defaultdict(lambda: collections.defaultdict(float))
disp = collections.defaultdict(set)
dur = collections.defaultdict(dict)
for f in sorted(glob.glob(f"{root}/p*/run_counter_collection.csv")):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("albedo::", "")
        agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
        disp[(k, f)].add(r["Dispatch_Id"])
        dur[k][(f, r["Dispatch_Id"])] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
        agg[k]["_lds"] = float(r["LDS_Block_Size"])
        agg[k]["_vgpr"] = float(r["VGPR_Count"]) + float(r.get("Accum_VGPR_Count", 0) or 0)
for k, c in agg.items():
    print(f"== {k}  dispatches/pass={len(disp[(k, sorted(glob.glob(root + '/p1/run_counter_collection.csv'))[0])]) if glob.glob(root + '/p1/run_counter_collection.csv') else '?'}")
    for n in sorted(c):
        print(f"   {n:28s} {c[n]:.4e}")
    if c.get("SQ_BUSY_CYCLES"):
        print(f"   avg waves resident/SE-cycle (LEVEL/BUSY): {c.get('SQ_LEVEL_WAVES', 0) / c['SQ_BUSY_CYCLES']:.2f}")
    if c.get("SQ_WAVE_CYCLES"):
        w = c["SQ_WAVE_CYCLES"]
        print(f"   wait_any {c.get('SQ_WAIT_ANY', 0) / w:.2f}  wait_inst {c.get('SQ_WAIT_INST_ANY', 0) / w:.2f}  active {c.get('SQ_ACTIVE_INST_ANY', 0) / w:.2f} of wave-cycles")
