"""Summarise hipcc -Rpass-analysis=kernel-resource-usage remarks: one line per kernel."""
import re, subprocess, sys
src = sys.argv[1]
out = subprocess.run(["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "-I../../include", "-I.", "--offload-arch=gfx950",
                      "-c", src, "-o", "/tmp/kres.o", "-Rpass-analysis=kernel-resource-usage"],
                     capture_output=True, text=True).stderr
cur = None
rows = {}
for line in out.splitlines():
    m = re.search(r"Function Name: (\S+)", line)
    if m:
        cur = m.group(1); rows[cur] = {}; continue
    m = re.search(r"remark: +([A-Za-z /\[\]]+?): (\d+)", line)
    if m and cur:
        rows[cur][m.group(1).strip()] = int(m.group(2))
pat = sys.argv[2] if len(sys.argv) > 2 else ""
for k, v in rows.items():
    if pat in k:
        print(f"{k[:60]:60s} vgpr {v.get('VGPRs',0):3d} agpr {v.get('AGPRs',0):3d} occ {v.get('Occupancy [waves/SIMD]',0)} "
              f"vspill {v.get('VGPRs Spill',0)} sspill {v.get('SGPRs Spill',0)} lds {v.get('LDS Size [bytes/block]',0)}")
