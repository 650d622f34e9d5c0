"""Static instruction mix of the kernels in a hipcc -S listing (gfx950).

usage: python tools/isa_count.py <file.s> <name-substring> [--blocks]
Prints per kernel: instructions by class (valu / mfma / salu / lds / vmem / other), VGPRs, and with
--blocks the same counts per basic block (label), to see where a kernel's VALU instructions sit.
"""
import collections
import re
import sys


def classify(op):
    if op.startswith("v_mfma"):
        return "mfma"
    if op.startswith("v_"):
        return "valu"
    if op.startswith("s_"):
        return "salu"
    if op.startswith("ds_"):
        return "lds"
    if op.startswith(("global_", "buffer_", "flat_", "scratch_")):
        return "vmem"
    return "other"


def main():
    path, pat = sys.argv[1], sys.argv[2]
    blocks = "--blocks" in sys.argv
    text = open(path).read()
    for m in re.finditer(r"\n(_Z\S+):[^\n]*\n(.*?)\n\.Lfunc_end", text, re.S):
        name, body = m.group(1), m.group(2)
        if pat not in name:
            continue
        tot = collections.Counter()
        per = collections.OrderedDict()
        cur = "entry"
        per[cur] = collections.Counter()
        for line in body.split("\n"):
            t = line.strip()
            if not t or t.startswith((";", ".")):
                if t.startswith(".LBB"):
                    cur = t.rstrip(":").split()[0]
                    per[cur] = collections.Counter()
                continue
            if t.endswith(":"):
                cur = t[:-1]
                per[cur] = collections.Counter()
                continue
            c = classify(t.split()[0])
            tot[c] += 1
            per[cur][c] += 1
        vg = re.search(re.escape(name) + r"\.num_vgpr, (\d+)", text)
        print(f"{name}  vgpr={vg.group(1) if vg else '?'}  {dict(tot)}")
        if blocks:
            for b, c in per.items():
                if c:
                    print(f"   {b:16s} {dict(c)}")


if __name__ == "__main__":
    main()
