"""Build-time check of rotate_bf_kernel's counted waits (albedo_amd/csrc/als_kernels.hip).

The kernel prefetches the next tile's X rows from asm and waits for them with s_waitcnt vmcnt(24)
(with the fused fp16 split: 3 stores per 16-column block J) or vmcnt(8) (1 store per J), leaving
the current tile's stores in flight.  That is exact only while the compiled J loop issues exactly
those stores and nothing else that counts in vmcnt, and never reads the prefetch registers before
the wait.  This script disassembles the object's gfx950 code and checks, after the in-loop
prefetch group:
  * per J: one global_store_dwordx4 (Z) and two global_store_dwordx2 (the fp16 hi / lo rows),
    the loop unrolled by a factor that divides NJ = 8;
  * no other vector-memory instruction (loads, scratch spills, buffer ops) anywhere after the
    prefetch group, and no scratch anywhere in the kernel;
  * no instruction after the prefetch group reads the prefetch destination registers.
usage: python tools/check_rotate_isa.py <als_kernels.o>   (exit 0: the waits are exact)
The Makefile rebuilds als_kernels.o with -DALBEDO_ROTATE_VMCNT0 (plain vmcnt(0) waits) when the
check fails.
"""
import os
import re
import subprocess
import sys
import tempfile

LLVM = "/opt/rocm/lib/llvm/bin"
SYM = "_ZN6albedo16rotate_bf_kernelILi128EEEvPKfPKDF16bPflS2_fPDF16_l"
NJ = 8


def disasm(obj):
    with tempfile.TemporaryDirectory() as td:
        fat, dev = os.path.join(td, "fat"), os.path.join(td, "dev.o")
        subprocess.run([f"{LLVM}/llvm-objcopy", f"--dump-section=.hip_fatbin={fat}", obj, os.path.join(td, "x.o")],
                       check=True, capture_output=True)
        subprocess.run([f"{LLVM}/clang-offload-bundler", "--unbundle", "--type=o", f"--input={fat}",
                        "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--output={dev}"], check=True, capture_output=True)
        out = subprocess.run([f"{LLVM}/llvm-objdump", "-d", f"--disassemble-symbols={SYM}", dev], check=True,
                             capture_output=True, text=True).stdout
    ins = []
    for line in out.splitlines():
        t = line.strip()
        if not t or t.startswith(("Disassembly", "0000")) or t.endswith(":"):
            continue
        ins.append(t.split("//")[0].strip())
    return ins


def regs(text):
    """VGPR numbers named in an operand string."""
    out = set()
    for a, b in re.findall(r"\bv\[(\d+):(\d+)\]", text):
        out.update(range(int(a), int(b) + 1))
    for a in re.findall(r"\bv(\d+)\b", text):
        out.add(int(a))
    return out


def check(ins):
    if not ins:
        return "kernel not found"
    if any(i.startswith(("scratch_", "buffer_")) for i in ins):
        return "scratch / buffer instructions in the kernel (spills count in vmcnt)"
    waits = [n for n, i in enumerate(ins) if re.match(r"s_waitcnt vmcnt\((8|24)\)$", i)]
    if len(waits) != 2:
        return f"expected the vmcnt(8) and vmcnt(24) waits, found {len(waits)}"
    # the in-loop prefetch group: the first 8 consecutive global_load_dwordx4 after the waits
    n = waits[-1]
    while n < len(ins) and not ins[n].startswith("global_load_dwordx4"):
        n += 1
    grp = []
    while n < len(ins) and len(grp) < 8:
        if ins[n].startswith("global_load_dwordx4"):
            grp.append(n)
        elif ins[n].startswith(("global_", "flat_")):
            return f"unexpected memory op inside the prefetch group: {ins[n]}"
        n += 1
    if len(grp) != 8:
        return f"prefetch group has {len(grp)} loads, expected 8"
    pre = set()
    for g in grp:
        pre |= regs(ins[g].split(",")[0])
    rest = ins[grp[-1] + 1:]
    z = sum(1 for i in rest if i.startswith("global_store_dwordx4"))
    h = sum(1 for i in rest if i.startswith("global_store_dwordx2"))
    other = [i for i in rest if i.startswith(("global_", "flat_")) and not i.startswith(("global_store_dwordx4",
                                                                                          "global_store_dwordx2"))]
    if other:
        return f"other vector-memory ops after the prefetch: {other[:3]}"
    if z == 0 or NJ % z or h != 2 * z:
        return f"J-loop stores per unrolled body: {z} x dwordx4, {h} x dwordx2 (need u and 2u, u | {NJ})"
    for i in rest:
        op, _, args = i.partition(" ")
        if not args:
            continue
        srcs = args if op.startswith(("global_store", "ds_write", "s_")) else args.partition(",")[2]
        if regs(srcs) & pre:
            return f"a prefetch register is read before its wait: {i}"
    return None


def main():
    err = check(disasm(sys.argv[1]))
    if err:
        print(f"check_rotate_isa: {err} -> rebuild with plain vmcnt(0) waits", file=sys.stderr)
        sys.exit(1)
    print("check_rotate_isa: counted waits exact")


if __name__ == "__main__":
    main()
