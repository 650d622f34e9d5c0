"""Static wait-state hazard check of a gfx950 device listing (hipcc --offload-device-only -S).

The compiler inserts the wait states CDNA needs between its own instructions, but it does not look
inside inline asm: a hand-written DPP instruction, or a compiler instruction feeding one, is checked
by nobody.  This scan re-checks every kernel of a listing against the rules below (the ones LLVM's
GCNHazardRecognizer applies on gfx950, restated) and prints each violation with the instructions
around it.  Wait states: one per instruction, N + 1 for `s_nop N`.

  DPP-VGPR   an instruction writes a VGPR that a DPP instruction reads (ANY of its VGPR sources,
             the tied accumulator of v_fmac/v_mac included, not only the DPP-permuted src0)
             within 2 wait states (checkDPPHazards: DppVgprWaitStates = 2)
  DPP-EXEC   a VALU instruction writes EXEC (v_cmpx*) within 5 wait states before a DPP
             instruction (DppExecWaitStates = 5)
  TRANS      a transcendental (v_rcp/v_rsq/v_sqrt/v_exp/v_log/v_sin/v_cos ...) writes a VGPR that
             the next non-transcendental VALU instruction reads (TransDefWaitstates = 1)
  DSTSEL     a VALU instruction writes part of a VGPR (SDWA dst_sel, op_sel dst bit, v_fma_mixhi)
             and the next VALU instruction reads it (hasDstSelForwardingHazard: 1 wait state)

Control flow: the predecessors of an instruction are the previous instruction (unless that is an
unconditional branch or s_endpgm) and, at a label, every branch to it; the backward walk follows
all of them.

usage: python tools/isa_hazards.py <file.s> [<file.s> ...] [--kernel SUBSTR] [--quiet]
exit status 1 when a violation is found (build() runs it on the shipped kernels).
"""
from __future__ import annotations

import re
import sys

DPP_RE = re.compile(r"\b(row_newbcast|row_shr|row_shl|row_ror|row_mirror|row_half_mirror|quad_perm|"
                    r"row_bcast|row_share|row_xmask|wave_shl|wave_shr|wave_rol|wave_ror)\b")
VREG_RE = re.compile(r"\bv\[(\d+):(\d+)\]|\bv(\d+)\b")
TRANS_OPS = ("v_rcp_", "v_rsq_", "v_sqrt_", "v_exp_", "v_log_", "v_sin_", "v_cos_", "v_rcp_iflag_")


def vregs(text):
    out = set()
    for m in VREG_RE.finditer(text):
        if m.group(3) is not None:
            out.add(int(m.group(3)))
        else:
            out.update(range(int(m.group(1)), int(m.group(2)) + 1))
    return out


class Ins:
    __slots__ = ("op", "args", "line", "asm", "lineno", "defs", "uses", "valu", "exec_w", "trans",
                 "dstsel", "dpp", "ws")

    def __init__(self, op, args, line, asm, lineno):
        self.op, self.args, self.line, self.asm, self.lineno = op, args, line, asm, lineno
        self.valu = op.startswith("v_")
        self.dpp = self.valu and (op.endswith("_dpp") or bool(DPP_RE.search(args)))
        self.trans = op.startswith(TRANS_OPS)
        self.ws = (int(args.strip(), 0) + 1) if op == "s_nop" else 1
        parts = [p.strip() for p in re.split(r",(?![^\[]*\])", args)] if args else []
        self.defs, self.uses = set(), set()
        if not parts:
            pass
        elif op.startswith(("global_store", "buffer_store", "flat_store", "scratch_store", "ds_write",
                            "ds_store", "global_atomic", "ds_add", "ds_max", "ds_min")) and "_rtn" not in op:
            for p in parts:
                self.uses |= vregs(p)
        elif op.startswith(("v_", "global_", "buffer_", "flat_", "scratch_", "ds_")):
            self.defs = vregs(parts[0])
            for p in parts[1:]:
                self.uses |= vregs(p)
            if op.startswith(("v_fmac", "v_mac", "v_dot2c", "v_pk_fmac")) or op.startswith("v_mfma"):
                self.uses |= self.defs  # tied accumulator (MFMA srcC may alias)
            if "v_cmpx" in op:
                self.exec_w = True
        else:
            for p in parts:
                self.uses |= vregs(p)
        self.exec_w = self.valu and ("v_cmpx" in op or (parts and parts[0] == "exec"))
        self.dstsel = self.valu and (op.startswith("v_fma_mixhi") or re.search(r"dst_sel:(WORD|BYTE)", args) is not None
                                     or re.search(r"op_sel:\[[01],[01],[01],1\]", args) is not None)


def parse(path, kfilter=None):
    kernels = []
    text = open(path).read()
    for m in re.finditer(r"\n(_Z\S+|[A-Za-z_]\w*):[^\n]*\n(.*?)\n\.Lfunc_end", text, re.S):
        name, body = m.group(1), m.group(2)
        if kfilter and kfilter not in name:
            continue
        if "s_endpgm" not in body:
            continue
        ins, labels, asm = [], {}, False
        base = text.count("\n", 0, m.start(2)) + 1
        for k, raw in enumerate(body.split("\n")):
            t = raw.split(";")[0].strip() if not raw.strip().startswith(";;#ASM") else raw.strip()
            if raw.strip().startswith(";;#ASMSTART"):
                asm = True
                continue
            if raw.strip().startswith(";;#ASMEND"):
                asm = False
                continue
            if not t or t.startswith("."):
                if t.startswith(".LBB") and t.endswith(":"):
                    labels[t[:-1]] = len(ins)
                continue
            if t.endswith(":"):
                labels[t[:-1]] = len(ins)
                continue
            sp = t.split(None, 1)
            ins.append(Ins(sp[0], sp[1] if len(sp) > 1 else "", t, asm, base + k))
        kernels.append((name, ins, labels))
    return kernels


def preds_of(ins, labels):
    at_label = {}
    for lab, idx in labels.items():
        at_label.setdefault(idx, []).append(lab)
    branch_to = {}
    for i, x in enumerate(ins):
        if x.op.startswith(("s_branch", "s_cbranch")):
            tgt = x.args.strip().split()[0] if x.args.strip() else ""
            if tgt in labels:
                branch_to.setdefault(labels[tgt], []).append(i)
    preds = []
    for i, x in enumerate(ins):
        p = []
        if i > 0 and not (ins[i - 1].op == "s_branch" or ins[i - 1].op == "s_endpgm"
                          or ins[i - 1].op.startswith("s_setpc")):
            p.append(i - 1)
        p += branch_to.get(i, [])
        preds.append(p)
    return preds


def walk_back(ins, preds, i, budget, hit):
    """Yield (index, waitstates_before_i) of instructions that can precede i within `budget` wait
    states; hit(j) is called for every such instruction, stopping that path when it returns True."""
    out = []
    seen = set()
    stack = [(p, 0) for p in preds[i]]
    while stack:
        j, ws = stack.pop()
        if (j, ws) in seen or ws >= budget:
            continue
        seen.add((j, ws))
        if hit(j, ws):
            out.append((j, ws))
            continue
        stack += [(p, ws + ins[j].ws) for p in preds[j]]
    return out


def check(path, kfilter=None, quiet=False):
    bad = 0
    for name, ins, labels in parse(path, kfilter):
        preds = preds_of(ins, labels)
        found = []
        for i, x in enumerate(ins):
            if x.dpp:
                need = x.uses
                for j, ws in walk_back(ins, preds, i, 2, lambda j, ws: bool(ins[j].defs & need)):
                    found.append(("DPP-VGPR", i, j, ws))
                for j, ws in walk_back(ins, preds, i, 5, lambda j, ws: ins[j].exec_w):
                    found.append(("DPP-EXEC", i, j, ws))
            if x.valu and not x.trans and x.uses:
                for j, ws in walk_back(ins, preds, i, 1, lambda j, ws: ins[j].trans and bool(ins[j].defs & x.uses)):
                    found.append(("TRANS", i, j, ws))
                for j, ws in walk_back(ins, preds, i, 1, lambda j, ws: ins[j].dstsel and bool(ins[j].defs & x.uses)):
                    found.append(("DSTSEL", i, j, ws))
        if found:
            bad += len(found)
            print(f"{path}: {name}: {len(found)} hazard(s)")
            if not quiet:
                for kind, i, j, ws in (found if "--all" in sys.argv else found[:40]):
                    a, b = ins[j], ins[i]
                    print(f"  {kind}: line {b.lineno} {'[asm] ' if b.asm else ''}{b.line}")
                    print(f"      after line {a.lineno} {'[asm] ' if a.asm else ''}{a.line}  ({ws} wait state(s) between)")
    return bad


def main():
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    kf = None
    if "--kernel" in sys.argv:
        kf = sys.argv[sys.argv.index("--kernel") + 1]
        args = [a for a in args if a != kf]
    quiet = "--quiet" in sys.argv
    total = sum(check(p, kf, quiet) for p in args)
    print(f"isa_hazards: {total} violation(s) in {len(args)} listing(s)")
    sys.exit(1 if total else 0)


if __name__ == "__main__":
    main()
