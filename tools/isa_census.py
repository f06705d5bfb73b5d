#!/usr/bin/env python3
"""Opcode-class census of one kernel's main loop from hipcc device assembly (tools only).

Usage: isa_census.py <kernel.s> [--path L1,L2,...]
  Prints every basic block of the function with its instruction counts per class and its
  successors; with --path, sums the classes over the listed blocks (the path one wave takes
  through one frame), counting each listed block once per occurrence.
Classes:
  fp32     f32 add/sub/mul/fma/fmac/fmamk/fmaak (VOP2/VOP3, DPP forms included), v_pk_* f32
  int_dft  integer butterflies of the first forward pass (v_add/sub_u32 with SDWA word selects
           and the plain int adds/subs that combine them)
  cvt      v_cvt_*
  mov      v_mov_b32 (incl. DPP movs), v_swap, v_permlane
  sel      v_cndmask
  addr     other VALU integer ops (shifts, and/or/xor, bitop3, bfe, lshl_add, mad_u32, ...)
  rfl      v_readfirstlane / v_readlane / v_writelane
  salu     s_* except waits, barrier, branches, nop
  lds      ds_*
  vmem     buffer_* / global_*
  ctl      s_waitcnt, s_barrier, s_nop, branches, s_setprio
"""
import re
import sys
from collections import Counter, OrderedDict

FP = re.compile(r"^v_(pk_)?(add|sub|subrev|mul|fma|fmac|fmamk|fmaak|mac|madmk|madak)_f32")


def classify(op, line):
    if op.startswith("v_"):
        if FP.match(op):
            return "fp32"
        if op.startswith("v_cvt"):
            return "cvt"
        if op.startswith(("v_mov", "v_swap", "v_permlane")):
            return "mov"
        if op.startswith("v_cndmask"):
            return "sel"
        if op.startswith(("v_readfirstlane", "v_readlane", "v_writelane")):
            return "rfl"
        if op.startswith(("v_add_u32", "v_sub_u32", "v_subrev_u32")) and ("sdwa" in op or "sext(" in line):
            return "int_dft"
        return "addr"
    if op.startswith("ds_"):
        return "lds"
    if op.startswith(("buffer_", "global_", "flat_")):
        return "vmem"
    if op.startswith(("s_waitcnt", "s_barrier", "s_nop", "s_branch", "s_cbranch", "s_setprio", "s_endpgm")):
        return "ctl"
    if op.startswith("s_"):
        return "salu"
    return "other"


def parse(path):
    blocks = OrderedDict()
    cur = "ENTRY"
    blocks[cur] = {"ops": [], "succ": []}
    order = [cur]
    for raw in open(path):
        line = raw.split(";")[0].rstrip()
        if not line.strip():
            m = re.match(r"^; %bb\.(\d+):", raw)
            if m:
                nxt = "bb." + m.group(1)
                blocks[cur]["succ"].append(nxt)
                cur = nxt
                blocks[cur] = {"ops": [], "succ": []}
                order.append(cur)
            continue
        m = re.match(r"^(\.LBB\w+):", line)
        if m:
            nxt = m.group(1)
            if blocks[cur]["ops"] and not blocks[cur]["ops"][-1][0].startswith("s_branch"):
                blocks[cur]["succ"].append(nxt)
            elif not blocks[cur]["ops"]:
                blocks[cur]["succ"].append(nxt)
            cur = nxt
            blocks[cur] = {"ops": [], "succ": []}
            order.append(cur)
            continue
        s = line.strip()
        if s.startswith(".") or s.endswith(":"):
            continue
        op = s.split()[0]
        blocks[cur]["ops"].append((op, s))
        if op.startswith(("s_branch", "s_cbranch")):
            blocks[cur]["succ"].append(s.split()[-1])
    return blocks, order


def census(ops):
    c = Counter()
    for op, s in ops:
        c[classify(op, s)] += 1
        if op.endswith("_e64") or ("_dpp" not in op and op.startswith("v_fma_f32")):
            c["(vop3)"] += 1
        if "_dpp" in op:
            c["(dpp)"] += 1
    return c


CLS = ["fp32", "int_dft", "cvt", "mov", "sel", "addr", "rfl", "salu", "lds", "vmem", "ctl", "other", "(vop3)", "(dpp)"]


def main():
    path = sys.argv[1]
    blocks, order = parse(path)
    want = None
    if "--path" in sys.argv:
        want = sys.argv[sys.argv.index("--path") + 1].split(",")
    if want is None:
        print("block".ljust(12) + "".join(k.rjust(8) for k in CLS) + "  succ")
        for b in order:
            c = census(blocks[b]["ops"])
            print(b.ljust(12) + "".join(str(c[k]).rjust(8) for k in CLS) + "  " + ",".join(blocks[b]["succ"]))
        return
    tot = Counter()
    for b in want:
        tot += census(blocks[b]["ops"])
    valu = sum(tot[k] for k in ["fp32", "int_dft", "cvt", "mov", "sel", "addr", "rfl"])
    print("path:", ",".join(want))
    for k in CLS:
        print(f"  {k:8s} {tot[k]:6d}" + (f"  ({100.0 * tot[k] / valu:5.1f} % of VALU)" if k in
                                           ["fp32", "int_dft", "cvt", "mov", "sel", "addr", "rfl"] else ""))
    print(f"  VALU     {valu:6d}")


if __name__ == "__main__":
    main()
