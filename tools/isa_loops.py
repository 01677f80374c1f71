#!/usr/bin/env python3
"""Per-loop instruction census of one kernel in a gfx950 `.s` file (hipcc --save-temps).

Usage: tools/isa_loops.py <file.s> <kernel-substring> [--dump LOOPLABEL]

For every backward branch (a loop) it prints the body's instruction count by class
(VALU f64 / other VALU / SALU / VMEM load / VMEM store / LDS / DPP / waitcnt), the
instructions per iteration and, with --frames F, per frame.  This is the ISA
evidence behind DESIGN.md §4's per-kernel VALU floors.
"""
import re
import sys
from collections import Counter


def kernel_lines(path, sub):
    lines = open(path).read().split("\n")
    start = None
    for i, ln in enumerate(lines):
        if start is None and re.match(r"^_Z\S*:", ln) and sub in ln:
            start = i
        elif start is not None and ln.startswith("\t.size") and sub in ln:
            return lines[start:i]
    raise SystemExit(f"kernel {sub} not found")


def classify(op):
    if op.startswith("s_waitcnt"):
        return "waitcnt"
    if op.startswith(("global_load", "buffer_load", "flat_load", "scratch_load")):
        return "vmem_ld"
    if op.startswith(("global_store", "buffer_store", "flat_store", "scratch_store", "global_atomic")):
        return "vmem_st"
    if op.startswith("ds_"):
        return "lds"
    if op.startswith("s_"):
        return "salu"
    if op.startswith("v_"):
        if "_f64" in op or op.startswith(("v_cvt_f64", "v_cvt_f32_f64", "v_cvt_i32_f64")):
            return "valu_f64"
        return "valu"
    return "other"


def main():
    path, sub = sys.argv[1], sys.argv[2]
    dump = sys.argv[sys.argv.index("--dump") + 1] if "--dump" in sys.argv else None
    body = kernel_lines(path, sub)
    labels = {}
    insts = []  # (label_or_None, op, text)
    for ln in body:
        m = re.match(r"^(\.LBB\S+):", ln)
        if m:
            labels[m.group(1)] = len(insts)
            continue
        s = ln.strip()
        if not s or s.startswith((";", ".")):
            continue
        op = s.split()[0]
        insts.append((op, s))
    total = Counter(classify(op) for op, _ in insts)
    print(f"{sub}: {len(insts)} instructions, {dict(total)}")
    for i, (op, s) in enumerate(insts):
        if op.startswith("s_cbranch") or op == "s_branch":
            tgt = s.split()[-1]
            if tgt in labels and labels[tgt] <= i:
                lo = labels[tgt]
                c = Counter(classify(o) for o, _ in insts[lo:i + 1])
                dpp = sum(1 for o, t in insts[lo:i + 1] if "dpp" in t or "quad_perm" in t)
                v = c["valu"] + c["valu_f64"]
                print(f"  loop {tgt} [{lo}..{i}] {i + 1 - lo} inst: valu {v} (f64 {c['valu_f64']}, dpp {dpp}) "
                      f"salu {c['salu']} vmem_ld {c['vmem_ld']} vmem_st {c['vmem_st']} lds {c['lds']} "
                      f"waitcnt {c['waitcnt']}")
                if dump == tgt:
                    for o, t in insts[lo:i + 1]:
                        print("     ", t)


if __name__ == "__main__":
    main()
