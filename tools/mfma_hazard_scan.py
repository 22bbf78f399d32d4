#!/usr/bin/env python3
"""Static scan of a hipcc -S listing for writes into the operand registers of an MFMA still in flight.

For every v_mfma instruction of one kernel, walk the following straight-line instructions (stop at a label) for
W wait states (one per instruction, N + 1 per s_nop N; MFMAs are skipped) and report a VALU / LDS / VMEM
instruction whose destination overlaps the MFMA's SrcA/SrcB, or its SrcC when SrcC != vDst (a true WAR: the
compiler treated the operand as read at issue). This is the pattern behind the split-Gram hazard fixed by
MFMA_DRAIN (als_kernels.hip); the scan lists candidates, it does not prove a hazard.

  hipcc --offload-arch=gfx950 -O3 -std=c++17 -I include -I <csrc> -S --cuda-device-only als_kernels.hip -o k.s
  python tools/mfma_hazard_scan.py k.s als_solve_mfmaILi64ELi2ELb1ELb0E [W=16]
"""
import collections
import re
import sys

REG = re.compile(r'([va])\[(\d+):(\d+)\]|([va])(\d+)\b')


def regs(op):
    m = REG.fullmatch(op.strip())
    if not m:
        return set()
    if m.group(1):
        return {(m.group(1), i) for i in range(int(m.group(2)), int(m.group(3)) + 1)}
    return {(m.group(4), int(m.group(5)))}


def kernel_body(lines, key):
    start = next(i for i, l in enumerate(lines)
                 if l.startswith("_Z") and key in l and l.split(";")[0].rstrip().endswith(":"))
    body = []
    for l in lines[start + 1:]:
        if l.startswith(".Lfunc_end"):
            break
        body.append(l)
    ins = []
    for l in body:
        t = l.strip()
        if not t or t.startswith((";", ".")) or t.split(";")[0].rstrip().endswith(":"):
            ins.append(("LABEL", []))
            continue
        op, _, rest = t.split(";")[0].partition(" ")
        ins.append((op, [o.strip() for o in rest.split(",")] if rest else []))
    return ins


def writes_vgpr(op):
    return op.startswith("v_") or "load" in op or op.startswith("ds_")


def scan(ins, window):
    hits = collections.Counter()
    examples = []
    for i, (op, ops) in enumerate(ins):
        if "v_mfma" not in op:
            continue
        dst, ab, c = regs(ops[0]), regs(ops[1]) | regs(ops[2]), regs(ops[3]) if len(ops) > 3 else set()
        ws = 0
        for j in range(i + 1, len(ins)):
            op2, ops2 = ins[j]
            if op2 == "LABEL":
                break
            if op2 == "s_nop":
                ws += int(ops2[0], 0) + 1
                continue
            if ws >= window:
                break
            ws += 1
            if "v_mfma" in op2 or not ops2 or not writes_vgpr(op2):
                continue
            d = regs(ops2[0])
            kind = "SrcC(!=vDst)" if d & (c - dst) else "SrcA/B" if d & ab else None
            if kind:
                hits[(op, kind)] += 1
                examples.append((ws, op, " ".join(ops), op2, " ".join(ops2[:2])))
                break
    return hits, examples


def main():
    path, key = sys.argv[1], sys.argv[2]
    window = int(sys.argv[3]) if len(sys.argv) > 3 else 16
    ins = kernel_body(open(path).read().split("\n"), key)
    hits, examples = scan(ins, window)
    print(f"{key}: {sum(hits.values())} candidate(s) within {window} wait states")
    for (op, kind), n in sorted(hits.items()):
        print(f"  {op:28s} {kind:14s} {n}")
    for e in examples[:8]:
        print(f"    +{e[0]:2d} ws  {e[1]} {e[2]}  <-  {e[3]} {e[4]}")


if __name__ == "__main__":
    main()
