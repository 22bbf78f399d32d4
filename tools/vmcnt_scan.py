#!/usr/bin/env python3
"""Static check of a kernel's straight-line regions for reads/writes of VGPRs that an outstanding vector load
will still write (RAW / WAW against the in-order vmcnt model).

  python tools/vmcnt_scan.py <file.s> <kernel symbol> [start_line end_line]

Walks the kernel's text in program order, keeping the list of issued-but-not-retired global/buffer loads
(retired oldest-first by `s_waitcnt vmcnt(N)`, all of them at labels/branches, which is conservative for a
loop body entered with vmcnt(0)), and reports every instruction that reads or writes a register one of them
will still write.
"""
import re
import sys


def regs(tok):
    m = re.fullmatch(r"v(\d+)", tok)
    if m:
        return {int(m.group(1))}
    m = re.fullmatch(r"v\[(\d+):(\d+)\]", tok)
    if m:
        return set(range(int(m.group(1)), int(m.group(2)) + 1))
    return set()


def main():
    path, sym = sys.argv[1], sys.argv[2]
    lines = open(path).read().split("\n")
    start = next(i for i, l in enumerate(lines) if l.startswith(sym + ":"))
    end = next(i for i in range(start, len(lines)) if lines[i].startswith(".Lfunc_end"))
    lo = int(sys.argv[3]) if len(sys.argv) > 3 else start
    hi = int(sys.argv[4]) if len(sys.argv) > 4 else end
    pending = []   # (line, dest regs)
    hits = 0
    for n in range(lo, hi):
        l = lines[n].split(";")[0].strip()
        if not l or l.startswith("."):
            if l.startswith(".LBB"):
                pending = []
            continue
        op = l.split()[0]
        ops = [t.strip() for t in l[len(op):].split(",")]
        ops = [t.split()[0] if t else t for t in ops]
        m = re.match(r"s_waitcnt.*vmcnt\((\d+)\)", l)
        if m:
            keep = int(m.group(1))
            if len(pending) > keep:
                pending = pending[len(pending) - keep:] if keep else []
            continue
        if op.startswith("s_cbranch") or op.startswith("s_branch"):
            continue
        if op.startswith(("global_load", "buffer_load")) and "lds" not in op:
            dst = regs(ops[0])
            for pl, pr in pending:
                if pr & dst:
                    print(f"{n + 1}: WAW load/load with line {pl + 1}: {l}")
                    hits += 1
            srcs = set().union(*[regs(t) for t in ops[1:]])
            for pl, pr in pending:
                if pr & srcs:
                    print(f"{n + 1}: RAW (address) with pending load line {pl + 1}: {l}")
                    hits += 1
            pending.append((n, dst))
            continue
        if op.startswith(("global_store", "buffer_store")):
            srcs = set().union(*[regs(t) for t in ops])
            dst = set()
        elif op.startswith(("s_", "ds_")) and not op.startswith("ds_"):
            continue
        else:
            dst = regs(ops[0]) if ops else set()
            srcs = set().union(*[regs(t) for t in ops[1:]]) if len(ops) > 1 else set()
        for pl, pr in pending:
            if pr & dst:
                print(f"{n + 1}: WAW with pending load line {pl + 1} ({lines[pl].strip()}): {l}")
                hits += 1
            if pr & srcs:
                print(f"{n + 1}: RAW with pending load line {pl + 1} ({lines[pl].strip()}): {l}")
                hits += 1
    print(f"{hits} hazards in lines {lo + 1}..{hi}")


if __name__ == "__main__":
    main()
