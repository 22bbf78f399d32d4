#!/usr/bin/env python3
"""Instruction mix of one kernel in a hipcc -S listing, split at the last MFMA (Gram | solve).

  python tools/isa_mix.py listing.s <kernel-substring>
"""
import collections
import sys


def main():
    path, key = sys.argv[1], sys.argv[2]
    lines = open(path).read().split("\n")
    start = next(i for i, l in enumerate(lines) if l.startswith("_Z") and key in l.split(":")[0] and l.split(":")[0].endswith("E") or (l.startswith("_Z") and key in l and l.rstrip().endswith(l.split(":")[0].split()[0] + ":")))
    body = []
    for l in lines[start + 1:]:
        if l.startswith(".Lfunc_end"):
            break
        body.append(l)
    mf = [k for k, l in enumerate(body) if "v_mfma" in l]
    parts = {"gram": body[:mf[-1] + 1] if mf else [], "solve": body[mf[-1] + 1:] if mf else body}
    for name, part in parts.items():
        c = collections.Counter()
        for l in part:
            t = l.strip().split()
            if not t or t[0].startswith((";", ".")) or t[0].endswith(":"):
                continue
            c[t[0]] += 1
        cls = collections.Counter()
        for op, n in c.items():
            k = ("mfma" if "mfma" in op else "valu" if op.startswith("v_") else "salu" if op.startswith("s_")
                 else "lds" if op.startswith("ds_") else "vmem" if op.startswith(("global_", "buffer_", "scratch_")) else "other")
            cls[k] += n
        print(f"== {name}: {sum(c.values())} instr  {dict(cls)}")
        for op, n in c.most_common(25):
            print(f"   {op:28s} {n}")


if __name__ == "__main__":
    main()
