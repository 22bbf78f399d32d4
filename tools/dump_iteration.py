#!/usr/bin/env python3
"""Factors after one full iteration (movie half, then user half) on the seeded Netflix-shape workload, saved for a
bitwise comparison of two library builds (CFK_ALS_LIB selects the build):

  CFK_ALS_LIB=.../build_x/libcfk_als.so python tools/dump_iteration.py --k 128 --out gpurun_out/x.npz
  python tools/dump_iteration.py --compare gpurun_out/a.npz gpurun_out/b.npz
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--k", type=int, default=128)
    ap.add_argument("--nnz", type=int, default=100_000_000)
    ap.add_argument("--out")
    ap.add_argument("--compare", nargs=2)
    args = ap.parse_args()
    import numpy as np
    if args.compare:
        a, b = (np.load(p) for p in args.compare)
        ok = True
        for side in ("M", "U"):
            x, y = a[side], b[side]
            diff = np.flatnonzero((x.view(np.uint32) != y.view(np.uint32)).any(axis=1))
            rel = float(np.max(np.abs(x - y)) / max(np.max(np.abs(x)), 1e-30))
            print(f"{side}: {len(diff)} of {len(x)} rows differ bitwise, max abs diff / max abs = {rel:.3e}")
            ok &= len(diff) == 0
        print("BITWISE EQUAL" if ok else "DIFFERENT")
        return 0 if ok else 1
    import __graft_entry__
    cfk = __graft_entry__.load_package()
    ds = cfk.Dataset.synthetic_netflix(480_189, 17_770, args.nnz, 0xA15, nthreads=16)
    eng = cfk.ALSEngine(args.k, "f32")
    for side in (0, 1):
        b = ds.shard_coo(side)
        eng.alloc_factors(side, b["n_slots"])
        eng.set_block_coo(side, b["n_rows"], b["rows"], b["cols"], b["ratings"], 0, ds.shard_info(1 - side)["n_slots"])
    eng.write_factors(1, ds.init_user_factors(args.k, 42))
    eng.solve_half(0, 0.05)
    eng.solve_half(1, 0.05)
    M, U = eng.read_factors(0), eng.read_factors(1)
    st = eng.integrity_status()
    np.savez(args.out, M=M, U=U)
    print(f"saved {args.out}: M {M.shape} U {U.shape}, integrity {st}")
    return 0


if __name__ == "__main__":
    sys.exit(main())
