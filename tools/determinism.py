#!/usr/bin/env python3
"""Bitwise determinism of the movie half on the full Netflix-shape workload: identical inputs solved repeatedly
(with the user half run in between, which reuses the shared partial-slot workspace) must give identical
factors. Variants are env settings applied at engine creation.

  [DET_K=128] [DET_REPS=3] [DET_USER_REPS=40] python tools/determinism.py [VAR=VAL[,VAR=VAL]] ...
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import numpy as np
    import torch
    import __graft_entry__
    cfk = __graft_entry__.load_package()
    ds = cfk.Dataset.synthetic_netflix(480_189, 17_770, 100_000_000, 0xA15, nthreads=16)
    k = int(os.environ.get("DET_K", "64"))
    U0 = ds.init_user_factors(k, 42)
    deg = np.diff(ds.shard_block(0)["row_ptr"])
    for v in (sys.argv[1:] or ["DEFAULT=1"]):
        saved = dict(os.environ)
        for kv in v.split(","):
            a, c = kv.split("=")
            os.environ[a] = c
        eng = cfk.ALSEngine(k, "f32")
        eng.use_torch_stream()
        for side in (0, 1):
            b = ds.shard_coo(side)
            eng.alloc_factors(side, b["n_slots"])
            eng.set_block_coo(side, b["n_rows"], b["rows"], b["cols"], b["ratings"], 0, ds.shard_info(1 - side)["n_slots"])
        os.environ.clear()
        os.environ.update(saved)
        Ms = []
        reps = int(os.environ.get("DET_REPS", "3"))
        for rep in range(reps):
            eng.write_factors(1, U0)
            eng.solve_half(0, 0.05)
            Ms.append(eng.read_factors(0))
            if rep == 1 or os.environ.get("DET_USER_EVERY_REP"):
                eng.solve_half(1, 0.05)      # the user half overwrites the shared partial slots
        blk0 = ds.shard_block(0)

        def fp64_err(i, x):
            # fp64 restatement of the movie update for row i (MFeatureCalculator.java:82-99) from U0
            cols = blk0["col"][blk0["row_ptr"][i]:blk0["row_ptr"][i + 1]]
            Y = U0[cols, :k].astype(np.float64)
            r = blk0["ratings"][blk0["row_ptr"][i]:blk0["row_ptr"][i + 1]].astype(np.float64)
            A = Y.T @ Y + np.float64(np.float32(0.05)) * len(cols) * np.eye(k)
            ref = np.linalg.solve(A, Y.T @ r)
            return float(np.max(np.abs(x[:k] - ref)) / np.max(np.abs(ref)))

        for r in range(1, reps):
            bad = np.nonzero(np.any(Ms[0] != Ms[r], axis=1))[0][:4]
            if len(bad):
                print(f"  vs fp64: rep0 {[fp64_err(i, Ms[0][i]) for i in bad]} rep{r} {[fp64_err(i, Ms[r][i]) for i in bad]}",
                      flush=True)
            rows = np.nonzero(np.any(Ms[0] != Ms[r], axis=1))[0]
            rel = [float(np.max(np.abs(Ms[0][i] - Ms[r][i])) / max(float(np.max(np.abs(Ms[0][i]))), 1e-30))
                   for i in rows[:12]]
            print(f"{v}: movie rep0 vs rep{r}: {len(rows)} differing rows {rows[:12].tolist()} rel {rel}; "
                  f"degrees {deg[rows][:12].tolist()}; "
                  f"stats {eng.block_stats(0)}", flush=True)
        ureps = int(os.environ.get("DET_USER_REPS", "0"))
        if ureps:
            # the user half repeated on the same movie factors (the pre-split, 3-wave path at k = 64): every
            # repetition must reproduce the first bitwise
            U_first, bad = None, []
            for rep in range(ureps):
                eng.solve_half(1, 0.05)
                U = eng.read_factors(1)
                if U_first is None:
                    U_first = U
                else:
                    bad.append(int(np.count_nonzero(np.any(U != U_first, axis=1))))
            print(f"{v}: user half x{ureps}: differing rows per repetition {bad}; total {sum(bad)}", flush=True)
        eng.close()


if __name__ == "__main__":
    main()
