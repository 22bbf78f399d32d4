#!/usr/bin/env python3
"""Bitwise determinism of the movie half on the full Netflix-shape workload: identical inputs solved repeatedly
(with the user half run in between, which reuses the shared partial-slot workspace) must give identical
factors. Variants are env settings applied at engine creation.

  [DET_K=128] python tools/determinism.py [VAR=VAL[,VAR=VAL]] ...
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
        for rep in range(3):
            eng.write_factors(1, U0)
            eng.solve_half(0, 0.05)
            Ms.append(eng.read_factors(0))
            if rep == 1:
                eng.solve_half(1, 0.05)      # the user half overwrites the shared partial slots
        for r in (1, 2):
            rows = np.nonzero(np.any(Ms[0] != Ms[r], axis=1))[0]
            print(f"{v}: movie rep0 vs rep{r}: {len(rows)} differing rows; degrees {deg[rows][:12].tolist()}; "
                  f"stats {eng.block_stats(0)}", flush=True)
        eng.close()


if __name__ == "__main__":
    main()
