#!/usr/bin/env python3
"""Cost of solving the user half in row-range chunks (the multi-GPU overlap path, app.py) on ONE GPU, without
any exchange: one shard of a G-way split of the Netflix-shape data, user half as one launch vs as C chunk
launches. The difference is what chunking adds to a rank's compute (launch tails), to weigh against the
all-gather time it hides.

  python tools/chunk_cost.py [--shards 8] [--chunks 1 2 4 8] [--k 64]
"""
import argparse
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shards", type=int, default=8)
    ap.add_argument("--chunks", type=int, nargs="+", default=[1, 2, 4, 8])
    ap.add_argument("--k", type=int, default=64)
    ap.add_argument("--reps", type=int, default=20)
    args = ap.parse_args()
    import torch
    import __graft_entry__
    cfk = __graft_entry__.load_package()
    ds = cfk.Dataset.synthetic_netflix(480_189, 17_770, 100_000_000, 0xA15, nthreads=16)
    G = args.shards
    out = {}
    for nc in args.chunks:
        app = cfk.ALSApp(G, args.k, 0.05, 1, precision="f32", seed=42, device=0, rank=0, world_size=G,
                         overlap_chunks=nc)
        # setup() shards for rank 0 of G; world_size > 1 makes it build the chunk plan, no collective is called
        app.setup(ds, check_duplicates=False)
        eng = app.engine
        S = app.info[1]["slots_per_shard"]

        def user_half():
            if app.chunk_slots is None:
                eng.solve_half(1, 0.05)
            else:
                for c in range(len(app.chunk_slots)):
                    eng.solve_half_chunk(1, 0.05, c)

        for _ in range(3):
            eng.solve_half(0, 0.05)
            user_half()
        torch.cuda.synchronize()
        ts = []
        for _ in range(args.reps):
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            user_half()
            b.record()
            torch.cuda.synchronize()
            ts.append(a.elapsed_time(b))
        out[nc] = {"median_ms": statistics.median(ts), "min_ms": min(ts), "chunks": len(app.chunk_slots or [0]),
                   "users": app.info[1]["n_rows"], "slots_per_shard": S}
        print(nc, json.dumps(out[nc]), flush=True)
        eng.close()
    print(json.dumps({"chunk_cost": out, "shards": G, "k": args.k}))


if __name__ == "__main__":
    main()
