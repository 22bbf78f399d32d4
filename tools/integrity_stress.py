#!/usr/bin/env python3
"""Split-row hand-off stress on the full Netflix-shape workload (k = 64 by default).

Runs ITERS full iterations (movie half + user half) on ONE engine, rewriting U0 from the host every
REWRITE iterations (the pattern of the round-1 determinism failures), and checks the partial-slot integrity
record (SlotCodec, als_kernels.hip) every CHECK iterations. Every movie half after a U0 rewrite is also
compared bitwise with the first one. Prints one JSON line.

  ITERS=500 REWRITE=5 CHECK=10 python tools/integrity_stress.py [k]
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import numpy as np
    import torch
    import __graft_entry__
    cfk = __graft_entry__.load_package()
    k = int(sys.argv[1]) if len(sys.argv) > 1 else 64
    iters = int(os.environ.get("ITERS", "500"))
    rewrite = int(os.environ.get("REWRITE", "5"))
    check = int(os.environ.get("CHECK", "10"))
    lam = 0.05
    ds = cfk.Dataset.synthetic_netflix(480_189, 17_770, 100_000_000, 0xA15, nthreads=16)
    U0 = ds.init_user_factors(k, 42)
    eng = cfk.ALSEngine(k, "f32")
    for side in (0, 1):
        b = ds.shard_coo(side)
        eng.alloc_factors(side, b["n_slots"])
        eng.set_block_coo(side, b["n_rows"], b["rows"], b["cols"], b["ratings"], 0, ds.shard_info(1 - side)["n_slots"])
    first_m = None
    mismatches = []
    records = []
    t0 = time.time()
    for it in range(iters):
        fresh = it % rewrite == 0
        if fresh:
            eng.write_factors(1, U0)
        eng.solve_half(0, lam)
        if fresh:
            M = eng.read_factors(0)
            if first_m is None:
                first_m = M
            else:
                rows = np.nonzero(np.any(M != first_m, axis=1))[0]
                if len(rows):
                    mismatches.append({"iter": it, "rows": rows[:8].tolist(), "n": int(len(rows))})
        eng.solve_half(1, lam)
        if (it + 1) % check == 0:
            rec = eng.integrity_status(reset=True)
            if rec[0]:
                records.append({"iter": it, "record": rec})
                print(f"iter {it}: integrity record {rec}", flush=True)
        if (it + 1) % 50 == 0:
            print(f"iter {it + 1}/{iters} t={time.time() - t0:.1f}s bad_records={len(records)} "
                  f"mismatching_fresh_halves={len(mismatches)}", flush=True)
    torch.cuda.synchronize()
    stats = eng.block_stats(0)
    eng.close()
    print(json.dumps({"integrity_stress": {"k": k, "iters": iters, "rewrite_every": rewrite, "check_every": check,
                                           "movie_block": stats, "bad_records": records,
                                           "fresh_movie_half_mismatches": mismatches,
                                           "seconds": time.time() - t0}}), flush=True)


if __name__ == "__main__":
    main()
