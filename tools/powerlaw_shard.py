#!/usr/bin/env python3
"""BASELINE configs[4] on one GPU: the per-GPU work of the 8-GPU power-law run (10M users x 1M items x 2B
ratings, k = 64, fp32), one id % G shard at a time.

Each rank of the G-GPU job holds the in-blocks of its shard of both sides and full replicas of both factor
matrices; its compute per iteration is a movie half over ~nnz/G ratings plus a user half over ~nnz/G ratings.
This tool builds exactly those blocks for the chosen shards on cuda:0, runs --steps full iterations per shard
(HIP-event device time of every launch), and prints one JSON line with the per-shard times; the G-GPU
iteration time is max over shards plus the exchange (reported separately: measured only by the driver's
multi-GPU run). Progress goes to stderr every step.

  python tools/powerlaw_shard.py [--users 10000000 --items 1000000 --nnz 2000000000] [--shards 0,3] [--G 8]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--users", type=int, default=10_000_000)
    ap.add_argument("--items", type=int, default=1_000_000)
    ap.add_argument("--nnz", type=int, default=2_000_000_000)
    ap.add_argument("--G", type=int, default=8)
    ap.add_argument("--shards", default="0")
    ap.add_argument("--k", type=int, default=64)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--seed", type=int, default=0xA15)
    args = ap.parse_args()
    import numpy as np
    import torch
    import __graft_entry__
    cfk = __graft_entry__.load_package()
    t0 = time.perf_counter()
    ds = cfk.Dataset.synthetic_powerlaw(args.users, args.items, args.nnz, args.seed, nthreads=16)
    log(f"generated {ds.counts()} in {time.perf_counter() - t0:.1f} s")
    G = args.G
    kp = cfk.factor_stride(args.k)
    u0 = ds.init_user_factors(args.k, 42, G)
    log(f"U0 ready ({time.perf_counter() - t0:.1f} s)")
    res = []
    for s in [int(x) for x in args.shards.split(",")]:
        t1 = time.perf_counter()
        eng = cfk.ALSEngine(args.k, "f32")
        eng.use_torch_stream()
        info = {}
        for side in (0, 1):
            blk = ds.shard_block(side, G, s)
            opp = ds.shard_info(1 - side, G, s)
            eng.alloc_factors(side, blk["n_slots"])
            eng.set_block(side, blk["row_ptr"], blk["col"], blk["ratings"], blk["row_offset"], opp["n_slots"])
            deg = np.diff(blk["row_ptr"])
            info[side] = {"rows": int(blk["n_rows"]), "nnz": int(blk["nnz"]), "max_row": int(deg.max()),
                          **eng.block_stats(side)}
            del blk
        eng.write_factors(1, u0)
        log(f"shard {s}: blocks in {time.perf_counter() - t1:.1f} s: {info}")
        eng.solve_half(0, 0.05)
        eng.solve_half(1, 0.05)
        torch.cuda.synchronize()
        eng.set_timing(True)
        for i in range(args.steps):
            eng.solve_half(0, 0.05)
            eng.solve_half(1, 0.05)
            torch.cuda.synchronize()
            log(f"shard {s}: step {i + 1}/{args.steps}")
        gm, rm, cm = eng.timing_collect(0)
        gu, ru, cu = eng.timing_collect(1)
        eng.close()
        ms = (gm + rm + gu + ru) / args.steps
        res.append({"shard": s, "ms_per_iteration": ms, "movie_ms": (gm + rm) / args.steps,
                    "user_ms": (gu + ru) / args.steps, "movie": info[0], "user": info[1],
                    "ratings_per_s_this_shard": (info[0]["nnz"] + info[1]["nnz"]) / 2 / (ms / 1e3)})
        log(json.dumps(res[-1]))
    worst = max(r["ms_per_iteration"] for r in res)
    print(json.dumps({"workload": f"powerlaw synthetic {args.users} users x {args.items} items x {args.nnz} ratings, "
                                  f"k={args.k}, fp32, shard(s) {args.shards} of G={G} on one MI355X",
                      "per_shard": res, "max_shard_ms_per_iteration": worst,
                      "G_gpu_ratings_per_s_compute_only": args.nnz / (worst / 1e3),
                      "note": f"exchange (RCCL all-gather of U {args.users * kp * 4 / 1e9:.2f} GB + M "
                              f"{args.items * kp * 4 / 1e9:.2f} GB per iteration) not included"}))


if __name__ == "__main__":
    main()
