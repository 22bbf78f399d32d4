#!/usr/bin/env python3
"""A/B kernel variants in ONE process with interleaved rounds (cdna_hip_programming.md §5.4 rule 24).

  python tools/kbench.py --variants "ALS_DUAL=1" "ALS_DUAL=0" [--rounds 5] [--nnz ...]
  CFK_ALS_LIB=collaborative-filtering-kafka_amd/build_debug/libcfk_als.so python tools/kbench.py \
      --variants "ALS_DEBUG_SKIP_SOLVE=0" "ALS_DEBUG_SKIP_SOLVE=1"   # Gram / solve split: debug build only

Each variant is a set of env settings read at engine creation / block upload. Prints per-variant median and
min device time (HIP events) of the main + reduce launches of each half on the Netflix-shape workload. Every
timed half starts from the same snapshot of real factor tables (two iterations from the seeded U0).
"""
from __future__ import annotations

import argparse
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--variants", nargs="+", default=["ALS_DUAL=1"])
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--k", type=int, default=64)
    ap.add_argument("--users", type=int, default=480_189)
    ap.add_argument("--movies", type=int, default=17_770)
    ap.add_argument("--nnz", type=int, default=100_000_000)
    ap.add_argument("--shard-of", type=int, default=1, help="G > 1: shard 0 of G (one rank's blocks, bench --shard-of)")
    args = ap.parse_args()
    import numpy as np
    import torch
    import __graft_entry__
    cfk = __graft_entry__.load_package()
    G = args.shard_of
    if G > 1:
        ds = cfk.Dataset.synthetic_shard("netflix", args.users, args.movies, args.nnz, 0xA15, G, 0, nthreads=16)
    else:
        ds = cfk.Dataset.synthetic_netflix(args.users, args.movies, args.nnz, 0xA15, nthreads=16)
    blocks = [ds.shard_block(0, G, 0), ds.shard_block(1, G, 0)]
    kp = cfk.factor_stride(args.k)

    def tables():
        return (torch.zeros((blocks[0]["n_slots"] + 1, kp), dtype=torch.float32, device="cuda"),
                torch.zeros((blocks[1]["n_slots"] + 1, kp), dtype=torch.float32, device="cuda"))

    def make_engine(env, M, U):
        saved = dict(os.environ)
        for kv in env.split(","):
            if kv:
                k, val = kv.split("=")
                os.environ[k] = val
        eng = cfk.ALSEngine(args.k, "f32")
        eng.use_torch_stream()
        eng.bind_factors(0, M)
        eng.bind_factors(1, U)
        for side in (0, 1):
            b = blocks[side]
            eng.set_block(side, b["row_ptr"], b["col"], b["ratings"], b["row_offset"], blocks[1 - side]["n_slots"])
        os.environ.clear()
        os.environ.update(saved)
        return eng

    # Canonical input state: two real iterations from the seeded U0 on a plain engine. Every timed half of every
    # variant starts from this snapshot in the variant's own tables, so a work-dropping variant (debug SKIP_SOLVE)
    # never feeds its garbage to another half, and every variant's MFMAs see the same data (MFMA power, and
    # so the clock, depends on the operand values).
    Ms, Us = tables()
    ref = make_engine("", Ms, Us)
    ref.write_factors(1, ds.init_user_factors(args.k, 42, G))
    for _ in range(2):
        ref.solve_half(0, 0.05)
        ref.solve_half(1, 0.05)
    torch.cuda.synchronize()
    del ref
    engines = []
    for v in args.variants:
        M, U = tables()
        engines.append((make_engine(v, M, U), M, U))
    res = {v: {"movie": [], "user": [], "movie_reduce": [], "user_reduce": []} for v in args.variants}
    for r in range(args.rounds + 1):   # round 0: warm-up
        for v, (e, M, U) in zip(args.variants, engines):
            e.set_timing(True)
            for side in (0, 1):
                M.copy_(Ms)
                U.copy_(Us)
                e.solve_half(side, 0.05)
            torch.cuda.synchronize()
            gm, rm, _ = e.timing_collect(0)
            gu, ru, _ = e.timing_collect(1)
            e.set_timing(False)
            if r == 0:
                continue
            res[v]["movie"].append(gm)
            res[v]["user"].append(gu)
            res[v]["movie_reduce"].append(rm)
            res[v]["user_reduce"].append(ru)
    # results of each variant's halves (both from the snapshot) against the first variant's
    outs = []
    for v, (e, M, U) in zip(args.variants, engines):
        res_v = []
        for side in (0, 1):
            M.copy_(Ms)
            U.copy_(Us)
            e.solve_half(side, 0.05)
            torch.cuda.synchronize()
            res_v.append((M if side == 0 else U).clone())
        outs.append(res_v)
    diffs = {}
    for v, r in zip(args.variants, outs):
        d = {}
        for side, name in ((0, "movie"), (1, "user")):
            ref_t, t = outs[0][side], r[side]
            d[name] = {"bitwise_equal": bool(torch.equal(ref_t, t)),
                       "max_abs_over_max": float((t - ref_t).abs().max() / ref_t.abs().max().clamp_min(1e-30)),
                       "finite": bool(torch.isfinite(t).all())}
        diffs[v] = d
        print("vs", args.variants[0], ":", v, json.dumps(d), flush=True)
    out = {}
    for v in args.variants:
        out[v] = {k: {"median_ms": statistics.median(x), "min_ms": min(x)} for k, x in res[v].items()}
        out[v]["total_median_ms"] = sum(out[v][k]["median_ms"] for k in ("movie", "user", "movie_reduce", "user_reduce"))
        print(v, json.dumps(out[v]), flush=True)
    print(json.dumps({"kbench": out, "nnz": args.nnz, "k": args.k, "diffs": diffs}))


if __name__ == "__main__":
    main()
