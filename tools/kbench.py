#!/usr/bin/env python3
"""A/B kernel variants in ONE process with interleaved rounds (cdna_hip_programming.md §5.4 rule 24).

  python tools/kbench.py --variants "ALS_DUAL=1" "ALS_DUAL=0" [--rounds 5] [--nnz ...]
  CFK_ALS_LIB=collaborative-filtering-kafka_amd/build_debug/libcfk_als.so python tools/kbench.py \
      --variants "ALS_DEBUG_SKIP_SOLVE=0" "ALS_DEBUG_SKIP_SOLVE=1"   # Gram / solve split: debug build only

Each variant is a set of env settings read at engine creation / block upload. Prints per-variant median and
min device time (HIP events) of the main + reduce launches of each half on the Netflix-shape workload.
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
    args = ap.parse_args()
    import numpy as np
    import torch
    import __graft_entry__
    cfk = __graft_entry__.load_package()
    ds = cfk.Dataset.synthetic_netflix(args.users, args.movies, args.nnz, 0xA15, nthreads=16)
    blocks = [ds.shard_block(0), ds.shard_block(1)]
    kp = cfk.factor_stride(args.k)
    U = torch.zeros((blocks[1]["n_slots"] + 1, kp), dtype=torch.float32, device="cuda")
    M = torch.zeros((blocks[0]["n_slots"] + 1, kp), dtype=torch.float32, device="cuda")
    engines = []
    for v in args.variants:
        saved = dict(os.environ)
        for kv in v.split(","):
            if kv:
                k, val = kv.split("=")
                os.environ[k] = val
        eng = cfk.ALSEngine(args.k, "f32")
        eng.use_torch_stream()
        eng.bind_factors(0, M)
        eng.bind_factors(1, U)
        for side in (0, 1):
            b = blocks[side]
            eng.set_block(side, b["row_ptr"], b["col"], b["ratings"], 0, blocks[1 - side]["n_slots"])
        os.environ.clear()
        os.environ.update(saved)
        engines.append(eng)
    engines[0].write_factors(1, ds.init_user_factors(args.k, 42))
    for e in engines:        # warm up every variant
        e.solve_half(0, 0.05)
        e.solve_half(1, 0.05)
    torch.cuda.synchronize()
    res = {v: {"movie": [], "user": [], "movie_reduce": [], "user_reduce": []} for v in args.variants}
    for r in range(args.rounds):
        for v, e in zip(args.variants, engines):
            e.set_timing(True)
            e.solve_half(0, 0.05)
            e.solve_half(1, 0.05)
            torch.cuda.synchronize()
            gm, rm, _ = e.timing_collect(0)
            gu, ru, _ = e.timing_collect(1)
            e.set_timing(False)
            res[v]["movie"].append(gm)
            res[v]["user"].append(gu)
            res[v]["movie_reduce"].append(rm)
            res[v]["user_reduce"].append(ru)
    out = {}
    for v in args.variants:
        out[v] = {k: {"median_ms": statistics.median(x), "min_ms": min(x)} for k, x in res[v].items()}
        out[v]["total_median_ms"] = sum(out[v][k]["median_ms"] for k in ("movie", "user", "movie_reduce", "user_reduce"))
        print(v, json.dumps(out[v]), flush=True)
    print(json.dumps({"kbench": out, "nnz": args.nnz, "k": args.k}))


if __name__ == "__main__":
    main()
