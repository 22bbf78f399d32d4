#!/usr/bin/env python3
"""bench.py -- ALS ratings/sec per full iteration, Netflix-shape k=64 fp32 on 1..8 MI355X (BASELINE.json).

  python bench.py [--gpus N] [--steps K] [--warmup W]
  python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 --master-port P \
      bench.py --gpus N --steps K --warmup W

A step = one full ALS iteration (movie half + RCCL all-gather + user half + RCCL all-gather) over the
synthetic Netflix-shape ratings (480,189 users x 17,770 movies x 1e8 ratings, k = 64, lambda = 0.05; seeded
generator). Inputs are resident in HBM before the timed region. The dataset is fixed as N grows
(strong scaling): users and movies are sharded by id % N, one process per GPU.

Prints ONE JSON line (rank 0). `roofline` covers the dominant kernel (the fused gather/Gram/solve launch of
each half) with the algorithmic bytes of SURVEY.md §8d, timed with HIP events on the stream the kernel is
launched on; `cpu_baseline` times the oracle's Java-float restatement of the reference hot path (the "port")
on a bounded sample of the same workload, rank 0 at N = 1 only.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0        # MI355X HBM3E spec (MI355X_MICROARCH.md)
FP32_PEAK_TFS = 157.3        # f32 vector = f32 MFMA dense peak


def half_bytes(nnz, n_rows, k, s=4):
    """SURVEY.md §8d algorithmic gather+Gram bytes of one half: factor row + col index + rating per entry,
    row_ptr, and the written factor rows."""
    return nnz * (s * k + 4 + 4) + 8 * (n_rows + 1) + s * k * n_rows


def half_flops(nnz, n_rows, k):
    return nnz * (k * k + 3 * k) + n_rows * (k ** 3 / 3 + 2 * k * k)


def cpu_baseline(ds, k, lam, seconds, threads):
    """The oracle's f32 (Java-float, EJML-order) restatement of MFeatureCalculator/UFeatureCalculator on a
    bounded random sample of rows of BOTH halves with equal rating counts R: ratings/s per full iteration =
    R / (t_movie_sample + t_user_sample)."""
    import numpy as np
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle   # checker / CPU baseline only
    oracle.build()
    rng = np.random.default_rng(1234)
    blocks = [ds.shard_block(0), ds.shard_block(1)]
    opp_f = [None, None]
    opp_f[0] = ds.init_user_factors(k, 42)                                      # movies read user factors
    opp_f[1] = rng.random((blocks[0]["n_rows"], k), dtype=np.float32)          # users read movie factors

    def sample(side, target):
        b = blocks[side]
        deg = np.diff(b["row_ptr"])
        order = rng.permutation(len(deg))
        csum = np.cumsum(deg[order])
        n = int(np.searchsorted(csum, target)) + 1
        rows = np.sort(order[:n])
        rp = np.zeros(n + 1, np.int64)
        np.cumsum(deg[rows], out=rp[1:])
        col = np.concatenate([b["col"][b["row_ptr"][r]:b["row_ptr"][r + 1]] for r in rows])
        rat = np.concatenate([b["ratings"][b["row_ptr"][r]:b["row_ptr"][r + 1]] for r in rows])
        side_obj = oracle.Side(ids=rows, row_ptr=rp, col=col, ratings=rat)
        return side_obj, int(rp[-1])

    def timed(target):
        t = 0.0
        got = []
        for side in (0, 1):
            s, r = sample(side, target)
            t0 = time.perf_counter()
            oracle.update_side(s, opp_f[side], lam, "f32", threads)
            t += time.perf_counter() - t0
            got.append(r)
        return t, min(got)

    target = 200_000
    t, r = timed(target)
    for _ in range(4):                      # grow the sample until it is ~`seconds` of CPU work
        if t >= 0.7 * seconds or target >= ds.nnz // 2:
            break
        target = int(min(ds.nnz // 2, target * seconds / max(t, 1e-3)))
        t, r = timed(target)
    return {"value": r / t, "unit": "ratings/s", "cores": threads, "kind": "port",
            "sample": f"oracle f32 (Java-float EJML-order restatement) on random rows of both halves, "
                      f"{r} ratings per half ({r / ds.nnz * 100:.2f}% of a half), {t:.1f} s, {threads} threads"}


def load_traffic():
    path = os.path.join(ROOT, "profiles", "traffic.json")
    if os.path.exists(path):
        try:
            return json.load(open(path))
        except Exception:
            return None
    return None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--k", type=int, default=64)
    ap.add_argument("--users", type=int, default=480_189)
    ap.add_argument("--movies", type=int, default=17_770)
    ap.add_argument("--nnz", type=int, default=100_000_000)
    ap.add_argument("--seed", type=int, default=0xA15)
    ap.add_argument("--lam", type=float, default=0.05)
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--overlap-chunks", type=int, default=4, help="user-half chunks per all-gather overlap (N > 1)")
    ap.add_argument("--rehearse-one-gpu", action="store_true",
                    help="N > 1 ranks all on cuda:0 over gloo: rehearses the multi-rank driver on a one-GPU box "
                         "(RCCL needs one GPU per rank); not a performance configuration")
    args = ap.parse_args()

    import numpy as np
    import torch
    import torch.distributed as dist
    import __graft_entry__
    cfk = __graft_entry__.load_package()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus and rank == 0:
        print(f"bench: WORLD_SIZE={world} but --gpus={args.gpus}; using WORLD_SIZE", file=sys.stderr)
    if args.rehearse_one_gpu:
        local = 0
    torch.cuda.set_device(local)
    if world > 1:
        if args.rehearse_one_gpu:
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=torch.device(f"cuda:{local}"))

    def barrier():
        if world > 1:
            dist.barrier()

    t_setup = time.perf_counter()
    ds = cfk.Dataset.synthetic_netflix(args.users, args.movies, args.nnz, args.seed, nthreads=min(16, os.cpu_count()))
    nm, nu, nnz = ds.counts()
    app = cfk.ALSApp(world, args.k, args.lam, args.steps, precision="f32", seed=42, device=local, rank=rank,
                     world_size=world, overlap_chunks=args.overlap_chunks).setup(ds, check_duplicates=False)
    t_setup = time.perf_counter() - t_setup

    for _ in range(args.warmup):
        app.iteration()
    torch.cuda.synchronize()
    barrier()
    app.engine.set_timing(True)
    barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        app.iteration()
    torch.cuda.synchronize()
    barrier()
    elapsed = time.perf_counter() - t0
    app.engine.set_timing(False)
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device="cpu" if args.rehearse_one_gpu else f"cuda:{local}")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    # per-kernel device time over the timed steps (HIP events on the launch stream)
    gm, rm, cm = app.engine.timing_collect("movie")
    gu, ru, cu = app.engine.timing_collect("user")
    mse = app.mse()

    if rank == 0:
        K = args.steps
        mi, ui = app.info[0], app.info[1]
        # algorithmic bytes of this rank's two halves (its shard), per step
        b_movie = half_bytes(mi["nnz"], mi["n_rows"], args.k)
        b_user = half_bytes(ui["nnz"], ui["n_rows"], args.k)
        t_main = (gm + gu) / 1000.0                       # s, main launches over K steps
        achieved = (b_movie + b_user) * K / t_main / 1e9 if t_main > 0 else None
        traffic = None
        tr = load_traffic()
        if tr and tr.get("k") == args.k and tr.get("nnz") == nnz and world == 1:
            traffic = tr.get("hbm_bytes_per_launch")
        flops = (half_flops(mi["nnz"], mi["n_rows"], args.k) + half_flops(ui["nnz"], ui["n_rows"], args.k)) * K
        roofline = {
            "bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": achieved / HBM_PEAK_GBS if achieved else None, "traffic": traffic,
            "kernel": "als_solve_mfma<64,2,split> (fused gather + split-bf16 MFMA Gram + in-wave tile LDL^T solve), main launch of each half",
            "algorithmic_bytes_per_launch": (b_movie + b_user) / 2,
            "avg_launch_ms": {"movie": gm / max(cm, 1), "user": gu / max(cu, 1)},
            "reduce_launch_ms": {"movie": rm / max(cm, 1), "user": ru / max(cu, 1)},
            "fp32_tflops": flops / t_main / 1e12 if t_main > 0 else None,
            "fp32_frac": flops / t_main / 1e12 / FP32_PEAK_TFS if t_main > 0 else None,
        }
        cpu = None
        if world == 1 and not args.no_cpu_baseline:
            cpu = cpu_baseline(ds, args.k, args.lam, args.cpu_seconds, min(16, os.cpu_count() or 1))
        value = nnz * K / elapsed
        line = {
            "metric": "ALS ratings/sec per full iteration, k=64 Netflix-shape, 1/2/4/8 MI355X",
            "value": value, "unit": "ratings/s", "n_gpus": world, "steps": K, "warmup": args.warmup,
            "ms_per_step": elapsed / K * 1000.0, "higher_is_better": True, "scaling": "strong",
            "vs_baseline": None, "dtype": "f32", "data": "synthetic (seeded Netflix-shape generator)",
            "config": {"workload": f"netflix-shape synthetic {nu} users x {nm} movies x {nnz} ratings, k={args.k}, "
                                   f"lambda={args.lam}, one step = one full ALS iteration",
                       "n_users": nu, "n_movies": nm, "nnz": nnz, "k": args.k, "lambda": args.lam,
                       "seed": args.seed, "partitions": world, "parallelism": f"id%{world} shards + RCCL all-gather"},
            "solves_per_s": (nm + nu) * K / elapsed,
            "mse_after": mse,
            "setup_s": t_setup,
            "roofline": roofline,
            "cpu_baseline": cpu,
        }
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
