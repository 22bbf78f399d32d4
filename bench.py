#!/usr/bin/env python3
"""bench.py -- ALS ratings/sec per full iteration, Netflix-shape k=64 fp32 on 1..8 MI355X (BASELINE.json).

  python bench.py [--gpus N] [--steps K] [--warmup W]
  python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 --master-port P \
      bench.py --gpus N --steps K --warmup W

A step = one full ALS iteration (movie half + RCCL all-gather + user half + RCCL all-gather) over the
synthetic Netflix-shape ratings (480,189 users x 17,770 movies x 1e8 ratings, k = 64, lambda = 0.05; seeded
generator). Inputs are resident in HBM before the timed region. The dataset is fixed as N grows
(strong scaling): users and movies are sharded by id % N, one process per GPU.

Prints ONE JSON line (rank 0). `roofline` describes the dominant kernel launch (the slower of the two halves'
fused gather/Gram/solve launches; both are under roofline.per_launch) with the algorithmic bytes of SURVEY.md
§8d, timed with HIP events on the stream the kernel is launched on; `cpu_baseline` times the oracle's
Java-float restatement of the reference hot path (the "port") on a bounded sample of the same workload, with
the reference's 4 stream threads (BaseKafkaApp.java:51) and with the box's CPU share, rank 0 at N = 1 only.
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
BF16_MFMA_PEAK_TFS = 2500.0  # dense bf16 MFMA peak (no sparsity)
MFMA_BF16_FLOP = 16 * 16 * 32 * 2   # one v_mfma_f32_16x16x32_bf16


def half_bytes(nnz, n_rows, k, s=4):
    """SURVEY.md §8d algorithmic gather+Gram bytes of one half: factor row + col index + rating per entry,
    row_ptr, and the written factor rows."""
    return nnz * (s * k + 4 + 4) + 8 * (n_rows + 1) + s * k * n_rows


def half_flops(nnz, n_rows, k):
    """Algorithmic Gram + RHS flops and solve flops of one half."""
    return nnz * (k * k + 3 * k), n_rows * (k ** 3 / 3 + 2 * k * k)


def mfma_per_block(kp, presplit):
    """v_mfma_f32_16x16x32_bf16 issued per 32-entry block by the split-bf16 Gram (als_kernels.hip): with C = kp/16
    feature blocks, every off-diagonal tile takes the six partial products hh, hm, mh, hl, lh, mm of the
    three-term split and every diagonal tile four (mm, hh and the folded hm + hl), plus 3 x C RHS MFMAs when
    the opposite table is pre-split (the RHS is a VALU FMA otherwise)."""
    c = kp // 16
    return 6 * (c * (c - 1) // 2) + 4 * c + (3 * c if presplit else 0)


def cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_baseline(ds, k, lam, seconds, thread_counts):
    """The oracle's f32 (Java-float, EJML-order) restatement of MFeatureCalculator/UFeatureCalculator on a
    bounded random sample of rows of BOTH halves with equal rating counts R: ratings/s per full iteration =
    R / (t_movie_sample + t_user_sample), once per thread count."""
    import numpy as np
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle   # checker / CPU baseline only
    oracle.build()
    rng = np.random.default_rng(1234)
    blocks = [ds.shard_block(0), ds.shard_block(1)]
    opp_f = [ds.init_user_factors(k, 42),                                        # movies read user factors
             rng.random((blocks[0]["n_rows"], k), dtype=np.float32)]            # users read movie factors

    def sample(side, target):
        b = blocks[side]
        deg = np.diff(b["row_ptr"])
        order = rng.permutation(len(deg))
        n = int(np.searchsorted(np.cumsum(deg[order]), target)) + 1
        rows = np.sort(order[:n])
        rp = np.zeros(n + 1, np.int64)
        np.cumsum(deg[rows], out=rp[1:])
        col = np.concatenate([b["col"][b["row_ptr"][r]:b["row_ptr"][r + 1]] for r in rows])
        rat = np.concatenate([b["ratings"][b["row_ptr"][r]:b["row_ptr"][r + 1]] for r in rows])
        return oracle.Side(ids=rows, row_ptr=rp, col=col, ratings=rat), int(rp[-1])

    def timed(target, threads):
        t, got = 0.0, []
        for side in (0, 1):
            s, r = sample(side, target)
            t0 = time.perf_counter()
            oracle.update_side(s, opp_f[side], lam, "f32", threads)
            t += time.perf_counter() - t0
            got.append(r)
        return t, min(got)

    runs = []
    for threads in thread_counts:
        target = 100_000
        t, r = timed(target, threads)
        for _ in range(4):                  # grow the sample until it is ~`seconds` of CPU work
            if t >= 0.7 * seconds or target >= ds.nnz // 2:
                break
            target = int(min(ds.nnz // 2, target * seconds / max(t, 1e-3)))
            t, r = timed(target, threads)
        runs.append({"threads": threads, "value": r / t, "ratings_per_half": r, "seconds": t})
    main = runs[0]
    return {"value": main["value"], "unit": "ratings/s", "cores": main["threads"], "kind": "port",
            "sample": f"oracle f32 (Java-float EJML-order restatement of MFeatureCalculator/UFeatureCalculator) on "
                      f"random rows of both halves, {main['ratings_per_half']} ratings per half "
                      f"({main['ratings_per_half'] / ds.nnz * 100:.2f}% of a half), {main['seconds']:.1f} s, "
                      f"{main['threads']} threads = the reference's NUM_STREAM_THREADS (BaseKafkaApp.java:51)",
            "runs": runs, "cpu_model": cpu_model(), "nproc": os.cpu_count(),
            "affinity_cpus": len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else None}


def load_traffic(k, nnz):
    path = os.path.join(ROOT, "profiles", "traffic.json" if k == 64 else f"traffic_k{k}.json")
    try:
        tr = json.load(open(path))
    except (OSError, ValueError):
        return None
    return tr if tr.get("k") == k and tr.get("nnz") == nnz else None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--k", type=int, default=64)
    ap.add_argument("--users", type=int, default=480_189)
    ap.add_argument("--movies", type=int, default=17_770)
    ap.add_argument("--nnz", type=int, default=100_000_000)
    ap.add_argument("--seed", type=int, default=0xA15)
    ap.add_argument("--lam", type=float, default=0.05)
    ap.add_argument("--cpu-seconds", type=float, default=7.0, help="CPU baseline seconds per thread count")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--overlap-chunks", type=int, default=4, help="user-half chunks per all-gather overlap (N > 1)")
    ap.add_argument("--rehearse-one-gpu", action="store_true",
                    help="N > 1 ranks all on cuda:0 over gloo: rehearses the multi-rank driver on a one-GPU box "
                         "(RCCL needs one GPU per rank); not a performance configuration")
    args = ap.parse_args()

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

    # per-half device time over the timed steps (HIP events on the launch stream), per half-iteration: with the
    # chunked user half (N > 1) one half is several launches, summed here
    K = args.steps
    eng = app.engine
    g_ms, r_ms = {}, {}
    for side in ("movie", "user"):
        g, r, _ = eng.timing_collect(side)
        g_ms[side], r_ms[side] = g / K, r / K
    mse = app.mse()

    if rank == 0:
        info = {"movie": app.info[0], "user": app.info[1]}
        tr = load_traffic(args.k, nnz) if world == 1 else None
        kp = eng.kp
        per = {}
        for si, side in enumerate(("movie", "user")):
            i = info[side]
            path = eng.block_path(si)
            blocks = eng.block_stats(si)["nnz_padded"] // 32
            dual = path.get("dual_rows_by_blocks", [0, 0, 0])
            main_blocks = blocks - sum((c + 1) * n for c, n in enumerate(dual))
            dual_mfma = sum(n * (cd * (cd + 1) // 2) * (kp // 32) * 6 for n, cd in zip(dual, (2, 4, 6)))
            b = half_bytes(i["nnz"], i["n_rows"], args.k)
            gram_f, solve_f = half_flops(i["nnz"], i["n_rows"], args.k)
            t_s = g_ms[side] / 1000.0
            mf = ((main_blocks * mfma_per_block(kp, path["presplit"]) + dual_mfma) * MFMA_BF16_FLOP
                  if path["gram_path"] == "mfma_split" else 0)
            achieved = b / t_s / 1e9
            per[side] = {
                "kernel": f"als_solve_mfma<{kp},{1 if kp == 128 else (3 if path['presplit'] else 2)},split,"
                          f"{'presplit' if path['presplit'] else 'on-the-fly split'}> + als_solve_dual (short rows)",
                "avg_launch_ms": g_ms[side], "reduce_launch_ms": r_ms[side],
                "algorithmic_bytes": b, "achieved": achieved, "frac": achieved / HBM_PEAK_GBS,
                "traffic": (tr or {}).get("per_side", {}).get(side),
                "alg_gram_tflops": gram_f / t_s / 1e12, "alg_solve_tflop_per_launch": solve_f / 1e12,
                "short_rows_entry_space": dual,
                # what bounds the launch (PMC passes in profiles/): the HBM fraction above is in
                # algorithmic bytes; the pre-split half reads an L2-resident table and is issue-bound instead
                "limit": ("issue: 64 MFMA + ~80 VALU per 32-entry block on one SIMD issue port, 3 waves/SIMD; "
                          "opposite table L2-resident (pre-split)") if path["presplit"] else
                         ("Infinity-Cache / fabric gather of the opposite factor rows" if kp <= 64 else
                          "HBM gather of the opposite factor rows + one-wave-per-SIMD solve"),
                "mfma_bf16": {"per_32_entry_block": mfma_per_block(kp, path["presplit"]),
                              "executed_tflops": mf / t_s / 1e12, "peak": BF16_MFMA_PEAK_TFS,
                              "frac": mf / t_s / 1e12 / BF16_MFMA_PEAK_TFS},
            }
        dom = max(per, key=lambda s: per[s]["avg_launch_ms"])
        d = per[dom]
        roofline = {
            "bound": "hbm", "achieved": d["achieved"], "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": d["frac"],
            "traffic": d["traffic"], "kernel": d["kernel"] + f" ({dom} half, the dominant launch)",
            "algorithmic_bytes_per_launch": d["algorithmic_bytes"], "avg_launch_ms": d["avg_launch_ms"],
            "both_halves": {"achieved": (per["movie"]["algorithmic_bytes"] + per["user"]["algorithmic_bytes"])
                            / ((g_ms["movie"] + g_ms["user"]) / 1000.0) / 1e9},
            "per_launch": per,
            "note": "achieved = SURVEY.md §8d algorithmic bytes / HIP-event launch time; traffic = PMC FETCH_SIZE x2 + "
                    "WRITE_SIZE per launch (profiles/traffic.json); mfma_bf16 = executed v_mfma_f32_16x16x32_bf16 "
                    "flops of the split Gram (each fp32 product = 3-term bf16 split: 6 partial products per "
                    "off-diagonal tile) against the dense bf16 peak",
        }
        cpu = None
        if world == 1 and not args.no_cpu_baseline:
            share = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
            share = min(share, int(os.environ.get("OMP_NUM_THREADS", "16") or 16), 16)
            cpu = cpu_baseline(ds, args.k, args.lam, args.cpu_seconds, [4] + ([share] if share != 4 else []))
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
