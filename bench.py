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
fused gather/Gram/solve launches; both are under roofline.per_launch), timed with HIP events on the stream the
kernel is launched on. Its `bound` is the launch's real limiter, from the rocprofv3 counters of the same build
(profiles/counters_k<k>.json, written by tools/prof_summary.py from a profiles/r03*/ pass): the pre-split user
half (LDS-DMA rows, transposed-read operands, no split VALU) and every KP = 128 launch are bound by the MFMA pipe
(achieved = the split-bf16 Gram's MFMA flops as issued, against the dense bf16 peak; gram_phase = the same over the
Gram's cycle share from the counters), the on-the-fly-split movie half at k = 64 by the fabric gather of the
opposite rows (counter bytes / time against the Infinity-Cache gather ceiling). The SURVEY.md §8d algorithmic-byte fraction
stays as a secondary field (cache-served gathers included, so it can exceed 1). `cpu_baseline` times the
oracle's Java-float restatement of the reference hot path (the "port", one C call per sampled half) on a bounded
sample of the same workload with the reference's 4 stream threads (BaseKafkaApp.java:51), the box's CPU share
and all `nproc` CPUs, rank 0 at N = 1 only.
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
# MI355X_MICROARCH.md "Indexed rows: gather into LDS": uniformly random rows of a 151 MB table (the 123 MB k = 64
# user table the movie half gathers sits between its 38 MB and 151 MB rows) are served at 7.4-7.9 TB/s chip-wide;
# rows every workgroup shares from the XCD's L2 (the 6.8 MB pre-split movie table of the user half: 91% L2 hits)
# at 16.8-18.8 TB/s
IC_GATHER_CEILING_GBS = 7900.0
L2_GATHER_CEILING_GBS = 18800.0
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
            "sample": f"oracle f32 (Java-float EJML-order restatement of MFeatureCalculator/UFeatureCalculator, "
                      f"oracle/als_oracle.c, ONE C call per half over the sampled rows) on uniformly random rows of "
                      f"both halves, {main['ratings_per_half']} ratings per half "
                      f"({main['ratings_per_half'] / ds.nnz * 100:.2f}% of a half), {main['seconds']:.1f} s, "
                      f"{main['threads']} threads = the reference's NUM_STREAM_THREADS (BaseKafkaApp.java:51). "
                      f"Representative: a row costs deg k^2 + k^3 / 3 flops, and rows drawn uniformly carry the "
                      f"half's own degree mix, so ratings / s over the sample estimates the full half's rate",
            "runs": runs, "cpu_model": cpu_model(), "nproc": os.cpu_count(),
            "affinity_cpus": len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else None}


def load_counters(k, nnz):
    """Per-launch rocprofv3 counters of this build at (k, nnz): profiles/counters_k<k>.json (tools/prof_summary.py)."""
    path = os.path.join(ROOT, "profiles", f"counters_k{k}.json")
    try:
        c = json.load(open(path))
    except (OSError, ValueError):
        return None
    return c if c.get("k") == k and c.get("nnz") == nnz else None


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
    ap.add_argument("--exchange", choices=("torch", "native"), default="torch",
                    help="N > 1: all-gathers through torch.distributed (RCCL) or through the engine's own RCCL "
                         "communicator behind the C ABI (als_comm_init / als_allgather_shard, the path a JNI caller "
                         "binds)")
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
    exchange = args.exchange if world > 1 and not args.rehearse_one_gpu else "torch"
    app = cfk.ALSApp(world, args.k, args.lam, args.steps, precision="f32", seed=42, device=local, rank=rank,
                     world_size=world, overlap_chunks=args.overlap_chunks,
                     exchange=exchange).setup(ds, check_duplicates=False)
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
        ctr = load_counters(args.k, nnz) if world == 1 else None
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
            c = (ctr or {}).get("per_side", {}).get(side, {})
            # bytes the launch requests from the memory hierarchy: the gathered opposite rows (pre-split: 384 B of
            # bf16 h/m/l pieces per padded entry; fp32 otherwise, also for the entry-space rows), column indices,
            # ratings (bf16 pairs on the pre-split path) and the written factor rows
            dual_entries = sum(32 * (c_ + 1) * n for c_, n in enumerate(dual))
            main_entries = main_blocks * 32
            row_b = 6 * kp if path["presplit"] else 4 * kp   # pre-split: bf16 h/m/l planes
            gathered = (main_entries * (row_b + 4 + (2 if path["presplit"] else 4)) + dual_entries * (4 * kp + 8)
                        + 4 * kp * i["n_rows"])
            d = {
                "kernel": f"als_solve_mfma<{kp},{1 if kp == 128 else (3 if path['presplit'] else 2)},split,"
                          f"{'presplit' if path['presplit'] else 'on-the-fly split'}> + als_solve_dual (short rows)",
                "avg_launch_ms": g_ms[side], "reduce_launch_ms": r_ms[side],
                "gathered_bytes": gathered,
                "mfma_bf16": {"per_32_entry_block": mfma_per_block(kp, path["presplit"]),
                              "flop_per_launch": mf, "executed_tflops": mf / t_s / 1e12, "peak": BF16_MFMA_PEAK_TFS,
                              "frac": mf / t_s / 1e12 / BF16_MFMA_PEAK_TFS},
                "algorithmic_bytes": {"bytes": b, "achieved_gbs": b / t_s / 1e9, "frac_of_hbm": b / t_s / 1e9 / HBM_PEAK_GBS,
                                      "note": "SURVEY.md §8d algorithmic bytes / launch time; cache-served gathers "
                                              "included, so it can exceed 1: not a bound"},
                "algorithmic_fp32": {"gram_flop": gram_f, "solve_flop": solve_f,
                                     "tflops": (gram_f + solve_f) / t_s / 1e12, "fp32_peak": FP32_PEAK_TFS},
                "short_rows_entry_space": dual,
            }
            if c:
                d["counters"] = c
                d["traffic"] = c.get("hbm_bytes")
            if kp <= 64 and not path["presplit"]:
                # the fabric gather of the opposite factor rows: L2 misses served by the Infinity Cache / HBM
                fab = c.get("hbm_bytes")
                d.update(bound="gather (Infinity Cache)", unit="GB/s", peak=IC_GATHER_CEILING_GBS,
                         achieved=(fab / t_s / 1e9) if fab else None,
                         limit="fabric gather of the opposite factor rows: PMC FETCH x2 + WRITE bytes / launch time "
                               "against the Infinity-Cache random-row gather ceiling (MI355X_MICROARCH.md)")
            elif path["presplit"]:
                # the pre-split Gram issues no split VALU (rows reach LDS by DMA, operands come back by transposed
                # reads): its limiter is the MFMA pipe; the solve phase after it is latency-bound (counters)
                d.update(bound="mfma", unit="TFLOP/s", peak=BF16_MFMA_PEAK_TFS, achieved=mf / t_s / 1e12,
                         limit="MFMA pipe: the split-bf16 Gram's v_mfma_f32_16x16x32_bf16 flops as issued (whole launch, "
                               "solve phase included) against the dense bf16 peak; gram_phase = the same flops over the "
                               "Gram's share of the launch cycles (counters.gram_only.cycles_frac); "
                               "counters.mfma_busy_frac = measured pipe-busy share at the sustained clock")
                gf = c.get("gram_only", {}).get("cycles_frac")
                if gf:
                    d["gram_phase"] = {"achieved_tflops": mf / (t_s * gf) / 1e12,
                                       "frac": mf / (t_s * gf) / 1e12 / BF16_MFMA_PEAK_TFS,
                                       "mfma_busy_frac": c.get("gram_only", {}).get("mfma_busy_frac")}
                d["gather_l2"] = {"achieved_gbs": gathered / t_s / 1e9, "peak": L2_GATHER_CEILING_GBS,
                                  "frac": gathered / t_s / 1e9 / L2_GATHER_CEILING_GBS}
            else:
                d.update(bound="mfma", unit="TFLOP/s", peak=BF16_MFMA_PEAK_TFS, achieved=mf / t_s / 1e12,
                         limit="MFMA pipe at one wave per SIMD: the split-bf16 Gram's v_mfma_f32_16x16x32_bf16 flops "
                               "as issued against the dense bf16 peak; counters.mfma_busy_frac = pipe-busy share")
            d["frac"] = d["achieved"] / d["peak"] if d.get("achieved") else None
            per[side] = d
        dom = max(per, key=lambda s: per[s]["avg_launch_ms"])
        d = per[dom]
        roofline = {
            "bound": "mfma" if d["bound"] == "mfma" else "hbm", "limiter": d["bound"],
            "achieved": d["achieved"], "peak": d["peak"],
            "unit": d["unit"], "frac": d["frac"], "traffic": d.get("traffic"),
            "kernel": d["kernel"] + f" ({dom} half, the dominant launch)", "limit": d["limit"],
            "avg_launch_ms": d["avg_launch_ms"], "counters": d.get("counters"), "gram_phase": d.get("gram_phase"),
            "algorithmic_bytes_frac": d["algorithmic_bytes"]["frac_of_hbm"],
            "both_halves_algorithmic_gbs": (per["movie"]["algorithmic_bytes"]["bytes"] +
                                            per["user"]["algorithmic_bytes"]["bytes"])
                                           / ((g_ms["movie"] + g_ms["user"]) / 1000.0) / 1e9,
            "per_launch": per,
            "counters_source": (ctr or {}).get("source"),
            "note": "achieved/frac: the dominant launch against its binding ceiling (limiter; bound = its memory "
                    "(hbm) or compute (mfma) side): the gathered bytes it requests / launch time against the chip's "
                    "gather ceiling for where those rows are served from (MI355X_MICROARCH.md), or executed MFMA "
                    "flops against the dense bf16 peak; traffic = PMC FETCH_SIZE x2 + WRITE_SIZE per launch (HBM / "
                    "Infinity Cache side); counters = rocprofv3 SQ passes of this build (whole launch, Gram only, and "
                    "their difference = the solve phase)",
        }
        cpu = None
        if world == 1 and not args.no_cpu_baseline:
            ncpu = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
            share = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or ncpu   # the box's CPU share (16 on one GPU)
            counts = []
            for t in (4, min(share, ncpu), ncpu):                   # reference's stream threads, share, nproc
                if t not in counts:
                    counts.append(t)
            cpu = cpu_baseline(ds, args.k, args.lam, args.cpu_seconds, counts)
        value = nnz * K / elapsed
        line = {
            "metric": "ALS ratings/sec per full iteration, k=64 Netflix-shape, 1/2/4/8 MI355X",
            "value": value, "unit": "ratings/s", "n_gpus": world, "steps": K, "warmup": args.warmup,
            "ms_per_step": elapsed / K * 1000.0, "higher_is_better": True, "scaling": "strong",
            "vs_baseline": None, "dtype": "f32", "data": "synthetic (seeded Netflix-shape generator)",
            "config": {"workload": f"netflix-shape synthetic {nu} users x {nm} movies x {nnz} ratings, k={args.k}, "
                                   f"lambda={args.lam}, one step = one full ALS iteration",
                       "n_users": nu, "n_movies": nm, "nnz": nnz, "k": args.k, "lambda": args.lam,
                       "seed": args.seed, "partitions": world, "parallelism": f"id%{world} shards + RCCL all-gather",
                       "exchange": exchange if world > 1 else None,
                       "overlap_chunks": args.overlap_chunks if world > 1 else None},
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
