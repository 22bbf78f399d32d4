#!/usr/bin/env python3
"""bench.py -- ALS ratings/sec per full iteration, Netflix-shape k=64 fp32 on 1..8 MI355X (BASELINE.json).

  python bench.py [--gpus N] [--steps K] [--warmup W] [--workload netflix|powerlaw] [--k 64|128]
                  [--exchange native|torch] [--movie-chunks C]
  python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 --master-port P \
      bench.py --gpus N --steps K --warmup W

A step = one full ALS iteration (movie half + RCCL all-gather + user half + RCCL all-gather) over seeded synthetic
ratings, inputs resident in HBM before the timed region:
  --workload netflix   (default, the metric's config) 480,189 users x 17,770 movies x 1e8 ratings, lambda = 0.05,
                       k = 64 (BASELINE configs[2]); --k 128 is configs[3];
  --workload powerlaw  10M users x 1M items x 2e9 ratings, k = 64 (BASELINE configs[4], an 8-GPU config).
The dataset is fixed as N grows (strong scaling): users and movies are sharded by id % N, one process per GPU, and
with N > 1 each process synthesizes only its shard's ratings (~2/N of them: als_dataset_synthetic_*_shard).

Prints ONE JSON line (rank 0). `roofline` describes the dominant kernel launch (the slower of the two halves' fused
gather/Gram/solve launches; both are under roofline.per_launch), timed with HIP events on the stream the kernel is
launched on, against the ceiling that binds it: the MFMA pipe (the Gram's MFMAs as issued against the dense
bf16/f16 peak) or the gather of the opposite factor rows (bytes requested / time against the chip's gather ceiling
for where those rows are served from), whichever the launch is closer to; the algorithmic fp32 TFLOP/s and the
SURVEY.md §8d algorithmic-byte rate are reported beside it. `counters` / `traffic` come from the rocprofv3 passes
of the SAME library build (profiles/counters_k<k>.json, stamped with the library's sha256; dropped when the hashes
differ). `cpu_baseline` times the oracle's Java-float restatement of the reference hot path (the "port") on a
bounded sample of the same workload with the reference's 4 stream threads (BaseKafkaApp.java:51) and the box's CPU
share, rank 0 at N = 1 only. `build` names the library that ran (path, sha256, the source digest it was built from).
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
HBM_MEASURED_GBS = 6290.0    # the guide's measured HBM rate (float4 copy, 79 % of the spec)
FP32_PEAK_TFS = 157.3        # f32 vector = f32 MFMA dense peak
MFMA16_PEAK_TFS = 2500.0     # dense bf16 / f16 MFMA peak (no sparsity; the f16 forms take the bf16 cycles)
# MI355X_MICROARCH.md "Indexed rows: gather into LDS": uniformly random rows of a 151 MB table (the 123 MB k = 64
# user table the movie half gathers sits between its 38 MB and 151 MB rows) are served at 7.4-7.9 TB/s chip-wide;
# rows every workgroup shares from the XCD's L2 at 16.8-18.8 TB/s there. This repository's own gather microbenchmark
# (tools/gather_bench.hip: 256-B rows in 8-KB blocks, 16 waves per CU, nothing else running) moves uniformly random rows
# of the 4.5 MB pre-split movie table at 22.0-22.2 TB/s (profiles/r05e/gather_bench.log, profiles/r06c/
# gather_bench_*.log; 25 TB/s with the Netflix popularity skew) and of a 123 MB table at 7.1-7.6 TB/s: the L2 ceiling is
# the higher measured uniform-row rate, so the fraction is not flattered by the guide's lower figure.
IC_GATHER_CEILING_GBS = 7900.0
L2_GATHER_CEILING_GBS = 22200.0
L2_RESIDENT_BYTES = 8 << 20  # a gathered table this small stays in every XCD's 4 MiB L2 to most of its rows
IC_RESIDENT_BYTES = 256 << 20   # Infinity Cache: a larger gathered table streams from HBM (configs[4]'s 2.56 GB U)
MFMA_FLOP = 16 * 16 * 32 * 2   # one v_mfma_f32_16x16x32_{bf16,f16}
WORKLOADS = {"netflix": (480_189, 17_770, 100_000_000), "powerlaw": (10_000_000, 1_000_000, 2_000_000_000)}


def half_bytes(nnz, n_rows, k, s=4):
    """SURVEY.md §8d algorithmic gather+Gram bytes of one half: factor row + col index + rating per entry,
    row_ptr, and the written factor rows."""
    return nnz * (s * k + 4 + 4) + 8 * (n_rows + 1) + s * k * n_rows


def half_flops(nnz, n_rows, k):
    """Algorithmic Gram + RHS flops and solve flops of one half."""
    return nnz * (k * k + 3 * k), n_rows * (k ** 3 / 3 + 2 * k * k)


def mfma_per_block(kp, presplit):
    """16x16x32 MFMAs issued per 32-entry block by the Gram (als_kernels.hip), C = kp/16 feature blocks:
    pre-split (scaled two-term fp16): 3 per off-diagonal tile (hh, hm, mh), 2 per diagonal tile (hh + the folded
    hm), 2 C for the RHS (h and m against the rh / rm rating columns); on-the-fly three-term bf16 split: 6 per
    off-diagonal tile, 4 per diagonal tile, RHS on the VALU."""
    c = kp // 16
    if presplit:
        return 3 * (c * (c - 1) // 2) + 2 * c + 2 * c
    return 6 * (c * (c - 1) // 2) + 4 * c


def served_from(table_bytes, interleaved):
    """Where a half's gathered opposite rows are served from, and that source's gather ceiling (GB/s): the XCD's L2
    (a table of <= 8 MB), the Infinity Cache (<= 256 MiB), beyond it a mix of IC and HBM ("hbm": the SURVEY.md §8d
    roofline binds), or -- a half with interleaved split rows -- the L2 as far as the walk in step keeps the
    IC-resident table's rows there ("l2_ic_walk", priced against the L2 ceiling: an upper bound)."""
    if interleaved:
        return "l2_ic_walk", L2_GATHER_CEILING_GBS
    if table_bytes <= L2_RESIDENT_BYTES:
        return "l2", L2_GATHER_CEILING_GBS
    if table_bytes <= IC_RESIDENT_BYTES:
        return "ic", IC_GATHER_CEILING_GBS
    return "hbm", HBM_PEAK_GBS


def bound_label(where):
    """roofline.bound of a gather-limited launch by where its rows are served from"""
    return "beyond_ic_mixed" if where == "hbm" else f"{where}_gather"


def cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_share():
    """CPUs this process may use: the affinity mask, capped by the cgroup CPU quota and by OMP_NUM_THREADS (the GPU
    box sets it to the box's share; nproc there shows the whole machine)."""
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    src = [f"affinity {n}"]
    try:
        q, p = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            c = max(1, int(int(q) / int(p)))
            src.append(f"cgroup cpu.max {c}")
            n = min(n, c)
    except (OSError, ValueError):
        pass
    omp = int(os.environ.get("OMP_NUM_THREADS", "0") or 0)
    if omp > 0:
        src.append(f"OMP_NUM_THREADS {omp}")
        n = min(n, omp)
    return n, ", ".join(src)


def cpu_baseline(ds, k, lam, seconds, thread_counts, share_src):
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
            "runs": runs, "cpu_model": cpu_model(), "cpu_share": share_src, "nproc": os.cpu_count()}


def build_record():
    """The library this process loaded: path, sha256, and the build stamp it carries (source digest)."""
    import __graft_entry__
    from cfk_amd import _lib
    path = os.path.realpath(_lib.LIB_PATH)
    rec = {"lib_path": os.path.relpath(path, ROOT), "lib_sha256": __graft_entry__.sha256_file(path),
           "device_code_sha256": __graft_entry__.device_code_sha256(path)}
    info = __graft_entry__.build_info("product")
    tree = __graft_entry__.source_digest()
    if info and info.get("lib_sha256") == rec["lib_sha256"]:
        rec["source_sha256"] = info.get("source_sha256")
        rec["source_matches_tree"] = info.get("source_sha256") == tree
    # the digest compiled into the binary itself (als_build_source_sha256): the source <-> binary link without the
    # build's own BUILD_INFO.json
    embedded = _lib.lib().als_build_source_sha256().decode() or None
    rec["binary_source_sha256"] = embedded
    rec["binary_matches_tree"] = embedded == tree if embedded else None
    return rec


def counters_path(k, workload="netflix", shard_of=0):
    """profiles/counters_k<k>.json for the metric's workload on the whole dataset, else
    counters_k<k>_<workload>[_shard<G>].json (tools/prof_summary.py counters_name writes the same names)"""
    if workload == "netflix" and not shard_of:
        return os.path.join(ROOT, "profiles", f"counters_k{k}.json")
    return os.path.join(ROOT, "profiles", f"counters_k{k}_{workload}" + (f"_shard{shard_of}" if shard_of else "") + ".json")


def load_counters(k, nnz, lib_sha, workload="netflix", shard_of=0, dev_sha=None):
    """Per-launch rocprofv3 counters at (k, nnz) of THIS library's kernels (profiles/counters_k<k>*.json, stamped by
    tools/prof_summary.py with the profiled library's sha256 and the sha256 of its device code): valid when either
    matches (a host-code-only rebuild keeps the kernels and so the counters). (counters, None) or (None, why they
    were dropped)."""
    path = counters_path(k, workload, shard_of)
    try:
        c = json.load(open(path))
    except (OSError, ValueError):
        return None, f"no {os.path.relpath(path, ROOT)}"
    if c.get("k") != k or c.get("nnz") != nnz:
        return None, f"{os.path.relpath(path, ROOT)} was profiled at k={c.get('k')} nnz={c.get('nnz')}"
    if c.get("lib_sha256") == lib_sha:
        return dict(c, matched_by="lib_sha256"), None
    if dev_sha and c.get("device_code_sha256") == dev_sha:
        return dict(c, matched_by="device_code_sha256"), None
    return None, (f"stale: {c.get('source')} profiled library {str(c.get('lib_sha256'))[:12]} != this build "
                  f"{lib_sha[:12]} (device code {str(c.get('device_code_sha256'))[:12]} != {str(dev_sha)[:12]})")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--workload", choices=tuple(WORKLOADS), default="netflix")
    ap.add_argument("--k", type=int, default=64)
    ap.add_argument("--users", type=int, default=None)
    ap.add_argument("--movies", type=int, default=None)
    ap.add_argument("--nnz", type=int, default=None)
    ap.add_argument("--seed", type=int, default=0xA15)
    ap.add_argument("--lam", type=float, default=0.05)
    ap.add_argument("--cpu-seconds", type=float, default=7.0, help="CPU baseline seconds per thread count")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--overlap-chunks", type=int, default=4, help="user-half chunks per all-gather overlap (N > 1)")
    ap.add_argument("--exchange", choices=("torch", "native"), default="native",
                    help="N > 1: all-gathers through the engine's own RCCL communicator behind the C ABI (default: "
                         "als_comm_init / als_allgather_shard, the path a JNI caller binds) or through "
                         "torch.distributed (RCCL); the one-GPU gloo rehearsal always uses torch")
    ap.add_argument("--movie-chunks", type=int, default=None,
                    help="N > 1: movie-half exchange chunks (default: --overlap-chunks once the movie table exceeds "
                         "64 MB, e.g. configs[4]; else 1)")
    ap.add_argument("--shard-of", type=int, default=0,
                    help="G > 1: run ONE rank's work of a G-GPU job on this GPU (shard --shard-rank of G, synthesized "
                         "alone, no exchange): the per-GPU compute of a sharded config such as configs[4] on 8 GPUs; "
                         "value = that rank's ratings per second")
    ap.add_argument("--shard-rank", type=int, default=0)
    ap.add_argument("--rehearse-one-gpu", action="store_true",
                    help="N > 1 ranks all on cuda:0 over gloo: rehearses the multi-rank driver on a one-GPU box "
                         "(RCCL needs one GPU per rank); not a performance configuration")
    args = ap.parse_args()
    users, movies, nnz_total = WORKLOADS[args.workload]
    users, movies = args.users or users, args.movies or movies
    nnz_total = args.nnz or nnz_total

    import torch
    import torch.distributed as dist
    import __graft_entry__
    cfk = __graft_entry__.load_package()
    from cfk_amd import _lib
    if hasattr(_lib.lib(), "als_debug_knobs_compiled"):   # exported by the diagnostics build only, whatever its path
        sys.exit(f"bench: {_lib.LIB_PATH} is the diagnostics build (work-dropping knobs compiled in): refused")

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    solo = args.shard_of > 1   # one rank of a G-GPU job, alone on this GPU
    if solo and world > 1:
        sys.exit("bench: --shard-of runs one process")
    if world != args.gpus and rank == 0:
        print(f"bench: WORLD_SIZE={world} but --gpus={args.gpus}; using WORLD_SIZE", file=sys.stderr)
    if args.rehearse_one_gpu:
        local = 0
    torch.cuda.set_device(local)
    if world > 1:
        if args.rehearse_one_gpu:
            dist.init_process_group("gloo")
        else:
            import datetime
            # torch's NCCL watchdog bounds its own collectives (the engine bounds the native exchange's waits)
            dist.init_process_group("nccl", device_id=torch.device(f"cuda:{local}"),
                                    timeout=datetime.timedelta(seconds=300))

    def barrier():
        if world > 1:
            dist.barrier()

    t_setup = time.perf_counter()
    # a progress line on stderr every 30 s until the timed steps start (a multi-minute configs[4] synthesis and block
    # build would otherwise print nothing for minutes)
    import threading
    setup_done = threading.Event()

    def heartbeat():
        while not setup_done.wait(30.0):
            print(f"bench: rank {rank} setting up, {time.perf_counter() - t_setup:.0f} s", file=sys.stderr, flush=True)
    threading.Thread(target=heartbeat, daemon=True).start()
    nthreads = min(16, os.cpu_count() or 1)
    if solo:
        ds = cfk.Dataset.synthetic_shard(args.workload, users, movies, nnz_total, args.seed, args.shard_of,
                                         args.shard_rank, nthreads)
    elif world > 1:   # this rank's ratings only (both sides' in-blocks of shard `rank`)
        ds = cfk.Dataset.synthetic_shard(args.workload, users, movies, nnz_total, args.seed, world, rank, nthreads)
    elif args.workload == "powerlaw":
        ds = cfk.Dataset.synthetic_powerlaw(users, movies, nnz_total, args.seed, nthreads=nthreads)
    else:
        ds = cfk.Dataset.synthetic_netflix(users, movies, nnz_total, args.seed, nthreads=nthreads)
    nm, nu, nnz_local = ds.counts()
    exchange = "none" if solo else args.exchange if world > 1 and not args.rehearse_one_gpu else "torch"
    gsim, rsim = (args.shard_of, args.shard_rank) if solo else (world, rank)
    app = cfk.ALSApp(gsim, args.k, args.lam, args.steps, precision="f32", seed=42, device=local, rank=rsim,
                     world_size=gsim, overlap_chunks=args.overlap_chunks, exchange=exchange,
                     movie_chunks=args.movie_chunks).setup(ds, check_duplicates=False)
    t_setup = time.perf_counter() - t_setup
    # ranks the exchange spans: the engine's own communicator (native) or the torch process group; RCCL unless the
    # one-GPU rehearsal runs the group over gloo
    exchange_world = (app.engine.comm_info()[0] if exchange == "native" else
                      dist.get_world_size() if world > 1 else 1)
    rccl_world = None if args.rehearse_one_gpu else exchange_world

    setup_done.set()
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
    app.engine.synchronize()   # bounded while an RCCL exchange is pending (als_comm_set_timeout): a hang is named
    torch.cuda.synchronize()
    barrier()
    elapsed = time.perf_counter() - t0
    app.engine.set_timing(False)
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device="cpu" if args.rehearse_one_gpu else f"cuda:{local}")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    # self-check of a sharded run: every rank's factor replicas bitwise equal, every integrity record clean
    # (CFK_BENCH_PERTURB_RANK=r: fault injection for tests/test_distributed.py -- rank r alters one word of its
    # user-factor replica before the check)
    pr = os.environ.get("CFK_BENCH_PERTURB_RANK")
    if pr is not None and world > 1 and int(pr) == rank:
        app.engine.synchronize()
        app.engine.factors[1][0, 0] += 1.0
    check = app.verify_replicas()

    # per-half device time over the timed steps (HIP events on the launch stream), per half-iteration: with the
    # chunked user half (N > 1) one half is several launches, summed here
    K = args.steps
    eng = app.engine
    g_ms, r_ms = {}, {}
    for side in ("movie", "user"):
        g, r, _ = eng.timing_collect(side)
        g_ms[side], r_ms[side] = g / K, r / K
    mse = app.mse() if not solo else None   # a lone shard's factors are not a model

    if rank == 0:
        build = build_record()
        info = {"movie": app.info[0], "user": app.info[1]}
        ctr, ctr_why = (load_counters(args.k, nnz_total, build["lib_sha256"], args.workload,
                                      args.shard_of if solo else 0, build["device_code_sha256"])
                        if world == 1 else (None, "N > 1"))
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
            mf = ((main_blocks * mfma_per_block(kp, path["presplit"]) + dual_mfma) * MFMA_FLOP
                  if path["gram_path"] == "mfma_split" else 0)
            c = (ctr or {}).get("per_side", {}).get(side, {})
            # bytes the launch requests from the memory hierarchy: the gathered opposite rows (4 kp B per padded
            # entry: fp32, or the fp16 h/m planes of the pre-split table -- the same size), column indices,
            # ratings (fp16 rh / rm pairs on the pre-split path) and the written factor rows
            dual_entries = sum(32 * (c_ + 1) * n for c_, n in enumerate(dual))
            main_entries = main_blocks * 32
            gathered = (main_entries * (4 * kp + 8) + dual_entries * (4 * kp + 8)
                        + 4 * kp * i["n_rows"])
            opp_rows = info["user" if side == "movie" else "movie"]["n_slots"] + 1
            table_bytes = opp_rows * 4 * kp
            # where the gathered rows are served from: the XCD's L2, the Infinity Cache, (beyond it) HBM -- or, on a
            # half with interleaved split rows, the L2 as far as the waves' walk of the
            # IC-resident table in step keeps its rows there: priced against the L2 gather ceiling (an upper bound;
            # the rest of the rows come from the IC)
            split = eng.split_info(si)
            where, gceil = served_from(table_bytes, split["interleaved_rows"] > 0)
            mfma_frac = mf / t_s / 1e12 / MFMA16_PEAK_TFS if mf else 0.0
            # rows of a table beyond the L2 are served by the Infinity Cache: measure them with the fabric-side counter
            # bytes of this build (L2 hits excluded) when profiled, else with the bytes requested (then an upper
            # bound that can exceed the ceiling by the L2 hit share)
            fab = c.get("hbm_bytes") if c else None
            if where == "hbm":   # the §8d roofline binds: algorithmic bytes against HBM peak
                g_bytes = b
            else:
                g_bytes = fab if (fab and where == "ic") else gathered
            gather_frac = g_bytes / t_s / 1e9 / gceil
            d = {
                # <KP, waves per SIMD, ...>: the instantiations launch_solve picks (als_kernels.hip, CFK_PS64_WAVES)
                "kernel": f"als_solve_mfma<{kp},{1 if kp == 128 else (4 if path['presplit'] else 2)},split,"
                          f"{'presplit f16' if path['presplit'] else 'on-the-fly bf16 split'}> + als_solve_dual "
                          f"(short rows)",
                "avg_launch_ms": g_ms[side], "reduce_launch_ms": r_ms[side],
                "mfma": {"per_32_entry_block": mfma_per_block(kp, path["presplit"]), "flop_per_launch": mf,
                         "executed_tflops": mf / t_s / 1e12, "peak": MFMA16_PEAK_TFS, "frac": mfma_frac},
                "gather": {"bytes_requested": gathered, "bytes": g_bytes,
                           "bytes_source": ("SURVEY.md §8d algorithmic bytes" if where == "hbm" else
                                            "PMC FETCH_SIZE x2 + WRITE_SIZE" if g_bytes is not gathered else "requested"),
                           "opposite_table_bytes": table_bytes, "served_from": where,
                           "achieved_gbs": g_bytes / t_s / 1e9, "ceiling_gbs": gceil, "frac": gather_frac,
                           "ceiling": {"l2": "L2-resident rows", "ic": "Infinity-Cache random rows",
                                       "hbm": "HBM peak (table beyond the Infinity Cache)",
                                       "l2_ic_walk": "L2-resident rows (an IC-resident table walked in step by "
                                                     "interleaved chunks)"}[where]},
                "split_rows": split,
                "algorithmic_bytes": {"bytes": b, "achieved_gbs": b / t_s / 1e9, "frac_of_hbm": b / t_s / 1e9 / HBM_PEAK_GBS,
                                      "note": "SURVEY.md §8d algorithmic bytes / launch time; cache-served gathers "
                                              "included, so it can exceed 1: not a bound"},
                "algorithmic_fp32": {"gram_flop": gram_f, "solve_flop": solve_f,
                                     "tflops": (gram_f + solve_f) / t_s / 1e12, "fp32_peak": FP32_PEAK_TFS,
                                     "note": "useful fp32 work; the split Gram issues several MFMA products per fp32 "
                                             "product, so executed_tflops > this"},
                "short_rows_entry_space": dual,
                "presplit": path["presplit"],
            }
            if c:
                d["counters"] = c
                d["traffic"] = c.get("hbm_bytes")
            if mfma_frac >= gather_frac:
                d.update(bound="mfma", unit="TFLOP/s", peak=MFMA16_PEAK_TFS, achieved=mf / t_s / 1e12, frac=mfma_frac,
                         limit="MFMA pipe: the Gram's 16x16x32 MFMA flops as issued (whole launch, solve phase "
                               "included) against the dense bf16/f16 peak")
            elif where == "hbm":
                # the table exceeds the IC, but its hot rows (the most active users) stay there: a mix of IC and
                # HBM service, so the algorithmic rate is reported against the spec peak AND the measured HBM rate
                d.update(bound=bound_label(where), unit="GB/s", peak=gceil, achieved=g_bytes / t_s / 1e9,
                         frac=gather_frac, frac_of_measured_hbm=g_bytes / t_s / 1e9 / HBM_MEASURED_GBS,
                         measured_hbm_gbs=HBM_MEASURED_GBS,
                         limit="SURVEY.md §8d algorithmic bytes per launch / launch time against the 8 TB/s HBM peak "
                               "(frac) and the guide's measured 6.29 TB/s (frac_of_measured_hbm); the gathered table "
                               "exceeds the 256 MiB Infinity Cache but its most active rows are served from it, so "
                               "this is a mixed IC/HBM figure, not a pure HBM bound")
            else:
                d.update(bound=bound_label(where), unit="GB/s", peak=gceil, achieved=g_bytes / t_s / 1e9,
                         frac=gather_frac,
                         limit="gather of the opposite factor rows: bytes requested per launch / launch time against "
                               f"the chip's {d['gather']['ceiling']} gather ceiling (MI355X_MICROARCH.md)")
            per[side] = d
        dom = max(per, key=lambda s: per[s]["avg_launch_ms"])
        d = per[dom]
        roofline = {
            "bound": d["bound"], "limiter": d["bound"],
            "achieved": d["achieved"], "peak": d["peak"],
            "unit": d["unit"], "frac": d["frac"], "traffic": d.get("traffic"),
            "frac_of_measured_hbm": d.get("frac_of_measured_hbm"),
            "kernel": d["kernel"] + f" ({dom} half, the dominant launch)", "limit": d["limit"],
            "avg_launch_ms": d["avg_launch_ms"], "counters": d.get("counters"),
            "counters_dropped": ctr_why,
            "algorithmic_fp32_tflops": d["algorithmic_fp32"]["tflops"],
            "algorithmic_bytes_frac": d["algorithmic_bytes"]["frac_of_hbm"],
            "both_halves_algorithmic_gbs": (per["movie"]["algorithmic_bytes"]["bytes"] +
                                            per["user"]["algorithmic_bytes"]["bytes"])
                                           / ((g_ms["movie"] + g_ms["user"]) / 1000.0) / 1e9,
            "per_launch": per,
            "counters_source": (ctr or {}).get("source"),
            "note": "achieved/frac: the dominant launch against the ceiling it is closest to (bound: mfma = "
                    "executed 16x16x32 MFMA flops against the dense bf16/f16 peak; l2_gather / ic_gather = the "
                    "gathered bytes it requests / launch time against the chip's gather ceiling for rows served from "
                    "the L2 / the Infinity Cache (MI355X_MICROARCH.md); l2_ic_walk_gather = an IC-resident table "
                    "walked in step by interleaved split rows, priced against the L2 ceiling; beyond_ic_mixed = "
                    "SURVEY.md §8d algorithmic bytes against the HBM peak and the measured HBM rate when the gathered "
                    "table exceeds the Infinity Cache); traffic = PMC FETCH_SIZE x2 + "
                    "WRITE_SIZE per launch; counters = rocprofv3 SQ passes of this build",
        }
        cpu = None
        if world == 1 and not solo and not args.no_cpu_baseline:
            share, share_src = cpu_share()
            counts = [4] + ([share] if share != 4 else [])      # reference's stream threads, the box's share
            cpu = cpu_baseline(ds, args.k, args.lam, args.cpu_seconds, counts, share_src)
        # whole-job ratings per second; --shard-of: this rank's share (its in-block entries, averaged over the halves)
        shard_nnz = (info["movie"]["nnz"] + info["user"]["nnz"]) / 2
        value = (shard_nnz if solo else nnz_total) * K / elapsed
        wl = (f"{args.workload}-shape synthetic {nu} users x {nm} movies x {nnz_total} ratings, k={args.k}, "
              f"lambda={args.lam}, one step = one full ALS iteration")
        line = {
            "metric": "ALS ratings/sec per full iteration, k=64 Netflix-shape, 1/2/4/8 MI355X",
            "value": value, "unit": "ratings/s", "n_gpus": world, "steps": K, "warmup": args.warmup,
            "ms_per_step": elapsed / K * 1000.0, "higher_is_better": True, "scaling": "strong",
            "vs_baseline": None, "dtype": "f32", "data": f"synthetic (seeded {args.workload}-shape generator)",
            "config": {"workload": wl, "workload_name": args.workload,
                       "n_users": nu, "n_movies": nm, "nnz": nnz_total, "nnz_this_rank": nnz_local, "k": args.k,
                       "lambda": args.lam, "seed": args.seed, "partitions": world,
                       "parallelism": f"id%{world} shards + RCCL all-gather",
                       "exchange": exchange if world > 1 else None, "rccl_world": rccl_world,
                       "exchange_world": exchange_world,
                       "overlap_chunks": args.overlap_chunks if world > 1 else None,
                       "movie_chunks": app.info[0]["n_chunks"] if world > 1 else None,
                       "rehearsal_gloo_one_gpu": bool(args.rehearse_one_gpu),
                       "shard_of": args.shard_of if solo else None, "shard_rank": args.shard_rank if solo else None,
                       "shard_ratings": shard_nnz if solo else None,
                       # main launches per half-iteration (one per slot chunk; tools/prof_summary.py groups the
                       # kernel trace by these)
                       "launches_per_half": {"movie": app.info[0]["n_chunks"], "user": app.info[1]["n_chunks"]}},
            "solves_per_s": ((info["movie"]["n_rows"] + info["user"]["n_rows"]) if solo else (nm + nu)) * K / elapsed,
            "projected_job_ratings_per_s_compute_only": value * args.shard_of if solo else None,
            "projection_note": ("this rank's rate x G: assumes balanced shards (id % G balances the Netflix shape; on the "
                                "power-law workload the heaviest items make rank 0 the longest) and leaves out the "
                                "exchange (DESIGN.md section 4)") if solo else None,
            "mse_after": mse,
            "replicas_agree": check["replicas_agree"], "integrity_clean": check["integrity_clean"],
            "replica_digest": check["digest"],
            "setup_s": t_setup,
            "build": build,
            "roofline": roofline,
            "cpu_baseline": cpu,
        }
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()
    if not (check["replicas_agree"] and check["integrity_clean"]):
        print(f"bench: rank {rank}: self-check failed: replicas_agree={check['replicas_agree']} "
              f"integrity_clean={check['integrity_clean']} ({check['integrity_failures']} bad partial slots)",
              file=sys.stderr, flush=True)
        sys.exit(3)


if __name__ == "__main__":
    main()
