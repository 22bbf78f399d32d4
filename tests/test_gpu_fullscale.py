"""GPU parity at the BASELINE.json configurations themselves (not only at test size).

- configs[2]: the full Netflix-shape workload (480,189 x 17,770 x 1e8, k = 64, fp32, 1 GPU). One movie half
  and one user half through the product path (ALSApp over libcfk_als.so), then sampled rows -- the 20 longest
  movie rows (split into PARTIAL chunks + a REDUCE task at chunk = nnz/4096), degree-1 users, the longest
  users and random rows -- against the fp64 oracle (oracle.update_rows_f64, the restatement of
  MFeatureCalculator.java:66-104 / UFeatureCalculator.java:66-104) and the oracle's fp32 EJML-order restatement
  (the reference's own fp32 error envelope).
- configs[3]: the same full Netflix-shape workload at k = 128 (KP = 128 variants: 36-tile split Gram, LDS tile
  solve, entry-space solve of rows of 1-3 padded blocks), sampled rows incl. the longest split rows and rows of
  every entry-space size; and k = 128 sharded over two ranks with the chunked (overlapped) user half at test size.
- configs[4] at FULL size: the 10M x 1M x 2B power-law matrix, shard 0 of G = 8 (both in-blocks of the shard plus
  full factor replicas on one GPU, exactly one rank's work of the 8-GPU job), with the heaviest items (millions of
  ratings, 100+ partial slots each) against the oracle; and a 1/40-scale shard.
Progress of the long tests goes to gpurun_out/fullscale_progress.log (a GPU run that prints nothing for minutes
looks hung).
"""
import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

LAM = 0.05


@pytest.fixture(autouse=True)
def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


def _sub_side(oracle_mod, blk, rows):
    """oracle.Side of the selected CSR rows (their entries in in-block order)."""
    rp = blk["row_ptr"]
    deg = np.diff(rp)[rows]
    sub_rp = np.zeros(len(rows) + 1, np.int64)
    np.cumsum(deg, out=sub_rp[1:])
    col = np.concatenate([blk["col"][rp[r]:rp[r + 1]] for r in rows])
    rat = np.concatenate([blk["ratings"][rp[r]:rp[r + 1]] for r in rows])
    return oracle_mod.Side(ids=np.asarray(rows, np.int64), row_ptr=sub_rp, col=col, ratings=rat)


def _check_rows(oracle_mod, blk, rows, got, opp, what):
    """fp64 oracle norm-relative error <= 1e-4, and within 3x the reference's own fp32 error on the same rows
    (test_gpu_parity.test_one_half_every_k_vs_oracle's bar)."""
    side = _sub_side(oracle_mod, blk, rows)
    ref = oracle_mod.update_rows_f64(blk["row_ptr"], blk["col"], blk["ratings"], rows, opp.astype(np.float64), LAM)
    ref32 = oracle_mod.update_side(side, opp.astype(np.float32), LAM, "f32")
    norm = np.linalg.norm(ref, axis=1)
    rel = np.linalg.norm(got[rows].astype(np.float64) - ref, axis=1) / norm
    rel_ref = np.linalg.norm(ref32 - ref, axis=1) / norm
    bad = rel > np.maximum(1e-4, 3 * rel_ref)
    assert not bad.any(), (what, [(int(rows[i]), int(np.diff(blk["row_ptr"])[rows[i]]), float(rel[i]),
                                   float(rel_ref[i])) for i in np.nonzero(bad)[0][:8]])
    return float(rel.max())


def _progress(msg):
    from conftest import ROOT
    d = os.path.join(ROOT, "gpurun_out")
    os.makedirs(d, exist_ok=True)
    with open(os.path.join(d, "fullscale_progress.log"), "a") as f:
        f.write(msg + "\n")


def _sample(blk, rng, n_long=20, n_rand=160, extra=()):
    deg = np.diff(blk["row_ptr"])
    longest = np.argsort(-deg, kind="stable")[:n_long]
    rand = rng.choice(len(deg), size=min(n_rand, len(deg)), replace=False)
    return np.unique(np.concatenate([longest, rand, np.asarray(extra, np.int64)])).astype(np.int64)


@pytest.mark.timeout(900)
@pytest.mark.parametrize("k", [64, 128])
def test_netflix_shape_full_size_sampled_rows(cfk, oracle_mod, k):
    """BASELINE configs[2] (k = 64) and configs[3] (k = 128) at full size through ALSApp (GPU block build, split
    rows at chunk = nnz/4096 with ~974 REDUCE rows, pre-split user half at k = 64, entry-space short rows)."""
    ds = cfk.Dataset.synthetic_netflix(480_189, 17_770, 100_000_000, 0xA15, nthreads=16)
    app = cfk.ALSApp(1, k, LAM, 1, precision="f32", seed=42).setup(ds, check_duplicates=False)
    eng = app.engine
    assert eng.block_stats(0)["n_reduce"] > 0                 # the real work plan has split rows
    U0 = ds.init_user_factors(k, 42)
    app.movie_half()
    M = eng.read_factors(0)
    app.user_half()
    U = eng.read_factors(1)
    assert eng.integrity_status() == [0, 0, 0, 0]
    _progress(f"netflix k={k}: halves done")
    rng = np.random.default_rng(2024)
    mblk = ds.shard_block(0)
    n_long = 20 if k == 64 else 12
    worst_m = _check_rows(oracle_mod, mblk, _sample(mblk, rng, n_long=n_long), M, U0, "movie")
    _progress(f"netflix k={k}: movie rows checked")
    ublk = ds.shard_block(1)
    udeg = np.diff(ublk["row_ptr"])
    # the entry-space sizes: 1, 2 and 3 padded blocks (k = 128 solves all three in entry space, k = 64 the first)
    extra = np.concatenate([np.nonzero(udeg == 1)[0][:40]] +
                           [rng.choice(np.nonzero((udeg > 32 * c) & (udeg <= 32 * (c + 1)))[0], 40, replace=False)
                            for c in range(3)])
    dual = eng.block_path(1)["dual_rows_by_blocks"]
    assert dual[0] > 0 and (k == 64 or min(dual) > 0), dual
    worst_u = _check_rows(oracle_mod, ublk, _sample(ublk, rng, extra=extra), U, M, "user")
    print(f"configs[{2 if k == 64 else 3}] full size k={k}: worst norm-rel movie {worst_m:.2e}, user {worst_u:.2e}")


@pytest.mark.timeout(900)
def test_powerlaw_full_2b_shard0_of_8(cfk, oracle_mod):
    """BASELINE configs[4] at full size: 10M users x 1M items x 2B ratings (log-normal sigma 1.5 users, Zipf items),
    shard 0 of G = 8 -- its ~250M-rating item and user in-blocks plus full factor replicas (U: 10M x 64) on one
    GPU, i.e. one rank's work of the 8-GPU job (MFeatureCalculator.java:66-104 over the heaviest items of the
    stress config). Checked against the fp64 oracle: the heaviest items (>= 1M ratings each, split into 100+
    PARTIAL chunks + a REDUCE task), random items, the longest and random users."""
    import time
    G = 8
    t0 = time.time()
    ds = cfk.Dataset.synthetic_powerlaw(10_000_000, 1_000_000, 2_000_000_000, 0xA15, nthreads=16)
    _progress(f"powerlaw 2B: generated in {time.time() - t0:.0f} s")
    eng = cfk.ALSEngine(64, "f32")
    info = [ds.shard_info(s, G, 0) for s in (0, 1)]
    for side in (0, 1):
        c = ds.shard_coo(side, G, 0)
        eng.alloc_factors(side, info[side]["n_slots"])
        eng.set_block_coo(side, c["n_rows"], c["rows"], c["cols"], c["ratings"], c["row_offset"],
                          info[1 - side]["n_slots"])
        del c
    _progress(f"powerlaw 2B: shard 0 blocks on the GPU at {time.time() - t0:.0f} s")
    assert eng.block_stats(0)["n_reduce"] > 0
    U0 = ds.init_user_factors(64, 42, G)                       # slot order of G shards, 10M x 64
    eng.write_factors(1, U0)
    eng.solve_half(0, LAM)
    Mfull = eng.read_factors(0)
    M = Mfull[info[0]["row_offset"]:info[0]["row_offset"] + info[0]["n_rows"]]
    mblk = ds.shard_block(0, G, 0)
    mdeg = np.diff(mblk["row_ptr"])
    heavy = np.nonzero(mdeg >= 1_000_000)[0]
    assert len(heavy) >= 4 and mdeg.max() >= 4_000_000, (len(heavy), int(mdeg.max()))
    rng = np.random.default_rng(7)
    pick = np.concatenate([np.argsort(-mdeg, kind="stable")[:8], rng.choice(heavy, min(8, len(heavy)), replace=False)])
    _progress(f"powerlaw 2B: item half solved at {time.time() - t0:.0f} s; {len(heavy)} items >= 1M ratings")
    worst_m = _check_rows(oracle_mod, mblk, _sample(mblk, rng, n_long=0, n_rand=120, extra=pick), M, U0, "item")
    _progress(f"powerlaw 2B: item rows checked at {time.time() - t0:.0f} s")
    del mblk, U0
    # user half of the shard against a random full item replica
    Mr = rng.random((info[0]["n_slots"], 64), dtype=np.float32)
    eng.write_factors(0, Mr)
    eng.solve_half(1, LAM)
    Ufull = eng.read_factors(1)
    U = Ufull[info[1]["row_offset"]:info[1]["row_offset"] + info[1]["n_rows"]]
    ublk = ds.shard_block(1, G, 0)
    worst_u = _check_rows(oracle_mod, ublk, _sample(ublk, rng, n_long=20, n_rand=200), U, Mr, "user")
    assert eng.integrity_status() == [0, 0, 0, 0]
    eng.close()
    _progress(f"powerlaw 2B: done at {time.time() - t0:.0f} s")
    print(f"configs[4] full 2B, shard 0 of 8: heaviest item {mdeg.max()} ratings, {len(heavy)} items >= 1M; worst "
          f"norm-rel item {worst_m:.2e}, user {worst_u:.2e}")


def test_powerlaw_shard_sampled_rows(cfk, oracle_mod):
    """BASELINE configs[4] scaled down (1M users x 50k items x 5e7 ratings, Zipf items, log-normal sigma 1.5
    users): shard 0 of G = 8 with full factor replicas, heavy items (>= 100k ratings) split into PARTIAL
    chunks + REDUCE tasks; sampled rows of both halves against the oracle."""
    G = 8
    ds = cfk.Dataset.synthetic_powerlaw(1_000_000, 50_000, 50_000_000, 0xA15, nthreads=16)
    eng = cfk.ALSEngine(64, "f32")
    info = [ds.shard_info(s, G, 0) for s in (0, 1)]
    for side in (0, 1):
        c = ds.shard_coo(side, G, 0)
        eng.alloc_factors(side, info[side]["n_slots"])
        eng.set_block_coo(side, c["n_rows"], c["rows"], c["cols"], c["ratings"], c["row_offset"],
                          info[1 - side]["n_slots"])
    mblk = ds.shard_block(0, G, 0)
    mdeg = np.diff(mblk["row_ptr"])
    assert mdeg.max() >= 100_000 and eng.block_stats(0)["n_reduce"] > 0
    rng = np.random.default_rng(7)
    U0 = ds.init_user_factors(64, 42, G)                       # slot order of G shards
    eng.write_factors(1, U0)
    eng.solve_half(0, LAM)
    Mfull = eng.read_factors(0)
    M = Mfull[info[0]["row_offset"]:info[0]["row_offset"] + info[0]["n_rows"]]
    heavy = np.nonzero(mdeg >= 100_000)[0]
    worst_m = _check_rows(oracle_mod, mblk, _sample(mblk, rng, extra=heavy), M, U0, "item")
    # user half of the shard against a full random item replica
    Mr = rng.random((info[0]["n_slots"], 64), dtype=np.float32)
    eng.write_factors(0, Mr)
    eng.solve_half(1, LAM)
    Ufull = eng.read_factors(1)
    U = Ufull[info[1]["row_offset"]:info[1]["row_offset"] + info[1]["n_rows"]]
    ublk = ds.shard_block(1, G, 0)
    worst_u = _check_rows(oracle_mod, ublk, _sample(ublk, rng), U, Mr, "user")
    assert eng.integrity_status() == [0, 0, 0, 0]
    eng.close()
    print(f"configs[4] shard: heaviest item {mdeg.max()} ratings; worst norm-rel item {worst_m:.2e}, "
          f"user {worst_u:.2e}")


def _sharded_worker(rank, world, port, out_dir, k):
    import sys
    from conftest import ROOT
    sys.path.insert(0, ROOT)
    import torch.distributed as dist
    import __graft_entry__
    cfk = __graft_entry__.load_package()
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    ds = cfk.Dataset.synthetic_netflix(n_users=3000, n_movies=400, nnz=90_000, seed=11, nthreads=8)
    app = cfk.ALSApp(world, k, LAM, 3, precision="f32", seed=9, device=0, rank=rank, world_size=world,
                     overlap_chunks=3)
    app.setup(ds)
    app.run()
    U, M = app.factors()
    np.savez(os.path.join(out_dir, f"rank{rank}.npz"), U=U, M=M, mse=app.mse())
    dist.destroy_process_group()


@pytest.mark.parametrize("k", [64, 128])
def test_sharded_two_ranks_chunked(tmp_path, oracle_mod, cfk, k):
    """BASELINE configs[3] path at test size: k = 128 (KP = 128 MFMA variants) sharded over 2 ranks (both on
    cuda:0, gloo carrying the all-gathers) with the user half in 3 overlapped chunks; MSE delta <= 1e-3 and
    factors within 1e-3 norm-relative of the fp64 oracle. At k = 64 the same run covers the chunked pre-split user
    half (3 waves per SIMD, packed bf16 rating pairs; chunk 0 prepares the pre-split table for the later chunks)."""
    import socket
    import torch.multiprocessing as mp
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    mp.spawn(_sharded_worker, args=(2, port, str(tmp_path), k), nprocs=2, join=True)
    ds = cfk.Dataset.synthetic_netflix(n_users=3000, n_movies=400, nnz=90_000, seed=11, nthreads=8)
    m, u, r = ds.ratings()
    b = oracle_mod.build_blocks(m, u, r)
    Uo, Mo = oracle_mod.run_als(b, k, LAM, 3, seed=9, precision="f64")
    mse_o = oracle_mod.mse(b, Uo, Mo)
    for rank in range(2):
        res = np.load(os.path.join(tmp_path, f"rank{rank}.npz"))
        assert abs(float(res["mse"]) - mse_o) <= 1e-3
        assert np.linalg.norm(res["U"] - Uo) / np.linalg.norm(Uo) < 1e-3
        assert np.linalg.norm(res["M"] - Mo) / np.linalg.norm(Mo) < 1e-3


def _shard_data_worker(rank, world, port, out_dir, workload, restricted):
    import sys
    from conftest import ROOT
    sys.path.insert(0, ROOT)
    import torch.distributed as dist
    import __graft_entry__
    cfk = __graft_entry__.load_package()
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    shape = (20_000, 1_500, 600_000)
    if restricted:
        ds = cfk.Dataset.synthetic_shard(workload, *shape, 5, world, rank, nthreads=8)
    elif workload == "powerlaw":
        ds = cfk.Dataset.synthetic_powerlaw(*shape, 5, nthreads=8)
    else:
        ds = cfk.Dataset.synthetic_netflix(*shape, 5, nthreads=8)
    app = cfk.ALSApp(world, 64, LAM, 3, precision="f32", seed=9, device=0, rank=rank, world_size=world,
                     overlap_chunks=2, movie_chunks=2)
    app.setup(ds, check_duplicates=False)
    app.run()
    U, M = app.factors()
    np.savez(os.path.join(out_dir, f"{workload}_{int(restricted)}_rank{rank}.npz"), U=U, M=M, mse=app.mse())
    dist.destroy_process_group()


@pytest.mark.parametrize("workload", ["netflix", "powerlaw"])
def test_two_ranks_on_shard_restricted_data(tmp_path, cfk, workload):
    """bench.py's multi-GPU data path at reduced size: each of 2 ranks (both on cuda:0, gloo carrying the
    all-gathers, both halves in 2 chunks: chunk-major movie and user slots) synthesizes ONLY its shard's ratings (als_dataset_synthetic_*_shard) and
    the factors and MSE are bitwise those of the same 2-rank run on the full dataset, and equal the 1-rank run's
    (same per-entity arithmetic; at this size every split row has the same chunking). Multi-GPU RCCL itself is
    measured only by the driver's 8-GPU run."""
    import socket
    import torch.multiprocessing as mp
    res = {}
    for restricted in (True, False):
        s = socket.socket()
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
        s.close()
        mp.spawn(_shard_data_worker, args=(2, port, str(tmp_path), workload, restricted), nprocs=2, join=True)
        res[restricted] = [np.load(os.path.join(tmp_path, f"{workload}_{int(restricted)}_rank{r}.npz")) for r in (0, 1)]
    shape = (20_000, 1_500, 600_000)
    ds = (cfk.Dataset.synthetic_powerlaw if workload == "powerlaw" else cfk.Dataset.synthetic_netflix)(*shape, 5, 8)
    app = cfk.ALSApp(1, 64, LAM, 3, precision="f32", seed=9).setup(ds, check_duplicates=False)
    app.run()
    U1, M1 = app.factors()
    for r in (0, 1):
        a, b = res[True][r], res[False][r]
        assert np.array_equal(a["U"], b["U"]) and np.array_equal(a["M"], b["M"]) and float(a["mse"]) == float(b["mse"])
        assert np.array_equal(a["U"], U1) and np.array_equal(a["M"], M1)
        assert abs(float(a["mse"]) - app.mse()) <= 1e-12 * app.mse()


def test_bench_rehearsal_two_ranks_shard_restricted(tmp_path):
    """bench.py itself as the driver's N = 2 run launches it (torch.distributed.run, one process per rank), both
    ranks on cuda:0 over gloo (--rehearse-one-gpu), on the power-law workload at reduced size: one JSON line whose
    MSE equals the 1-rank bench line's, each rank holding ~2/N of the ratings."""
    import json
    import socket
    import subprocess
    import sys
    from conftest import ROOT
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    common = ["--workload", "powerlaw", "--users", "20000", "--movies", "1500", "--nnz", "600000", "--steps", "3",
              "--warmup", "1", "--no-cpu-baseline"]
    env = dict(os.environ, OMP_NUM_THREADS="8")
    two = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
                          "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.join(ROOT, "bench.py"),
                          "--gpus", "2", "--rehearse-one-gpu"] + common, capture_output=True, text=True, timeout=300,
                         env=env, cwd=ROOT)
    assert two.returncode == 0, two.stderr[-3000:]
    one = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + common, capture_output=True, text=True,
                         timeout=300, env=env, cwd=ROOT)
    assert one.returncode == 0, one.stderr[-3000:]
    l2 = json.loads([x for x in two.stdout.splitlines() if x.startswith("{")][-1])
    l1 = json.loads([x for x in one.stdout.splitlines() if x.startswith("{")][-1])
    assert l2["n_gpus"] == 2 and l2["config"]["exchange_world"] == 2 and l2["config"]["nnz"] == 600_000
    assert l2["config"]["nnz_this_rank"] < 0.75 * 600_000
    assert abs(l2["mse_after"] - l1["mse_after"]) <= 1e-9 * l1["mse_after"]
    assert l1["build"]["lib_sha256"] == l2["build"]["lib_sha256"]
    # the self-check of a sharded run: replicas bitwise equal on both ranks, integrity clean
    assert l2["replicas_agree"] is True and l2["integrity_clean"] is True and len(l2["replica_digest"]) == 2
    # fault injection: rank 1 alters one word of its replica -> replicas_agree false, exit status 3
    bad = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
                          "--master-addr", "127.0.0.1", "--master-port", str(port + 1), os.path.join(ROOT, "bench.py"),
                          "--gpus", "2", "--rehearse-one-gpu"] + common, capture_output=True, text=True, timeout=300,
                         env=dict(env, CFK_BENCH_PERTURB_RANK="1"), cwd=ROOT)
    assert bad.returncode != 0 and "self-check failed" in bad.stderr, bad.stderr[-2000:]
    lb = json.loads([x for x in bad.stdout.splitlines() if x.startswith("{")][-1])
    assert lb["replicas_agree"] is False and lb["integrity_clean"] is True
    if not os.environ.get("CFK_ALS_LIB"):   # the product library (an A/B variant carries no build stamp)
        assert l1["build"]["source_matches_tree"] and l1["build"]["binary_matches_tree"]
