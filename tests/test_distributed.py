"""CPU rehearsal of the multi-GPU path with torch.distributed + gloo, world_size 2, 3 and 4.

The per-shard solve is injected (an oracle-backed stand-in with the ALSEngine interface): what is under
test here is the product's distributed driver -- id % G sharding into slot order, the per-half
all_gather_into_tensor into the factor replicas (sentinel row excluded), the MSE all-reduce and the final
slot -> ascending-id permutation. Every rank must reproduce the single-process oracle run exactly (fp64).
The same driver runs over RCCL (backend "nccl") on the GPUs; see bench.py.
"""
import os
import socket

import numpy as np
import pytest
import torch

from conftest import GOLDEN, ROOT


class OracleShardEngine:
    """ALSEngine-shaped CPU stand-in: torch CPU factor tensors (+ sentinel row), oracle per-row update."""

    def __init__(self, k, precision, device):
        import oracle
        self.oracle = oracle
        self.k = k
        self.kp = k
        self.dtype = torch.float64
        self.factors = [None, None]
        self.blocks = [None, None]
        self.layout = [(0, 0), (0, 0)]
        self.chunks = [None, None]

    def set_row_layout(self, side, rows_per_chunk, chunk_stride):
        self.layout[side] = (int(rows_per_chunk), int(chunk_stride))

    def _rows(self, side, lo, hi):
        """factor rows of local rows [lo, hi) under the side's slot layout (als_set_row_layout)"""
        off = self.blocks[side][3]
        i = np.arange(lo, hi)
        rpc, stride = self.layout[side]
        return off + i if rpc == 0 else off + (i // rpc) * stride + i % rpc

    def use_torch_stream(self):
        pass

    def synchronize(self):
        pass

    def alloc_factors(self, side, n):
        self.factors[side] = torch.zeros((n + 1, self.kp), dtype=self.dtype)
        return self.factors[side]

    def set_block(self, side, row_ptr, col, ratings, row_offset, n_opp_rows):
        self.blocks[side] = (np.asarray(row_ptr, np.int64), np.asarray(col, np.int32), np.asarray(ratings, np.int16),
                             int(row_offset), int(n_opp_rows))

    def write_factors(self, side, host, row0=0):
        self.factors[side][row0:row0 + len(host), :self.k] = torch.from_numpy(np.asarray(host, np.float64))

    def read_factors(self, side, row0=0, n_rows=None):
        n = self.factors[side].shape[0] - 1 - row0 if n_rows is None else n_rows
        return self.factors[side][row0:row0 + n, :self.k].numpy().copy()

    def solve_half(self, side, lam):
        rp, col, rat, off, n_opp = self.blocks[side]
        opp = self.factors[1 - side][:n_opp].numpy()
        s = self.oracle.Side(ids=np.arange(len(rp) - 1), row_ptr=rp, col=col, ratings=rat)
        out = self.oracle.update_side(s, opp, lam, "f64", 1)
        self.factors[side][self._rows(side, 0, len(out))] = torch.from_numpy(out)

    def set_chunks(self, side, bounds):
        self.chunks[side] = [(int(bounds[c]), int(bounds[c + 1])) for c in range(len(bounds) - 1)]

    def solve_half_chunk(self, side, lam, c):
        rp, col, rat, off, n_opp = self.blocks[side]
        lo, hi = self.chunks[side][c]
        opp = self.factors[1 - side][:n_opp].numpy()
        sub = rp[lo:hi + 1] - rp[lo]
        s = self.oracle.Side(ids=np.arange(hi - lo), row_ptr=sub, col=col[rp[lo]:rp[hi]], ratings=rat[rp[lo]:rp[hi]])
        out = self.oracle.update_side(s, opp, lam, "f64", 1)
        self.factors[side][self._rows(side, lo, hi)] = torch.from_numpy(out)

    def sq_error(self, side):
        rp, col, rat, off, n_opp = self.blocks[0]
        s = self.oracle.Side(ids=np.arange(len(rp) - 1), row_ptr=rp, col=col, ratings=rat)
        rows = self._rows(0, 0, len(rp) - 1)
        return self.oracle.sq_error(s, self.factors[0][rows].numpy(), self.factors[1][:n_opp].numpy())


def _worker(rank, world, port, path, out_dir, chunks=4, movie_chunks=None):
    import sys
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import torch.distributed as dist
    import __graft_entry__
    cfk = __graft_entry__.load_package()
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    ds = cfk.Dataset.load_netflix(path)
    app = cfk.ALSApp(4, 10, 0.05, 3, precision="f64", seed=42, rank=rank, world_size=world, overlap_chunks=chunks,
                     movie_chunks=movie_chunks)
    app.setup(ds, engine_factory=OracleShardEngine)
    app.run()
    U, M = app.factors()
    mse = app.mse()
    np.savez(os.path.join(out_dir, f"rank{rank}.npz"), U=U, M=M, mse=mse)
    dist.destroy_process_group()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.parametrize("world,chunks,movie_chunks", [(2, 1, None), (2, 4, None), (2, 4, 3), (3, 3, 2), (4, 7, None)])
def test_sharded_driver_matches_single_process(cfk, oracle_mod, tiny_path, tmp_path, world, chunks, movie_chunks):
    """chunks > 1: the user half is solved in row-range chunks over chunk-major user slots; each chunk's
    all-gather (async, one contiguous all_gather_into_tensor) overlaps the next chunk's solve. movie_chunks > 1:
    the movie half the same way (chunk-major movie slots; automatic above ALSApp.MOVIE_CHUNK_BYTES)."""
    import torch.multiprocessing as mp
    mp.spawn(_worker, args=(world, _free_port(), tiny_path, str(tmp_path), chunks, movie_chunks), nprocs=world,
             join=True)
    m, u, r = oracle_mod.parse_netflix(tiny_path)
    b = oracle_mod.build_blocks(m, u, r)
    Uo, Mo = oracle_mod.run_als(b, 10, 0.05, 3, seed=42, precision="f64")
    mse_o = oracle_mod.mse(b, Uo, Mo)
    for rank in range(world):
        res = np.load(os.path.join(tmp_path, f"rank{rank}.npz"))
        np.testing.assert_allclose(res["U"], Uo, rtol=1e-12, atol=1e-12)
        np.testing.assert_allclose(res["M"], Mo, rtol=1e-12, atol=1e-12)
        # f64 factors -> sum of squared errors in f64 (the stand-in); oracle MSE uses fp32 predictions
        assert abs(float(res["mse"]) - mse_o) < 1e-6


def _check_worker(rank, world, port, path, out_dir, perturb_rank):
    """ALSApp.verify_replicas (bench.py's self-check of a sharded run) over gloo: after the run, and after rank
    `perturb_rank` alters one word of its user-factor replica (-1: none)."""
    import json
    import sys
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import torch.distributed as dist
    import __graft_entry__
    cfk = __graft_entry__.load_package()
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    ds = cfk.Dataset.load_netflix(path)
    app = cfk.ALSApp(4, 10, 0.05, 2, precision="f64", seed=42, rank=rank, world_size=world, overlap_chunks=2)
    app.setup(ds, engine_factory=OracleShardEngine)
    app.run()
    before = app.verify_replicas()
    if rank == perturb_rank:
        app.engine.factors[1][3, 1] += 1e-9
    after = app.verify_replicas()
    with open(os.path.join(out_dir, f"check{rank}.json"), "w") as f:
        json.dump({"before": before, "after": after}, f)
    dist.destroy_process_group()


@pytest.mark.parametrize("world,perturb", [(2, 1), (3, 0), (3, -1)])
def test_replica_self_check(tiny_path, tmp_path, world, perturb):
    """The multi-GPU run's self-check (bench.py fields replicas_agree / integrity_clean): every rank's replicas of both
    factor matrices agree bitwise after the exchange; one word changed on one rank flips replicas_agree on EVERY rank
    (bench.py then exits with status 3), the digests of the other ranks unchanged."""
    import json
    import torch.multiprocessing as mp
    mp.spawn(_check_worker, args=(world, _free_port(), tiny_path, str(tmp_path), perturb), nprocs=world, join=True)
    res = [json.load(open(os.path.join(tmp_path, f"check{r}.json"))) for r in range(world)]
    for r in res:
        assert r["before"]["replicas_agree"] and r["before"]["integrity_clean"], r
        assert r["after"]["replicas_agree"] == (perturb < 0), r
        assert r["after"]["integrity_clean"]
    assert len({tuple(r["before"]["digest"]) for r in res}) == 1
    for i, r in enumerate(res):
        assert (r["after"]["digest"] == r["before"]["digest"]) == (i != perturb)
