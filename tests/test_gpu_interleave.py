"""Interleaved split rows of the movie half (ALS_INTERLEAVE) against the contiguous plan and
the oracle.

The interleaved plan changes the work plan, not the arithmetic of an update (MFeatureCalculator.java:66-104): a long
row's blocks are permuted chunk-major, each interleaved chunk is one PARTIAL task of the pre-split fp16 Gram (as the
user half), and the row's REDUCE task sums the chunks in order and solves. So the interleaved half must agree with the
contiguous plan and the fp64 oracle within the fp32 envelope, repeat bitwise, keep every partial slot intact and give
the same squared error (the permuted layout is also what als_sq_error walks).
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


def _engine(cfk, blocks, k, ilv, ranges=False):
    saved = {v: os.environ.get(v) for v in ("ALS_INTERLEAVE", "ALS_XCD_RANGES")}
    os.environ["ALS_INTERLEAVE"] = "1" if ilv else "0"
    os.environ["ALS_XCD_RANGES"] = "1" if ranges else "0"
    try:
        eng = cfk.ALSEngine(k, "f32")
    finally:
        for v, old in saved.items():
            if old is None:
                del os.environ[v]
            else:
                os.environ[v] = old
    eng.use_torch_stream()
    eng.alloc_factors(0, blocks[0]["n_slots"])
    eng.alloc_factors(1, blocks[1]["n_slots"])
    for side in (0, 1):
        b = blocks[side]
        eng.set_block(side, b["row_ptr"], b["col"], b["ratings"], 0, blocks[1 - side]["n_slots"])
    return eng


@pytest.mark.timeout(600)
def test_interleaved_matches_contiguous_plan_and_oracle(cfk, oracle_mod):
    """Netflix-shape at 1/8 scale (60k users x 2,200 movies x 12.5M ratings, k = 64), ALS_INTERLEAVE=1 forced (the
    table is below the auto threshold): the movie half of the interleaved engine vs the contiguous-plan engine from the
    same U, both against the fp64 oracle on rows of every length (the longest split in several chunks), bitwise repeat,
    clean integrity record, equal squared error; then a user half from each engine's M."""
    from test_gpu_fullscale import _check_rows
    ds = cfk.Dataset.synthetic_netflix(60_000, 2_200, 12_500_000, seed=0xA15, nthreads=16)
    blocks = [ds.shard_block(0), ds.shard_block(1)]
    k = 64
    sw = _engine(cfk, blocks, k, True)
    pl = _engine(cfk, blocks, k, False)
    info = sw.split_info(0)
    assert info["interleaved_rows"] > 0 and info["chunk_tasks"] > info["interleaved_rows"] and info["presplit"], info
    assert pl.split_info(0)["interleaved_rows"] == 0
    u0 = ds.init_user_factors(k, 42)
    for e in (sw, pl):
        e.write_factors(1, u0)
        e.solve_half(0, LAM)
    m_sw = sw.read_factors(0)
    m_pl = pl.read_factors(0)
    assert sw.integrity_status() == [0, 0, 0, 0]
    # both plans vs the fp64 oracle: the 20 longest (interleaved, several chunks) and random rows, within 3x the
    # reference's own fp32 error on the same rows (the first half from U0 is the worst-conditioned one)
    deg = np.diff(blocks[0]["row_ptr"])
    rng = np.random.default_rng(5)
    rows = np.unique(np.concatenate([np.argsort(-deg)[:20], rng.choice(len(deg), 120, replace=False)]))
    e_sw = _check_rows(oracle_mod, blocks[0], rows, m_sw, u0.astype(np.float64), "interleaved movie half")
    e_pl = _check_rows(oracle_mod, blocks[0], rows, m_pl, u0.astype(np.float64), "contiguous movie half")
    assert e_sw <= 3 * max(e_pl, 1e-7), (e_sw, e_pl)
    # bitwise repeat of the paced launch (static schedule, fixed chunk order)
    sw.write_factors(1, u0)
    sw.solve_half(0, LAM)
    assert np.array_equal(sw.read_factors(0), m_sw)
    # the squared error of the SAME factors over the permuted in-block equals the contiguous layout's (the same
    # entries, fp64 sums in another order)
    sw.write_factors(0, m_pl)
    se_sw, n_sw = sw.sq_error(0)
    se_pl, n_pl = pl.sq_error(0)
    assert n_sw == n_pl == ds.nnz
    assert abs(se_sw - se_pl) <= 1e-10 * se_pl, (se_sw, se_pl)
    sw.write_factors(0, m_sw)
    # the user half reads the interleaved engine's M like any other: sampled users vs the oracle on that M
    sw.solve_half(1, LAM)
    u_sw = sw.read_factors(1)
    udeg = np.diff(blocks[1]["row_ptr"])
    urows = np.unique(np.concatenate([np.argsort(-udeg)[:10], rng.choice(len(udeg), 200, replace=False)]))
    _check_rows(oracle_mod, blocks[1], urows, u_sw, m_sw.astype(np.float64), "user half after the interleaved M")
    assert sw.integrity_status() == [0, 0, 0, 0]


@pytest.mark.timeout(300)
def test_interleaved_plan_covers_every_entry_once(cfk):
    """The interleaved block's work plan: every rating is in exactly one task (the squared error counts nnz), every row
    longer than the chunk is interleaved, and a small block (the opposite table under the auto threshold) keeps the
    contiguous plan by default."""
    ds = cfk.Dataset.synthetic_netflix(30_000, 1_000, 6_000_000, seed=0xA16, nthreads=16)
    blocks = [ds.shard_block(0), ds.shard_block(1)]
    auto = cfk.ALSEngine(64, "f32")
    auto.alloc_factors(0, blocks[0]["n_slots"])
    auto.alloc_factors(1, blocks[1]["n_slots"])
    auto.set_block(0, blocks[0]["row_ptr"], blocks[0]["col"], blocks[0]["ratings"], 0, blocks[1]["n_slots"])
    assert auto.split_info(0)["interleaved_rows"] == 0   # 30k x 256 B user table: the L2s hold it
    sw = _engine(cfk, blocks, 64, True)
    info = sw.split_info(0)
    deg = np.diff(blocks[0]["row_ptr"])
    assert info["interleaved_rows"] == int((deg > info["chunk"]).sum()) > 0, info
    assert info["chunk_tasks"] == int(np.ceil(deg[deg > info["chunk"]] / info["chunk"]).sum())
    assert sw.block_stats(0)["n_reduce"] == info["interleaved_rows"]
    sw.write_factors(1, ds.init_user_factors(64, 42))
    sw.solve_half(0, LAM)
    se, n = sw.sq_error(0)
    assert n == ds.nnz and np.isfinite(se)
    # k = 128: a block whose long rows hold far fewer than 4 chunks of 16,384 entries per resident wave (every shard of
    # the Netflix shape) takes the 4,096-entry chunk, capped by the contiguous chunk length
    sw128 = _engine(cfk, blocks, 128, True)
    i128 = sw128.split_info(0)
    assert i128["chunk"] == min(4096, sw128.block_path(0)["chunk"]) and i128["interleaved_rows"] > 0, i128
    assert i128["interleaved_rows"] == int((deg > i128["chunk"]).sum())


@pytest.mark.timeout(300)
def test_xcd_range_pieces_cover_every_entry_and_match_the_oracle(cfk, oracle_mod):
    """ALS_XCD_RANGES: each long row cut into 8 opposite-slot ranges before the interleave, the
    chunks of range x ordered onto the workgroups of one XCD. Same arithmetic per chunk, another summation order: every
    entry in exactly one task, one REDUCE per long row, at least one chunk per range a row reaches, results against the
    fp64 oracle within 3x the plain interleaved plan's error, bitwise repeat, clean integrity record."""
    from test_gpu_fullscale import _check_rows
    ds = cfk.Dataset.synthetic_netflix(30_000, 1_000, 6_000_000, seed=0xA16, nthreads=16)
    blocks = [ds.shard_block(0), ds.shard_block(1)]
    k = 64
    rg = _engine(cfk, blocks, k, True, ranges=True)
    sw = _engine(cfk, blocks, k, True)
    deg = np.diff(blocks[0]["row_ptr"])
    i_rg, i_sw = rg.split_info(0), sw.split_info(0)
    assert i_rg["interleaved_rows"] == i_sw["interleaved_rows"] == int((deg > i_rg["chunk"]).sum()) > 0
    assert i_rg["chunk_tasks"] >= i_sw["chunk_tasks"]
    assert rg.block_stats(0)["n_reduce"] == i_rg["interleaved_rows"]
    u0 = ds.init_user_factors(k, 42)
    for e in (rg, sw):
        e.write_factors(1, u0)
        e.solve_half(0, LAM)
    m_rg, m_sw = rg.read_factors(0), sw.read_factors(0)
    assert rg.integrity_status() == [0, 0, 0, 0]
    rng = np.random.default_rng(7)
    rows = np.unique(np.concatenate([np.argsort(-deg)[:20], rng.choice(len(deg), 100, replace=False)]))
    e_rg = _check_rows(oracle_mod, blocks[0], rows, m_rg, u0.astype(np.float64), "XCD-range movie half")
    e_sw = _check_rows(oracle_mod, blocks[0], rows, m_sw, u0.astype(np.float64), "interleaved movie half")
    assert e_rg <= 3 * max(e_sw, 1e-7), (e_rg, e_sw)
    rg.write_factors(1, u0)
    rg.solve_half(0, LAM)
    assert np.array_equal(rg.read_factors(0), m_rg)
    rg.write_factors(0, m_sw)
    se_rg, n_rg = rg.sq_error(0)
    sw.write_factors(0, m_sw)
    se_sw, n_sw = sw.sq_error(0)
    assert n_rg == n_sw == ds.nnz and abs(se_rg - se_sw) <= 1e-10 * se_sw, (se_rg, se_sw)
