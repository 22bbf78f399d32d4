"""GPU: the split-row hand-off check (PARTIAL -> REDUCE partial slots) and the reference's full rating range.

- Every partial slot is stored keyed by its launch generation with a check word (SlotCodec, als_kernels.hip);
  a REDUCE task that reads a slot its PARTIAL task's writes have not reached -- including a slot left over
  from an earlier launch with identical numbers -- fails the check and the engine's next synchronising call
  returns ALS_ERR_INTEGRITY.
- Ratings are Java shorts (Short.parseShort, NetflixDataFormatProducer.java:50; (float) of the short,
  MFeatureCalculator.java:80): every Gram path must be exact for |r| up to 32768, not only for 1..5.
"""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

LAM = 0.05


@pytest.fixture(autouse=True)
def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


def _engine(cfk, k, precision, side, blk, n_opp, opp_f):
    eng = cfk.ALSEngine(k, precision)
    eng.alloc_factors(1 - side, n_opp)
    eng.alloc_factors(side, max(1, blk["n_rows"]))
    eng.set_block(side, blk["row_ptr"], blk["col"], blk["ratings"], 0, n_opp)
    eng.write_factors(1 - side, opp_f)
    return eng


def _split_row_data(cfk, oracle_mod, ratings=None, seed=3):
    ds = cfk.Dataset.synthetic_netflix(n_users=2000, n_movies=150, nnz=60_000, seed=seed, nthreads=8)
    m, u, r = ds.ratings()
    if ratings is not None:
        r = np.random.default_rng(seed).choice(np.asarray(ratings, np.int16), size=len(r))
        ds = cfk.Dataset.from_ratings(m, u, r)
    return ds, oracle_mod.build_blocks(m, u, r)


def test_integrity_clean_on_split_rows(cfk, oracle_mod, monkeypatch):
    """Split rows (chunk 64: every movie row of degree > 64 becomes PARTIAL tasks + a REDUCE task), repeated
    halves: no slot ever fails its check, and the record is readable."""
    monkeypatch.setenv("ALS_CHUNK", "64")
    ds, b = _split_row_data(cfk, oracle_mod)
    for k, prec in ((64, "f32"), (128, "f32"), (10, "f64")):
        F = np.random.default_rng(1).random((len(b.user.ids), k))
        F = F.astype(np.float32 if prec == "f32" else np.float64)
        eng = _engine(cfk, k, prec, 0, ds.shard_block(0), len(b.user.ids), F)
        assert eng.block_stats(0)["n_reduce"] > 0
        for _ in range(5):
            eng.solve_half(0, LAM)
        eng.synchronize()
        assert eng.integrity_status() == [0, 0, 0, 0]
        eng.close()


@pytest.mark.parametrize("k,prec", [(64, "f32"), (128, "f32"), (32, "f32"), (10, "f64")])
def test_integrity_check_catches_foreign_slots(cfk, oracle_mod, monkeypatch, k, prec):
    """Fault injection: the REDUCE launch decodes with another launch's generation (ALS_DEBUG_REDUCE_GEN_SKEW),
    which is exactly what a slot still holding an earlier launch's sums looks like. Every such read must be
    caught, reported with its slot and row, and cleared by a reset."""
    monkeypatch.setenv("ALS_CHUNK", "64")
    monkeypatch.setenv("ALS_DEBUG_REDUCE_GEN_SKEW", "1")
    ds, b = _split_row_data(cfk, oracle_mod)
    F = np.random.default_rng(2).random((len(b.user.ids), k)).astype(np.float32 if prec == "f32" else np.float64)
    eng = _engine(cfk, k, prec, 0, ds.shard_block(0), len(b.user.ids), F)
    st = eng.block_stats(0)
    eng.solve_half(0, LAM)
    from cfk_amd._lib import ALSError
    with pytest.raises(ALSError, match="ALS_ERR_INTEGRITY"):
        eng.read_factors(0)
    rec = eng.integrity_status(reset=True)
    # every REDUCE task fails (the record counts failing REDUCE tasks)
    n_slots = st["n_tasks"] - (len(b.movie.ids) - st["n_reduce"])
    assert rec[0] == st["n_reduce"], (rec, st)
    assert rec[2] < n_slots and rec[3] < len(b.movie.ids)
    assert eng.integrity_status() == [0, 0, 0, 0]
    eng.read_factors(0)   # cleared: synchronising calls succeed again
    eng.close()


def _check_vs_oracle(got32, ref, ref32):
    """test_gpu_parity.test_one_half_every_k_vs_oracle's bar: within the reference's own fp32 envelope."""
    norm = np.linalg.norm(ref, axis=1)
    zero = norm == 0                      # every rating of the row is 0: the solution is exactly 0
    assert np.all(got32[zero] == 0)
    got32, ref, ref32, norm = got32[~zero], ref[~zero], ref32[~zero], norm[~zero]
    rel = np.linalg.norm(got32 - ref, axis=1) / norm
    rel_ref = np.linalg.norm(ref32 - ref, axis=1) / norm
    assert np.percentile(rel, 99) <= max(2 * np.percentile(rel_ref, 99), 2e-5), (np.percentile(rel, 99),)
    assert rel.max() <= max(3 * rel_ref.max(), 1e-4), (rel.max(), rel_ref.max())


@pytest.mark.parametrize("k", [64, 128])
@pytest.mark.parametrize("presplit_env", [None, "1", "0"])
def test_extreme_short_ratings_every_path(cfk, oracle_mod, monkeypatch, k, presplit_env):
    """Ratings from {-32768, -1, 0, 257, 32767} (257 and 32767 are not bf16 numbers): both halves at k = 64 and
    128 against the fp64 oracle. The user half at k = 64 is the pre-split candidate (small movie table); the
    engine must not feed these ratings to its bf16 RHS operand, even when ALS_PRESPLIT=1 asks for it."""
    if presplit_env is not None:
        monkeypatch.setenv("ALS_PRESPLIT", presplit_env)
    ds, b = _split_row_data(cfk, oracle_mod, ratings=[-32768, -1, 0, 257, 32767], seed=5)
    rng = np.random.default_rng(k)
    for side, rows, opp in ((0, b.movie, b.user), (1, b.user, b.movie)):
        F = rng.random((len(opp.ids), k))
        ref = oracle_mod.update_side(rows, F, LAM, "f64")
        ref32 = oracle_mod.update_side(rows, F.astype(np.float32), LAM, "f32")
        eng = _engine(cfk, k, "f32", side, ds.shard_block(side), len(opp.ids), F.astype(np.float32))
        assert not eng.block_path(side)["presplit"]          # |r| > 256: never the bf16 RHS operand
        eng.solve_half(side, LAM)
        got = eng.read_factors(side)
        eng.close()
        _check_vs_oracle(got, ref, ref32)


def test_presplit_path_with_bf16_exact_extreme_ratings(cfk, oracle_mod):
    """Ratings in [-256, 256] are bf16 numbers: the pre-split user half (k = 64, small movie table) stays on its
    MFMA RHS and must still be within the reference's fp32 envelope."""
    ds, b = _split_row_data(cfk, oracle_mod, ratings=[-256, -255, -1, 0, 1, 255, 256], seed=6)
    F = np.random.default_rng(9).random((len(b.movie.ids), 64))
    ref = oracle_mod.update_side(b.user, F, LAM, "f64")
    ref32 = oracle_mod.update_side(b.user, F.astype(np.float32), LAM, "f32")
    eng = _engine(cfk, 64, "f32", 1, ds.shard_block(1), len(b.movie.ids), F.astype(np.float32))
    bp = eng.block_path(1)
    assert bp["gram_path"] == "mfma_split" and bp["presplit"]
    eng.solve_half(1, LAM)
    got = eng.read_factors(1)
    eng.close()
    _check_vs_oracle(got, ref, ref32)
