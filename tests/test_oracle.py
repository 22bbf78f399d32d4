"""CPU: pin the oracle (the checker) before anything is compared against it.

The reference ships no tests/golden vectors and its Java/Kafka path cannot run here, so the
oracle is pinned by: exact-rational known answers, the reference's own calculate_mse.py output on an
oracle CSV, the README's published MSE values (loose: unseeded reference init), and f32/f64 agreement.
"""
import gzip
import json
import os

import numpy as np
import pytest

from conftest import GOLDEN, max_rel


def _one_row_side(oracle, Y, r):
    """A one-entity in-block whose opposite factor rows are Y (n x k), ratings r."""
    n = len(Y)
    return oracle.Side(ids=np.array([1]), row_ptr=np.array([0, n], np.int64), col=np.arange(n, dtype=np.int32),
                       ratings=np.asarray(r, np.int16))


def test_known_answers_exact_rational(oracle_mod):
    cases = json.load(open(os.path.join(GOLDEN, "known_answers.json")))
    for c in cases:
        side = _one_row_side(oracle_mod, c["Y"], c["r"])
        Y = np.asarray(c["Y"], np.float64)
        x64 = oracle_mod.update_side(side, Y, 0.05, "f64")[0]
        np.testing.assert_allclose(x64, c["x"], rtol=1e-12, atol=1e-14)
        x32 = oracle_mod.update_side(side, Y.astype(np.float32), 0.05, "f32")[0]
        np.testing.assert_allclose(x32, c["x"], rtol=2e-4, atol=1e-5)


def test_u01_range_and_determinism(oracle_mod):
    vals = [oracle_mod.u01(42, i, f) for i in range(200) for f in range(1, 8)]
    assert all(0.0 <= v < 1.0 for v in vals)
    assert vals == [oracle_mod.u01(42, i, f) for i in range(200) for f in range(1, 8)]
    assert abs(np.mean(vals) - 0.5) < 0.05


def test_parse_and_blocks_tiny(oracle_mod, tiny_path):
    m, u, r = oracle_mod.parse_netflix(tiny_path)
    assert len(r) == 3415            # SURVEY §8a (README.md:211 claims 3,989)
    b = oracle_mod.build_blocks(m, u, r, 4)
    assert len(b.movie.ids) == 426 and len(b.user.ids) == 302
    # movie in-block order = file order (MRatings2BlocksProcessor.java:52-58)
    first = b.movie.row_ptr[0], b.movie.row_ptr[1]
    assert first == (0, 1) and b.user.ids[b.movie.col[0]] == 915
    # out-blocks: partitions of dependents in first-appearance order (MRatings2BlocksProcessor.java:54-56)
    for row in range(len(b.movie.ids)):
        deps = b.user.ids[b.movie.col[b.movie.row_ptr[row]:b.movie.row_ptr[row + 1]]]
        expect = []
        for d in deps:
            if d % 4 not in expect:
                expect.append(int(d % 4))
        assert b.movie.out_blocks[row] == expect


def test_readme_published_mse(oracle_mod, tiny_path, medium_path):
    """README.md:207-212: k=5, 7 iterations, lambda=0.05 -> tiny MSE 0.265, medium MSE 0.577 (unseeded init)."""
    for path, published, tol in ((tiny_path, 0.265, 0.025), (medium_path, 0.577, 0.012)):
        m, u, r = oracle_mod.parse_netflix(path)
        b = oracle_mod.build_blocks(m, u, r, 4)
        mses = []
        for seed in (1, 2, 3):
            U, M = oracle_mod.run_als(b, 5, 0.05, 7, seed=seed)
            mses.append(oracle_mod.mse(b, U, M))
        assert abs(np.mean(mses) - published) < tol, (path, mses)


def test_f32_port_tracks_f64(oracle_mod, medium_path):
    """Java-float restatement vs f64: MSE delta far inside the north star's 1e-3 fast-mode bound."""
    m, u, r = oracle_mod.parse_netflix(medium_path)
    b = oracle_mod.build_blocks(m, u, r, 4)
    U64, M64 = oracle_mod.run_als(b, 10, 0.05, 10, seed=42, precision="f64")
    U32, M32 = oracle_mod.run_als(b, 10, 0.05, 10, seed=42, precision="f32")
    assert abs(oracle_mod.mse(b, U64, M64) - oracle_mod.mse(b, U32, M32)) < 1e-5
    assert np.linalg.norm(U64 - U32) / np.linalg.norm(U64) < 1e-4


def test_golden_regenerates(oracle_mod, tiny_path):
    g = np.load(os.path.join(GOLDEN, "tiny_k10_n10_p4_seed42_f64.npz"))
    m, u, r = oracle_mod.parse_netflix(tiny_path)
    b = oracle_mod.build_blocks(m, u, r, 4)
    U, M = oracle_mod.run_als(b, 10, 0.05, 10, seed=42)
    assert max_rel(U, g["U"]) == 0.0 and max_rel(M, g["M"]) == 0.0
    assert oracle_mod.mse(b, U, M) == float(g["mse"])


def test_reference_calculate_mse_pins_csv_and_mse(oracle_mod, tiny_path, tmp_path):
    """The reference's scripts/calculate_mse.py printed this MSE for the oracle's CSV (make_golden.py)."""
    ref = json.load(open(os.path.join(GOLDEN, "tiny_k5_n7_seed42_mse_reference.json")))
    csv = tmp_path / "pred.csv"
    csv.write_bytes(gzip.open(os.path.join(GOLDEN, "tiny_k5_n7_seed42_prediction.csv.gz")).read())
    assert oracle_mod.mse_from_csv(tiny_path, str(csv)) == pytest.approx(ref["mse"], rel=1e-14)
    # regenerating the CSV reproduces the committed bytes
    m, u, r = oracle_mod.parse_netflix(tiny_path)
    b = oracle_mod.build_blocks(m, u, r, 4)
    U, M = oracle_mod.run_als(b, 5, 0.05, 7, seed=42)
    out = tmp_path / "regen.csv"
    oracle_mod.save_dense_csv(oracle_mod.prediction_matrix(U, M), str(out))
    assert out.read_bytes() == csv.read_bytes()
    # the observed-cell MSE of the fp32 prediction matrix equals the script's number
    assert oracle_mod.mse(b, U, M) == pytest.approx(ref["mse"], rel=1e-12)


def test_java_double_format(oracle_mod):
    f = oracle_mod.java_double_str
    assert f(float(np.float32(3.52))) == "3.5199999809265137"
    assert f(1.0) == "1.0" and f(100.0) == "100.0" and f(0.001) == "0.001"
    assert f(1e-5) == "1.0E-5" and f(1e7) == "1.0E7" and f(-2.5e-10) == "-2.5E-10" and f(0.0) == "0.0"


def test_ejml_invert_branches(oracle_mod):
    """CommonOps_FDRM.invert (MFeatureCalculator.java:98): UnrolledInverseFromMinor_FDRM for k <= 5, LU beyond.
    Both restated branches invert regularised Gram systems to f64 round-off, and the k = 2, 3 cofactor forms equal,
    bit for bit in float, the library's inv2 / inv3 expressions (scale by 1/max|a|, cofactors, det over scale)."""
    rng = np.random.default_rng(11)
    for k in range(1, 9):
        Y = rng.random((3 * k + 2, k))
        A = Y.T @ Y + 0.05 * len(Y) * np.eye(k)
        inv = oracle_mod.ejml_invert(A, "f64")
        assert np.abs(inv - np.linalg.inv(A)).max() <= 1e-12 * np.abs(np.linalg.inv(A)).max(), k
        inv32 = oracle_mod.ejml_invert(A.astype(np.float32), "f32")
        assert np.abs(inv32 - np.linalg.inv(A)).max() <= 1e-4 * np.abs(np.linalg.inv(A)).max(), k
    f = np.float32
    for k in (2, 3):
        Y = rng.random((7, k)).astype(f)
        A = (Y.T @ Y + f(0.35) * np.eye(k, dtype=f)).astype(f)
        mx = np.abs(A).max()
        sc = f(1) / mx
        a = A * sc
        if k == 2:
            m = np.array([[a[1, 1], -a[1, 0]], [-a[0, 1], a[0, 0]]], f)
            det = (a[0, 0] * m[0, 0] + a[0, 1] * m[0, 1]) / sc
        else:
            m = np.empty((3, 3), f)
            m[0, 0] = a[1, 1] * a[2, 2] - a[1, 2] * a[2, 1]
            m[0, 1] = -(a[1, 0] * a[2, 2] - a[1, 2] * a[2, 0])
            m[0, 2] = a[1, 0] * a[2, 1] - a[1, 1] * a[2, 0]
            m[1, 0] = -(a[0, 1] * a[2, 2] - a[0, 2] * a[2, 1])
            m[1, 1] = a[0, 0] * a[2, 2] - a[0, 2] * a[2, 0]
            m[1, 2] = -(a[0, 0] * a[2, 1] - a[0, 1] * a[2, 0])
            m[2, 0] = a[0, 1] * a[1, 2] - a[0, 2] * a[1, 1]
            m[2, 1] = -(a[0, 0] * a[1, 2] - a[0, 2] * a[1, 0])
            m[2, 2] = a[0, 0] * a[1, 1] - a[0, 1] * a[1, 0]
            det = ((a[0, 0] * m[0, 0] + a[0, 1] * m[0, 1]) + a[0, 2] * m[0, 2]) / sc
        want = (m / det).T.astype(f)
        got = oracle_mod.ejml_invert(A, "f32")
        assert np.array_equal(got, want), (k, got, want)
