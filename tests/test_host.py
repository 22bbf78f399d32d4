"""CPU: the C-ABI library loads and exports every declared symbol; the native host data layer (ingest,
in-blocks, sharding, U0, CSV) matches the oracle exactly; error behaviour. No kernel launches here."""
import gzip
import os
import re
import subprocess

import numpy as np
import pytest

from conftest import GOLDEN, ROOT


def _declared_symbols():
    names = []
    for h in ("als.h", "als_host.h"):
        src = open(os.path.join(ROOT, "include", h)).read()
        names += re.findall(r"^\s*(?:int|int64_t|float|const char\*)\s+(als_\w+)\s*\(", src, flags=re.M)
    return names


def test_library_exports_every_declared_symbol(cfk):
    from cfk_amd import _lib
    L = _lib.lib()
    declared = _declared_symbols()
    assert len(declared) >= 30
    for name in declared:
        assert hasattr(L, name), name
    assert sorted(declared) == sorted(_lib.exported_symbols())
    nm = subprocess.run(["nm", "-D", "--defined-only", _lib.LIB_PATH], capture_output=True, text=True).stdout
    for name in declared:
        assert re.search(rf"\bT {name}\b", nm), name
    assert L.als_abi_version() == 3


def test_library_carries_its_source_digest(cfk):
    """A library built by __graft_entry__.build() has the digest of the sources it was compiled from inside the
    binary (als_build_source_sha256), equal to its BUILD_INFO.json stamp; an unstamped developer build returns ""."""
    import __graft_entry__
    from cfk_amd import _lib
    embedded = _lib.lib().als_build_source_sha256().decode()
    info = __graft_entry__.build_info("product")
    if info and info.get("lib_sha256") == __graft_entry__.sha256_file(os.path.realpath(_lib.LIB_PATH)):
        assert embedded == info["source_sha256"]
    assert embedded == "" or re.fullmatch(r"[0-9a-f]{64}", embedded), embedded


def test_kernels_are_gfx950_code_objects(cfk):
    from cfk_amd import _lib
    blob = open(_lib.LIB_PATH, "rb").read()
    assert b"hipv4-amdgcn-amd-amdhsa--gfx950" in blob      # the fat binary carries a gfx950 code object


def test_ingest_and_blocks_match_oracle(cfk, oracle_mod, tiny_path, medium_path):
    for path in (tiny_path, medium_path):
        ds = cfk.Dataset.load_netflix(path)
        m, u, r = oracle_mod.parse_netflix(path)
        mm, uu, rr = ds.ratings()
        assert np.array_equal(mm, m) and np.array_equal(uu, u) and np.array_equal(rr, r)
        b = oracle_mod.build_blocks(m, u, r, 4)
        assert ds.count_duplicates() == 0
        for side, o in ((0, b.movie), (1, b.user)):
            blk = ds.shard_block(side)
            assert np.array_equal(blk["row_ptr"], o.row_ptr)
            assert np.array_equal(blk["col"], o.col)
            assert np.array_equal(blk["ratings"], o.ratings)
            assert np.array_equal(blk["row_ids"], o.ids)
            assert np.array_equal(ds.ids(side), o.ids)


@pytest.mark.parametrize("G", [1, 2, 3, 4, 8])
def test_shards_partition_by_id_mod_g(cfk, medium_path, G):
    """PureModStreamPartitioner: shard = raw id % G; slots are shard-major; shards cover every rating once."""
    ds = cfk.Dataset.load_netflix(medium_path)
    full = {s: ds.shard_block(s) for s in (0, 1)}
    for side in (0, 1):
        ids = ds.ids(side)
        slots = ds.slots(side, G)
        info0 = ds.shard_info(side, G, 0)
        S = info0["slots_per_shard"]
        assert np.array_equal(slots // S, ids % G)
        assert len(np.unique(slots)) == len(ids) and slots.max() < G * S
        opp_slots = ds.slots(1 - side, G)
        total = 0
        for sh in range(G):
            blk = ds.shard_block(side, G, sh)
            assert blk["row_offset"] == sh * S
            assert np.all(blk["row_ids"] % G == sh) and np.all(np.diff(blk["row_ids"]) > 0)
            total += blk["nnz"]
            # every row equals the unsharded row with opposite indices mapped to slots
            dense = np.searchsorted(ids, blk["row_ids"])
            for i in range(0, blk["n_rows"], max(1, blk["n_rows"] // 50)):
                d = dense[i]
                f0, f1 = full[side]["row_ptr"][d], full[side]["row_ptr"][d + 1]
                c0, c1 = blk["row_ptr"][i], blk["row_ptr"][i + 1]
                assert np.array_equal(blk["col"][c0:c1], opp_slots[full[side]["col"][f0:f1]])
                assert np.array_equal(blk["ratings"][c0:c1], full[side]["ratings"][f0:f1])
        assert total == ds.nnz


def test_u0_matches_oracle(cfk, oracle_mod, tiny_path):
    ds = cfk.Dataset.load_netflix(tiny_path)
    m, u, r = oracle_mod.parse_netflix(tiny_path)
    b = oracle_mod.build_blocks(m, u, r)
    for k in (1, 5, 10, 64):
        assert np.array_equal(ds.init_user_factors(k, 42), oracle_mod.init_user_features(b.user, k, 42))
    for G in (2, 4):
        U0 = ds.init_user_factors(10, 42, G)
        assert np.array_equal(U0[ds.slots(1, G)], oracle_mod.init_user_features(b.user, 10, 42))
    assert cfk.u01(42, 7, 3) == oracle_mod.u01(42, 7, 3)


def test_prediction_csv_matches_oracle_bytes(cfk, oracle_mod, tiny_path, tmp_path):
    """Native writer == oracle EJML/Java layout byte for byte; the reference's calculate_mse.py MSE holds."""
    import json
    m, u, r = oracle_mod.parse_netflix(tiny_path)
    b = oracle_mod.build_blocks(m, u, r, 4)
    U, M = oracle_mod.run_als(b, 5, 0.05, 7, seed=42)
    out = tmp_path / "p.csv"
    cfk.write_prediction_csv(str(out), U.astype(np.float32), M.astype(np.float32))
    golden = gzip.open(os.path.join(GOLDEN, "tiny_k5_n7_seed42_prediction.csv.gz")).read()
    assert out.read_bytes() == golden
    ref = json.load(open(os.path.join(GOLDEN, "tiny_k5_n7_seed42_mse_reference.json")))
    assert oracle_mod.mse_from_csv(tiny_path, str(out)) == pytest.approx(ref["mse"], rel=1e-14)


def java_float_dots(U, M):
    """FeatureCollector's fp32 U M^T with Java float semantics: every product and partial sum rounded."""
    U = np.asarray(U, np.float32)
    M = np.asarray(M, np.float32)
    total = np.zeros((U.shape[0], M.shape[0]), np.float32)
    for f in range(U.shape[1]):
        total = (total + np.outer(U[:, f], M[:, f]).astype(np.float32)).astype(np.float32)
    return total


def test_prediction_matrix_csv_writer(cfk, oracle_mod, tiny_path, tmp_path):
    """als_write_prediction_matrix_csv(P) == als_write_prediction_csv(U, M) byte for byte when P holds the
    Java-float dots (the GPU collector's output contract, checked bitwise in tests/test_gpu_parity.py)."""
    m, u, r = oracle_mod.parse_netflix(tiny_path)
    b = oracle_mod.build_blocks(m, u, r, 4)
    U, M = oracle_mod.run_als(b, 5, 0.05, 7, seed=42)
    a, c = tmp_path / "a.csv", tmp_path / "c.csv"
    cfk.write_prediction_csv(str(a), U.astype(np.float32), M.astype(np.float32))
    cfk.write_prediction_matrix_csv(str(c), java_float_dots(U, M))
    assert a.read_bytes() == c.read_bytes()


def test_synthetic_powerlaw_generator(cfk):
    """configs[4] shape at small scale: exact nnz, no duplicates, every entity rated, heavy-tailed items."""
    ds = cfk.Dataset.synthetic_powerlaw(20_000, 2_000, 2_000_000, 5, 4)
    assert ds.counts() == (2_000, 20_000, 2_000_000) and ds.count_duplicates() == 0
    deg = np.diff(ds.shard_block(0)["row_ptr"])
    assert deg.min() >= 1 and deg.max() > 20 * np.median(deg)


@pytest.mark.parametrize("workload", ["powerlaw", "netflix"])
def test_shard_restricted_synthesis_equals_the_full_dataset(cfk, workload):
    """One process of the G-GPU bench holds only its shard's ratings (als_dataset_synthetic_*_shard): every query
    the sharded driver makes for its shard -- both sides' COO in-blocks, shard geometry, slot layout (chunked too),
    U0 -- equals the full dataset's."""
    nu, nm, nnz, G = 20_000, 1_500, 600_000, 3
    full = (cfk.Dataset.synthetic_powerlaw if workload == "powerlaw" else cfk.Dataset.synthetic_netflix)(
        nu, nm, nnz, 5, 4)
    full.set_slot_chunks(1, 2)
    u0 = full.init_user_factors(16, 42, G)
    for shard in range(G):
        part = cfk.Dataset.synthetic_shard(workload, nu, nm, nnz, 5, G, shard, nthreads=3)
        part.set_slot_chunks(1, 2)
        assert part.counts()[:2] == (nm, nu) and part.counts()[2] < nnz
        for side in (0, 1):
            assert part.shard_info(side, G, shard) == full.shard_info(side, G, shard)
            assert part.slot_layout(side, G) == full.slot_layout(side, G)
            a, b = part.shard_coo(side, G, shard), full.shard_coo(side, G, shard)
            for key in ("rows", "cols", "ratings"):
                assert np.array_equal(a[key], b[key]), (shard, side, key)
        assert np.array_equal(part.init_user_factors(16, 42, G), u0)


def test_synthetic_generator_shape(cfk):
    ds = cfk.Dataset.synthetic_netflix(n_users=20_000, n_movies=2_000, nnz=400_000, seed=5, nthreads=4)
    nm, nu, nnz = ds.counts()
    assert (nm, nu, nnz) == (2_000, 20_000, 400_000)
    assert ds.count_duplicates() == 0
    deg_m = np.diff(ds.shard_block(0)["row_ptr"])
    deg_u = np.diff(ds.shard_block(1)["row_ptr"])
    assert deg_m.min() >= 1 and deg_u.min() >= 1
    assert deg_m.max() > 8 * np.median(deg_m)           # heavy-tailed movies
    _, _, r = ds.ratings()
    hist = np.bincount(r, minlength=6)[1:] / len(r)
    assert np.allclose(hist, [0.0455, 0.0978, 0.2837, 0.3351, 0.2380], atol=0.01)
    # deterministic in the seed and independent of the thread count
    ds2 = cfk.Dataset.synthetic_netflix(n_users=20_000, n_movies=2_000, nnz=400_000, seed=5, nthreads=1)
    assert all(np.array_equal(a, b) for a, b in zip(ds.ratings(), ds2.ratings()))


def test_error_behaviour(cfk, tmp_path):
    from cfk_amd._lib import ALSError
    bad = tmp_path / "bad.txt"
    bad.write_text("1:\n5,3,2005-01-01\nnot-a-rating-line\n")
    with pytest.raises(ALSError, match="ALS_ERR_PARSE"):
        cfk.Dataset.load_netflix(str(bad))
    with pytest.raises(ALSError, match="ALS_ERR_IO"):
        cfk.Dataset.load_netflix(str(tmp_path / "missing.txt"))
    dup = cfk.Dataset.from_ratings([1, 1, 2], [7, 7, 7], [3, 4, 5])
    assert dup.count_duplicates() == 1
    with pytest.raises(ALSError, match="ALS_ERR_INVALID_ARGUMENT"):
        cfk.Dataset.from_ratings([1, -1], [7, 8], [3, 4])
    # engine creation without a GPU (or with bad args) fails loudly instead of falling back
    with pytest.raises(ALSError):
        cfk.ALSEngine(0, "f32")
    with pytest.raises(ALSError, match="ALS_ERR_UNSUPPORTED"):
        cfk.ALSEngine(1025, "f32")         # 1..1024 (beyond 128 fp32 / 64 fp64: the generic path)
    with pytest.raises(ALSError, match="ALS_ERR_UNSUPPORTED"):
        cfk.ALSEngine(2000, "f64")


def test_cli_arguments_missing_message():
    app = os.path.join(ROOT, "collaborative-filtering-kafka_amd", "build", "als_app")
    res = subprocess.run([app, "4", "10"], capture_output=True, text=True)
    assert res.returncode == 0 and "ARGUMENTS MISSING" in res.stdout      # ALSAppRunner.java:11-14


def test_shard_coo_is_arrival_order_of_the_in_blocks(cfk, tiny_path):
    """A stable sort of the COO export by row reproduces the host CSR in-blocks exactly (the contract the GPU
    block build of als_set_block_coo relies on)."""
    ds = cfk.Dataset.load_netflix(tiny_path)
    for G, shard in ((1, 0), (3, 1), (4, 3)):
        for side in (0, 1):
            csr = ds.shard_block(side, G, shard)
            coo = ds.shard_coo(side, G, shard)
            order = np.argsort(coo["rows"], kind="stable")
            assert np.array_equal(np.bincount(coo["rows"], minlength=csr["n_rows"]), np.diff(csr["row_ptr"]))
            assert np.array_equal(coo["cols"][order], csr["col"])
            assert np.array_equal(coo["ratings"][order], csr["ratings"])


def test_loader_long_lines_and_line_terminators(cfk, oracle_mod, tmp_path):
    """BufferedReader.readLine (NetflixDataFormatProducer.java:44): lines of any length (a rating line with a
    200 KB date field, far beyond any fixed buffer), and "\\n", "\\r\\n" and a lone "\\r" all end a line. The
    loader must read exactly what the oracle's universal-newline parse reads."""
    long_date = "2005-09-06" + "x" * 200_000
    text = ("1:\n6,3," + long_date + "\n7,4,2005-01-01\r\n8,5,2005-01-02\r2:\r\n6,1\n"
            "9,2," + long_date + "\r7,5,2004-12-31")          # last line without a terminator
    p = tmp_path / "long.txt"
    p.write_bytes(text.encode())
    ds = cfk.Dataset.load_netflix(str(p))
    m, u, r = ds.ratings()
    mo, uo, ro = oracle_mod.parse_netflix(str(p))
    assert list(m) == list(mo) == [1, 1, 1, 2, 2, 2]
    assert list(u) == list(uo) == [6, 7, 8, 6, 9, 7]
    assert list(r) == list(ro) == [3, 4, 5, 1, 2, 5]
