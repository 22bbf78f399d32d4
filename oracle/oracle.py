"""CPU ORACLE -- TEST INFRASTRUCTURE ONLY.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may import this
module, and only as the checker (or the timed CPU baseline). The product package
(``collaborative-filtering-kafka_amd/``) never imports it.

Python restatement of the reference topology around the hot path; the per-entity arithmetic lives in
``als_oracle.c`` (see its header). Each function cites the reference file:line it follows
(paths relative to the reference's ``src/main/java/de/hpi/collaborativefilteringkafka/``).

Pinning (see DESIGN.md "Oracle"): the reference ships no tests or golden vectors and its Java/Kafka path
cannot run here (no JDK), so the oracle is pinned by (1) exact-rational known-answer systems
(tests/golden/known_answers.json), (2) the reference's own ``scripts/calculate_mse.py`` run on this
oracle's CSV output (tests/golden/*_mse_reference.json), and (3) the README's published MSE values
(README.md:211-212), which are loose because the reference's init is unseeded.
"""
from __future__ import annotations

import ctypes
import os
import subprocess
from dataclasses import dataclass, field

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "build", "liboracle.so")
_lib = None


def build() -> str:
    """Compile the C restatement (gcc) into oracle/build/liboracle.so."""
    subprocess.run(["make", "-s", "-C", _HERE], check=True)
    return _LIB_PATH


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        L = ctypes.CDLL(_LIB_PATH)
        i64p = ctypes.POINTER(ctypes.c_int64)
        i32p = ctypes.POINTER(ctypes.c_int32)
        i16p = ctypes.POINTER(ctypes.c_int16)
        f32p = ctypes.POINTER(ctypes.c_float)
        f64p = ctypes.POINTER(ctypes.c_double)
        L.oracle_u01.restype = ctypes.c_float
        L.oracle_u01.argtypes = [ctypes.c_uint64, ctypes.c_int64, ctypes.c_int32]
        L.oracle_init_user_features.restype = None
        L.oracle_init_user_features.argtypes = [ctypes.c_int64, i64p, i64p, i16p, ctypes.c_int,
                                                ctypes.c_uint64, f32p]
        for suf, fp in (("f32", f32p), ("f64", f64p)):
            fn = getattr(L, "oracle_update_" + suf)
            fn.restype = ctypes.c_int
            fn.argtypes = [ctypes.c_int64, i64p, i32p, i16p, fp, ctypes.c_int, ctypes.c_float, fp,
                           ctypes.c_int]
            fn = getattr(L, "oracle_sq_error_" + suf)
            fn.restype = ctypes.c_double
            fn.argtypes = [ctypes.c_int64, i64p, i32p, i16p, fp, fp, ctypes.c_int, i64p]
        L.oracle_update_rows_f64.restype = ctypes.c_int
        L.oracle_update_rows_f64.argtypes = [ctypes.c_int64, i64p, i64p, i32p, i16p, f64p, ctypes.c_int,
                                             ctypes.c_float, f64p]
        L.oracle_invert_f64.restype = ctypes.c_int
        L.oracle_invert_f64.argtypes = [f64p, ctypes.c_int]
        L.oracle_invert_f32.restype = ctypes.c_int
        L.oracle_invert_f32.argtypes = [f32p, ctypes.c_int]
        L.oracle_max_threads.restype = ctypes.c_int
        _lib = L
    return _lib


def _p(a, ct):
    return a.ctypes.data_as(ctypes.POINTER(ct))


# ------------------------------------------------------------------------------------------------
# Ingest: NetflixDataFormatProducer.runProducer (producers/NetflixDataFormatProducer.java:44-60)
# ------------------------------------------------------------------------------------------------
def parse_netflix(path: str):
    """Return (movie_ids, user_ids, ratings) int arrays in file (= producer send) order.

    ``row.endsWith(":")`` starts a movie (``Integer.parseInt(row.split(":")[0])``); any other line is
    ``userId,rating,date`` -> ``(Integer.parseInt(split[0]), Short.parseShort(split[1]))``.
    """
    movies, users, ratings = [], [], []
    current = -1
    with open(path, "r") as f:
        for line in f:
            row = line.rstrip("\r\n")
            if row.endswith(":"):
                current = int(row.split(":")[0])
            else:
                split = row.split(",")
                movies.append(current)
                users.append(int(split[0]))
                ratings.append(int(split[1]))
    return (np.asarray(movies, np.int64), np.asarray(users, np.int64), np.asarray(ratings, np.int16))


# ------------------------------------------------------------------------------------------------
# Block build: MRatings2BlocksProcessor.process (:48-69) and URatings2BlocksProcessor.process (:72-92)
# ------------------------------------------------------------------------------------------------
@dataclass
class Side:
    ids: np.ndarray            # ascending raw ids of entities with >=1 rating (dense index = position)
    row_ptr: np.ndarray        # int64 [n+1]
    col: np.ndarray            # int32 dense index into the opposite side
    ratings: np.ndarray        # int16
    out_blocks: list = field(default_factory=list)   # per row: partitions in first-appearance order


@dataclass
class Blocks:
    movie: Side
    user: Side


def build_blocks(movie_ids, user_ids, ratings, num_partitions: int = 1) -> Blocks:
    """In-blocks = ordered (otherId, rating) lists (CSR rows); out-blocks = ordered partition sets.

    Movie rows keep arrival (= file) order (MRatings2BlocksProcessor.java:52-58). User rows are filled
    from the re-keyed stream (MRatings2BlocksProcessor.java:71); the reference interleaves P upstream
    tasks non-deterministically, this restatement uses the P=1 interleaving (file order), which is one
    of the reference's admissible orders.
    """
    m_uniq = np.unique(movie_ids)
    u_uniq = np.unique(user_ids)
    m_dense = np.searchsorted(m_uniq, movie_ids)
    u_dense = np.searchsorted(u_uniq, user_ids)

    def csr(row_dense, col_dense, n_rows, col_raw):
        order = np.argsort(row_dense, kind="stable")   # stable: keeps arrival order inside a row
        counts = np.bincount(row_dense, minlength=n_rows)
        row_ptr = np.zeros(n_rows + 1, np.int64)
        np.cumsum(counts, out=row_ptr[1:])
        col = col_dense[order].astype(np.int32)
        rat = ratings[order].astype(np.int16)
        out_blocks = []
        raw = col_raw[order]
        for r in range(n_rows):
            seen = []
            for other in raw[row_ptr[r]:row_ptr[r + 1]]:
                p = int(other) % num_partitions        # PureModStreamPartitioner.java:9-10
                if p not in seen:
                    seen.append(p)
            out_blocks.append(seen)
        return row_ptr, col, rat, out_blocks

    mrp, mcol, mrat, mout = csr(m_dense, u_dense, len(m_uniq), user_ids)
    urp, ucol, urat, uout = csr(u_dense, m_dense, len(u_uniq), movie_ids)
    return Blocks(Side(m_uniq, mrp, mcol, mrat, mout), Side(u_uniq, urp, ucol, urat, uout))


# ------------------------------------------------------------------------------------------------
# U0: UFeatureInitializer.process (:43-56)
# ------------------------------------------------------------------------------------------------
def init_user_features(user: Side, k: int, seed: int) -> np.ndarray:
    out = np.zeros((len(user.ids), k), np.float32)
    ids = np.ascontiguousarray(user.ids, np.int64)
    lib().oracle_init_user_features(len(ids), _p(ids, ctypes.c_int64), _p(user.row_ptr, ctypes.c_int64),
                                    _p(user.ratings, ctypes.c_int16), k, seed, _p(out, ctypes.c_float))
    return out


def u01(seed: int, raw_id: int, feature: int) -> float:
    return lib().oracle_u01(seed, raw_id, feature)


# ------------------------------------------------------------------------------------------------
# Hot path: {M,U}FeatureCalculator.process solve block (:66-104), whole side at once
# ------------------------------------------------------------------------------------------------
def update_side(side: Side, opp: np.ndarray, lam: float, precision: str = "f64", nthreads: int = 0) -> np.ndarray:
    k = opp.shape[1]
    n = len(side.row_ptr) - 1
    if precision == "f64":
        opp = np.ascontiguousarray(opp, np.float64)
        out = np.zeros((n, k), np.float64)
        fn, ct = lib().oracle_update_f64, ctypes.c_double
    else:
        opp = np.ascontiguousarray(opp, np.float32)
        out = np.zeros((n, k), np.float32)
        fn, ct = lib().oracle_update_f32, ctypes.c_float
    nt = nthreads if nthreads > 0 else lib().oracle_max_threads()
    rc = fn(n, _p(side.row_ptr, ctypes.c_int64), _p(side.col, ctypes.c_int32), _p(side.ratings, ctypes.c_int16),
            _p(opp, ct), k, float(np.float32(lam)), _p(out, ct), nt)
    assert rc == 0
    return out


def ejml_invert(a: np.ndarray, precision: str = "f64") -> np.ndarray:
    """CommonOps_FDRM.invert (MFeatureCalculator.java:98) as restated in als_oracle.c: cofactors for k <= 5
    (UnrolledInverseFromMinor_FDRM), the LU solver beyond."""
    dt, fn, ct = (np.float64, lib().oracle_invert_f64, ctypes.c_double) if precision == "f64" else \
        (np.float32, lib().oracle_invert_f32, ctypes.c_float)
    out = np.ascontiguousarray(a, dt).copy()
    assert fn(_p(out, ct), out.shape[0]) == 0
    return out


def update_rows_f64(row_ptr, col, ratings, rows, opp, lam):
    """Oracle update for a selected subset of CSR rows (spot checks at full size)."""
    rows = np.ascontiguousarray(rows, np.int64)
    opp = np.ascontiguousarray(opp, np.float64)
    k = opp.shape[1]
    out = np.zeros((len(rows), k), np.float64)
    rc = lib().oracle_update_rows_f64(len(rows), _p(rows, ctypes.c_int64),
                                      _p(np.ascontiguousarray(row_ptr, np.int64), ctypes.c_int64),
                                      _p(np.ascontiguousarray(col, np.int32), ctypes.c_int32),
                                      _p(np.ascontiguousarray(ratings, np.int16), ctypes.c_int16),
                                      _p(opp, ctypes.c_double), k, float(np.float32(lam)), _p(out, ctypes.c_double))
    assert rc == 0
    return out


def sq_error(side: Side, row_f: np.ndarray, col_f: np.ndarray):
    k = row_f.shape[1]
    cnt = ctypes.c_int64(0)
    if row_f.dtype == np.float64:
        se = lib().oracle_sq_error_f64(len(side.row_ptr) - 1, _p(side.row_ptr, ctypes.c_int64),
                                       _p(side.col, ctypes.c_int32), _p(side.ratings, ctypes.c_int16),
                                       _p(np.ascontiguousarray(row_f), ctypes.c_double),
                                       _p(np.ascontiguousarray(col_f, np.float64), ctypes.c_double), k,
                                       ctypes.byref(cnt))
    else:
        se = lib().oracle_sq_error_f32(len(side.row_ptr) - 1, _p(side.row_ptr, ctypes.c_int64),
                                       _p(side.col, ctypes.c_int32), _p(side.ratings, ctypes.c_int16),
                                       _p(np.ascontiguousarray(row_f, np.float32), ctypes.c_float),
                                       _p(np.ascontiguousarray(col_f, np.float32), ctypes.c_float), k,
                                       ctypes.byref(cnt))
    return se, cnt.value


# ------------------------------------------------------------------------------------------------
# Topology: ALSApp.getTopology (:115-163) iteration semantics + FeatureCollector (:72-110)
# ------------------------------------------------------------------------------------------------
def run_als(blocks: Blocks, k: int, lam: float, iterations: int, seed: int = 42, precision: str = "f64",
            nthreads: int = 0, u0: np.ndarray | None = None):
    """U0 -> for i in 0..N-1: M_i = update(movies | U_i); U_{i+1} = update(users | M_i).

    Final output is (U_N, M_{N-1}) (MFeatureCalculator.java:117-123 sends M_{N-1} to movie-features-N,
    UFeatureCalculator.java:117-123 sends U_N to user-features-N). Unlike the reference (iteration number
    parsed from the last topic-name character, MFeatureCalculator.java:107), any N is allowed.
    """
    U = init_user_features(blocks.user, k, seed) if u0 is None else u0
    U = U.astype(np.float64 if precision == "f64" else np.float32)
    M = None
    for _ in range(iterations):
        M = update_side(blocks.movie, U, lam, precision, nthreads)
        U = update_side(blocks.user, M, lam, precision, nthreads)
    return U, M


def prediction_matrix(U: np.ndarray, M: np.ndarray) -> np.ndarray:
    """FeatureCollector.calculatePredictionMatrix (:90-101): fp32 U.M^T widened to double.

    EJML MatrixMatrixMult_FDRM.multTransB is a sequential float dot (total = 0; total += a*b), restated with
    element-wise float32 numpy ops (one rounding per * and +, features in ascending order)."""
    U32 = U.astype(np.float32)
    M32 = M.astype(np.float32)
    P = np.zeros((U32.shape[0], M32.shape[0]), np.float32)
    for f in range(U32.shape[1]):
        P += U32[:, f:f + 1] * M32[None, :, f]
    return P.astype(np.float64)


def java_double_str(v: float) -> str:
    """Java Double.toString layout over the shortest round-trip digits: plain decimal with at least one
    fraction digit for 1e-3 <= |v| < 1e7, otherwise ``d.dddE<exp>``."""
    import decimal
    import math
    if math.isnan(v):
        return "NaN"
    if math.isinf(v):
        return "Infinity" if v > 0 else "-Infinity"
    if v == 0.0:
        return "-0.0" if math.copysign(1.0, v) < 0 else "0.0"
    sign, digits, exp = decimal.Decimal(repr(v)).as_tuple()
    ds = "".join(map(str, digits)).rstrip("0") or "0"
    exp10 = exp + len(digits) - 1               # value = d.ddd * 10^exp10
    a = abs(v)
    if 1e-3 <= a < 1e7:
        if exp10 >= 0:
            ip = ds[:exp10 + 1].ljust(exp10 + 1, "0")
            fp = ds[exp10 + 1:] or "0"
            out = ip + "." + fp
        else:
            out = "0." + "0" * (-exp10 - 1) + ds
    else:
        out = ds[0] + "." + (ds[1:] or "0") + "E" + str(exp10)
    return ("-" if sign else "") + out


def save_dense_csv(P: np.ndarray, path: str) -> None:
    """EJML MatrixIO.saveDenseCSV layout (FeatureCollector.java:103-106): header ``rows cols real``,
    then per row every value (Double.toString) followed by one space."""
    with open(path, "w") as f:
        f.write(f"{P.shape[0]} {P.shape[1]} real\n")
        for row in P:
            f.write("".join(java_double_str(float(v)) + " " for v in row))
            f.write("\n")


def mse_from_csv(ratings_path: str, csv_path: str) -> float:
    """scripts/calculate_mse.py:11-90 restated (users sorted -> rows; movies in file order -> columns)."""
    m, u, r = parse_netflix(ratings_path)
    users = np.unique(u)
    movies_in_order = []
    for mid in m:
        if not movies_in_order or movies_in_order[-1] != mid:
            movies_in_order.append(int(mid))
    col_of = {mid: c for c, mid in enumerate(movies_in_order)}
    rows = np.searchsorted(users, u)
    cols = np.asarray([col_of[int(x)] for x in m])
    P = []
    with open(csv_path) as f:
        for line in f:
            if "real" in line:
                continue
            P.append([float(c) for c in line.strip().split(" ")])
    P = np.asarray(P)
    d = r.astype(np.float64) - P[rows, cols]
    return float(np.sum(d * d) / len(d))


def mse(blocks: Blocks, U: np.ndarray, M: np.ndarray) -> float:
    """MSE over observed ratings with fp32 predictions (FeatureCollector.java:92 + calculate_mse.py:78-90)."""
    se, cnt = sq_error(blocks.movie, M.astype(np.float32), U.astype(np.float32))
    return se / cnt
