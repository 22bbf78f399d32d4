"""Row f3 / §8b: the JNI shim (integration/jni/cfk_als_jni.c, the binding AlsNative.java declares) EXECUTED.

There is no JDK in this image, so the unchanged shim is compiled against a test-only jni.h together with a mock JVM
(tests/jni: a copying JVM with per-thread JNIEnvs, pending exceptions, bounds- and type-checked array regions, release
modes honoured) and every Java_* entry point is called through ctypes exactly as the JVM would call it.

CPU (no GPU needed): every native of AlsNative.java is exported; als_status -> StreamsException carrying
als_last_error(); IllegalArgumentException on shape errors before any C ABI call; the collector CSV through
writePredictionMatrixCsv is byte-identical to the oracle's restatement of FeatureCollector.java:103-106.

GPU: the re-plumbed topology's use of the binding (TaskEngine.java: one engine per (stream task, side), compacted
opposite slots from the partition's in-blocks, one solveHalf per partition and half) on the tiny sample at P = 4,
k = 10, N = 10: 8 engines on one GPU driven by 4 host threads at once (BaseKafkaApp.java:51: 4 stream threads),
fp64 parity mode against tests/golden/tiny_k10_n10_p4_seed42_f64.npz within the north-star bar, fp32 within the fast
mode bar, and repeated threaded runs bitwise equal. Reference: MFeatureCalculator.java:49-136, ALSApp.java:115-151.
"""
from __future__ import annotations

import ctypes
import os
import threading

import numpy as np
import pytest

from conftest import GOLDEN, ROOT, max_rel

JNI_LIB = os.path.join(ROOT, "tests", "jni", "build", "libcfk_jni_mock.so")
PREFIX = "Java_de_hpi_collaborativefilteringkafka_nativeals_AlsNative_"
T_BYTE, T_SHORT, T_INT, T_LONG, T_FLOAT, T_DOUBLE = 1, 2, 3, 4, 5, 6
NP_TYPE = {np.int8: T_BYTE, np.int16: T_SHORT, np.int32: T_INT, np.int64: T_LONG, np.float32: T_FLOAT,
           np.float64: T_DOUBLE}
LAM = 0.05
P = 4            # NUM_PARTITIONS of the tiny config (BASELINE configs[0])
THREADS = 4      # BaseKafkaApp.java:51 NUM_STREAM_THREADS

_v, _i, _i64, _f = ctypes.c_void_p, ctypes.c_int, ctypes.c_int64, ctypes.c_float
# Java signature -> ctypes argument types after (JNIEnv*, jclass); arrays and strings are mock object handles
NATIVES = {
    "abiVersion": (_i, []), "deviceCount": (_i, []), "create": (_i64, [_i, _i, _i]), "destroy": (None, [_i64]),
    "setBlockCoo": (None, [_i64, _i, _i64, _i64, _i64, _v, _v, _v]), "allocFactors": (None, [_i64, _i, _i64]),
    "writeFactors": (None, [_i64, _i, _i64, _v, _i]), "readFactors": (None, [_i64, _i, _i64, _v, _i]),
    "writeFactorsF64": (None, [_i64, _i, _i64, _v, _i]), "readFactorsF64": (None, [_i64, _i, _i64, _v, _i]),
    "solveHalf": (None, [_i64, _i, _f]), "synchronize": (None, [_i64]), "commUniqueId": (_v, []),
    "commInit": (None, [_i64, _i, _i, _v]), "commSetTimeout": (None, [_i64, _i64]), "allgatherShard": (None, [_i64, _i, _i64, _i64]),
    "predict": (None, [_i64, _v, _v, _v]), "writePredictionMatrixCsv": (None, [_v, _v, _i64, _i64]),
}


class JavaException(Exception):
    def __init__(self, cls: str, msg: str):
        super().__init__(f"{cls}: {msg}")
        self.cls, self.msg = cls, msg


class MockJVM:
    """The JVM side of AlsNative: per-thread JNIEnv, Java arrays as mock objects, natives called by name."""

    def __init__(self):
        self.L = ctypes.CDLL(JNI_LIB)
        L = self.L
        L.mock_env_new.restype = _v
        L.mock_env_free.argtypes = [_v]
        L.mock_exception.argtypes = [_v, ctypes.c_char_p, _i, ctypes.c_char_p, _i, _i]
        L.mock_env_stats.argtypes = [_v, ctypes.POINTER(ctypes.c_long)]
        L.mock_array_new.restype = _v
        L.mock_array_new.argtypes = [_i, _i64, _v]
        L.mock_array_len.restype = _i64
        L.mock_array_len.argtypes = [_v]
        L.mock_array_read.argtypes = [_v, _v]
        L.mock_string_new.restype = _v
        L.mock_string_new.argtypes = [ctypes.c_char_p]
        L.mock_obj_free.argtypes = [_v]
        for name, (res, args) in NATIVES.items():
            fn = getattr(L, PREFIX + name)
            fn.restype = res
            fn.argtypes = [_v, _v] + args
        self._tls = threading.local()
        self._envs = []
        self._lock = threading.Lock()

    def env(self):
        e = getattr(self._tls, "env", None)
        if e is None:
            e = self.L.mock_env_new()
            self._tls.env = e
            with self._lock:
                self._envs.append(e)
        return e

    def stats(self, env=None) -> dict:
        out = (ctypes.c_long * 5)()
        self.L.mock_env_stats(env or self.env(), out)
        return dict(zip(("calls", "critical", "copies", "violations", "open_critical"), list(out)))

    def all_stats(self) -> list[dict]:
        return [self.stats(e) for e in self._envs]

    def call(self, name: str, *args):
        """A static native call: (env, jclass = NULL, args...); a pending exception is raised (and cleared)."""
        env = self.env()
        r = getattr(self.L, PREFIX + name)(env, None, *args)
        cls, msg = ctypes.create_string_buffer(256), ctypes.create_string_buffer(2048)
        if self.L.mock_exception(env, cls, 256, msg, 2048, 1):
            raise JavaException(cls.value.decode(), msg.value.decode())
        return r

    # Java arrays (copied in, as `new float[]{...}` would be)
    def array(self, a: np.ndarray):
        a = np.ascontiguousarray(a)
        return self.L.mock_array_new(NP_TYPE[a.dtype.type], a.size, a.ctypes.data_as(_v))

    def array_zeros(self, dtype, n: int):
        return self.L.mock_array_new(NP_TYPE[np.dtype(dtype).type], n, None)

    def read(self, arr, dtype) -> np.ndarray:
        out = np.zeros(self.L.mock_array_len(arr), dtype)
        self.L.mock_array_read(arr, out.ctypes.data_as(_v))
        return out

    def string(self, s: str):
        return self.L.mock_string_new(s.encode())

    def free(self, *objs):
        for o in objs:
            self.L.mock_obj_free(o)


@pytest.fixture(scope="module")
def jvm(cfk):
    cfk._lib.lib()            # libcfk_als.so first (after torch: one HIP runtime), then the shim that links it
    if not os.path.exists(JNI_LIB):
        pytest.fail(f"{JNI_LIB} not built (__graft_entry__.build() runs make -C tests/jni)")
    return MockJVM()


# ---------------------------------------------------------------------------------------------------------------
# CPU: the binding's surface and its error mapping
# ---------------------------------------------------------------------------------------------------------------
def test_every_java_native_is_exported(jvm):
    import re
    src = open(os.path.join(ROOT, "integration", "java", "de", "hpi", "collaborativefilteringkafka", "nativeals",
                            "AlsNative.java")).read()
    natives = set(re.findall(r"public\s+static\s+native\s+[\w\[\]]+\s+(\w+)\s*\(", src))
    assert natives == set(NATIVES), sorted(natives ^ set(NATIVES))
    for n in natives:
        assert hasattr(jvm.L, PREFIX + n)
    assert jvm.call("abiVersion") == 3


def test_status_becomes_streams_exception_with_last_error(jvm):
    with pytest.raises(JavaException) as ei:
        jvm.call("create", 0, 10, 7)                  # precision 7: ALS_ERR_INVALID_ARGUMENT before any device call
    assert ei.value.cls == "org/apache/kafka/streams/errors/StreamsException"
    assert "als_engine_create: als_status 1" in ei.value.msg and "precision must be ALS_F32 or ALS_F64" in ei.value.msg
    with pytest.raises(JavaException, match="num_features must be >= 1"):
        jvm.call("create", 0, 0, 0)
    jvm.call("destroy", 0)                            # als_engine_destroy(NULL) is a no-op, no exception
    with pytest.raises(JavaException, match="als_comm_set_timeout: als_status 1"):
        jvm.call("commSetTimeout", 0, 1000)           # NULL engine: ALS_ERR_INVALID_ARGUMENT
    assert jvm.stats()["violations"] == 0


def test_shape_errors_throw_illegal_argument_before_the_abi(jvm):
    a3, a2 = jvm.array(np.zeros(3, np.int32)), jvm.array(np.zeros(2, np.int32))
    s3 = jvm.array(np.zeros(3, np.int16))
    f7, f6 = jvm.array(np.zeros(7, np.float32)), jvm.array(np.zeros(6, np.float32))
    cases = [("setBlockCoo", (0, 0, 3, 0, 3, a3, a2, s3), "differ in length"),
             ("writeFactors", (0, 0, 0, f7, 2), "multiple of ld"),
             ("readFactors", (0, 0, 0, f6, 0), "multiple of ld"),
             ("writeFactorsF64", (0, 0, 0, f7, 2), "multiple of ld"),
             ("predict", (0, jvm.array(np.zeros(2, np.int64)), jvm.array(np.zeros(2, np.int64)), f7), "userRows.length"),
             ("commInit", (0, 2, 0, jvm.array(np.zeros(5, np.int8))), "128 bytes"),
             ("writePredictionMatrixCsv", (jvm.string("/nonexistent/x.csv"), f7, 2, 3), "nUsers * nMovies")]
    for name, args, what in cases:
        with pytest.raises(JavaException) as ei:
            jvm.call(name, *args)
        assert ei.value.cls == "java/lang/IllegalArgumentException" and what in ei.value.msg, (name, ei.value)
    st = jvm.stats()
    assert st["violations"] == 0 and st["open_critical"] == 0


def test_prediction_csv_through_the_shim_matches_the_oracle(jvm, oracle_mod, tmp_path):
    """writePredictionMatrixCsv (FeatureCollector.java:103-106): GetStringUTFChars + GetFloatArrayElements with
    JNI_ABORT (the writer only reads), bytes equal to the oracle's saveDenseCSV restatement."""
    rng = np.random.default_rng(3)
    Pm = (rng.standard_normal((7, 5)) * 10.0 ** rng.integers(-4, 8, (7, 5))).astype(np.float32)
    arr = jvm.array(Pm.ravel())
    path = str(tmp_path / "prediction_matrix_jni.csv")
    jvm.call("writePredictionMatrixCsv", jvm.string(path), arr, 7, 5)
    ref = str(tmp_path / "oracle.csv")
    oracle_mod.save_dense_csv(Pm.astype(np.float64), ref)
    assert open(path, "rb").read() == open(ref, "rb").read()
    assert np.array_equal(jvm.read(arr, np.float32), Pm.ravel())      # JNI_ABORT: the Java array is untouched
    with pytest.raises(JavaException, match="als_write_prediction_matrix_csv: als_status 6"):
        jvm.call("writePredictionMatrixCsv", jvm.string("/nonexistent-dir/x.csv"), arr, 7, 5)
    assert jvm.stats()["violations"] == 0


# ---------------------------------------------------------------------------------------------------------------
# GPU: the TaskEngine pattern, 8 engines, 4 threads
# ---------------------------------------------------------------------------------------------------------------
class TaskEngineMirror:
    """TaskEngine.java over the mock JVM: the engine of (partition p, side), its compacted opposite slots
    (ensureBlocks, :87-115), the staged opposite rows of an iteration (stage, :118-130) and the half (solve,
    :137-146: writeFactors, ONE solveHalf, readFactors)."""

    def __init__(self, jvm: MockJVM, side: int, part: int, rows, opp, k: int, precision: int):
        self.jvm, self.side, self.k, self.precision = jvm, side, k, precision
        ids = rows.ids
        self.local = np.nonzero(ids % P == part)[0]           # dense rows of this partition, ascending id
        r, c, v, slots = [], [], [], {}
        for i, d in enumerate(self.local):                     # in-block order = arrival order
            lo, hi = rows.row_ptr[d], rows.row_ptr[d + 1]
            for q in range(lo, hi):
                o = int(rows.col[q])                           # dense opposite index (= opposite id order)
                r.append(i)
                c.append(slots.setdefault(o, len(slots)))
                v.append(int(rows.ratings[q]))
        self.opp_dense = np.array(sorted(slots, key=slots.get), np.int64)   # slot -> dense opposite row
        self.coo = (np.array(r, np.int32), np.array(c, np.int32), np.array(v, np.int16))
        self.h = jvm.call("create", 0, k, precision)

    def ensure_blocks(self):
        j = self.jvm
        j.call("allocFactors", self.h, 1 - self.side, len(self.opp_dense))
        j.call("allocFactors", self.h, self.side, len(self.local))
        arrs = [j.array(a) for a in self.coo]
        j.call("setBlockCoo", self.h, self.side, len(self.local), 0, len(self.opp_dense), *arrs)
        j.free(*arrs)

    def solve(self, opp_full: np.ndarray, lam: float) -> np.ndarray:
        j, k = self.jvm, self.k
        f64 = self.precision == 1
        staged = j.array(np.ascontiguousarray(opp_full[self.opp_dense], np.float64 if f64 else np.float32).ravel())
        j.call("writeFactorsF64" if f64 else "writeFactors", self.h, 1 - self.side, 0, staged, k)
        j.call("solveHalf", self.h, self.side, lam)
        out = j.array_zeros(np.float64 if f64 else np.float32, len(self.local) * k)
        j.call("readFactorsF64" if f64 else "readFactors", self.h, self.side, 0, out, k)
        res = j.read(out, np.float64 if f64 else np.float32).reshape(len(self.local), k)
        j.free(staged, out)
        return res

    def release(self):
        self.jvm.call("destroy", self.h)


def _kafka_mirror(jvm, blocks, U0, k, iters, precision):
    """ALSApp.java:115-151 over P = 4 partitions: per half, each of THREADS host threads drives its partition's
    engine of that side (writeFactors / solveHalf / readFactors) concurrently; halves separated by a barrier
    (every solve of a half needs the whole previous half, the readiness rule of TaskEngine.stage)."""
    eng = [[TaskEngineMirror(jvm, s, p, blocks.movie if s == 0 else blocks.user,
                             blocks.user if s == 0 else blocks.movie, k, precision) for p in range(P)]
           for s in (0, 1)]
    dt = np.float64 if precision == 1 else np.float32
    U = U0.astype(dt).copy()
    M = np.zeros((len(blocks.movie.ids), k), dt)
    barrier = threading.Barrier(THREADS)
    errors = []

    def worker(t):
        try:
            for s in (0, 1):
                eng[s][t].ensure_blocks()
            for _ in range(iters):
                res = eng[0][t].solve(U, LAM)                  # MFeatureCalculator-i of partition t
                M[eng[0][t].local] = res
                barrier.wait()
                U[eng[1][t].local] = eng[1][t].solve(M, LAM)   # UFeatureCalculator-i (reads M only)
                barrier.wait()
            for s in (0, 1):
                eng[s][t].release()
        except BaseException as ex:                            # noqa: BLE001 -- surfaced by the main thread
            errors.append(ex)
            barrier.abort()

    threads = [threading.Thread(target=worker, args=(t,)) for t in range(THREADS)]
    for th in threads:
        th.start()
    for th in threads:
        th.join(timeout=300)
    assert not any(th.is_alive() for th in threads), "JNI mirror threads hung"
    if errors:
        raise errors[0]
    return U, M


@pytest.fixture(scope="module")
def tiny_blocks(oracle_mod, tiny_path):
    m, u, r = oracle_mod.parse_netflix(tiny_path)
    b = oracle_mod.build_blocks(m, u, r, P)
    return b, oracle_mod.init_user_features(b.user, 10, 42)


@pytest.mark.gpu
def test_taskengine_pattern_8_engines_4_threads_f64_golden(jvm, tiny_blocks, oracle_mod):
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    b, U0 = tiny_blocks
    U, M = _kafka_mirror(jvm, b, U0, 10, 10, precision=1)
    g = np.load(os.path.join(GOLDEN, "tiny_k10_n10_p4_seed42_f64.npz"))
    assert max_rel(U, g["U"]) <= 1e-6 and max_rel(M, g["M"]) <= 1e-6
    mse = oracle_mod.mse(b, U, M)
    assert abs(mse - float(g["mse"])) / float(g["mse"]) <= 1e-6
    st = jvm.all_stats()
    assert all(s["violations"] == 0 and s["open_critical"] == 0 and s["critical"] == 0 for s in st), st


@pytest.mark.gpu
def test_taskengine_pattern_f32_fast_mode_and_bitwise_repeatable(jvm, tiny_blocks, oracle_mod):
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    b, U0 = tiny_blocks
    g = np.load(os.path.join(GOLDEN, "tiny_k10_n10_p4_seed42_f64.npz"))
    runs = [_kafka_mirror(jvm, b, U0, 10, 10, precision=0) for _ in range(3)]
    U, M = runs[0]
    assert abs(oracle_mod.mse(b, U, M) - float(g["mse"])) <= 1e-3
    assert np.linalg.norm(U - g["U"]) / np.linalg.norm(g["U"]) < 1e-3
    for U2, M2 in runs[1:]:
        assert np.array_equal(U, U2) and np.array_equal(M, M2)   # interleaving of the 4 threads changes nothing
    # k = 64 through the same binding (MFMA path): one threaded run per precision-32 engine set, 2 iterations
    Uk, Mk = _kafka_mirror(jvm, b, oracle_mod.init_user_features(b.user, 64, 42), 64, 2, precision=0)
    Uo, Mo = oracle_mod.run_als(b, 64, LAM, 2, seed=42, precision="f64")
    assert abs(oracle_mod.mse(b, Uk, Mk) - oracle_mod.mse(b, Uo, Mo)) <= 1e-3


@pytest.mark.gpu
def test_device_errors_surface_as_streams_exception(jvm):
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    h = jvm.call("create", 0, 16, 0)
    with pytest.raises(JavaException) as ei:
        jvm.call("solveHalf", h, 0, 0.05)                      # no block uploaded: ALS_ERR_STATE
    assert ei.value.cls == "org/apache/kafka/streams/errors/StreamsException"
    assert "als_status 5" in ei.value.msg and "no block set" in ei.value.msg
    rows, cols = jvm.array(np.array([0], np.int32)), jvm.array(np.array([9], np.int32))
    with pytest.raises(JavaException, match="als_status 1"):   # opposite slot out of range: rejected on the host
        jvm.call("setBlockCoo", h, 0, 1, 0, 4, rows, cols, jvm.array(np.array([5], np.int16)))
    jvm.call("destroy", h)
    assert jvm.stats()["violations"] == 0


@pytest.mark.gpu
@pytest.mark.parametrize("f64", [False, True])
def test_read_factors_with_ld_beyond_k_keeps_padding_columns(jvm, f64):
    """readFactors[F64] with ld > num_features: columns k..ld-1 of the caller's array keep their values (the shim
    fills its buffer from the Java array before als_read_factors, which writes only the first k per row), as the
    Panama binding (AlsFfm.readFactors) leaves them."""
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    k, ld, n = 3, 5, 4
    dt = np.float64 if f64 else np.float32
    h = jvm.call("create", 0, k, 1 if f64 else 0)
    try:
        jvm.call("allocFactors", h, 0, n)
        src = (np.arange(n * k, dtype=dt) + 1.0) / 7.0
        jvm.call("writeFactorsF64" if f64 else "writeFactors", h, 0, 0, jvm.array(src), k)
        init = np.full(n * ld, -7.25, dt)
        out = jvm.array(init)
        jvm.call("readFactorsF64" if f64 else "readFactors", h, 0, 0, out, ld)
        got = jvm.read(out, dt).reshape(n, ld)
        assert np.array_equal(got[:, :k], src.reshape(n, k))
        assert np.all(got[:, k:] == -7.25)
    finally:
        jvm.call("destroy", h)
    assert jvm.stats()["violations"] == 0
