"""Python mirror of the reference's hot-path surface, over the C ABI of libcfk_als.so.

Reference interface (paths under src/main/java/de/hpi/collaborativefilteringkafka/):
  - ``Dataset``           ingest + in-block build + partition key: producers/NetflixDataFormatProducer.java:44-60,
                          processors/MRatings2BlocksProcessor.java:48-69, processors/URatings2BlocksProcessor.java:72-92,
                          producers/PureModStreamPartitioner.java:9-10 (all computed natively in als_dataset.cpp)
  - ``ALSEngine``         one partition's MFeatureCalculator / UFeatureCalculator solve state
                          (processors/MFeatureCalculator.java:49-136, processors/UFeatureCalculator.java:49-136)

Device memory is torch-owned (factor matrices are torch tensors bound into the engine) so that
``torch.distributed`` (RCCL over xGMI) can all-gather straight into the matrices the kernels read.
"""
from __future__ import annotations

import ctypes

import numpy as np
import torch

from . import _lib
from ._lib import F32, F64, SIDE_MOVIE, SIDE_USER, call, ptr

SIDES = {"movie": SIDE_MOVIE, "user": SIDE_USER}


def _side(s) -> int:
    return SIDES[s] if isinstance(s, str) else int(s)


def factor_stride(k: int, precision: str = "f32") -> int:
    """Padded factor-row stride of an engine (als_factor_stride): 16 / 32 / 64 / 128 on the wave-per-row kernels,
    the next multiple of 16 on the generic path (fp32 k > 128, fp64 k > 64)."""
    if k > (64 if precision == "f64" else 128):
        return (k + 15) // 16 * 16
    return 16 if k <= 16 else 32 if k <= 32 else 64 if k <= 64 else 128


class Dataset:
    """Ratings in arrival order plus the derived in-blocks (native; see include/als_host.h)."""

    def __init__(self, handle):
        self._h = ctypes.c_void_p(handle)

    # -- constructors ---------------------------------------------------------------------------
    @classmethod
    def load_netflix(cls, path: str) -> "Dataset":
        h = ctypes.c_void_p()
        call("als_dataset_load_netflix", path.encode(), ctypes.byref(h))
        return cls(h.value)

    @classmethod
    def from_ratings(cls, movie_ids, user_ids, ratings) -> "Dataset":
        m = np.ascontiguousarray(movie_ids, np.int32)
        u = np.ascontiguousarray(user_ids, np.int32)
        r = np.ascontiguousarray(ratings, np.int16)
        h = ctypes.c_void_p()
        call("als_dataset_from_ratings", len(m), ptr(m, ctypes.c_int32), ptr(u, ctypes.c_int32),
             ptr(r, ctypes.c_int16), ctypes.byref(h))
        return cls(h.value)

    @classmethod
    def synthetic_netflix(cls, n_users=480_189, n_movies=17_770, nnz=100_000_000, seed=0xA15, nthreads=0) -> "Dataset":
        h = ctypes.c_void_p()
        call("als_dataset_synthetic_netflix", n_users, n_movies, nnz, seed, nthreads, ctypes.byref(h))
        return cls(h.value)

    @classmethod
    def synthetic_powerlaw(cls, n_users=10_000_000, n_items=1_000_000, nnz=2_000_000_000, seed=0xA15,
                           nthreads=0) -> "Dataset":
        """BASELINE configs[4]: log-normal user activity (sigma 1.5), Zipf item popularity."""
        h = ctypes.c_void_p()
        call("als_dataset_synthetic_powerlaw", n_users, n_items, nnz, seed, nthreads, ctypes.byref(h))
        return cls(h.value)

    @classmethod
    def synthetic_shard(cls, workload: str, n_users: int, n_movies: int, nnz: int, seed: int, n_shards: int,
                        shard: int, nthreads: int = 0) -> "Dataset":
        """The same synthetic dataset restricted to the ratings of shard `shard` of n_shards (both sides' in-blocks of
        that rank): what one process of the G-GPU job needs, ~2/G of the ratings (include/als_host.h)."""
        h = ctypes.c_void_p()
        fn = {"netflix": "als_dataset_synthetic_netflix_shard", "powerlaw": "als_dataset_synthetic_powerlaw_shard"}
        call(fn[workload], n_users, n_movies, nnz, seed, nthreads, n_shards, shard, ctypes.byref(h))
        return cls(h.value)

    def close(self):
        if self._h and self._h.value:
            _lib.lib().als_dataset_destroy(self._h)
            self._h = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # -- queries ----------------------------------------------------------------------------------
    def counts(self):
        nm, nu, nnz = ctypes.c_int64(), ctypes.c_int64(), ctypes.c_int64()
        call("als_dataset_counts", self._h, ctypes.byref(nm), ctypes.byref(nu), ctypes.byref(nnz))
        return nm.value, nu.value, nnz.value

    @property
    def n_movies(self):
        return self.counts()[0]

    @property
    def n_users(self):
        return self.counts()[1]

    @property
    def nnz(self):
        return self.counts()[2]

    def ids(self, side) -> np.ndarray:
        side = _side(side)
        n = self.counts()[0 if side == SIDE_MOVIE else 1]
        out = np.zeros(n, np.int64)
        call("als_dataset_ids", self._h, side, ptr(out, ctypes.c_int64))
        return out

    def ratings(self):
        n = self.nnz
        m = np.zeros(n, np.int32)
        u = np.zeros(n, np.int32)
        r = np.zeros(n, np.int16)
        call("als_dataset_ratings", self._h, ptr(m, ctypes.c_int32), ptr(u, ctypes.c_int32), ptr(r, ctypes.c_int16))
        return m, u, r

    def count_duplicates(self) -> int:
        d = ctypes.c_int64()
        call("als_dataset_count_duplicates", self._h, ctypes.byref(d))
        return d.value

    def shard_info(self, side, n_shards=1, shard=0) -> dict:
        v = [ctypes.c_int64() for _ in range(5)]
        call("als_dataset_shard_info", self._h, _side(side), n_shards, shard, *[ctypes.byref(x) for x in v])
        keys = ("n_rows", "row_offset", "nnz", "slots_per_shard", "n_slots")
        return dict(zip(keys, (x.value for x in v)))

    def set_slot_chunks(self, side, n_chunks: int):
        """Chunk-major slot layout of `side` with n_chunks chunks (include/als_host.h "Slot layout")."""
        call("als_dataset_set_slot_chunks", self._h, _side(side), int(n_chunks))

    def slot_layout(self, side, n_shards=1) -> tuple[int, int]:
        """(slots per shard and chunk Sc, chunks C) of `side` under n_shards shards."""
        sc, c = ctypes.c_int64(), ctypes.c_int()
        call("als_dataset_slot_layout", self._h, _side(side), n_shards, ctypes.byref(sc), ctypes.byref(c))
        return sc.value, c.value

    def shard_block(self, side, n_shards=1, shard=0) -> dict:
        """In-block CSR of one shard: rows in ascending id, entries in arrival order, cols = opposite slots."""
        info = self.shard_info(side, n_shards, shard)
        rp = np.zeros(info["n_rows"] + 1, np.int64)
        col = np.zeros(info["nnz"], np.int32)
        rat = np.zeros(info["nnz"], np.int16)
        ids = np.zeros(info["n_rows"], np.int64)
        call("als_dataset_shard_block", self._h, _side(side), n_shards, shard, ptr(rp, ctypes.c_int64),
             ptr(col, ctypes.c_int32), ptr(rat, ctypes.c_int16), ptr(ids, ctypes.c_int64))
        info.update(row_ptr=rp, col=col, ratings=rat, row_ids=ids)
        return info

    def shard_coo(self, side, n_shards=1, shard=0) -> dict:
        """The shard's ratings as COO (local row, opposite slot, rating) in arrival order."""
        info = self.shard_info(side, n_shards, shard)
        rows = np.zeros(info["nnz"], np.int32)
        cols = np.zeros(info["nnz"], np.int32)
        rat = np.zeros(info["nnz"], np.int16)
        call("als_dataset_shard_coo", self._h, _side(side), n_shards, shard, ptr(rows, ctypes.c_int32),
             ptr(cols, ctypes.c_int32), ptr(rat, ctypes.c_int16))
        info.update(rows=rows, cols=cols, ratings=rat)
        return info

    def slots(self, side, n_shards=1) -> np.ndarray:
        side = _side(side)
        n = self.counts()[0 if side == SIDE_MOVIE else 1]
        out = np.zeros(n, np.int64)
        call("als_dataset_slots", self._h, side, n_shards, ptr(out, ctypes.c_int64))
        return out

    def feature_messages(self, side, n_partitions: int, factors: np.ndarray) -> tuple[bytes, np.ndarray, np.ndarray]:
        """The out-block fan-out of one half as Kafka FeatureMessage records (MFeatureCalculator.java:122-131):
        (concatenated payload, record keys = target partitions, byte offsets with a final end offset).
        factors: one row per entity of `side` in ascending raw-id order."""
        F = np.ascontiguousarray(factors, np.float32)
        k = F.shape[1]
        length = ctypes.c_int64()
        n_msg = ctypes.c_int64()
        call("als_encode_feature_messages", self._h, _side(side), n_partitions, k, None, k, None, 0,
             ctypes.byref(length), ctypes.byref(n_msg), None, None, 0)
        out = np.zeros(max(length.value, 1), np.uint8)
        keys = np.zeros(n_msg.value, np.int32)
        offs = np.zeros(n_msg.value + 1, np.int64)
        call("als_encode_feature_messages", self._h, _side(side), n_partitions, k, ptr(F, ctypes.c_float), k,
             ptr(out, ctypes.c_uint8), length.value, ctypes.byref(length), ctypes.byref(n_msg),
             ptr(keys, ctypes.c_int32), ptr(offs, ctypes.c_int64), n_msg.value)
        offs[-1] = length.value
        return out[:length.value].tobytes(), keys, offs

    def init_user_factors(self, k: int, seed: int = 42, n_shards: int = 1, ld: int | None = None) -> np.ndarray:
        """U0 in slot order (UFeatureInitializer.java:50-56 with the shared seeded generator)."""
        ld = k if ld is None else ld
        n_slots = self.shard_info(SIDE_USER, n_shards, 0)["n_slots"]
        out = np.zeros((n_slots, ld), np.float32)
        call("als_dataset_init_user_factors", self._h, k, seed, n_shards, ptr(out, ctypes.c_float), ld, n_slots)
        return out


def u01(seed: int, raw_id: int, feature: int) -> float:
    return _lib.lib().als_u01(seed, raw_id, feature)


def write_prediction_csv(path: str, U: np.ndarray, M: np.ndarray) -> None:
    """FeatureCollector.calculatePredictionMatrix + saveDenseCSV (FeatureCollector.java:90-110)."""
    U = np.ascontiguousarray(U, np.float32)
    M = np.ascontiguousarray(M, np.float32)
    k = U.shape[1]
    call("als_write_prediction_csv", path.encode(), ptr(U, ctypes.c_float), U.shape[0], k, ptr(M, ctypes.c_float),
         M.shape[0], k, k)


def write_prediction_matrix_csv(path: str, P: np.ndarray) -> None:
    """The collector's CSV from an already computed prediction matrix (e.g. ALSEngine.predict)."""
    P = np.ascontiguousarray(P, np.float32)
    call("als_write_prediction_matrix_csv", path.encode(), ptr(P, ctypes.c_float), P.shape[0], P.shape[1])


def encode_feature_message(entity_id: int, deps, features) -> bytes:
    """FeatureMessageSerializer (FeatureMessageSerializer.java:27-37): big-endian wire bytes."""
    d = np.ascontiguousarray(deps if deps is not None else [], np.int32)
    f = np.ascontiguousarray(features, np.float32)
    n = _lib.lib().als_feature_message_size(d.size, f.size)
    out = np.zeros(n, np.uint8)
    call("als_feature_message_encode", entity_id, ptr(d, ctypes.c_int32), d.size, ptr(f, ctypes.c_float), f.size,
         ptr(out, ctypes.c_uint8), n, None)
    return out.tobytes()


def decode_feature_message(data: bytes, num_features: int) -> tuple[int, np.ndarray, np.ndarray]:
    """FeatureMessageDeserializer (FeatureMessageDeserializer.java:30-56) -> (id, dependent ids, features)."""
    buf = np.frombuffer(data, np.uint8).copy()
    eid = ctypes.c_int32()
    nd = ctypes.c_int64()
    call("als_feature_message_decode", ptr(buf, ctypes.c_uint8), buf.size, num_features, ctypes.byref(eid), None, 0,
         ctypes.byref(nd), None)
    deps = np.zeros(nd.value, np.int32)
    f = np.zeros(num_features, np.float32)
    call("als_feature_message_decode", ptr(buf, ctypes.c_uint8), buf.size, num_features, None,
         ptr(deps, ctypes.c_int32), nd.value, None, ptr(f, ctypes.c_float))
    return eid.value, deps, f


def encode_id_rating(entity_id: int, rating: int) -> bytes:
    """IdRatingPairMessageSerializer (IdRatingPairMessageSerializer.java:24-33): 6 big-endian bytes."""
    out = np.zeros(6, np.uint8)
    call("als_id_rating_encode", entity_id, rating, ptr(out, ctypes.c_uint8))
    return out.tobytes()


def decode_id_rating(data: bytes) -> tuple[int, int]:
    buf = np.frombuffer(data, np.uint8).copy()
    eid = ctypes.c_int32()
    r = ctypes.c_int16()
    call("als_id_rating_decode", ptr(buf, ctypes.c_uint8), buf.size, ctypes.byref(eid), ctypes.byref(r))
    return eid.value, r.value


class ALSEngine:
    """One device engine: the in-blocks of this rank's shard of both sides + bound factor matrices."""

    def __init__(self, k: int, precision: str = "f32", device: int = 0):
        if precision not in ("f32", "f64"):
            raise ValueError("precision must be 'f32' or 'f64'")
        self.k = k
        self.precision = precision
        self.device = device
        self.dtype = torch.float32 if precision == "f32" else torch.float64
        self.np_dtype = np.float32 if precision == "f32" else np.float64
        h = ctypes.c_void_p()
        call("als_engine_create", device, k, F32 if precision == "f32" else F64, ctypes.byref(h))
        self._h = h
        self.kp = _lib.lib().als_factor_stride(self._h)
        self.factors = [None, None]    # torch tensors [n_slots, kp]
        # the factor tables are torch tensors (torch.zeros fill, RCCL all-gathers): launch on torch's current
        # stream from the start so every access is ordered (als.h ordering contract); set_stream-style calls
        # may move it later
        self.use_torch_stream()

    def close(self):
        if self._h and self._h.value:
            _lib.lib().als_engine_destroy(self._h)
            self._h = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def use_torch_stream(self, stream: torch.cuda.Stream | None = None):
        s = stream if stream is not None else torch.cuda.current_stream(self.device)
        if s.cuda_stream == 0:
            # torch's default stream is the NULL stream: launch there too (a NULL handle passed to
            # als_engine_set_stream would select a private non-blocking stream, unordered with torch's work
            # and with the RCCL collectives that wait on torch's current stream)
            call("als_engine_use_default_stream", self._h)
        else:
            call("als_engine_set_stream", self._h, ctypes.c_void_p(s.cuda_stream))

    def set_block(self, side, row_ptr, col, ratings, row_offset: int, n_opp_rows: int):
        rp = np.ascontiguousarray(row_ptr, np.int64)
        c = np.ascontiguousarray(col, np.int32)
        r = np.ascontiguousarray(ratings, np.int16)
        call("als_set_block", self._h, _side(side), len(rp) - 1, row_offset, n_opp_rows, ptr(rp, ctypes.c_int64),
             ptr(c, ctypes.c_int32), ptr(r, ctypes.c_int16))

    def set_block_coo(self, side, n_rows: int, rows, cols, ratings, row_offset: int, n_opp_rows: int):
        """Same block from arrival-order COO; the in-block sort and layout run on the GPU."""
        r = np.ascontiguousarray(rows, np.int32)
        c = np.ascontiguousarray(cols, np.int32)
        v = np.ascontiguousarray(ratings, np.int16)
        call("als_set_block_coo", self._h, _side(side), n_rows, row_offset, n_opp_rows, len(r),
             ptr(r, ctypes.c_int32), ptr(c, ctypes.c_int32), ptr(v, ctypes.c_int16))

    def bind_factors(self, side, tensor: torch.Tensor):
        """Bind a [n_rows + 1, kp] tensor: rows [0, n_rows) are the factors, the last row is the engine's
        all-zero sentinel (gathered by in-block padding entries; never written)."""
        side = _side(side)
        if tensor.dtype != self.dtype or tensor.dim() != 2 or tensor.shape[1] != self.kp or not tensor.is_contiguous():
            raise ValueError(f"factor tensor must be contiguous [n + 1, {self.kp}] {self.dtype}")
        if tensor.device.type != "cuda":
            raise ValueError("factor tensor must live on the GPU")
        call("als_bind_factors", self._h, side, ctypes.c_void_p(tensor.data_ptr()), tensor.shape[0] - 1)
        self.factors[side] = tensor

    def alloc_factors(self, side, n_rows: int) -> torch.Tensor:
        t = torch.zeros((n_rows + 1, self.kp), dtype=self.dtype, device=f"cuda:{self.device}")
        self.bind_factors(side, t)
        return t

    def write_factors(self, side, host: np.ndarray, row0: int = 0):
        h = np.ascontiguousarray(host, self.np_dtype)
        call("als_write_factors", self._h, _side(side), row0, h.shape[0], h.ctypes.data_as(ctypes.c_void_p), h.shape[1])

    def read_factors(self, side, row0: int = 0, n_rows: int | None = None) -> np.ndarray:
        side = _side(side)
        if n_rows is None:
            n_rows = self.factors[side].shape[0] - 1 - row0
        out = np.zeros((n_rows, self.k), self.np_dtype)
        call("als_read_factors", self._h, side, row0, n_rows, out.ctypes.data_as(ctypes.c_void_p), self.k)
        return out

    def solve_half(self, side, lam: float):
        """MFeatureCalculator (side='movie') / UFeatureCalculator (side='user') for every row of the block."""
        call("als_solve_half", self._h, _side(side), float(np.float32(lam)))

    def set_chunks(self, side, row_bounds):
        """Split the side's block into row-range chunks (local rows; row_bounds[0] = 0, [-1] = n_rows)."""
        b = np.ascontiguousarray(row_bounds, np.int64)
        call("als_set_chunks", self._h, _side(side), len(b) - 1, ptr(b, ctypes.c_int64))

    def solve_half_chunk(self, side, lam: float, chunk: int):
        call("als_solve_half_chunk", self._h, _side(side), float(np.float32(lam)), int(chunk))

    # -- multi-GPU exchange through the C ABI (RCCL over xGMI, als.h) -------------------------------------
    @staticmethod
    def comm_unique_id() -> bytes:
        buf = ctypes.create_string_buffer(128)
        call("als_comm_unique_id", buf, 128)
        return buf.raw

    def comm_init(self, world: int, rank: int, unique_id: bytes):
        buf = ctypes.create_string_buffer(bytes(unique_id), 128)
        call("als_comm_init", self._h, world, rank, buf)

    @staticmethod
    def comm_init_group(engines: list["ALSEngine"]):
        """One process driving len(engines) GPUs (one engine per device)."""
        arr = (ctypes.c_void_p * len(engines))(*[e._h.value for e in engines])
        call("als_comm_init_group", arr, len(engines))

    def comm_info(self) -> tuple[int, int]:
        w, r = ctypes.c_int(), ctypes.c_int()
        call("als_comm_info", self._h, ctypes.byref(w), ctypes.byref(r))
        return w.value, r.value

    def allgather_shard(self, side, slots_per_chunk: int, chunk: int = 0):
        """All-gather chunk `chunk` of `side` (every shard's slots_per_chunk rows of it, one contiguous region of
        the chunk-major layout) into this engine's replica; an unchunked side: its slots per shard, chunk 0."""
        call("als_allgather_shard", self._h, _side(side), int(slots_per_chunk), int(chunk))

    def set_row_layout(self, side, rows_per_chunk: int, chunk_stride: int):
        """Local row i -> factor row row_offset + (i // rows_per_chunk) * chunk_stride + i % rows_per_chunk."""
        call("als_set_row_layout", self._h, _side(side), int(rows_per_chunk), int(chunk_stride))

    def comm_wait(self):
        call("als_comm_wait", self._h)

    def comm_set_timeout(self, timeout_ms: int):
        """Bound (ms) on the engine's host waits while it has a communicator (als_comm_set_timeout)."""
        call("als_comm_set_timeout", self._h, int(timeout_ms))

    def predict(self, user_rows, movie_rows) -> np.ndarray:
        """FeatureCollector's U M^T (Java-float dots) for the given factor rows, on the GPU."""
        ur = np.ascontiguousarray(user_rows, np.int64)
        mr = np.ascontiguousarray(movie_rows, np.int64)
        out = np.zeros((len(ur), len(mr)), np.float32)
        call("als_predict", self._h, ptr(ur, ctypes.c_int64), len(ur), ptr(mr, ctypes.c_int64), len(mr),
             ptr(out, ctypes.c_float))
        return out

    def sq_error(self, side="movie"):
        se = ctypes.c_double()
        cnt = ctypes.c_int64()
        call("als_sq_error", self._h, _side(side), ctypes.byref(se), ctypes.byref(cnt))
        return se.value, cnt.value

    def synchronize(self):
        call("als_synchronize", self._h)

    def integrity_status(self, reset: bool = False) -> list[int]:
        """[REDUCE tasks that found a bad slot, generation, slot, row] of the first failure (0s when none)."""
        rec = (ctypes.c_uint32 * 4)()
        call("als_integrity_status", self._h, rec, 1 if reset else 0)
        return list(rec)

    def set_timing(self, on: bool):
        call("als_set_timing", self._h, 1 if on else 0)

    def timing_collect(self, side):
        g, r, n = ctypes.c_double(), ctypes.c_double(), ctypes.c_int64()
        call("als_timing_collect", self._h, _side(side), ctypes.byref(g), ctypes.byref(r), ctypes.byref(n))
        return g.value, r.value, n.value

    def debug_partials(self) -> np.ndarray:
        """The partial-slot workspace as raw 32-bit words (diagnostics)."""
        n = ctypes.c_int64()
        call("als_debug_copy_partials", self._h, None, 0, ctypes.byref(n))
        out = np.zeros(n.value // 4, np.uint32)
        call("als_debug_copy_partials", self._h, out.ctypes.data_as(ctypes.c_void_p), n.value, ctypes.byref(n))
        return out

    def block_path(self, side) -> dict:
        """Gram variant of the side's block: gram_path ('valu' | 'mfma_f32' | 'mfma_split'), presplit, chunk."""
        g, p, c, d = ctypes.c_int(), ctypes.c_int(), ctypes.c_int64(), (ctypes.c_int64 * 3)()
        call("als_block_path", self._h, _side(side), ctypes.byref(g), ctypes.byref(p), ctypes.byref(c), d)
        return {"gram_path": ("valu", "mfma_f32", "mfma_split", "generic")[g.value], "presplit": bool(p.value),
                "chunk": c.value,
                "dual_rows": sum(d), "dual_rows_by_blocks": list(d)}

    def split_info(self, side) -> dict:
        """Split-row plan of the side's block (als_block_split_info): rows split into interleaved chunks, their chunk
        tasks, the chunk length (entries), whether the half gathers the pre-split table."""
        v = (ctypes.c_int64 * 4)()
        call("als_block_split_info", self._h, _side(side), v)
        return {"interleaved_rows": v[0], "chunk_tasks": v[1], "chunk": v[2], "presplit": bool(v[3])}

    def block_stats(self, side):
        a, b, c = ctypes.c_int64(), ctypes.c_int64(), ctypes.c_int64()
        call("als_block_stats", self._h, _side(side), ctypes.byref(a), ctypes.byref(b), ctypes.byref(c))
        return {"n_tasks": a.value, "n_reduce": b.value, "nnz_padded": c.value}
