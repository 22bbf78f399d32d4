"""ALSApp: the reference topology's iteration semantics on 1..G GPUs (one process per GPU).

Reference: apps/ALSApp.java:41-48 (configuration), :115-163 (the unrolled ALS loop),
processors/UFeatureInitializer.java:36-66 (U0 after the EOF barrier), processors/FeatureCollector.java:72-110.

Bulk-synchronous restatement: U0 -> for i in 0..N-1 { M_i = solve(movies | U_i); U_{i+1} = solve(users | M_i) }.
The reference fires each entity's solve as soon as its last factor row arrives (MFeatureCalculator.java:65);
every solve of a half depends only on the previous half's factors, so the results are identical.
Final output = (U_N, M_{N-1}) as in the reference's movie-features-N / user-features-N topics.

Multi-GPU: entities are sharded by raw id % G (PureModStreamPartitioner.java:9-10 with numPartitions = G,
equal to (id % P) % G when G divides P). Every rank holds its shard's in-blocks and a full replica of both
factor matrices in slot order; each half-iteration ends with ONE RCCL all-gather (torch.distributed, backend
"nccl" = RCCL over xGMI) of the updated shard -- the replacement for the feature topics' block-to-block
fan-out (ALSApp.java:105-148, README.md:157).
"""
from __future__ import annotations

import time

import numpy as np
import torch

from .engine import ALSEngine, Dataset, SIDE_MOVIE, SIDE_USER


def _table_digest(t: torch.Tensor) -> int:
    """Bitwise digest of a factor table (all rows incl. the sentinel): sum over its 32-bit words w_i of
    w_i * (2 i + 1) * 0x9E3779B1 in wrapping int64 -- any change of one word changes it."""
    w = t.detach().contiguous().view(torch.int32).flatten().to(torch.int64)
    i = torch.arange(w.numel(), dtype=torch.int64, device=w.device)
    return int((w * ((2 * i + 1) * 0x9E3779B1)).sum().item())


class ALSApp:
    # a movie factor table above this is exchanged in chunks (N > 1): configs[4]'s 256 MB item table (all-gather ~1.7 ms
    # at G = 8), not the 9 MB k = 128 Netflix one -- its 4 chunk launches cost more in launch tails than the overlap of a
    # ~0.1 ms all-gather saves (one rank's k = 128 movie half at G = 2: 7.2 ms in 4 launches vs 5.4 ms in one,
    # profiles/r06a)
    MOVIE_CHUNK_BYTES = 64 << 20

    def __init__(self, num_partitions: int, num_features: int, als_lambda: float, num_als_iterations: int,
                 num_movies: int | None = None, num_users: int | None = None, *, precision: str = "f32",
                 seed: int = 42, device: int = 0, rank: int = 0, world_size: int = 1, group=None,
                 overlap_chunks: int = 4, exchange: str = "torch", movie_chunks: int | None = None):
        self.NUM_PARTITIONS = num_partitions
        self.NUM_FEATURES = num_features
        self.ALS_LAMBDA = float(np.float32(als_lambda))     # Float.parseFloat (ALSAppRunner.java:19)
        self.NUM_ALS_ITERATIONS = num_als_iterations
        self.NUM_MOVIES = num_movies
        self.NUM_USERS = num_users
        self.precision = precision
        self.seed = seed
        self.device = device
        self.rank = rank
        self.world = world_size
        self.group = group
        self.engine = None
        self.ds = None
        self.info = [None, None]
        # user half on > 1 GPU: solve in `overlap_chunks` row ranges and all-gather each range while the
        # next one is solved (1 = one launch, then one all-gather)
        self.overlap_chunks = max(1, int(overlap_chunks))
        # movie half on > 1 GPU: the same chunked exchange once the movie table is large (None: overlap_chunks
        # chunks when the movie factor table exceeds MOVIE_CHUNK_BYTES, e.g. configs[4]'s 1M items; 1 = unchunked)
        self.movie_chunks = None if movie_chunks is None else max(1, int(movie_chunks))
        self.chunk_slots = [None, None]   # per side: chunk indices of a chunked half, or None
        # "torch": torch.distributed collectives on the factor tensors (backend "nccl" = RCCL); "native": the
        # engine's own RCCL communicator through the C ABI (als_comm_init / als_allgather_shard), the path a
        # JNI caller uses. The rendezvous (sharing the RCCL unique id) uses the torch process group either way.
        # "none": no exchange at all -- one rank of a sharded run timed alone (its halves, not the all-gathers).
        if exchange not in ("torch", "native", "none"):
            raise ValueError("exchange must be 'torch', 'native' or 'none'")
        self.exchange = exchange

    # -------------------------------------------------------------------------------------------------
    def setup(self, ds: Dataset, check_duplicates: bool = True, engine_factory=None,
              block_build: str = "device") -> "ALSApp":
        """Blocks of this rank's shard + factor replicas + U0 (UFeatureInitializer after the EOF barrier).

        ``engine_factory(k, precision, device)`` replaces the HIP engine with another object of the same
        interface; only the multi-rank CPU rehearsal tests (gloo) use it, to exercise the sharding and the
        all-gather on machines without a GPU. The product path is always the HIP engine."""
        nm, nu, nnz = ds.counts()
        if self.NUM_MOVIES is not None and (nm, nu) != (self.NUM_MOVIES, self.NUM_USERS):
            raise ValueError(f"NUM_MOVIES/NUM_USERS = {self.NUM_MOVIES}/{self.NUM_USERS} but the dataset rates "
                             f"{nm} movies and {nu} users (the reference collector would never fire, "
                             f"FeatureCollector.java:43)")
        if check_duplicates and ds.count_duplicates():
            raise ValueError("duplicate (user, movie) pairs: the reference never completes such an entity "
                             "(MFeatureCalculator.java:65)")
        self.ds = ds
        # user half on > 1 GPU in `overlap_chunks` row ranges: chunk-major user slots (include/als_host.h "Slot
        # layout"), so each range's exchange is one contiguous all-gather; the movie half too once its table is big
        kp = (self.NUM_FEATURES + 15) // 16 * 16
        if self.world == 1:
            n_chunks = [1, 1]
        else:
            mc = self.movie_chunks
            if mc is None:
                mc = self.overlap_chunks if nm * kp * 4 > self.MOVIE_CHUNK_BYTES else 1
            n_chunks = [mc, self.overlap_chunks]
        ds.set_slot_chunks(SIDE_USER, n_chunks[SIDE_USER])
        ds.set_slot_chunks(SIDE_MOVIE, n_chunks[SIDE_MOVIE])
        if engine_factory is None:
            torch.cuda.set_device(self.device)
            eng = ALSEngine(self.NUM_FEATURES, self.precision, self.device)
        else:
            eng = engine_factory(self.NUM_FEATURES, self.precision, self.device)
        eng.use_torch_stream()
        for side in (SIDE_MOVIE, SIDE_USER):
            opp = ds.shard_info(1 - side, self.world, self.rank)
            if block_build == "device" and hasattr(eng, "set_block_coo"):
                # block builders on the GPU: arrival-order COO -> stable radix sort by row (als_set_block_coo)
                blk = ds.shard_coo(side, self.world, self.rank)
                eng.alloc_factors(side, blk["n_slots"])
                eng.set_block_coo(side, blk["n_rows"], blk["rows"], blk["cols"], blk["ratings"], blk["row_offset"],
                                  opp["n_slots"])
            else:
                blk = ds.shard_block(side, self.world, self.rank)
                eng.alloc_factors(side, blk["n_slots"])
                eng.set_block(side, blk["row_ptr"], blk["col"], blk["ratings"], blk["row_offset"], opp["n_slots"])
            sc, nc = ds.slot_layout(side, self.world)
            blk["slots_per_chunk"], blk["n_chunks"] = sc, nc
            if nc > 1:
                eng.set_row_layout(side, sc, self.world * sc)
            self.info[side] = {k: blk[k] for k in ("n_rows", "row_offset", "nnz", "slots_per_shard", "n_slots",
                                                   "slots_per_chunk", "n_chunks")}
        for side in (SIDE_MOVIE, SIDE_USER):
            nc = self.info[side]["n_chunks"]
            if nc > 1:
                sc, n = self.info[side]["slots_per_chunk"], self.info[side]["n_rows"]
                # chunk c = this rank's local rows [c Sc, (c+1) Sc) = factor rows [c G Sc + rank Sc, + Sc)
                self.chunk_slots[side] = list(range(nc))
                eng.set_chunks(side, [min(c * sc, n) for c in range(nc)] + [n])
        u0 = ds.init_user_factors(self.NUM_FEATURES, self.seed, self.world)
        eng.write_factors(SIDE_USER, u0)
        if self.exchange == "native" and self.world > 1:
            import torch.distributed as dist
            uid = [eng.comm_unique_id() if self.rank == 0 else None]
            dist.broadcast_object_list(uid, src=0, group=self.group)
            eng.comm_init(self.world, self.rank, uid[0])
        self.engine = eng
        self.nnz_total = nnz
        return self

    # -------------------------------------------------------------------------------------------------
    def _stream_ordered(self) -> bool:
        """RCCL ("nccl") orders its kernels after the work already queued on the current stream. gloo on CUDA
        tensors reads them with host-side copies, so the engine's stream is drained before each collective."""
        import torch.distributed as dist
        if not hasattr(self, "_ordered"):
            self._ordered = dist.get_backend(self.group) == "nccl"
        return self._ordered

    def _allgather(self, side: int, chunk: int = 0):
        """Exchange chunk `chunk` of `side` (the whole shard when the side is unchunked): one all-gather of the G
        ranks' Sc-row pieces, which are contiguous in the chunk-major slot layout."""
        if self.world == 1 or self.exchange == "none":   # "none": one rank's work alone (bench.py --shard-of)
            return
        sc = self.info[side]["slots_per_chunk"]
        if self.exchange == "native":
            self.engine.allgather_shard(side, sc, chunk)
            return
        import torch.distributed as dist
        if not self._stream_ordered():
            self.engine.synchronize()
        full = self.engine.factors[side]            # [n_slots + 1, kp]: last row = sentinel, not exchanged
        base = chunk * self.world * sc
        return dist.all_gather_into_tensor(full[base:base + self.world * sc],
                                           full[base + self.rank * sc:base + (self.rank + 1) * sc],
                                           group=self.group, async_op=True)

    def _half(self, side):
        if self.chunk_slots[side] is None:
            self.engine.solve_half(side, self.ALS_LAMBDA)
            w = self._allgather(side)
            if w is not None:
                w.wait()
            return
        # chunk c's all-gather (RCCL, ordered after chunk c's solve on the stream) overlaps chunk c+1's solve
        works = []
        for c in self.chunk_slots[side]:
            self.engine.solve_half_chunk(side, self.ALS_LAMBDA, c)
            works.append(self._allgather(side, c))
        for w in works:
            if w is not None:
                w.wait()

    def movie_half(self):
        """MFeatureCalculator-i over this rank's movies + all-gather (movie-features-i topic)."""
        self._half(SIDE_MOVIE)

    def user_half(self):
        """UFeatureCalculator-i over this rank's users + all-gather (user-features-(i+1) topic)."""
        self._half(SIDE_USER)

    def iteration(self):
        self.movie_half()
        self.user_half()

    def run(self, iterations: int | None = None) -> float:
        n = self.NUM_ALS_ITERATIONS if iterations is None else iterations
        self.engine.synchronize()
        t0 = time.perf_counter()
        for _ in range(n):
            self.iteration()
        self.engine.synchronize()
        return time.perf_counter() - t0

    # -------------------------------------------------------------------------------------------------
    def verify_replicas(self) -> dict:
        """Self-check of a sharded run (N > 1), after the exchange has settled: every rank's full replicas of both
        factor matrices must be bitwise identical (what the all-gathers promise: the reference's feature topics
        deliver the same rows to every partition, ALSApp.java:105-148), and every rank's partial-slot integrity
        record clean. One digest per side and rank -- a position-weighted int64 sum of the tables' 32-bit words --
        compared by MIN/MAX all-reduces. Returns {"replicas_agree", "integrity_clean", "digest": [movie, user],
        "integrity_failures"}; at N = 1 trivially true (one replica)."""
        self.engine.synchronize()
        digests = [_table_digest(self.engine.factors[s]) for s in (SIDE_MOVIE, SIDE_USER)]
        bad = int(self.engine.integrity_status()[0]) if hasattr(self.engine, "integrity_status") else 0
        if self.world == 1 or self.exchange == "none":
            return {"replicas_agree": True, "integrity_clean": bad == 0, "digest": [f"{d:016x}" for d in digests],
                    "integrity_failures": bad}
        import torch.distributed as dist
        dev = "cpu" if dist.get_backend(self.group) == "gloo" else self.engine.factors[0].device
        t = torch.tensor(digests + [bad], dtype=torch.int64, device=dev)
        hi, lo = t.clone(), t.clone()
        dist.all_reduce(hi, op=dist.ReduceOp.MAX, group=self.group)
        dist.all_reduce(lo, op=dist.ReduceOp.MIN, group=self.group)
        agree = bool(torch.equal(hi[:2], lo[:2]))
        return {"replicas_agree": agree, "integrity_clean": int(hi[2]) == 0,
                "digest": [f"{d & 0xFFFFFFFFFFFFFFFF:016x}" for d in digests], "integrity_failures": int(hi[2])}

    def factors(self):
        """(U, M) in ascending raw-id order (FeatureCollector.constructFeatureMatrices, :72-88)."""
        U = self.engine.read_factors(SIDE_USER)
        M = self.engine.read_factors(SIDE_MOVIE)
        return U[self.ds.slots(SIDE_USER, self.world)], M[self.ds.slots(SIDE_MOVIE, self.world)]

    def prediction_matrix(self) -> np.ndarray:
        """FeatureCollector.calculatePredictionMatrix (FeatureCollector.java:90-101): users x movies, both in
        ascending id order, computed on the GPU from the (gathered) factor replicas."""
        return self.engine.predict(self.ds.slots(SIDE_USER, self.world), self.ds.slots(SIDE_MOVIE, self.world))

    def sq_error(self):
        """Sum of squared errors over all observed ratings (all ranks) and the rating count."""
        se, cnt = self.engine.sq_error(SIDE_MOVIE)
        if self.world > 1:
            import torch.distributed as dist
            t = torch.tensor([se, float(cnt)], dtype=torch.float64, device=self.engine.factors[0].device)
            dist.all_reduce(t, group=self.group)
            se, cnt = float(t[0]), int(t[1])
        return se, cnt

    def mse(self) -> float:
        se, cnt = self.sq_error()
        return se / cnt
