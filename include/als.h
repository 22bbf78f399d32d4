/*
 * als.h -- C ABI of the MI355X-native ALS engine (libcfk_als.so).
 *
 * Drop-in boundary for the reference's one hot path: the per-movie / per-user regularised least-squares
 * feature update that the Kafka Streams processors run
 *     MFeatureCalculator.process   src/main/java/de/hpi/collaborativefilteringkafka/processors/MFeatureCalculator.java:49-136
 *     UFeatureCalculator.process   .../processors/UFeatureCalculator.java:49-136
 * whose arithmetic sits behind EJML CommonOps_FDRM (multTransA / scale / identity / add / invert / mult,
 * MFeatureCalculator.java:85-99). A re-plumbed processor buffers its partition's half-iteration (the EOF
 * barrier, UFeatureInitializer.java:37-41) and makes ONE als_solve_half() call instead of one EJML solve per
 * entity. The JNI / Panama binding a maintainer adds on the Java side is shown in INTEGRATION.md.
 *
 * Conventions
 *  - Plain C types only; every function returns an als_status (0 = ALS_OK) and never throws or longjmps
 *    across the ABI. als_last_error() returns the calling thread's last message. (The reference ignores
 *    EJML invert's boolean, MFeatureCalculator.java:98; this ABI reports failures instead.)
 *  - One engine = one (device, num_features, precision). Engines are independent; one engine must not be
 *    used from two threads at once (the reference runs each task's process() single-threaded,
 *    BaseKafkaApp.java:51, so one engine per stream task / GPU is the intended use).
 *  - "side" selects the entity type whose rows are recomputed: ALS_SIDE_MOVIE rows are solved from user
 *    factors (MFeatureCalculator), ALS_SIDE_USER rows from movie factors (UFeatureCalculator).
 *  - Factor matrices live in device memory with a padded row stride (als_factor_stride(): 16, 32, 64 or
 *    128 elements, or num_features rounded up to 16 beyond that); columns >= num_features are kept at zero.
 */
#ifndef CFK_ALS_H
#define CFK_ALS_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define ALS_ABI_VERSION 3

typedef enum {
    ALS_OK = 0,
    ALS_ERR_INVALID_ARGUMENT = 1,
    ALS_ERR_UNSUPPORTED = 2,
    ALS_ERR_DEVICE = 3,        /* HIP runtime error */
    ALS_ERR_OUT_OF_MEMORY = 4,
    ALS_ERR_STATE = 5,         /* call order violated (e.g. solve before a block was set) */
    ALS_ERR_IO = 6,
    ALS_ERR_PARSE = 7,
    ALS_ERR_DATA = 8,          /* input that hangs the reference (duplicate pair, count mismatch) */
    ALS_ERR_INTEGRITY = 9,     /* a split row's REDUCE task read a partial slot this launch had not written
                                  (als_integrity_status); the results of that half are not trustworthy */
    ALS_ERR_COMM = 10          /* RCCL error (als_comm_*, als_allgather_shard) */
} als_status;

typedef enum { ALS_SIDE_MOVIE = 0, ALS_SIDE_USER = 1 } als_side;
typedef enum { ALS_F32 = 0, ALS_F64 = 1 } als_precision;

typedef struct als_engine als_engine;

/* ---- version / errors --------------------------------------------------------------------------- */
int         als_abi_version(void);
const char* als_last_error(void);
/* sha256 of the sources (csrc/, include/) the library was compiled from, as stamped by the build
 * (__graft_entry__.build); "" for an unstamped developer build. */
const char* als_build_source_sha256(void);
int         als_device_count(int* n);

/* ---- engine lifetime ---------------------------------------------------------------------------- */
/* Replaces the per-task processor state of MFeatureCalculator/UFeatureCalculator.init (:29-46).
 * num_features = ALSApp.NUM_FEATURES (ALSApp.java:18), 1..1024: up to 128 (f64: 64) on the wave-per-row kernels,
 * beyond that on the generic workgroup-per-row path (ALSAppRunner.java:18 accepts any value). */
int als_engine_create(int device, int num_features, int precision, als_engine** out);
int als_engine_destroy(als_engine* e);
/* Launch on a caller-provided hipStream_t (e.g. torch's current stream); NULL = engine-owned stream.
 * Ordering contract: the engine orders its own work on its stream only. A caller that reads or writes a bound
 * factor buffer (als_bind_factors) from other work -- torch ops, RCCL collectives -- must issue that work on
 * the engine's stream or synchronise (als_synchronize) in between. */
int als_engine_set_stream(als_engine* e, void* hip_stream);
/* Launch on the device's NULL (legacy default) stream: the stream torch launches on when no other stream is
 * current (its handle is 0, which als_engine_set_stream would read as "engine-owned"). The engine's kernels are
 * then ordered with torch's work and with RCCL collectives issued against that stream. */
int als_engine_use_default_stream(als_engine* e);
int als_factor_stride(const als_engine* e);

/* ---- in-block upload (constant over all iterations, README.md:146-147) ---------------------------- */
/* Replaces the state stores m-inblocks-uid / m-inblocks-ratings (resp. u-*) that
 * MRatings2BlocksProcessor.java:48-69 / URatings2BlocksProcessor.java:72-92 fill: one CSR row per entity
 * of this partition, entries in in-block order. Row i is solved into factor row (row_offset + i) of
 * `side`; col_idx[] are rows of the opposite side's factor matrix (0 <= col < n_opp_rows).
 * Host pointers; copied to the device once. */
int als_set_block(als_engine* e, int side, int64_t n_rows, int64_t row_offset, int64_t n_opp_rows,
                  const int64_t* row_ptr, const int32_t* col_idx, const int16_t* ratings);

/* The same block from COO triples in arrival order (rows[t] = local row, cols[t] = opposite row, ratings[t]):
 * the stable sort into in-block order (= arrival order per row, MRatings2BlocksProcessor.java:53-69) and the
 * padded layout are done on the GPU (radix sort by row), replacing the host-side CSR build for large data.
 * Host pointers; results identical to als_set_block on the equivalent CSR. nnz < 2^31 per call. */
int als_set_block_coo(als_engine* e, int side, int64_t n_rows, int64_t row_offset, int64_t n_opp_rows, int64_t nnz,
                      const int32_t* rows, const int32_t* cols, const int16_t* ratings);

/* ---- factor matrices (device resident) ---------------------------------------------------------- */
/* Engine-owned buffer of n_total_rows x stride elements (zeroed), plus one hidden all-zero sentinel row
 * after the last row (in-block padding entries gather it instead of being masked). */
int als_alloc_factors(als_engine* e, int side, int64_t n_total_rows);
/* Caller-owned device buffer (e.g. a torch tensor) of n_total_rows + 1 rows, row stride =
 * als_factor_stride(e), padding columns zero; the engine zeroes row n_total_rows (the sentinel) here and
 * never writes it, so callers must not either. Lets a collective (RCCL all-gather) write straight into the
 * matrix the engine reads. */
int als_bind_factors(als_engine* e, int side, void* device_ptr, int64_t n_total_rows);
int als_factors_device_ptr(const als_engine* e, int side, void** device_ptr, int64_t* n_total_rows);
/* Host <-> device copies of rows [row0, row0+n_rows) with a host row stride of src_ld/dst_ld elements
 * (>= num_features); element type = float (ALS_F32) or double (ALS_F64). */
int als_write_factors(als_engine* e, int side, int64_t row0, int64_t n_rows, const void* host_src, int64_t src_ld);
int als_read_factors(als_engine* e, int side, int64_t row0, int64_t n_rows, void* host_dst, int64_t dst_ld);

/* ---- THE HOT PATH ------------------------------------------------------------------------------- */
/* For every row j of `side`'s block: gather Y_S = opposite factor rows of its in-block, form
 * A = Y_S^T Y_S + lambda * n_j * I and V = Y_S^T r, solve A m_j = V and store m_j. A is SPD because lambda * n_j > 0:
 * the MFMA paths (fp32 k <= 128, fp64 k <= 64) factor it as a Jacobi-scaled block LDL^T on the 16 x 16 Gram tiles
 * with a pivot-gated refinement step, the generic path (wider k) by Cholesky; EJML's LU inverse (the reference,
 * CommonOps_FDRM.invert) is restated in the oracle. == MFeatureCalculator.java:66-104 / UFeatureCalculator.java:66-104
 * for the whole partition. Asynchronous on the engine's stream. */
int als_solve_half(als_engine* e, int side, float lambda);

/* Row-range chunks of a half (multi-GPU overlap). als_set_chunks splits `side`'s block into n_chunks
 * ranges of its local rows, row_bounds[0] = 0 <= ... <= row_bounds[n_chunks] = n_rows; the union of the
 * chunk launches is exactly als_solve_half. Lets the caller all-gather chunk c of the updated shard over
 * RCCL while chunk c+1 is solved -- the per-partition fan-out of the reference's feature topics
 * (ALSApp.java:105-148) overlapped with compute. Replaces any previous chunking of that side. The chunks of
 * one half are solved in ascending order starting with chunk 0, and the opposite factor replica (the half's
 * input) does not change between them: chunk 0 prepares it (the pre-split copy), later chunks reuse that. */
int als_set_chunks(als_engine* e, int side, int n_chunks, const int64_t* row_bounds);
int als_solve_half_chunk(als_engine* e, int side, float lambda, int chunk);
/* Chunk-major slot layout of `side`'s rows (after als_set_block, which resets it): local row i is solved into
 * factor row row_offset + (i / rows_per_chunk) * chunk_stride + i % rows_per_chunk (rows_per_chunk = 0: the
 * contiguous row_offset + i). With Sc = rows_per_chunk and chunk_stride = G Sc, the rows of chunk c of every
 * shard are contiguous (als_host.h "Slot layout"). */
int als_set_row_layout(als_engine* e, int side, int64_t rows_per_chunk, int64_t chunk_stride);

/* ---- multi-GPU: shards + RCCL all-gather over xGMI ------------------------------------------------
 * Replaces the per-iteration feature topics (ALSApp.java:105-151): entities are sharded by raw id % G
 * (PureModStreamPartitioner.java:9-10) into chunk-major slots (als_host.h "Slot layout": slot = (r / Sc) G Sc +
 * shard Sc + r % Sc for rank r in the shard, Sc = slots per shard and chunk; one chunk: slot = shard S + r), every
 * engine holds its shard's in-blocks and a full replica of both factor matrices, and each half ends with one
 * all-gather per chunk of the updated shard. One engine per GPU; either one process per GPU (unique id from
 * als_comm_unique_id on one process, shared by the caller, then als_comm_init on every process) or one process
 * driving G GPUs (als_comm_init_group). The exchange is enqueued on the engine's stream after its solve. */
int als_comm_unique_id(void* id_out, int nbytes);   /* nbytes >= 128 */
int als_comm_init(als_engine* e, int world, int rank, const void* unique_id);
int als_comm_init_group(als_engine** engines, int n);
int als_comm_info(const als_engine* e, int* world, int* rank);
/* Gather chunk `chunk` of `side` -- factor rows [chunk G Sc, (chunk + 1) G Sc), this engine's Sc rows at
 * chunk G Sc + rank Sc -- into every engine's replica: one in-place ncclAllGather (Sc = slots_per_chunk; an
 * unchunked side passes its S slots per shard and chunk 0). A single host thread driving several engines
 * wraps its per-engine calls in als_comm_group_start / als_comm_group_end; the engines' completion events are
 * then recorded at the outermost group end, where RCCL places the grouped collectives on their streams. A no-op
 * for an engine without a communicator (G = 1). */
int als_allgather_shard(als_engine* e, int side, int64_t slots_per_chunk, int64_t chunk);
int als_comm_group_start(void);
int als_comm_group_end(void);
/* The all-gathers run on the engine's own communication stream, after the solve that produced the shard and
 * overlapping any later solve that does not depend on them (e.g. the next user-half chunk); the engine orders
 * its next solve of the other side, and every synchronising call, after them. Work issued by the caller on
 * the engine's stream that reads the gathered replicas (e.g. torch ops) must call als_comm_wait first. */
int als_comm_wait(als_engine* e);
/* Bound on every host wait of an engine with a communicator (default 120 000 ms, or ALS_COMM_TIMEOUT_S): a collective
 * that never completes (a peer gone, mismatched calls) would hang the caller of a synchronising call. On expiry the
 * communicator is aborted and the call fails with ALS_ERR_COMM naming the last all-gather issued (side, chunk); the
 * engine is then unusable for the exchange. timeout_ms <= 0: unbounded. (No reference counterpart: the reference's
 * lost messages hang silently, README.md:241; SURVEY.md section 5 asks for a timeout on collectives.) */
int als_comm_set_timeout(als_engine* e, int64_t timeout_ms);

/* FeatureCollector's prediction matrix (FeatureCollector.java:90-101) from the resident factors:
 * host_out[u * n_movies + m] = U[user_rows[u]] . M[movie_rows[m]] as a Java float dot (fp32 products and
 * sums rounded separately, features in order -- EJML multTransB), so the CSV written from it carries the
 * reference's digits. Rows are factor-matrix rows (slots); pass them in ascending-id order for the
 * collector's layout (FeatureCollector.java:72-88). Synchronous. */
int als_predict(als_engine* e, const int64_t* user_rows, int64_t n_users, const int64_t* movie_rows,
                int64_t n_movies, float* host_out);

/* Sum of (r - x_row . y_col)^2 over the block's observed ratings and their count (the RMSE/MSE
 * reduction of scripts/calculate_mse.py:78-90 computed on the device from the factors). Synchronous. */
int als_sq_error(als_engine* e, int side, double* sum_sq_error, int64_t* count);

/* Waits for the engine's stream. Like every synchronising call (als_read_factors, als_sq_error, als_predict)
 * it returns ALS_ERR_INTEGRITY once a REDUCE task has found a partial slot that its PARTIAL task's writes had
 * not reached (each slot is stored keyed by the launch generation with a check word). */
int als_synchronize(als_engine* e);
/* The integrity record: record[0] = REDUCE tasks that found a bad slot so far, record[1..3] = launch generation, slot
 * and local row of the first; reset != 0 clears it. Synchronising. */
int als_integrity_status(als_engine* e, uint32_t* record, int reset);
/* Device-time accounting with HIP events on the engine's stream (non-blocking while enabled): every
 * als_solve_half records its gram/solve launch and its reduce launch; als_timing_collect waits for the
 * recorded events of `side`, returns their summed milliseconds and call count, and clears them. */
int als_set_timing(als_engine* e, int enabled);
int als_timing_collect(als_engine* e, int side, double* ms_gram, double* ms_reduce, int64_t* n_calls);
/* Diagnostics: copies up to max_bytes of the partial-slot workspace (the PARTIAL tasks' encoded sums of the
 * last half) to host memory and reports its size. Synchronising. */
int als_debug_copy_partials(als_engine* e, void* host_dst, int64_t max_bytes, int64_t* bytes);
/* Gram variant of `side`'s block: gram_path 0 = LDS-staged VALU (fp64, fp32 k < 32), 1 = fp32 MFMA
 * (v_mfma_f32_16x16x4_f32), 2 = split MFMA (fp32 operands split exactly into narrow terms); presplit = 1 when the
 * opposite table is gathered as the pre-split scaled two-term fp16 copy (h + m per value, RHS on the MFMAs too),
 * 0 when each gathered fp32 row is split on the fly into three bf16 terms; chunk = entries per contiguous PARTIAL
 * task of a split row (interleaved split rows: als_block_split_info); n_dual_rows[3] = short rows
 * of 1, 2 and 3 padded blocks solved in entry space, (Y Y^T + lambda n I) alpha = r, m = Y^T alpha (the same
 * solution as the k x k system). */
int als_block_path(const als_engine* e, int side, int* gram_path, int* presplit, int64_t* chunk, int64_t* n_dual_rows);
/* Work-plan statistics of the uploaded block (tasks, partial slots, padded nnz). */
int als_block_stats(const als_engine* e, int side, int64_t* n_tasks, int64_t* n_reduce, int64_t* nnz_padded);
/* Split-row plan of the uploaded block (a launch-shape query with no reference counterpart):
 * info[0] = rows split into interleaved chunks (0: contiguous chunks, the plan of halves whose opposite table fits the
 * L2s), [1] their chunk tasks, [2] the chunk length in entries, [3] 1 when the half gathers the pre-split table. */
int als_block_split_info(const als_engine* e, int side, int64_t info[4]);

#ifdef __cplusplus
}
#endif
#endif /* CFK_ALS_H */
