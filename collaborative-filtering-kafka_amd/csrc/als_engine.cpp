// als_engine.cpp -- the C ABI of include/als.h: engine lifetime, in-block upload + work plan, factor
// buffers, and the half-iteration launch. See include/als.h for the reference interface each entry
// point replaces.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <chrono>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "als.h"
#include "als_internal.h"

using cfk::Path;
using cfk::Task;

namespace {

thread_local std::string g_last_error;

int fail(int code, const char* fmt, ...) {
    char buf[1024];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof(buf), fmt, ap);
    va_end(ap);
    g_last_error = buf;
    return code;
}

#define HIP_TRY(expr)                                                                              \
    do {                                                                                           \
        hipError_t _e = (expr);                                                                    \
        if (_e != hipSuccess)                                                                      \
            return fail(ALS_ERR_DEVICE, "%s failed: %s (%s:%d)", #expr, hipGetErrorString(_e),     \
                        __FILE__, __LINE__);                                                       \
    } while (0)

struct Block {
    bool set = false;
    int64_t n_rows = 0, row_offset = 0, n_opp_rows = 0, nnz = 0, nnz_padded = 0;
    int32_t* d_col = nullptr;
    float* d_rat = nullptr;
    uint32_t* d_rat_pk = nullptr;   // pre-split blocks: ratings as fp16 rh / rm pairs (the Gram's RHS operand)
    int32_t* d_col_ps = nullptr;    // pre-split blocks: column indices in the LDS-DMA gather order
    Task* d_tasks = nullptr;        // FULL + PARTIAL, sorted by work (longest first)
    Task* d_reduce = nullptr;       // REDUCE
    int32_t n_tasks = 0, n_reduce = 0, n_slots = 0;
    double* d_task_se = nullptr;    // per-task squared-error partials
    std::vector<Task> h_tasks, h_reduce;   // host copies of the work plan (chunking re-sorts them)
    Task* d_ctasks = nullptr;       // chunk-major FULL + PARTIAL tasks (LPT inside each chunk)
    Task* d_creduce = nullptr;      // chunk-major REDUCE tasks
    std::vector<int32_t> coff, croff;   // chunk c = d_ctasks[coff[c], coff[c+1]), d_creduce[croff[c], ...)
    // short rows solved in entry space (cfk::launch_dual), by entry-tile count cd = 2 (1 block) / 4 (2 blocks)
    Task* d_dual[3] = {nullptr, nullptr, nullptr};
    int32_t n_dual[3] = {0, 0, 0};
    std::vector<Task> h_dual[3];
    Task* d_cdual[3] = {nullptr, nullptr, nullptr};
    std::vector<int32_t> cdoff[3];
    Task* d_sq_tasks = nullptr;     // every FULL + PARTIAL task incl. the short rows (als_sq_error)
    int32_t n_sq = 0;
    bool presplit = false;          // gather a pre-split (scaled fp16 h/m) copy of the opposite table
    // interleaved split rows: rows longer than ilv_chunk entries, blocks permuted chunk-major
    int64_t ilv_rows = 0, ilv_tasks = 0, ilv_chunk = 0;
    // chunk-major slot layout (als_set_row_layout): local row i -> factor row row_offset + (i / rows_per_chunk) *
    // chunk_stride + i % rows_per_chunk; rows_per_chunk = 0: row_offset + i
    int64_t rows_per_chunk = 0, chunk_stride = 0;
    int64_t factor_row(int64_t i) const {
        return rows_per_chunk > 0 ? row_offset + (i / rows_per_chunk) * chunk_stride + i % rows_per_chunk
                                  : row_offset + i;
    }
};

struct TimingRec {
    int side;
    hipEvent_t ev[3];
};

struct Factors {
    void* ptr = nullptr;
    int64_t n_rows = 0;
    bool owned = false;
};

}  // namespace

namespace cfk_detail {
void set_last_error(const std::string& s) { g_last_error = s; }
}  // namespace cfk_detail

struct als_engine {
    int device = 0;
    int k = 0, kp = 0;
    int precision = ALS_F32;
    Path path = Path::VALU;
    hipStream_t stream = nullptr;
    bool own_stream = false;
    Block blk[2];
    Factors fac[2];
    void* d_partials = nullptr;
    size_t partial_bytes = 0;
    int64_t generic_slabs = 0;      // generic path: Gram slabs in d_partials
    void* d_split = nullptr;        // pre-split opposite table (cfk::launch_presplit), sized for the larger need
    size_t split_bytes = 0;
    uint32_t* d_amax = nullptr;     // bits of the pre-split table's largest |x| (cfk::launch_absmax): its scale
    void* h_stage = nullptr;        // pinned staging of als_write_factors / als_read_factors (copy kernels)
    size_t stage_bytes = 0;
    uint32_t* d_integrity = nullptr;   // cfk::INTEGRITY_WORDS: partial slots that failed their check
    int cu_count = 0;               // compute units of the device: the range guard's fallback grid
    // ALS_INTERLEAVE: interleaved split rows + pre-split Gram for halves whose opposite table outgrows the L2s
    // (-1 auto, 0 off, 1 wherever the pre-split Gram exists)
    int interleave = -1;
    // ALS_XCD_RANGES: an interleaved half's long rows are cut by opposite-slot range into 8 pieces whose chunks run on
    // the XCD of that range (-1 auto: KP = 64 and an opposite table within 128 MiB, 0 off, 1 on)
    int xcd_ranges = -1;
    uint32_t gen = 0;               // launch generation of the next PARTIAL/REDUCE pair
    int32_t debug_flags = 0;        // debug build only (CFK_DEBUG_KNOBS): ALS_DEBUG_SKIP_SOLVE / _REFINE
    uint32_t debug_gen_skew = 0;    // debug build only: ALS_DEBUG_REDUCE_GEN_SKEW=n, REDUCE decodes with generation
                                    // + n (tests the integrity check: every slot reads as written by another launch)
    // ALS_REFINE_MIN_PIVOT (cfk::SolveArgs): 0.45 keeps the worst per-row error ratio to the reference's own fp32
    // path where always refining puts it (0.41, tools/refine_accuracy.py; 0.30 lets it reach 1.2), and skips the
    // step for nearly every Netflix-shape row (k = 128 user half 17.7 -> 14.9 ms); > 1 always refines
    float refine_min_pivot = 0.45f;
    int32_t debug_extra_lds = 0;    // debug build only: ALS_DEBUG_EXTRA_LDS=bytes of unused LDS per main-launch
                                    // workgroup (occupancy sweeps of the MFMA kernels)
    bool debug_fixed_gen = false;   // debug build only: ALS_DEBUG_FIXED_GEN=1, every launch uses generation 1, so
                                    // partial slots of repeated launches are bitwise comparable (diagnostics)
    ncclComm_t comm = nullptr;      // RCCL communicator over the G engines (one per GPU) of a sharded run
    int world = 1, rank = 0;
    hipStream_t comm_stream = nullptr;   // all-gathers run here, overlapping the next chunk's solve
    hipEvent_t solved = nullptr;         // recorded on `stream` before each all-gather
    hipEvent_t gathered[2] = {nullptr, nullptr};   // last all-gather of each side, on comm_stream
    bool gather_pending[2] = {false, false};
    int64_t comm_timeout_ms = 120000;    // bound of host waits while a communicator exists (als_comm_set_timeout)
    int last_gather_side = -1;           // the last all-gather issued (for the timeout's message)
    int64_t last_gather_chunk = -1, last_gather_rows = 0;
    // Entry-space (als_solve_dual) launches run on side_stream, forked from and joined back into `stream`, so
    // they fill the CUs the main launch's tail leaves idle (ALS_DUAL_SIDE=0: same stream, after the main launch)
    bool dual_side = true;
    hipStream_t side_stream = nullptr;
    hipEvent_t fork = nullptr, join = nullptr;
    bool timing = false;
    std::vector<hipEvent_t> ev_pool;
    std::vector<TimingRec> pending;
    size_t elem() const { return precision == ALS_F64 ? 8 : 4; }
};

namespace {

int check_engine(const als_engine* e) {
    if (!e) return fail(ALS_ERR_INVALID_ARGUMENT, "engine is NULL");
    return ALS_OK;
}

// Drain the engine's stream and read the partial-slot integrity record (cfk::SlotCodec): a REDUCE task that
// found a slot it could not see freshly written by this launch's PARTIAL task makes every later synchronising
// call fail until als_integrity_status(..., reset = 1).
// Order the engine's stream after the pending all-gathers of the given sides (comm_stream -> stream).
int wait_gathers(als_engine* e, bool movie, bool user) {
    const bool want[2] = {movie, user};
    for (int s = 0; s < 2; ++s)
        if (want[s] && e->gather_pending[s]) {
            HIP_TRY(hipStreamWaitEvent(e->stream, e->gathered[s], 0));
            e->gather_pending[s] = false;
        }
    return ALS_OK;
}

// Host wait for the engine's stream, bounded while the engine has a communicator: on expiry the communicator is
// aborted (so that its kernels end) and the call fails naming the last all-gather issued.
int stream_wait(als_engine* e, hipStream_t s) {
    if (!e->comm || e->comm_timeout_ms <= 0) {
        HIP_TRY(hipStreamSynchronize(s));
        return ALS_OK;
    }
    const auto t0 = std::chrono::steady_clock::now();
    for (int spin = 0;; ++spin) {
        const hipError_t st = hipStreamQuery(s);
        if (st == hipSuccess) return ALS_OK;
        if (st != hipErrorNotReady) return fail(ALS_ERR_DEVICE, "stream wait: %s", hipGetErrorString(st));
        const int64_t ms =
            std::chrono::duration_cast<std::chrono::milliseconds>(std::chrono::steady_clock::now() - t0).count();
        if (ms > e->comm_timeout_ms) {
            (void)ncclCommAbort(e->comm);
            e->comm = nullptr;
            return fail(ALS_ERR_COMM,
                        "rank %d of %d: the engine's stream did not complete within %lld ms; the last RCCL all-gather "
                        "issued was side %s chunk %lld (%lld rows per shard); communicator aborted",
                        e->rank, e->world, (long long)e->comm_timeout_ms,
                        e->last_gather_side == ALS_SIDE_MOVIE ? "movie" : e->last_gather_side == ALS_SIDE_USER ? "user"
                                                                                                              : "none",
                        (long long)e->last_gather_chunk, (long long)e->last_gather_rows);
        }
        if (spin < 1000) std::this_thread::yield();
        else std::this_thread::sleep_for(std::chrono::microseconds(50));
    }
}

int sync_checked(als_engine* e) {
    if (int r = wait_gathers(e, true, true)) return r;
    if (int r = stream_wait(e, e->stream)) return r;
    uint32_t rec[cfk::INTEGRITY_WORDS];
    HIP_TRY(hipMemcpy(rec, e->d_integrity, sizeof(rec), hipMemcpyDeviceToHost));
    if (rec[0] != 0)
        return fail(ALS_ERR_INTEGRITY,
                    "%u REDUCE tasks found partial slots that failed their check (first: launch generation %u, slot "
                    "%u, row %u): partial sums its PARTIAL task's writes had not reached",
                    rec[0], rec[1], rec[2], rec[3]);
    return ALS_OK;
}
int check_side(int side) {
    if (side != ALS_SIDE_MOVIE && side != ALS_SIDE_USER)
        return fail(ALS_ERR_INVALID_ARGUMENT, "side must be ALS_SIDE_MOVIE (0) or ALS_SIDE_USER (1), got %d", side);
    return ALS_OK;
}

void free_block(Block& b) {
    (void)hipFree(b.d_col);
    (void)hipFree(b.d_rat);
    (void)hipFree(b.d_rat_pk);
    (void)hipFree(b.d_col_ps);
    (void)hipFree(b.d_tasks);
    (void)hipFree(b.d_reduce);
    (void)hipFree(b.d_task_se);
    (void)hipFree(b.d_ctasks);
    (void)hipFree(b.d_creduce);
    for (int c = 0; c < 3; ++c) {
        (void)hipFree(b.d_dual[c]);
        (void)hipFree(b.d_cdual[c]);
    }
    (void)hipFree(b.d_sq_tasks);
    b = Block();
}

// Chunk length (entries, multiple of 4) above which a row is split into PARTIAL tasks + a REDUCE task.
// Aim for enough wave-tasks to fill 256 CUs several times over while keeping partial traffic small.
int64_t chunk_entries(int64_t nnz_padded) {
    constexpr int64_t B = cfk::BLOCK_ENTRIES;
    if (const char* env = getenv("ALS_CHUNK")) {
        long v = atol(env);
        if (v >= 1) return (v + B - 1) / B * B;
    }
    // nnz/4096 (24.5k entries at Netflix shape; kbench: movie half + REDUCE 3.38 -> 3.19 ms against the
    // former nnz/24576 <= 8192, fewer 11-KB partial slots and REDUCE solves), still nnz-proportional so a
    // G-way shard keeps enough tasks for load balance
    int64_t c = nnz_padded / 4096;
    c = std::max<int64_t>(c, 1024);
    c = std::min<int64_t>(c, 32768);
    return (c + B - 1) / B * B;
}

}  // namespace

extern "C" {

int als_abi_version(void) { return ALS_ABI_VERSION; }

int als_device_count(int* n) {
    if (!n) return fail(ALS_ERR_INVALID_ARGUMENT, "n is NULL");
    *n = 0;
    HIP_TRY(hipGetDeviceCount(n));
    return ALS_OK;
}
const char* als_last_error(void) { return g_last_error.c_str(); }

#define CFK_STR2(x) #x
#define CFK_STR(x) CFK_STR2(x)
const char* als_build_source_sha256(void) {
#ifdef CFK_SOURCE_SHA256
    return &CFK_STR(CFK_SOURCE_SHA256)[1];   // "h<digest>": an identifier token, the h dropped
#else
    return "";
#endif
}

int als_engine_create(int device, int num_features, int precision, als_engine** out) {
    if (!out) return fail(ALS_ERR_INVALID_ARGUMENT, "out is NULL");
    *out = nullptr;
    if (precision != ALS_F32 && precision != ALS_F64)
        return fail(ALS_ERR_INVALID_ARGUMENT, "precision must be ALS_F32 or ALS_F64");
    if (num_features < 1) return fail(ALS_ERR_INVALID_ARGUMENT, "num_features must be >= 1, got %d", num_features);
    // padded row stride: 16 / 32 / 64 / 128 for the wave-per-row kernels, beyond them (fp32 k > 128, fp64 k > 64:
    // the generic workgroup-per-row path) the next multiple of 16; the reference accepts any NUM_FEATURES
    // (ALSAppRunner.java:18), this build up to 1024
    if (num_features > 1024)
        return fail(ALS_ERR_UNSUPPORTED, "num_features=%d: this build supports 1..1024", num_features);
    const bool generic = num_features > (precision == ALS_F64 ? 64 : 128);
    int kp = num_features <= 16 ? 16 : num_features <= 32 ? 32 : num_features <= 64 ? 64 : 128;
    if (generic) kp = (num_features + 15) / 16 * 16;
    // MFMA Gram only where the accumulation is a real dense contraction (k >= 32, north star); fp64 and
    // small k use the LDS-staged VALU Gram. fp32 Gram products via the exact split (Path::MFMA_SPLIT) by default;
    // ALS_GRAM=f32 selects the v_mfma_f32_16x16x4_f32 path (same accumulator layout, 2.3x the Gram time).
    Path path = generic ? Path::GENERIC : (precision == ALS_F32 && num_features >= 32) ? Path::MFMA_SPLIT : Path::VALU;
    if (path == Path::MFMA_SPLIT)
        if (const char* env = getenv("ALS_GRAM"))
            if (!strcmp(env, "f32")) path = Path::MFMA;
    if (const char* env = getenv("ALS_FORCE_VALU"))
        if (env[0] == '1' && !generic) path = Path::VALU;
    if (!cfk::variant_available(precision, kp, path))
        return fail(ALS_ERR_UNSUPPORTED, "no kernel variant for precision=%d kp=%d", precision, kp);
    int ndev = 0;
    HIP_TRY(hipGetDeviceCount(&ndev));
    if (device < 0 || device >= ndev) return fail(ALS_ERR_INVALID_ARGUMENT, "device %d out of range (%d devices)", device, ndev);
    HIP_TRY(hipSetDevice(device));
    als_engine* e = new als_engine();
    e->device = device;
    e->k = num_features;
    e->kp = kp;
    e->precision = precision;
    e->path = path;
#ifdef CFK_DEBUG_KNOBS
    // work-dropping diagnostics: compiled only into the tools' debug build (Makefile target `debug`), never into
    // the product library
    if (const char* env = getenv("ALS_DEBUG_SKIP_SOLVE"))
        if (env[0] == '1') e->debug_flags |= cfk::SOLVE_FLAG_SKIP_SOLVE;
    if (const char* env = getenv("ALS_DEBUG_SKIP_REFINE"))
        if (env[0] == '1') e->debug_flags |= cfk::SOLVE_FLAG_SKIP_REFINE;
    // integrity fault injection / slot-level diagnostics (tests/test_gpu_integrity.py, tools/split_diag.py): they
    // weaken the partial-slot check, so they exist in the debug build only
    if (const char* env = getenv("ALS_DEBUG_REDUCE_GEN_SKEW")) e->debug_gen_skew = (uint32_t)atoi(env);
    if (const char* env = getenv("ALS_DEBUG_FIXED_GEN")) e->debug_fixed_gen = env[0] == '1';
    if (const char* env = getenv("ALS_DEBUG_EXTRA_LDS")) e->debug_extra_lds = atoi(env);
#endif
    if (const char* env = getenv("ALS_REFINE_MIN_PIVOT")) {
        // the product library can only refine MORE often than the validated gate (> 1: every row); thresholds
        // below 0.45 drop accuracy (tools/refine_accuracy.py) and are accepted by the debug build only
        e->refine_min_pivot = (float)atof(env);
#ifndef CFK_DEBUG_KNOBS
        e->refine_min_pivot = std::max(e->refine_min_pivot, 0.45f);
#endif
    }
    if (const char* env = getenv("ALS_DUAL_SIDE")) e->dual_side = env[0] != '0';
    if (const char* env = getenv("ALS_INTERLEAVE")) e->interleave = env[0] == '0' ? 0 : 1;
    if (const char* env = getenv("ALS_XCD_RANGES")) e->xcd_ranges = env[0] == '0' ? 0 : 1;
    if (const char* env = getenv("ALS_COMM_TIMEOUT_S")) e->comm_timeout_ms = (int64_t)(atof(env) * 1000.0);
    hipError_t st = hipStreamCreateWithFlags(&e->stream, hipStreamNonBlocking);
    if (st != hipSuccess) {
        delete e;
        return fail(ALS_ERR_DEVICE, "hipStreamCreate: %s", hipGetErrorString(st));
    }
    e->own_stream = true;
    st = hipDeviceGetAttribute(&e->cu_count, hipDeviceAttributeMultiprocessorCount, device);
    if (st == hipSuccess) st = hipMalloc((void**)&e->d_integrity, cfk::INTEGRITY_WORDS * sizeof(uint32_t));
    if (st == hipSuccess) st = hipMemset(e->d_integrity, 0, cfk::INTEGRITY_WORDS * sizeof(uint32_t));
    if (st == hipSuccess) st = hipMalloc((void**)&e->d_amax, 2 * sizeof(uint32_t));
    if (st != hipSuccess) {
        (void)hipStreamDestroy(e->stream);
        (void)hipFree(e->d_integrity);
        (void)hipFree(e->d_amax);
        delete e;
        return fail(ALS_ERR_DEVICE, "integrity record: %s", hipGetErrorString(st));
    }
    *out = e;
    return ALS_OK;
}

int als_engine_destroy(als_engine* e) {
    if (!e) return ALS_OK;
    (void)hipSetDevice(e->device);
    (void)hipStreamSynchronize(e->stream);
    for (auto& b : e->blk) free_block(b);
    for (auto& f : e->fac)
        if (f.owned) (void)hipFree(f.ptr);
    (void)hipFree(e->d_partials);
    (void)hipFree(e->d_split);
    (void)hipHostFree(e->h_stage);
    (void)hipFree(e->d_integrity);
    (void)hipFree(e->d_amax);
    for (auto& rec : e->pending)
        for (auto ev : rec.ev) (void)hipEventDestroy(ev);
    for (auto ev : e->ev_pool) (void)hipEventDestroy(ev);
    if (e->comm_stream) (void)hipStreamSynchronize(e->comm_stream);
    if (e->comm) (void)ncclCommDestroy(e->comm);
    if (e->comm_stream) (void)hipStreamDestroy(e->comm_stream);
    for (auto ev : {e->solved, e->gathered[0], e->gathered[1]})
        if (ev) (void)hipEventDestroy(ev);
    if (e->side_stream) {
        (void)hipStreamSynchronize(e->side_stream);
        (void)hipStreamDestroy(e->side_stream);
    }
    for (auto ev : {e->fork, e->join})
        if (ev) (void)hipEventDestroy(ev);
    if (e->own_stream) (void)hipStreamDestroy(e->stream);
    delete e;
    return ALS_OK;
}

int als_engine_set_stream(als_engine* e, void* hip_stream) {
    if (int r = check_engine(e)) return r;
    HIP_TRY(hipSetDevice(e->device));
    if (e->own_stream) {
        HIP_TRY(hipStreamSynchronize(e->stream));
        HIP_TRY(hipStreamDestroy(e->stream));
        e->own_stream = false;
        e->stream = nullptr;
    }
    if (hip_stream) {
        e->stream = (hipStream_t)hip_stream;
    } else {
        HIP_TRY(hipStreamCreateWithFlags(&e->stream, hipStreamNonBlocking));
        e->own_stream = true;
    }
    return ALS_OK;
}

int als_engine_use_default_stream(als_engine* e) {
    if (int r = check_engine(e)) return r;
    HIP_TRY(hipSetDevice(e->device));
    if (e->own_stream) {
        HIP_TRY(hipStreamSynchronize(e->stream));
        HIP_TRY(hipStreamDestroy(e->stream));
        e->own_stream = false;
    }
    e->stream = nullptr;   // hipStream_t 0: the legacy default stream
    return ALS_OK;
}

int als_factor_stride(const als_engine* e) { return e ? e->kp : 0; }

}  // extern "C"

namespace {

int ensure_stage(als_engine* e) {
    constexpr size_t STAGE = 32u << 20;
    if (!e->h_stage) {
        HIP_TRY(hipHostMalloc(&e->h_stage, STAGE, hipHostMallocDefault));
        e->stage_bytes = STAGE;
    }
    return ALS_OK;
}

int check_block_shape(als_engine* e, int64_t n_rows, int64_t row_offset, int64_t n_opp_rows) {
    if (n_rows < 0 || row_offset < 0 || n_opp_rows < 0)
        return fail(ALS_ERR_INVALID_ARGUMENT, "negative size (n_rows=%lld row_offset=%lld n_opp_rows=%lld)",
                    (long long)n_rows, (long long)row_offset, (long long)n_opp_rows);
    if (n_rows > INT32_MAX) return fail(ALS_ERR_UNSUPPORTED, "n_rows exceeds 2^31-1");
    if (n_opp_rows >= INT32_MAX) return fail(ALS_ERR_UNSUPPORTED, "n_opp_rows must be < 2^31-1 (int32 column indices)");
    if ((n_opp_rows + 1) * (int64_t)e->kp * (int64_t)e->elem() > (int64_t)UINT32_MAX)
        return fail(ALS_ERR_UNSUPPORTED, "opposite factor matrix exceeds 4 GiB (32-bit gather offsets)");
    return ALS_OK;
}

// Padded entries of a row of degree d (every row starts on a 32-entry block).
inline int64_t padded(int64_t d) { return (d + cfk::BLOCK_ENTRIES - 1) / cfk::BLOCK_ENTRIES * cfk::BLOCK_ENTRIES; }

// Interleaved split rows: on a half whose opposite table outgrows the L2s but fits the Infinity
// Cache (the 123 / 246 MB user table of the Netflix-shape movie half at k = 64 / 128, the 256 MB item table of the
// power-law user half), a row longer than the returned length (entries) is split into
// nc = ceil(d / length) chunks of INTERLEAVED blocks -- chunk c = blocks c, c + nc, c + 2 nc, ... of the row -- so
// that every chunk covers the row's whole range of opposite slots. With the chunks dispatched together (longest
// first) the waves of an XCD then walk the opposite table in step and find its rows in their L2. Such a half gathers
// the pre-split table (the fp16 Gram). 0: contiguous chunks at chunk_entries() (the other halves).
int64_t interleave_chunk(const als_engine* e, int64_t n_opp_rows, const std::vector<int64_t>& deg) {
    const int64_t sb = (n_opp_rows + 1) * (int64_t)cfk::presplit_row_bytes(e->kp);
    if (e->interleave == 0 || e->path != Path::MFMA_SPLIT || (e->kp != 64 && e->kp != 128)) return 0;
    if (n_opp_rows + 1 >= (1 << 24) || sb > (int64_t)UINT32_MAX) return 0;   // the pre-split gather's offsets
    // auto: a table the L2s cannot hold (> 32 MB) that the 256 MiB Infinity Cache still holds; beyond the IC (configs[4]'s
    // 2.56 GB user table) the contiguous chunks read the long rows' near-dense user ranges in order and win (item half
    // of the power-law shard: 8.87 vs 14.6 ms interleaved, profiles/r06a)
    if (e->interleave < 0 && (sb <= (32ll << 20) || sb > (256ll << 20))) return 0;
    auto long_work = [&](int64_t t) {   // entries in rows longer than t
        int64_t w = 0;
        for (int64_t d : deg) w += d > t ? d : 0;
        return w;
    };
    // the walk in step needs many chunks in flight: resident waves of the pre-split launch (4 per SIMD at KP = 64, 1 at
    // KP = 128). Chunk length (kbench, Netflix shape, movie half + its REDUCE, profiles/r06a): k = 64, whole data:
    // 8,192 / 10,240 / 12,288 / 16,384 / 24,576 entries 2.07 / 2.04 / 2.06 / 2.16 / 2.29 ms (contiguous chunks: 2.98);
    // one rank's shard of G = 2 / 4 / 8 (fewer chunks than twice the resident waves): 1.52 / 0.95 / 0.66 ms at the
    // best length vs 1.58 / 0.90 / 0.47 contiguous -- so k = 64 interleaves only with >= 1.5 x the resident waves of
    // chunks. k = 128 (whole data 4,096 / 8,192 / 16,384: 5.76 / 5.32 / 5.06 ms, contiguous 6.67; shards of G = 2 / 4
    // / 8 at 8,192: 4.92 / 2.55 / 1.37 vs 5.25 / 2.77 / 1.50) always. Round 6 (profiles/r06c/xcd2_*.log, movie half +
    // REDUCE): whole data 16,384 / 8,192 / 4,096: 5.07 / 5.26 / 5.71 ms; shards of G = 2 / 4 / 8 at 4,096: 4.17 / 2.36 /
    // ~1.40 ms vs 4.98 / 2.57 / 1.39 at 8,192 (2,048: 4.13 / 2.29 / 1.40; its REDUCE launch doubles) -- so 16,384 when
    // the long rows hold over ~4 chunks of it per resident wave (the whole Netflix shape), else 4,096.
    const int64_t conc = (int64_t)std::max(1, e->cu_count) * (e->kp == 128 ? 4 : 16);
    int64_t len;
    if (e->kp == 64) {
        len = 10240;
        // the concurrency rule holds for the 123 MB user table of a Netflix shard; the 256 MB item table of the
        // power-law shard's user half interleaves whatever its long-row work (9.43 -> 7.38 ms, profiles/r06a; the rule
        // alone had turned it off again: 9.47-9.57 ms, profiles/r06c/ranges_bench_ab)
        if (e->interleave < 0 && sb <= (128ll << 20) && long_work(len) < len * conc * 3 / 2) return 0;
    } else {
        len = long_work(16384) >= 16384 * 4 * conc ? 16384 : 4096;
    }
#ifdef CFK_DEBUG_KNOBS
    if (const char* v = getenv("ALS_ILV_CHUNK")) len = std::max(32L, atol(v));
#endif
    return (len + cfk::BLOCK_ENTRIES - 1) / cfk::BLOCK_ENTRIES * cfk::BLOCK_ENTRIES;
}

// Work plan of a block whose padded in-block (d_col / d_rat, device, already laid out) has row degrees deg[]
// and row starts begin[]: FULL / PARTIAL / REDUCE tasks, longest first; uploads the plan, takes ownership of
// d_col / d_rat and sizes the partial and pre-split workspaces.
int finish_block(als_engine* e, int side, int64_t n_rows, int64_t row_offset, int64_t n_opp_rows, int64_t nnz,
                 const std::vector<int64_t>& deg, const std::vector<int64_t>& begin, int32_t* d_col, float* d_rat) {
    const int64_t nnz_padded = begin[n_rows];
    auto drop = [&]() {
        (void)hipFree(d_col);
        (void)hipFree(d_rat);
    };
    // the generic path's workgroup takes a whole row of any length: no split rows
    const int64_t chunk = e->path == Path::GENERIC ? INT64_MAX : chunk_entries(nnz_padded);
    std::vector<Task> tasks, reduce, stasks;
    int64_t slots = 0;
    // Interleaved split rows: the long rows' blocks are permuted chunk-major (chunk c = blocks c, c + nc, ... of the
    // row, in order), each chunk one PARTIAL task of whole blocks (the row's last, padded block is the last block of
    // its chunk, so nent counts exactly the chunk's real entries), one REDUCE per row.
    // (no longer than the contiguous chunk: a small block keeps enough tasks for load balance)
    const int64_t ilv = std::min(interleave_chunk(e, n_opp_rows, deg), chunk);
    std::vector<int32_t> perm;
    std::vector<int8_t> srange;   // XCD range of each interleaved chunk task (ranges only)
    int64_t ilv_rows = 0;
    // XCD ranges (ALS_XCD_RANGES): a long row's blocks are first grouped by the opposite slot of their first entry
    // into X = 8 ranges of the opposite table (a row's entries ascend by slot, so each range is a run of its blocks),
    // then each range's blocks are interleaved into chunks as below. Chunk tasks of range x all run on one XCD (the
    // task order below), so that XCD's L2 serves 1/8 of the table instead of every XCD fetching all of it.
    // Measured (profiles/r06c/ranges_*.log): the k = 64 Netflix-shape movie half (123 MB user table, one launch) 2.00
    // -> 1.80 ms, iteration 4.73 -> 4.60 ms; the k = 128 movie half (246 MB) and the power-law shard's chunked item-table
    // half (256 MB) a little slower, shards of G = 2 / 4 slower than their contiguous plan -- so auto = KP = 64 with an
    // opposite table within 128 MiB (each XCD's range within 16 MiB).
    constexpr int XR = 8;
    const bool ranges = ilv > 0 && n_opp_rows > 0 &&
                        (e->xcd_ranges > 0 ||
                         (e->xcd_ranges < 0 && e->kp == 64 &&
                          (n_opp_rows + 1) * (int64_t)cfk::presplit_row_bytes(e->kp) <= (128ll << 20)));
    std::vector<int32_t> bfirst;   // opposite slot of every block's first entry (physical position 0 of the block)
    if (ranges && nnz_padded > 0) {
        bfirst.resize((size_t)(nnz_padded / cfk::BLOCK_ENTRIES));
        hipError_t st = hipMemcpy2D(bfirst.data(), 4, d_col, cfk::BLOCK_ENTRIES * 4, 4, bfirst.size(),
                                    hipMemcpyDeviceToHost);
        if (st != hipSuccess) {
            drop();
            return fail(ALS_ERR_DEVICE, "set_block: block heads: %s", hipGetErrorString(st));
        }
    }
    if (ilv > 0) {
        constexpr int64_t BE = cfk::BLOCK_ENTRIES;
        std::vector<int64_t> piece[XR];
        for (int64_t i = 0; i < n_rows; ++i) {
            const int64_t d = deg[i];
            if (d <= ilv) continue;
            if (perm.empty()) {
                perm.resize((size_t)(nnz_padded / BE));
                for (size_t q = 0; q < perm.size(); ++q) perm[q] = (int32_t)q;
            }
            ++ilv_rows;
            const int64_t nb = (d + BE - 1) / BE, b0 = begin[i] / BE;
            for (auto& v : piece) v.clear();
            for (int64_t q = 0; q < nb; ++q) {
                const int x = ranges ? (int)std::min<int64_t>(XR - 1, (int64_t)bfirst[(size_t)(b0 + q)] * XR / n_opp_rows)
                                     : 0;
                piece[x].push_back(q);
            }
            Task t{};
            t.row = (int32_t)i;
            t.ndeg = (int32_t)d;
            t.kind = cfk::TASK_PARTIAL;
            const int64_t first = slots;
            int64_t pos = 0;
            for (int x = 0; x < XR; ++x) {
                const std::vector<int64_t>& pb = piece[x];
                if (pb.empty()) continue;
                const int64_t np = (int64_t)pb.size();
                const bool has_last = pb.back() == nb - 1;   // the row's padded block: last of its chunk below
                const int64_t pent = BE * np - (has_last ? BE * nb - d : 0);
                const int64_t nc = (pent + ilv - 1) / ilv;
                for (int64_t c = 0; c < nc; ++c) {
                    const int64_t p0 = pos;
                    bool last = false;
                    for (int64_t y = c; y < np; y += nc) {
                        perm[(size_t)(b0 + pos++)] = (int32_t)(b0 + pb[(size_t)y]);
                        last = pb[(size_t)y] == nb - 1;
                    }
                    const int64_t cnt = pos - p0;
                    const int64_t nent = last ? BE * (cnt - 1) + (d - BE * (nb - 1)) : BE * cnt;
                    Task p = t;
                    p.begin = begin[i] + BE * p0;
                    p.nent = (int32_t)nent;
                    p.nsteps = (int32_t)((nent + 3) / 4);
                    p.slot = (int32_t)slots++;
                    stasks.push_back(p);
                    srange.push_back((int8_t)x);
                }
            }
            Task r = t;
            r.begin = 0;
            r.slot = (int32_t)first;
            r.nsteps = (int32_t)(slots - first);
            r.kind = cfk::TASK_REDUCE;
            reduce.push_back(r);
        }
    }
    const int64_t ilv_tasks = (int64_t)stasks.size();
    for (int64_t i = 0; i < n_rows; ++i) {
        if (ilv > 0 && deg[i] > ilv) continue;   // interleaved above
        const int64_t d = deg[i];
        Task t{};
        t.row = (int32_t)i;
        t.ndeg = (int32_t)d;
        if (d <= chunk) {
            t.begin = begin[i];
            t.nsteps = (int32_t)((d + 3) / 4);
            t.nent = (int32_t)d;
            t.slot = -1;
            t.kind = cfk::TASK_FULL;
            tasks.push_back(t);
        } else {
            const int64_t first = slots;
            for (int64_t o = 0; o < d; o += chunk) {
                Task p = t;
                p.begin = begin[i] + o;
                p.nsteps = (int32_t)((std::min(chunk, d - o) + 3) / 4);
                p.nent = (int32_t)std::min(chunk, d - o);
                p.slot = (int32_t)slots++;
                p.kind = cfk::TASK_PARTIAL;
                tasks.push_back(p);
            }
            Task r = t;
            r.begin = 0;
            r.slot = (int32_t)first;
            r.nsteps = (int32_t)(slots - first);
            r.kind = cfk::TASK_REDUCE;
            reduce.push_back(r);
        }
    }
    // Short rows in entry space (split-bf16 path): rows of <= 3 blocks at KP = 128, 1 block at KP = 64 solve the
    // (padded entries)^2 system of als_solve_dual instead of the KP x KP one. Only rows with n <= k entries: then
    // Y Y^T + lambda n I_n has the nonzero spectrum of Y^T Y + lambda n I_k plus nothing smaller, so the same
    // conditioning; with n > k the n x n system would carry n - k eigenvalues lambda n only (singular at
    // lambda = 0 where the reference's k x k system is not). ALS_DUAL=0 turns it off.
    std::vector<Task> sq_all = stasks;
    sq_all.insert(sq_all.end(), tasks.begin(), tasks.end());
    std::vector<Task> dual[3];
    {
        const int max_cd = e->path != Path::MFMA_SPLIT ? 0 : e->kp == 128 ? 6 : e->kp == 64 ? 2 : 0;
        bool on = max_cd > 0;
        if (const char* env = getenv("ALS_DUAL")) on = on && env[0] != '0';
        if (on) {
            std::vector<Task> keep;
            for (const Task& t : tasks) {
                const int cd = 2 * ((t.nent + cfk::BLOCK_ENTRIES - 1) / cfk::BLOCK_ENTRIES);
                if (t.kind == cfk::TASK_FULL && t.ndeg > 0 && t.ndeg <= e->k && cd <= max_cd)
                    dual[cd / 2 - 1].push_back(t);
                else
                    keep.push_back(t);
            }
            tasks.swap(keep);
        }
    }
    if (slots > INT32_MAX || tasks.size() > (size_t)INT32_MAX) {
        drop();
        return fail(ALS_ERR_UNSUPPORTED, "too many tasks / partial slots");
    }
    // Longest tasks first (LPT): the grid drains with a short tail.
    std::stable_sort(tasks.begin(), tasks.end(), [](const Task& a, const Task& b) { return a.nsteps > b.nsteps; });
#ifdef CFK_DEBUG_KNOBS
    // ALS_TASK_ORDER=random / stagger[:W] (measurement knobs, debug build only): a seeded shuffle of the main launch's
    // tasks, or LPT windows alternating between its longer and shorter half
    if (const char* env = getenv("ALS_TASK_ORDER")) {
        if (std::strncmp(env, "stagger", 7) == 0) {
            // windows of W tasks (W = stagger:<W>, default 1024 = one 4-wave workgroup per CU) alternate between the
            // longer and the shorter half of the LPT list: co-resident waves of a CU run tasks of different lengths
            const size_t W = env[7] == ':' ? (size_t)std::max(1, atoi(env + 8)) : 1024;
            const size_t h = (tasks.size() + 1) / 2;
            std::vector<Task> out;
            out.reserve(tasks.size());
            size_t ia = 0, ib = h;
            while (ia < h || ib < tasks.size()) {
                for (size_t q = 0; q < W && ia < h; ++q) out.push_back(tasks[ia++]);
                for (size_t q = 0; q < W && ib < tasks.size(); ++q) out.push_back(tasks[ib++]);
            }
            tasks.swap(out);
        }
        if (std::strcmp(env, "random") == 0) {
            uint64_t x = 0x9e3779b97f4a7c15ull;
            for (size_t i = tasks.size(); i > 1; --i) {
                x ^= x << 13;
                x ^= x >> 7;
                x ^= x << 17;
                std::swap(tasks[i - 1], tasks[(size_t)(x % i)]);
            }
        }
    }
#endif
    std::stable_sort(reduce.begin(), reduce.end(), [](const Task& a, const Task& b) { return a.nsteps > b.nsteps; });
    for (auto& d : dual)
        std::stable_sort(d.begin(), d.end(), [](const Task& a, const Task& b) { return a.nsteps > b.nsteps; });

    // the interleaved chunks join the plain tasks, longest first
    if (!stasks.empty() && ranges) {
        // XCD ranges: workgroup w runs on the XCD of w % 8 (round-robin placement; speed only, never correctness), so
        // the workgroups at positions w = 8 j + x take range x's chunk tasks (queue x). The plain (whole-row) tasks have
        // no range: each goes, longest first, to the queue of least work among those still short of an equal share of
        // the task count, so the queues stay aligned to the round-robin. Every queue is longest first.
        std::vector<Task> q[XR];
        int64_t work[XR] = {};
        for (size_t t = 0; t < stasks.size(); ++t) {
            q[srange[t]].push_back(stasks[t]);
            work[srange[t]] += stasks[t].nsteps;
        }
        const int64_t total = (int64_t)(stasks.size() + tasks.size());
        const int64_t wgs = (total + 3) / 4;
        for (const Task& t : tasks) {   // already longest first
            int best = -1;
            for (int x = 0; x < XR; ++x) {
                const int64_t cap = 4 * ((wgs - x + XR - 1) / XR);   // tasks of the workgroups at w = x mod 8
                if ((int64_t)q[x].size() < cap && (best < 0 || work[x] < work[best])) best = x;
            }
            if (best < 0) best = (int)(std::min_element(work, work + XR) - work);
            q[best].push_back(t);
            work[best] += t.nsteps;
        }
        std::vector<Task> out;
        out.reserve((size_t)total);
        for (int x = 0; x < XR; ++x)
            std::stable_sort(q[x].begin(), q[x].end(), [](const Task& a, const Task& b) { return a.nsteps > b.nsteps; });
        for (size_t j = 0;; j += 4) {
            bool any = false;
            for (int x = 0; x < XR; ++x)
                for (size_t u = j; u < j + 4 && u < q[x].size(); ++u) {
                    out.push_back(q[x][u]);
                    any = true;
                }
            if (!any) break;
        }
        tasks.swap(out);
    } else if (!stasks.empty()) {
        tasks.insert(tasks.begin(), stasks.begin(), stasks.end());
        std::stable_sort(tasks.begin(), tasks.end(), [](const Task& a, const Task& b) { return a.nsteps > b.nsteps; });
    }

    hipError_t st0 = hipSetDevice(e->device);
    if (st0 == hipSuccess) st0 = hipStreamSynchronize(e->stream);
    if (st0 == hipSuccess && !perm.empty()) {
        // the long rows' blocks chunk-major (before the pre-split packing below derives its arrays from them)
        int32_t *d_perm = nullptr, *col2 = nullptr;
        float* rat2 = nullptr;
        st0 = hipMalloc((void**)&d_perm, perm.size() * 4);
        if (st0 == hipSuccess) st0 = hipMalloc((void**)&col2, (size_t)nnz_padded * 4);
        if (st0 == hipSuccess) st0 = hipMalloc((void**)&rat2, (size_t)nnz_padded * 4);
        if (st0 == hipSuccess) st0 = hipMemcpy(d_perm, perm.data(), perm.size() * 4, hipMemcpyHostToDevice);
        if (st0 == hipSuccess)
            st0 = cfk::launch_permute_blocks(d_col, d_rat, col2, rat2, d_perm, (int64_t)perm.size(), nullptr);
        if (st0 == hipSuccess) st0 = hipDeviceSynchronize();
        (void)hipFree(d_perm);
        if (st0 == hipSuccess) {
            std::swap(d_col, col2);
            std::swap(d_rat, rat2);
        }
        (void)hipFree(col2);
        (void)hipFree(rat2);
    }
    if (st0 != hipSuccess) {
        drop();
        return fail(ALS_ERR_DEVICE, "set_block: %s", hipGetErrorString(st0));
    }
    Block& blk = e->blk[side];
    free_block(blk);
    blk.d_col = d_col;
    blk.d_rat = d_rat;
    blk.n_rows = n_rows;
    blk.row_offset = row_offset;
    blk.n_opp_rows = n_opp_rows;
    blk.nnz = nnz;
    blk.nnz_padded = nnz_padded;
    blk.n_tasks = (int32_t)tasks.size();
    blk.n_reduce = (int32_t)reduce.size();
    blk.n_slots = (int32_t)slots;
    // Pre-split opposite table (scaled two-term fp16, cfk::launch_presplit, once per half) for the MFMA Gram: 4 KP
    // bytes per row (the fp32 row's size), 3 MFMAs per tile instead of the on-the-fly bf16 split's 6, no split VALU
    // (the rows reach LDS by DMA and the MFMA operands come back with transposed reads). Chosen where the Gram is
    // MFMA-bound: always at KP = 128, and at KP = 64 for a cache-resident opposite table (<= 8 MB: the 17,770-row
    // movie table of the user half, 2.99 vs 4.37 ms). The KP = 64 movie half gathers the 123 MB user table at the
    // Infinity-Cache ceiling either way, and the split pass over that table would cost more than it saves (3.08 vs
    // 3.01 ms; kbench). ALS_PRESPLIT=0/1 forces it off/on.
    {
        const int64_t sb = (n_opp_rows + 1) * (int64_t)cfk::presplit_row_bytes(e->kp);
        const bool ps_kp = e->path == Path::MFMA_SPLIT && (e->kp == 64 || e->kp == 128);
        bool ps = ps_kp && (e->kp == 128 || sb <= (8ll << 20) || ilv > 0);
        if (const char* env = getenv("ALS_PRESPLIT")) ps = ps_kp && env[0] == '1';
        // the pre-split gather forms 32-bit byte offsets row * presplit_row_bytes with a 24-bit multiply: both the
        // row (< 2^24) and the offset (< 2^32) must fit, also when ALS_PRESPLIT=1 forces the path
        if (n_opp_rows + 1 >= (1 << 24) || sb > (int64_t)UINT32_MAX) ps = false;
        blk.presplit = ps;
        if (ps && (size_t)sb > e->split_bytes) {
            (void)hipFree(e->d_split);
            e->d_split = nullptr;
            e->split_bytes = 0;
            hipError_t st = hipMalloc(&e->d_split, (size_t)sb);
            if (st != hipSuccess) return fail(ALS_ERR_OUT_OF_MEMORY, "pre-split hipMalloc(%lld): %s", (long long)sb,
                                              hipGetErrorString(st));
            e->split_bytes = (size_t)sb;
        }
        if (ps && nnz_padded > 0) {
            // the RHS operand's ratings, packed once (setup time): fp16 rh pairs, then rm pairs
            hipError_t st = hipMalloc((void**)&blk.d_rat_pk, (size_t)nnz_padded * 4);
            if (st != hipSuccess) return fail(ALS_ERR_OUT_OF_MEMORY, "hipMalloc(%lld): %s", (long long)nnz_padded * 4,
                                              hipGetErrorString(st));
            st = cfk::launch_pack_ratings(blk.d_rat, blk.d_rat_pk, nnz_padded / 2, nullptr);
            // and the column indices in the order of the LDS-DMA gather (one 16-B load per loader row)
            if (st == hipSuccess) st = hipMalloc((void**)&blk.d_col_ps, (size_t)nnz_padded * 4);
            if (st == hipSuccess) st = cfk::launch_pack_cols_ps(blk.d_col, blk.d_col_ps, nnz_padded, nullptr);
            if (st == hipSuccess) st = hipDeviceSynchronize();
            if (st != hipSuccess) return fail(ALS_ERR_DEVICE, "pack ratings: %s", hipGetErrorString(st));
        }
    }
    auto up = [&](void** dst, const void* src, size_t bytes) -> int {
        if (bytes == 0) return ALS_OK;
        hipError_t st = hipMalloc(dst, bytes);
        if (st != hipSuccess) return fail(ALS_ERR_OUT_OF_MEMORY, "hipMalloc(%zu): %s", bytes, hipGetErrorString(st));
        st = hipMemcpy(*dst, src, bytes, hipMemcpyHostToDevice);
        if (st != hipSuccess) return fail(ALS_ERR_DEVICE, "hipMemcpy: %s", hipGetErrorString(st));
        return ALS_OK;
    };
    int r;
    if ((r = up((void**)&blk.d_tasks, tasks.data(), tasks.size() * sizeof(Task)))) return r;
    blk.ilv_rows = ilv_rows;
    blk.ilv_tasks = ilv_tasks;
    blk.ilv_chunk = ilv;
    if ((r = up((void**)&blk.d_reduce, reduce.data(), reduce.size() * sizeof(Task)))) return r;
    for (int c = 0; c < 3; ++c) {
        if ((r = up((void**)&blk.d_dual[c], dual[c].data(), dual[c].size() * sizeof(Task)))) return r;
        blk.n_dual[c] = (int32_t)dual[c].size();
        blk.h_dual[c] = std::move(dual[c]);
    }
    if ((r = up((void**)&blk.d_sq_tasks, sq_all.data(), sq_all.size() * sizeof(Task)))) return r;
    blk.n_sq = (int32_t)sq_all.size();
    if (!sq_all.empty()) HIP_TRY(hipMalloc((void**)&blk.d_task_se, sq_all.size() * sizeof(double)));
    blk.h_tasks = std::move(tasks);
    blk.h_reduce = std::move(reduce);
    // Partial workspace sized for the larger side (the generic path: its per-workgroup Gram slabs, when the packed
    // triangle does not fit in LDS -- up to 1024 workgroups within 4 GiB)
    size_t need = (size_t)slots * cfk::partial_words_per_lane(e->precision, e->kp, e->path) * 64 * e->elem();
    if (e->path == Path::GENERIC) {
        const cfk::GenericPlan gp = cfk::generic_plan(e->precision, e->kp);
        if (!gp.g_in_lds) {
            const int64_t slab = gp.slab_elems * (int64_t)e->elem();
            e->generic_slabs = std::max<int64_t>(1, std::min<int64_t>(1024, (4ll << 30) / slab));
            need = (size_t)(e->generic_slabs * slab);
        }
    }
    if (need > e->partial_bytes) {
        (void)hipFree(e->d_partials);
        e->d_partials = nullptr;
        e->partial_bytes = 0;
        hipError_t st = hipMalloc(&e->d_partials, need);
        if (st != hipSuccess) return fail(ALS_ERR_OUT_OF_MEMORY, "partials hipMalloc(%zu): %s", need, hipGetErrorString(st));
        e->partial_bytes = need;
    }
    blk.set = true;
    return ALS_OK;
}

}  // namespace

extern "C" {

int als_set_block(als_engine* e, int side, int64_t n_rows, int64_t row_offset, int64_t n_opp_rows,
                  const int64_t* row_ptr, const int32_t* col_idx, const int16_t* ratings) {
    if (int r = check_engine(e)) return r;
    if (int r = check_side(side)) return r;
    if (int r = check_block_shape(e, n_rows, row_offset, n_opp_rows)) return r;
    if (n_rows > 0 && !row_ptr) return fail(ALS_ERR_INVALID_ARGUMENT, "row_ptr is NULL");
    const int64_t nnz = n_rows > 0 ? row_ptr[n_rows] : 0;
    if (n_rows > 0 && row_ptr[0] != 0) return fail(ALS_ERR_INVALID_ARGUMENT, "row_ptr[0] must be 0");
    if (nnz > 0 && (!col_idx || !ratings)) return fail(ALS_ERR_INVALID_ARGUMENT, "col_idx/ratings NULL");
    // Validate the block on the host: a bad index would fault the GPU.
    std::vector<int64_t> deg(n_rows), begin(n_rows + 1);
    int64_t o = 0;
    for (int64_t i = 0; i < n_rows; ++i) {
        const int64_t d = row_ptr[i + 1] - row_ptr[i];
        if (d < 0) return fail(ALS_ERR_INVALID_ARGUMENT, "row_ptr not monotone at row %lld", (long long)i);
        if (d > INT32_MAX / 2) return fail(ALS_ERR_UNSUPPORTED, "row %lld has %lld entries", (long long)i, (long long)d);
        deg[i] = d;
        begin[i] = o;
        o += padded(d);
    }
    begin[n_rows] = o;
    for (int64_t t = 0; t < nnz; ++t)
        if (col_idx[t] < 0 || col_idx[t] >= n_opp_rows)
            return fail(ALS_ERR_INVALID_ARGUMENT, "col_idx[%lld]=%d outside [0, %lld)", (long long)t, col_idx[t],
                        (long long)n_opp_rows);
    // Padded, block-interleaved device in-block (see cfk::block_position): every row starts on a
    // 32-entry block; padding entries point at the sentinel zero row (col = n_opp_rows) with rating 0.
    std::vector<int32_t> col(o, (int32_t)n_opp_rows);
    std::vector<float> rat(o, 0.f);
    for (int64_t i = 0; i < n_rows; ++i)
        for (int64_t t = 0; t < deg[i]; ++t) {
            const int64_t pos = begin[i] + cfk::block_position(t);
            col[pos] = col_idx[row_ptr[i] + t];
            rat[pos] = (float)ratings[row_ptr[i] + t];
        }
    HIP_TRY(hipSetDevice(e->device));
    int32_t* d_col = nullptr;
    float* d_rat = nullptr;
    if (o > 0) {
        hipError_t st = hipMalloc((void**)&d_col, o * 4);
        if (st == hipSuccess) st = hipMalloc((void**)&d_rat, o * 4);
        if (st == hipSuccess) st = hipMemcpy(d_col, col.data(), o * 4, hipMemcpyHostToDevice);
        if (st == hipSuccess) st = hipMemcpy(d_rat, rat.data(), o * 4, hipMemcpyHostToDevice);
        if (st != hipSuccess) {
            (void)hipFree(d_col);
            (void)hipFree(d_rat);
            return fail(ALS_ERR_OUT_OF_MEMORY, "in-block upload: %s", hipGetErrorString(st));
        }
    }
    return finish_block(e, side, n_rows, row_offset, n_opp_rows, nnz, deg, begin, d_col, d_rat);
}

int als_set_block_coo(als_engine* e, int side, int64_t n_rows, int64_t row_offset, int64_t n_opp_rows, int64_t nnz,
                      const int32_t* rows, const int32_t* cols, const int16_t* ratings) {
    if (int r = check_engine(e)) return r;
    if (int r = check_side(side)) return r;
    if (int r = check_block_shape(e, n_rows, row_offset, n_opp_rows)) return r;
    if (nnz < 0) return fail(ALS_ERR_INVALID_ARGUMENT, "nnz < 0");
    if (nnz > 0 && (!rows || !cols || !ratings)) return fail(ALS_ERR_INVALID_ARGUMENT, "rows/cols/ratings NULL");
    if (nnz >= INT32_MAX) return fail(ALS_ERR_UNSUPPORTED, "nnz per block must be < 2^31-1 (shard the side)");
    HIP_TRY(hipSetDevice(e->device));
    std::vector<int64_t> deg, begin;
    int32_t* d_col = nullptr;
    float* d_rat = nullptr;
    std::string err;
    const int code = cfk::build_block_device(rows, cols, ratings, nnz, n_rows, n_opp_rows, e->stream, deg, begin,
                                             &d_col, &d_rat, err);
    if (code != ALS_OK) return fail(code, "als_set_block_coo: %s", err.c_str());
    return finish_block(e, side, n_rows, row_offset, n_opp_rows, nnz, deg, begin, d_col, d_rat);
}

int als_alloc_factors(als_engine* e, int side, int64_t n_total_rows) {
    if (int r = check_engine(e)) return r;
    if (int r = check_side(side)) return r;
    if (n_total_rows < 0) return fail(ALS_ERR_INVALID_ARGUMENT, "n_total_rows < 0");
    HIP_TRY(hipSetDevice(e->device));
    Factors& f = e->fac[side];
    if (f.owned) (void)hipFree(f.ptr);
    f = Factors();
    const size_t bytes = (size_t)(n_total_rows + 1) * e->kp * e->elem();   // + sentinel zero row
    hipError_t st = hipMalloc(&f.ptr, bytes);
    if (st != hipSuccess) return fail(ALS_ERR_OUT_OF_MEMORY, "factors hipMalloc(%zu): %s", bytes, hipGetErrorString(st));
    f.owned = true;
    f.n_rows = n_total_rows;
    HIP_TRY(hipMemsetAsync(f.ptr, 0, bytes, e->stream));
    HIP_TRY(hipStreamSynchronize(e->stream));
    return ALS_OK;
}

int als_bind_factors(als_engine* e, int side, void* device_ptr, int64_t n_total_rows) {
    if (int r = check_engine(e)) return r;
    if (int r = check_side(side)) return r;
    if (!device_ptr || n_total_rows < 0) return fail(ALS_ERR_INVALID_ARGUMENT, "bad device buffer");
    Factors& f = e->fac[side];
    if (f.owned) (void)hipFree(f.ptr);
    f.ptr = device_ptr;
    f.n_rows = n_total_rows;
    f.owned = false;
    // the sentinel row after the last factor row must read as zeros (padding entries gather it). The buffer's
    // owner may still have work on it queued on another stream (e.g. torch's zero fill): drain the device first,
    // so the memset and every later engine access are ordered after it.
    HIP_TRY(hipSetDevice(e->device));
    HIP_TRY(hipDeviceSynchronize());
    HIP_TRY(hipMemsetAsync((char*)device_ptr + (size_t)n_total_rows * e->kp * e->elem(), 0, (size_t)e->kp * e->elem(),
                           e->stream));
    HIP_TRY(hipStreamSynchronize(e->stream));
    return ALS_OK;
}

int als_factors_device_ptr(const als_engine* e, int side, void** device_ptr, int64_t* n_total_rows) {
    if (int r = check_engine(e)) return r;
    if (int r = check_side(side)) return r;
    if (device_ptr) *device_ptr = e->fac[side].ptr;
    if (n_total_rows) *n_total_rows = e->fac[side].n_rows;
    return ALS_OK;
}

int als_write_factors(als_engine* e, int side, int64_t row0, int64_t n_rows, const void* host_src, int64_t src_ld) {
    if (int r = check_engine(e)) return r;
    if (int r = check_side(side)) return r;
    const Factors& f = e->fac[side];
    if (!f.ptr) return fail(ALS_ERR_STATE, "factors of side %d not allocated/bound", side);
    if (row0 < 0 || n_rows < 0 || row0 + n_rows > f.n_rows) return fail(ALS_ERR_INVALID_ARGUMENT, "row range out of bounds");
    if (src_ld < e->k) return fail(ALS_ERR_INVALID_ARGUMENT, "src_ld (%lld) < num_features (%d)", (long long)src_ld, e->k);
    if (n_rows == 0) return ALS_OK;
    if (!host_src) return fail(ALS_ERR_INVALID_ARGUMENT, "host_src is NULL");
    HIP_TRY(hipSetDevice(e->device));
    if (int r = wait_gathers(e, true, true)) return r;
    const size_t es = e->elem();
    // Rows are packed kp wide (padding columns zero) into pinned staging and written by a copy kernel
    // (cfk::launch_upload) on the engine's stream: see copy16 in als_kernels.hip.
    const size_t row_bytes = (size_t)e->kp * es;
    if (int r = ensure_stage(e)) return r;
    HIP_TRY(hipStreamSynchronize(e->stream));   // the staging buffer may still feed an earlier copy
    const int64_t rows_per = (int64_t)(e->stage_bytes / row_bytes);
    for (int64_t r = 0; r < n_rows; r += rows_per) {
        const int64_t nr = std::min(rows_per, n_rows - r);
        char* stage = (char*)e->h_stage;
        const char* src = (const char*)host_src + (size_t)r * src_ld * es;
        for (int64_t i = 0; i < nr; ++i) {
            std::memcpy(stage + i * row_bytes, src + (size_t)i * src_ld * es, (size_t)e->k * es);
            std::memset(stage + i * row_bytes + (size_t)e->k * es, 0, row_bytes - (size_t)e->k * es);
        }
        HIP_TRY(cfk::launch_upload(stage, (char*)f.ptr + (size_t)(row0 + r) * row_bytes, (size_t)nr * row_bytes,
                                   e->stream));
        HIP_TRY(hipStreamSynchronize(e->stream));   // the staging buffer is reused by the next chunk
    }
    return ALS_OK;
}

int als_read_factors(als_engine* e, int side, int64_t row0, int64_t n_rows, void* host_dst, int64_t dst_ld) {
    if (int r = check_engine(e)) return r;
    if (int r = check_side(side)) return r;
    const Factors& f = e->fac[side];
    if (!f.ptr) return fail(ALS_ERR_STATE, "factors of side %d not allocated/bound", side);
    if (row0 < 0 || n_rows < 0 || row0 + n_rows > f.n_rows) return fail(ALS_ERR_INVALID_ARGUMENT, "row range out of bounds");
    if (dst_ld < e->k) return fail(ALS_ERR_INVALID_ARGUMENT, "dst_ld (%lld) < num_features (%d)", (long long)dst_ld, e->k);
    if (n_rows == 0) return ALS_OK;
    if (!host_dst) return fail(ALS_ERR_INVALID_ARGUMENT, "host_dst is NULL");
    HIP_TRY(hipSetDevice(e->device));
    if (int r = sync_checked(e)) return r;
    const size_t es = e->elem();
    // Read back the way the kernels wrote: a copy kernel (cfk::launch_download) moves whole kp-wide rows into
    // pinned staging, the host keeps the first k columns; the same path as als_write_factors in reverse.
    const size_t row_bytes = (size_t)e->kp * es;
    if (int r = ensure_stage(e)) return r;
    const int64_t rows_per = (int64_t)(e->stage_bytes / row_bytes);
    for (int64_t r = 0; r < n_rows; r += rows_per) {
        const int64_t nr = std::min(rows_per, n_rows - r);
        HIP_TRY(cfk::launch_download((const char*)f.ptr + (size_t)(row0 + r) * row_bytes, e->h_stage,
                                     (size_t)nr * row_bytes, e->stream));
        HIP_TRY(hipStreamSynchronize(e->stream));
        const char* stage = (const char*)e->h_stage;
        char* dst = (char*)host_dst + (size_t)r * dst_ld * es;
        for (int64_t i = 0; i < nr; ++i)
            std::memcpy(dst + (size_t)i * dst_ld * es, stage + i * row_bytes, (size_t)e->k * es);
    }
    return ALS_OK;
}

namespace {

// One half (or one chunk of it): the FULL + PARTIAL launch, then the REDUCE launch.
struct DualLaunch {
    const Task* t[3] = {nullptr, nullptr, nullptr};
    int32_t n[3] = {0, 0, 0};
};

int launch_half(als_engine* e, int side, float lambda, const Task* tasks, int32_t n_tasks, const Task* reduce,
                int32_t n_reduce, bool first_chunk, const DualLaunch& dl) {
    Block& b = e->blk[side];
    const Factors& self = e->fac[side];
    const Factors& opp = e->fac[1 - side];
    if (!self.ptr || !opp.ptr) return fail(ALS_ERR_STATE, "als_solve_half: factor matrices not allocated/bound");
    if (b.n_rows > 0 && b.factor_row(b.n_rows - 1) >= self.n_rows)
        return fail(ALS_ERR_STATE, "block rows (last at factor row %lld) exceed factor rows %lld",
                    (long long)b.factor_row(b.n_rows - 1), (long long)self.n_rows);
    if (b.n_opp_rows != opp.n_rows)   // the padding entries gather row n_opp_rows: it must be the sentinel
        return fail(ALS_ERR_STATE, "block was set for %lld opposite rows, the opposite factor matrix has %lld",
                    (long long)b.n_opp_rows, (long long)opp.n_rows);
    if (!(lambda >= 0.f)) return fail(ALS_ERR_INVALID_ARGUMENT, "lambda must be >= 0");
    HIP_TRY(hipSetDevice(e->device));
    // the solve reads the opposite replica: wait for its all-gather; a whole half / first chunk also rewrites
    // this side's rows, which an earlier all-gather of this side may still be sending
    if (int r = wait_gathers(e, side == ALS_SIDE_USER || first_chunk, side == ALS_SIDE_MOVIE || first_chunk)) return r;
    cfk::SolveArgs a{};
    a.tasks = tasks;
    a.n_tasks = n_tasks;
    a.k = e->k;
    a.col = b.d_col;
    a.rat = b.d_rat;
    a.opp = opp.ptr;
    a.out = self.ptr;
    a.row_offset = b.row_offset;
    a.rows_per_chunk = (int32_t)b.rows_per_chunk;
    a.chunk_stride = b.chunk_stride;
    a.partials = e->d_partials;
    a.scratch_slabs = e->generic_slabs;
    a.lambda = lambda;
    a.sentinel = (int32_t)b.n_opp_rows;
    a.flags = e->path == Path::VALU ? 0 : e->debug_flags;
    if (++e->gen == 0) e->gen = 1;
    a.gen = e->debug_fixed_gen ? 1u : e->gen;
    a.integrity = e->d_integrity;
    a.refine_min_pivot = e->refine_min_pivot;
    a.extra_lds = e->debug_extra_lds;
    TimingRec rec{side, {nullptr, nullptr, nullptr}};
    if (e->timing) {
        for (auto& ev : rec.ev) {
            if (!e->ev_pool.empty()) {
                ev = e->ev_pool.back();
                e->ev_pool.pop_back();
            } else {
                HIP_TRY(hipEventCreate(&ev));
            }
        }
        HIP_TRY(hipEventRecord(rec.ev[0], e->stream));
    }
    const bool any_dual = dl.n[0] > 0 || dl.n[1] > 0 || dl.n[2] > 0;
    const bool side_dual = any_dual && e->dual_side;
    if (side_dual) {   // the dual launches read the fp32 opposite table only: fork before the pre-split
        if (!e->side_stream) {
            HIP_TRY(hipStreamCreateWithFlags(&e->side_stream, hipStreamNonBlocking));
            HIP_TRY(hipEventCreateWithFlags(&e->fork, hipEventDisableTiming));
            HIP_TRY(hipEventCreateWithFlags(&e->join, hipEventDisableTiming));
        }
        HIP_TRY(hipEventRecord(e->fork, e->stream));
    }
    if (b.presplit) {
        // the opposite replica is the half's input and does not change between its chunks (als.h): chunk 0
        // converts it, later chunks reuse the conversion
        if (first_chunk) {
            const int64_t n_floats = (b.n_opp_rows + 1) * (int64_t)e->kp;
            HIP_TRY(cfk::launch_absmax((const float*)opp.ptr, n_floats, e->kp, e->d_amax, e->stream));
            HIP_TRY(cfk::launch_presplit(e->kp, (const float*)opp.ptr, e->d_split, b.n_opp_rows + 1, e->d_amax,
                                         e->stream));
        }
        a.opp_split = e->d_split;
        a.rat_pk = b.d_rat_pk;
        a.rat_lo_off = b.nnz_padded / 2;
        a.col_ps = b.d_col_ps;
        a.amax = e->d_amax;
    }
    HIP_TRY(cfk::launch_solve(e->precision, e->kp, e->path, a, e->stream, b.presplit, false));
    if (b.presplit) {
        // the range guard's fallback: the same tasks on the fp32 table with the on-the-fly split, a launch whose
        // waves exit at once unless the opposite table is out of the pre-split's range (cfk::presplit_ok)
        cfk::SolveArgs f = a;
        f.presplit_fallback = 1;
        f.grid_cap = 4 * e->cu_count;
        HIP_TRY(cfk::launch_solve(e->precision, e->kp, e->path, f, e->stream, false, false));
    }
    if (side_dual) HIP_TRY(hipStreamWaitEvent(e->side_stream, e->fork, 0));
    for (int c = 0; c < 3; ++c)
        if (dl.n[c] > 0) {
            cfk::SolveArgs d = a;
            d.tasks = dl.t[c];
            d.n_tasks = dl.n[c];
            HIP_TRY(cfk::launch_dual(e->kp, 2 * (c + 1), d, side_dual ? e->side_stream : e->stream));
        }
    if (side_dual) {
        HIP_TRY(hipEventRecord(e->join, e->side_stream));
        HIP_TRY(hipStreamWaitEvent(e->stream, e->join, 0));
    }
    if (e->timing) HIP_TRY(hipEventRecord(rec.ev[1], e->stream));
    if (n_reduce > 0) {
        a.tasks = reduce;
        a.n_tasks = n_reduce;
        a.gen += e->debug_gen_skew;
        HIP_TRY(cfk::launch_solve(e->precision, e->kp, e->path, a, e->stream, false, true));
    }
    if (e->timing) {
        HIP_TRY(hipEventRecord(rec.ev[2], e->stream));
        e->pending.push_back(rec);
    }
    return ALS_OK;
}

}  // namespace

int als_solve_half(als_engine* e, int side, float lambda) {
    if (int r = check_engine(e)) return r;
    if (int r = check_side(side)) return r;
    Block& b = e->blk[side];
    if (!b.set) return fail(ALS_ERR_STATE, "als_solve_half: no block set for side %d", side);
    DualLaunch dl;
    for (int c = 0; c < 3; ++c) {
        dl.t[c] = b.d_dual[c];
        dl.n[c] = b.n_dual[c];
    }
    return launch_half(e, side, lambda, b.d_tasks, b.n_tasks, b.d_reduce, b.n_reduce, true, dl);
}

int als_set_chunks(als_engine* e, int side, int n_chunks, const int64_t* row_bounds) {
    if (int r = check_engine(e)) return r;
    if (int r = check_side(side)) return r;
    Block& b = e->blk[side];
    if (!b.set) return fail(ALS_ERR_STATE, "als_set_chunks: no block set for side %d", side);
    if (n_chunks < 1 || !row_bounds) return fail(ALS_ERR_INVALID_ARGUMENT, "n_chunks must be >= 1 with row_bounds");
    if (row_bounds[0] != 0 || row_bounds[n_chunks] != b.n_rows)
        return fail(ALS_ERR_INVALID_ARGUMENT, "row_bounds must run from 0 to n_rows (%lld)", (long long)b.n_rows);
    for (int c = 0; c < n_chunks; ++c)
        if (row_bounds[c + 1] < row_bounds[c]) return fail(ALS_ERR_INVALID_ARGUMENT, "row_bounds not monotone");
    auto chunk_of = [&](int32_t row) {
        return (int)(std::upper_bound(row_bounds, row_bounds + n_chunks + 1, (int64_t)row) - row_bounds) - 1;
    };
    // stable partition by chunk keeps the longest-first order inside every chunk
    auto split = [&](const std::vector<Task>& in, std::vector<Task>& out, std::vector<int32_t>& off) {
        std::vector<std::vector<Task>> per(n_chunks);
        for (const Task& t : in) per[chunk_of(t.row)].push_back(t);
        off.assign(n_chunks + 1, 0);
        out.clear();
        for (int c = 0; c < n_chunks; ++c) {
            out.insert(out.end(), per[c].begin(), per[c].end());
            off[c + 1] = (int32_t)out.size();
        }
    };
    std::vector<Task> ct, cr, cdl[3];
    split(b.h_tasks, ct, b.coff);
    split(b.h_reduce, cr, b.croff);
    for (int c = 0; c < 3; ++c) split(b.h_dual[c], cdl[c], b.cdoff[c]);
    HIP_TRY(hipSetDevice(e->device));
    HIP_TRY(hipStreamSynchronize(e->stream));
    (void)hipFree(b.d_ctasks);
    (void)hipFree(b.d_creduce);
    b.d_ctasks = b.d_creduce = nullptr;
    if (!ct.empty()) {
        HIP_TRY(hipMalloc((void**)&b.d_ctasks, ct.size() * sizeof(Task)));
        HIP_TRY(hipMemcpy(b.d_ctasks, ct.data(), ct.size() * sizeof(Task), hipMemcpyHostToDevice));
    }
    if (!cr.empty()) {
        HIP_TRY(hipMalloc((void**)&b.d_creduce, cr.size() * sizeof(Task)));
        HIP_TRY(hipMemcpy(b.d_creduce, cr.data(), cr.size() * sizeof(Task), hipMemcpyHostToDevice));
    }
    for (int c = 0; c < 3; ++c) {
        (void)hipFree(b.d_cdual[c]);
        b.d_cdual[c] = nullptr;
        if (!cdl[c].empty()) {
            HIP_TRY(hipMalloc((void**)&b.d_cdual[c], cdl[c].size() * sizeof(Task)));
            HIP_TRY(hipMemcpy(b.d_cdual[c], cdl[c].data(), cdl[c].size() * sizeof(Task), hipMemcpyHostToDevice));
        }
    }
    return ALS_OK;
}

int als_solve_half_chunk(als_engine* e, int side, float lambda, int chunk) {
    if (int r = check_engine(e)) return r;
    if (int r = check_side(side)) return r;
    Block& b = e->blk[side];
    if (!b.set || b.coff.empty()) return fail(ALS_ERR_STATE, "als_solve_half_chunk: no chunks set for side %d", side);
    if (chunk < 0 || chunk + 1 >= (int)b.coff.size())
        return fail(ALS_ERR_INVALID_ARGUMENT, "chunk %d out of range (%d chunks)", chunk, (int)b.coff.size() - 1);
    DualLaunch dl;
    for (int c = 0; c < 3; ++c) {
        dl.t[c] = b.d_cdual[c] + b.cdoff[c][chunk];
        dl.n[c] = b.cdoff[c][chunk + 1] - b.cdoff[c][chunk];
    }
    return launch_half(e, side, lambda, b.d_ctasks + b.coff[chunk], b.coff[chunk + 1] - b.coff[chunk],
                       b.d_creduce + b.croff[chunk], b.croff[chunk + 1] - b.croff[chunk], chunk == 0, dl);
}

int als_predict(als_engine* e, const int64_t* user_rows, int64_t n_users, const int64_t* movie_rows,
                int64_t n_movies, float* host_out) {
    if (int r = check_engine(e)) return r;
    if (n_users < 0 || n_movies < 0) return fail(ALS_ERR_INVALID_ARGUMENT, "negative counts");
    if (n_users == 0 || n_movies == 0) return ALS_OK;
    if (!user_rows || !movie_rows || !host_out) return fail(ALS_ERR_INVALID_ARGUMENT, "NULL pointer");
    const Factors& U = e->fac[ALS_SIDE_USER];
    const Factors& M = e->fac[ALS_SIDE_MOVIE];
    if (!U.ptr || !M.ptr) return fail(ALS_ERR_STATE, "als_predict: factor matrices not allocated/bound");
    for (int64_t i = 0; i < n_users; ++i)
        if (user_rows[i] < 0 || user_rows[i] >= U.n_rows) return fail(ALS_ERR_INVALID_ARGUMENT, "user row out of range");
    for (int64_t i = 0; i < n_movies; ++i)
        if (movie_rows[i] < 0 || movie_rows[i] >= M.n_rows) return fail(ALS_ERR_INVALID_ARGUMENT, "movie row out of range");
    if ((n_users + 15) / 16 > 65535) return fail(ALS_ERR_UNSUPPORTED, "at most 1,048,560 users per call (call per user range)");
    HIP_TRY(hipSetDevice(e->device));
    if (int r = wait_gathers(e, true, true)) return r;
    int64_t *d_u = nullptr, *d_m = nullptr;
    float* d_out = nullptr;
    const size_t ob = (size_t)n_users * (size_t)n_movies * sizeof(float);
    auto cleanup = [&]() {
        (void)hipFree(d_u);
        (void)hipFree(d_m);
        (void)hipFree(d_out);
    };
    hipError_t st = hipMalloc((void**)&d_u, n_users * sizeof(int64_t));
    if (st == hipSuccess) st = hipMalloc((void**)&d_m, n_movies * sizeof(int64_t));
    if (st == hipSuccess) st = hipMalloc((void**)&d_out, ob);
    if (st != hipSuccess) {
        cleanup();
        return fail(ALS_ERR_OUT_OF_MEMORY, "als_predict: hipMalloc: %s", hipGetErrorString(st));
    }
    st = hipMemcpyAsync(d_u, user_rows, n_users * sizeof(int64_t), hipMemcpyHostToDevice, e->stream);
    if (st == hipSuccess) st = hipMemcpyAsync(d_m, movie_rows, n_movies * sizeof(int64_t), hipMemcpyHostToDevice, e->stream);
    if (st == hipSuccess)
        st = cfk::launch_predict(e->precision, U.ptr, M.ptr, e->kp, e->k, d_u, n_users, d_m, n_movies, d_out, e->stream);
    if (st == hipSuccess) st = hipMemcpyAsync(host_out, d_out, ob, hipMemcpyDeviceToHost, e->stream);
    if (st == hipSuccess) st = hipStreamSynchronize(e->stream);
    cleanup();
    if (st != hipSuccess) return fail(ALS_ERR_DEVICE, "als_predict: %s", hipGetErrorString(st));
    return sync_checked(e);
}

int als_sq_error(als_engine* e, int side, double* sum_sq_error, int64_t* count) {
    if (int r = check_engine(e)) return r;
    if (int r = check_side(side)) return r;
    Block& b = e->blk[side];
    if (!b.set) return fail(ALS_ERR_STATE, "als_sq_error: no block set for side %d", side);
    const Factors& self = e->fac[side];
    const Factors& opp = e->fac[1 - side];
    if (!self.ptr || !opp.ptr) return fail(ALS_ERR_STATE, "als_sq_error: factor matrices not allocated/bound");
    HIP_TRY(hipSetDevice(e->device));
    if (int r = wait_gathers(e, true, true)) return r;
    cfk::SqErrArgs a{};
    a.tasks = b.d_sq_tasks;
    a.n_tasks = b.n_sq;
    a.col = b.d_col;
    a.rat = b.d_rat;
    a.opp = opp.ptr;
    a.self = self.ptr;
    a.row_offset = b.row_offset;
    a.rows_per_chunk = (int32_t)b.rows_per_chunk;
    a.chunk_stride = b.chunk_stride;
    a.task_se = b.d_task_se;
    a.sentinel = (int32_t)b.n_opp_rows;
    HIP_TRY(cfk::launch_sq_error(e->precision, e->kp, a, e->stream));
    std::vector<double> se(b.n_sq);
    if (b.n_sq > 0)
        HIP_TRY(hipMemcpyAsync(se.data(), b.d_task_se, se.size() * sizeof(double), hipMemcpyDeviceToHost, e->stream));
    if (int r = sync_checked(e)) return r;
    double s = 0.0;
    for (double v : se) s += v;   // fixed (task) order: deterministic
    if (sum_sq_error) *sum_sq_error = s;
    if (count) *count = b.nnz;
    return ALS_OK;
}

int als_synchronize(als_engine* e) {
    if (int r = check_engine(e)) return r;
    HIP_TRY(hipSetDevice(e->device));
    return sync_checked(e);
}

int als_integrity_status(als_engine* e, uint32_t* record, int reset) {
    if (int r = check_engine(e)) return r;
    HIP_TRY(hipSetDevice(e->device));
    if (int r = wait_gathers(e, true, true)) return r;
    if (int r = stream_wait(e, e->stream)) return r;
    uint32_t rec[cfk::INTEGRITY_WORDS];
    HIP_TRY(hipMemcpy(rec, e->d_integrity, sizeof(rec), hipMemcpyDeviceToHost));
    if (record) std::memcpy(record, rec, sizeof(rec));
    if (reset) HIP_TRY(hipMemset(e->d_integrity, 0, sizeof(rec)));
    return ALS_OK;
}

int als_set_timing(als_engine* e, int enabled) {
    if (int r = check_engine(e)) return r;
    e->timing = enabled != 0;
    return ALS_OK;
}

int als_timing_collect(als_engine* e, int side, double* ms_gram, double* ms_reduce, int64_t* n_calls) {
    if (int r = check_engine(e)) return r;
    if (int r = check_side(side)) return r;
    HIP_TRY(hipSetDevice(e->device));
    double g = 0, rd = 0;
    int64_t n = 0;
    std::vector<TimingRec> keep;
    for (auto& rec : e->pending) {
        if (rec.side != side) {
            keep.push_back(rec);
            continue;
        }
        HIP_TRY(hipEventSynchronize(rec.ev[2]));
        float m1 = 0, m2 = 0;
        HIP_TRY(hipEventElapsedTime(&m1, rec.ev[0], rec.ev[1]));
        HIP_TRY(hipEventElapsedTime(&m2, rec.ev[1], rec.ev[2]));
        g += m1;
        rd += m2;
        ++n;
        for (auto ev : rec.ev) e->ev_pool.push_back(ev);
    }
    e->pending.swap(keep);
    if (ms_gram) *ms_gram = g;
    if (ms_reduce) *ms_reduce = rd;
    if (n_calls) *n_calls = n;
    return ALS_OK;
}

int als_debug_copy_partials(als_engine* e, void* host_dst, int64_t max_bytes, int64_t* bytes) {
    if (int r = check_engine(e)) return r;
    HIP_TRY(hipSetDevice(e->device));
    HIP_TRY(hipStreamSynchronize(e->stream));
    const int64_t n = std::min<int64_t>(max_bytes, (int64_t)e->partial_bytes);
    if (bytes) *bytes = (int64_t)e->partial_bytes;
    if (host_dst && n > 0) HIP_TRY(hipMemcpy(host_dst, e->d_partials, (size_t)n, hipMemcpyDeviceToHost));
    return ALS_OK;
}

// ---- multi-GPU exchange (RCCL over xGMI) ---------------------------------------------------------------
#define NCCL_TRY(expr)                                                                                     \
    do {                                                                                                   \
        ncclResult_t _r = (expr);                                                                          \
        if (_r != ncclSuccess)                                                                             \
            return fail(ALS_ERR_COMM, "%s failed: %s (%s:%d)", #expr, ncclGetErrorString(_r), __FILE__,     \
                        __LINE__);                                                                         \
    } while (0)

static int comm_streams(als_engine* e) {
    HIP_TRY(hipSetDevice(e->device));
    HIP_TRY(hipStreamCreateWithFlags(&e->comm_stream, hipStreamNonBlocking));
    HIP_TRY(hipEventCreateWithFlags(&e->solved, hipEventDisableTiming));
    for (auto& ev : e->gathered) HIP_TRY(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
    return ALS_OK;
}

// Caller-level RCCL groups (als_comm_group_start / _end, one host thread driving several engines): inside a
// group a collective is only placed on its stream at the OUTERMOST ncclGroupEnd, so the "gathered" event of an
// all-gather issued inside a group must be recorded after that end, not at the call (recorded earlier it would
// order nothing). The thread's open-group depth and the (engine, side) pairs whose record is deferred:
thread_local int g_group_depth = 0;
thread_local std::vector<std::pair<als_engine*, int>> g_group_gathers;

static int record_gathered(als_engine* e, int side) {
    HIP_TRY(hipSetDevice(e->device));
    HIP_TRY(hipEventRecord(e->gathered[side], e->comm_stream));
    e->gather_pending[side] = true;
    return ALS_OK;
}

int als_comm_unique_id(void* id_out, int nbytes) {
    if (!id_out || nbytes < (int)sizeof(ncclUniqueId))
        return fail(ALS_ERR_INVALID_ARGUMENT, "unique id buffer must hold %d bytes", (int)sizeof(ncclUniqueId));
    ncclUniqueId id;
    NCCL_TRY(ncclGetUniqueId(&id));
    std::memcpy(id_out, &id, sizeof(id));
    return ALS_OK;
}

int als_comm_init(als_engine* e, int world, int rank, const void* unique_id) {
    if (int r = check_engine(e)) return r;
    if (world < 1 || rank < 0 || rank >= world || !unique_id)
        return fail(ALS_ERR_INVALID_ARGUMENT, "bad world/rank/unique_id (world %d, rank %d)", world, rank);
    if (e->comm) return fail(ALS_ERR_STATE, "engine already has a communicator");
    HIP_TRY(hipSetDevice(e->device));
    ncclUniqueId id;
    std::memcpy(&id, unique_id, sizeof(id));
    NCCL_TRY(ncclCommInitRank(&e->comm, world, id, rank));
    e->world = world;
    e->rank = rank;
    return comm_streams(e);
}

int als_comm_init_group(als_engine** engines, int n) {
    if (!engines || n < 1) return fail(ALS_ERR_INVALID_ARGUMENT, "need >= 1 engines");
    std::vector<int> devs(n);
    for (int i = 0; i < n; ++i) {
        if (int r = check_engine(engines[i])) return r;
        if (engines[i]->comm) return fail(ALS_ERR_STATE, "engine %d already has a communicator", i);
        devs[i] = engines[i]->device;
        for (int j = 0; j < i; ++j)
            if (devs[j] == devs[i]) return fail(ALS_ERR_INVALID_ARGUMENT, "engines %d and %d share device %d", j, i, devs[i]);
    }
    std::vector<ncclComm_t> comms(n);
    NCCL_TRY(ncclCommInitAll(comms.data(), n, devs.data()));
    for (int i = 0; i < n; ++i) {
        engines[i]->comm = comms[i];
        engines[i]->world = n;
        engines[i]->rank = i;
        if (int r = comm_streams(engines[i])) return r;
    }
    return ALS_OK;
}

int als_comm_info(const als_engine* e, int* world, int* rank) {
    if (int r = check_engine(e)) return r;
    if (world) *world = e->world;
    if (rank) *rank = e->rank;
    return ALS_OK;
}

int als_comm_group_start(void) {
    NCCL_TRY(ncclGroupStart());
    ++g_group_depth;
    return ALS_OK;
}

int als_comm_group_end(void) {
    if (g_group_depth <= 0) return fail(ALS_ERR_STATE, "als_comm_group_end without als_comm_group_start");
    const ncclResult_t r = ncclGroupEnd();
    if (--g_group_depth > 0) {
        if (r != ncclSuccess) return fail(ALS_ERR_COMM, "ncclGroupEnd failed: %s", ncclGetErrorString(r));
        return ALS_OK;
    }
    // outermost end: the grouped all-gathers are on their streams now; record their events behind them
    std::vector<std::pair<als_engine*, int>> touched;
    touched.swap(g_group_gathers);
    if (r != ncclSuccess) return fail(ALS_ERR_COMM, "ncclGroupEnd failed: %s", ncclGetErrorString(r));
    for (auto& eg : touched)
        if (int rc = record_gathered(eg.first, eg.second)) return rc;
    return ALS_OK;
}

int als_allgather_shard(als_engine* e, int side, int64_t slots_per_chunk, int64_t chunk) {
    if (int r = check_engine(e)) return r;
    if (int r = check_side(side)) return r;
    if (e->world == 1 && !e->comm) return ALS_OK;   // one shard: the replica is the matrix
    if (!e->comm) return fail(ALS_ERR_STATE, "als_allgather_shard: no communicator (als_comm_init)");
    const Factors& f = e->fac[side];
    if (!f.ptr) return fail(ALS_ERR_STATE, "factors of side %d not allocated/bound", side);
    const int64_t Sc = slots_per_chunk;
    if (Sc < 0 || chunk < 0 || (chunk + 1) * Sc * e->world > f.n_rows)
        return fail(ALS_ERR_INVALID_ARGUMENT, "chunk %lld of %lld slots per shard x %d shards exceeds %lld rows",
                    (long long)chunk, (long long)Sc, e->world, (long long)f.n_rows);
    if (Sc == 0) return ALS_OK;
    HIP_TRY(hipSetDevice(e->device));
    // after this engine's solve (stream) on comm_stream; the next solve that reads this side waits for it
    HIP_TRY(hipEventRecord(e->solved, e->stream));
    HIP_TRY(hipStreamWaitEvent(e->comm_stream, e->solved, 0));
    const ncclDataType_t dt = e->precision == ALS_F64 ? ncclFloat64 : ncclFloat32;
    const size_t row = (size_t)e->kp * e->elem();
    // chunk-major slots: chunk c holds the G shards' Sc-row pieces back to back, so its exchange is ONE
    // contiguous in-place all-gather
    char* cbase = (char*)f.ptr + (size_t)chunk * (size_t)(Sc * e->world) * row;
    e->last_gather_side = side;
    e->last_gather_chunk = chunk;
    e->last_gather_rows = Sc;
    NCCL_TRY(ncclAllGather(cbase + (size_t)e->rank * Sc * row, cbase, (size_t)Sc * e->kp, dt, e->comm,
                           e->comm_stream));
    if (g_group_depth > 0) {   // placed on the stream at the outermost group end: record the event there
        g_group_gathers.emplace_back(e, side);
        return ALS_OK;
    }
    return record_gathered(e, side);
}

int als_set_row_layout(als_engine* e, int side, int64_t rows_per_chunk, int64_t chunk_stride) {
    if (int r = check_engine(e)) return r;
    if (int r = check_side(side)) return r;
    Block& b = e->blk[side];
    if (!b.set) return fail(ALS_ERR_STATE, "als_set_row_layout: no block set for side %d", side);
    if (rows_per_chunk < 0 || (rows_per_chunk > 0 && chunk_stride < rows_per_chunk) || rows_per_chunk > INT32_MAX)
        return fail(ALS_ERR_INVALID_ARGUMENT, "rows_per_chunk %lld / chunk_stride %lld", (long long)rows_per_chunk,
                    (long long)chunk_stride);
    b.rows_per_chunk = rows_per_chunk;
    b.chunk_stride = rows_per_chunk > 0 ? chunk_stride : 0;
    return ALS_OK;
}

int als_comm_wait(als_engine* e) {
    if (int r = check_engine(e)) return r;
    HIP_TRY(hipSetDevice(e->device));
    return wait_gathers(e, true, true);
}

int als_comm_set_timeout(als_engine* e, int64_t timeout_ms) {
    if (int r = check_engine(e)) return r;
    e->comm_timeout_ms = timeout_ms;
    return ALS_OK;
}

int als_block_path(const als_engine* e, int side, int* gram_path, int* presplit, int64_t* chunk, int64_t* n_dual_rows) {
    if (int r = check_engine(e)) return r;
    if (int r = check_side(side)) return r;
    const Block& b = e->blk[side];
    if (gram_path) *gram_path = (int)e->path;
    if (presplit) *presplit = b.presplit ? 1 : 0;
    if (chunk) *chunk = b.set ? chunk_entries(b.nnz_padded) : 0;
    if (n_dual_rows)
        for (int c = 0; c < 3; ++c) n_dual_rows[c] = b.n_dual[c];
    return ALS_OK;
}

int als_block_stats(const als_engine* e, int side, int64_t* n_tasks, int64_t* n_reduce, int64_t* nnz_padded) {
    if (int r = check_engine(e)) return r;
    if (int r = check_side(side)) return r;
    const Block& b = e->blk[side];
    if (n_tasks) *n_tasks = b.n_tasks + b.n_dual[0] + b.n_dual[1] + b.n_dual[2];
    if (n_reduce) *n_reduce = b.n_reduce;
    if (nnz_padded) *nnz_padded = b.nnz_padded;
    return ALS_OK;
}

int als_block_split_info(const als_engine* e, int side, int64_t info[4]) {
    if (int r = check_engine(e)) return r;
    if (int r = check_side(side)) return r;
    if (!info) return fail(ALS_ERR_INVALID_ARGUMENT, "info is NULL");
    const Block& b = e->blk[side];
    info[0] = b.ilv_rows;
    info[1] = b.ilv_tasks;
    info[2] = b.ilv_chunk;
    info[3] = b.presplit ? 1 : 0;
    return ALS_OK;
}

}  // extern "C"

#ifdef CFK_DEBUG_KNOBS
// Debug build only (not in include/als.h): present iff the work-dropping / fault-injection knobs are compiled in
// (bench.py refuses a library that exports it, whatever its path).
extern "C" int als_debug_knobs_compiled(void) { return 1; }
#endif
