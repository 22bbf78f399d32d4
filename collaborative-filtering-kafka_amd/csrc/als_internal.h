// Internal declarations shared by the engine (als_engine.cpp) and the kernels (als_kernels.hip).
#pragma once
#include <cstdint>
#include <string>
#include <vector>

#include <hip/hip_runtime.h>

namespace cfk {

// One wave-sized unit of work of a half-iteration (host-built once per uploaded block, README.md:146-147:
// the rating blocks never change, so the work plan is fixed for every iteration).
//   kind FULL    : gather rows [begin, begin + 4*nsteps) of the padded in-block, accumulate Gram + RHS,
//                  regularise, Cholesky-solve, store factor row `row`.
//   kind PARTIAL : same gather/accumulate over one chunk of a long row; store the raw per-lane
//                  accumulators into partial slot `slot` (no solve).
//   kind REDUCE  : sum partial slots [slot, slot + nsteps) of row `row` in fixed order, then solve + store.
enum TaskKind : int32_t { TASK_FULL = 0, TASK_PARTIAL = 1, TASK_REDUCE = 2 };

// Device in-block layout: each row is padded to whole blocks of BLOCK_ENTRIES = 32 entries; padding entries
// hold col = n_opp_rows (the sentinel zero row kept after the last factor row) and rating 0, so they add
// nothing and need no masking in the kernels. Entry e of a
// row is consumed by sub-step t = e / 4 (one MFMA K=4 step) in lane group g = e % 4; inside a block the
// entries are stored group-major ([g][t], t < 8) so that one lane fetches the column indices of its 8
// sub-steps with two 16-byte loads.
constexpr int BLOCK_SUBSTEPS = 8;
constexpr int BLOCK_ENTRIES = 4 * BLOCK_SUBSTEPS;
__host__ __device__ constexpr int64_t block_position(int64_t e) {
    const int64_t blk = e / BLOCK_ENTRIES, w = e % BLOCK_ENTRIES;
    return blk * BLOCK_ENTRIES + (w % 4) * BLOCK_SUBSTEPS + w / 4;
}

struct alignas(16) Task {
    int64_t begin;   // entry offset into the padded col/rating arrays (multiple of BLOCK_ENTRIES)
    int32_t nsteps;  // FULL/PARTIAL: sub-steps holding real entries (ceil(n/4)); the task spans
                     // ceil(nsteps / BLOCK_SUBSTEPS) blocks. REDUCE: number of partial slots
    int32_t row;     // local row of the block (factor row = row_offset + row)
    int32_t slot;    // PARTIAL: slot written; REDUCE: first slot read; FULL: -1
    int32_t ndeg;    // true in-block size n_j (lambda * n_j * I, MFeatureCalculator.java:92-95)
    int32_t kind;
    int32_t nent;    // FULL/PARTIAL: real entries in this task's range (logical indices [0, nent))
};
static_assert(sizeof(Task) == 32, "Task layout");

struct SolveArgs {
    const Task* tasks;
    int32_t n_tasks;
    int32_t k;              // true number of features (<= KP)
    const int32_t* col;     // padded in-block opposite indices (-1 = padding)
    const float* rat;       // padded ratings (0 = padding)
    const void* opp;        // opposite factor matrix [n_opp][KP]
    void* out;              // this side's factor matrix [n_total][KP]
    int64_t row_offset;     // first factor row of this block
    void* partials;         // partial-slot workspace
    float lambda;
    int32_t sentinel;       // index of the opposite side's all-zero sentinel row (= n_opp_rows)
    int32_t flags;          // SOLVE_FLAG_* (diagnostics only; 0 in production)
    const void* opp_split;  // MFMA_SPLIT + presplit: the opposite table as fp16 h/m planes (als_presplit)
    uint32_t gen;           // launch generation (PARTIAL and its REDUCE share it): keys the partial-slot encoding
    uint32_t* integrity;    // device record of partial slots that failed their check (see als_kernels.hip)
    float refine_min_pivot; // MFMA tile solve: skip the refinement step when every scaled pivot >= this (> 1: never)
    const uint32_t* rat_pk; // presplit: the padded ratings r = rh + rm as fp16 pairs (entries 2i, 2i+1): the rh pairs,
                            //   then (at rat_lo_off words) the rm pairs; both exact for every Java short
    const int32_t* col_ps;  // presplit: the padded column indices permuted per block for the LDS-DMA gather
                            //   (launch_pack_cols_ps: lane group r of a block loads its 4 rows with one 16-B load)
    int32_t rows_per_chunk; // chunk-major slots (als_set_row_layout): 0 = factor row row_offset + row, else
    int64_t chunk_stride;   //   row_offset + (row / rows_per_chunk) * chunk_stride + row % rows_per_chunk
    int64_t rat_lo_off;     // presplit: words from the rh pairs to the rm pairs (nnz_padded / 2)
    const uint32_t* amax;   // presplit: range statistics of the opposite table (als_absmax): [0] bits of its largest
                            //   |x| (the split scale), [1] ~bits of its smallest nonzero row maximum
    int32_t presplit_fallback;  // the on-the-fly split launch guarding a pre-split half: it runs only when the table
                                //   is out of the pre-split's range (presplit_ok(amax) false), else exits at once
    int64_t scratch_slabs;  // generic path: workgroup slabs in `partials` (its Gram when it does not fit in LDS)
    int32_t grid_cap;       // workgroups of a grid-stride launch (the range guard's fallback): CUs x 4
    int32_t extra_lds;      // diagnostics (debug build's ALS_DEBUG_EXTRA_LDS, else 0): unused dynamic LDS per workgroup
};
// Factor row of local row `row` under the block's slot layout (wave-uniform: scalar arithmetic, once per task).
__host__ __device__ inline int64_t factor_row(int64_t row_offset, int32_t rows_per_chunk, int64_t chunk_stride,
                                              int32_t row) {
    if (rows_per_chunk <= 0) return row_offset + row;
    const int32_t q = row / rows_per_chunk;
    return row_offset + (int64_t)q * chunk_stride + (row - q * rows_per_chunk);
}
// Partial-slot integrity record (device, 4 words): [0] REDUCE tasks that found a bad slot, [1] generation, [2] slot,
// [3] row of the first failure. Read back by every synchronising call of the engine.
constexpr int INTEGRITY_WORDS = 4;
// Diagnostic: skip the k x k solve after the Gram (stores the Gram diagonal instead) -- used by
// tools/kbench.py to split a launch's time into Gram and solve. Only the debug build (CFK_DEBUG_KNOBS) can set
// these flags; the product library never does.
constexpr int32_t SOLVE_FLAG_SKIP_SOLVE = 1;
constexpr int32_t SOLVE_FLAG_SKIP_REFINE = 2;   // diagnostic: no refinement step (accuracy experiments)

struct SqErrArgs {
    const Task* tasks;      // FULL + PARTIAL tasks (they cover every entry exactly once)
    int32_t n_tasks;
    const int32_t* col;
    const float* rat;
    const void* opp;
    const void* self;
    int64_t row_offset;
    double* task_se;        // [n_tasks]
    int32_t sentinel;
    int32_t rows_per_chunk; // slot layout as SolveArgs
    int64_t chunk_stride;
};

// Gram paths: VALU (LDS-staged, fp32 k < 32 and all fp64), MFMA (v_mfma_f32_16x16x4_f32, exact f32
// products), MFMA_SPLIT (fp32 operands split into narrow terms, fp32 accumulation: fp32-accurate products at a
// multiple of the f32 MFMA rate): on the fly into three bf16 terms (six v_mfma_f32_16x16x32_bf16 partial products
// per tile), or -- presplit -- once per half into a scaled two-term fp16 table (three v_mfma_f32_16x16x32_f16).
// GENERIC: any num_features beyond the wave-per-row kernels (fp32 k > 128, fp64 k > 64): one workgroup per row,
// the Gram's packed lower triangle in LDS (or a per-workgroup global slab) and a workgroup Cholesky.
enum class Path : int { VALU = 0, MFMA = 1, MFMA_SPLIT = 2, GENERIC = 3 };
// Launch geometry of the generic path for (precision, kp): LDS or slab Gram, staged rows per batch, dynamic LDS.
struct GenericPlan {
    bool g_in_lds;
    int batch;
    int64_t lds_bytes;
    int64_t slab_elems;   // elements per workgroup slab of SolveArgs::partials (0 when the Gram is in LDS)
};
GenericPlan generic_plan(int precision, int kp);
hipError_t launch_generic(int precision, int kp, const SolveArgs& a, hipStream_t s);

// Launch helpers (defined in als_kernels.hip). Return hipSuccess or the launch error.
// The variant (and its occupancy) follows from (precision, kp, path, presplit). presplit: the Gram reads the pre-split
// opposite table (a.opp_split). reduce: `a.tasks` are REDUCE tasks (launched after the FULL/PARTIAL launch of the
// same half).
hipError_t launch_solve(int precision, int kp, Path path, const SolveArgs& a, hipStream_t s, bool presplit,
                        bool reduce);
// Block permutation of the in-block (32-entry blocks): dst block i <- src block perm[i] (cols and ratings).
hipError_t launch_permute_blocks(const int32_t* col, const float* rat, int32_t* col_out, float* rat_out,
                                 const int32_t* perm, int64_t n_blocks, hipStream_t s);
// Short rows in entry space (als_solve_dual): fp32 split path, kp 64 with cd 2, kp 128 with cd 2 or 4 (rows of
// 16 * cd padded entries, i.e. cd / 2 blocks); `a.tasks` are FULL tasks of such rows.
hipError_t launch_dual(int kp, int cd, const SolveArgs& a, hipStream_t s);
// Pre-split of an fp32 [n_rows][kp] factor table (kp = 64 or 128, sentinel row included) into the two fp16 terms
// the presplit Gram stages in LDS: row r = presplit_row_bytes(kp) = 4 kp bytes (the fp32 row's size) at r * 4 kp =
// two planes (h, m) of 2 kp bytes, plane position 16 b + j (b = 0..kp/16-1, j = 0..15) holding feature (kp/16) j + b
// scaled by 2^s, so the 16 values one transposed LDS read hands to a 16-lane group (features (kp/16) j + b,
// j = 0..15) are 32 contiguous bytes. launch_absmax writes the table's range statistics to amax[0..1] first (zeroed
// here, on the stream); the presplit kernel and the Gram derive s from it (als_kernels.hip, split_exp).
__host__ __device__ constexpr int presplit_row_bytes(int kp) { return 4 * kp; }
hipError_t launch_absmax(const float* src, int64_t n_floats, int kp, uint32_t* amax /* 2 words */, hipStream_t s);
hipError_t launch_presplit(int kp, const float* src, void* dst, int64_t n_rows, const uint32_t* amax, hipStream_t s);
// padded column indices -> the per-block order of the presplit gather (n_entries = nnz_padded)
hipError_t launch_pack_cols_ps(const int32_t* col, int32_t* dst, int64_t n_entries, hipStream_t s);
// padded fp32 ratings r -> fp16 pairs of rh = f16(r) at dst[0, n_pairs) and of rm = r - rh at dst[n_pairs, 2 n_pairs)
// (n_pairs = nnz_padded / 2; exact for every integer |r| <= 2^22, so for every Java short)
hipError_t launch_pack_ratings(const float* rat, uint32_t* dst, int64_t n_pairs, hipStream_t s);
// bytes % 16 == 0; host_pinned must stay valid until the stream has passed the copy
hipError_t launch_upload(const void* host_pinned, void* dst, size_t bytes, hipStream_t s);
hipError_t launch_download(const void* src, void* host_pinned, size_t bytes, hipStream_t s);
// out[u][m] = Java-float dot of U row urows[u] and M row mrows[m] (device arrays; out row-major n_u x n_m).
hipError_t launch_predict(int precision, const void* U, const void* M, int kp, int k, const int64_t* urows,
                          int64_t n_u, const int64_t* mrows, int64_t n_m, float* out, hipStream_t s);
hipError_t launch_sq_error(int precision, int kp, const SqErrArgs& a, hipStream_t s);
// Per-lane accumulator words (elements of the engine precision) of one partial slot: nacc * 64.
int partial_words_per_lane(int precision, int kp, Path path);
// In-block build on the device (als_build.hip): host COO (local row, opposite slot, rating) in arrival order ->
// stable radix sort by row -> the padded block-interleaved d_col / d_rat of als_set_block, row degrees and
// padded row starts back on the host (for the work plan). Returns an als_status; on failure `err` says why and
// nothing is left allocated.
int build_block_device(const int32_t* rows, const int32_t* cols, const int16_t* ratings, int64_t nnz, int64_t n_rows,
                       int64_t n_opp_rows, hipStream_t s, std::vector<int64_t>& deg, std::vector<int64_t>& begin,
                       int32_t** d_col, float** d_rat, std::string& err);
// Host-side check that a (precision, kp, path) variant is compiled in.
bool variant_available(int precision, int kp, Path path);

}  // namespace cfk
