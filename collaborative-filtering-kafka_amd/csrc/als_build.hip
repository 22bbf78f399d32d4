// als_build.hip -- in-block (CSR) build on the GPU: the block-builder processors
// MRatings2BlocksProcessor.java:48-69 / URatings2BlocksProcessor.java:72-92 append each arriving rating to its
// entity's id and rating lists, i.e. an in-block row keeps ARRIVAL order. Here the ratings of a partition
// arrive as COO triples (local row, opposite slot, rating) and one stable radix sort by row on the device
// (hipCUB/rocPRIM onesweep; stable, so arrival order survives inside a row) replaces the per-entity list
// appends; a scatter kernel then writes the padded, block-interleaved layout the solve kernels read
// (cfk::block_position, sentinel padding), so the only host work left is the per-row work plan.
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include "als.h"
#include "als_internal.h"

namespace cfk {
namespace {

__global__ void validate_iota(const int32_t* __restrict__ rows, const int32_t* __restrict__ cols, int64_t nnz,
                              int64_t n_rows, int64_t n_opp, int32_t* __restrict__ idx, unsigned* __restrict__ bad) {
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= nnz) return;
    idx[t] = (int32_t)t;
    const int32_t r = rows[t], c = cols[t];
    if (r < 0 || r >= n_rows) atomicOr(bad, 1u);
    if (c < 0 || c >= n_opp) atomicOr(bad, 2u);
}

__global__ void row_degrees(const int32_t* __restrict__ rows_sorted, int64_t nnz, int32_t* __restrict__ deg) {
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= nnz) return;
    // the last entry of every run of equal (sorted) rows records the run's inclusive end
    const int32_t r = rows_sorted[t];
    if (t + 1 == nnz || rows_sorted[t + 1] != r) deg[r] = (int32_t)(t + 1);   // inclusive end
}

__global__ void fill_padding(int32_t* __restrict__ col, float* __restrict__ rat, int64_t n, int32_t sentinel) {
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= n) return;
    col[t] = sentinel;
    rat[t] = 0.f;
}

__global__ void scatter_block(const int32_t* __restrict__ rows_sorted, const int32_t* __restrict__ idx_sorted,
                              const int32_t* __restrict__ cols, const int16_t* __restrict__ ratings, int64_t nnz,
                              const int64_t* __restrict__ row_start, const int64_t* __restrict__ begin,
                              int32_t* __restrict__ col_out, float* __restrict__ rat_out) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= nnz) return;
    const int32_t r = rows_sorted[i];
    const int32_t src = idx_sorted[i];
    const int64_t pos = begin[r] + block_position(i - row_start[r]);
    col_out[pos] = cols[src];
    rat_out[pos] = (float)ratings[src];
}

unsigned grid_for(int64_t n) { return (unsigned)((n + 255) / 256); }

}  // namespace

int build_block_device(const int32_t* rows, const int32_t* cols, const int16_t* ratings, int64_t nnz, int64_t n_rows,
                       int64_t n_opp_rows, hipStream_t s, std::vector<int64_t>& deg, std::vector<int64_t>& begin,
                       int32_t** d_col_out, float** d_rat_out, std::string& err) {
    *d_col_out = nullptr;
    *d_rat_out = nullptr;
    deg.assign(n_rows, 0);
    begin.assign(n_rows + 1, 0);
    int32_t *d_rows = nullptr, *d_cols = nullptr, *d_idx = nullptr, *d_rows_s = nullptr, *d_idx_s = nullptr;
    int32_t *d_end = nullptr, *d_col = nullptr;
    int16_t* d_r16 = nullptr;
    float* d_rat = nullptr;
    int64_t *d_start = nullptr, *d_begin = nullptr;
    unsigned* d_bad = nullptr;
    void* d_tmp = nullptr;
    auto release = [&](bool keep_out) {
        for (void* p : {(void*)d_rows, (void*)d_cols, (void*)d_idx, (void*)d_rows_s, (void*)d_idx_s, (void*)d_end,
                        (void*)d_r16, (void*)d_start, (void*)d_begin, (void*)d_bad, d_tmp})
            (void)hipFree(p);
        if (!keep_out) {
            (void)hipFree(d_col);
            (void)hipFree(d_rat);
        }
    };
    hipError_t st = hipSuccess;
    auto ok = [&](hipError_t e, const char* what) {
        if (e != hipSuccess && st == hipSuccess) {
            st = e;
            err = std::string(what) + ": " + hipGetErrorString(e);
        }
        return st == hipSuccess;
    };
    const size_t n4 = (size_t)nnz * 4;
    if (nnz > 0) {
        if (!ok(hipMalloc((void**)&d_rows, n4), "hipMalloc") || !ok(hipMalloc((void**)&d_cols, n4), "hipMalloc") ||
            !ok(hipMalloc((void**)&d_r16, (size_t)nnz * 2), "hipMalloc") || !ok(hipMalloc((void**)&d_idx, n4), "hipMalloc") ||
            !ok(hipMalloc((void**)&d_rows_s, n4), "hipMalloc") || !ok(hipMalloc((void**)&d_idx_s, n4), "hipMalloc") ||
            !ok(hipMalloc((void**)&d_bad, sizeof(unsigned)), "hipMalloc")) {
            release(false);
            return ALS_ERR_OUT_OF_MEMORY;
        }
        ok(hipMemcpyAsync(d_rows, rows, n4, hipMemcpyHostToDevice, s), "upload");
        ok(hipMemcpyAsync(d_cols, cols, n4, hipMemcpyHostToDevice, s), "upload");
        ok(hipMemcpyAsync(d_r16, ratings, (size_t)nnz * 2, hipMemcpyHostToDevice, s), "upload");
        ok(hipMemsetAsync(d_bad, 0, sizeof(unsigned), s), "memset");
        if (st == hipSuccess) {
            validate_iota<<<grid_for(nnz), 256, 0, s>>>(d_rows, d_cols, nnz, n_rows, n_opp_rows, d_idx, d_bad);
            ok(hipGetLastError(), "validate");
        }
        unsigned bad = 0;
        ok(hipMemcpyAsync(&bad, d_bad, sizeof(unsigned), hipMemcpyDeviceToHost, s), "download");
        ok(hipStreamSynchronize(s), "sync");
        if (st != hipSuccess) {
            release(false);
            return ALS_ERR_DEVICE;
        }
        if (bad) {
            err = (bad & 1) ? "a row index is outside [0, n_rows)" : "a column index is outside [0, n_opp_rows)";
            release(false);
            return ALS_ERR_INVALID_ARGUMENT;
        }
        // stable LSD radix sort of (row, arrival index) over the bits the row count needs
        int end_bit = 1;
        while (end_bit < 31 && ((int64_t)1 << end_bit) < n_rows) ++end_bit;
        size_t tmp_bytes = 0;
        ok(hipcub::DeviceRadixSort::SortPairs(nullptr, tmp_bytes, d_rows, d_rows_s, d_idx, d_idx_s, (int)nnz, 0, end_bit, s),
           "radix sort sizing");
        if (st == hipSuccess && !ok(hipMalloc(&d_tmp, tmp_bytes), "hipMalloc")) {
            release(false);
            return ALS_ERR_OUT_OF_MEMORY;
        }
        ok(hipcub::DeviceRadixSort::SortPairs(d_tmp, tmp_bytes, d_rows, d_rows_s, d_idx, d_idx_s, (int)nnz, 0, end_bit, s),
           "radix sort");
        // inclusive end of every non-empty row's run -> degrees on the host
        std::vector<int32_t> ends(n_rows, -1);
        if (st == hipSuccess && n_rows > 0) {
            if (!ok(hipMalloc((void**)&d_end, (size_t)n_rows * 4), "hipMalloc")) {
                release(false);
                return ALS_ERR_OUT_OF_MEMORY;
            }
            ok(hipMemsetAsync(d_end, 0xff, (size_t)n_rows * 4, s), "memset");
            if (st == hipSuccess) {
                row_degrees<<<grid_for(nnz), 256, 0, s>>>(d_rows_s, nnz, d_end);
                ok(hipGetLastError(), "row_degrees");
            }
            ok(hipMemcpyAsync(ends.data(), d_end, (size_t)n_rows * 4, hipMemcpyDeviceToHost, s), "download");
            ok(hipStreamSynchronize(s), "sync");
        }
        if (st != hipSuccess) {
            release(false);
            return ALS_ERR_DEVICE;
        }
        // rows are dense in [0, n_rows): start of row r = end of the previous non-empty row
        int64_t prev_end = 0;
        for (int64_t r = 0; r < n_rows; ++r) {
            if (ends[r] >= 0) {
                deg[r] = (int64_t)ends[r] - prev_end;
                prev_end = ends[r];
            }
        }
    }
    std::vector<int64_t> start(n_rows + 1, 0);
    for (int64_t r = 0; r < n_rows; ++r) {
        if (deg[r] > INT32_MAX / 2) {
            err = "a row has more than 2^30 entries";
            release(false);
            return ALS_ERR_UNSUPPORTED;
        }
        start[r + 1] = start[r] + deg[r];
        begin[r + 1] = begin[r] + (deg[r] + BLOCK_ENTRIES - 1) / BLOCK_ENTRIES * BLOCK_ENTRIES;
    }
    const int64_t padded = begin[n_rows];
    if (padded > 0) {
        if (!ok(hipMalloc((void**)&d_col, (size_t)padded * 4), "hipMalloc") ||
            !ok(hipMalloc((void**)&d_rat, (size_t)padded * 4), "hipMalloc") ||
            !ok(hipMalloc((void**)&d_start, (size_t)(n_rows + 1) * 8), "hipMalloc") ||
            !ok(hipMalloc((void**)&d_begin, (size_t)(n_rows + 1) * 8), "hipMalloc")) {
            release(false);
            return ALS_ERR_OUT_OF_MEMORY;
        }
        ok(hipMemcpyAsync(d_start, start.data(), (size_t)(n_rows + 1) * 8, hipMemcpyHostToDevice, s), "upload");
        ok(hipMemcpyAsync(d_begin, begin.data(), (size_t)(n_rows + 1) * 8, hipMemcpyHostToDevice, s), "upload");
        if (st == hipSuccess) {
            fill_padding<<<grid_for(padded), 256, 0, s>>>(d_col, d_rat, padded, (int32_t)n_opp_rows);
            ok(hipGetLastError(), "fill");
        }
        if (st == hipSuccess && nnz > 0) {
            scatter_block<<<grid_for(nnz), 256, 0, s>>>(d_rows_s, d_idx_s, d_cols, d_r16, nnz, d_start, d_begin, d_col,
                                                        d_rat);
            ok(hipGetLastError(), "scatter");
        }
        ok(hipStreamSynchronize(s), "sync");
    }
    if (st != hipSuccess) {
        release(false);
        return ALS_ERR_DEVICE;
    }
    release(true);
    *d_col_out = d_col;
    *d_rat_out = d_rat;
    return ALS_OK;
}

}  // namespace cfk
