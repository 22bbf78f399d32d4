// Gather microbenchmark (diagnostics, not part of the library): random 256-B rows of a factor-table-sized buffer
// gathered in 32-row blocks (one block = 8 KB = the pre-split KP = 64 Gram's per-block image) by every wave of a
// full grid, three ways:
//   0  LDS-DMA: 8 global_load_lds_dwordx4 per block (1 KB each), s_waitcnt vmcnt(0), then 8 ds_read_b128
//   1  register gather + LDS: 8 global_load_dwordx4 per lane, then 8 ds_write_b128 and 8 ds_read_b128
//   2  register gather only: 8 global_load_dwordx4 per lane, XOR-folded into one register
//   4  LDS-DMA with the rows hashed from (wave, block, lane) instead of loaded: no index loads (8 instead of 10
//      vector-memory instructions per block), uniform rows
//   3  LDS-DMA with the rows below HOT left out of the DMA (exec-masked lanes: rows an LDS-resident hot-row cache
//      would serve), the reads as mode 0
// over uniform rows and over the Netflix-shape movie popularity (rank + 321)^-1.85 (ids = popularity ranks, so
// "row < HOT" is the HOT most popular rows).
// one block in flight per wave (DEPTH 1; the index loads of a block follow the previous block's wait, so a deeper
// pipeline would need its own counted waits). Prints GB/s for each mode and table size.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/gather_bench.hip -o build/gather_bench
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>
#include <random>
#include <cmath>
#include <algorithm>

#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); return 1; } } while (0)

typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
typedef int i32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) void lds_void;

constexpr int ROW = 256, BLK_ROWS = 32, WAVES = 4;
constexpr int IMG = BLK_ROWS * ROW;   // 8 KB per block

// idx layout: [block][g = lane >> 4][m = 0..7] = row of entry 4 m + g of the block
template <int MODE, int DEPTH>
__global__ __launch_bounds__(64 * WAVES) void gather(const char* __restrict__ table, const int* __restrict__ idx,
                                                     int nblk_per_wave, unsigned* __restrict__ sink, int hot) {
    __shared__ __attribute__((aligned(1024))) char img[WAVES][DEPTH][IMG];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int gw = blockIdx.x * WAVES + wave;
    const int g = lane >> 4, c = lane & 15;
    const int* ip = idx + ((int64_t)gw * nblk_per_wave) * 32 + g * 8;
    unsigned acc = 0;
    auto load_rows = [&](int b, int (&rows)[8]) {
        if constexpr (MODE == 4) {
            for (int m = 0; m < 8; ++m) {
                uint32_t x = (uint32_t)(gw * 977 + b) * 0x9E3779B1u ^ (uint32_t)(g * 8 + m) * 0x85EBCA77u;
                x ^= x >> 15;
                x *= 0x2C1B3C6Du;
                x ^= x >> 12;
                rows[m] = (int)(x % (uint32_t)hot);   // mode 4: hot = the table's row count
            }
            return;
        }
        const i32x4 r0 = *(const i32x4*)(ip + (int64_t)b * 32);
        const i32x4 r1 = *(const i32x4*)(ip + (int64_t)b * 32 + 4);
        for (int m = 0; m < 4; ++m) { rows[m] = r0[m]; rows[4 + m] = r1[m]; }
    };
    if constexpr (MODE == 0 || MODE == 3 || MODE == 4) {
        auto issue = [&](int b, char* im) {
            int rows[8];
            load_rows(b, rows);
#pragma unroll
            for (int m = 0; m < 8; ++m)
                if (MODE != 3 || rows[m] >= hot)
                    __builtin_amdgcn_global_load_lds((const void*)(table + (int64_t)rows[m] * ROW + c * 16),
                                                     (lds_void*)(im + m * 1024), 16, 0, 0);
        };
        issue(0, img[wave][0]);
        if (DEPTH > 1 && nblk_per_wave > 1) issue(1, img[wave][DEPTH - 1]);
        for (int b = 0; b < nblk_per_wave; ++b) {
            char* im = img[wave][b % DEPTH];
            if (DEPTH > 1 && b + 1 < nblk_per_wave) asm volatile("s_waitcnt vmcnt(10)" ::: "memory");
            else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            u32x4 v = {0, 0, 0, 0};
#pragma unroll
            for (int m = 0; m < 8; ++m) v ^= *(const u32x4*)(im + m * 1024 + lane * 16);
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            acc ^= v[0] ^ v[1] ^ v[2] ^ v[3];
            if (b + DEPTH < nblk_per_wave) issue(b + DEPTH, im);
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    } else {
        u32x4 d[DEPTH][8];
        auto issue = [&](int b, u32x4 (&dd)[8]) {
            int rows[8];
            load_rows(b, rows);
#pragma unroll
            for (int m = 0; m < 8; ++m) dd[m] = *(const u32x4*)(table + (int64_t)rows[m] * ROW + c * 16);
        };
        issue(0, d[0]);
        if (DEPTH > 1 && nblk_per_wave > 1) issue(1, d[DEPTH - 1]);
        for (int b = 0; b < nblk_per_wave; ++b) {
            u32x4 (&cur)[8] = d[b % DEPTH];
            u32x4 v = {0, 0, 0, 0};
            if constexpr (MODE == 1) {
                char* im = img[wave][0];
#pragma unroll
                for (int m = 0; m < 8; ++m) *(u32x4*)(im + m * 1024 + lane * 16) = cur[m];
#pragma unroll
                for (int m = 0; m < 8; ++m) v ^= *(const u32x4*)(im + m * 1024 + ((lane * 16 + 272) & 1023));
            } else {
#pragma unroll
                for (int m = 0; m < 8; ++m) v ^= cur[m];
            }
            acc ^= v[0] ^ v[1] ^ v[2] ^ v[3];
            if (b + DEPTH < nblk_per_wave) issue(b + DEPTH, cur);
        }
    }
    if (acc == 0x12345678u) sink[gw] = acc;   // keeps the loads live
}

template <int MODE, int DEPTH>
int run(const char* table, const int* idx, int grid, int nblk, unsigned* sink, const char* label, int64_t tbytes,
        int hot = 0) {
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    gather<MODE, DEPTH><<<grid, 64 * WAVES>>>(table, idx, nblk, sink, hot);
    CHECK(hipDeviceSynchronize());
    float best = 1e30f;
    for (int it = 0; it < 5; ++it) {
        CHECK(hipEventRecord(e0));
        gather<MODE, DEPTH><<<grid, 64 * WAVES>>>(table, idx, nblk, sink, hot);
        CHECK(hipEventRecord(e1));
        CHECK(hipEventSynchronize(e1));
        float ms;
        CHECK(hipEventElapsedTime(&ms, e0, e1));
        best = ms < best ? ms : best;
    }
    const double bytes = (double)grid * WAVES * nblk * IMG;
    printf("table %7.1f MB  %-28s hot %4d depth %d: %.3f ms  %.2f TB/s  %.1f GB/s per CU (block bytes incl. hot rows)\n",
           tbytes / 1e6, label, hot, DEPTH, best, bytes / best / 1e9, bytes / best / 1e6 / 256);
    return 0;
}

int main() {
    const int cus = 256, wg_per_cu = 4, grid = cus * wg_per_cu;   // 16 waves per CU
    const int nblk = 200;
    const int64_t nrows_idx = (int64_t)grid * WAVES * nblk * 32;
    int* d_idx;
    unsigned* d_sink;
    CHECK(hipMalloc(&d_idx, nrows_idx * 4));
    CHECK(hipMalloc(&d_sink, (size_t)grid * WAVES * 4));
    for (int64_t rows : {17771LL, 480190LL}) {
        const int64_t tbytes = rows * ROW;
        char* d_table;
        CHECK(hipMalloc(&d_table, tbytes));
        CHECK(hipMemset(d_table, 1, tbytes));
        std::vector<int> h(nrows_idx);
        std::mt19937 rng(7);
        std::uniform_int_distribution<int> dist(0, (int)rows - 1);
        for (auto& x : h) x = dist(rng);
        CHECK(hipMemcpy(d_idx, h.data(), nrows_idx * 4, hipMemcpyHostToDevice));
        if (run<0, 1>(d_table, d_idx, grid, nblk, d_sink, "LDS-DMA", tbytes)) return 1;
        if (run<1, 1>(d_table, d_idx, grid, nblk, d_sink, "register + ds_write", tbytes)) return 1;
        if (run<2, 1>(d_table, d_idx, grid, nblk, d_sink, "register only", tbytes)) return 1;
        if (run<4, 1>(d_table, d_idx, grid, nblk, d_sink, "LDS-DMA, no index loads", tbytes, (int)rows)) return 1;
        if (rows == 17771) {
            // Netflix-shape popularity: id = rank, P(rank) ~ (rank + 321)^-1.85 (inverse CDF of the continuous law)
            std::uniform_real_distribution<double> U(0.0, 1.0);
            const double a = 321.0, e = 0.85, top = std::pow(a, -e), bot = std::pow(a + rows, -e);
            for (auto& x : h) {
                const double r = std::pow(top - U(rng) * (top - bot), -1.0 / e) - a;
                x = std::min<int>((int)rows - 1, std::max(0, (int)r));
            }
            CHECK(hipMemcpy(d_idx, h.data(), nrows_idx * 4, hipMemcpyHostToDevice));
            for (int hot : {0, 64, 112, 240, 480}) {
                int64_t n = 0;
                for (auto x : h) n += x < hot;
                printf("zipf: rows < %d = %.3f of the gathers\n", hot, (double)n / (double)h.size());
                if (run<3, 1>(d_table, d_idx, grid, nblk, d_sink, "zipf LDS-DMA, hot rows skipped", tbytes, hot))
                    return 1;
            }
            if (run<2, 1>(d_table, d_idx, grid, nblk, d_sink, "zipf register only", tbytes)) return 1;
        }
        CHECK(hipFree(d_table));
    }
    printf("gather_bench done\n");
    return 0;
}
