// xcd_coherence.hip -- does a kernel see rows that ANOTHER XCD wrote in the previous kernel on the same stream,
// when its own XCD's L2 still holds an older copy of those rows?
//
// Per round g (all on one stream):
//   R(g): every workgroup on XCD x reads rows r with r % 8 == x (its L2 now holds them, value g-1)
//   W(g): every workgroup on XCD x writes rows r with r % 8 == (x + 1) % 8 (value g): rows of residue j are
//         written by XCD j-1, never by the XCD that reads them
//   C(g): every workgroup on XCD x re-reads rows r % 8 == x and counts entries != g
// A kernel boundary that leaves a reader's L2 copy in place shows up as a non-zero count.
//   hipcc --offload-arch=gfx950 -O3 tools/xcd_coherence.hip -o tools/xcd_coherence && tools/xcd_coherence [rounds]
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CHECK(x)                                                                             \
    do {                                                                                     \
        hipError_t e_ = (x);                                                                 \
        if (e_ != hipSuccess) {                                                              \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                          \
            return 1;                                                                        \
        }                                                                                    \
    } while (0)

constexpr int ROWS = 8192;      // x 64 floats = 2 MiB: fits one XCD's 4 MiB L2
constexpr int COLS = 64;

__device__ __forceinline__ int xcc_id() { return __builtin_amdgcn_s_getreg((3 << 11) | 20) & 7; }

__global__ void read_rows(const float* __restrict__ x, float* __restrict__ sink) {
    const int xc = xcc_id();
    float s = 0.f;
    for (int r = xc; r < ROWS; r += 8)
        for (int c = threadIdx.x; c < COLS; c += blockDim.x) s += x[r * COLS + c];
    sink[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ void write_rows(float* __restrict__ x, float g, int shift) {
    const int xc = xcc_id();
    for (int r = (xc + shift) & 7; r < ROWS; r += 8)
        for (int c = threadIdx.x; c < COLS; c += blockDim.x) x[r * COLS + c] = g;
}

__global__ void check_rows(const float* __restrict__ x, float g, unsigned* __restrict__ bad) {
    const int xc = xcc_id();
    unsigned n = 0;
    for (int r = xc; r < ROWS; r += 8)
        for (int c = threadIdx.x; c < COLS; c += blockDim.x) n += x[r * COLS + c] != g;
    if (n) atomicAdd(bad, n);
}

__global__ void census(unsigned* __restrict__ seen) {
    if (threadIdx.x == 0) atomicOr(seen, 1u << xcc_id());
}

int main(int argc, char** argv) {
    const int rounds = argc > 1 ? atoi(argv[1]) : 200;
    const int blocks = 1024, threads = 64;
    float *x, *sink;
    unsigned *bad, *seen;
    CHECK(hipMalloc(&x, ROWS * COLS * sizeof(float)));
    CHECK(hipMalloc(&sink, blocks * threads * sizeof(float)));
    CHECK(hipMalloc(&bad, sizeof(unsigned)));
    CHECK(hipMalloc(&seen, sizeof(unsigned)));
    CHECK(hipMemset(x, 0, ROWS * COLS * sizeof(float)));
    CHECK(hipMemset(bad, 0, sizeof(unsigned)));
    CHECK(hipMemset(seen, 0, sizeof(unsigned)));
    census<<<blocks, threads>>>(seen);
    unsigned s = 0;
    CHECK(hipMemcpy(&s, seen, sizeof(s), hipMemcpyDeviceToHost));
    printf("XCDs seen by a %d-block grid: mask 0x%02x\n", blocks, s);
    hipStream_t st;
    CHECK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
    for (int shift = 0; shift < 2; ++shift) {
        unsigned total = 0, bad_rounds = 0;
        for (int g = 1; g <= rounds; ++g) {
            CHECK(hipMemsetAsync(bad, 0, sizeof(unsigned), st));
            read_rows<<<blocks, threads, 0, st>>>(x, sink);
            write_rows<<<blocks, threads, 0, st>>>(x, (float)g, shift ? 1 : 0);
            check_rows<<<blocks, threads, 0, st>>>(x, (float)g, bad);
            unsigned b = 0;
            CHECK(hipMemcpyAsync(&b, bad, sizeof(b), hipMemcpyDeviceToHost, st));
            CHECK(hipStreamSynchronize(st));
            total += b;
            bad_rounds += b != 0;
        }
        printf("%s: %d rounds, %u rounds with stale entries, %u stale entry reads in total\n",
               shift ? "writer XCD != reader XCD" : "writer XCD == reader XCD (control)", rounds, bad_rounds, total);
    }
    CHECK(hipStreamDestroy(st));
    return 0;
}
