// First-touch check: does a kernel's write into freshly hipMalloc'd memory always survive?
// Each trial allocates a new buffer, fills it with a trial-specific pattern by a kernel (vector stores),
// runs a second kernel that checks the pattern on the device and counts mismatching dwords, then frees it.
//   hipcc --offload-arch=gfx950 -O2 tools/first_touch.hip -o tools/first_touch && tools/first_touch [trials] [MB]
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

__global__ void fill(unsigned* p, size_t n, unsigned seed) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        p[i] = seed ^ (unsigned)(i * 2654435761u);
}

__global__ void check(const unsigned* p, size_t n, unsigned seed, unsigned long long* bad, unsigned long long* zero) {
    unsigned long long b = 0, z = 0;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        const unsigned v = p[i];
        if (v != (seed ^ (unsigned)(i * 2654435761u))) {
            ++b;
            z += v == 0;
        }
    }
    if (b) {
        atomicAdd(bad, b);
        atomicAdd(zero, z);
    }
}

int main(int argc, char** argv) {
    const int trials = argc > 1 ? atoi(argv[1]) : 200;
    const size_t mb = argc > 2 ? (size_t)atol(argv[2]) : 280;
    unsigned long long *d_bad, *d_zero;
    if (hipMalloc(&d_bad, 8) != hipSuccess || hipMalloc(&d_zero, 8) != hipSuccess) return 2;
    unsigned long long total_bad = 0, bad_trials = 0;
    for (int t = 0; t < trials; ++t) {
        const size_t bytes = (mb << 20) + (size_t)(t % 7) * 4096 * 33;   // vary the size a little
        const size_t n = bytes / 4;
        unsigned* p = nullptr;
        if (hipMalloc(&p, bytes) != hipSuccess) { fprintf(stderr, "hipMalloc failed\n"); return 2; }
        (void)hipMemset(d_bad, 0, 8);
        (void)hipMemset(d_zero, 0, 8);
        fill<<<4096, 256>>>(p, n, 0x9E3779B9u * (t + 1));
        check<<<4096, 256>>>(p, n, 0x9E3779B9u * (t + 1), d_bad, d_zero);
        unsigned long long bad = 0, zero = 0;
        (void)hipMemcpy(&bad, d_bad, 8, hipMemcpyDeviceToHost);
        (void)hipMemcpy(&zero, d_zero, 8, hipMemcpyDeviceToHost);
        if (bad) {
            ++bad_trials;
            total_bad += bad;
            printf("trial %d: %llu of %zu dwords wrong (%llu of them zero)\n", t, bad, n, zero);
        }
        (void)hipFree(p);
        if (t % 50 == 0) { printf("trial %d done\n", t); fflush(stdout); }
    }
    printf("first_touch: %d trials x %zu MB, %llu trials with wrong dwords, %llu wrong dwords\n", trials, mb,
           bad_trials, total_bad);
    return 0;
}
