// als_kernels.hip -- hand-written gfx950 (CDNA4) kernels for the ALS half-iteration.
//
// Hot path being replaced: MFeatureCalculator.java:66-104 / UFeatureCalculator.java:66-104 (EJML fp32
// multTransA -> add(lambda * n * I) -> invert -> mult, one entity at a time). Here one 64-lane wave owns
// one Task (cfk::Task, see als_internal.h): it gathers the opposite factor rows of its in-block entries,
// accumulates the Gram matrix Y^T Y and RHS Y^T r, and -- for FULL / REDUCE tasks -- regularises and
// Cholesky-solves the k x k system inside the wave, writing one factor row.
//
// Gram accumulation paths:
//   MFMA (fp32, KP = 32 / 64): v_mfma_f32_16x16x4_f32. Lane l = (g = l>>4, j = l&15) holds entry g of a
//        4-entry sub-step and gathers the 16-B (KP=64) / 8-B (KP=32) piece [C*j, C*j+C) of that entry's
//        factor row, so a 16-lane group reads one whole row (coalesced). With C = KP/16 components per lane,
//        tile (b1,b2) = mfma(A = y[b1], B = y[b2]) accumulates G[C*i + b1][C*j' + b2]; only b1 <= b2 tiles
//        are issued (10 of 16 at KP=64: G is symmetric), each gathered register feeds C MFMAs directly (no
//        LDS, no shuffles). RHS is a per-lane VALU FMA, reduced across the 4 groups at the end.
//   VALU (fp32 KP = 16, all fp64): 64 gathered rows are staged in LDS (coalesced 16-B vector loads), then
//        each lane accumulates KP*KP/64 Gram entries of one row from LDS broadcasts.
// Solve: the Gram is canonicalised into a per-wave LDS matrix G[KP][KP+1]; lane j loads row j, adds
// lambda*n_j to the diagonal, and runs a right-looking Cholesky with L's column broadcast through LDS,
// then forward / backward substitution with v_readlane broadcasts (L transposed once through LDS).
#include <hip/hip_runtime.h>

#include <type_traits>

#include "als_internal.h"

namespace cfk {
namespace {

constexpr int WAVES = 4;       // waves (tasks) per 256-thread workgroup
constexpr int RSTAGE = 64;     // VALU path: rows staged per LDS block

typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef double f64x2 __attribute__((ext_vector_type(2)));

template <class T> struct Vec16;
template <> struct Vec16<float> { typedef f32x4 type; static constexpr int N = 4; };
template <> struct Vec16<double> { typedef f64x2 type; static constexpr int N = 2; };

template <int C> struct VecC;
template <> struct VecC<2> { typedef f32x2 type; };
template <> struct VecC<4> { typedef f32x4 type; };

// Same-wave LDS hand-off: the hardware keeps one wave's DS operations in order; this only stops the
// compiler from moving LDS accesses across the point.
__device__ __forceinline__ void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

__device__ __forceinline__ float bcast(float v, int src) {
    return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), src));
}
__device__ __forceinline__ double bcast(double v, int src) {
    const long long b = __double_as_longlong(v);
    const int lo = __builtin_amdgcn_readlane((int)(unsigned)(b & 0xffffffffll), src);
    const int hi = __builtin_amdgcn_readlane((int)(b >> 32), src);
    return __longlong_as_double(((long long)hi << 32) | (long long)(unsigned)lo);
}
__device__ __forceinline__ int uni(int v) { return __builtin_amdgcn_readfirstlane(v); }
// Fresh copy of a per-lane value the optimizer cannot see through: stops LLVM from CSE-ing the 3*KP
// lane-vs-step comparisons of the unrolled solve into live SGPR masks (which spill).
__device__ __forceinline__ int opaque(int v) {
    asm volatile("" : "+v"(v));
    return v;
}

__device__ __forceinline__ Task load_task(const Task* p) {
    Task t = *p;
    t.begin = ((int64_t)uni((int)(t.begin >> 32)) << 32) | (int64_t)(uint32_t)uni((int)(uint32_t)t.begin);
    t.nsteps = uni(t.nsteps);
    t.row = uni(t.row);
    t.slot = uni(t.slot);
    t.ndeg = uni(t.ndeg);
    t.kind = uni(t.kind);
    return t;
}

// ---------------------------------------------------------------------------------------------------
// Per-wave LDS carve-up
// ---------------------------------------------------------------------------------------------------
__host__ __device__ constexpr int round16(int b) { return (b + 15) & ~15; }

template <class T, int KP, Path P>
struct WaveLds {
    static constexpr int LD = KP + 1;                                 // conflict-free row and column reads
    static constexpr int G_BYTES = round16(KP * LD * (int)sizeof(T));
    static constexpr int STAGE_BYTES = (P == Path::VALU) ? round16(RSTAGE * KP * (int)sizeof(T)) : 0;
    static constexpr int MAIN_BYTES = G_BYTES > STAGE_BYTES ? G_BYTES : STAGE_BYTES;   // staging aliases G
    static constexpr int RHS_OFF = MAIN_BYTES;
    static constexpr int BC_OFF = RHS_OFF + round16(KP * (int)sizeof(T));
    static constexpr int SIDX_OFF = BC_OFF + round16(KP * (int)sizeof(T));
    static constexpr int SRAT_OFF = SIDX_OFF + ((P == Path::VALU) ? round16(RSTAGE * 4) : 0);
    static constexpr int BYTES = SRAT_OFF + ((P == Path::VALU) ? round16(RSTAGE * (int)sizeof(T)) : 0);
};

// ---------------------------------------------------------------------------------------------------
// In-wave Cholesky solve (lane j = row j), shared by both paths
// ---------------------------------------------------------------------------------------------------
template <class T, int KP>
__device__ __forceinline__ void solve_store(T* G, const T* rhs_l, T* bc, const Task& tk, const SolveArgs& a,
                                            int lane) {
    constexpr int LD = KP + 1;
    const int j = lane;
    const bool act = j < KP;
    const int jr = act ? j : 0;
    T* out = (T*)a.out + (a.row_offset + tk.row) * (int64_t)KP;

    if (tk.ndeg == 0) {   // cannot occur in the reference (entities exist only once rated); defined as 0
        if (act) out[j] = T(0);
        return;
    }

    T av[KP];
#pragma unroll
    for (int i = 0; i < KP; ++i) av[i] = G[jr * LD + i];
    T y = act ? rhs_l[jr] : T(0);

    // A + lambda * (n * I): fp32 mirrors add(A, lambda, n*I) (MFeatureCalculator.java:91-95) -> lambda*(float)n
    const T reg = (T)a.lambda * (T)tk.ndeg;
    const bool real_feature = j < a.k;
#pragma unroll
    for (int i = 0; i < KP; ++i) {
        const int jo = opaque(j);
        if (i == jo) av[i] = real_feature ? av[i] + reg : T(1);   // padded features: identity rows
    }

    // Right-looking Cholesky: after step p lane j holds L[j][0..p] in av[0..p]. Column p of L is
    // broadcast through a KP-word LDS vector read back 16 B at a time; sched_barriers keep the compiler
    // from hoisting later steps' reads (which would blow the register budget).
    using BV = typename Vec16<T>::type;
    constexpr int BN = Vec16<T>::N;
    T dinv = T(0);
#pragma unroll
    for (int p = 0; p < KP; ++p) {
        const int jo = opaque(j);
        const T d = sqrt(bcast(av[p], p));
        const T id = T(1) / d;
        const T l = (jo > p) ? av[p] * id : ((jo == p) ? d : T(0));
        av[p] = l;
        dinv = (jo == p) ? id : dinv;
        if (act) bc[j] = l;
        wave_sync();
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int q = ((p + 1) / BN) * BN; q < KP; q += BN) {
            const BV b = *(const BV*)(bc + q);
#pragma unroll
            for (int c = 0; c < BN; ++c)
                if (q + c > p) av[q + c] -= b[c] * l;
            if ((q / BN) % 4 == 3) __builtin_amdgcn_sched_barrier(0);
        }
        wave_sync();
        __builtin_amdgcn_sched_barrier(0);
    }
    // Forward substitution L y = b (lane j owns row j of L).
#pragma unroll
    for (int p = 0; p < KP; ++p) {
        const int jo = opaque(j);
        const T yp = bcast(y, p) * bcast(dinv, p);
        y = (jo == p) ? yp : ((jo > p) ? y - av[p] * yp : y);
    }
    // Transpose L through LDS: lane j then owns column j (av[i] = L[i][j]).
    if (act) {
#pragma unroll
        for (int i = 0; i < KP; ++i) G[j * LD + i] = av[i];
    }
    wave_sync();
#pragma unroll
    for (int i = 0; i < KP; ++i) av[i] = G[i * LD + jr];
    // Backward substitution L^T x = y.
#pragma unroll
    for (int p = KP - 1; p >= 0; --p) {
        const int jo = opaque(j);
        const T xp = bcast(y, p) * bcast(dinv, p);
        y = (jo == p) ? xp : ((jo < p) ? y - av[p] * xp : y);
    }
    if (act) out[j] = (j < a.k) ? y : T(0);
}

// ---------------------------------------------------------------------------------------------------
// MFMA Gram path (fp32, KP = 16*C with C in {2, 4})
// ---------------------------------------------------------------------------------------------------
template <int C>
struct MfmaAcc {
    static constexpr int NT = C * (C + 1) / 2;     // upper-triangular tiles (b1 <= b2)
    static constexpr int NWORDS = NT * 4 + C;       // per-lane words of one partial slot
    f32x4 g[NT];
    float rhs[C];
};

template <int C>
__host__ __device__ constexpr int tile_index(int b1, int b2) { return b1 * C - (b1 * (b1 - 1)) / 2 + (b2 - b1); }

template <int KP>
__global__ __launch_bounds__(256) void als_solve_mfma(SolveArgs a) {
    constexpr int C = KP / 16;
    using Acc = MfmaAcc<C>;
    using VT = typename VecC<C>::type;
    using L = WaveLds<float, KP, Path::MFMA>;
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];

    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int tid = blockIdx.x * WAVES + wave;
    if (tid >= a.n_tasks) return;   // wave-uniform; no workgroup barriers are used below
    const Task tk = load_task(a.tasks + tid);
    unsigned char* wl = smem + wave * L::BYTES;
    float* G = (float*)wl;
    float* rhs_l = (float*)(wl + L::RHS_OFF);
    float* bc = (float*)(wl + L::BC_OFF);

    const int g = lane >> 4, j = lane & 15;
    Acc acc;
#pragma unroll
    for (int p = 0; p < Acc::NT; ++p) acc.g[p] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int c = 0; c < C; ++c) acc.rhs[c] = 0.f;

    float* part = (float*)a.partials;
    if (tk.kind == TASK_REDUCE) {
        // Fixed-order sum of the row's partial slots ([word][lane] layout, coalesced).
        for (int s = 0; s < tk.nsteps; ++s) {
            const float* src = part + (int64_t)(tk.slot + s) * (Acc::NWORDS * 64) + lane;
#pragma unroll
            for (int p = 0; p < Acc::NT; ++p)
#pragma unroll
                for (int r = 0; r < 4; ++r) acc.g[p][r] += src[(p * 4 + r) * 64];
#pragma unroll
            for (int c = 0; c < C; ++c) acc.rhs[c] += src[(Acc::NT * 4 + c) * 64];
        }
    } else {
        const float* opp = (const float*)a.opp;
        const int n = tk.nsteps;
        const int32_t* cp = a.col + tk.begin + g;
        const float* rp = a.rat + tk.begin + g;
        constexpr int U = 4;
        int idx_c[U], idx_n[U];
        float r_c[U], r_n[U];
        VT y_c[U], y_n[U];
        auto load_idx = [&](int t0, int (&idx)[U], float (&r)[U]) {
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const int t = t0 + u;
                idx[u] = (t < n) ? cp[4 * t] : -1;
                r[u] = (t < n) ? rp[4 * t] : 0.f;
            }
        };
        auto gather = [&](const int (&idx)[U], VT (&y)[U]) {
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const int id = idx[u] < 0 ? 0 : idx[u];
                const VT v = *(const VT*)(opp + (int64_t)id * KP + C * j);
                y[u] = idx[u] < 0 ? VT(0.f) : v;
            }
        };
        load_idx(0, idx_c, r_c);
        gather(idx_c, y_c);
        load_idx(U, idx_n, r_n);
        for (int t0 = 0; t0 < n; t0 += U) {
            gather(idx_n, y_n);                 // next block's rows in flight under this block's MFMAs
            int idx_nn[U];
            float r_nn[U];
            load_idx(t0 + 2 * U, idx_nn, r_nn);
#pragma unroll
            for (int u = 0; u < U; ++u) {
                if (t0 + u < n) {               // wave-uniform
#pragma unroll
                    for (int b1 = 0; b1 < C; ++b1)
#pragma unroll
                        for (int b2 = b1; b2 < C; ++b2)
                            acc.g[tile_index<C>(b1, b2)] = __builtin_amdgcn_mfma_f32_16x16x4f32(
                                y_c[u][b1], y_c[u][b2], acc.g[tile_index<C>(b1, b2)], 0, 0, 0);
#pragma unroll
                    for (int c = 0; c < C; ++c) acc.rhs[c] += r_c[u] * y_c[u][c];
                }
            }
#pragma unroll
            for (int u = 0; u < U; ++u) {
                y_c[u] = y_n[u];
                r_c[u] = r_n[u];
                idx_n[u] = idx_nn[u];
                r_n[u] = r_nn[u];
            }
        }
    }

    if (tk.kind == TASK_PARTIAL) {
        float* dst = part + (int64_t)tk.slot * (Acc::NWORDS * 64) + lane;
#pragma unroll
        for (int p = 0; p < Acc::NT; ++p)
#pragma unroll
            for (int r = 0; r < 4; ++r) dst[(p * 4 + r) * 64] = acc.g[p][r];
#pragma unroll
        for (int c = 0; c < C; ++c) dst[(Acc::NT * 4 + c) * 64] = acc.rhs[c];
        return;
    }

    // Canonicalise: tile (b1,b2) lane (g,j) reg r holds G[C*(4g+r)+b1][C*j+b2]; mirror off-diagonal tiles.
    constexpr int LD = KP + 1;
#pragma unroll
    for (int b1 = 0; b1 < C; ++b1)
#pragma unroll
        for (int b2 = b1; b2 < C; ++b2)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const float v = acc.g[tile_index<C>(b1, b2)][r];
                const int row = C * (4 * g + r) + b1, col = C * j + b2;
                G[row * LD + col] = v;
                if (b1 != b2) G[col * LD + row] = v;
            }
#pragma unroll
    for (int c = 0; c < C; ++c) {
        float v = acc.rhs[c];
        v += __shfl_xor(v, 16);
        v += __shfl_xor(v, 32);
        if (g == 0) rhs_l[C * j + c] = v;
    }
    wave_sync();
    solve_store<float, KP>(G, rhs_l, bc, tk, a, lane);
}

// ---------------------------------------------------------------------------------------------------
// VALU Gram path (LDS-staged rows), fp32 and fp64
// ---------------------------------------------------------------------------------------------------
template <class T, int KP>
__global__ __launch_bounds__(256) void als_solve_valu(SolveArgs a) {
    constexpr int LPR = 64 / KP;            // lanes per Gram row
    constexpr int E = KP / LPR;             // Gram entries per lane (= KP*KP/64)
    constexpr int NWORDS = E + 1;           // + RHS
    constexpr int VN = Vec16<T>::N;         // elements per 16-B vector
    constexpr int V = KP / VN;              // 16-B vectors per factor row
    using VT = typename Vec16<T>::type;
    using L = WaveLds<T, KP, Path::VALU>;
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];

    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int tid = blockIdx.x * WAVES + wave;
    if (tid >= a.n_tasks) return;
    const Task tk = load_task(a.tasks + tid);
    unsigned char* wl = smem + wave * L::BYTES;
    T* G = (T*)wl;
    T* stage = (T*)wl;   // aliases G: staging is dead before the Gram is canonicalised
    T* rhs_l = (T*)(wl + L::RHS_OFF);
    T* bc = (T*)(wl + L::BC_OFF);
    int32_t* sidx = (int32_t*)(wl + L::SIDX_OFF);
    T* srat = (T*)(wl + L::SRAT_OFF);

    const int arow = lane / LPR, c0 = (lane % LPR) * E;
    T acc[E];
#pragma unroll
    for (int e = 0; e < E; ++e) acc[e] = T(0);
    T rhs = T(0);

    T* part = (T*)a.partials;
    if (tk.kind == TASK_REDUCE) {
        for (int s = 0; s < tk.nsteps; ++s) {
            const T* src = part + (int64_t)(tk.slot + s) * (NWORDS * 64) + lane;
#pragma unroll
            for (int e = 0; e < E; ++e) acc[e] += src[e * 64];
            rhs += src[E * 64];
        }
    } else {
        const T* opp = (const T*)a.opp;
        const int n = tk.nsteps * 4;
        for (int base = 0; base < n; base += RSTAGE) {
            const int e = base + lane;
            int idx = -1;
            T r = T(0);
            if (e < n) {
                idx = a.col[tk.begin + e];
                r = (T)a.rat[tk.begin + e];
            }
            sidx[lane] = idx;
            srat[lane] = r;
            wave_sync();
#pragma unroll
            for (int q = 0; q < V; ++q) {       // RSTAGE * V vectors, 64 per instruction
                const int pair = q * 64 + lane;
                const int t = pair / V, v = pair % V;
                const int id = sidx[t];
                const VT val = *(const VT*)(opp + (int64_t)(id < 0 ? 0 : id) * KP + v * VN);
                *(VT*)(stage + t * KP + v * VN) = id < 0 ? VT(T(0)) : val;
            }
            wave_sync();
            const int nt = (n - base) < RSTAGE ? (n - base) : RSTAGE;
            for (int t = 0; t < nt; ++t) {
                const T ya = stage[t * KP + arow];
#pragma unroll
                for (int e2 = 0; e2 < E; ++e2) acc[e2] += ya * stage[t * KP + c0 + e2];
                rhs += srat[t] * ya;
            }
            wave_sync();
        }
    }

    if (tk.kind == TASK_PARTIAL) {
        T* dst = part + (int64_t)tk.slot * (NWORDS * 64) + lane;
#pragma unroll
        for (int e = 0; e < E; ++e) dst[e * 64] = acc[e];
        dst[E * 64] = rhs;
        return;
    }

    constexpr int LD = KP + 1;
#pragma unroll
    for (int e = 0; e < E; ++e) G[arow * LD + c0 + e] = acc[e];
    if (lane % LPR == 0) rhs_l[arow] = rhs;
    wave_sync();
    solve_store<T, KP>(G, rhs_l, bc, tk, a, lane);
}

// ---------------------------------------------------------------------------------------------------
// Squared-error reduction over observed ratings (RMSE numerator; scripts/calculate_mse.py:78-90)
// ---------------------------------------------------------------------------------------------------
template <class T, int KP>
__global__ __launch_bounds__(256) void als_sq_error_kernel(SqErrArgs a) {
    constexpr int VN = Vec16<T>::N;
    constexpr int LPE = KP / VN;            // lanes per entry (one 16-B piece each)
    constexpr int EPS = 64 / LPE;           // entries per wave step
    using VT = typename Vec16<T>::type;
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int tid = blockIdx.x * WAVES + wave;
    if (tid >= a.n_tasks) return;
    const Task tk = load_task(a.tasks + tid);
    const int es = lane / LPE, v = lane % LPE;
    const T* self = (const T*)a.self + (a.row_offset + tk.row) * (int64_t)KP;
    const T* opp = (const T*)a.opp;
    const VT x = *(const VT*)(self + v * VN);
    const int n = tk.nsteps * 4;
    double se = 0.0;
    for (int base = 0; base < n; base += EPS) {
        const int e = base + es;
        int idx = -1;
        float r = 0.f;
        if (e < n) {
            idx = a.col[tk.begin + e];
            r = a.rat[tk.begin + e];
        }
        const VT y = *(const VT*)(opp + (int64_t)(idx < 0 ? 0 : idx) * KP + v * VN);
        T dot = T(0);
#pragma unroll
        for (int c = 0; c < VN; ++c) dot += x[c] * y[c];
#pragma unroll
        for (int m = 1; m < LPE; m <<= 1) dot += __shfl_xor(dot, m);
        if (v == 0 && idx >= 0) {
            const double d = (double)r - (double)dot;
            se += d * d;
        }
    }
#pragma unroll
    for (int m = 1; m < 64; m <<= 1) se += __shfl_xor(se, m);
    if (lane == 0) a.task_se[tid] = se;
}

int blocks_for(int n_tasks) { return (n_tasks + WAVES - 1) / WAVES; }

template <class T, int KP, Path P>
hipError_t launch_solve_t(const SolveArgs& a, hipStream_t s) {
    if (a.n_tasks <= 0) return hipSuccess;
    constexpr int bytes = WAVES * WaveLds<T, KP, P>::BYTES;
    if constexpr (P == Path::MFMA) {
        static_assert(std::is_same<T, float>::value, "MFMA path is fp32");
        static bool attr = false;
        if (!attr) {
            hipError_t e = hipFuncSetAttribute((const void*)als_solve_mfma<KP>,
                                               hipFuncAttributeMaxDynamicSharedMemorySize, bytes);
            if (e != hipSuccess) return e;
            attr = true;
        }
        als_solve_mfma<KP><<<blocks_for(a.n_tasks), 256, bytes, s>>>(a);
    } else {
        static bool attr = false;
        if (!attr) {
            hipError_t e = hipFuncSetAttribute((const void*)als_solve_valu<T, KP>,
                                               hipFuncAttributeMaxDynamicSharedMemorySize, bytes);
            if (e != hipSuccess) return e;
            attr = true;
        }
        als_solve_valu<T, KP><<<blocks_for(a.n_tasks), 256, bytes, s>>>(a);
    }
    return hipGetLastError();
}

template <class T, int KP>
hipError_t launch_sq_t(const SqErrArgs& a, hipStream_t s) {
    if (a.n_tasks <= 0) return hipSuccess;
    als_sq_error_kernel<T, KP><<<blocks_for(a.n_tasks), 256, 0, s>>>(a);
    return hipGetLastError();
}

}  // namespace

bool variant_available(int precision, int kp, Path path) {
    if (precision == 0) {
        if (path == Path::MFMA) return kp == 32 || kp == 64;
        return kp == 16 || kp == 32 || kp == 64;
    }
    return path == Path::VALU && (kp == 16 || kp == 32 || kp == 64);
}

int partial_words_per_lane(int precision, int kp, Path path) {
    if (path == Path::MFMA) {
        const int c = kp / 16;
        return (c * (c + 1) / 2) * 4 + c;
    }
    return kp * kp / 64 + 1;
}

hipError_t launch_solve(int precision, int kp, Path path, const SolveArgs& a, hipStream_t s) {
    if (precision == 0) {
        if (path == Path::MFMA) {
            if (kp == 32) return launch_solve_t<float, 32, Path::MFMA>(a, s);
            if (kp == 64) return launch_solve_t<float, 64, Path::MFMA>(a, s);
        } else {
            if (kp == 16) return launch_solve_t<float, 16, Path::VALU>(a, s);
            if (kp == 32) return launch_solve_t<float, 32, Path::VALU>(a, s);
            if (kp == 64) return launch_solve_t<float, 64, Path::VALU>(a, s);
        }
    } else if (path == Path::VALU) {
        if (kp == 16) return launch_solve_t<double, 16, Path::VALU>(a, s);
        if (kp == 32) return launch_solve_t<double, 32, Path::VALU>(a, s);
        if (kp == 64) return launch_solve_t<double, 64, Path::VALU>(a, s);
    }
    return hipErrorInvalidValue;
}

hipError_t launch_sq_error(int precision, int kp, const SqErrArgs& a, hipStream_t s) {
    if (precision == 0) {
        if (kp == 16) return launch_sq_t<float, 16>(a, s);
        if (kp == 32) return launch_sq_t<float, 32>(a, s);
        if (kp == 64) return launch_sq_t<float, 64>(a, s);
    } else {
        if (kp == 16) return launch_sq_t<double, 16>(a, s);
        if (kp == 32) return launch_sq_t<double, 32>(a, s);
        if (kp == 64) return launch_sq_t<double, 64>(a, s);
    }
    return hipErrorInvalidValue;
}

}  // namespace cfk
