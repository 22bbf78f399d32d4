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
// Solve: the Gram is canonicalised into a per-wave packed lower triangle in LDS (KP*(KP+1)/2 words); lane j
// loads row j, adds lambda*n_j to the diagonal, and runs a right-looking Cholesky: the two look-ahead
// columns of every step are broadcast with v_readlane (so the pivot chain never waits on LDS) and the bulk
// of L's column goes through a KP-word LDS vector read back 16 B at a time; forward substitution is fused
// into the factorisation; L is transposed once through the packed triangle for the backward substitution.
#include <hip/hip_runtime.h>

#include <mutex>
#include <type_traits>
#include <utility>
#include <vector>

#include "als_internal.h"

namespace cfk {
namespace {

constexpr int WAVES = 4;       // waves (tasks) per 256-thread workgroup
constexpr int RSTAGE = 64;     // VALU path: rows staged per LDS block

typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x8 __attribute__((ext_vector_type(8)));
typedef double f64x2 __attribute__((ext_vector_type(2)));

typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
typedef unsigned u32x2 __attribute__((ext_vector_type(2)));

template <class T> struct Vec16;
template <> struct Vec16<float> { typedef f32x4 type; static constexpr int N = 4; };
template <> struct Vec16<double> { typedef f64x2 type; static constexpr int N = 2; };

template <int C> struct VecC;
template <> struct VecC<2> { typedef f32x2 type; };
template <> struct VecC<4> { typedef f32x4 type; };
template <> struct VecC<8> { typedef f32x8 type; };

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
// Compile-time loop: f(std::integral_constant<int, i>) for i in [B, E). Every index derived from i is a
// constant expression, so register arrays are never indexed dynamically (no scratch).
template <int B, int E, class F>
__device__ __forceinline__ void static_for(F&& f) {
    if constexpr (B < E) {
        f(std::integral_constant<int, B>{});
        static_for<B + 1, E>(f);
    }
}
// Fresh copy of a per-lane value the optimizer cannot see through: stops LLVM from CSE-ing the 3*KP
// lane-vs-step comparisons of the unrolled solve into live SGPR masks (which spill).
__device__ __forceinline__ int opaque(int v) {
    asm volatile("" : "+v"(v));
    return v;
}
// Materialise a value here: keeps LLVM from sinking a step's rank-1 updates into deferred FMA chains at the
// next use (MachineSink ignores sched_barrier), which multiplies live registers in the unrolled solve.
__device__ __forceinline__ void pin(float& v) { asm volatile("" : "+v"(v)); }
__device__ __forceinline__ void pin(double& v) { asm volatile("" : "+v"(v)); }
__device__ __forceinline__ void pin(unsigned& v) { asm volatile("" : "+v"(v)); }

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
// Partial-slot integrity. A PARTIAL task stores word w of lane l of slot s as bits ^ key(gen, s, l, w) plus
// one check word (the wrap-around sum of the plain words); its REDUCE task decodes with the SAME launch
// generation and re-sums. A slot line the REDUCE cannot see freshly written -- never written, left over
// from an earlier launch (which, on identical inputs, would hold identical numbers and be invisible to any
// comparison of results), or torn -- decodes to noise and fails the check; the failure is counted in
// SolveArgs::integrity and the engine's next synchronising call reports it (ALS_ERR_INTEGRITY).
// ---------------------------------------------------------------------------------------------------
__device__ __forceinline__ uint32_t mix32(uint32_t x) {
    x ^= x >> 16;
    x *= 0x7feb352du;
    x ^= x >> 15;
    x *= 0x846ca68bu;
    x ^= x >> 16;
    return x;
}
__device__ __forceinline__ uint32_t slot_key(uint32_t gen, int32_t slot, int lane) {
    return mix32(gen * 0x9e3779b1u ^ mix32((uint32_t)slot * 64u + (uint32_t)lane));
}
constexpr uint32_t WORD_KEY_STEP = 0x632be5abu;
struct SlotCodec {
    uint32_t key, sum = 0;
    __device__ __forceinline__ float enc(float v, int w) {
        const uint32_t b = __float_as_uint(v);
        sum += b;
        return __uint_as_float(b ^ (key + (uint32_t)w * WORD_KEY_STEP));
    }
    __device__ __forceinline__ float dec(float v, int w) {
        const uint32_t b = __float_as_uint(v) ^ (key + (uint32_t)w * WORD_KEY_STEP);
        sum += b;
        return __uint_as_float(b);
    }
    __device__ __forceinline__ double enc(double v, int w) {
        const uint64_t b = (uint64_t)__double_as_longlong(v);
        sum += (uint32_t)b + (uint32_t)(b >> 32);
        const uint64_t k = key + (uint32_t)w * WORD_KEY_STEP;
        return __longlong_as_double((long long)(b ^ (k | (k << 32))));
    }
    __device__ __forceinline__ double dec(double v, int w) {
        const uint64_t k = key + (uint32_t)w * WORD_KEY_STEP;
        const uint64_t b = (uint64_t)__double_as_longlong(v) ^ (k | (k << 32));
        sum += (uint32_t)b + (uint32_t)(b >> 32);
        return __longlong_as_double((long long)b);
    }
    // check word (element w of the slot), stored keyed like the data words
    template <class T>
    __device__ __forceinline__ T check_word(int w) const {
        const uint32_t c = sum ^ (key + (uint32_t)w * WORD_KEY_STEP);
        if constexpr (sizeof(T) == 4) return __uint_as_float(c);
        else return __longlong_as_double((long long)(uint64_t)c);
    }
    template <class T>
    __device__ __forceinline__ bool check_ok(T stored, int w) const {
        uint32_t c;
        if constexpr (sizeof(T) == 4) c = __float_as_uint(stored);
        else c = (uint32_t)(uint64_t)__double_as_longlong(stored);
        return (c ^ (key + (uint32_t)w * WORD_KEY_STEP)) == sum;
    }
};
// Vector-memory atomics only, from the first failing lane (slot = the first slot that lane found bad).
__device__ __forceinline__ void report_bad_slot(uint32_t* rec, uint32_t gen, int32_t slot, int32_t row, bool bad,
                                                int lane) {
    const uint64_t m = __ballot(bad);
    if (m == 0) return;
    if (lane == (int)__builtin_ctzll(m)) {
        const uint32_t n = atomicAdd(rec, 1u);
        if (n == 0) {
            atomicExch(rec + 1, gen);
            atomicExch(rec + 2, (uint32_t)slot);
            atomicExch(rec + 3, (uint32_t)row);
        }
    }
}

// ---------------------------------------------------------------------------------------------------
// Per-wave LDS carve-up
// ---------------------------------------------------------------------------------------------------
__host__ __device__ constexpr int round16(int b) { return (b + 15) & ~15; }

template <class T, int KP, Path P>
struct WaveLds {
    static constexpr int G_BYTES = round16(KP * (KP + 1) / 2 * (int)sizeof(T));   // packed lower triangle
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
// packed lower-triangular index (c <= r)
__host__ __device__ constexpr int tri(int r, int c) { return r * (r + 1) / 2 + c; }

// Pivot of one Cholesky step: d = sqrt(a), dinv = 1/sqrt(a). fp32 uses v_rsq_f32 (1 ulp; the fp32 fast mode
// is held to an MSE bound), fp64 keeps correctly rounded sqrt and division for the 1e-6 parity mode.
__device__ __forceinline__ void pivot(float a, float& d, float& dinv) {
    dinv = __builtin_amdgcn_rsqf(a);
    d = a * dinv;
}
__device__ __forceinline__ void pivot(double a, double& d, double& dinv) {
    d = sqrt(a);
    dinv = 1.0 / d;
}

// Lane j owns row j of A and computes row j of L. A lane never needs an entry right of its diagonal
// (i > j): those registers may hold anything finite, which makes the solve nearly select-free -- every
// step runs the same instructions on all lanes; only the per-step uniform results (1/L[p][p], the forward
// and backward solution components) are dropped into lane p with one compare + select; the row load and
// the transposition are unpredicated LDS accesses.
template <class T, int KP>
__device__ __forceinline__ void solve_store(T* P, const T* rhs_l, T* bc, const Task& tk, const SolveArgs& a,
                                            int lane) {
    using BV = typename Vec16<T>::type;
    constexpr int BN = Vec16<T>::N;
    static_assert(KP <= 64, "one row per lane");
    const int j = lane;
    const bool act = j < KP;
    const int jr = act ? j : KP - 1;
    T* out = (T*)a.out + factor_row(a.row_offset, a.rows_per_chunk, a.chunk_stride, tk.row) * (int64_t)KP;

    if (tk.ndeg == 0) {   // cannot occur in the reference (entities exist only once rated); defined as 0
        if (act) out[j] = T(0);
        return;
    }

    // A + lambda * (n * I) on the packed diagonal: fp32 mirrors add(A, lambda, n*I)
    // (MFeatureCalculator.java:91-95) -> A[j][j] + lambda*(float)n; padded features get an identity row.
    const T reg = (T)a.lambda * (T)tk.ndeg;
    const int rowbase = tri(jr, 0);
    if (act) {
        const T dd = P[rowbase + jr];
        P[rowbase + jr] = (j < a.k) ? dd + reg : T(1);
    }
    wave_sync();
    // Row j, entries 0..KP-1 read straight through the packed triangle: entries i > j land in the next
    // rows' storage (finite, never used). rowbase + i <= tri(KP-1, 0) + KP-1: always in bounds.
    T av[KP];
#pragma unroll
    for (int i = 0; i < KP; ++i) av[i] = P[rowbase + i];
    T y = act ? rhs_l[jr] : T(0);

    T dinv = T(0), z = T(0);     // lane p: 1/L[p][p] and the forward solution z_p
    T rs_cur, l;
    {
        T d;
        pivot(bcast(av[0], 0), d, rs_cur);
        l = av[0] * rs_cur;       // lane 0 gets ~L[0][0]; lanes > 0 L[j][0]
        av[0] = l;
    }
    static_for<0, KP>([&](auto P_) {
        constexpr int p = decltype(P_)::value;
        // forward substitution with column p: z_p = y_p / L[p][p]; y_j -= L[j][p] z_p (lanes > p; lane p
        // and lanes < p update registers they no longer need)
        const T zp = bcast(y, p) * rs_cur;
        const bool me = opaque(j) == p;
        z = me ? zp : z;
        dinv = me ? rs_cur : dinv;
        y -= l * zp;
        // look-ahead columns p+1, p+2 through v_readlane: the next pivots never wait on LDS
        if constexpr (p + 1 < KP) av[p + 1] -= bcast(l, p + 1) * l;
        if constexpr (p + 2 < KP) av[p + 2] -= bcast(l, p + 2) * l;
        // next pivot (p+1): lane p+1 gets ~L[p+1][p+1], lanes > p+1 L[j][p+1]
        T l_next = T(0), rs_next = T(0);
        if constexpr (p + 1 < KP) {
            T d;
            pivot(bcast(av[p + 1], p + 1), d, rs_next);
            l_next = av[p + 1] * rs_next;
            av[p + 1] = l_next;
        }
        // bulk trailing update of columns >= p+3: L[i][p] broadcast through LDS, 16 B per read,
        // double-buffered so that reads of the next chunk are in flight under this chunk's FMAs
        if constexpr (p + 3 < KP) {
            wave_sync();
            if (act) bc[j] = l;
            wave_sync();
            constexpr int CH = 4;                              // 16-B vectors per chunk
            constexpr int q0 = ((p + 3) / BN) * BN;
            constexpr int nvec = (KP - q0) / BN;
            constexpr int nch = (nvec + CH - 1) / CH;
            BV buf[2][CH];
            static_for<0, (CH < nvec ? CH : nvec)>([&](auto V_) {
                constexpr int v = decltype(V_)::value;
                buf[0][v] = *(const BV*)(bc + q0 + v * BN);
            });
            static_for<0, nch>([&](auto C_) {
                constexpr int c = decltype(C_)::value;
                if constexpr (c + 1 < nch) {
                    static_for<0, CH>([&](auto V_) {
                        constexpr int v = decltype(V_)::value;
                        if constexpr ((c + 1) * CH + v < nvec)
                            buf[(c + 1) & 1][v] = *(const BV*)(bc + q0 + ((c + 1) * CH + v) * BN);
                    });
                }
                static_for<0, CH>([&](auto V_) {
                    constexpr int v = decltype(V_)::value;
                    if constexpr (c * CH + v < nvec) {
                        static_for<0, BN>([&](auto E_) {
                            constexpr int e = decltype(E_)::value;
                            constexpr int i = q0 + (c * CH + v) * BN + e;
                            if constexpr (i >= p + 3) av[i] -= buf[c & 1][v][e] * l;
                        });
                    }
                });
                __builtin_amdgcn_sched_barrier(0);
            });
        }
        static_for<p + 1, KP>([&](auto I_) { pin(av[decltype(I_)::value]); });
        l = l_next;
        rs_cur = rs_next;
        __builtin_amdgcn_sched_barrier(0);
    });
    // Transpose L through the packed triangle: lane j writes its row into ITS OWN segment only -- the
    // right-of-diagonal (garbage) entries i > j go to min(i, j) = the lane's diagonal slot, written before
    // the valid diagonal (descending i; same address, so program order holds). Then lane j reads column j.
    wave_sync();
    if (act) {
#pragma unroll
        for (int i = KP - 1; i >= 0; --i) P[rowbase + min(i, jr)] = av[i];
    }
    wave_sync();
#pragma unroll
    for (int i = 0; i < KP; ++i) av[i] = P[tri(i, 0) + jr];   // = L[i][j] for i >= j; garbage above
    // Backward substitution L^T x = z (column-oriented, p descending): x_p = z'_p / L[p][p],
    // z'_j -= L[p][j] x_p for j < p.
    T x = T(0);
#pragma unroll
    for (int p = KP - 1; p >= 0; --p) {
        const T xp = bcast(z, p) * bcast(dinv, p);
        x = (opaque(j) == p) ? xp : x;
        z -= av[p] * xp;
    }
    if (act) out[j] = (j < a.k) ? x : T(0);
}

// ---------------------------------------------------------------------------------------------------
// MFMA Gram path (fp32, KP = 16*C with C in {2, 4})
// ---------------------------------------------------------------------------------------------------
// Exact three-term bf16 split of two fp32 values, packed as bf16 pairs (element 0 = x0 in the low half):
// x = h + m + l with h = bf16_rn(x), m = bf16_rn(x - h), l = bf16_rn(x - h - m). Each residual is exact in
// fp32 and |m| <= 2^-9 |x|, |l| <= 2^-18 |x|, so the dropped partial products m*l, l*m, l*l of x*y are
// below 2^-26 |x y| -- under the fp32 rounding of the product itself -- and every bf16 x bf16 partial
// product is exact in the fp32 MFMA accumulation. 11 VALU instructions per pair.
__device__ __forceinline__ unsigned pk_bf16(float a, float b) {
    return __builtin_bit_cast(unsigned, __builtin_convertvector(f32x2{a, b}, bf16x2));
}
__device__ __forceinline__ void split3(float x0, float x1, unsigned& h, unsigned& m, unsigned& l) {
    h = pk_bf16(x0, x1);
    const float r0 = x0 - __uint_as_float(h << 16), r1 = x1 - __uint_as_float(h & 0xffff0000u);
    m = pk_bf16(r0, r1);
    const float s0 = r0 - __uint_as_float(m << 16), s1 = r1 - __uint_as_float(m & 0xffff0000u);
    l = pk_bf16(s0, s1);
}
__device__ __forceinline__ bf16x8 as_bf16x8(const u32x4& v) { return __builtin_bit_cast(bf16x8, v); }
// One 32-entry block of a bf16 partial product: D += A^T B over k = 32 (lane (g, i) element e <-> entry 8g + e).
__device__ __forceinline__ f32x4 mfma_k32(const u32x4& a, const u32x4& b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(as_bf16x8(a), as_bf16x8(b), c, 0, 0, 0);
}

// Two-term fp16 split of the pre-split tables (als_presplit): x' = x 2^s (s = split_exp of the table's largest |x|,
// so |x'| <= 2^14), h = f16_rn(x'), m = f16_rn(x' - h). x' - h is exact in fp32 and |x' - h - m| <= 2^-22 |x'|, so
// h + m carries 22 significant bits of every value. A product is taken as hh + hm + mh (the dropped mm and the
// representation error are <= 3 2^-22 |x'y'|); every fp16 x fp16 partial product is exact in the fp32 MFMA
// accumulation. Against the three-term bf16 split (six products) this halves the Gram MFMAs. Its accuracy, with the
// rest of the solve exact: per-row error 0.07-0.08x the reference's own fp32 EJML error on every test block, equal
// to rounding the inputs to fp32; the fp32 solve, not the Gram, sets the error.
typedef _Float16 f16x2 __attribute__((ext_vector_type(2)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
__device__ __forceinline__ void split2(float x0, float x1, unsigned& h, unsigned& m) {
    const f16x2 hv = __builtin_convertvector(f32x2{x0, x1}, f16x2);
    const f32x2 hf = __builtin_convertvector(hv, f32x2);
    const f16x2 mv = __builtin_convertvector(f32x2{x0 - hf[0], x1 - hf[1]}, f16x2);
    h = __builtin_bit_cast(unsigned, hv);
    m = __builtin_bit_cast(unsigned, mv);
}
__device__ __forceinline__ f32x4 mfma_f16(const u32x4& a, const u32x4& b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(f16x8, a), __builtin_bit_cast(f16x8, b), c, 0, 0,
                                                  0);
}
// Scale exponent s of a pre-split table from the bits of its largest |x| (als_absmax): 2^s max|x| <= 2^14 < the fp16
// maximum 65504 (no overflow at any rounding), and the table's values use the whole fp16 range (m stays normal for
// |x| >= 2^-17 max|x|). A zero, infinite or NaN maximum keeps s = 0; s is clamped so 2^s and 2^-2s stay usable.
__device__ __forceinline__ int split_exp(uint32_t maxbits) {
    if (maxbits == 0 || maxbits >= 0x7f800000u) return 0;
    int e = (int)(maxbits >> 23) - 127;          // max in [2^e, 2^(e+1)) (normal)
    if (e == -127) e = -126;                     // subnormal maximum
    else if (maxbits & 0x7fffffu) e += 1;        // e = ceil(log2(max))
    const int s = 14 - e;
    return s < -100 ? -100 : (s > 100 ? 100 : s);
}
// Close a group of v_mfma_f32_16x16x32_bf16: the compiler lets VALU instructions overwrite an MFMA's
// A/B/C registers one instruction after it (it models the operands as read at issue), which on gfx950
// intermittently corrupted the Gram (found as run-to-run differences in ~0.1% of rows, tools/determinism.py).
// Every split step therefore issues its MFMAs as one group (sched_barrier before it) and ends it with 16
// wait states before any later instruction may touch the operand registers: bitwise deterministic, same speed.
#ifndef CFK_DRAIN_NOPS
#define CFK_DRAIN_NOPS 2
#endif
#define MFMA_DRAIN()                                                          \
    do {                                                                      \
        __builtin_amdgcn_sched_barrier(0);                                    \
        static_for<0, CFK_DRAIN_NOPS>([&](auto) { asm volatile("s_nop 7"); }); \
        __builtin_amdgcn_sched_barrier(0);                                    \
    } while (0)
// RHS of the on-the-fly split path: computed before its block's MFMA group and materialised there. Computed
// after it (and with SLP-vectorised packed-fp32 VALU), LLVM deferred the RHS products into v_pk_mul /
// v_pk_add_f32 chains next to the next block's MFMAs, and on gfx950 that intermittently lost ~1/3 of RHS
// component 3 in lanes 48..63 of a wave (tools/split_diag.py: 5 of 5 captured failures had this signature;
// 9 wrong movie rows in 300 Netflix-shape halves). Both this and building the kernels without SLP
// vectorisation (Makefile) remove it (0 in 300 halves each).

template <int C>
struct MfmaAcc {
    static constexpr int NT = C * (C + 1) / 2;     // upper-triangular tiles (b1 <= b2)
    static constexpr int NWORDS = NT * 4 + C;       // per-lane words of one partial slot
    f32x4 g[NT];
    float rhs[C];
};

template <int C>
__host__ __device__ constexpr int tile_index(int b1, int b2) { return b1 * C - (b1 * (b1 - 1)) / 2 + (b2 - b1); }

// Diagonal tiles of the split Gram: hm + mh = X + X^T and hl + lh = Y + Y^T with X = h m^T, Y = h l^T, so the
// split paths accumulate X + Y per diagonal tile in E (2 MFMAs instead of 4 per block) and fold
// G_bb += E_b + E_b^T once per task: 8 of the 60 Gram MFMAs per block saved.

// G_bb += E_b + E_b^T. E^T via v_mfma_f32_16x16x4_f32 against the identity: with both operands in accumulator
// layout the four k-slices compute D += E^T I (see solve_tiles), each output one exact product plus C.
template <int C>
__device__ __forceinline__ void fold_diag(MfmaAcc<C>& acc, f32x4 (&E)[C], int lane) {
    f32x4 I;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        float v = ((lane >> 4) * 4 + r == (lane & 15)) ? 1.f : 0.f;
        pin(v);
        I[r] = v;
    }
    f32x4 D[C];
#pragma unroll
    for (int b = 0; b < C; ++b)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            float v = acc.g[tile_index<C>(b, b)][r] + E[b][r];
            float e = E[b][r];
            pin(v);
            pin(e);
            D[b][r] = v;
            E[b][r] = e;
        }
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int b = 0; b < C; ++b) {
        f32x4 t = D[b];
#pragma unroll
        for (int s = 0; s < 4; ++s) t = __builtin_amdgcn_mfma_f32_16x16x4f32(E[b][s], I[s], t, 0, 0, 0);
        acc.g[tile_index<C>(b, b)] = t;
    }
    MFMA_DRAIN();
}

// The same fold with E^T read back transposed from the wave's free LDS image (the pre-split Gram's) instead of 4 C
// v_mfma_f32_16x16x4_f32 against the identity: (acc + E) + E^T in the same order, bitwise the MFMA fold (each of its
// outputs is one exact product plus zeros). The pre-split path uses it (k = 64 / 128 user half -1.6 / -1.8 % in three
// interleaved rounds, profiles/r05e/e26_*.log). Bank-conflict-free image (round 6): lane (g, c) stores its column
// piece E[4g .. 4g+3][c] as one ds_write_b128 at dword 20 c + 4 g of its tile's 1280-B region, so the eight lanes of
// every b128 write group cover the 32 banks once; lane (g, c) then reads E[c][4g + r] with ds_read_b32 at dword
// 20 (4g + r) + 4 (c >> 2) + (c & 3) = 80 g + 20 r + c: 32 distinct banks per 32-lane group. (Round 5 read a
// 16-dword-stride image: 4-way conflicts, SQ_LDS_BANK_CONFLICT 0.118 of the user launch's LDS cycles.)
constexpr int FOLD_TILE_BYTES = 1280;
template <int C>
__device__ __forceinline__ void fold_diag_lds(MfmaAcc<C>& acc, const f32x4 (&E)[C], int lane, unsigned char* img) {
    static_assert(C * FOLD_TILE_BYTES <= 2 * C * 1024, "fold image within the wave's LDS-DMA image");
    const int g = lane >> 4, c = lane & 15;
#pragma unroll
    for (int b = 0; b < C; ++b) *(f32x4*)(img + b * FOLD_TILE_BYTES + (20 * c + 4 * g) * 4) = E[b];
    wave_sync();
    const int rd = (80 * g + c) * 4;
#pragma unroll
    for (int b = 0; b < C; ++b) {
        f32x4 t = acc.g[tile_index<C>(b, b)];
#pragma unroll
        for (int r = 0; r < 4; ++r)
            t[r] = (t[r] + E[b][r]) + *(const float*)(img + b * FOLD_TILE_BYTES + rd + r * 80);
        acc.g[tile_index<C>(b, b)] = t;
    }
    wave_sync();
}

// ---------------------------------------------------------------------------------------------------
// Cross-lane moves on the 4 x 16 lane grid (row g = lane >> 4, column c = lane & 15), VALU-only (no LDS)
// ---------------------------------------------------------------------------------------------------
// value of lane (g, L) at every lane of row g (DPP row_newbcast)
template <int L>
__device__ __forceinline__ float row_lane_bcast(float v) {
    return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x150 + L, 0xf, 0xf, false));
}
// value of lane (G, c) at every lane (g, c): one ds_bpermute through the LDS crossbar (no LDS storage).
// Measured 3-5% faster on the solve-heavy user half than the v_permlane16/32_swap pair it replaced (the
// swaps clobber both operands, which cost register copies and hazard NOPs on every sweep step).
template <int G>
__device__ __forceinline__ float col_bcast(float v) {
    const int addr = ((int)(__lane_id() & 15) + 16 * G) * 4;
    return __int_as_float(__builtin_amdgcn_ds_bpermute(addr, __float_as_int(v)));
}

// sum over the 4 rows at each column, result in every row
__device__ __forceinline__ float col_sum(float v) {
    const int x = __float_as_int(v);
    const auto s16 = __builtin_amdgcn_permlane16_swap(x, x, false, false);
    const float y = __int_as_float((int)s16[0]) + __int_as_float((int)s16[1]);
    const auto s32 = __builtin_amdgcn_permlane32_swap(__float_as_int(y), __float_as_int(y), false, false);
    return __int_as_float((int)s32[0]) + __int_as_float((int)s32[1]);
}
// inclusive row_shr scan: lane (g, 15) ends with the sum over row g
__device__ __forceinline__ float row_sum_to_last(float v) {
    v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x111, 0xf, 0xf, true));
    v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x112, 0xf, 0xf, true));
    v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x114, 0xf, 0xf, true));
    v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x118, 0xf, 0xf, true));
    return v;
}

// Sweep operator (Goodnight) over all 16 pivots of one 16 x 16 tile in MFMA accumulator layout
// (lane (g, c), register r holds a[4g + r][c]): in place a -> -a^{-1}. Step p:
//   a[i][j] -= a[i][p] a[p][j] / d,  a[i][p] = a[i][p] / d,  a[p][j] = a[p][j] / d,  a[p][p] = -1 / d.
// Column p reaches each row by DPP row_newbcast, row p each column by two permlane swaps. The pivot row /
// column rules fold into the same four FMAs by offsetting a[p][p] by -1 in the broadcast operands:
// a[i][p] + a[i][p] (d - 1)(-1/d) = a[i][p] / d. That FMA is accurate to a few ulp only while d <= 1,
// which the caller guarantees by Jacobi-scaling the system to a unit diagonal (every later pivot is a
// Schur-complement diagonal of a unit-diagonal SPD matrix, so it stays in (0, 1]).
// The four row broadcasts are fused into the FMAs (v_fmac_f32_dpp row_newbcast, one instruction per register
// instead of a v_mov_b32_dpp + v_fmac_f32 pair; k = 64 / 128 user half -3 %, profiles/r05e/e18_*.log).
// A DPP read of a VGPR needs 2 wait states after a VALU write of it, and the compiler's hazard recognizer does not
// see VALU writes inside inline asm: the block waits 2 states before its first DPP read (the previous step's writes)
// and after its last write (a compiler-placed DPP or lane op reading the results next).
template <int L>
__device__ __forceinline__ void fmac_rowbcast4(f32x4& a, float t) {
    float a0 = a[0], a1 = a[1], a2 = a[2], a3 = a[3];
    asm("s_nop 1\n\t"
        "v_fmac_f32_dpp %0, %0, %4 row_newbcast:%5 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f32_dpp %1, %1, %4 row_newbcast:%5 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f32_dpp %2, %2, %4 row_newbcast:%5 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f32_dpp %3, %3, %4 row_newbcast:%5 row_mask:0xf bank_mask:0xf\n\t"
        "s_nop 1"
        : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3)
        : "v"(t), "i"(L));
    a[0] = a0;
    a[1] = a1;
    a[2] = a2;
    a[3] = a3;
}
// lane L ? x : v with the lane mask a scalar constant (s_mov): the compiler's select re-derived the mask by a
// v_cmp at every pivot step (one vector instruction, and a 2-state hazard before the v_cndmask reading it).
// AFTER_DPP: ends with the 2 wait states a following DPP read of the result needs (see fmac_rowbcast4).
template <int L, bool AFTER_DPP>
__device__ __forceinline__ float select_lane(float v, float x) {
    float r;
    if constexpr (AFTER_DPP)
        asm("v_cndmask_b32_e64 %0, %1, %2, %3\n\ts_nop 1" : "=v"(r) : "v"(v), "v"(x), "s"((uint64_t)1 << L));
    else
        asm("v_cndmask_b32_e64 %0, %1, %2, %3" : "=v"(r) : "v"(v), "v"(x), "s"((uint64_t)1 << L));
    return r;
}
template <int p>
__device__ __forceinline__ void sweep_step(f32x4& a, int lane, float& nrd_min) {
    constexpr int pg = p >> 2, pr = p & 3;
    const float nrd = __builtin_amdgcn_rcpf(-bcast(a[pr], 16 * pg + p));   // -1 / d
    nrd_min = fminf(nrd_min, nrd);                                          // -1 / (smallest pivot)
    // the pivot lane's d - 1 (read next by v_readlane / ds_bpermute / the DPP block, which waits its own 2 states)
    a[pr] = select_lane<16 * pg + p, false>(a[pr], a[pr] - 1.f);
    const float t = col_bcast<pg>(a[pr]) * nrd;   // a[p][c] (d - 1 at c = p) * (-1/d)
    fmac_rowbcast4<p>(a, t);                       // a[4g + r][c] += a[4g + r][p] t[c]
    a[pr] = select_lane<16 * pg + p, true>(a[pr], nrd);
    (void)lane;
}
__device__ __forceinline__ void sweep_tile(f32x4& a, int lane, float& nrd_min) {
    static_for<0, 16>([&](auto P_) { sweep_step<decltype(P_)::value>(a, lane, nrd_min); });
}

// D + X^T Y of two 16 x 16 tiles in accumulator layout (the solve's block products): four v_mfma_f32_16x16x4_f32
// (exact fp32 products, 128 MFMA cycles)
__device__ __forceinline__ f32x4 tile_tn(const f32x4& X, const f32x4& Y, f32x4 D) {
#pragma unroll
    for (int s = 0; s < 4; ++s) D = __builtin_amdgcn_mfma_f32_16x16x4f32(X[s], Y[s], D, 0, 0, 0);
    return D;
}

// Lookahead schedule of the block factorisation: step P first finishes block column P + 1
// (V'_{P,P+1} and the update of T_{P+1,P+1}), so the 16-step sweep of T_{P+1,P+1} -- a dependent chain of
// broadcasts, latency-bound -- can start at once, and the rest of step P's MFMA work (block columns J >= P + 2) is
// issued between its steps. Items of step P, J descending, per J: V'_PJ = S_P T_PJ, then T_IJ += T_PI^T V'_PJ for
// I = P + 1 .. J (the same single update per tile as the plain order: bitwise equal results).
__host__ __device__ constexpr int la_items(int C, int P) {
    int n = 0;
    for (int J = C - 1; J >= P + 2; --J) n += 1 + (J - P);
    return n;
}
__host__ __device__ constexpr int la_item_J(int C, int P, int t) {
    for (int J = C - 1; J >= P + 2; --J) {
        if (t < 1 + J - P) return J;
        t -= 1 + J - P;
    }
    return -1;
}
__host__ __device__ constexpr int la_item_I(int C, int P, int t) {   // -1: the V'_PJ item of its J
    for (int J = C - 1; J >= P + 2; --J) {
        if (t < 1 + J - P) return t == 0 ? -1 : P + t;
        t -= 1 + J - P;
    }
    return -2;
}
// waves per SIMD of the pre-split KP = 64 kernel (register budget 512 / waves; LDS 16 x 8.25 KB at 4; 3 waves:
// 3.05 vs 2.83 ms user half, profiles/r05e/ab_k64_waves4_vs_3.log)
constexpr int PS64_WAVES = 4;

// Block LDL^T solve on the Gram tiles left in the MFMA accumulators (no LDS copy of the matrix).
// With C = KP/16 the accumulators hold G' = P G P^T (feature f = C*i + b at position 16*b + i) as upper
// tiles T_IJ (I <= J) in accumulator layout; MFMA operands read straight from those registers because for
// 16x16x4 the A/B slice s of lane (g, c) is "register s" of a tile read as X[4g+s][c] -- the k index runs
// over the rows of the tile, which is exactly what T_PI^T V and A^{-1} T need. Per block column P:
//   S = sweep(T_PP) = -T_PP^{-1};  V'_PJ = S T_PJ (= -T_PP^{-1} T_PJ);  T_IJ += T_PI^T V'_PJ (P < I <= J);
//   forward  b_I += V'_PI^T b_P,  u_P = S b_P;  backward  x_P = -u_P + sum_{I>P} V'_PI x_I.
// The explicit block inverses cost accuracy on ill-conditioned diagonal blocks (forward error grows with
// cond(T_PP), not just cond(A)), so the solve ends with one step of iterative refinement against the
// (scaled, regularised) Gram kept in registers: r = b - A x, x += solve(r). That brings the fp32 error
// below the reference's own fp32 LU (tests/test_gpu_parity.py). Vectors are held "lane (g, j) = element j"
// of each block; buf is KP floats of per-wave LDS.
// Tile storage of the solve. Up to KP = 64 the tiles stay in the MFMA accumulator registers (RegTiles), and so do
// they at KP = 128 on the pre-split path, which keeps no copy of the system (RowResidual); the other KP = 128 paths
// (36 tiles = 144 registers per copy, plus the kept copy) hold the working tiles in per-wave LDS ([tile][lane][reg]),
// loaded a tile at a time (LdsTiles).
template <int C>
struct RegTiles {
    f32x4* t;
    __device__ __forceinline__ f32x4 get(int i) const { return t[i]; }
    __device__ __forceinline__ void put(int i, const f32x4& v) { t[i] = v; }
};
template <int C>
struct RegStore {
    f32x4 t[MfmaAcc<C>::NT];
    __device__ __forceinline__ f32x4 get(int i) const { return t[i]; }
    __device__ __forceinline__ void put(int i, const f32x4& v) { t[i] = v; }
};
// KP = 128 working tiles: [tile][lane][reg] so a tile moves with one ds_read_b128 / ds_write_b128 per lane
// (kbench, k = 128: user half 23.3 -> 20.5 ms against a [tile][reg][lane] b32 layout, at the cost of 3 VGPR spills)
struct LdsTiles {
    float* p;   // per-wave base + 4 * lane
    __device__ __forceinline__ f32x4 get(int i) const { return *(const f32x4*)(p + i * 256); }
    __device__ __forceinline__ void put(int i, const f32x4& v) { *(f32x4*)(p + i * 256) = v; }
};
template <int C>
constexpr bool tiles_in_lds() { return C > 4; }
template <int C>
constexpr int tile_lds_floats() { return tiles_in_lds<C>() ? MfmaAcc<C>::NT * 4 * 64 : 0; }

// Logical in-block entry index of physical position q of a row's padded range (inverse of block_position).
__device__ __forceinline__ int logical_entry(int q) {
    const int w = q % BLOCK_ENTRIES;
    return q - w + (w % BLOCK_SUBSTEPS) * 4 + w / BLOCK_SUBSTEPS;
}

// Tag for solve_tiles' A0: keep NO copy of the system; a refinement step (rare: every Netflix-shape user row passes
// the pivot gate, tools/refine_accuracy.py) forms its residual from the factor rows instead, r = b - D (G (D x) +
// lambda n D x) with G z = sum_e y_e (y_e . z) over the row's entries. G z uses the exact fp32 rows; b is the RHS
// the Gram pass accumulated, which on the pre-split path comes from the split (h + m) values, so the step corrects
// the Gram's 2^-22 representation error but not the RHS's. Frees the copy's registers (4 waves per SIMD on the
// pre-split KP = 64 path instead of 3).
struct RowResidual {
    __device__ __forceinline__ void put(int, const f32x4&) {}
};

// T: working tiles (RegTiles / LdsTiles), A0: kept copy of the scaled system (RegStore / LdsTiles), or RowResidual.
// DUAL: the system is the entry Gram of a short row (als_solve_dual): unknown 16b + j = the row's entry at
// physical position 16b + j, real when that entry exists (padding entries get an identity row), and the
// solution alpha goes to buf[16b + j] (read by the caller after a wave_sync) instead of a factor row.
// u: the units of the tiles and the RHS -- the Gram terms are u^2 times the true ones and the RHS u times (the
// pre-split Gram's table scale; 1 elsewhere). A' = D A D and D b do not depend on u (D scales by 1/u), so the
// factorisation and the scaled solution are the same; the regularisation is added as lambda n u^2 and the solution
// leaves in true units as D x' u.
template <int C, bool DUAL = false, class TT, class KT>
__device__ __forceinline__ void solve_tiles(TT& T, KT& A0, const float (&rhs_acc)[C], float* buf, const Task& tk,
                                            const SolveArgs& a, int lane, float u = 1.f) {
    const int g = lane >> 4, j = lane & 15;
    float* out = (float*)a.out + factor_row(a.row_offset, a.rows_per_chunk, a.chunk_stride, tk.row) * (int64_t)(16 * C);
    auto is_real = [&](int b) { return DUAL ? logical_entry(16 * b + j) < tk.nent : C * j + b < a.k; };
    auto emit = [&](const float (&xs)[C]) {   // xs = solution in the scaled variables, times scol
        if constexpr (DUAL) {
            wave_sync();
            if (g == 0) {
#pragma unroll
                for (int b = 0; b < C; ++b) buf[16 * b + j] = is_real(b) ? xs[b] : 0.f;
            }
        } else if (g == 0) {
            using VT = typename VecC<C>::type;
            VT o;
#pragma unroll
            for (int b = 0; b < C; ++b) o[b] = is_real(b) ? xs[b] : 0.f;
            *(VT*)(out + C * j) = o;
        }
    };
    if (tk.ndeg == 0) {   // cannot occur in the reference (entities exist only once rated); defined as 0
        if (DUAL) {
            float z[C] = {};
            emit(z);
        } else if (g == 0) {
#pragma unroll
            for (int b = 0; b < C; ++b) out[C * j + b] = 0.f;
        }
        return;
    }
    // A + lambda * (n * I) (fp32, MFeatureCalculator.java:91-95: A[f][f] + lambda*(float)n); padded features
    // get an identity row (their Gram rows/columns are exactly zero: padded factor columns are zero).
    // Then Jacobi scaling A' = D A D, b' = D b, x = D x' with D = diag(A)^{-1/2}: lane (g, j) of block b
    // needs s for column j (scol) and for rows 4g..4g+3 (srow), exchanged through buf.
    const float reg = a.lambda * (float)tk.ndeg * (u * u);
    const int jr = j & 3;
    const bool diag_lane = opaque(j >> 2) == g;   // lane holds a diagonal entry, in register j & 3
    float scol[C];
#pragma unroll
    for (int b = 0; b < C; ++b) {
        f32x4 t = T.get(tile_index<C>(b, b));
        const bool real = is_real(b);
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const bool diag = diag_lane && jr == r;
            t[r] = diag ? (real ? t[r] + reg : 1.f) : t[r];
        }
        T.put(tile_index<C>(b, b), t);
        float dv = t[0];
#pragma unroll
        for (int r = 1; r < 4; ++r) dv = (jr == r) ? t[r] : dv;
        if (diag_lane) buf[16 * b + j] = __builtin_amdgcn_rsqf(dv);
    }
    wave_sync();
#pragma unroll
    for (int b = 0; b < C; ++b) scol[b] = buf[16 * b + j];
#pragma unroll
    for (int I = 0; I < C; ++I) {
        const f32x4 srow = *(const f32x4*)(buf + 16 * I + 4 * g);   // s for rows 4g .. 4g + 3 of block I
#pragma unroll
        for (int J = I; J < C; ++J) {
            f32x4 t = T.get(tile_index<C>(I, J));
#pragma unroll
            for (int r = 0; r < 4; ++r) t[r] *= srow[r] * scol[J];
            T.put(tile_index<C>(I, J), t);
            A0.put(tile_index<C>(I, J), t);
        }
    }
    wave_sync();
    float b0[C];
#pragma unroll
    for (int b = 0; b < C; ++b) b0[b] = col_sum(rhs_acc[b]) * scol[b];

    // ---- factorisation (matrix part only), lookahead schedule ----
    float nrd_min = -1.f;
    {
        {
            f32x4 S0 = T.get(tile_index<C>(0, 0));
            sweep_tile(S0, lane, nrd_min);
            T.put(tile_index<C>(0, 0), S0);
        }
        static_for<0, C - 1>([&](auto P_) {
            constexpr int P = decltype(P_)::value;
            const f32x4 S = T.get(tile_index<C>(P, P));   // -T_PP^{-1}
            const f32x4 orig = T.get(tile_index<C>(P, P + 1));
            const f32x4 v1 = tile_tn(S, orig, f32x4{0.f, 0.f, 0.f, 0.f});
            f32x4 D = tile_tn(orig, v1, T.get(tile_index<C>(P + 1, P + 1)));
            T.put(tile_index<C>(P, P + 1), v1);
            constexpr int m = la_items(C, P);
            f32x4 vcur = {0.f, 0.f, 0.f, 0.f};
            auto item = [&](auto T_) {
                constexpr int t = decltype(T_)::value;
                constexpr int J = la_item_J(C, P, t), I = la_item_I(C, P, t);
                if constexpr (I < 0) {
                    vcur = tile_tn(S, T.get(tile_index<C>(P, J)), f32x4{0.f, 0.f, 0.f, 0.f});
                } else {
                    // T_PI: I = P + 1 was replaced by V'_{P,P+1} above (orig keeps it); P + 1 < I <= J is still the
                    // original (replaced only when its own, later, J group ends)
                    const f32x4 TPI = (I == P + 1) ? orig : T.get(tile_index<C>(P, I));
                    T.put(tile_index<C>(I, J), tile_tn(TPI, vcur, T.get(tile_index<C>(I, J))));
                    if constexpr (I == J) T.put(tile_index<C>(P, J), vcur);   // block row P now holds V'_PJ
                }
            };
            // the sweep of T_{P+1,P+1} with step P's remaining items between its 16 pivot steps
            static_for<0, 16>([&](auto Q_) {
                constexpr int q = decltype(Q_)::value;
                sweep_step<q>(D, lane, nrd_min);
                static_for<q * m / 16, (q + 1) * m / 16>(item);
            });
            T.put(tile_index<C>(P + 1, P + 1), D);
        });
    }

    // ---- x = A^{-1} rhs with the factorisation ----
    auto solve_vec = [&](const float (&rhs)[C], float (&x)[C]) {
        float bw[C], u[C];
#pragma unroll
        for (int b = 0; b < C; ++b) bw[b] = rhs[b];
        static_for<0, C>([&](auto P_) {
            constexpr int P = decltype(P_)::value;
            const f32x4 S = T.get(tile_index<C>(P, P));
            wave_sync();
            if (g == 0) buf[j] = bw[P];           // b_P[4g + r] into every lane of row g
            wave_sync();
            const f32x4 bb = *(const f32x4*)(buf + 4 * g);
            float su = 0.f;
#pragma unroll
            for (int r = 0; r < 4; ++r) su += S[r] * bb[r];
            u[P] = col_sum(su);
            static_for<P + 1, C>([&](auto I_) {
                constexpr int I = decltype(I_)::value;
                const f32x4 V = T.get(tile_index<C>(P, I));
                float sb = 0.f;
#pragma unroll
                for (int r = 0; r < 4; ++r) sb += V[r] * bb[r];
                bw[I] += col_sum(sb);
            });
        });
        static_for<0, C>([&](auto Q_) {
            constexpr int P = C - 1 - decltype(Q_)::value;
            if constexpr (P == C - 1) {
                x[P] = -u[P];
            } else {
                f32x4 w = {0.f, 0.f, 0.f, 0.f};
                static_for<P + 1, C>([&](auto I_) {
                    constexpr int I = decltype(I_)::value;
                    const f32x4 V = T.get(tile_index<C>(P, I));
#pragma unroll
                    for (int r = 0; r < 4; ++r) w[r] += V[r] * x[I];
                });
#pragma unroll
                for (int r = 0; r < 4; ++r) w[r] = row_sum_to_last(w[r]);
                wave_sync();
                if (j == 15) *(f32x4*)(buf + 4 * g) = w;
                wave_sync();
                x[P] = buf[j] - u[P];
            }
        });
    };
    float x[C];
    solve_vec(b0, x);
    // Well-conditioned systems skip the refinement step: every pivot of the scaled (unit-diagonal) system is a
    // Schur-complement diagonal in (0, 1]; when the smallest is >= a.refine_min_pivot the block factorisation's
    // error is already below the reference's own fp32 LU error. The test is wave-uniform.
    if (-1.f / nrd_min >= a.refine_min_pivot) {
        float xs[C];
#pragma unroll
        for (int b = 0; b < C; ++b) xs[b] = x[b] * scol[b] * u;
        emit(xs);
        return;
    }
    if (a.flags & SOLVE_FLAG_SKIP_REFINE) {   // diagnostics only
        float xs[C];
#pragma unroll
        for (int b = 0; b < C; ++b) xs[b] = x[b] * scol[b] * u;
        emit(xs);
        return;
    }

    // ---- one refinement step: r = b - A x, x += A^{-1} r ----
    float r[C];
    if constexpr (std::is_same<KT, RowResidual>::value) {
        static_assert(!DUAL, "row residual: primal systems only");
        // z = D x (lane (g, j), block b: feature C j + b, the layout of a C-float piece of a factor row)
        float z[C], acc[C];
#pragma unroll
        for (int b = 0; b < C; ++b) {
            z[b] = x[b] * scol[b] * u;   // true units
            acc[b] = 0.f;
        }
        using VT = typename VecC<C>::type;
        typedef int i32x4 __attribute__((ext_vector_type(4)));
        const char* obase = (const char*)a.opp + (uint32_t)(C * j * sizeof(float));
        const int32_t* cb = a.col + tk.begin + 8 * g;   // group g: physical entries 8 g .. 8 g + 7 of each block
        const int nblk = (tk.nsteps + BLOCK_SUBSTEPS - 1) / BLOCK_SUBSTEPS;
        for (int blk = 0; blk < nblk; ++blk) {
            const i32x4 c0 = *(const i32x4*)(cb + blk * BLOCK_ENTRIES);
            const i32x4 c1 = *(const i32x4*)(cb + blk * BLOCK_ENTRIES + 4);
#pragma unroll
            for (int t = 0; t < 8; ++t) {   // padding entries read the zero sentinel row
                const uint32_t row = (uint32_t)(t < 4 ? c0[t] : c1[t - 4]);
                const VT y = *(const VT*)(obase + row * (uint32_t)(16 * C * sizeof(float)));
                float p = 0.f;
#pragma unroll
                for (int b = 0; b < C; ++b) p += y[b] * z[b];
                p = row_lane_bcast<15>(row_sum_to_last(p));   // y_e . z over the 16 lanes of the row group
#pragma unroll
                for (int b = 0; b < C; ++b) acc[b] += y[b] * p;
            }
        }
        const float reg = a.lambda * (float)tk.ndeg;
#pragma unroll
        for (int b = 0; b < C; ++b) {
            const float gz = col_sum(acc[b]);
            r[b] = b0[b] - (is_real(b) ? scol[b] * u * (gz + reg * z[b]) : x[b]);   // padded features: identity rows
        }
    } else {
    wave_sync();
    if (g == 0) {
#pragma unroll
        for (int b = 0; b < C; ++b) buf[16 * b + j] = x[b];
    }
    wave_sync();
    f32x4 xr[C];                                   // x_b[4g + q] in row g
#pragma unroll
    for (int b = 0; b < C; ++b) xr[b] = *(const f32x4*)(buf + 16 * b + 4 * g);
    float res[C];
    f32x4 w[C];
#pragma unroll
    for (int b = 0; b < C; ++b) {
        res[b] = 0.f;
        w[b] = f32x4{0.f, 0.f, 0.f, 0.f};
    }
#pragma unroll
    for (int I = 0; I < C; ++I)
#pragma unroll
        for (int J = I; J < C; ++J) {
            const f32x4 t = A0.get(tile_index<C>(I, J));
#pragma unroll
            for (int q = 0; q < 4; ++q) w[I][q] += t[q] * x[J];            // rows of block I
            if (I != J) {
                float s = 0.f;
#pragma unroll
                for (int q = 0; q < 4; ++q) s += t[q] * xr[I][q];          // (A_IJ^T x_I) at column c
                res[J] += s;
            }
        }
#pragma unroll
    for (int b = 0; b < C; ++b)
#pragma unroll
        for (int q = 0; q < 4; ++q) w[b][q] = row_sum_to_last(w[b][q]);
    wave_sync();
    if (j == 15) {
#pragma unroll
        for (int b = 0; b < C; ++b) *(f32x4*)(buf + 16 * b + 4 * g) = w[b];
    }
    wave_sync();
#pragma unroll
    for (int b = 0; b < C; ++b) r[b] = b0[b] - buf[16 * b + j] - (C > 1 ? col_sum(res[b]) : 0.f);
    }
    float dx[C];
    solve_vec(r, dx);
    float xs[C];
#pragma unroll
    for (int b = 0; b < C; ++b) xs[b] = (x[b] + dx[b]) * scol[b] * u;
    emit(xs);
}

// Waves (tasks) per workgroup of the MFMA kernel: 4, or 2 at KP = 128, whose 72 KB of per-wave LDS tiles
// allow two 2-wave workgroups per CU (one wave per SIMD, which its register use allows anyway).
template <int KP>
constexpr int mfma_waves() { return WAVES; }

// Range statistics of a table for the pre-split Gram, from the bits of |x| (non-negative floats order as unsigned
// integers): out[0] = the largest |x| (the split scale, split_exp), out[1] = ~(the smallest nonzero row maximum) (a
// max of complements is a min; 0 = no nonzero row). Grid-stride over 16-B vectors, vpr vectors per row (a row's
// vectors are consecutive lanes of one wave: the grid stride is a multiple of 64), workgroup reduction, one
// vector-memory atomicMax per workgroup and word. out[0..1] are zeroed before the launch.
__global__ __launch_bounds__(256) void als_absmax(const u32x4* __restrict__ src, int64_t n4, int vpr,
                                                  uint32_t* __restrict__ out) {
    uint32_t m = 0, rmin = 0xffffffffu;
    const int64_t stride = (int64_t)gridDim.x * 256;
    for (int64_t i0 = (int64_t)blockIdx.x * 256 + (threadIdx.x & ~63); i0 < n4; i0 += stride) {
        const int64_t i = i0 + (threadIdx.x & 63);
        uint32_t v = 0;
        if (i < n4) {
            const u32x4 x = src[i] & 0x7fffffffu;
            v = max(max(x[0], x[1]), max(x[2], x[3]));
        }
        m = max(m, v);
        for (int o = 1; o < vpr; o <<= 1) v = max(v, (uint32_t)__shfl_xor((int)v, o));   // the row's maximum
        if (v != 0 && i < n4) rmin = min(rmin, v);
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        m = max(m, (uint32_t)__shfl_xor((int)m, o));
        rmin = min(rmin, (uint32_t)__shfl_xor((int)rmin, o));
    }
    // one atomic per workgroup: thousands of same-address atomics serialise (53 us for the 4.5 MB M table)
    __shared__ uint32_t wm[4], wr[4];
    if ((threadIdx.x & 63) == 0) {
        wm[threadIdx.x >> 6] = m;
        wr[threadIdx.x >> 6] = rmin;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        m = max(max(wm[0], wm[1]), max(wm[2], wm[3]));
        rmin = min(min(wr[0], wr[1]), min(wr[2], wr[3]));
        if (m != 0) atomicMax(out, m);
        if (rmin != 0xffffffffu) atomicMax(out + 1, ~rmin);
    }
}
// The pre-split (table-wide scale, two fp16 terms) keeps ~22 significant bits for values within 2^-17 of the table's
// largest |x| and falls toward the fp16 subnormal floor below; it serves a half only when every nonzero row's
// maximum is within PRESPLIT_RANGE of the table's. Otherwise that half's Gram runs on the fp32 table with the
// on-the-fly three-term bf16 split (an 8-bit exponent per value): the pre-split kernels exit at once and the
// guarded on-the-fly launch after them does the work (SolveArgs::presplit_fallback).
constexpr float PRESPLIT_RANGE = 65536.f;
__device__ __forceinline__ bool presplit_ok(const uint32_t* st) {
    const uint32_t mx = st[0], rc = st[1];
    if (mx >= 0x7f800000u) return false;   // inf / NaN in the table: the fp32 path propagates it as the reference would
    if (rc == 0) return true;              // no nonzero row
    return __uint_as_float(mx) <= PRESPLIT_RANGE * __uint_as_float(~rc);
}

// fp32 table -> fp16 h/m planes (presplit_row_bytes(KP) per row, als_internal.h) at the table's scale 2^s: thread
// (row, b, jh) splits features C (8 jh + i) + b, i = 0..7, and writes 16 B per plane at plane position 16 b + 8 jh.
template <int KP>
__global__ __launch_bounds__(256) void als_presplit(const float* __restrict__ src, unsigned* __restrict__ dst,
                                                   int64_t n_threads, const uint32_t* __restrict__ amax) {
    constexpr int C = KP / 16;
    const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (t >= n_threads) return;
    const int sc = split_exp(*amax);
    const int64_t row = t / (2 * C);
    const int b = (int)(t % (2 * C)) >> 1, jh = (int)(t & 1);
    const float* s = src + row * KP + C * 8 * jh + b;
    u32x4 h, m;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        unsigned hh, mm;
        split2(ldexpf(s[C * (2 * i)], sc), ldexpf(s[C * (2 * i + 1)], sc), hh, mm);
        h[i] = hh;
        m[i] = mm;
    }
    unsigned* o = dst + row * (presplit_row_bytes(KP) / 4) + (16 * b + 8 * jh) / 2;
    *(u32x4*)o = h;
    *(u32x4*)(o + KP / 2) = m;   // plane stride 2 KP bytes
}
// In-block column indices in the order of the LDS-DMA gather: inside a 32-entry block, word 4 r + x (r = 0..7,
// x = 0..3) holds the column of entry k = 16 (x >> 1) + 8 (r >> 2) + 4 (x & 1) + (r & 3), so the 8 lanes of loader
// row r fetch the rows of their 4 DMA instructions with one 16-B load.
__global__ __launch_bounds__(256) void als_pack_cols_ps(const int32_t* __restrict__ col, int32_t* __restrict__ dst,
                                                       int64_t n) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    const int w = (int)(i & 31), r = w >> 2, x = w & 3;
    const int k = 16 * (x >> 1) + 8 * (r >> 2) + 4 * (x & 1) + (r & 3);
    dst[i] = col[(i & ~(int64_t)31) + k];
}

// A PARTIAL task's raw accumulators -> its partial slot ([word][lane], keyed words + check word, SlotCodec).
template <int C>
__device__ __forceinline__ void store_partial(const SolveArgs& a, const Task& tk, const MfmaAcc<C>& acc, int lane) {
    using Acc = MfmaAcc<C>;
    constexpr int SLOT_WORDS = Acc::NWORDS + 1;   // + integrity check word
    float* dst = (float*)a.partials + (int64_t)tk.slot * (SLOT_WORDS * 64) + lane;
    SlotCodec cd{slot_key(a.gen, tk.slot, lane)};
#pragma unroll
    for (int p = 0; p < Acc::NT; ++p)
#pragma unroll
        for (int r = 0; r < 4; ++r) dst[(p * 4 + r) * 64] = cd.enc(acc.g[p][r], p * 4 + r);
#pragma unroll
    for (int c = 0; c < C; ++c) dst[(Acc::NT * 4 + c) * 64] = cd.enc(acc.rhs[c], Acc::NT * 4 + c);
    dst[Acc::NWORDS * 64] = cd.check_word<float>(Acc::NWORDS);
}

// Pre-split fp16 Gram of one FULL / PARTIAL task into acc (tiles, RHS) and E (the diagonal tiles' h m^T terms,
// folded by the caller), in the table's scaled units: Gram terms times 2^(2 sc), the RHS times 2^sc; returns sc.
// The caller brings a PARTIAL task's sums back to true units for its slot and lets a FULL task's solve work in the
// scaled ones (solve_tiles' u: the scaled system is the same after the Jacobi scaling), which saves the 72 ldexp of
// the unscaling at KP = 64. img: the wave's 2 C KB LDS image (1-KB aligned); buf: its KP floats.
template <int KP>
__device__ __forceinline__ int gram_presplit(const SolveArgs& a, const Task& tk, MfmaAcc<KP / 16>& acc,
                                             f32x4 (&E)[KP / 16], unsigned char* img, float* buf, int lane) {
    constexpr int C = KP / 16;
    constexpr int B = BLOCK_SUBSTEPS;
    const int g = lane >> 4, j = lane & 15;
    const int nblk = (tk.nsteps + B - 1) / B;
    // Two-term fp16 Gram over a PRE-SPLIT opposite table (als_presplit, once per half: the scaled h/m fp16
    // terms of every factor row, split2). Tile (b1, b2) takes hh + hm + mh (3 MFMAs), a diagonal tile hh + E
    // with E = h m^T folded as E + E^T once per task (2 MFMAs). The RHS Y^T r is 2 MFMAs per feature block on
    // B[k][c] = rh_k (columns 0-7) / rm_k (columns 8-15), r = rh + rm exact in fp16 for every Java short:
    // column 0 + column 8 = Y_b^T r. KP = 64: 34 MFMAs per 32-entry block (the on-the-fly bf16 split: 52
    // + VALU RHS); KP = 128: 116 (200 + VALU RHS).
    static_assert(C == 4 || C == 8, "pre-split Gram: KP = 64 or 128");
    typedef int i32x4 __attribute__((ext_vector_type(4)));
    constexpr int NPL = 2;                 // planes h, m
    const char* tbase = (const char*)a.opp_split;
    const int sc = split_exp(*a.amax);     // the table's scale 2^sc (wave-uniform scalar load)
    f32x4 racc[C];
#pragma unroll
    for (int b = 0; b < C; ++b) racc[b] = f32x4{0.f, 0.f, 0.f, 0.f};
    // the block's MFMAs on operands P[plane h/m][feature block b] (entries 8g..8g+7 of feature C j + b as
    // fp16 pairs) and the fp16 rating pairs R of the same entries (rh or rm by the lane's column)
    // FIRST (the task's first block): every accumulator's first MFMA takes the inline constant 0 as its C operand,
    // so the 72 zeroing moves of the accumulators (KP = 64) are not needed on this path
    auto mfma_block = [&](const u32x4 (&P)[NPL][C], const u32x4& R, auto FIRST_) {
        constexpr bool FIRST = decltype(FIRST_)::value;
        const f32x4 zero = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int b1 = 0; b1 < C; ++b1)
#pragma unroll
            for (int b2 = b1; b2 < C; ++b2) {
                f32x4 t = FIRST ? zero : acc.g[tile_index<C>(b1, b2)];
                if (b1 == b2) {
                    E[b1] = mfma_f16(P[0][b1], P[1][b1], FIRST ? zero : E[b1]);
                } else {
                    t = mfma_f16(P[0][b1], P[1][b2], t);
                    t = mfma_f16(P[1][b1], P[0][b2], t);
                }
                t = mfma_f16(P[0][b1], P[0][b2], t);
                acc.g[tile_index<C>(b1, b2)] = t;
            }
#pragma unroll
        for (int b = 0; b < C; ++b) {
            f32x4 t = FIRST ? zero : racc[b];
            t = mfma_f16(P[1][b], R, t);
            t = mfma_f16(P[0][b], R, t);
            racc[b] = t;
        }
        MFMA_DRAIN();
    };
    // LDS image of one 32-entry block per wave (2 C KB: 8 KB at KP = 64, 16 KB at KP = 128): 2 C LDS-DMA
    // instructions (plane pl, 128-B plane half ph, entry quarter m) of 1 KB, instruction = 8 rows x one
    // 128-B half plane, lane 8 r + i holding 16-B chunk i ^ 2 (r >> 1) of the row of entry
    // k = 16 (m >> 1) + 8 (r >> 2) + 4 (m & 1) + (r & 3): whole cache lines per row for the address unit (8
    // lines per instruction), and a chunk swizzle that makes the transposed reads conflict-free. Operand
    // (pl, b) of lane (g, 4 q + p) = two ds_read_b64_tr_b16 (h = 0, 1: entries 8 g + 4 h + 0..3), lane
    // 4 q + p addressing entry 8 g + 4 h + q, plane positions 16 b + 4 p .. + 3 (features C j + b,
    // j = 4 p .. 4 p + 3); the 16 lanes of a group receive features j = 0..15 of their 4 entries: exactly
    // the MFMA A/B operand, no lane movement.
    typedef short s16x4 __attribute__((ext_vector_type(4)));
    typedef __attribute__((address_space(3))) void lds_void;
    typedef __attribute__((address_space(3))) s16x4 lds_s16x4;
    constexpr int NH = C / 4;              // 128-B halves per plane
    const int r8 = lane >> 3;
    const uint32_t ld_off = 16u * (uint32_t)((lane & 7) ^ (2 * (r8 >> 1)));
    const int q = (lane >> 2) & 3, p = lane & 3, rr = 4 * (g & 1) + q;
    uint32_t rd[4];   // per feature block b & 3 (the 128-B half b >> 2 is an immediate)
#pragma unroll
    for (int b = 0; b < 4; ++b)
        rd[b] = 2048u * (uint32_t)(g >> 1) + 16u * (uint32_t)(8 * rr + ((2 * b + (p >> 1)) ^ (2 * (rr >> 1)))) +
                8u * (uint32_t)(p & 1);
    // per-plane table bases kept in SGPRs (opaque to the optimiser: folded into the per-lane offset they
    // would force 64-bit addresses; an LDS-DMA takes no immediate offset here, it would move the LDS
    // destination too), so every DMA takes the saddr form with one 32-bit lane offset per row
    const char* tpl[NPL * NH];
#pragma unroll
    for (int x = 0; x < NPL * NH; ++x) {
        tpl[x] = tbase + (x / NH) * 2 * KP + (x % NH) * 128;
        asm volatile("" : "+s"(tpl[x]));
    }
    auto issue = [&](const i32x4& cv) {
        static_for<0, 4>([&](auto M_) {
            constexpr int m = decltype(M_)::value;
            // 24-bit multiply: pre-split tables are host-checked < 2^24 rows and < 4 GiB
            const uint32_t vo = __umul24((uint32_t)cv[m], (uint32_t)presplit_row_bytes(KP)) + ld_off;
            static_for<0, NPL * NH>([&](auto X_) {
                constexpr int x = decltype(X_)::value;   // plane x / NH, half x % NH
                __builtin_amdgcn_global_load_lds((const void*)(tpl[x] + vo),
                                                 (lds_void*)(img + (x * 4 + m) * 1024), 16, 0, 0);
            });
        });
    };
    auto read1 = [&](auto PL_, auto B_) {
        constexpr int pl = decltype(PL_)::value, b = decltype(B_)::value;
        u32x4 P;
        static_for<0, 2>([&](auto H_) {
            constexpr int h = decltype(H_)::value;
            const s16x4 v = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
                (lds_s16x4*)(img + rd[b & 3] + ((pl * NH + (b >> 2)) * 4 + h) * 1024));
            const u32x2 w = __builtin_bit_cast(u32x2, v);
            P[2 * h] = w[0];
            P[2 * h + 1] = w[1];
        });
        return P;
    };
    auto read = [&](u32x4 (&P)[NPL][C]) {
        static_for<0, NPL>([&](auto PL_) {
            static_for<0, C>([&](auto B_) { P[decltype(PL_)::value][decltype(B_)::value] = read1(PL_, B_); });
        });
    };
    if (nblk > 0) {
        const int lastb = nblk - 1;
        const i32x4* cp = (const i32x4*)(a.col_ps + tk.begin) + r8;          // + 8 per block
        // rating pairs of the lane's column half: rh (columns 0-7) or rm (columns 8-15)
        const u32x4* rp = (const u32x4*)(a.rat_pk + (j >= 8 ? a.rat_lo_off : 0) + (tk.begin >> 1)) + g;
        i32x4 cv = cp[0];
        u32x4 Rn = rp[0];
        issue(cv);
        cv = cp[8 * min(1, lastb)];
        auto step = [&](int b, auto FIRST_) {
            const u32x4 R = Rn;
            // every vector-memory op of this wave done: this block's LDS-DMA (and the column / rating loads
            // the DMA issue and the MFMAs below need anyway) -- explicit, not left to the compiler's tracking
            // of LDS-DMA writes (tests/test_isa_guard.py checks it)
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            u32x4 P[NPL][C];
            read(P);
            // the operands are in registers before the image is overwritten by the next block's DMA
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            if (b < lastb) issue(cv);
            cv = cp[8 * min(b + 2, lastb)];
            Rn = rp[4 * min(b + 1, lastb)];
            __builtin_amdgcn_sched_barrier(0);
            mfma_block(P, R, FIRST_);
            __builtin_amdgcn_sched_barrier(0);
        };
        step(0, std::true_type{});
        for (int b = 1; b < nblk; ++b) step(b, std::false_type{});
    }
    // RHS tiles (row i of block b = feature C i + b; column 0 = Y^T rh, column 8 = Y^T rm) -> the per-lane
    // partial layout of the other paths: lane (0, j) holds feature C j + b, the other rows zero (col_sum
    // restores it). The lane's (g, j) derived afresh (opaque): kept live across the Gram loop, one spilled.
    const int lane2 = opaque(lane), g2 = lane2 >> 4, j2 = lane2 & 15;
    wave_sync();
#pragma unroll
    for (int b = 0; b < C; ++b) {
        f32x4 v = racc[b];
#pragma unroll
        for (int r = 0; r < 4; ++r)   // lane (g, 8) += lane (g, 0): DPP row_shr:8
            v[r] += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v[r]), 0x118, 0xf, 0xf, false));
        if (j2 == 8) *(f32x4*)(buf + 16 * b + 4 * g2) = v;
    }
    wave_sync();
#pragma unroll
    for (int b = 0; b < C; ++b) acc.rhs[b] = (g2 == 0) ? buf[16 * b + j2] : 0.f;
    wave_sync();
    return sc;
}

// REDUCE = true: the launch of a half's REDUCE tasks (sum of partial slots + solve), compiled apart from the
// gather kernel so neither carries the other's code and registers.
// GRIDLOOP: a grid-stride loop over the tasks (the range guard's fallback launch, whose grid is capped: when the
// pre-split serves the half, as it nearly always does, its waves exit without a full-size grid's dispatch cost).
template <int KP, int MINW, bool SPLIT, bool PRESPLIT = false, bool REDUCE = false, bool GRIDLOOP = false>
__global__ __launch_bounds__(64 * mfma_waves<KP>(), MINW) void als_solve_mfma(SolveArgs a) {
    constexpr int C = KP / 16;
    constexpr int NW = mfma_waves<KP>();
    using Acc = MfmaAcc<C>;
    using VT = typename VecC<C>::type;
    __shared__ __attribute__((aligned(16))) float sbuf[NW][KP];
    // KP = 128 keeps the solve's working tiles in per-wave LDS, except on the pre-split path: its solve keeps no copy
    // of the system (RowResidual), which leaves the registers for the tiles themselves (user half 11.4 -> 10.5 ms)
    constexpr bool TILES_LDS = tiles_in_lds<C>() && !(PRESPLIT && !REDUCE);
    constexpr int TL = TILES_LDS ? tile_lds_floats<C>() : 0;
    __shared__ __attribute__((aligned(16))) float tiles_lds[NW][TL > 0 ? TL : 1];
    (void)tiles_lds;
    // pre-split Gram: one block's LDS image per wave (LDS-DMA target)
    constexpr int STAGE = (PRESPLIT && !REDUCE) ? 2 * C * 1024 : 16;
    __shared__ __attribute__((aligned(1024))) unsigned char stage_lds[NW][STAGE];
    (void)stage_lds;

    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    // the table-range guard (presplit_ok): a pre-split launch serves the half only in range, its guarded on-the-fly
    // fallback only out of range (one scalar load per wave; the other launch's waves exit here)
    if constexpr (!REDUCE && SPLIT) {
        if (PRESPLIT ? !presplit_ok(a.amax) : (a.presplit_fallback && presplit_ok(a.amax))) return;
    }
    // one task per wave (wave-uniform; no workgroup barriers are used below)
    auto task = [&](const int tid) {
        const Task tk = load_task(a.tasks + tid);
        float* buf = sbuf[wave];

        const int g = lane >> 4, j = lane & 15;
        Acc acc;
#pragma unroll
        for (int p = 0; p < Acc::NT; ++p) acc.g[p] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int c = 0; c < C; ++c) acc.rhs[c] = 0.f;
        f32x4 E[C];   // split paths: h m^T + h l^T of the diagonal tiles (fold_diag)
#pragma unroll
        for (int c = 0; c < C; ++c) E[c] = f32x4{0.f, 0.f, 0.f, 0.f};

        float* part = (float*)a.partials;
        constexpr int SLOT_WORDS = Acc::NWORDS + 1;   // + integrity check word
        int ps_sc = 0;   // pre-split Gram: its sums are in units of 2^(2 ps_sc) (tiles) and 2^ps_sc (RHS)
        if constexpr (REDUCE) {
            // Fixed-order sum of the row's partial slots ([word][lane] layout, coalesced), each decoded and checked.
            bool bad = false;
            int32_t bad_slot = -1;
            for (int s = 0; s < tk.nsteps; ++s) {
                const float* src = part + (int64_t)(tk.slot + s) * (SLOT_WORDS * 64) + lane;
                SlotCodec cd{slot_key(a.gen, tk.slot + s, lane)};
                // the whole slot's loads are issued before the first use: left to the scheduler under the KP = 128
                // register pressure they went out one at a time (load, wait, add: 0.44 ms for 974 rows)
                float w[SLOT_WORDS];
#pragma unroll
                for (int q = 0; q < SLOT_WORDS; ++q) w[q] = src[q * 64];
                __builtin_amdgcn_sched_barrier(0);
#pragma unroll
                for (int p = 0; p < Acc::NT; ++p)
#pragma unroll
                    for (int r = 0; r < 4; ++r) acc.g[p][r] += cd.dec(w[p * 4 + r], p * 4 + r);
#pragma unroll
                for (int c = 0; c < C; ++c) acc.rhs[c] += cd.dec(w[Acc::NT * 4 + c], Acc::NT * 4 + c);
                const bool ok = cd.check_ok(w[Acc::NWORDS], Acc::NWORDS);
                if (!ok && !bad) bad_slot = tk.slot + s;
                bad |= !ok;
            }
            report_bad_slot(a.integrity, a.gen, bad_slot, tk.row, bad, lane);
        } else {
            // Gather pipeline over blocks of B = 8 sub-steps (32 entries, layout [g][t], see block_position):
            // lane (g, j) loads the 8 column indices / ratings of its group with two 16-B loads, issued one
            // block ahead of that block's gathers, which are issued one block ahead of their MFMAs. The loop
            // body is branch-free, so vmcnt retires in program order with 8 gathers (8 KB per wave) still in
            // flight under each block's 80 MFMAs.
            constexpr int B = BLOCK_SUBSTEPS;
            const float* opp = (const float*)a.opp;
            const int n = tk.nsteps;
            const int nblk = (n + B - 1) / B;
            const int32_t* cb = a.col + tk.begin + g * B;
            const float* rb = a.rat + tk.begin + g * B;
            typedef int i32x4 __attribute__((ext_vector_type(4)));
            struct Idx { i32x4 i[2]; f32x4 r[2]; };
            auto load_idx = [&](int blk, Idx& x) {
                const int32_t* c = cb + (int64_t)blk * BLOCK_ENTRIES;
                const float* r = rb + (int64_t)blk * BLOCK_ENTRIES;
                x.i[0] = *(const i32x4*)c;
                x.i[1] = *(const i32x4*)(c + 4);
                x.r[0] = *(const f32x4*)r;
                x.r[1] = *(const f32x4*)(r + 4);
            };
            // unconditional: padding entries index the sentinel zero row; 32-bit unsigned byte offsets (host-checked:
            // opposite table <= 4 GiB, e.g. 16.7M rows at k = 64)
            // wave-uniform table base + 32-bit per-lane byte offsets (row << log2(row bytes), + this lane's piece): the
            // loads take the saddr form, one v_lshl_add_u32 per gathered row instead of a 64-bit address per lane
            const char* obase = (const char*)opp;
            const uint32_t lane_off = (uint32_t)(C * j * sizeof(float));
            constexpr int ROW_SHIFT = __builtin_ctz(KP * sizeof(float));
            auto gather = [&](const Idx& x, VT (&y)[B]) {
#pragma unroll
                for (int t = 0; t < B; ++t)
                    y[t] = *(const VT*)(obase + (((uint32_t)x.i[t >> 2][t & 3] << ROW_SHIFT) + lane_off));
            };
            auto mfma_step = [&](const VT& y, float r) {
#pragma unroll
                for (int b1 = 0; b1 < C; ++b1)
#pragma unroll
                    for (int b2 = b1; b2 < C; ++b2)
                        acc.g[tile_index<C>(b1, b2)] = __builtin_amdgcn_mfma_f32_16x16x4f32(
                            y[b1], y[b2], acc.g[tile_index<C>(b1, b2)], 0, 0, 0);
#pragma unroll
                for (int c = 0; c < C; ++c) acc.rhs[c] += r * y[c];
            };
            if constexpr (PRESPLIT) {
                ps_sc = gram_presplit<KP>(a, tk, acc, E, stage_lds[uni(wave)], buf, lane);
            } else if constexpr (SPLIT) {
                // Split-bf16 Gram: one v_mfma_f32_16x16x32_bf16 consumes a whole 32-entry block. Lane (g, j)
                // holds A[i = j][k = 8g + t] = y_t[C*j + b] (its own gathered piece, component b, entry t of its
                // group): with the interleaved feature order (f = C*i + b) the operands need no lane movement,
                // and the accumulators come out in exactly the layout of the f32 path (tile (b1, b2) holds
                // G[C*i + b1][C*j' + b2]), so the solve, the partial slots and the REDUCE pass are shared.
                // Padding entries gather the sentinel zero row with rating 0, so the last block needs no mask.
                typedef int i32x4 __attribute__((ext_vector_type(4)));
                struct Cols { i32x4 i[2]; };
                struct Rats { f32x4 r[2]; };
                auto load_cols = [&](int blk, Cols& x) {
                    const int32_t* c = cb + (int64_t)blk * BLOCK_ENTRIES;
                    x.i[0] = *(const i32x4*)c;
                    x.i[1] = *(const i32x4*)(c + 4);
                };
                auto load_rats = [&](int blk, Rats& x) {
                    const float* r = rb + (int64_t)blk * BLOCK_ENTRIES;
                    x.r[0] = *(const f32x4*)r;
                    x.r[1] = *(const f32x4*)(r + 4);
                };
                auto gather_blk = [&](const Cols& x, VT (&y)[B]) {
#pragma unroll
                    for (int t = 0; t < B; ++t)
                        y[t] = *(const VT*)(obase + (((uint32_t)x.i[t >> 2][t & 3] << ROW_SHIFT) + lane_off));
                };
                auto split_step = [&](const VT (&y)[B], const Rats& x) {
                    u32x4 H[C], M[C], L[C];
#pragma unroll
                    for (int b = 0; b < C; ++b)
#pragma unroll
                        for (int q = 0; q < 4; ++q) {
                            unsigned h, m, l;
                            split3(y[2 * q][b], y[2 * q + 1][b], h, m, l);
                            pin(h);
                            pin(m);
                            pin(l);
                            H[b][q] = h;
                            M[b][q] = m;
                            L[b][q] = l;
                        }
                    // the RHS before the MFMA group, materialised (see the RHS note at MFMA_DRAIN)
#pragma unroll
                    for (int t = 0; t < B; ++t)
#pragma unroll
                        for (int c = 0; c < C; ++c) acc.rhs[c] += x.r[t >> 2][t & 3] * y[t][c];
#pragma unroll
                    for (int c = 0; c < C; ++c) pin(acc.rhs[c]);
                    // the operands are materialised above (pin: MachineSink ignores sched_barrier), so the MFMA group
                    // below contains no VALU that could overwrite an operand register of an MFMA in flight
                    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
                    for (int b1 = 0; b1 < C; ++b1)
#pragma unroll
                        for (int b2 = b1; b2 < C; ++b2) {
                            f32x4 t = acc.g[tile_index<C>(b1, b2)];
                            t = mfma_k32(M[b1], M[b2], t);
                            if (b1 == b2) {
                                f32x4 e = E[b1];
                                e = mfma_k32(H[b1], L[b1], e);
                                e = mfma_k32(H[b1], M[b1], e);
                                E[b1] = e;
                            } else {
                                t = mfma_k32(H[b1], L[b2], t);
                                t = mfma_k32(L[b1], H[b2], t);
                                t = mfma_k32(H[b1], M[b2], t);
                                t = mfma_k32(M[b1], H[b2], t);
                            }
                            t = mfma_k32(H[b1], H[b2], t);
                            acc.g[tile_index<C>(b1, b2)] = t;
                        }
                    MFMA_DRAIN();
                };
                // Two blocks per trip with ping-pong buffers (no register rotation): column indices are loaded two
                // blocks ahead of their gathers' use, gathers and ratings one block ahead of their MFMAs.
                // Invariant at the loop top: Y0/R0 in flight for block b, I1 = columns of b+1, I0 = columns of b+2.
                if (C > 4 && nblk > 0) {
                    // KP = 128, one wave per SIMD: no second wave hides the split VALU behind this wave's MFMAs, so
                    // the wave interleaves them itself. The tiles are issued column by column (column c = tiles
                    // (b1 <= c, c): 6c + 4 MFMAs), and the split of feature block c + 1 -- the only new operand
                    // column c + 1 needs -- plus a share of the RHS FMAs run in the issue gaps of column c's MFMAs
                    // (an MFMA holds vector issue for 8 of its 16 cycles: two VALU per gap). Column 7's gaps split
                    // feature block 0 of the next block. No operand register dies before column 7 and all of them
                    // are kept allocated past the closing drain (keep_alive), so no VALU result can land in a
                    // register an MFMA in flight still reads. Same products, same accumulation order per tile and
                    // per RHS component as split_step: bitwise equal results.
                    Cols I0, I1;
                    Rats R0, R1;
                    VT Y0[B], Y1[B];
                    u32x4 H[C], M[C], L[C];
                    const int lastb = nblk - 1;
                    auto split_feat = [&](const VT (&y)[B], int c, u32x4& h4, u32x4& m4, u32x4& l4) {
#pragma unroll
                        for (int q = 0; q < 4; ++q) {
                            unsigned h, m, l;
                            split3(y[2 * q][c], y[2 * q + 1][c], h, m, l);
                            h4[q] = h;
                            m4[q] = m;
                            l4[q] = l;
                        }
                    };
                    auto keep_alive = [&]() {
#pragma unroll
                        for (int b = 0; b < C; ++b) asm volatile("" ::"v"(H[b]), "v"(M[b]), "v"(L[b]));
                    };
                    // one block: y/x = this block, yn = the next block (its feature block 0 is split here) when NEXT
                    auto block = [&](const VT (&y)[B], const Rats& x, const VT (&yn)[B], auto next_) {
                        constexpr bool NEXT = decltype(next_)::value;
                        u32x4 hn, mn, ln;
                        static_for<0, C>([&](auto C_) {
                            constexpr int c = decltype(C_)::value;
#pragma unroll
                            for (int b1 = 0; b1 <= c; ++b1) {
                                f32x4 t = acc.g[tile_index<C>(b1, c)];
                                t = mfma_k32(M[b1], M[c], t);
                                if (b1 == c) {
                                    f32x4 e = E[b1];
                                    e = mfma_k32(H[b1], L[b1], e);
                                    e = mfma_k32(H[b1], M[b1], e);
                                    E[b1] = e;
                                } else {
                                    t = mfma_k32(H[b1], L[c], t);
                                    t = mfma_k32(L[b1], H[c], t);
                                    t = mfma_k32(H[b1], M[c], t);
                                    t = mfma_k32(M[b1], H[c], t);
                                }
                                t = mfma_k32(H[b1], H[c], t);
                                acc.g[tile_index<C>(b1, c)] = t;
                            }
                            if constexpr (c + 1 < C) split_feat(y, c + 1, H[c + 1], M[c + 1], L[c + 1]);
                            // RHS components 0-1 in column 5's gaps, 2-4 in column 6's, 5-7 in column 7's
                            constexpr int r0 = c == 5 ? 0 : c == 6 ? 2 : c == 7 ? 5 : C;
                            constexpr int r1 = c == 5 ? 2 : c == 6 ? 5 : c == 7 ? 8 : C;
#pragma unroll
                            for (int f = r0; f < r1; ++f)
#pragma unroll
                                for (int t = 0; t < B; ++t) acc.rhs[f] += x.r[t >> 2][t & 3] * y[t][f];
                            if constexpr (NEXT && c == C - 1) split_feat(yn, 0, hn, mn, ln);
                            static_for<0, 6 * c + 4>([&](auto) {
                                __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);   // 1 MFMA
                                __builtin_amdgcn_sched_group_barrier(0x002, 2, 0);   // 2 VALU
                            });
                            __builtin_amdgcn_sched_barrier(0);
                        });
                        MFMA_DRAIN();
                        keep_alive();
                        __builtin_amdgcn_sched_barrier(0);
                        if constexpr (NEXT) {
                            H[0] = hn;
                            M[0] = mn;
                            L[0] = ln;
                        }
                    };
                    using Yes = std::integral_constant<bool, true>;
                    using No = std::integral_constant<bool, false>;
                    // one block per trip, staging rotated (two blocks per trip with ping-pong buffers made the
                    // register allocator shuffle the 144 accumulator registers at every back edge)
                    load_cols(0, I0);
                    load_cols(min(1, lastb), I1);
                    gather_blk(I0, Y0);
                    load_rats(0, R0);
                    split_feat(Y0, 0, H[0], M[0], L[0]);
                    for (int b = 0; b < lastb; ++b) {
                        gather_blk(I1, Y1);
                        load_rats(b + 1, R1);
                        load_cols(min(b + 2, lastb), I1);
                        __builtin_amdgcn_sched_barrier(0);
                        block(Y0, R0, Y1, Yes{});
#pragma unroll
                        for (int t = 0; t < B; ++t) Y0[t] = Y1[t];
                        R0 = R1;
                    }
                    block(Y0, R0, Y1, No{});
                } else if (nblk > 0) {
                    Cols I0, I1;
                    Rats R0, R1;
                    VT Y0[B], Y1[B];
                    const int lastb = nblk - 1;
                    load_cols(0, I0);
                    load_cols(min(1, lastb), I1);
                    gather_blk(I0, Y0);
                    load_rats(0, R0);
                    load_cols(min(2, lastb), I0);
                    int b = 0;
                    for (; b + 2 < nblk; b += 2) {
                        gather_blk(I1, Y1);
                        load_rats(b + 1, R1);
                        load_cols(min(b + 3, lastb), I1);
                        __builtin_amdgcn_sched_barrier(0);
                        split_step(Y0, R0);
                        __builtin_amdgcn_sched_barrier(0);
                        gather_blk(I0, Y0);
                        load_rats(b + 2, R0);
                        load_cols(min(b + 4, lastb), I0);
                        __builtin_amdgcn_sched_barrier(0);
                        split_step(Y1, R1);
                        __builtin_amdgcn_sched_barrier(0);
                    }
                    if (nblk - b == 2) {
                        gather_blk(I1, Y1);
                        load_rats(b + 1, R1);
                        __builtin_amdgcn_sched_barrier(0);
                        split_step(Y0, R0);
                        split_step(Y1, R1);
                    } else {
                        split_step(Y0, R0);
                    }
                }
            } else if constexpr (C > 4) {
                // KP = 128: 288 MFMAs per block, so half a block of prefetch (4 gathered rows per lane in
                // flight) covers the gather latency and halves the staging registers (the 36 accumulator
                // tiles already take 144). Stage = 4 sub-steps = one 16-B index/rating vector per lane.
                constexpr int H = B / 2;
                auto gather_half = [&](const Idx& x, auto h_, VT (&y)[H]) {
                    constexpr int h = decltype(h_)::value;
#pragma unroll
                    for (int t = 0; t < H; ++t)
                        y[t] = *(const VT*)(obase + (((uint32_t)x.i[h][t] << ROW_SHIFT) + lane_off));
                };
                using H0 = std::integral_constant<int, 0>;
                using H1 = std::integral_constant<int, 1>;
                if (nblk > 0) {
                    Idx x_c, x_n;
                    VT y_c[H], y_n[H];
                    load_idx(0, x_c);
                    load_idx(nblk > 1 ? 1 : 0, x_n);
                    gather_half(x_c, H0{}, y_c);
                    for (int b = 0; b + 1 < nblk; ++b) {
                        gather_half(x_c, H1{}, y_n);
                        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
                        for (int t = 0; t < H; ++t) mfma_step(y_c[t], x_c.r[0][t]);
                        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
                        for (int t = 0; t < H; ++t) y_c[t] = y_n[t];
                        Idx x_nn;
                        load_idx(b + 2 < nblk ? b + 2 : nblk - 1, x_nn);   // clamped: always a valid address
                        gather_half(x_n, H0{}, y_n);
                        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
                        for (int t = 0; t < H; ++t) mfma_step(y_c[t], x_c.r[1][t]);
                        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
                        for (int t = 0; t < H; ++t) y_c[t] = y_n[t];
                        x_c = x_n;
                        x_n = x_nn;
                    }
                    const int last = n - (nblk - 1) * B;
                    gather_half(x_c, H1{}, y_n);
#pragma unroll
                    for (int t = 0; t < H; ++t)
                        if (t < last) mfma_step(y_c[t], x_c.r[0][t]);     // wave-uniform
#pragma unroll
                    for (int t = 0; t < H; ++t)
                        if (H + t < last) mfma_step(y_n[t], x_c.r[1][t]);
                }
            } else if (nblk > 0) {
                Idx x_c, x_n;
                VT y_c[B], y_n[B];
                load_idx(0, x_c);
                load_idx(nblk > 1 ? 1 : 0, x_n);
                gather(x_c, y_c);
                for (int b = 0; b + 1 < nblk; ++b) {
                    Idx x_nn;
                    load_idx(b + 2 < nblk ? b + 2 : nblk - 1, x_nn);   // clamped: always a valid address
                    gather(x_n, y_n);
                    // keep the prefetch above the MFMAs: without this the scheduler sinks the gathers below
                    // them (saving registers) and every block waits out a full memory latency
                    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
                    for (int t = 0; t < B; ++t) mfma_step(y_c[t], x_c.r[t >> 2][t & 3]);
                    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
                    for (int t = 0; t < B; ++t) y_c[t] = y_n[t];
                    x_c = x_n;
                    x_n = x_nn;
                }
                const int last = n - (nblk - 1) * B;     // sub-steps with real entries in the last block
#pragma unroll
                for (int t = 0; t < B; ++t)
                    if (t < last) mfma_step(y_c[t], x_c.r[t >> 2][t & 3]);   // wave-uniform
            }
        }

        if constexpr (SPLIT && !REDUCE) {
            if constexpr (PRESPLIT)
                // the image is free after the Gram; the fold's lane addresses are derived afresh (opaque: kept live
                // across the Gram loop, one of them spilled at 128 VGPRs)
                fold_diag_lds<C>(acc, E, opaque(lane), stage_lds[uni(wave)]);
            else
                fold_diag<C>(acc, E, lane);
        }

        // Pre-split units: a PARTIAL task's slot holds true units (the REDUCE launch sums slots unscaled); a FULL task
        // solves in units of 2^keep (solve_tiles' u), keep = sc clamped to +-30 so that lambda n 2^(2 keep) stays a
        // normal float (a table far from unit scale, rare, pays the ldexp of the difference). Powers of two: exact.
        float u = 1.f;
        if constexpr (PRESPLIT && !REDUCE) {
            const int keep = tk.kind == TASK_PARTIAL ? 0 : min(max(ps_sc, -30), 30);
            if (ps_sc != keep) {   // wave-uniform
                const int d = ps_sc - keep;
#pragma unroll
                for (int p = 0; p < Acc::NT; ++p)
#pragma unroll
                    for (int r = 0; r < 4; ++r) acc.g[p][r] = ldexpf(acc.g[p][r], -2 * d);
#pragma unroll
                for (int c = 0; c < C; ++c) acc.rhs[c] = ldexpf(acc.rhs[c], -d);
            }
            u = ldexpf(1.f, keep);
        }
        if (!REDUCE && tk.kind == TASK_PARTIAL) {
            store_partial<C>(a, tk, acc, lane);
            return;
        }
        if (a.flags & SOLVE_FLAG_SKIP_SOLVE) {   // diagnostics (kbench): Gram only
            float* out = (float*)a.out + factor_row(a.row_offset, a.rows_per_chunk, a.chunk_stride, tk.row) * (int64_t)KP;
            if (lane < 16) {
#pragma unroll
                for (int b = 0; b < C; ++b) out[C * lane + b] = acc.g[tile_index<C>(b, b)][0] + acc.rhs[b];
            }
            return;
        }
        if constexpr (TILES_LDS) {
            LdsTiles T{tiles_lds[wave] + 4 * lane};
            RegStore<C> A0;
#pragma unroll
            for (int p = 0; p < Acc::NT; ++p) T.put(p, acc.g[p]);
            solve_tiles<C>(T, A0, acc.rhs, buf, tk, a, lane);
        } else if constexpr (PRESPLIT && !REDUCE) {
            RegTiles<C> T{acc.g};
            RowResidual A0;
            solve_tiles<C>(T, A0, acc.rhs, buf, tk, a, lane, u);
        } else {
            RegTiles<C> T{acc.g};
            RegStore<C> A0;
            solve_tiles<C>(T, A0, acc.rhs, buf, tk, a, lane);
        }
    };
    if constexpr (GRIDLOOP) {
        for (int tid = blockIdx.x * NW + wave; tid < a.n_tasks; tid += gridDim.x * NW) task(tid);
    } else {
        const int tid = blockIdx.x * NW + wave;
        if (tid < a.n_tasks) task(tid);
    }
}

// ---------------------------------------------------------------------------------------------------
// Short rows in entry space (fp32, split-bf16 MFMA)
// ---------------------------------------------------------------------------------------------------
// For a row with n <= 16 * CD entries (its 1 or 2 padded 32-entry blocks, CD = 2 or 4) the update
//   m = (Y^T Y + lambda n I_k)^{-1} Y^T r      (MFeatureCalculator.java:85-99, Y = the n x k gathered rows)
// equals  m = Y^T alpha  with  (Y Y^T + lambda n I_n) alpha = r  (push-through identity; the same nonzero
// spectrum and conditioning), an n x n system instead of k x k: at k = 128 a 64-entry user costs a 64 x 64
// solve instead of 128 x 128. The entry Gram Y Y^T needs no operand transposition: lane (g, i) loads the 32-B
// piece [32s + 8g, 32s + 8g + 8) of entry 16I + i's factor row, which is directly the A (and B) operand
// "row i, k = 8g..8g+7" of v_mfma_f32_16x16x32_bf16 for feature chunk s, split exactly into h/m/l bf16 terms
// as on the primal path. Entries are in physical (padded, block-interleaved) order; padding entries gather
// the zero sentinel row with rating 0 and get an identity row (solve_tiles<DUAL>), so alpha is 0 there.
template <int KP, int CD>
__global__ __launch_bounds__(64 * WAVES, CD <= 4 ? 2 : 1) void als_solve_dual(SolveArgs a) {
    constexpr int NS = KP / 32;      // 32-feature chunks = MFMA K steps
    constexpr int NF = KP / 64;      // output features per lane
    using Acc = MfmaAcc<CD>;
    __shared__ __attribute__((aligned(16))) float sbuf[WAVES][16 * CD];
    constexpr int TL = tile_lds_floats<CD>();
    __shared__ __attribute__((aligned(16))) float tiles_lds[WAVES][TL > 0 ? TL : 1];
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int tid = blockIdx.x * WAVES + wave;
    if (tid >= a.n_tasks) return;   // wave-uniform; no workgroup barriers below
    const Task tk = load_task(a.tasks + tid);
    float* buf = sbuf[wave];
    const int g = lane >> 4, i = lane & 15;
    const float* opp = (const float*)a.opp;
    int cidx[CD];
    float rr[CD];
#pragma unroll
    for (int I = 0; I < CD; ++I) {
        cidx[I] = a.col[tk.begin + 16 * I + i];
        rr[I] = a.rat[tk.begin + 16 * I + i];
    }
    f32x4 acc[Acc::NT];
#pragma unroll
    for (int p = 0; p < Acc::NT; ++p) acc[p] = f32x4{0.f, 0.f, 0.f, 0.f};
    const char* obase = (const char*)(opp + 8 * g);
    auto load = [&](int s, f32x8 (&y)[CD]) {
#pragma unroll
        for (int I = 0; I < CD; ++I)
            y[I] = *(const f32x8*)(obase + (uint32_t)cidx[I] * (uint32_t)(KP * sizeof(float)) + s * 128);
    };
    f32x8 yc[CD], yn[CD];
    load(0, yc);
#pragma unroll
    for (int s = 0; s < NS; ++s) {
        if (s + 1 < NS) load(s + 1, yn);
        u32x4 H[CD], M[CD], L[CD];
#pragma unroll
        for (int I = 0; I < CD; ++I)
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                unsigned h, m, l;
                split3(yc[I][2 * q], yc[I][2 * q + 1], h, m, l);
                pin(h);
                pin(m);
                pin(l);
                H[I][q] = h;
                M[I][q] = m;
                L[I][q] = l;
            }
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int I = 0; I < CD; ++I)
#pragma unroll
            for (int J = I; J < CD; ++J) {
                f32x4 t = acc[tile_index<CD>(I, J)];
                t = mfma_k32(M[I], M[J], t);
                t = mfma_k32(H[I], L[J], t);
                t = mfma_k32(L[I], H[J], t);
                t = mfma_k32(H[I], M[J], t);
                t = mfma_k32(M[I], H[J], t);
                t = mfma_k32(H[I], H[J], t);
                acc[tile_index<CD>(I, J)] = t;
            }
        MFMA_DRAIN();
        if (s + 1 < NS) {
#pragma unroll
            for (int I = 0; I < CD; ++I) yc[I] = yn[I];
        }
    }
    // right-hand side r in the per-lane partial layout of solve_tiles (element j of block b on row g = 0)
    float rhs[CD];
#pragma unroll
    for (int b = 0; b < CD; ++b) rhs[b] = g == 0 ? rr[b] : 0.f;
    if constexpr (tiles_in_lds<CD>()) {   // CD = 6: 21 working tiles in per-wave LDS, as the KP = 128 primal solve
        LdsTiles T{tiles_lds[wave] + 4 * lane};
        RegStore<CD> A0;
#pragma unroll
        for (int p = 0; p < Acc::NT; ++p) T.put(p, acc[p]);
        solve_tiles<CD, true>(T, A0, rhs, buf, tk, a, lane);
    } else {
        RegTiles<CD> T{acc};
        RegStore<CD> A0;
        solve_tiles<CD, true>(T, A0, rhs, buf, tk, a, lane);
    }
    wave_sync();
    // m = Y^T alpha: lane l owns features l + 64 f; entries with alpha = 0 (padding, or exactly 0) are skipped
    float xo[NF];
#pragma unroll
    for (int f = 0; f < NF; ++f) xo[f] = 0.f;
#pragma unroll
    for (int I = 0; I < CD; ++I)
#pragma unroll
        for (int e = 0; e < 16; ++e) {
            const float al = buf[16 * I + e];
            const int c = __builtin_amdgcn_readlane(cidx[I], e);
            const float* row = opp + (int64_t)c * KP + lane;
#pragma unroll
            for (int f = 0; f < NF; ++f) xo[f] += row[64 * f] * al;
        }
    float* out = (float*)a.out + factor_row(a.row_offset, a.rows_per_chunk, a.chunk_stride, tk.row) * (int64_t)KP + lane;
#pragma unroll
    for (int f = 0; f < NF; ++f) out[64 * f] = (lane + 64 * f < a.k) ? xo[f] : 0.f;
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
    constexpr int SLOT_WORDS = NWORDS + 1;   // + integrity check word (SlotCodec)
    if (tk.kind == TASK_REDUCE) {
        bool bad = false;
        int32_t bad_slot = -1;
        for (int s = 0; s < tk.nsteps; ++s) {
            const T* src = part + (int64_t)(tk.slot + s) * (SLOT_WORDS * 64) + lane;
            SlotCodec cd{slot_key(a.gen, tk.slot + s, lane)};
#pragma unroll
            for (int e = 0; e < E; ++e) acc[e] += cd.dec(src[e * 64], e);
            rhs += cd.dec(src[E * 64], E);
            const bool ok = cd.check_ok(src[NWORDS * 64], NWORDS);
            if (!ok && !bad) bad_slot = tk.slot + s;
            bad |= !ok;
        }
        report_bad_slot(a.integrity, a.gen, bad_slot, tk.row, bad, lane);
    } else {
        const T* opp = (const T*)a.opp;
        const int n = (tk.nsteps + BLOCK_SUBSTEPS - 1) / BLOCK_SUBSTEPS * BLOCK_ENTRIES;   // task span
        for (int base = 0; base < n; base += RSTAGE) {
            const int e = base + lane;
            int idx = a.sentinel;
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
                const int id = sidx[t];   // padding entries gather the sentinel zero row
                *(VT*)(stage + t * KP + v * VN) = *(const VT*)(opp + (int64_t)id * KP + v * VN);
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
        T* dst = part + (int64_t)tk.slot * (SLOT_WORDS * 64) + lane;
        SlotCodec cd{slot_key(a.gen, tk.slot, lane)};
#pragma unroll
        for (int e = 0; e < E; ++e) dst[e * 64] = cd.enc(acc[e], e);
        dst[E * 64] = cd.enc(rhs, E);
        dst[NWORDS * 64] = cd.check_word<T>(NWORDS);
        return;
    }

#pragma unroll
    for (int e = 0; e < E; ++e)
        if (c0 + e <= arow) G[tri(arow, 0) + c0 + e] = acc[e];   // packed lower triangle
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
    const T* self = (const T*)a.self + factor_row(a.row_offset, a.rows_per_chunk, a.chunk_stride, tk.row) * (int64_t)KP;
    const T* opp = (const T*)a.opp;
    const VT x = *(const VT*)(self + v * VN);
    const int n = (tk.nsteps + BLOCK_SUBSTEPS - 1) / BLOCK_SUBSTEPS * BLOCK_ENTRIES;   // task span
    double se = 0.0;
    for (int base = 0; base < n; base += EPS) {
        const int e = base + es;
        int idx = a.sentinel;
        float r = 0.f;
        if (e < n) {
            idx = a.col[tk.begin + e];
            r = a.rat[tk.begin + e];
        }
        const VT y = *(const VT*)(opp + (int64_t)idx * KP + v * VN);
        T dot = T(0);
#pragma unroll
        for (int c = 0; c < VN; ++c) dot += x[c] * y[c];
#pragma unroll
        for (int m = 1; m < LPE; m <<= 1) dot += __shfl_xor(dot, m);
        // logical entry index of physical position e (block_position inverse): skip the padding
        const int w = e % BLOCK_ENTRIES;
        const int logical = e - w + (w % BLOCK_SUBSTEPS) * 4 + w / BLOCK_SUBSTEPS;
        if (v == 0 && e < n && logical < tk.nent) {
            const double d = (double)r - (double)dot;
            se += d * d;
        }
    }
#pragma unroll
    for (int m = 1; m < 64; m <<= 1) se += __shfl_xor(se, m);
    if (lane == 0) a.task_se[tid] = se;
}

// ---------------------------------------------------------------------------------------------------
// Collector prediction matrix (FeatureCollector.java:90-101): P[u][m] = sum_f U[u][f] * M[m][f] in fp32 with
// Java float semantics -- each product and each partial sum rounded separately, features in order (EJML
// MatrixMatrixMult_FDRM.multTransB's sequential dot; no FMA contraction) -- so that the CSV digits are the
// reference's. 16 x 16 cells per workgroup, the 16 + 16 factor rows staged in LDS.
// ---------------------------------------------------------------------------------------------------
template <class T>
__global__ __launch_bounds__(256) void als_predict_kernel(const T* __restrict__ U, const T* __restrict__ M, int kp,
                                                          int k, const int64_t* __restrict__ urows, int64_t n_u,
                                                          const int64_t* __restrict__ mrows, int64_t n_m,
                                                          float* __restrict__ out) {
    __shared__ float su[16][129], sm[16][129];
    const int tx = threadIdx.x & 15, ty = threadIdx.x >> 4;
    const int64_t u0 = (int64_t)blockIdx.y * 16, m0 = (int64_t)blockIdx.x * 16;
    for (int i = threadIdx.x; i < 16 * k; i += 256) {
        const int r = i / k, f = i % k;
        su[r][f] = (u0 + r < n_u) ? (float)U[urows[u0 + r] * kp + f] : 0.f;   // f64 factors reach the
        sm[r][f] = (m0 + r < n_m) ? (float)M[mrows[m0 + r] * kp + f] : 0.f;   // collector as floats
    }
    __syncthreads();
    const int64_t u = u0 + ty, m = m0 + tx;
    if (u >= n_u || m >= n_m) return;
    float total = 0.f;
    {
#pragma clang fp contract(off)
        for (int f = 0; f < k; ++f) total = total + su[ty][f] * sm[tx][f];   // rounded product, rounded sum
    }
    out[u * n_m + m] = total;
}

// ---------------------------------------------------------------------------------------------------
// Generic path: any num_features beyond the wave-per-row kernels (fp32 k > 128, fp64 k > 64)
// ---------------------------------------------------------------------------------------------------
// One 256-thread workgroup per row (FULL tasks only: the work plan never splits a row on this path), grid-stride
// over the rows. MFeatureCalculator.java:85-99 for that row: the Gram's lower triangle and the RHS accumulated over
// LDS-staged batches of gathered factor rows, A + lambda n I (padded features: identity), a right-looking Cholesky
// (one pivot column per step, the trailing update spread over the workgroup), forward and backward substitution.
// G_LDS: the packed lower triangle lives in LDS (kp <= 256 fp32, <= 128 fp64); otherwise in a per-workgroup slab
// of `scratch` (slab elements each). Not a benchmark configuration: correctness for every k (ALSAppRunner.java:18
// accepts any NUM_FEATURES), at the cost of O(k^2) LDS traffic per gathered row.
template <class T, bool G_LDS>
__global__ __launch_bounds__(256) void als_solve_generic(SolveArgs a, int kp, int batch, T* __restrict__ scratch,
                                                         int64_t slab) {
    extern __shared__ __attribute__((aligned(16))) unsigned char gsmem[];
    const int tid = threadIdx.x;
    const int64_t ntri = (int64_t)kp * (kp + 1) / 2;
    T* G = G_LDS ? (T*)gsmem : scratch + (int64_t)blockIdx.x * slab;   // packed lower triangle, tri(i, j)
    T* stage = (T*)gsmem + (G_LDS ? ((ntri + 1) & ~(int64_t)1) : 0); // batch x kp gathered rows
    __shared__ T vec[1024 + 1];                                         // RHS / solution (kp <= 1024) + pivot
    // fp64: the refinement step's residual / correction and per-entry residuals of a batch (batch <= 64)
    __shared__ T res[std::is_same<T, double>::value ? 1024 : 1];
    __shared__ T tb[std::is_same<T, double>::value ? 64 : 1];
    const T* opp = (const T*)a.opp;
    auto tri_ = [](int64_t i, int64_t j) { return i * (i + 1) / 2 + j; };
    for (int task = blockIdx.x; task < a.n_tasks; task += gridDim.x) {
        const Task tk = a.tasks[task];
        T* out = (T*)a.out + factor_row(a.row_offset, a.rows_per_chunk, a.chunk_stride, tk.row) * (int64_t)kp;
        for (int64_t x = tid; x < ntri; x += 256) G[x] = T(0);
        for (int i = tid; i < kp; i += 256) vec[i] = T(0);
        __syncthreads();
        const int n = (tk.nsteps + BLOCK_SUBSTEPS - 1) / BLOCK_SUBSTEPS * BLOCK_ENTRIES;   // padded span
        for (int base = 0; base < n; base += batch) {
            const int nb = min(batch, n - base);
            for (int x = tid; x < nb * kp; x += 256) {   // padding entries gather the zero sentinel row
                const int e = x / kp, f = x - e * kp;
                stage[x] = opp[(int64_t)a.col[tk.begin + base + e] * kp + f];
            }
            __syncthreads();
            for (int i = tid; i < kp; i += 256) {
                T acc = vec[i];
                for (int e = 0; e < nb; ++e) acc += (T)a.rat[tk.begin + base + e] * stage[e * kp + i];
                vec[i] = acc;
            }
            for (int64_t x = tid; x < ntri; x += 256) {
                // row i of the packed triangle holding x: i (i + 1) / 2 <= x
                int64_t i = (int64_t)((sqrt(8.0 * (double)x + 1.0) - 1.0) / 2.0);
                while (i * (i + 1) / 2 > x) --i;
                while ((i + 1) * (i + 2) / 2 <= x) ++i;
                const int64_t j = x - i * (i + 1) / 2;
                T acc = G[x];
                for (int e = 0; e < nb; ++e) acc += stage[e * kp + i] * stage[e * kp + j];
                G[x] = acc;
            }
            __syncthreads();
        }
        if (tk.ndeg == 0) {   // cannot occur in the reference; defined as 0 (as the other paths)
            for (int i = tid; i < kp; i += 256) out[i] = T(0);
            __syncthreads();
            continue;
        }
        const T reg = (T)a.lambda * (T)tk.ndeg;   // A + lambda * (float) n on the diagonal (MFeatureCalculator.java:91-95)
        for (int i = tid; i < kp; i += 256) {
            const int64_t d = tri_(i, i);
            G[d] = i < a.k ? G[d] + reg : T(1);
        }
        __syncthreads();
        for (int j = 0; j < kp; ++j) {   // Cholesky: column j of L, then the trailing update
            if (tid == 0) {
                const T d = sqrt(G[tri_(j, j)]);
                G[tri_(j, j)] = d;
                vec[1024] = d;
            }
            __syncthreads();
            const T d = vec[1024];
            for (int i = j + 1 + tid; i < kp; i += 256) G[tri_(i, j)] /= d;
            __syncthreads();
            const int m = kp - j - 1;
            for (int64_t x = tid; x < (int64_t)m * m; x += 256) {
                const int i = j + 1 + (int)(x / m), l = j + 1 + (int)(x % m);
                if (l <= i) G[tri_(i, l)] -= G[tri_(i, j)] * G[tri_(l, j)];
            }
            __syncthreads();
        }
        auto chol_solve = [&](T* v) {   // v <- (L L^T)^{-1} v
            for (int j = 0; j < kp; ++j) {   // forward: L y = v
                const T y = v[j] / G[tri_(j, j)];
                __syncthreads();
                if (tid == 0) v[j] = y;
                for (int i = j + 1 + tid; i < kp; i += 256) v[i] -= G[tri_(i, j)] * y;
                __syncthreads();
            }
            for (int j = kp - 1; j >= 0; --j) {   // backward: L^T x = y
                const T x = v[j] / G[tri_(j, j)];
                __syncthreads();
                if (tid == 0) v[j] = x;
                for (int i = tid; i < j; i += 256) v[i] -= G[tri_(j, i)] * x;
                __syncthreads();
            }
        };
        chol_solve(vec);
        if constexpr (std::is_same<T, double>::value) {
            // fp64 parity mode: one step of iterative refinement, x += (L L^T)^{-1} (b - A x), with the residual
            // formed from the rows themselves (A x = Y^T (Y x) + lambda n x; the triangle now holds L):
            // b - A x = sum_e y_e (r_e - y_e . x) - lambda n x. The Cholesky's own error on the near-zero elements
            // of a wide solution (~cond * eps of the row norm) drops by about cond.
            for (int i = tid; i < kp; i += 256) res[i] = -(i < a.k ? reg : T(1)) * vec[i];
            __syncthreads();
            const int wv = tid >> 6, ln = tid & 63;
            for (int base = 0; base < n; base += batch) {
                const int nb = min(batch, n - base);
                for (int x = tid; x < nb * kp; x += 256) {
                    const int e = x / kp, f = x - e * kp;
                    stage[x] = opp[(int64_t)a.col[tk.begin + base + e] * kp + f];
                }
                __syncthreads();
                for (int e = wv; e < nb; e += 4) {   // t_e = r_e - y_e . x, one wave per entry
                    T d = T(0);
                    for (int f = ln; f < kp; f += 64) d += stage[e * kp + f] * vec[f];
#pragma unroll
                    for (int o = 32; o > 0; o >>= 1) d += __shfl_xor(d, o);
                    if (ln == 0) tb[e] = (T)a.rat[tk.begin + base + e] - d;
                }
                __syncthreads();
                for (int i = tid; i < kp; i += 256) {
                    T acc = res[i];
                    for (int e = 0; e < nb; ++e) acc += stage[e * kp + i] * tb[e];
                    res[i] = acc;
                }
                __syncthreads();
            }
            chol_solve(res);
            for (int i = tid; i < kp; i += 256) vec[i] += res[i];
            __syncthreads();
        }
        for (int i = tid; i < kp; i += 256) out[i] = i < a.k ? vec[i] : T(0);
        __syncthreads();
    }
}

// Squared error of the generic path (any kp): one wave per task, lane = feature stripe.
template <class T>
__global__ __launch_bounds__(256) void als_sq_error_generic(SqErrArgs a, int kp) {
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int tid = blockIdx.x * WAVES + wave;
    if (tid >= a.n_tasks) return;
    const Task tk = load_task(a.tasks + tid);
    const T* self = (const T*)a.self + factor_row(a.row_offset, a.rows_per_chunk, a.chunk_stride, tk.row) * (int64_t)kp;
    const T* opp = (const T*)a.opp;
    double se = 0.0;
    const int n = (tk.nsteps + BLOCK_SUBSTEPS - 1) / BLOCK_SUBSTEPS * BLOCK_ENTRIES;
    for (int e = 0; e < n; ++e) {
        const int w = e % BLOCK_ENTRIES;
        const int logical = e - w + (w % BLOCK_SUBSTEPS) * 4 + w / BLOCK_SUBSTEPS;
        if (logical >= tk.nent) continue;   // wave-uniform
        const T* y = opp + (int64_t)a.col[tk.begin + e] * kp;
        T dot = T(0);
        for (int f = lane; f < kp; f += 64) dot += self[f] * y[f];
#pragma unroll
        for (int m = 1; m < 64; m <<= 1) dot += __shfl_xor(dot, m);
        const double d = (double)a.rat[tk.begin + e] - (double)dot;
        se += d * d;
    }
    if (lane == 0) a.task_se[tid] = se;
}

// Collector dot products for any k (FeatureCollector.java:90-101, Java-float order): one thread per cell.
template <class T>
__global__ __launch_bounds__(256) void als_predict_generic(const T* __restrict__ U, const T* __restrict__ M, int kp,
                                                           int k, const int64_t* __restrict__ urows, int64_t n_u,
                                                           const int64_t* __restrict__ mrows, int64_t n_m,
                                                           float* __restrict__ out) {
    const int64_t cell = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (cell >= n_u * n_m) return;
    const int64_t u = cell / n_m, m = cell % n_m;
    const T* x = U + urows[u] * kp;
    const T* y = M + mrows[m] * kp;
    float total = 0.f;
    {
#pragma clang fp contract(off)
        for (int f = 0; f < k; ++f) total = total + (float)x[f] * (float)y[f];
    }
    out[cell] = total;
}

int blocks_for(int n_tasks) { return (n_tasks + WAVES - 1) / WAVES; }

// hipFuncAttributeMaxDynamicSharedMemorySize of one kernel on the current device, raised to `bytes` when a launch
// needs more than was set there before (engines of several devices and host threads launch concurrently: the
// per-(kernel, device) high-water mark is kept under a lock).
hipError_t ensure_dyn_lds(const void* fn, int bytes) {
    constexpr int MAXDEV = 64;
    static std::mutex mu;
    static std::vector<std::pair<const void*, std::vector<int>>> tab;   // per kernel: bytes set per device
    int dev = 0;
    hipError_t e = hipGetDevice(&dev);
    if (e != hipSuccess) return e;
    if (dev < 0 || dev >= MAXDEV) return hipErrorInvalidDevice;
    std::lock_guard<std::mutex> g(mu);
    std::vector<int>* set = nullptr;
    for (auto& x : tab)
        if (x.first == fn) set = &x.second;
    if (!set) {
        tab.emplace_back(fn, std::vector<int>(MAXDEV, 0));
        set = &tab.back().second;
    }
    if (bytes <= (*set)[dev]) return hipSuccess;
    e = hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, bytes);
    if (e == hipSuccess) (*set)[dev] = bytes;
    return e;
}

template <class T, int KP, Path P, int MINW = 1, bool PRESPLIT = false>
hipError_t launch_solve_t(const SolveArgs& a, hipStream_t s, bool reduce) {
    if (a.n_tasks <= 0) return hipSuccess;
    constexpr int bytes = WAVES * WaveLds<T, KP, P>::BYTES;
    if constexpr (P == Path::MFMA || P == Path::MFMA_SPLIT) {
        static_assert(std::is_same<T, float>::value, "MFMA paths are fp32");
        constexpr int nw = mfma_waves<KP>();
        const unsigned grid = (unsigned)((a.n_tasks + nw - 1) / nw);
        const size_t dyn = (size_t)a.extra_lds;   // debug build only: unused LDS per workgroup (occupancy sweeps)
        constexpr bool SPLIT = P == Path::MFMA_SPLIT;
        if (reduce) {   // one REDUCE kernel per KP: the partial slots have the same layout on every Gram path
            als_solve_mfma<KP, MINW, false, false, true><<<grid, 64 * nw, 0, s>>>(a);
        } else if constexpr (!PRESPLIT && SPLIT) {
            if (a.presplit_fallback)   // the range guard's fallback: grid-stride over a capped grid
                als_solve_mfma<KP, MINW, true, false, false, true>
                    <<<std::min<unsigned>(grid, (unsigned)std::max(1, a.grid_cap)), 64 * nw, dyn, s>>>(a);
            else
                als_solve_mfma<KP, MINW, true, false><<<grid, 64 * nw, dyn, s>>>(a);
        } else {
            als_solve_mfma<KP, MINW, SPLIT, PRESPLIT><<<grid, 64 * nw, dyn, s>>>(a);
        }
    } else {
        hipError_t e = ensure_dyn_lds((const void*)als_solve_valu<T, KP>, bytes);
        if (e != hipSuccess) return e;
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

// dst block i <- src block perm[i]: 32 columns + 32 ratings per block, one 64-lane wave per block (16 B per lane)
__global__ __launch_bounds__(256) void als_permute_blocks(const int32_t* __restrict__ col, const float* __restrict__ rat,
                                                         int32_t* __restrict__ col_out, float* __restrict__ rat_out,
                                                         const int32_t* __restrict__ perm, int64_t n_blocks) {
    const int64_t blk = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (blk >= n_blocks) return;
    const int l = threadIdx.x & 63;
    const int64_t src = (int64_t)perm[blk] * BLOCK_ENTRIES;
    const int64_t dst = blk * BLOCK_ENTRIES;
    if (l < 8) ((u32x4*)(col_out + dst))[l] = ((const u32x4*)(col + src))[l];
    else if (l < 16) ((u32x4*)(rat_out + dst))[l - 8] = ((const u32x4*)(rat + src))[l - 8];
}
hipError_t launch_permute_blocks(const int32_t* col, const float* rat, int32_t* col_out, float* rat_out,
                                 const int32_t* perm, int64_t n_blocks, hipStream_t s) {
    if (n_blocks <= 0) return hipSuccess;
    als_permute_blocks<<<(unsigned)((n_blocks + 3) / 4), 256, 0, s>>>(col, rat, col_out, rat_out, perm, n_blocks);
    return hipGetLastError();
}


bool variant_available(int precision, int kp, Path path) {
    if (path == Path::GENERIC) return kp % 16 == 0 && kp <= 1024;
    if (precision == 0) {
        if (path == Path::MFMA || path == Path::MFMA_SPLIT) return kp == 32 || kp == 64 || kp == 128;
        return kp == 16 || kp == 32 || kp == 64;
    }
    return path == Path::VALU && (kp == 16 || kp == 32 || kp == 64);
}

int partial_words_per_lane(int precision, int kp, Path path) {
    if (path == Path::GENERIC) return 0;   // rows are never split on the generic path
    if (path == Path::MFMA || path == Path::MFMA_SPLIT) {
        const int c = kp / 16;
        return (c * (c + 1) / 2) * 4 + c + 1;   // accumulators + RHS + check word
    }
    return kp * kp / 64 + 1 + 1;
}

hipError_t launch_predict(int precision, const void* U, const void* M, int kp, int k, const int64_t* urows,
                          int64_t n_u, const int64_t* mrows, int64_t n_m, float* out, hipStream_t s) {
    if (n_u <= 0 || n_m <= 0) return hipSuccess;
    if (k > 128) {   // generic path: one thread per cell
        const int64_t cells = n_u * n_m;
        if ((cells + 255) / 256 > INT32_MAX) return hipErrorInvalidValue;
        const unsigned g = (unsigned)((cells + 255) / 256);
        if (precision == 0)
            als_predict_generic<float><<<g, 256, 0, s>>>((const float*)U, (const float*)M, kp, k, urows, n_u, mrows, n_m, out);
        else
            als_predict_generic<double><<<g, 256, 0, s>>>((const double*)U, (const double*)M, kp, k, urows, n_u, mrows,
                                                           n_m, out);
        return hipGetLastError();
    }
    if ((n_m + 15) / 16 > INT32_MAX || (n_u + 15) / 16 > 65535) return hipErrorInvalidValue;
    const dim3 grid((unsigned)((n_m + 15) / 16), (unsigned)((n_u + 15) / 16));
    if (precision == 0)
        als_predict_kernel<float><<<grid, 256, 0, s>>>((const float*)U, (const float*)M, kp, k, urows, n_u, mrows, n_m, out);
    else
        als_predict_kernel<double><<<grid, 256, 0, s>>>((const double*)U, (const double*)M, kp, k, urows, n_u, mrows, n_m,
                                                        out);
    return hipGetLastError();
}

// Host <-> device factor-table copies as KERNEL accesses: each lane moves 16 B between pinned host memory
// (zero-copy, non-temporal) and device memory, so the factor tables are only ever written and read through
// the same cache path as the solve kernels' own accesses (no SDMA engine in between). This keeps every access
// to a factor table on one documented ordering path: kernels on the engine's stream.
__global__ __launch_bounds__(256) void copy16(const u32x4* __restrict__ src, u32x4* __restrict__ dst, int64_t n,
                                              int to_host) {
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        if (to_host) __builtin_nontemporal_store(src[i], dst + i);
        else dst[i] = __builtin_nontemporal_load(src + i);
    }
}

hipError_t launch_copy(const void* src, void* dst, size_t bytes, int to_host, hipStream_t s) {
    if (bytes == 0) return hipSuccess;
    if (bytes % 16 != 0) return hipErrorInvalidValue;
    const int64_t n = (int64_t)(bytes / 16);
    const int64_t blocks = std::min<int64_t>((n + 255) / 256, 4096);
    copy16<<<(unsigned)blocks, 256, 0, s>>>((const u32x4*)src, (u32x4*)dst, n, to_host);
    return hipGetLastError();
}
hipError_t launch_upload(const void* host_pinned, void* dst, size_t bytes, hipStream_t s) {
    return launch_copy(host_pinned, dst, bytes, 0, s);
}
hipError_t launch_download(const void* src, void* host_pinned, size_t bytes, hipStream_t s) {
    return launch_copy(src, host_pinned, bytes, 1, s);
}

// r = rh + rm with rh = f16_rn(r), rm = r - rh: both exact fp16 for integers |r| <= 2^22 (every Java short)
__global__ __launch_bounds__(256) void als_pack_ratings(const float* __restrict__ rat, uint32_t* __restrict__ dst,
                                                        int64_t n_pairs) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= n_pairs) return;
    unsigned h, m;
    split2(rat[2 * i], rat[2 * i + 1], h, m);
    dst[i] = h;
    dst[n_pairs + i] = m;
}
hipError_t launch_pack_ratings(const float* rat, uint32_t* dst, int64_t n_pairs, hipStream_t s) {
    if (n_pairs <= 0) return hipSuccess;
    als_pack_ratings<<<(unsigned)((n_pairs + 255) / 256), 256, 0, s>>>(rat, dst, n_pairs);
    return hipGetLastError();
}
hipError_t launch_absmax(const float* src, int64_t n_floats, int kp, uint32_t* amax, hipStream_t s) {
    hipError_t e = hipMemsetAsync(amax, 0, 2 * sizeof(uint32_t), s);
    if (e != hipSuccess || n_floats <= 0) return e;
    if (n_floats % kp || kp % 4 || kp / 4 > 64 || (kp / 4 & (kp / 4 - 1))) return hipErrorInvalidValue;   // whole rows
    const int64_t n4 = n_floats / 4;
    // >= 8 vectors per thread, at most 512 workgroups (= atomics)
    const int64_t blocks = std::max<int64_t>(1, std::min<int64_t>((n4 + 2047) / 2048, 512));
    als_absmax<<<(unsigned)blocks, 256, 0, s>>>((const u32x4*)src, n4, kp / 4, amax);
    return hipGetLastError();
}
hipError_t launch_presplit(int kp, const float* src, void* dst, int64_t n_rows, const uint32_t* amax, hipStream_t s) {
    const int64_t threads = n_rows * 2 * (kp / 16);
    if (threads <= 0) return hipSuccess;
    const unsigned grid = (unsigned)((threads + 255) / 256);
    if (kp == 64) als_presplit<64><<<grid, 256, 0, s>>>(src, (unsigned*)dst, threads, amax);
    else if (kp == 128) als_presplit<128><<<grid, 256, 0, s>>>(src, (unsigned*)dst, threads, amax);
    else return hipErrorInvalidValue;   // the pre-split Gram is built for KP = 64 and 128
    return hipGetLastError();
}
hipError_t launch_pack_cols_ps(const int32_t* col, int32_t* dst, int64_t n_entries, hipStream_t s) {
    if (n_entries <= 0) return hipSuccess;
    if (n_entries % BLOCK_ENTRIES) return hipErrorInvalidValue;
    als_pack_cols_ps<<<(unsigned)((n_entries + 255) / 256), 256, 0, s>>>(col, dst, n_entries);
    return hipGetLastError();
}

hipError_t launch_dual(int kp, int cd, const SolveArgs& a, hipStream_t s) {
    if (a.n_tasks <= 0) return hipSuccess;
    const unsigned grid = (unsigned)blocks_for(a.n_tasks);
    if (kp == 64 && cd == 2) als_solve_dual<64, 2><<<grid, 64 * WAVES, 0, s>>>(a);
    else if (kp == 128 && cd == 2) als_solve_dual<128, 2><<<grid, 64 * WAVES, 0, s>>>(a);
    else if (kp == 128 && cd == 4) als_solve_dual<128, 4><<<grid, 64 * WAVES, 0, s>>>(a);
    else if (kp == 128 && cd == 6) als_solve_dual<128, 6><<<grid, 64 * WAVES, 0, s>>>(a);
    else return hipErrorInvalidValue;
    return hipGetLastError();
}

hipError_t launch_solve(int precision, int kp, Path path, const SolveArgs& a, hipStream_t s, bool presplit,
                        bool reduce) {
    if (path == Path::GENERIC) return reduce ? hipErrorInvalidValue : launch_generic(precision, kp, a, s);
    if (precision == 0) {
        // occupancy (waves per SIMD) per variant: KP <= 64 two, the pre-split KP = 64 Gram four (PS64_WAVES),
        // KP = 128 one
        if (path == Path::MFMA) {
            if (kp == 32) return launch_solve_t<float, 32, Path::MFMA, 2>(a, s, reduce);
            if (kp == 64) return launch_solve_t<float, 64, Path::MFMA, 2>(a, s, reduce);
            if (kp == 128) return launch_solve_t<float, 128, Path::MFMA, 1>(a, s, reduce);
        } else if (path == Path::MFMA_SPLIT) {
            if (kp == 32) return launch_solve_t<float, 32, Path::MFMA_SPLIT, 2>(a, s, reduce);
            if (kp == 64 && presplit) return launch_solve_t<float, 64, Path::MFMA_SPLIT, PS64_WAVES, true>(a, s, reduce);
            if (kp == 64) return launch_solve_t<float, 64, Path::MFMA_SPLIT, 2>(a, s, reduce);
            if (kp == 128 && presplit) return launch_solve_t<float, 128, Path::MFMA_SPLIT, 1, true>(a, s, reduce);
            if (kp == 128) return launch_solve_t<float, 128, Path::MFMA_SPLIT, 1>(a, s, reduce);
        } else {
            if (kp == 16) return launch_solve_t<float, 16, Path::VALU>(a, s, reduce);
            if (kp == 32) return launch_solve_t<float, 32, Path::VALU>(a, s, reduce);
            if (kp == 64) return launch_solve_t<float, 64, Path::VALU>(a, s, reduce);
        }
    } else if (path == Path::VALU) {
        if (kp == 16) return launch_solve_t<double, 16, Path::VALU>(a, s, reduce);
        if (kp == 32) return launch_solve_t<double, 32, Path::VALU>(a, s, reduce);
        if (kp == 64) return launch_solve_t<double, 64, Path::VALU>(a, s, reduce);
    }
    return hipErrorInvalidValue;
}

GenericPlan generic_plan(int precision, int kp) {
    GenericPlan p{};
    const int64_t elem = precision == 0 ? 4 : 8;
    const int64_t ntri = (int64_t)kp * (kp + 1) / 2;
    const int64_t tri_b = ((ntri + 1) & ~(int64_t)1) * elem;
    // LDS minus the kernel's static vectors (RHS / solution; fp64: the refinement's residual and batch residuals)
    const int64_t avail = 160 * 1024 - 1025 * elem - (precision == 0 ? 2 * 4 : (1024 + 64) * 8);
    const int64_t row_b = (int64_t)kp * elem;
    if (tri_b + 8 * row_b <= avail) {
        p.g_in_lds = true;
        p.batch = (int)std::min<int64_t>(64, (avail - tri_b) / row_b);
        p.lds_bytes = tri_b + p.batch * row_b;
        p.slab_elems = 0;
    } else {
        p.g_in_lds = false;
        p.batch = (int)std::max<int64_t>(1, std::min<int64_t>(64, (64 * 1024) / row_b));
        p.lds_bytes = p.batch * row_b;
        p.slab_elems = ntri + 1;
    }
    return p;
}

template <class T, bool L>
hipError_t launch_generic_t(const GenericPlan& p, int kp, const SolveArgs& a, hipStream_t s) {
    hipError_t e = ensure_dyn_lds((const void*)als_solve_generic<T, L>, (int)p.lds_bytes);
    if (e != hipSuccess) return e;
    int64_t grid = std::min<int64_t>(a.n_tasks, 4096);
    if (!L) grid = std::min<int64_t>(grid, a.scratch_slabs);
    if (grid <= 0) return hipErrorInvalidValue;
    als_solve_generic<T, L><<<(unsigned)grid, 256, (size_t)p.lds_bytes, s>>>(a, kp, p.batch, (T*)a.partials,
                                                                             p.slab_elems);
    return hipGetLastError();
}

hipError_t launch_generic(int precision, int kp, const SolveArgs& a, hipStream_t s) {
    if (a.n_tasks <= 0) return hipSuccess;
    if (kp > 1024 || kp % 16) return hipErrorInvalidValue;
    const GenericPlan p = generic_plan(precision, kp);
    if (precision == 0)
        return p.g_in_lds ? launch_generic_t<float, true>(p, kp, a, s) : launch_generic_t<float, false>(p, kp, a, s);
    return p.g_in_lds ? launch_generic_t<double, true>(p, kp, a, s) : launch_generic_t<double, false>(p, kp, a, s);
}

hipError_t launch_sq_error(int precision, int kp, const SqErrArgs& a, hipStream_t s) {
    if (kp > 128 || (precision == 1 && kp > 64)) {   // generic path
        if (a.n_tasks <= 0) return hipSuccess;
        if (precision == 0) als_sq_error_generic<float><<<blocks_for(a.n_tasks), 256, 0, s>>>(a, kp);
        else als_sq_error_generic<double><<<blocks_for(a.n_tasks), 256, 0, s>>>(a, kp);
        return hipGetLastError();
    }
    if (precision == 0) {
        if (kp == 16) return launch_sq_t<float, 16>(a, s);
        if (kp == 32) return launch_sq_t<float, 32>(a, s);
        if (kp == 64) return launch_sq_t<float, 64>(a, s);
        if (kp == 128) return launch_sq_t<float, 128>(a, s);
    } else {
        if (kp == 16) return launch_sq_t<double, 16>(a, s);
        if (kp == 32) return launch_sq_t<double, 32>(a, s);
        if (kp == 64) return launch_sq_t<double, 64>(a, s);
    }
    return hipErrorInvalidValue;
}

}  // namespace cfk
