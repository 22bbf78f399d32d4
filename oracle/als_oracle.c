/*
 * CPU ORACLE -- TEST INFRASTRUCTURE ONLY.
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's `cpu_baseline` leg may load this
 * library, and only as the checker / the timed CPU baseline. The product path
 * (collaborative-filtering-kafka_amd/) never links, loads or calls it.
 *
 * Plain-C restatement of the reference's per-entity ALS feature update, i.e. the solve block of
 *   src/main/java/de/hpi/collaborativefilteringkafka/processors/MFeatureCalculator.java:66-104
 *   src/main/java/de/hpi/collaborativefilteringkafka/processors/UFeatureCalculator.java:66-104
 * which, through EJML 0.38 CommonOps_FDRM (third-party, NOT vendored in /root/reference; restated
 * from its published algorithm), computes for every entity row j with in-block Y_S (n_j x k, rows in
 * in-block order) and ratings r:
 *     V  = Y_S^T r                      CommonOps_FDRM.multTransA      (MFeatureCalculator.java:86)
 *     A  = Y_S^T Y_S                    CommonOps_FDRM.multTransA      (:89)
 *     A' = A + lambda * ((float)n_j I)  CommonOps_FDRM.scale/identity/add (:91-95)
 *     A'^-1                             CommonOps_FDRM.invert  -> LinearSolverLu_FDRM over
 *                                       LUDecompositionAlt_FDRM (JAMA-style Crout LU, partial
 *                                       pivoting), inverse = LU solve against each unit column (:98)
 *     m_j = A'^-1 V                     CommonOps_FDRM.mult (:99)
 * in the same operation order. Two precisions:
 *   - f32: every operation rounded to float exactly as Java float arithmetic (no FMA contraction;
 *          build with -ffp-contract=off). This is the "port" CPU baseline of the reference arithmetic.
 *   - f64: the identical algorithm in double with lambda = (double)(float)lambda (ALSAppRunner.java:19
 *          parses lambda with Float.parseFloat). This is the parity oracle (north star: factor max-rel
 *          <= 1e-6, MSE rel <= 1e-6).
 * CommonOps_FDRM.invert dispatches on the size: k <= UnrolledInverseFromMinor_FDRM.MAX (5) inverts by cofactors
 * (k = 1: 1/a), larger k by the LU solver above. Both are restated (minor_invert_* below for k <= 5).
 *
 * Also restated:
 *   - the U0 initialiser (UFeatureInitializer.java:50-56): f[0] = (float)mean(ratings) (mean in double),
 *     f[1..k-1] uniform [0,1). The reference draws unseeded Math.random(); the build replaces it with a
 *     shared seeded counter-based generator (splitmix64 of (seed, raw user id, feature)), restated here
 *     independently of the product code so both sides can be compared bit-for-bit.
 *   - the squared-error sum over observed ratings behind scripts/calculate_mse.py:78-90, with the
 *     prediction formed as FeatureCollector.java:92 does (fp32 multTransB: sequential float dot).
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#ifdef _OPENMP
#include <omp.h>
#endif

/* ------------------------------------------------------------------------------------------------ */
/* Seeded initial user features (replacement for Math.random(), UFeatureInitializer.java:55)        */
/* ------------------------------------------------------------------------------------------------ */
static uint64_t oracle_mix64(uint64_t z) {
    z += 0x9E3779B97F4A7C15ULL;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    return z ^ (z >> 31);
}

/* uniform float in [0,1) with 24 random bits: exact in float, never rounds up to 1.0f */
float oracle_u01(uint64_t seed, int64_t raw_id, int32_t feature) {
    uint64_t h = oracle_mix64(seed ^ oracle_mix64((uint64_t)raw_id * 0x100000001B3ULL + (uint64_t)(uint32_t)feature));
    return (float)(h >> 40) * (1.0f / 16777216.0f);
}

/* UFeatureInitializer.java:50-56 for n_users rows (row i = user raw id user_ids[i]) */
void oracle_init_user_features(int64_t n_users, const int64_t* user_ids, const int64_t* row_ptr,
                               const int16_t* ratings, int k, uint64_t seed, float* out /* n_users x k */) {
    for (int64_t u = 0; u < n_users; ++u) {
        int64_t b = row_ptr[u], e = row_ptr[u + 1];
        int64_t sum = 0;
        for (int64_t t = b; t < e; ++t) sum += ratings[t];
        /* DoubleStream.average(): exact for short ratings; .orElse(1.0) for an empty list */
        double mean = (e > b) ? (double)sum / (double)(e - b) : 1.0;
        out[u * k + 0] = (float)mean;
        for (int f = 1; f < k; ++f) out[u * k + f] = oracle_u01(seed, user_ids[u], f);
    }
}

/* ------------------------------------------------------------------------------------------------ */
/* EJML LinearSolverLu_FDRM / LUDecompositionAlt_FDRM restated, templated by macro on the scalar     */
/* ------------------------------------------------------------------------------------------------ */
#define DEFINE_LU_INVERT(T, SUFFIX, ABS)                                                                \
    /* LUDecompositionAlt_FDRM.decompose (JAMA Crout, partial pivoting), LU in place, row-major n x n */ \
    static void lu_decompose_##SUFFIX(T* lu, int n, int* indx, T* col) {                                \
        for (int j = 0; j < n; ++j) {                                                                   \
            for (int i = 0; i < n; ++i) col[i] = lu[i * n + j];                                         \
            for (int i = 0; i < n; ++i) {                                                               \
                int kmax = i < j ? i : j;                                                               \
                T s = (T)0;                                                                             \
                for (int kk = 0; kk < kmax; ++kk) s += lu[i * n + kk] * col[kk];                        \
                col[i] -= s;                                                                            \
                lu[i * n + j] = col[i];                                                                 \
            }                                                                                           \
            int p = j;                                                                                  \
            T mx = ABS(col[p]);                                                                         \
            for (int i = j + 1; i < n; ++i) {                                                           \
                T v = ABS(col[i]);                                                                      \
                if (v > mx) { p = i; mx = v; }                                                          \
            }                                                                                           \
            if (p != j) {                                                                               \
                for (int c = 0; c < n; ++c) {                                                           \
                    T t = lu[p * n + c]; lu[p * n + c] = lu[j * n + c]; lu[j * n + c] = t;              \
                }                                                                                       \
            }                                                                                           \
            indx[j] = p;                                                                                \
            T ljj = lu[j * n + j];                                                                      \
            if (ljj != (T)0)                                                                            \
                for (int i = j + 1; i < n; ++i) lu[i * n + j] /= ljj;                                   \
        }                                                                                               \
    }                                                                                                   \
    /* LUDecompositionBase_FDRM._solveVectorInternal + TriangularSolver_FDRM.solveU */                 \
    static void lu_solve_vec_##SUFFIX(const T* lu, int n, const int* indx, T* vv) {                     \
        int ii = 0;                                                                                     \
        for (int i = 0; i < n; ++i) {                                                                   \
            int ip = indx[i];                                                                           \
            T sum = vv[ip];                                                                             \
            vv[ip] = vv[i];                                                                             \
            if (ii != 0) {                                                                              \
                for (int j = ii - 1; j < i; ++j) sum -= lu[i * n + j] * vv[j];                          \
            } else if (sum != (T)0) {                                                                   \
                ii = i + 1;                                                                             \
            }                                                                                           \
            vv[i] = sum;                                                                                \
        }                                                                                               \
        for (int i = n - 1; i >= 0; --i) {                                                              \
            T sum = vv[i];                                                                              \
            for (int j = i + 1; j < n; ++j) sum -= lu[i * n + j] * vv[j];                               \
            vv[i] = sum / lu[i * n + i];                                                                \
        }                                                                                               \
    }                                                                                                   \
    /* CommonOps_FDRM.invert -> LinearSolverLuBase.invert: column j of A^-1 = LU solve of e_j */        \
    static void lu_invert_##SUFFIX(T* a, int n, T* lu, int* indx, T* col) {                             \
        memcpy(lu, a, sizeof(T) * (size_t)n * (size_t)n);                                               \
        lu_decompose_##SUFFIX(lu, n, indx, col);                                                        \
        for (int j = 0; j < n; ++j) {                                                                   \
            for (int i = 0; i < n; ++i) col[i] = (T)0;                                                  \
            col[j] = (T)1;                                                                              \
            lu_solve_vec_##SUFFIX(lu, n, indx, col);                                                    \
            for (int i = 0; i < n; ++i) a[i * n + j] = col[i];                                          \
        }                                                                                               \
    }

DEFINE_LU_INVERT(float, f32, fabsf)
DEFINE_LU_INVERT(double, f64, fabs)

/* ------------------------------------------------------------------------------------------------ */
/* EJML UnrolledInverseFromMinor_FDRM / _DDRM restated (CommonOps_FDRM.invert for 2 <= k <= 5)        */
/* ------------------------------------------------------------------------------------------------ */
/* inv(mat): scale = 1 / max|a| over all entries (the first entry, then strictly larger ones in storage order),
 * a_ij *= scale; cofactor m_ij = (-1)^(i+j) det(minor without row i, column j), each minor determinant written
 * out as the library's generated code does -- Laplace expansion along the minor's first row, terms left to
 * right with alternating signs (+ a*(..) - b*(..) + ...), 2 x 2 determinants as (a*d - b*c), a negative cofactor
 * as -( .. ); det = (a11*m11 + a12*m12 + ... + a1k*m1k) / scale; inv[j][i] = m_ij / det. The same expression
 * shapes evaluated in float (f32, no contraction) or double (f64). */
#define DEFINE_MINOR_INVERT(T, SUFFIX, ABS)                                                              \
    static T minor_det_##SUFFIX(const T* a, int n, const int* rows, const int* cols, int m) {            \
        if (m == 1) return a[rows[0] * n + cols[0]];                                                     \
        if (m == 2)                                                                                      \
            return a[rows[0] * n + cols[0]] * a[rows[1] * n + cols[1]] -                                 \
                   a[rows[0] * n + cols[1]] * a[rows[1] * n + cols[0]];                                  \
        T total = (T)0;                                                                                  \
        for (int c = 0; c < m; ++c) {                                                                    \
            int sub[4], q = 0;                                                                           \
            for (int x = 0; x < m; ++x)                                                                  \
                if (x != c) sub[q++] = cols[x];                                                          \
            const T term = a[rows[0] * n + cols[c]] * minor_det_##SUFFIX(a, n, rows + 1, sub, m - 1);    \
            total = (c == 0) ? term : ((c & 1) ? total - term : total + term);                           \
        }                                                                                                \
        return total;                                                                                    \
    }                                                                                                    \
    static void minor_invert_##SUFFIX(T* data, int n) {                                                  \
        if (n == 1) { data[0] = (T)1 / data[0]; return; }                                                \
        T max = ABS(data[0]);                                                                            \
        for (int i = 1; i < n * n; ++i) {                                                                \
            T v = ABS(data[i]);                                                                          \
            if (v > max) max = v;                                                                        \
        }                                                                                                \
        const T scale = (T)1 / max;                                                                      \
        T a[25], m[25];                                                                                  \
        for (int i = 0; i < n * n; ++i) a[i] = data[i] * scale;                                          \
        for (int i = 0; i < n; ++i)                                                                      \
            for (int j = 0; j < n; ++j) {                                                                \
                int rows[4], cols[4], q = 0;                                                             \
                for (int x = 0; x < n; ++x)                                                              \
                    if (x != i) rows[q++] = x;                                                           \
                q = 0;                                                                                   \
                for (int x = 0; x < n; ++x)                                                              \
                    if (x != j) cols[q++] = x;                                                           \
                const T d = minor_det_##SUFFIX(a, n, rows, cols, n - 1);                                 \
                m[i * n + j] = ((i + j) & 1) ? -(d) : d;                                                 \
            }                                                                                            \
        T det = a[0] * m[0];                                                                             \
        for (int j = 1; j < n; ++j) det = det + a[j] * m[j];                                             \
        det = det / scale;                                                                               \
        for (int i = 0; i < n; ++i)                                                                      \
            for (int j = 0; j < n; ++j) data[j * n + i] = m[i * n + j] / det;                            \
    }                                                                                                    \
    /* CommonOps_FDRM.invert(mat): cofactors up to UnrolledInverseFromMinor_FDRM.MAX = 5, else LU */      \
    static void ejml_invert_##SUFFIX(T* a, int n, T* lu, int* indx, T* col) {                            \
        if (n <= 5) minor_invert_##SUFFIX(a, n);                                                         \
        else lu_invert_##SUFFIX(a, n, lu, indx, col);                                                    \
    }

DEFINE_MINOR_INVERT(float, f32, fabsf)
DEFINE_MINOR_INVERT(double, f64, fabs)

/* the inverse alone (tests: known-answer matrices through both EJML branches) */
int oracle_invert_f64(double* a, int n) {
    if (n < 1 || n > 1024) return 1;
    double* lu = (double*)malloc(sizeof(double) * ((size_t)n * n + n));
    int* indx = (int*)malloc(sizeof(int) * (size_t)n);
    if (!lu || !indx) { free(lu); free(indx); return 2; }
    ejml_invert_f64(a, n, lu, indx, lu + (size_t)n * n);
    free(lu);
    free(indx);
    return 0;
}
int oracle_invert_f32(float* a, int n) {
    if (n < 1 || n > 1024) return 1;
    float* lu = (float*)malloc(sizeof(float) * ((size_t)n * n + n));
    int* indx = (int*)malloc(sizeof(int) * (size_t)n);
    if (!lu || !indx) { free(lu); free(indx); return 2; }
    ejml_invert_f32(a, n, lu, indx, lu + (size_t)n * n);
    free(lu);
    free(indx);
    return 0;
}

/* ------------------------------------------------------------------------------------------------ */
/* The per-entity update (MFeatureCalculator.java:66-104), one CSR row per entity                   */
/* ------------------------------------------------------------------------------------------------ */
#define DEFINE_UPDATE(T, SUFFIX)                                                                         \
    static void update_row_##SUFFIX(int64_t b, int64_t e, const int32_t* col_idx, const int16_t* ratings, \
                                    const T* opp, int k, T lam, T* out, T* ws) {                         \
        T* A = ws;                      /* k*k */                                                        \
        T* LU = A + (size_t)k * k;       /* k*k */                                                        \
        T* V = LU + (size_t)k * k;       /* k   */                                                        \
        T* col = V + k;                 /* k   */                                                        \
        int* indx = (int*)(col + k);     /* k ints */                                                     \
        int64_t n = e - b;                                                                              \
        if (n == 0) { for (int f = 0; f < k; ++f) out[f] = (T)0; return; }                              \
        /* V = multTransA(Y_S, r): V[i] = sum_j Y[j][i] * r[j], j ascending (MatrixVectorMult) */        \
        for (int i = 0; i < k; ++i) V[i] = (T)0;                                                         \
        for (int i = 0; i < k * k; ++i) A[i] = (T)0;                                                     \
        for (int64_t t = b; t < e; ++t) {                                                               \
            const T* y = opp + (int64_t)col_idx[t] * k;                                                  \
            T r = (T)ratings[t];                                                                         \
            for (int i = 0; i < k; ++i) V[i] += y[i] * r;                                                \
            /* A = multTransA(Y_S, Y_S): A[i][l] = sum_j Y[j][i] * Y[j][l], j ascending */                \
            for (int i = 0; i < k; ++i) {                                                                \
                T yi = y[i];                                                                             \
                for (int l = 0; l < k; ++l) A[i * k + l] += yi * y[l];                                   \
            }                                                                                            \
        }                                                                                                \
        /* A + lambda * ((T)n * I)  (scale(n, identity) then add(A, lambda, N)) */                      \
        T reg = lam * (T)n;                                                                              \
        for (int i = 0; i < k; ++i) A[i * k + i] += reg;                                                 \
        ejml_invert_##SUFFIX(A, k, LU, indx, col);                                                       \
        /* m = mult(A^-1, V): total = A[i][0]*V[0]; total += A[i][j]*V[j] */                              \
        for (int i = 0; i < k; ++i) {                                                                    \
            T total = A[i * k] * V[0];                                                                   \
            for (int j = 1; j < k; ++j) total += A[i * k + j] * V[j];                                    \
            out[i] = total;                                                                              \
        }                                                                                                \
    }                                                                                                    \
    int oracle_update_##SUFFIX(int64_t n_rows, const int64_t* row_ptr, const int32_t* col_idx,         \
                               const int16_t* ratings, const T* opp, int k, float lambda, T* out,       \
                               int nthreads) {                                                           \
        if (k <= 0 || n_rows < 0) return 1;                                                              \
        T lam = (T)lambda;                                                                               \
        size_t ws_bytes = sizeof(T) * (2 * (size_t)k * k + 2 * (size_t)k) + sizeof(int) * (size_t)k + 64; \
        (void)nthreads;                                                                                  \
        _Pragma("omp parallel num_threads(nthreads > 0 ? nthreads : 1)")                                 \
        {                                                                                                \
            T* ws = (T*)malloc(ws_bytes);                                                                \
            _Pragma("omp for schedule(dynamic, 1)")                                                     \
            for (int64_t r = 0; r < n_rows; ++r)                                                         \
                update_row_##SUFFIX(row_ptr[r], row_ptr[r + 1], col_idx, ratings, opp, k, lam,           \
                                    out + r * (int64_t)k, ws);                                           \
            free(ws);                                                                                    \
        }                                                                                                \
        return 0;                                                                                        \
    }

DEFINE_UPDATE(float, f32)
DEFINE_UPDATE(double, f64)

/* Same update for an explicit list of rows (used to spot-check huge configs on sampled rows). */
int oracle_update_rows_f64(int64_t n_sel, const int64_t* sel_rows, const int64_t* row_ptr,
                           const int32_t* col_idx, const int16_t* ratings, const double* opp, int k,
                           float lambda, double* out /* n_sel x k */) {
    size_t ws_bytes = sizeof(double) * (2 * (size_t)k * k + 2 * (size_t)k) + sizeof(int) * (size_t)k + 64;
    int rc = 0;
#pragma omp parallel
    {
        double* ws = (double*)malloc(ws_bytes);
        if (!ws) {
#pragma omp atomic write
            rc = 2;
        }
#pragma omp for schedule(dynamic, 1)
        for (int64_t s = 0; s < n_sel; ++s) {
            int64_t r = sel_rows[s];
            if (ws)
                update_row_f64(row_ptr[r], row_ptr[r + 1], col_idx, ratings, opp, k, (double)lambda, out + s * k,
                               ws);
        }
        free(ws);
    }
    return rc;
}

/* ------------------------------------------------------------------------------------------------ */
/* Squared error over observed ratings (calculate_mse.py:78-90 with FeatureCollector.java:92 preds) */
/* ------------------------------------------------------------------------------------------------ */
double oracle_sq_error_f32(int64_t n_rows, const int64_t* row_ptr, const int32_t* col_idx,
                           const int16_t* ratings, const float* row_f, const float* col_f, int k,
                           int64_t* count) {
    double se = 0.0;
    int64_t c = 0;
    for (int64_t r = 0; r < n_rows; ++r) {
        const float* x = row_f + r * (int64_t)k;
        for (int64_t t = row_ptr[r]; t < row_ptr[r + 1]; ++t) {
            const float* y = col_f + (int64_t)col_idx[t] * k;
            float total = 0.0f;
            for (int f = 0; f < k; ++f) total += x[f] * y[f];
            double d = (double)ratings[t] - (double)total;
            se += d * d;
            ++c;
        }
    }
    if (count) *count = c;
    return se;
}

double oracle_sq_error_f64(int64_t n_rows, const int64_t* row_ptr, const int32_t* col_idx,
                           const int16_t* ratings, const double* row_f, const double* col_f, int k,
                           int64_t* count) {
    double se = 0.0;
    int64_t c = 0;
    for (int64_t r = 0; r < n_rows; ++r) {
        const double* x = row_f + r * (int64_t)k;
        for (int64_t t = row_ptr[r]; t < row_ptr[r + 1]; ++t) {
            const double* y = col_f + (int64_t)col_idx[t] * k;
            double total = 0.0;
            for (int f = 0; f < k; ++f) total += x[f] * y[f];
            double d = (double)ratings[t] - total;
            se += d * d;
            ++c;
        }
    }
    if (count) *count = c;
    return se;
}

int oracle_max_threads(void) {
#ifdef _OPENMP
    return omp_get_max_threads();
#else
    return 1;
#endif
}
