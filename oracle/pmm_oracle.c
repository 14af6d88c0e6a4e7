/*
 * pmm_oracle.c -- CPU restatement of the reference's `.pmm.topk` / `.pmm.matmul`
 * numerics (NivekNey/polars-matmul v0.1.4).
 *
 * TEST INFRASTRUCTURE ONLY.  Only tests/, __graft_entry__.smoke() and the
 * cpu_baseline leg of bench.py may load this library, and only as the checker
 * or the timed CPU baseline.  The product path (polars-matmul_amd/) never links
 * or calls it.
 *
 * What is restated, and from where (paths are into the reference tree):
 *   - Metric parsing / direction ............ src/metrics.rs:20-36
 *   - row L2 norms (ndarray 1-D `dot`) ...... src/metrics.rs:368-393
 *       ndarray 0.16 `unrolled_dot` (third-party, not vendored; recalled):
 *       8 partial sums p0..p7 over chunks of 8, combined
 *       sum=(p0+p4); sum+=(p1+p5); sum+=(p2+p6); sum+=(p3+p7); then the
 *       scalar tail, no FMA contraction.  Built with -ffp-contract=off.
 *   - GEMM  S = Q * C^T ...................... src/metrics.rs:204-255 (f32),
 *       :40-97 (f64), zero-copy variants :111-202.  The arithmetic lives in
 *       faer 0.19 (third-party, version unpinned: Cargo.lock is gitignored).
 *       Restated as one k-ordered fused-multiply-add chain per output
 *       element; faer's blocking order is NOT pinned by any reference test,
 *       so GEMM outputs are compared within the reference's rtol=1e-5.
 *   - cosine / euclidean epilogue ............ src/metrics.rs:314-365 (f32),
 *       :258-311 (f64): s /= (qn*cn) with norm threshold 1e-6 (f32) /
 *       1e-10 (f64); euclid = sqrt(max((qsq+csq) - 2*dot, 0)).
 *   - per-row top-k ........................... src/topk.rs:42-75 (f32), :6-39
 *       select_nth_unstable_by + truncate + sort_by.  The reference leaves
 *       the order of equal scores (and NaN placement) unspecified
 *       (partial_cmp -> Equal).  This restatement fixes the total order
 *       (score best-first, NaN last, then lower corpus index first), which
 *       is one of the orders the reference may produce.
 *   - k clipping, f32->f64 score widening ... src/matmul.rs:443-447
 *
 * Structure mirrors the reference: multithreaded GEMM (faer's rayon pool),
 * then a single-threaded epilogue over the materialised M x N matrix, then
 * a single-threaded per-row select.  That is what the cpu_baseline times.
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <ctype.h>
#ifdef _OPENMP
#include <omp.h>
#endif

#define METRIC_COSINE 0
#define METRIC_DOT 1
#define METRIC_EUCLIDEAN 2

/* ---- metrics.rs:20-27  Metric::from_str (lower-cased, "l2" alias) ---- */
int oracle_metric_from_str(const char *s) {
    char buf[32];
    size_t n = strlen(s);
    if (n >= sizeof(buf)) return -1;
    for (size_t i = 0; i <= n; i++) buf[i] = (char)tolower((unsigned char)s[i]);
    if (strcmp(buf, "cosine") == 0) return METRIC_COSINE;
    if (strcmp(buf, "dot") == 0) return METRIC_DOT;
    if (strcmp(buf, "euclidean") == 0 || strcmp(buf, "l2") == 0) return METRIC_EUCLIDEAN;
    return -1;
}

/* metrics.rs:30-35 */
int oracle_higher_is_better(int metric) { return metric != METRIC_EUCLIDEAN; }

/* ---- ndarray unrolled_dot restatement (f32 / f64) ---- */
static float udot_f32(const float *x, const float *y, int64_t n) {
    float sum = 0.0f;
    float p0 = 0, p1 = 0, p2 = 0, p3 = 0, p4 = 0, p5 = 0, p6 = 0, p7 = 0;
    int64_t i = 0;
    for (; i + 8 <= n; i += 8) {
        p0 = p0 + x[i + 0] * y[i + 0];
        p1 = p1 + x[i + 1] * y[i + 1];
        p2 = p2 + x[i + 2] * y[i + 2];
        p3 = p3 + x[i + 3] * y[i + 3];
        p4 = p4 + x[i + 4] * y[i + 4];
        p5 = p5 + x[i + 5] * y[i + 5];
        p6 = p6 + x[i + 6] * y[i + 6];
        p7 = p7 + x[i + 7] * y[i + 7];
    }
    sum = sum + (p0 + p4);
    sum = sum + (p1 + p5);
    sum = sum + (p2 + p6);
    sum = sum + (p3 + p7);
    for (; i < n; i++) sum = sum + x[i] * y[i];
    return sum;
}

static double udot_f64(const double *x, const double *y, int64_t n) {
    double sum = 0.0;
    double p0 = 0, p1 = 0, p2 = 0, p3 = 0, p4 = 0, p5 = 0, p6 = 0, p7 = 0;
    int64_t i = 0;
    for (; i + 8 <= n; i += 8) {
        p0 = p0 + x[i + 0] * y[i + 0];
        p1 = p1 + x[i + 1] * y[i + 1];
        p2 = p2 + x[i + 2] * y[i + 2];
        p3 = p3 + x[i + 3] * y[i + 3];
        p4 = p4 + x[i + 4] * y[i + 4];
        p5 = p5 + x[i + 5] * y[i + 5];
        p6 = p6 + x[i + 6] * y[i + 6];
        p7 = p7 + x[i + 7] * y[i + 7];
    }
    sum = sum + (p0 + p4);
    sum = sum + (p1 + p5);
    sum = sum + (p2 + p6);
    sum = sum + (p3 + p7);
    for (; i < n; i++) sum = sum + x[i] * y[i];
    return sum;
}

/* metrics.rs:382-393 compute_norms_f32 / compute_squared_norms_f32 */
void oracle_norms_f32(const float *a, int64_t rows, int64_t d, int squared, float *out) {
    for (int64_t r = 0; r < rows; r++) {
        float v = udot_f32(a + r * d, a + r * d, d);
        out[r] = squared ? v : sqrtf(v);
    }
}

/* metrics.rs:368-379 compute_norms_f64 / compute_squared_norms_f64 */
void oracle_norms_f64(const double *a, int64_t rows, int64_t d, int squared, double *out) {
    for (int64_t r = 0; r < rows; r++) {
        double v = udot_f64(a + r * d, a + r * d, d);
        out[r] = squared ? v : sqrt(v);
    }
}

/* ---- GEMM S = Q * C^T (metrics.rs:204-255 / :160-202), k-ordered FMA chain.
 * C is transposed once (D x N) so the inner loop vectorises over j while each
 * output element still sees exactly fma(q[k], c[k], acc) for k = 0..D-1. */
#define JB 256
#define IB 4
void oracle_gemm_f32(const float *q, int64_t m, const float *c, int64_t n, int64_t d,
                     float *s, int nthreads) {
    float *ct = (float *)malloc(sizeof(float) * (size_t)(n * d));
#ifdef _OPENMP
    if (nthreads <= 0) nthreads = omp_get_max_threads();
#pragma omp parallel for num_threads(nthreads) schedule(static)
#endif
    for (int64_t j = 0; j < n; j++)
        for (int64_t kk = 0; kk < d; kk++) ct[kk * n + j] = c[j * d + kk];

    int64_t nib = (m + IB - 1) / IB, njb = (n + JB - 1) / JB;
#ifdef _OPENMP
#pragma omp parallel for num_threads(nthreads) schedule(dynamic, 1) collapse(2)
#endif
    for (int64_t ib = 0; ib < nib; ib++) {
        for (int64_t jb = 0; jb < njb; jb++) {
            float acc[IB][JB];
            int64_t i0 = ib * IB, j0 = jb * JB;
            int64_t ni = (m - i0) < IB ? (m - i0) : IB;
            int64_t nj = (n - j0) < JB ? (n - j0) : JB;
            memset(acc, 0, sizeof(acc));
            for (int64_t kk = 0; kk < d; kk++) {
                const float *crow = ct + kk * n + j0;
                for (int64_t r = 0; r < ni; r++) {
                    float a = q[(i0 + r) * d + kk];
                    float *ar = acc[r];
                    for (int64_t j = 0; j < nj; j++) ar[j] = fmaf(a, crow[j], ar[j]);
                }
            }
            for (int64_t r = 0; r < ni; r++)
                memcpy(s + (i0 + r) * n + j0, acc[r], sizeof(float) * (size_t)nj);
        }
    }
    free(ct);
}

void oracle_gemm_f64(const double *q, int64_t m, const double *c, int64_t n, int64_t d,
                     double *s, int nthreads) {
    double *ct = (double *)malloc(sizeof(double) * (size_t)(n * d));
#ifdef _OPENMP
    if (nthreads <= 0) nthreads = omp_get_max_threads();
#pragma omp parallel for num_threads(nthreads) schedule(static)
#endif
    for (int64_t j = 0; j < n; j++)
        for (int64_t kk = 0; kk < d; kk++) ct[kk * n + j] = c[j * d + kk];
    int64_t nib = (m + IB - 1) / IB, njb = (n + JB - 1) / JB;
#ifdef _OPENMP
#pragma omp parallel for num_threads(nthreads) schedule(dynamic, 1) collapse(2)
#endif
    for (int64_t ib = 0; ib < nib; ib++) {
        for (int64_t jb = 0; jb < njb; jb++) {
            double acc[IB][JB];
            int64_t i0 = ib * IB, j0 = jb * JB;
            int64_t ni = (m - i0) < IB ? (m - i0) : IB;
            int64_t nj = (n - j0) < JB ? (n - j0) : JB;
            memset(acc, 0, sizeof(acc));
            for (int64_t kk = 0; kk < d; kk++) {
                const double *crow = ct + kk * n + j0;
                for (int64_t r = 0; r < ni; r++) {
                    double a = q[(i0 + r) * d + kk];
                    double *ar = acc[r];
                    for (int64_t j = 0; j < nj; j++) ar[j] = fma(a, crow[j], ar[j]);
                }
            }
            for (int64_t r = 0; r < ni; r++)
                memcpy(s + (i0 + r) * n + j0, acc[r], sizeof(double) * (size_t)nj);
        }
    }
    free(ct);
}

/* ---- epilogue, metrics.rs:329-343 (cosine f32) and :347-362 (euclid f32) ---- */
void oracle_epilogue_f32(float *s, int64_t m, int64_t n, int metric,
                         const float *qn, const float *cn) {
    if (metric == METRIC_COSINE) {
        for (int64_t i = 0; i < m; i++) {
            float q = qn[i];
            float *row = s + i * n;
            if (q > 1e-6f) {
                for (int64_t j = 0; j < n; j++) {
                    float c = cn[j];
                    if (c > 1e-6f) row[j] /= q * c;
                    else row[j] = 0.0f;
                }
            } else {
                for (int64_t j = 0; j < n; j++) row[j] = 0.0f;
            }
        }
    } else if (metric == METRIC_EUCLIDEAN) {
        for (int64_t i = 0; i < m; i++) {
            float *row = s + i * n;
            for (int64_t j = 0; j < n; j++) {
                float sq = qn[i] + cn[j] - 2.0f * row[j];
                /* Rust f32::max: a NaN argument yields the other argument */
                float mx = (sq > 0.0f) ? sq : 0.0f;
                row[j] = sqrtf(mx);
            }
        }
    }
}

/* metrics.rs:276-308 (f64) */
void oracle_epilogue_f64(double *s, int64_t m, int64_t n, int metric,
                         const double *qn, const double *cn) {
    if (metric == METRIC_COSINE) {
        for (int64_t i = 0; i < m; i++) {
            double q = qn[i];
            double *row = s + i * n;
            if (q > 1e-10) {
                for (int64_t j = 0; j < n; j++) {
                    double c = cn[j];
                    if (c > 1e-10) row[j] /= q * c;
                    else row[j] = 0.0;
                }
            } else {
                for (int64_t j = 0; j < n; j++) row[j] = 0.0;
            }
        }
    } else if (metric == METRIC_EUCLIDEAN) {
        for (int64_t i = 0; i < m; i++) {
            double *row = s + i * n;
            for (int64_t j = 0; j < n; j++) {
                double sq = qn[i] + cn[j] - 2.0 * row[j];
                double mx = (sq > 0.0) ? sq : 0.0;
                row[j] = sqrt(mx);
            }
        }
    }
}

/* ---- total order used for selection ----
 * key: monotone map of the ranking value (score if higher_is_better, else
 * -score) onto unsigned integers; -0 is folded onto +0 and NaN maps to 0,
 * the lowest key, so NaN scores rank last.  Larger key = better; equal keys
 * break to the lower corpus index. */
typedef struct { uint64_t key; uint32_t idx; uint32_t pad; } ent_t;

static inline uint64_t okey_f32(float v) {
    if (v != v) return 0;
    if (v == 0.0f) v = 0.0f;
    uint32_t u;
    memcpy(&u, &v, 4);
    u = (u & 0x80000000u) ? ~u : (u | 0x80000000u);
    return (uint64_t)u;
}
static inline uint64_t okey_f64(double v) {
    if (v != v) return 0;
    if (v == 0.0) v = 0.0;
    uint64_t u;
    memcpy(&u, &v, 8);
    u = (u & 0x8000000000000000ull) ? ~u : (u | 0x8000000000000000ull);
    return u;
}
static inline int better(const ent_t *a, const ent_t *b) {
    return a->key > b->key || (a->key == b->key && a->idx < b->idx);
}
static int cmp_ent(const void *pa, const void *pb) {
    const ent_t *a = (const ent_t *)pa, *b = (const ent_t *)pb;
    if (better(a, b)) return -1;
    if (better(b, a)) return 1;
    return 0;
}

/* quickselect: put the k best entries in e[0..k) (unordered) */
static void select_k(ent_t *e, int64_t n, int64_t k) {
    int64_t lo = 0, hi = n - 1;
    uint64_t rng = 0x9E3779B97F4A7C15ull;
    while (lo < hi) {
        rng ^= rng << 13; rng ^= rng >> 7; rng ^= rng << 17;
        int64_t p = lo + (int64_t)(rng % (uint64_t)(hi - lo + 1));
        ent_t piv = e[p];
        e[p] = e[hi]; e[hi] = piv;
        int64_t st = lo;
        for (int64_t i = lo; i < hi; i++) {
            if (better(&e[i], &piv)) { ent_t t = e[i]; e[i] = e[st]; e[st] = t; st++; }
        }
        ent_t t = e[st]; e[st] = e[hi]; e[hi] = t;
        if (st == k - 1 || st == k) { if (st == k) { /* e[0..k) are the k best */ } return; }
        if (st < k) lo = st + 1; else hi = st - 1;
    }
}

/* topk.rs:42-75 select_topk_with_scores_f32 (single-threaded, per row) */
void oracle_select_topk_f32(const float *s, int64_t m, int64_t n, int64_t k,
                            int higher_is_better, uint32_t *out_idx, float *out_score) {
    if (k <= 0 || n <= 0) return;
    ent_t *e = (ent_t *)malloc(sizeof(ent_t) * (size_t)n);
    for (int64_t i = 0; i < m; i++) {
        const float *row = s + i * n;
        for (int64_t j = 0; j < n; j++) {
            float v = higher_is_better ? row[j] : -row[j];
            e[j].key = okey_f32(v);
            e[j].idx = (uint32_t)j;
        }
        if (k < n) select_k(e, n, k);
        qsort(e, (size_t)k, sizeof(ent_t), cmp_ent);
        for (int64_t j = 0; j < k; j++) {
            out_idx[i * k + j] = e[j].idx;
            out_score[i * k + j] = row[e[j].idx];
        }
    }
    free(e);
}

/* topk.rs:6-39 select_topk_with_scores (f64) */
void oracle_select_topk_f64(const double *s, int64_t m, int64_t n, int64_t k,
                            int higher_is_better, uint32_t *out_idx, double *out_score) {
    if (k <= 0 || n <= 0) return;
    ent_t *e = (ent_t *)malloc(sizeof(ent_t) * (size_t)n);
    for (int64_t i = 0; i < m; i++) {
        const double *row = s + i * n;
        for (int64_t j = 0; j < n; j++) {
            double v = higher_is_better ? row[j] : -row[j];
            e[j].key = okey_f64(v);
            e[j].idx = (uint32_t)j;
        }
        if (k < n) select_k(e, n, k);
        qsort(e, (size_t)k, sizeof(ent_t), cmp_ent);
        for (int64_t j = 0; j < k; j++) {
            out_idx[i * k + j] = e[j].idx;
            out_score[i * k + j] = row[e[j].idx];
        }
    }
    free(e);
}

/* ---- the reference's per-row select with Rust's own algorithm (timing) ----
 * src/topk.rs:42-75 per row: a Vec<(usize, f32)> of all N entries (16 bytes
 * each), `select_nth_unstable_by(k - 1, cmp)`, `truncate(k)`, a stable
 * `sort_by(cmp)`, with cmp = partial_cmp -> Equal (so is_less(a, b) is
 * a.score > b.score for higher-is-better, a.score < b.score otherwise; false
 * whenever a NaN is involved).  select_nth_unstable_by lives in Rust's core
 * library (core::slice::select, the toolchain's, not vendored; recalled):
 * introselect over at most 16 rounds of
 *   - pivot: choose_pivot -- median of 3 at len/8 * {0, 4, 7}, recursively
 *     (median3_rec) for len >= 64;
 *   - partition: swap the pivot to the front, a branchless cyclic Lomuto pass
 *     over the rest (each element moved into the left run, the displaced
 *     element into the previous position: two moves per element, the
 *     comparison result added to the run length), pivot swapped to the
 *     boundary;
 *   - a chosen pivot not less than the previous round's pivot (runs of equal
 *     keys): partition by <= and skip the equal run;
 *   - len <= 16: insertion sort; index 0 / len - 1: a min / max scan;
 * then a deterministic fallback (median of medians in Rust; a full sort
 * here -- never reached on the benchmark's random rows).  This is the
 * CPU baseline's select (oracle.topk_blas, bench.py); the checker keeps
 * select_k above and its fixed total order.  The two differ only in the
 * order of equal scores, which the reference leaves unspecified. */
typedef struct { uint64_t idx; float s; uint32_t pad; } rs_ent;  /* (usize, f32) */
typedef struct { double s; uint64_t idx; } rs_ent64;            /* (usize, f64) */

#define RS_SELECT_IMPL(NAME, T)                                                              \
static inline int NAME##_lt(const T *a, const T *b, int desc) {                              \
    return desc ? (a->s > b->s) : (a->s < b->s);                                             \
}                                                                                            \
static inline int NAME##_le(const T *a, const T *b, int desc) { /* !is_less(b, a) */         \
    return !NAME##_lt(b, a, desc);                                                           \
}                                                                                            \
static void NAME##_insertion(T *v, size_t len, int desc) {                                   \
    for (size_t i = 1; i < len; i++) {                                                       \
        T x = v[i];                                                                          \
        size_t j = i;                                                                        \
        while (j > 0 && NAME##_lt(&x, &v[j - 1], desc)) { v[j] = v[j - 1]; j--; }            \
        v[j] = x;                                                                            \
    }                                                                                        \
}                                                                                            \
static const T *NAME##_med3(const T *a, const T *b, const T *c, int desc) {                  \
    int x = NAME##_lt(a, b, desc), y = NAME##_lt(a, c, desc);                                \
    if (x == y) { int z = NAME##_lt(b, c, desc); return (z ^ x) ? c : b; }                   \
    return a;                                                                                \
}                                                                                            \
static const T *NAME##_med3_rec(const T *a, const T *b, const T *c, size_t n, int desc) {    \
    if (n * 8 >= 64) {                                                                       \
        size_t n8 = n / 8;                                                                   \
        a = NAME##_med3_rec(a, a + n8 * 4, a + n8 * 7, n8, desc);                            \
        b = NAME##_med3_rec(b, b + n8 * 4, b + n8 * 7, n8, desc);                            \
        c = NAME##_med3_rec(c, c + n8 * 4, c + n8 * 7, n8, desc);                            \
    }                                                                                        \
    return NAME##_med3(a, b, c, desc);                                                       \
}                                                                                            \
static size_t NAME##_choose_pivot(const T *v, size_t len, int desc) {                        \
    size_t n8 = len / 8;                                                                     \
    const T *p = len < 64 ? NAME##_med3(v, v + n8 * 4, v + n8 * 7, desc)                     \
                          : NAME##_med3_rec(v, v + n8 * 4, v + n8 * 7, n8, desc);            \
    return (size_t)(p - v);                                                                  \
}                                                                                            \
/* v[0] = pivot; cyclic branchless Lomuto over v[1..len); returns num_lt      \
 * (one loop per (direction, <= vs <) so the comparison is branch-free) */                   \
static inline __attribute__((always_inline)) size_t NAME##_part_body(T *w, size_t n, const T *pv, \
                                                                     const int desc, const int le) { \
    size_t num_lt = 0;                                                                       \
    if (n == 0) return 0;                                                                    \
    const T saved = w[0];                                                                    \
    T *gap = w;                                                                              \
    for (size_t i = 1; i < n; i++) {                                                         \
        T *r = w + i;                                                                        \
        const int lt = le ? NAME##_le(r, pv, desc) : NAME##_lt(r, pv, desc);                 \
        T *left = w + num_lt;                                                                \
        *gap = *left;                                                                        \
        *left = *r;                                                                          \
        gap = r;                                                                             \
        num_lt += (size_t)lt;                                                                \
    }                                                                                        \
    const int lt = le ? NAME##_le(&saved, pv, desc) : NAME##_lt(&saved, pv, desc);           \
    T *left = w + num_lt;                                                                    \
    *gap = *left;                                                                            \
    *left = saved;                                                                           \
    return num_lt + (size_t)lt;                                                              \
}                                                                                            \
static size_t NAME##_partition(T *v, size_t len, size_t piv, int desc, int le) {            \
    T t = v[0]; v[0] = v[piv]; v[piv] = t;                                                   \
    const T pv = v[0];                                                                       \
    size_t num_lt;                                                                           \
    if (desc) num_lt = le ? NAME##_part_body(v + 1, len - 1, &pv, 1, 1)                      \
                          : NAME##_part_body(v + 1, len - 1, &pv, 1, 0);                     \
    else num_lt = le ? NAME##_part_body(v + 1, len - 1, &pv, 0, 1)                           \
                     : NAME##_part_body(v + 1, len - 1, &pv, 0, 0);                          \
    t = v[0]; v[0] = v[num_lt]; v[num_lt] = t;                                               \
    return num_lt;                                                                           \
}                                                                                            \
static int NAME##_cmp_desc(const void *a, const void *b) {                                   \
    const T *x = (const T *)a, *y = (const T *)b;                                            \
    return NAME##_lt(x, y, 1) ? -1 : NAME##_lt(y, x, 1) ? 1 : 0;                             \
}                                                                                            \
static int NAME##_cmp_asc(const void *a, const void *b) {                                    \
    const T *x = (const T *)a, *y = (const T *)b;                                            \
    return NAME##_lt(x, y, 0) ? -1 : NAME##_lt(y, x, 0) ? 1 : 0;                             \
}                                                                                            \
static void NAME##_select_nth(T *v, size_t len, size_t index, int desc) {                    \
    if (index >= len) return;                                                                \
    if (index == len - 1 || index == 0) {                                                    \
        /* max_index / min_index scan: the last (first) position by is_less */               \
        size_t best = 0;                                                                     \
        for (size_t i = 1; i < len; i++)                                                     \
            if (index == 0 ? NAME##_lt(&v[i], &v[best], desc) : !NAME##_lt(&v[i], &v[best], desc)) \
                best = i;                                                                    \
        T t = v[index]; v[index] = v[best]; v[best] = t;                                     \
        return;                                                                              \
    }                                                                                        \
    int limit = 16;                                                                          \
    const T *anc = NULL;                                                                     \
    T anc_v;                                                                                 \
    while (1) {                                                                              \
        if (len <= 16) { if (len >= 2) NAME##_insertion(v, len, desc); return; }             \
        if (limit == 0) {                                                                    \
            qsort(v, len, sizeof(T), desc ? NAME##_cmp_desc : NAME##_cmp_asc);               \
            return;                                                                          \
        }                                                                                    \
        limit--;                                                                             \
        size_t piv = NAME##_choose_pivot(v, len, desc);                                      \
        if (anc && !NAME##_lt(anc, &v[piv], desc)) {                                         \
            size_t num_le = NAME##_partition(v, len, piv, desc, 1);                          \
            if (index <= num_le) return;                                                     \
            v += num_le + 1; len -= num_le + 1; index -= num_le + 1;                         \
            anc = NULL;                                                                      \
            continue;                                                                        \
        }                                                                                    \
        size_t num_lt = NAME##_partition(v, len, piv, desc, 0);                              \
        if (index < num_lt) { len = num_lt; }                                                \
        else if (index > num_lt) {                                                           \
            anc_v = v[num_lt]; anc = &anc_v;                                                 \
            v += num_lt + 1; len -= num_lt + 1; index -= num_lt + 1;                         \
        } else return;                                                                       \
    }                                                                                        \
}                                                                                            \
/* stable sort of the k kept (Rust's sort_by: insertion sort for short runs) */             \
static void NAME##_stable_sort(T *v, size_t len, T *tmp, int desc) {                         \
    if (len <= 20) { NAME##_insertion(v, len, desc); return; }                               \
    size_t h = len / 2;                                                                      \
    NAME##_stable_sort(v, h, tmp, desc);                                                     \
    NAME##_stable_sort(v + h, len - h, tmp, desc);                                           \
    memcpy(tmp, v, h * sizeof(T));                                                           \
    size_t i = 0, j = h, o = 0;                                                              \
    while (i < h && j < len) v[o++] = NAME##_lt(&v[j], &tmp[i], desc) ? v[j++] : tmp[i++];   \
    while (i < h) v[o++] = tmp[i++];                                                         \
}

RS_SELECT_IMPL(rs32, rs_ent)
RS_SELECT_IMPL(rs64, rs_ent64)

void oracle_select_topk_rs_f32(const float *s, int64_t m, int64_t n, int64_t k,
                               int higher_is_better, uint32_t *out_idx, float *out_score) {
    if (k <= 0 || n <= 0) return;
    rs_ent *e = (rs_ent *)malloc(sizeof(rs_ent) * (size_t)n);
    rs_ent *tmp = (rs_ent *)malloc(sizeof(rs_ent) * (size_t)k);
    for (int64_t i = 0; i < m; i++) {
        const float *row = s + i * n;
        for (int64_t j = 0; j < n; j++) { e[j].idx = (uint64_t)j; e[j].s = row[j]; }  /* enumerate().collect() */
        rs32_select_nth(e, (size_t)n, (size_t)(k - 1), higher_is_better);
        rs32_stable_sort(e, (size_t)k, tmp, higher_is_better);
        for (int64_t j = 0; j < k; j++) {
            out_idx[i * k + j] = (uint32_t)e[j].idx;
            out_score[i * k + j] = e[j].s;
        }
    }
    free(tmp);
    free(e);
}

void oracle_select_topk_rs_f64(const double *s, int64_t m, int64_t n, int64_t k,
                               int higher_is_better, uint32_t *out_idx, double *out_score) {
    if (k <= 0 || n <= 0) return;
    rs_ent64 *e = (rs_ent64 *)malloc(sizeof(rs_ent64) * (size_t)n);
    rs_ent64 *tmp = (rs_ent64 *)malloc(sizeof(rs_ent64) * (size_t)k);
    for (int64_t i = 0; i < m; i++) {
        const double *row = s + i * n;
        for (int64_t j = 0; j < n; j++) { e[j].idx = (uint64_t)j; e[j].s = row[j]; }
        rs64_select_nth(e, (size_t)n, (size_t)(k - 1), higher_is_better);
        rs64_stable_sort(e, (size_t)k, tmp, higher_is_better);
        for (int64_t j = 0; j < k; j++) {
            out_idx[i * k + j] = (uint32_t)e[j].idx;
            out_score[i * k + j] = e[j].s;
        }
    }
    free(tmp);
    free(e);
}

/* metrics.rs:314-365 compute_similarity_matrix_f32 into caller buffer s (m*n) */
void oracle_similarity_f32(const float *q, int64_t m, const float *c, int64_t n, int64_t d,
                           int metric, float *s, int nthreads) {
    float *qn = NULL, *cn = NULL;
    if (metric != METRIC_DOT) {
        int sq = metric == METRIC_EUCLIDEAN;
        qn = (float *)malloc(sizeof(float) * (size_t)(m > 0 ? m : 1));
        cn = (float *)malloc(sizeof(float) * (size_t)(n > 0 ? n : 1));
        oracle_norms_f32(q, m, d, sq, qn);
        oracle_norms_f32(c, n, d, sq, cn);
    }
    oracle_gemm_f32(q, m, c, n, d, s, nthreads);
    if (metric != METRIC_DOT) oracle_epilogue_f32(s, m, n, metric, qn, cn);
    free(qn);
    free(cn);
}

void oracle_similarity_f64(const double *q, int64_t m, const double *c, int64_t n, int64_t d,
                           int metric, double *s, int nthreads) {
    double *qn = NULL, *cn = NULL;
    if (metric != METRIC_DOT) {
        int sq = metric == METRIC_EUCLIDEAN;
        qn = (double *)malloc(sizeof(double) * (size_t)(m > 0 ? m : 1));
        cn = (double *)malloc(sizeof(double) * (size_t)(n > 0 ? n : 1));
        oracle_norms_f64(q, m, d, sq, qn);
        oracle_norms_f64(c, n, d, sq, cn);
    }
    oracle_gemm_f64(q, m, c, n, d, s, nthreads);
    if (metric != METRIC_DOT) oracle_epilogue_f64(s, m, n, metric, qn, cn);
    free(qn);
    free(cn);
}

/* matmul.rs:420-448 compute_topk_indices_scores, f32 branch.  k is clipped to n
 * by the caller convention (matmul.rs:443); returns the clipped k.  Scores are
 * widened to f64 as matmul.rs:447 does. */
int64_t oracle_topk_f32(const float *q, int64_t m, const float *c, int64_t n, int64_t d,
                        int64_t k, int metric, int nthreads, uint32_t *out_idx, double *out_score) {
    if (k > n) k = n;
    if (m <= 0 || k <= 0) return k;
    float *s = (float *)malloc(sizeof(float) * (size_t)(m * n));
    float *sc = (float *)malloc(sizeof(float) * (size_t)(m * k));
    oracle_similarity_f32(q, m, c, n, d, metric, s, nthreads);
    oracle_select_topk_f32(s, m, n, k, oracle_higher_is_better(metric), out_idx, sc);
    for (int64_t i = 0; i < m * k; i++) out_score[i] = (double)sc[i];
    free(sc);
    free(s);
    return k;
}

int64_t oracle_topk_f64(const double *q, int64_t m, const double *c, int64_t n, int64_t d,
                        int64_t k, int metric, int nthreads, uint32_t *out_idx, double *out_score) {
    if (k > n) k = n;
    if (m <= 0 || k <= 0) return k;
    double *s = (double *)malloc(sizeof(double) * (size_t)(m * n));
    oracle_similarity_f64(q, m, c, n, d, metric, s, nthreads);
    oracle_select_topk_f64(s, m, n, k, oracle_higher_is_better(metric), out_idx, out_score);
    free(s);
    return k;
}

/* Exact score of given (query row, corpus row) pairs, element by element the
 * value oracle_similarity_f32 would hold at S[i][idx[i][j]]: the same
 * k-ordered fmaf chain (metrics.rs:204-255 as restated above), the same
 * norms (metrics.rs:382-393) and epilogue (metrics.rs:314-365).  Used by the
 * full-size parity tests to re-score every returned (row, index) without
 * materialising the M x N matrix.  idx 0xFFFFFFFF (an empty slot) -> NaN. */
void oracle_pair_scores_f32(const float *q, int64_t m, const float *c, int64_t n, int64_t d,
                            int metric, const uint32_t *idx, int64_t k, int nthreads,
                            float *out) {
#ifdef _OPENMP
    if (nthreads <= 0) nthreads = omp_get_max_threads();
#pragma omp parallel for num_threads(nthreads) schedule(dynamic, 16)
#endif
    for (int64_t i = 0; i < m; i++) {
        const float *qr = q + i * d;
        const int sq = metric == METRIC_EUCLIDEAN;
        float qn = 0.0f;
        if (metric != METRIC_DOT) {
            qn = udot_f32(qr, qr, d);
            if (!sq) qn = sqrtf(qn);
        }
        for (int64_t j = 0; j < k; j++) {
            const uint32_t id = idx[i * k + j];
            if ((int64_t)id >= n) {
                out[i * k + j] = NAN;
                continue;
            }
            const float *cr = c + (int64_t)id * d;
            float acc = 0.0f;
            for (int64_t kk = 0; kk < d; kk++) acc = fmaf(qr[kk], cr[kk], acc);
            if (metric == METRIC_DOT) {
                out[i * k + j] = acc;
                continue;
            }
            float cn = udot_f32(cr, cr, d);
            if (!sq) cn = sqrtf(cn);
            float s = acc;
            oracle_epilogue_f32(&s, 1, 1, metric, &qn, &cn);
            out[i * k + j] = s;
        }
    }
}
