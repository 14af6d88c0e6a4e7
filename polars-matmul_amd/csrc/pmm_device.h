// pmm_device.h -- device-side building blocks shared by the gfx950 kernels
// (pmm_kernels.hip: f32 / f64 paths; pmm_bf16.hip: bf16 compute path):
// ordered selection keys, wave primitives, the reference-order norms and
// epilogue arithmetic, the pre-filter bound, buffer-resource LDS-DMA helpers
// and candidate-buffer compaction.  Not installed.
#pragma once
#include "pmm_internal.h"

#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>

namespace pmm {

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef double f64x4 __attribute__((ext_vector_type(4)));
typedef double f64x2 __attribute__((ext_vector_type(2)));
typedef unsigned long long u64;

#define LDS_AS __attribute__((address_space(3)))
#define GLB_AS __attribute__((address_space(1)))

// ===========================================================================
// Ordered keys.  The selection order is a total order on (score, index):
// best score first, NaN last, equal scores -> lower corpus index first.  A
// score maps to an unsigned key that is monotone in the ranking value
// (score for cosine/dot, -distance for euclidean); -0 folds onto +0 and NaN
// maps to 0.  A candidate is the 64-bit composite (key << 32) | ~index, so a
// single unsigned compare implements the whole order and every composite in
// a row is unique.
// ===========================================================================
__device__ __forceinline__ uint32_t okey32(float v) {
  if (v != v) return 0u;
  uint32_t u = __float_as_uint(v);
  if ((u << 1) == 0u) u = 0u;
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
__device__ __forceinline__ float dekey32(uint32_t k) {
  if (k == 0u) return __uint_as_float(0x7FC00000u);
  return __uint_as_float((k & 0x80000000u) ? (k & 0x7FFFFFFFu) : ~k);
}
__device__ __forceinline__ u64 okey64(double v) {
  if (v != v) return 0ull;
  u64 u = (u64)__double_as_longlong(v);
  if ((u << 1) == 0ull) u = 0ull;
  return (u & 0x8000000000000000ull) ? ~u : (u | 0x8000000000000000ull);
}
__device__ __forceinline__ double dekey64(u64 k) {
  if (k == 0ull) return __longlong_as_double(0x7FF8000000000000ll);
  return __longlong_as_double((long long)((k & 0x8000000000000000ull) ? (k & 0x7FFFFFFFFFFFFFFFull) : ~k));
}

// ===========================================================================
// Wave primitives (wave64).
// ===========================================================================
__device__ __forceinline__ void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  asm volatile("" ::: "memory");
}
__device__ __forceinline__ int lanes_below(u64 mask) {
  return (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(mask >> 32),
                                        __builtin_amdgcn_mbcnt_lo((uint32_t)mask, 0u));
}

// Bitonic sort, best (largest) first, of P (power of two) u64 in LDS by one wave.
__device__ inline void wave_sort_desc_u64(u64 *s, int P, int lane) {
  for (int size = 2; size <= P; size <<= 1) {
    for (int stride = size >> 1; stride > 0; stride >>= 1) {
      for (int i = lane; i < (P >> 1); i += 64) {
        const int x0 = ((i & ~(stride - 1)) << 1) | (i & (stride - 1));
        const int x1 = x0 + stride;
        const u64 a = s[x0], b = s[x1];
        const bool desc = (x0 & size) == 0;
        if (desc ? (a < b) : (a > b)) {
          s[x0] = b;
          s[x1] = a;
        }
      }
      wave_sync();
    }
  }
}

__device__ __forceinline__ u64 wave_max_u64(u64 v) {
#pragma unroll
  for (int o = 32; o; o >>= 1) {
    const u64 w = __shfl_xor(v, o);
    v = v > w ? v : w;
  }
  return v;
}
__device__ __forceinline__ u64 wave_min_u64(u64 v) {
#pragma unroll
  for (int o = 32; o; o >>= 1) {
    const u64 w = __shfl_xor(v, o);
    v = v < w ? v : w;
  }
  return v;
}
// Exact k-th largest of the keys a wave holds E per lane (0 = empty slot;
// at least k non-empty), by bitwise construction from the most significant
// bit where the keys differ: the largest v with #{x >= v} >= k, stopping as
// soon as exactly k keys are >= v (the k-th is then the least of them).  One
// compare per key and one popcount per 64 keys per bit, no LDS: far cheaper
// than sorting the buffer to find one rank.  The keys of one row are
// distinct (the corpus index rides in the low bits).
// The wave-wide reductions' results as scalars (every lane holds the same
// value; the compiler cannot prove it): the bit loop below then runs on
// scalar bounds and scalar control flow instead of per-lane copies under
// exec-mask bookkeeping (8 vector instructions per bit at E = 8, was 15).
// Round 6, alternated on one box (profiles/r6_merge/kth_uniform_ab.txt):
// c4 kernel 131.3 / 131.5 -> 130.9 / 130.9 ms (its compactions), merges
// and c3 unchanged.  Callers run the selection with the whole wave active.
__device__ __forceinline__ u64 wave_uniform_u64(u64 v) {
  // (the builtin returns int: through uint32_t, or the low word sign-extends)
  return ((u64)(uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)(v >> 32)) << 32) |
         (u64)(uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)v);
}
__device__ __forceinline__ uint32_t wave_uniform_u32(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_readfirstlane(v);
}
template <int E>
__device__ inline u64 wave_kth_u64(const u64 (&x)[E], int k) {
  u64 mx = 0ull, mn = ~0ull;
#pragma unroll
  for (int e = 0; e < E; e++) {
    if (x[e] > mx) mx = x[e];
    if (x[e] != 0ull && x[e] < mn) mn = x[e];
  }
  mx = wave_uniform_u64(wave_max_u64(mx));
  mn = wave_uniform_u64(wave_min_u64(mn));
  if (mx == 0ull) return 0ull;
  const u64 diff = mx ^ mn;
  int b = diff ? 63 - __builtin_clzll(diff) : -1;
  u64 v = (b >= 0) ? (mx & ~((2ull << b) - 1ull)) : mx;  // the keys' common prefix
  for (; b >= 0; b--) {
    const u64 c = v | (1ull << b);
    int cnt = 0;
#pragma unroll
    for (int e = 0; e < E; e++) cnt += __popcll(__ballot(x[e] >= c));
    if (cnt >= k) {
      v = c;
      if (cnt == k) break;
    }
  }
  u64 t = ~0ull;
#pragma unroll
  for (int e = 0; e < E; e++)
    if (x[e] >= v && x[e] < t) t = x[e];
  return wave_min_u64(t);
}
// The same selection over 32-bit keys (0 = empty): the largest v with
// #{x >= v} >= k, i.e. the k-th largest key (ties allowed).  Half the compare
// work of the 64-bit form; the threshold seeds use it on the score part of
// their composite keys (a lower bound of the composite k-th is all they need).
template <int E>
__device__ inline uint32_t wave_kth_u32(const uint32_t (&x)[E], int k) {
  uint32_t mx = 0u, mn = ~0u;
#pragma unroll
  for (int e = 0; e < E; e++) {
    mx = x[e] > mx ? x[e] : mx;
    if (x[e] != 0u && x[e] < mn) mn = x[e];
  }
#pragma unroll
  for (int o = 32; o; o >>= 1) {
    const uint32_t a = __shfl_xor(mx, o), c = __shfl_xor(mn, o);
    mx = a > mx ? a : mx;
    mn = c < mn ? c : mn;
  }
  mx = wave_uniform_u32(mx);
  mn = wave_uniform_u32(mn);
  if (mx == 0u) return 0u;
  const uint32_t diff = mx ^ mn;
  int b = diff ? 31 - __builtin_clz(diff) : -1;
  uint32_t v = (b >= 0) ? (mx & ~((2u << b) - 1u)) : mx;  // (b = 31: 2u << 31 wraps to 0, v = 0)
  for (; b >= 0; b--) {
    const uint32_t c = v | (1u << b);
    int cnt = 0;
#pragma unroll
    for (int e = 0; e < E; e++) cnt += __popcll(__ballot(x[e] >= c));
    if (cnt >= k) {
      v = c;
      if (cnt == k) break;
    }
  }
  uint32_t t = ~0u;
#pragma unroll
  for (int e = 0; e < E; e++)
    if (x[e] >= v && x[e] < t) t = x[e];
#pragma unroll
  for (int o = 32; o; o >>= 1) {
    const uint32_t a = __shfl_xor(t, o);
    t = a < t ? a : t;
  }
  return t;
}
// Seeded threshold from the score part of a row's sample keys: every key
// whose score key is at least the k-th largest passes ((kth << 32) - 1 is
// below each of them, whatever its index part), so it is an exact lower bound
// of the row's final k-th composite.  0 (accept all) when the sample has fewer
// than k scores that are not NaN.
template <int E>
__device__ __forceinline__ u64 seed_threshold(const u64 (&x)[E], int k) {
  uint32_t h[E];
  int nz = 0;
#pragma unroll
  for (int e = 0; e < E; e++) {
    h[e] = (uint32_t)(x[e] >> 32);
    nz += __popcll(__ballot(h[e] != 0u));
  }
  if (nz < k) return 0ull;
  const uint32_t t = wave_kth_u32<E>(h, k);
  return t ? ((u64)t << 32) - 1ull : 0ull;
}

// Store the non-empty keys >= t of x packed (lane order) through st(pos, key);
// returns their count.
template <int E, typename Store>
__device__ inline int wave_keep_ge(const u64 (&x)[E], u64 t, Store st, int lane) {
  int base = 0;
  const u64 t1 = t ? t : 1ull;  // (x >= max(t, 1): x != 0 and x >= t in one compare)
#pragma unroll
  for (int e = 0; e < E; e++) {
    const bool keep = x[e] >= t1;
    const u64 m = __ballot(keep);
    if (keep) st(base + lanes_below(m), x[e]);
    base += __popcll(m);
  }
  return base;
}

// 16-byte entry for the materialised (row-select) path: f64 keys need all
// 64 bits, so the index rides alongside.
struct __attribute__((aligned(16))) Ent {
  u64 key;
  uint32_t idx;
  uint32_t pad;
};
__device__ __forceinline__ bool ent_better(const Ent &a, const Ent &b) {
  return a.key > b.key || (a.key == b.key && a.idx < b.idx);
}
__device__ inline void wave_sort_desc_ent(Ent *s, int P, int lane) {
  for (int size = 2; size <= P; size <<= 1) {
    for (int stride = size >> 1; stride > 0; stride >>= 1) {
      for (int i = lane; i < (P >> 1); i += 64) {
        const int x0 = ((i & ~(stride - 1)) << 1) | (i & (stride - 1));
        const int x1 = x0 + stride;
        const Ent a = s[x0], b = s[x1];
        const bool desc = (x0 & size) == 0;
        if (desc ? ent_better(b, a) : ent_better(a, b)) {
          s[x0] = b;
          s[x1] = a;
        }
      }
      wave_sync();
    }
  }
}

__device__ __forceinline__ int next_pow2_dev(int x) {
  int p = 64;
  while (p < x) p <<= 1;
  return p;
}

// ===========================================================================
// Row norms in ndarray's `unrolled_dot` order (src/metrics.rs:368-393 ->
// ndarray 0.16 unrolled_dot): accumulator j sums x[8t+j]^2 sequentially,
// combined as ((((0+(p0+p4))+(p1+p5))+(p2+p6))+(p3+p7)) then the scalar tail.
// 8 lanes per row, lane j owns accumulator p_j -> bit-identical to the
// reference's norms (no FMA: the file is built with -ffp-contract=off).
// ===========================================================================
template <typename T>
__device__ __forceinline__ T sqrt_rn(T x);
// f32: __builtin_sqrtf (llvm.sqrt.f32, correctly rounded under hipcc's default
// -fhip-fp32-correctly-rounded-divide-sqrt), as Rust's f32::sqrt.  NOT
// __fsqrt_rn: without OCML_BASIC_ROUNDED_OPERATIONS that is the 1-ulp native
// v_sqrt_f32 (it differed from the oracle on 15% of norms).
template <>
__device__ __forceinline__ float sqrt_rn<float>(float x) { return __builtin_sqrtf(x); }
template <>
__device__ __forceinline__ double sqrt_rn<double>(double x) { return __dsqrt_rn(x); }

// TI = stored element type (f32, f64, or bf16 for the bf16 compute path, whose
// norms are those of the bf16-rounded rows, accumulated in f32).
// 8 lanes per row; gt = the thread's index over this array's rows * 8.
template <typename T, typename TI = T>
__device__ __forceinline__ void norms_rows(const TI *__restrict__ a, int64_t rows, int64_t d,
                                           int64_t ld, int squared, T *__restrict__ out,
                                           T *__restrict__ inv, int64_t gt) {
  const int64_t row = gt >> 3;
  const int j = threadIdx.x & 7;
  const bool valid = row < rows;
  const TI *p = a + (valid ? row : 0) * ld;
  const int64_t d8 = d & ~(int64_t)7;
  T acc = (T)0;
  if (valid) {
    // 8 loads in flight per lane (a plain loop waited for each: 32 exposed
    // latencies per row at d = 256); the sum keeps its order
    int64_t i = j;
    for (; i + 56 < d8; i += 64) {
      T x[8];
#pragma unroll
      for (int u = 0; u < 8; u++) x[u] = (T)p[i + 8 * u];
#pragma unroll
      for (int u = 0; u < 8; u++) acc = acc + x[u] * x[u];
    }
    for (; i < d8; i += 8) {
      const T x = (T)p[i];
      acc = acc + x * x;
    }
  }
  const int base = (int)(threadIdx.x & 63) & ~7;
  T pp[8];
#pragma unroll
  for (int t = 0; t < 8; t++) pp[t] = __shfl(acc, base + t, 64);
  if (valid && j == 0) {
    T sum = (T)0;
    sum = sum + (pp[0] + pp[4]);
    sum = sum + (pp[1] + pp[5]);
    sum = sum + (pp[2] + pp[6]);
    sum = sum + (pp[3] + pp[7]);
    for (int64_t i = d8; i < d; i++) {
      const T x = (T)p[i];
      sum = sum + x * x;
    }
    const T v = squared ? sum : sqrt_rn<T>(sum);
    out[row] = v;
    // pre-filter column factor (see prefilter_bound): cosine 1/norm (0 for the
    // reference's zero-norm rule); euclidean the squared norm shrunk by 2^-18
    // so 2*dot - factor over-estimates qsq - sq by more than its rounding.
    if (inv) inv[row] = squared ? v * (T)(1.0 - 0x1p-18) : ((v > (T)1e-6) ? (T)1 / v : (T)0);
  }
}

template <typename T, typename TI = T>
__global__ __launch_bounds__(256) void norms_kernel(const TI *__restrict__ a, int64_t rows,
                                                    int64_t d, int64_t ld, int squared,
                                                    T *__restrict__ out, T *__restrict__ inv) {
  norms_rows<T, TI>(a, rows, d, ld, squared, out, inv, (int64_t)blockIdx.x * blockDim.x + threadIdx.x);
}

// Query and corpus norms in one launch: blocks [0, qblocks) take the query
// rows, blocks [qblocks, nblocks) the corpus rows (same arithmetic as two
// norms_kernel launches), and any blocks past nblocks zero `zn` 16-byte words
// at `zero` (the fused top-k's counters, so no separate fill launch).
template <typename T>
__global__ __launch_bounds__(256) void norms_pair_kernel(const T *__restrict__ q, int64_t m, int64_t ldq,
                                                         T *__restrict__ qout, const T *__restrict__ c,
                                                         int64_t n, int64_t ldc, T *__restrict__ cout,
                                                         T *__restrict__ cinv, int64_t d, int squared,
                                                         unsigned qblocks, unsigned nblocks,
                                                         uint4 *__restrict__ zero, int64_t zn) {
  if (blockIdx.x < qblocks) {
    norms_rows<T, T>(q, m, d, ldq, squared, qout, nullptr, (int64_t)blockIdx.x * blockDim.x + threadIdx.x);
  } else if (blockIdx.x < nblocks) {
    norms_rows<T, T>(c, n, d, ldc, squared, cout, cinv,
                     (int64_t)(blockIdx.x - qblocks) * blockDim.x + threadIdx.x);
  } else {
    const int64_t stride = (int64_t)(gridDim.x - nblocks) * blockDim.x;
    for (int64_t i = (int64_t)(blockIdx.x - nblocks) * blockDim.x + threadIdx.x; i < zn; i += stride)
      zero[i] = make_uint4(0u, 0u, 0u, 0u);
  }
}

// ===========================================================================
// Epilogue arithmetic, exactly as the reference orders it.
//   cosine   (metrics.rs:329-343): q>1e-6 && c>1e-6 ? dot / (q*c) : 0
//   euclid   (metrics.rs:347-362): sqrt(max((qsq + csq) - 2*dot, 0)),
//            Rust f32::max returns the non-NaN operand -> NaN becomes 0.
// ===========================================================================
template <int METRIC>
__device__ __forceinline__ float exact_score(float dot, float qv, float cv) {
  if (METRIC == kMetricDot) return dot;
  if (METRIC == kMetricCosine) {
    if (qv > 1e-6f && cv > 1e-6f) return __fdiv_rn(dot, __fmul_rn(qv, cv));
    return 0.0f;
  }
  const float sq = __fsub_rn(__fadd_rn(qv, cv), 2.0f * dot);
  const float mx = (sq > 0.0f) ? sq : 0.0f;
  return __builtin_sqrtf(mx);  // correctly rounded (see sqrt_rn)
}
template <int METRIC>
__device__ __forceinline__ double exact_score_f64(double dot, double qv, double cv) {
  if (METRIC == kMetricDot) return dot;
  if (METRIC == kMetricCosine) {
    if (qv > 1e-10 && cv > 1e-10) return __ddiv_rn(dot, __dmul_rn(qv, cv));
    return 0.0;
  }
  const double sq = __dsub_rn(__dadd_rn(qv, cv), 2.0 * dot);
  const double mx = (sq > 0.0) ? sq : 0.0;
  return __dsqrt_rn(mx);
}

// Pre-filter.  For every score the hot epilogue computes ONE value
//   dot:    pv = dot                     (exact)
//   cosine: pv = dot * (1/cn)            (= score * qn within 5 ulp)
//   euclid: pv = 2*dot - csq*(1-2^-18)   (>= qsq - sq - rounding)
// and keeps the element iff !(pv < L), with the per-row bound L derived from
// the row's current k-th composite `thr` and the row norm qv (cosine: ||q||,
// euclid: ||q||^2).  L is loose by a margin that covers every rounding step,
// so the pre-filter never rejects a true candidate; survivors are re-scored
// exactly and compared as composites.  NaN pv always passes (!(NaN < L)).
template <int METRIC>
__device__ __forceinline__ float prefilter_bound(u64 thr, float qv) {
  const float inf = __builtin_inff();
  if (thr == ~0ull) return inf;                 // padding row: reject all
  const uint32_t tk = (uint32_t)(thr >> 32);
  if (tk == 0u) return -inf;                    // row not full: accept all
  const float v = dekey32(tk);                  // ranking value of the k-th
  if (METRIC == kMetricDot) return v;
  if (METRIC == kMetricCosine) {
    if (!(qv > 1e-6f)) return (0.0f >= v) ? -inf : inf;  // zero-norm row: every score is 0
    const float lo = v - (fabsf(v) * 0x1p-19f + 0x1p-100f);
    const float L = lo * qv;
    return L - (fabsf(L) * 0x1p-20f + 0x1p-100f);
  }
  const float dist = -v;
  const float hi = dist * dist * (1.0f + 0x1p-20f) + 0x1p-100f;
  const float L = qv - hi;
  return L - ((fabsf(qv) + hi) * 0x1p-18f + 0x1p-100f);
}

// Pre-filter difference of one score (bf16 kernels): >= 0 (or NaN) iff the
// score may enter the row's top-k (see prefilter_bound); a rounded difference
// keeps the sign of the exact one.
template <int METRIC>
__device__ __forceinline__ float prefilter_diff(float v, float cv, float lo) {
  if (METRIC == kMetricDot) return v - lo;
  if (METRIC == kMetricCosine) return fmaf(v, cv, -lo);
  return fmaf(2.0f, v, -cv) - lo;
}

__device__ __forceinline__ int acc_row(int e, int h) { return (e & 3) + 8 * (e >> 2) + 4 * h; }

__device__ __forceinline__ __amdgpu_buffer_rsrc_t make_rsrc(const void *base, int64_t bytes) {
  const int nrec = bytes <= 0 ? 0 : (int)(bytes > 0x7FFFFFFFll ? 0x7FFFFFFFll : bytes);
  return __builtin_amdgcn_make_buffer_rsrc((void *)base, (short)0, nrec, 0x00020000);
}

__device__ __forceinline__ void dma16(__amdgpu_buffer_rsrc_t r, char *lds, uint32_t voff,
                                      uint32_t soff) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (LDS_AS void *)lds, 16, voff, soff, 0, 0);
}

// Wave-level compaction of one row's candidate buffer: sort, keep the best k,
// raise the row threshold to the k-th composite and publish it (atomicMax)
// so later units of the same row prune with it.
__device__ inline void compact_row(const GemmF32Args &a, int s, int grow, u64 *thr_slot,
                                   unsigned *cnt_slot, u64 *scr, int lane) {
  u64 *base = a.cand + ((int64_t)grow * a.S + s) * a.capg;
  const int n = (int)*cnt_slot;
  const int P = a.capg;
  if (P <= 512 && n > a.k) {
    // select, don't sort: the buffer is unordered; keep its best k and
    // raise the threshold to the k-th
    u64 x[8];
#pragma unroll
    for (int e = 0; e < 8; e++) {
      const int i = lane + 64 * e;
      x[e] = (i < n) ? __hip_atomic_load(base + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0ull;
    }
    const u64 nt = wave_kth_u64<8>(x, a.k);  // (the ballots consumed every load)
    wave_keep_ge<8>(x, nt, [&](int pos, u64 v) __attribute__((always_inline)) { base[pos] = v; }, lane);
    wave_sync();
    if (lane == 0) {
      *cnt_slot = (unsigned)a.k;
      if (nt > *thr_slot) *thr_slot = nt;
      atomicMax(a.gthr + grow, nt);
    }
    wave_sync();
    return;
  }
  for (int i = lane; i < P; i += 64)
    scr[i] = (i < n) ? __hip_atomic_load(base + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                     : 0ull;
  wave_sync();
  wave_sort_desc_u64(scr, P, lane);
  const int kk = min(a.k, n);
  for (int i = lane; i < kk; i += 64) base[i] = scr[i];
  const u64 nt = (n >= a.k) ? scr[a.k - 1] : 0ull;
  wave_sync();
  if (lane == 0) {
    *cnt_slot = (unsigned)kk;
    if (nt > *thr_slot) *thr_slot = nt;
    if (nt) atomicMax(a.gthr + grow, nt);
  }
  wave_sync();
}

}  // namespace pmm
