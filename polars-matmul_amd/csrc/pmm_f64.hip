// pmm_f64.hip -- the f64 branch of `.pmm.topk` without the M x N matrix:
// compute_similarity_matrix (src/metrics.rs:258-311: faer f64 GEMM, then
// cosine / euclidean in the reference's operation order with the 1e-10 norm
// threshold) + select_topk_with_scores (src/topk.rs:6-39), reached from
// src/matmul.rs:449-468 -- what every Polars Float64 column takes.
//
// The corpus is scanned in column chunks.  Each chunk is one launch of the
// f64 MFMA GEMM (v_mfma_f64_16x16x4_f64, K in natural order) whose epilogue
// computes the exact score of every element and appends it to its row's
// candidate buffer when it beats the row's threshold (the k-th best entry so
// far under the total order: score best-first, NaN last, lower index first);
// between chunks one wave per row sorts its buffer, keeps the best k and
// raises the threshold to the k-th.  Chunks grow with the columns seen, so a
// chunk is expected to add about g*k survivors per row (g chosen so the buffer
// stays half empty).  A row whose buffer overflows is reported and the call
// falls back to the materialised path (pmm_capi.hip), so the result is exact
// whatever the data.
#include "pmm_device.h"

namespace pmm {

__device__ __forceinline__ u64 f64_key(double v, int metric) {
  return okey64(metric == kMetricEuclidean ? -v : v);
}
__device__ __forceinline__ double f64_unkey(u64 k, int metric) {
  const double v = dekey64(k);
  return metric == kMetricEuclidean ? 0.0 - v : v;  // +0.0 for a zero distance
}

// ---------------------------------------------------------------------------
// GEMM + epilogue + threshold append.  64 x 64 tile per 4-wave workgroup, each
// wave 32 x 32 (2 x 2 MFMA tiles).  K step s of a 16-K chunk: lane (i = lane &
// 15, kq = lane >> 4) feeds A[row i][k0 + 4 s + kq] and B[col i][k0 + 4 s + kq],
// so the four MFMAs of a chunk see k0 .. k0 + 15 in natural order.  Operands
// load straight from global memory (L2), the next chunk's while this one's
// MFMAs run.  C/D layout: col = lane & 15, row = (lane >> 4) + 4 * reg.
// ---------------------------------------------------------------------------
template <int METRIC>
__global__ __launch_bounds__(256) void gemm_f64_topk_kernel(F64TopkArgs a) {
  constexpr bool XF = METRIC != kMetricDot;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int i = lane & 15, kq = lane >> 4;
  const int row0 = blockIdx.y * 64 + (wid >> 1) * 32;
  const int lc0 = blockIdx.x * 64 + (wid & 1) * 32;  // column within the chunk
  const double *ap[2], *bp[2];
#pragma unroll
  for (int t = 0; t < 2; t++) {
    ap[t] = a.q + (int64_t)min(row0 + 16 * t + i, a.M - 1) * a.ldq + kq;
    bp[t] = a.c + (int64_t)(a.col0 + min(lc0 + 16 * t + i, a.ncol - 1)) * a.ldc + kq;
  }
  f64x4 acc[2][2];
#pragma unroll
  for (int ti = 0; ti < 2; ti++)
#pragma unroll
    for (int tj = 0; tj < 2; tj++) acc[ti][tj] = (f64x4){0.0, 0.0, 0.0, 0.0};
  double av[2][4], bv[2][4];
#pragma unroll
  for (int t = 0; t < 2; t++)
#pragma unroll
    for (int s = 0; s < 4; s++) {
      av[t][s] = ap[t][4 * s];
      bv[t][s] = bp[t][4 * s];
    }
  for (int k0 = 0; k0 < a.D; k0 += 16) {
    double an[2][4], bn[2][4];
    const int kn = k0 + 16 < a.D ? k0 + 16 : k0;  // (the last chunk re-reads itself)
#pragma unroll
    for (int t = 0; t < 2; t++)
#pragma unroll
      for (int s = 0; s < 4; s++) {
        an[t][s] = ap[t][kn + 4 * s];
        bn[t][s] = bp[t][kn + 4 * s];
      }
#pragma unroll
    for (int s = 0; s < 4; s++)
#pragma unroll
      for (int ti = 0; ti < 2; ti++)
#pragma unroll
        for (int tj = 0; tj < 2; tj++)
          acc[ti][tj] = __builtin_amdgcn_mfma_f64_16x16x4f64(av[ti][s], bv[tj][s], acc[ti][tj], 0, 0, 0);
#pragma unroll
    for (int t = 0; t < 2; t++)
#pragma unroll
      for (int s = 0; s < 4; s++) {
        av[t][s] = an[t][s];
        bv[t][s] = bn[t][s];
      }
  }
  // epilogue: exact score, key, compare with the row's k-th, append
#pragma unroll
  for (int ti = 0; ti < 2; ti++)
#pragma unroll
    for (int r = 0; r < 4; r++) {
      const int row = row0 + 16 * ti + kq + 4 * r;
      if (row >= a.M) continue;
      const u64 tk = a.tkey[row];
      const uint32_t tx = a.tidx[row];
      const double qv = XF ? a.qn[row] : 0.0;
#pragma unroll
      for (int tj = 0; tj < 2; tj++) {
        const int lc = lc0 + 16 * tj + i;
        if (lc >= a.ncol) continue;
        const uint32_t gcol = (uint32_t)(a.col0 + lc);
        const double v = acc[ti][tj][r];
        const double sc = XF ? exact_score_f64<METRIC>(v, qv, a.cn[gcol]) : v;
        const u64 key = f64_key(sc, METRIC);
        if (key > tk || (key == tk && gcol < tx)) {
          const unsigned pos = atomicAdd(a.cnt + row, 1u);
          if (pos < (unsigned)a.cap) {
            Ent e;
            e.key = key;
            e.idx = gcol;
            e.pad = 0u;
            a.cand[(int64_t)row * a.cap + pos] = e;
          }
        }
      }
    }
}

hipError_t launch_gemm_f64_topk(const F64TopkArgs &a, hipStream_t s) {
  if (a.M <= 0 || a.ncol <= 0) return hipSuccess;
  const dim3 grid((a.ncol + 63) / 64, (a.M + 63) / 64), blk(256);
  if (a.metric == kMetricCosine) gemm_f64_topk_kernel<kMetricCosine><<<grid, blk, 0, s>>>(a);
  else if (a.metric == kMetricEuclidean) gemm_f64_topk_kernel<kMetricEuclidean><<<grid, blk, 0, s>>>(a);
  else gemm_f64_topk_kernel<kMetricDot><<<grid, blk, 0, s>>>(a);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------
// Per-row buffer select, one wave per row: sort the row's entries in LDS
// (bitonic over the next power of two), then
//   mode 0 (between chunks): keep the best k at the buffer's start, count =
//          min(count, k), threshold = the k-th entry (accept-all while fewer);
//   mode 1 (final): write the best k, best first (src/topk.rs:6-39 order).
// A count above the capacity means entries were dropped: *overflow is set and
// the host discards the result.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void f64_select_kernel(F64SelArgs a) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int wpb = blockDim.x >> 6;
  const int row = blockIdx.x * wpb + wid;
  if (row >= a.M) return;
  Ent *scr = (Ent *)smem + (size_t)wid * a.P;
  int n = (int)a.cnt[row];
  if (n > a.cap) {
    if (lane == 0) atomicOr(a.overflow, 1u);
    n = a.cap;
  }
  const int P2 = min(a.P, next_pow2_dev(n));
  const Ent* src = a.cand + (int64_t)row * a.cap;
  for (int j = lane; j < P2; j += 64) {
    Ent e;
    if (j < n) {
      e = src[j];
    } else {
      e.key = 0ull;
      e.idx = 0xFFFFFFFFu;
      e.pad = 0u;
    }
    scr[j] = e;
  }
  wave_sync();
  wave_sort_desc_ent(scr, P2, lane);
  const int kk = min(a.k, n);
  if (a.mode == 0) {
    Ent *dst = a.cand + (int64_t)row * a.cap;
    for (int j = lane; j < kk; j += 64) dst[j] = scr[j];
    if (lane == 0) {
      a.cnt[row] = (unsigned)kk;
      if (n >= a.k) {
        a.tkey[row] = scr[a.k - 1].key;
        a.tidx[row] = scr[a.k - 1].idx;
      } else {
        a.tkey[row] = 0ull;
        a.tidx[row] = 0xFFFFFFFFu;
      }
    }
  } else {
    for (int j = lane; j < a.k; j += 64) {
      const bool ok = j < kk;
      a.out_idx[(int64_t)row * a.k + j] = ok ? scr[j].idx + a.index_base : 0xFFFFFFFFu;
      a.out_score[(int64_t)row * a.k + j] = ok ? f64_unkey(scr[j].key, a.metric) : __longlong_as_double(0x7FF8000000000000ll);
    }
  }
}

// thresholds to accept-all, counts to 0
__global__ __launch_bounds__(256) void f64_reset_kernel(u64 *tkey, uint32_t *tidx, unsigned *cnt, int m,
                                                        unsigned *overflow) {
  const int r = blockIdx.x * blockDim.x + threadIdx.x;
  if (r == 0) *overflow = 0u;
  if (r < m) {
    tkey[r] = 0ull;
    tidx[r] = 0xFFFFFFFFu;
    cnt[r] = 0u;
  }
}

hipError_t launch_f64_reset(u64 *tkey, uint32_t *tidx, unsigned *cnt, int m, unsigned *overflow, hipStream_t s) {
  f64_reset_kernel<<<(m + 255) / 256, 256, 0, s>>>(tkey, tidx, cnt, m, overflow);
  return hipGetLastError();
}

hipError_t launch_f64_select(const F64SelArgs &a, hipStream_t s) {
  if (a.M <= 0) return hipSuccess;
  const size_t per_wave = (size_t)a.P * sizeof(Ent);
  int wpb = (int)(131072 / per_wave);
  wpb = wpb < 1 ? 1 : (wpb > 4 ? 4 : wpb);
  const size_t lds = (size_t)wpb * per_wave;
  static bool attr = false;
  if (!attr) {
    hipError_t e = hipFuncSetAttribute((const void *)f64_select_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                                       160 * 1024);
    if (e != hipSuccess) return e;
    attr = true;
  }
  f64_select_kernel<<<(unsigned)((a.M + wpb - 1) / wpb), wpb * 64, lds, s>>>(a);
  return hipGetLastError();
}

}  // namespace pmm
