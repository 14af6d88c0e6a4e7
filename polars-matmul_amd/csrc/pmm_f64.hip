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
// The f64 GEMM tile (store mode and the fused top-k share it, so both paths
// compute every dot product identically).  64 x 64 tile per 4-wave
// workgroup, each wave 32 x 32 = 2 x 2 v_mfma_f64_16x16x4_f64 tiles.  K runs
// in chunks of 16 through a double-buffered LDS image stored k-major
// (As[k][row]), so at K step s of a chunk lane (i = lane & 15, kq = lane >> 4)
// reads A[row i][k0 + 4 s + kq] and B[col i][k0 + 4 s + kq] with one
// ds_read_b64 each: the four MFMAs of a chunk see k0 .. k0 + 15 in natural
// order.  Rows of 16 + 64 doubles: the kq = 0 and kq = 1 half-waves of a read
// land on disjoint banks.  Global loads: each thread one 32-byte run (row t/4,
// k 4(t%4) .. +3) of A and of B per chunk, the next chunk's in flight while
// this chunk's MFMAs run.  C/D layout: col = lane & 15, row = (lane >> 4) + 4 reg.
// ---------------------------------------------------------------------------
constexpr int kF64LdsRow = 80;                              // doubles per LDS row (64 + pad)
constexpr int kF64LdsBuf = 16 * kF64LdsRow;                 // one operand's chunk

__device__ __forceinline__ void f64_tile(const double *__restrict__ q, int64_t ldq, int mrows,
                                         const double *__restrict__ c, int64_t ldc, int ncols, int D,
                                         f64x4 (&acc)[2][2], double *lds) {
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int i = lane & 15, kq = lane >> 4;
  const int wr = (wid >> 1) * 32, wc = (wid & 1) * 32;
  // this thread's staging run: row / column lr, k 4 lk .. 4 lk + 3 of a chunk
  const int lr = tid >> 2, lk = (tid & 3) * 4;
  const double *ga = q + (int64_t)min(lr, mrows - 1) * ldq + lk;
  const double *gb = c + (int64_t)min(lr, ncols - 1) * ldc + lk;
  double *As = lds, *Bs = lds + 2 * kF64LdsBuf;
#pragma unroll
  for (int ti = 0; ti < 2; ti++)
#pragma unroll
    for (int tj = 0; tj < 2; tj++) acc[ti][tj] = (f64x4){0.0, 0.0, 0.0, 0.0};
  f64x2 ra0 = *(const f64x2 *)ga, ra1 = *(const f64x2 *)(ga + 2);
  f64x2 rb0 = *(const f64x2 *)gb, rb1 = *(const f64x2 *)(gb + 2);
  auto put = [&](int buf) __attribute__((always_inline)) {
    double *a = As + buf * kF64LdsBuf + lk * kF64LdsRow + lr;
    double *b = Bs + buf * kF64LdsBuf + lk * kF64LdsRow + lr;
    a[0] = ra0[0];
    a[kF64LdsRow] = ra0[1];
    a[2 * kF64LdsRow] = ra1[0];
    a[3 * kF64LdsRow] = ra1[1];
    b[0] = rb0[0];
    b[kF64LdsRow] = rb0[1];
    b[2 * kF64LdsRow] = rb1[0];
    b[3 * kF64LdsRow] = rb1[1];
  };
  put(0);
  __syncthreads();
  const int nch = D / 16;
  for (int ch = 0; ch < nch; ch++) {
    const int buf = ch & 1;
    if (ch + 1 < nch) {
      const int ko = (ch + 1) * 16;
      ra0 = *(const f64x2 *)(ga + ko);
      ra1 = *(const f64x2 *)(ga + ko + 2);
      rb0 = *(const f64x2 *)(gb + ko);
      rb1 = *(const f64x2 *)(gb + ko + 2);
    }
    const double *a = As + buf * kF64LdsBuf + kq * kF64LdsRow + wr + i;
    const double *b = Bs + buf * kF64LdsBuf + kq * kF64LdsRow + wc + i;
#pragma unroll
    for (int s = 0; s < 4; s++) {
      const double a0 = a[4 * s * kF64LdsRow], a1 = a[4 * s * kF64LdsRow + 16];
      const double b0 = b[4 * s * kF64LdsRow], b1 = b[4 * s * kF64LdsRow + 16];
      acc[0][0] = __builtin_amdgcn_mfma_f64_16x16x4f64(a0, b0, acc[0][0], 0, 0, 0);
      acc[0][1] = __builtin_amdgcn_mfma_f64_16x16x4f64(a0, b1, acc[0][1], 0, 0, 0);
      acc[1][0] = __builtin_amdgcn_mfma_f64_16x16x4f64(a1, b0, acc[1][0], 0, 0, 0);
      acc[1][1] = __builtin_amdgcn_mfma_f64_16x16x4f64(a1, b1, acc[1][1], 0, 0, 0);
    }
    if (ch + 1 < nch) put(buf ^ 1);
    __syncthreads();
  }
}

// Tile order of the 1-D grid (both kernels below).  Consecutive workgroups
// go to the 8 XCDs in turn, and each XCD has its own L2, so workgroup b works
// on logical tile x * ceil(T / 8) + b / 8 (x = b % 8): every XCD walks a
// contiguous stretch of the logical order, which takes the row blocks in
// groups of kF64GroupRows (row block fastest inside a group, then the column
// block): the ~128 workgroups an XCD holds at once share 8 row tiles and ~16
// column tiles, 3 MB at D = 256, instead of streaming every corpus tile once
// per row block (a column-block-fastest 2-D grid re-read the corpus from HBM
// M / 64 times).
constexpr int kF64GroupRows = 8;
__device__ __forceinline__ bool f64_tile_of(int nR, int nC, int &r, int &c) {
  const int64_t T = (int64_t)nR * nC;
  const int64_t per = (T + 7) / 8;
  const int64_t L = (int64_t)(blockIdx.x % 8) * per + blockIdx.x / 8;
  if (L >= T) return false;
  const int64_t span = (int64_t)kF64GroupRows * nC;
  const int64_t g = L / span, w = L - g * span;
  const int gr = (int)min<int64_t>(kF64GroupRows, nR - g * kF64GroupRows);  // rows in this group
  r = (int)(g * kF64GroupRows + w % gr);
  c = (int)(w / gr);
  return true;
}
__host__ static inline unsigned f64_grid(int nR, int nC) {
  return (unsigned)(((int64_t)nR * nC + 7) / 8 * 8);
}

// Store mode (`.pmm.matmul` f64, src/metrics.rs:40-157; and the materialised
// top-k path's transformed scores, :258-311).
template <int METRIC, int XF>
__global__ __launch_bounds__(256) void gemm_f64_store_kernel(const double *__restrict__ q, int64_t ldq,
                                                             const double *__restrict__ c, int64_t ldc,
                                                             const double *__restrict__ qn,
                                                             const double *__restrict__ cn, int M, int N, int D,
                                                             double *__restrict__ out, int64_t ldo) {
  __shared__ double lds[2 * 2 * kF64LdsBuf];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int i = lane & 15, kq = lane >> 4;
  int rb, cbk;
  if (!f64_tile_of((M + 63) / 64, (N + 63) / 64, rb, cbk)) return;
  const int r0 = rb * 64, c0 = cbk * 64;
  f64x4 acc[2][2];
  f64_tile(q + (int64_t)r0 * ldq, ldq, M - r0, c + (int64_t)c0 * ldc, ldc, N - c0, D, acc, lds);
  const int row0 = r0 + (wid >> 1) * 32, col0 = c0 + (wid & 1) * 32;
#pragma unroll
  for (int ti = 0; ti < 2; ti++)
#pragma unroll
    for (int tj = 0; tj < 2; tj++)
#pragma unroll
      for (int r = 0; r < 4; r++) {
        const int grow = row0 + 16 * ti + kq + 4 * r;
        const int gcol = col0 + 16 * tj + i;
        if (grow < M && gcol < N) {
          const double v = acc[ti][tj][r];
          out[(int64_t)grow * ldo + gcol] = XF ? exact_score_f64<METRIC>(v, qn[grow], cn[gcol]) : v;
        }
      }
}

hipError_t launch_gemm_f64_store(const double *q, int64_t ldq, const double *c, int64_t ldc,
                                 const double *qn, const double *cn, int M, int N, int D,
                                 int metric, int store_metric, double *out, int64_t ldo,
                                 hipStream_t s) {
  if (M <= 0 || N <= 0) return hipSuccess;
  const dim3 grid(f64_grid((M + 63) / 64, (N + 63) / 64)), blk(256);
  if (!store_metric || metric == kMetricDot)
    gemm_f64_store_kernel<kMetricDot, 0><<<grid, blk, 0, s>>>(q, ldq, c, ldc, qn, cn, M, N, D, out, ldo);
  else if (metric == kMetricCosine)
    gemm_f64_store_kernel<kMetricCosine, 1><<<grid, blk, 0, s>>>(q, ldq, c, ldc, qn, cn, M, N, D, out, ldo);
  else
    gemm_f64_store_kernel<kMetricEuclidean, 1><<<grid, blk, 0, s>>>(q, ldq, c, ldc, qn, cn, M, N, D, out, ldo);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------
// Fused top-k pass over one column chunk: the tile above, then per element
// the exact score (reference order), its key, and an append to the row's
// buffer when it beats the row's threshold.
// ---------------------------------------------------------------------------
template <int METRIC>
__global__ __launch_bounds__(256) void gemm_f64_topk_kernel(F64TopkArgs a) {
  constexpr bool XF = METRIC != kMetricDot;
  __shared__ double lds[2 * 2 * kF64LdsBuf];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int i = lane & 15, kq = lane >> 4;
  int rb, cbk;
  if (!f64_tile_of((a.M + 63) / 64, (a.ncol + 63) / 64, rb, cbk)) return;
  const int r0 = rb * 64, lc0w = cbk * 64;  // lc: column within the chunk
  f64x4 acc[2][2];
  f64_tile(a.q + (int64_t)r0 * a.ldq, a.ldq, a.M - r0, a.c + (int64_t)(a.col0 + lc0w) * a.ldc, a.ldc,
           a.ncol - lc0w, a.D, acc, lds);
  const int row0 = r0 + (wid >> 1) * 32, lc0 = lc0w + (wid & 1) * 32;
  if (a.accept_all) {
    // the first chunk (ncol <= cap): every element at its own column's slot
    // (the counts were set to ncol by the reset; no atomics)
#pragma unroll
    for (int ti = 0; ti < 2; ti++)
#pragma unroll
      for (int r = 0; r < 4; r++) {
        const int row = row0 + 16 * ti + kq + 4 * r;
        if (row >= a.M) continue;
        const double qv = XF ? a.qn[row] : 0.0;
#pragma unroll
        for (int tj = 0; tj < 2; tj++) {
          const int lc = lc0 + 16 * tj + i;
          if (lc >= a.ncol) continue;
          const uint32_t gcol = (uint32_t)(a.col0 + lc);
          const double sc = XF ? exact_score_f64<METRIC>(acc[ti][tj][r], qv, a.cn[gcol]) : acc[ti][tj][r];
          Ent e;
          e.key = f64_key(sc, METRIC);
          e.idx = gcol;
          e.pad = 0u;
          a.cand[(int64_t)row * a.cap + lc] = e;
        }
      }
    return;
  }
  // Later chunks: every element's key and pass flag first, then one buffer
  // reservation per (row, wave) -- the 16 lanes of a row group share it --
  // with all eight in flight, then the appends.  (An atomicAdd per passing
  // element waited one memory round trip per (row block, register) step:
  // 0.22 ms for the GEMM at c1 f64 against 0.12 ms in store mode.)
  u64 key[2][4][2];
  bool ps[2][4][2];
#pragma unroll
  for (int ti = 0; ti < 2; ti++)
#pragma unroll
    for (int r = 0; r < 4; r++) {
      const int row = row0 + 16 * ti + kq + 4 * r;
      const bool rv = row < a.M;
      const u64 tk = rv ? a.tkey[row] : ~0ull;
      const uint32_t tx = rv ? a.tidx[row] : 0u;
      const double qv = (XF && rv) ? a.qn[row] : 0.0;
#pragma unroll
      for (int tj = 0; tj < 2; tj++) {
        const int lc = lc0 + 16 * tj + i;
        const bool cv = rv && lc < a.ncol;
        const uint32_t gcol = (uint32_t)(a.col0 + lc);
        const double v = acc[ti][tj][r];
        const double sc = XF ? exact_score_f64<METRIC>(v, qv, cv ? a.cn[gcol] : 0.0) : v;
        key[ti][r][tj] = f64_key(sc, METRIC);
        ps[ti][r][tj] = cv && (key[ti][r][tj] > tk || (key[ti][r][tj] == tk && gcol < tx));
      }
    }
  const u64 grp = 0xFFFFull << (16 * kq);
  const u64 below = (1ull << lane) - 1ull;
  unsigned base[2][4];
#pragma unroll
  for (int ti = 0; ti < 2; ti++)
#pragma unroll
    for (int r = 0; r < 4; r++) {
      const u64 m0 = __ballot(ps[ti][r][0]) & grp, m1 = __ballot(ps[ti][r][1]) & grp;
      const unsigned n = (unsigned)(__popcll(m0) + __popcll(m1));
      unsigned b0 = 0u;
      if (i == 0 && n != 0u) b0 = atomicAdd(a.cnt + row0 + 16 * ti + kq + 4 * r, n);
      base[ti][r] = b0;
    }
#pragma unroll
  for (int ti = 0; ti < 2; ti++)
#pragma unroll
    for (int r = 0; r < 4; r++) {
      const int row = row0 + 16 * ti + kq + 4 * r;
      const unsigned b0 = (unsigned)__shfl((int)base[ti][r], lane & 48, 64);
      const u64 m0 = __ballot(ps[ti][r][0]) & grp, m1 = __ballot(ps[ti][r][1]) & grp;
#pragma unroll
      for (int tj = 0; tj < 2; tj++) {
        if (!ps[ti][r][tj]) continue;
        const unsigned pos = b0 + (tj ? (unsigned)(__popcll(m0) + __popcll(m1 & below)) : (unsigned)__popcll(m0 & below));
        if (pos < (unsigned)a.cap) {
          Ent e;
          e.key = key[ti][r][tj];
          e.idx = (uint32_t)(a.col0 + lc0 + 16 * tj + i);
          e.pad = 0u;
          a.cand[(int64_t)row * a.cap + pos] = e;
        }
      }
    }
}

hipError_t launch_gemm_f64_topk(const F64TopkArgs &a, hipStream_t s) {
  if (a.M <= 0 || a.ncol <= 0) return hipSuccess;
  const dim3 grid(f64_grid((a.M + 63) / 64, (a.ncol + 63) / 64)), blk(256);
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
constexpr int kF64SelE = 16;  // selection path: buffers of up to 1024 entries in registers
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
  const Ent* src = a.cand + (int64_t)row * a.cap;
  if (n > a.k && n <= 64 * kF64SelE) {
    // Selection instead of a sort of the whole buffer: the k-th key by
    // ballots (wave_kth_u64, the value with multiplicity), then among the
    // entries tied at it the (k - #greater)-th smallest index.  The kept set
    // {key > tk} + {key == tk, idx <= tx} is exactly the sort's first k.
    // NaN scores (key 0) outnumbering n - k fall through to the sort.
    u64 x[kF64SelE];
    uint32_t ix[kF64SelE];
#pragma unroll
    for (int e = 0; e < kF64SelE; e++) {
      const int j = lane + 64 * e;
      x[e] = 0ull;
      ix[e] = 0xFFFFFFFFu;
      if (j < n) {
        const Ent en = src[j];
        x[e] = en.key;
        ix[e] = en.idx;
      }
    }
    int nz = 0;
#pragma unroll
    for (int e = 0; e < kF64SelE; e++) nz += __popcll(__ballot(x[e] != 0ull));
    if (nz >= a.k) {
      const u64 tk = wave_kth_u64<kF64SelE>(x, a.k);
      int gt = 0;
#pragma unroll
      for (int e = 0; e < kF64SelE; e++) gt += __popcll(__ballot(x[e] > tk));
      u64 y[kF64SelE];
#pragma unroll
      for (int e = 0; e < kF64SelE; e++) y[e] = x[e] == tk ? (u64)(~ix[e]) : 0ull;
      const uint32_t tx = ~(uint32_t)wave_kth_u64<kF64SelE>(y, a.k - gt);
      Ent *dst = a.mode == 0 ? a.cand + (int64_t)row * a.cap : scr;
      int base = 0;
#pragma unroll
      for (int e = 0; e < kF64SelE; e++) {
        const bool keep = x[e] > tk || (x[e] == tk && ix[e] <= tx);
        const u64 msk = __ballot(keep);
        if (keep) {
          Ent en;
          en.key = x[e];
          en.idx = ix[e];
          en.pad = 0u;
          dst[base + lanes_below(msk)] = en;
        }
        base += __popcll(msk);
      }
      if (a.mode == 0) {
        if (lane == 0) {
          a.cnt[row] = (unsigned)a.k;
          a.tkey[row] = tk;
          a.tidx[row] = tx;
        }
        return;
      }
      // final: sort the k kept entries only
      const int P2 = next_pow2_dev(a.k);
      for (int j = a.k + lane; j < P2; j += 64) {
        Ent e;
        e.key = 0ull;
        e.idx = 0xFFFFFFFFu;
        e.pad = 0u;
        scr[j] = e;
      }
      wave_sync();
      wave_sort_desc_ent(scr, P2, lane);
      for (int j = lane; j < a.k; j += 64) {
        a.out_idx[(int64_t)row * a.k + j] = scr[j].idx + a.index_base;
        a.out_score[(int64_t)row * a.k + j] = f64_unkey(scr[j].key, a.metric);
      }
      return;
    }
  }
  const int P2 = min(a.P, next_pow2_dev(n));
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

// thresholds to accept-all, counts to cnt0 (the first chunk's width)
__global__ __launch_bounds__(256) void f64_reset_kernel(u64 *tkey, uint32_t *tidx, unsigned *cnt, int m,
                                                        unsigned cnt0) {
  const int r = blockIdx.x * blockDim.x + threadIdx.x;
  if (r < m) {
    tkey[r] = 0ull;
    tidx[r] = 0xFFFFFFFFu;
    cnt[r] = cnt0;
  }
}

hipError_t launch_f64_reset(u64 *tkey, uint32_t *tidx, unsigned *cnt, int m, unsigned cnt0, hipStream_t s) {
  f64_reset_kernel<<<(m + 255) / 256, 256, 0, s>>>(tkey, tidx, cnt, m, cnt0);
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
