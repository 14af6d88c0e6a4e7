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
// compute every dot product identically).  Four waves in 2 x 2; each wave
// owns W x W v_mfma_f64_16x16x4_f64 tiles (16W x 16W outputs), so the
// workgroup's tile is 32W x 32W: W = 2 -> 64 x 64, W = 4 -> 128 x 128 (half
// the operand bytes per flop, four times the MFMAs per LDS fragment pair).
// K runs in chunks of 16 through a double-buffered LDS image stored k-major
// (As[k][row]), so at K step s of a chunk lane (i = lane & 15, kq = lane >> 4)
// reads A[row][k0 + 4 s + kq] and B[col][k0 + 4 s + kq] with one ds_read_b64
// each: the four MFMAs of a chunk see k0 .. k0 + 15 in natural order, whatever
// W is (so every W returns the same bits).  Rows of 32W + 16 doubles: the
// kq = 0 and kq = 1 half-waves of a read land on disjoint banks.  Global loads:
// each thread W / 2 32-byte runs (rows t/4 + 64j, k 4(t%4) .. +3) of A and of
// B per chunk, the next chunk's in flight while this chunk's MFMAs run.
// C/D layout: col = lane & 15, row = (lane >> 4) + 4 reg.
// ---------------------------------------------------------------------------
template <int W>
struct F64T {
  static constexpr int R = 32 * W;         // rows (= columns) of a workgroup tile
  static constexpr int LR = R + 16;        // doubles per LDS k-row
  static constexpr int BUF = 16 * LR;      // one operand's K chunk
  static constexpr int LDS = 2 * 2 * BUF;  // two operands, double-buffered
  static constexpr int NRUN = W / 2;       // staging runs per thread per operand
  static_assert(W == 2 || W == 4, "64 x 64 or 128 x 128 workgroup tiles");
};

template <int W>
__device__ __forceinline__ void f64_tile(const double *__restrict__ q, int64_t ldq, int mrows,
                                         const double *__restrict__ c, int64_t ldc, int ncols, int D,
                                         f64x4 (&acc)[W][W], double *lds) {
  using T = F64T<W>;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int i = lane & 15, kq = lane >> 4;
  const int wr = (wid >> 1) * 16 * W, wc = (wid & 1) * 16 * W;
  // this thread's staging runs: rows / columns lr + 64 j, k 4 lk .. 4 lk + 3 of a chunk
  const int lr = tid >> 2, lk = (tid & 3) * 4;
  const double *ga[T::NRUN], *gb[T::NRUN];
#pragma unroll
  for (int j = 0; j < T::NRUN; j++) {
    ga[j] = q + (int64_t)min(lr + 64 * j, mrows - 1) * ldq + lk;
    gb[j] = c + (int64_t)min(lr + 64 * j, ncols - 1) * ldc + lk;
  }
  double *As = lds, *Bs = lds + 2 * T::BUF;
#pragma unroll
  for (int ti = 0; ti < W; ti++)
#pragma unroll
    for (int tj = 0; tj < W; tj++) acc[ti][tj] = (f64x4){0.0, 0.0, 0.0, 0.0};
  f64x2 ra[T::NRUN][2], rb[T::NRUN][2];
  auto load = [&](int ko) __attribute__((always_inline)) {
#pragma unroll
    for (int j = 0; j < T::NRUN; j++) {
      ra[j][0] = *(const f64x2 *)(ga[j] + ko);
      ra[j][1] = *(const f64x2 *)(ga[j] + ko + 2);
      rb[j][0] = *(const f64x2 *)(gb[j] + ko);
      rb[j][1] = *(const f64x2 *)(gb[j] + ko + 2);
    }
  };
  auto put = [&](int buf) __attribute__((always_inline)) {
#pragma unroll
    for (int j = 0; j < T::NRUN; j++) {
      double *a = As + buf * T::BUF + lk * T::LR + lr + 64 * j;
      double *b = Bs + buf * T::BUF + lk * T::LR + lr + 64 * j;
      a[0] = ra[j][0][0];
      a[T::LR] = ra[j][0][1];
      a[2 * T::LR] = ra[j][1][0];
      a[3 * T::LR] = ra[j][1][1];
      b[0] = rb[j][0][0];
      b[T::LR] = rb[j][0][1];
      b[2 * T::LR] = rb[j][1][0];
      b[3 * T::LR] = rb[j][1][1];
    }
  };
  load(0);
  put(0);
  __syncthreads();
  const int nch = D / 16;
  for (int ch = 0; ch < nch; ch++) {
    const int buf = ch & 1;
    if (ch + 1 < nch) load((ch + 1) * 16);
    const double *a = As + buf * T::BUF + kq * T::LR + wr + i;
    const double *b = Bs + buf * T::BUF + kq * T::LR + wc + i;
#pragma unroll
    for (int s = 0; s < 4; s++) {
      double av[W], bv[W];
#pragma unroll
      for (int t = 0; t < W; t++) {
        av[t] = a[4 * s * T::LR + 16 * t];
        bv[t] = b[4 * s * T::LR + 16 * t];
      }
#pragma unroll
      for (int ti = 0; ti < W; ti++)
#pragma unroll
        for (int tj = 0; tj < W; tj++)
          acc[ti][tj] = __builtin_amdgcn_mfma_f64_16x16x4f64(av[ti], bv[tj], acc[ti][tj], 0, 0, 0);
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
// block): the workgroups an XCD holds at once share 8 row tiles and a few
// column tiles instead of streaming every corpus tile once per row block (a
// column-block-fastest 2-D grid re-read the corpus from HBM M / 64 times).
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
  constexpr int W = 2;
  using T = F64T<W>;
  __shared__ double lds[T::LDS];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int i = lane & 15, kq = lane >> 4;
  int rb, cbk;
  if (!f64_tile_of((M + T::R - 1) / T::R, (N + T::R - 1) / T::R, rb, cbk)) return;
  const int r0 = rb * T::R, c0 = cbk * T::R;
  f64x4 acc[W][W];
  f64_tile<W>(q + (int64_t)r0 * ldq, ldq, M - r0, c + (int64_t)c0 * ldc, ldc, N - c0, D, acc, lds);
  const int row0 = r0 + (wid >> 1) * 16 * W, col0 = c0 + (wid & 1) * 16 * W;
#pragma unroll
  for (int ti = 0; ti < W; ti++)
#pragma unroll
    for (int tj = 0; tj < W; tj++)
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
  constexpr int R = F64T<2>::R;
  const dim3 grid(f64_grid((M + R - 1) / R, (N + R - 1) / R)), blk(256);
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
template <int METRIC, int W>
__global__ __launch_bounds__(256, W == 4 ? 2 : 1) void gemm_f64_topk_kernel(F64TopkArgs a) {
  using T = F64T<W>;
  constexpr bool XF = METRIC != kMetricDot;
  __shared__ double lds[T::LDS];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int i = lane & 15, kq = lane >> 4;
  int rb, cbk;
  if (!f64_tile_of((a.M + T::R - 1) / T::R, (a.ncol + T::R - 1) / T::R, rb, cbk)) return;
  const int r0 = rb * T::R, lc0w = cbk * T::R;  // lc: column within the chunk
  f64x4 acc[W][W];
  f64_tile<W>(a.q + (int64_t)r0 * a.ldq, a.ldq, a.M - r0, a.c + (int64_t)(a.col0 + lc0w) * a.ldc, a.ldc,
              a.ncol - lc0w, a.D, acc, lds);
  const int row0 = r0 + (wid >> 1) * 16 * W, lc0 = lc0w + (wid & 1) * 16 * W;
  if (a.accept_all) {
    // the first chunk (ncol <= cap): every element at its own column's slot
    // (the counts were set to ncol by the reset; no atomics)
#pragma unroll
    for (int ti = 0; ti < W; ti++)
#pragma unroll
      for (int r = 0; r < 4; r++) {
        const int row = row0 + 16 * ti + kq + 4 * r;
        if (row >= a.M) continue;
        const double qv = XF ? a.qn[row] : 0.0;
#pragma unroll
        for (int tj = 0; tj < W; tj++) {
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
  // Later chunks, one 16-row block (ti) at a time: every element's key and
  // pass flag first, then one buffer reservation per (row, wave) -- the 16
  // lanes of a row group share it -- with the block's four in flight, then
  // the appends.  (An atomicAdd per passing element waited one memory round
  // trip per (row block, register) step: 0.22 ms for the GEMM at c1 f64
  // against 0.12 ms in store mode.)
  const u64 grp = 0xFFFFull << (16 * kq);
  const u64 below = (1ull << lane) - 1ull;
  // Cosine: the exact score is a division; an element whose dot is below
  // bm * cn -- bm = ts * qn * (1 -+ 2^-49), ts the row's threshold score --
  // scores strictly below ts (the three roundings of the bound and the two of
  // the score are covered 13u > 4u), so it is dropped without the division.
  // No bound (NaN: never below) for an accept-all row, a zero threshold, a
  // zero-norm row or column (score 0 whatever the dot), or a NaN.
  const double kNaN = __longlong_as_double(0x7FF8000000000000ll);
  double cnf[W];
#pragma unroll
  for (int tj = 0; tj < W; tj++) {
    const int lc = lc0 + 16 * tj + i;
    const double cvv = (METRIC == kMetricCosine && lc < a.ncol) ? a.cn[a.col0 + lc] : 0.0;
    // (a column factor in [1e-10, 2^100] and a row bound |bm| in [2^-900,
    // 2^900] keep bm * cn a normal double, where the rounding margin below
    // holds; outside, NaN: no skip, the exact division decides)
    cnf[tj] = (cvv > 1e-10 && cvv < 0x1p100) ? cvv : kNaN;
  }
#pragma unroll
  for (int ti = 0; ti < W; ti++) {
    u64 key[4][W];
    bool ps[4][W];
#pragma unroll
    for (int r = 0; r < 4; r++) {
      const int row = row0 + 16 * ti + kq + 4 * r;
      const bool rv = row < a.M;
      const u64 tk = rv ? a.tkey[row] : ~0ull;
      const uint32_t tx = rv ? a.tidx[row] : 0u;
      const double qv = (XF && rv) ? a.qn[row] : 0.0;
      double bm = kNaN;
      if (METRIC == kMetricCosine) {
        const double ts = dekey64(tk);
        const double tq = __dmul_rn(ts, qv);
        if (qv > 1e-10 && ts != 0.0 && fabs(tq) > 0x1p-900 && fabs(tq) < 0x1p900)
          bm = __dmul_rn(tq, ts > 0.0 ? 1.0 - 0x1p-49 : 1.0 + 0x1p-49);
      }
#pragma unroll
      for (int tj = 0; tj < W; tj++) {
        const int lc = lc0 + 16 * tj + i;
        const bool cv = rv && lc < a.ncol;
        const uint32_t gcol = (uint32_t)(a.col0 + lc);
        const double v = acc[ti][tj][r];
        key[r][tj] = 0ull;
        ps[r][tj] = false;
        if (METRIC == kMetricCosine && v < __dmul_rn(bm, cnf[tj])) continue;
        const double sc = XF ? exact_score_f64<METRIC>(v, qv, cv ? a.cn[gcol] : 0.0) : v;
        key[r][tj] = f64_key(sc, METRIC);
        ps[r][tj] = cv && (key[r][tj] > tk || (key[r][tj] == tk && gcol < tx));
      }
    }
    unsigned base[4];
#pragma unroll
    for (int r = 0; r < 4; r++) {
      unsigned n = 0u;
#pragma unroll
      for (int tj = 0; tj < W; tj++) n += (unsigned)__popcll(__ballot(ps[r][tj]) & grp);
      unsigned b0 = 0u;
      if (i == 0 && n != 0u) b0 = atomicAdd(a.cnt + row0 + 16 * ti + kq + 4 * r, n);
      base[r] = b0;
    }
#pragma unroll
    for (int r = 0; r < 4; r++) {
      const int row = row0 + 16 * ti + kq + 4 * r;
      unsigned pos = (unsigned)__shfl((int)base[r], lane & 48, 64);
#pragma unroll
      for (int tj = 0; tj < W; tj++) {
        const u64 m = __ballot(ps[r][tj]) & grp;
        if (ps[r][tj] && pos + (unsigned)__popcll(m & below) < (unsigned)a.cap) {
          Ent e;
          e.key = key[r][tj];
          e.idx = (uint32_t)(a.col0 + lc0 + 16 * tj + i);
          e.pad = 0u;
          a.cand[(int64_t)row * a.cap + pos + __popcll(m & below)] = e;
        }
        pos += (unsigned)__popcll(m);
      }
    }
  }
}

// 64 x 64 tiles: 128 x 128 ones (W = 4, two waves per SIMD, half the
// operand bytes per flop) measured slower at 4096 x 1M x 256: the fused GEMM
// 43.0 vs 39.7-39.8 ms per step, alternated on one box
// (profiles/r5_f64/ab.txt) -- the f64 kernel is bound by its issue, not its
// operand stream.  PMM_F64_TILE=128 (per call) keeps them for tests / A/B.

template <int W>
static hipError_t launch_gemm_f64_topk_w(const F64TopkArgs &a, hipStream_t s) {
  constexpr int R = F64T<W>::R;
  const dim3 grid(f64_grid((a.M + R - 1) / R, (a.ncol + R - 1) / R)), blk(256);
  if (a.metric == kMetricCosine) gemm_f64_topk_kernel<kMetricCosine, W><<<grid, blk, 0, s>>>(a);
  else if (a.metric == kMetricEuclidean) gemm_f64_topk_kernel<kMetricEuclidean, W><<<grid, blk, 0, s>>>(a);
  else gemm_f64_topk_kernel<kMetricDot, W><<<grid, blk, 0, s>>>(a);
  return hipGetLastError();
}

hipError_t launch_gemm_f64_topk(const F64TopkArgs &a, hipStream_t s) {
  if (a.M <= 0 || a.ncol <= 0) return hipSuccess;
  // (PMM_F64_TILE=64 / 128 forces one size, per call: tests and A/B runs)
  const char *e = getenv("PMM_F64_TILE");
  const int force = e ? atoi(e) : 0;
  if (force == 128) return launch_gemm_f64_topk_w<4>(a, s);
  return launch_gemm_f64_topk_w<2>(a, s);
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

// ---------------------------------------------------------------------------
// k-way merge of G sorted f64 lists per row (the corpus-sharded f64 path:
// every device's f64 top-k of its shard, gathered into [G][m][k] index and
// score planes on the root).  LPR = next_pow2(G) lanes per row, lane g holding
// list g's head; per output position the row's best head under the f64
// path's total order (key okey64(score) best-first -- NaN and empty slots at
// key 0 -- then the lower index; empty slots carry 0xFFFFFFFF, so they come
// last) by log2(LPR) shuffle steps, and the winning list advances.  The
// winner writes the entry as its list holds it (bit for bit the one-device
// value).  Each list's next entry is loaded ahead of its next win.
// ---------------------------------------------------------------------------
template <int LPR>
__global__ __launch_bounds__(256) void f64_kway_merge_kernel(F64MergeArgs a) {
  const int lane = threadIdx.x & 63;
  constexpr int RPW = 64 / LPR;
  const int wave = (int)((blockIdx.x * blockDim.x + threadIdx.x) >> 6);
  const int row = wave * RPW + lane / LPR;
  const int g = lane % LPR;
  if (wave * RPW >= a.M) return;  // whole wave exits
  const bool live = row < a.M && g < a.G;
  const int64_t base = live ? (int64_t)g * a.list_stride + (int64_t)row * a.k : 0;
  const double nan = __longlong_as_double(0x7FF8000000000000ll);
  auto ld = [&](int p, uint32_t &id, double &sc) __attribute__((always_inline)) {
    const bool ok = live && p < a.k;
    const int64_t o = ok ? base + p : 0;
    id = a.gi[o];
    sc = a.gs[o];
    if (!ok) id = 0xFFFFFFFFu;
  };
  uint32_t hid, nid;
  double hsc, nsc;
  ld(0, hid, hsc);
  ld(1, nid, nsc);
  int ptr = 0;
  for (int j = 0; j < a.k; j++) {
    const u64 hk = hid != 0xFFFFFFFFu ? f64_key(hsc, a.metric) : 0ull;
    u64 mk = hk;
    uint32_t mi = hid;
#pragma unroll
    for (int o = 1; o < LPR; o <<= 1) {
      const u64 ok2 = __shfl_xor(mk, o);
      const uint32_t oi2 = (uint32_t)__shfl_xor((int)mi, o);
      if (ok2 > mk || (ok2 == mk && oi2 < mi)) {
        mk = ok2;
        mi = oi2;
      }
    }
    // the lists' (key, index) pairs are distinct (disjoint shard rows), so
    // one lane wins -- or, past every list's end, all lanes hold the same
    // empty slot and write the same empty entry
    if (live && hk == mk && hid == mi) {
      a.out_idx[(int64_t)row * a.k + j] = hid;
      a.out_score[(int64_t)row * a.k + j] = hid != 0xFFFFFFFFu ? hsc : nan;
      ptr++;
      hid = nid;
      hsc = nsc;
      ld(ptr + 1, nid, nsc);
    }
  }
}

hipError_t launch_f64_merge(const F64MergeArgs &a, hipStream_t s) {
  if (a.M <= 0 || a.k <= 0) return hipSuccess;
  int lpr = 1;
  while (lpr < a.G) lpr <<= 1;
  if (lpr > 64) return hipErrorInvalidValue;
  const int64_t waves = ((int64_t)a.M * lpr + 63) / 64;
  const unsigned grid = (unsigned)((waves + 3) / 4);
  switch (lpr) {
    case 1: f64_kway_merge_kernel<1><<<grid, 256, 0, s>>>(a); break;
    case 2: f64_kway_merge_kernel<2><<<grid, 256, 0, s>>>(a); break;
    case 4: f64_kway_merge_kernel<4><<<grid, 256, 0, s>>>(a); break;
    case 8: f64_kway_merge_kernel<8><<<grid, 256, 0, s>>>(a); break;
    case 16: f64_kway_merge_kernel<16><<<grid, 256, 0, s>>>(a); break;
    case 32: f64_kway_merge_kernel<32><<<grid, 256, 0, s>>>(a); break;
    default: f64_kway_merge_kernel<64><<<grid, 256, 0, s>>>(a); break;
  }
  return hipGetLastError();
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
