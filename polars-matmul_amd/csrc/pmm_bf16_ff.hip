// pmm_bf16_ff.hip -- host side of the fire-and-forget 256-row bf16 kernel
// (pmm_bf16_ff_kernel.h; one instantiation per padded-D step count in
// pmm_bf16_ff_ks.hip) and its bucketing pass.
#include "pmm_bf16_ff_kernel.h"

#include <hip/hip_runtime.h>

namespace pmm {

size_t gemm_bf16_ff_lds_bytes(int D) {
  switch (D / 128) {
    case 1: return ff::Carve<1>::BYTES;
    case 2: return ff::Carve<2>::BYTES;
    case 3: return ff::Carve<3>::BYTES;
    case 4: return ff::Carve<4>::BYTES;
    case 5: return ff::Carve<5>::BYTES;
    case 6: return ff::Carve<6>::BYTES;
    default: return 0;
  }
}

hipError_t launch_bf16_ff_ks1(const GemmF32Args &a, int grid, size_t lds, hipStream_t s);
hipError_t launch_bf16_ff_ks2(const GemmF32Args &a, int grid, size_t lds, hipStream_t s);
hipError_t launch_bf16_ff_ks3(const GemmF32Args &a, int grid, size_t lds, hipStream_t s);
hipError_t launch_bf16_ff_ks4(const GemmF32Args &a, int grid, size_t lds, hipStream_t s);
hipError_t launch_bf16_ff_ks5(const GemmF32Args &a, int grid, size_t lds, hipStream_t s);
hipError_t launch_bf16_ff_ks6(const GemmF32Args &a, int grid, size_t lds, hipStream_t s);

hipError_t launch_gemm_bf16_ff(const GemmF32Args &a, int grid, hipStream_t s) {
  const size_t lds = (a.D % 128 == 0) ? gemm_bf16_ff_lds_bytes(a.D) : 0;
  // the kernel's shapes: whole 128-wide K steps, every unit's tiles inside
  // the corpus, every query block inside QB, split units only (no whole-block
  // runs), regions to write into, and a column that fits the item's 26 bits
  if (lds == 0 || lds > 160 * 1024 || a.tps < 1 || (int64_t)a.ntiles * ff::BN < a.N ||
      (int64_t)(a.ntiles - 1) * ff::BN >= a.N || (int64_t)a.QB * ff::BM < a.M || grid < 1 || a.qb_full != 0 ||
      a.N >= (1 << 26) || !a.ffreg || !a.ffcnt || a.ffcap < 1)
    return hipErrorInvalidValue;
  switch (a.D / 128) {
    case 1: return launch_bf16_ff_ks1(a, grid, lds, s);
    case 2: return launch_bf16_ff_ks2(a, grid, lds, s);
    case 3: return launch_bf16_ff_ks3(a, grid, lds, s);
    case 4: return launch_bf16_ff_ks4(a, grid, lds, s);
    case 5: return launch_bf16_ff_ks5(a, grid, lds, s);
    case 6: return launch_bf16_ff_ks6(a, grid, lds, s);
    default: return hipErrorInvalidValue;
  }
}

// ---------------------------------------------------------------------------
// Bucketing pass: workgroup (query block qb, wave w) takes the S regions of
// its 64 rows (one per split unit), re-scores every item exactly -- the
// reference's operation order on the main pass's raw dot (exact_score) --
// keeps those whose composite key beats the row's threshold (the guess - 1)
// and appends them to the row's candidate list of that split (LDS counters).
// A row is exact when it kept at least k candidates and nothing of it was
// dropped (no region or list overflow); the others are listed for a re-run.
// ---------------------------------------------------------------------------
template <int METRIC>
__global__ __launch_bounds__(256) void ff_bucket_kernel(GemmF32Args a, unsigned *fb_count, int *fb_rows) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  constexpr bool XFORM = METRIC != kMetricDot;
  unsigned *cnt_l = (unsigned *)smem;        // [64][S]
  int *bad_l = (int *)(cnt_l + 64 * a.S);    // [64]
  const int tid = threadIdx.x;
  const int qb = (int)blockIdx.x / ff::NW, w = (int)blockIdx.x % ff::NW;
  const int wrow0 = qb * ff::BM + w * ff::RW;
  for (int i = tid; i < 64 * a.S; i += 256) cnt_l[i] = 0u;
  if (tid < 64) bad_l[tid] = 0;
  __syncthreads();
  for (int s = 0; s < a.S; s++) {
    const int64_t r = (int64_t)(s * a.QB + qb) * ff::NW + w;
    const unsigned n = a.ffcnt[r];
    if (n > (unsigned)a.ffcap) {  // items were dropped: every row of the region re-runs
      if (tid < 64) bad_l[tid] = 1;
    }
    const unsigned nn = n < (unsigned)a.ffcap ? n : (unsigned)a.ffcap;
    const unsigned long long *reg = a.ffreg + r * a.ffcap;
    for (unsigned i = tid; i < nn; i += 256) {
      const u64 it = reg[i];
      const float v = __uint_as_float((uint32_t)it);
      const uint32_t hi = (uint32_t)(it >> 32);
      const int row = (int)(hi >> 26), col = (int)(hi & 0x3FFFFFFu);
      const int grow = wrow0 + row;
      if (grow >= a.M) continue;
      const float sc = exact_score<METRIC>(v, XFORM ? a.qn[grow] : 0.0f, XFORM ? a.cn[col] : 0.0f);
      const u64 comp = ((u64)okey32(METRIC == kMetricEuclidean ? -sc : sc) << 32) | (u64)(~(uint32_t)col);
      if (comp > a.gthr[grow]) {
        const unsigned pos = atomicAdd(cnt_l + row * a.S + s, 1u);
        if (pos < (unsigned)a.capg) a.cand[((int64_t)grow * a.S + s) * a.capg + pos] = comp;
      }
    }
  }
  __syncthreads();
  if (tid < 64) {
    const int grow = wrow0 + tid;
    if (grow < a.M) {
      unsigned tot = 0;
      int bad = bad_l[tid];
      for (int s = 0; s < a.S; s++) {
        const unsigned c = cnt_l[tid * a.S + s];
        if (c > (unsigned)a.capg) bad = 1;
        const unsigned cc = c < (unsigned)a.capg ? c : (unsigned)a.capg;
        a.cnt[(int64_t)grow * a.S + s] = cc;
        tot += cc;
      }
      if (bad || tot < (unsigned)a.k) {
        const unsigned j = atomicAdd(fb_count, 1u);
        fb_rows[j] = grow;
      }
    }
  }
}

hipError_t launch_ff_bucket(const GemmF32Args &a, unsigned *fb_count, int *fb_rows, hipStream_t s) {
  if (a.M <= 0) return hipSuccess;
  const unsigned grid = (unsigned)(a.QB * ff::NW);
  // (many splits per query block -- few query rows over a long corpus -- take
  // more than the default 64 KiB of counters)
  const size_t lds = (size_t)64 * a.S * 4 + 64 * 4;
  if (lds > 160 * 1024) return hipErrorInvalidValue;
  if (lds > 64 * 1024) {
    static bool attr_set[3] = {false, false, false};
    if (!attr_set[a.metric]) {
      const void *fn = a.metric == kMetricCosine ? (const void *)ff_bucket_kernel<kMetricCosine>
                       : a.metric == kMetricDot  ? (const void *)ff_bucket_kernel<kMetricDot>
                                                 : (const void *)ff_bucket_kernel<kMetricEuclidean>;
      hipError_t e = hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
      if (e != hipSuccess) return e;
      attr_set[a.metric] = true;
    }
  }
  if (a.metric == kMetricCosine) ff_bucket_kernel<kMetricCosine><<<grid, 256, lds, s>>>(a, fb_count, fb_rows);
  else if (a.metric == kMetricDot) ff_bucket_kernel<kMetricDot><<<grid, 256, lds, s>>>(a, fb_count, fb_rows);
  else ff_bucket_kernel<kMetricEuclidean><<<grid, 256, lds, s>>>(a, fb_count, fb_rows);
  return hipGetLastError();
}

// The re-run's row gather (query rows listed in rows[0..r) into a dense
// block) and list scatter (the re-run's lists back to those rows).
__global__ __launch_bounds__(256) void ff_gather_rows_kernel(const uint16_t *__restrict__ q, int64_t ldq,
                                                             const int *__restrict__ rows, int r,
                                                             uint16_t *__restrict__ dst) {
  const int i = blockIdx.x;
  if (i >= r) return;
  const uint16_t *src = q + (int64_t)rows[i] * ldq;
  for (int64_t j = threadIdx.x; j < ldq; j += 256) dst[(int64_t)i * ldq + j] = src[j];
}
__global__ __launch_bounds__(256) void ff_scatter_lists_kernel(const uint32_t *__restrict__ oi,
                                                               const float *__restrict__ os,
                                                               const int *__restrict__ rows, int r, int k,
                                                               uint32_t *__restrict__ out_idx,
                                                               float *__restrict__ out_score) {
  const int i = blockIdx.x;
  if (i >= r) return;
  const int64_t row = rows[i];
  for (int j = threadIdx.x; j < k; j += 256) {
    out_idx[row * k + j] = oi[(int64_t)i * k + j];
    out_score[row * k + j] = os[(int64_t)i * k + j];
  }
}
hipError_t launch_ff_gather_rows(const uint16_t *q, int64_t ldq, const int *rows, int r, uint16_t *dst,
                                 hipStream_t s) {
  if (r <= 0) return hipSuccess;
  ff_gather_rows_kernel<<<r, 256, 0, s>>>(q, ldq, rows, r, dst);
  return hipGetLastError();
}
hipError_t launch_ff_scatter_lists(const uint32_t *oi, const float *os, const int *rows, int r, int k,
                                   uint32_t *out_idx, float *out_score, hipStream_t s) {
  if (r <= 0) return hipSuccess;
  ff_scatter_lists_kernel<<<r, 256, 0, s>>>(oi, os, rows, r, k, out_idx, out_score);
  return hipGetLastError();
}

}  // namespace pmm
