// pmm_bf16.hip -- bf16 compute path of the fused top-k (PMM_COMPUTE_BF16;
// BASELINE configs[3]: 100k x 1M x 768 bf16 cosine k=100, CDNA4 bf16 MFMA with
// f32 accumulation).
//
// Scores are those of the bf16-rounded embeddings: Q and C are rounded to
// bf16 (round to nearest even), S = Q.C^T runs on v_mfma_f32_32x32x16_bf16
// (f32 accumulation), the norms are the f32 norms of the bf16 rows in the
// reference's order, and the metric epilogue and per-row top-k are the f32
// path's (exact_score / prefilter_bound / candidate buffers / merge), so the
// result is the exact top-k of the bf16 vectors up to f32 accumulation order.
//
// Why a different kernel shape than the f32 path: a bf16 MFMA does 8x the
// work of the f32 one per operand byte, so the f32 kernel's 256 x 256 tile with
// both operands re-streamed through LDS would need ~20 TB/s from L2 + MALL.
// Here each wave keeps its 32 query rows x D in registers for a whole work
// unit (D <= 768: 4 registers per 16 columns of D), so only corpus tiles
// stream: 128 query rows x 128 corpus columns per workgroup, 4 waves (one per
// SIMD), corpus K-steps of 128 bf16 (32 KiB per step) through a 3-slot LDS-DMA
// ring with counted vmcnt waits (the next-but-one step is always in flight).
#include "pmm_device.h"

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace pmm {

typedef __attribute__((__vector_size__(8 * sizeof(__bf16)))) __bf16 bf16x8;

namespace {
constexpr int NW = kBf16NW;                  // waves per workgroup (1 per SIMD)
constexpr int NB = kBf16BN / 32;             // 32x32 accumulators per wave
constexpr int BN = kBf16BN;                  // corpus columns per tile
constexpr int BM = kBf16BM;                  // query rows per workgroup
constexpr int NST = 3;                       // LDS ring slots
constexpr int KB = 256;                      // bytes of a row per K-step (128 bf16)
constexpr int KSUB = KB / 32;                // MFMA substeps (K = 16) per K-step
constexpr int STAGE = BN * KB;               // BN corpus rows x 128 bf16
constexpr int BPIECES = STAGE / 1024 / NW;   // 1 KiB LDS-DMA pieces per wave per step
constexpr int OFF_THR = NST * STAGE;
constexpr int OFF_CNT = OFF_THR + BM * 8;
constexpr int OFF_QEX = OFF_CNT + BM * 4;
constexpr int OFF_LO = OFF_QEX + BM * 4;
constexpr int OFF_CV = OFF_LO + BM * 4;      // pre-filter column factors, 2 tiles
constexpr int OFF_UNIT = OFF_CV + 2 * BN * 4;
constexpr int OFF_SCR = OFF_UNIT + 16;
static_assert(OFF_SCR % 16 == 0, "LDS carve must stay 16-byte aligned");
constexpr int CV_PER_WAVE = BN / NW;          // pre-filter factors DMA'd per wave per tile
static_assert(CV_PER_WAVE <= 64, "one 4-byte DMA per lane covers a wave's factors");
}  // namespace

size_t gemm_bf16_lds_bytes(int capg) { return (size_t)OFF_SCR + (size_t)NW * capg * 8; }

// ---------------------------------------------------------------------------
// f32 -> bf16 with zero padding: one thread per 8 output elements.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void f32_to_bf16_kernel(const float *__restrict__ src,
                                                          int64_t rows, int64_t d, int64_t lds,
                                                          uint16_t *__restrict__ dst, int64_t ldd) {
  const int64_t per_row = ldd >> 3;
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= rows * per_row) return;
  const int64_t r = t / per_row;
  const int64_t c0 = (t - r * per_row) * 8;
  bf16x8 v;
#pragma unroll
  for (int j = 0; j < 8; j++) {
    const int64_t c = c0 + j;
    // plain cast: v_cvt_pk_bf16_f32, round to nearest even, NaN stays NaN
    v[j] = (c < d) ? (__bf16)src[r * lds + c] : (__bf16)0.0f;
  }
  *(bf16x8 *)(dst + r * ldd + c0) = v;
}

hipError_t launch_f32_to_bf16(const float *src, int64_t rows, int64_t d, int64_t lds, uint16_t *dst,
                              int64_t ldd, hipStream_t s) {
  if (rows <= 0) return hipSuccess;
  const int64_t threads = rows * (ldd >> 3);
  f32_to_bf16_kernel<<<(unsigned)((threads + 255) / 256), 256, 0, s>>>(src, rows, d, lds, dst, ldd);
  return hipGetLastError();
}

hipError_t launch_norms_bf16(const uint16_t *a, int64_t rows, int64_t d, int64_t ld, int squared,
                             float *out, float *inv, hipStream_t s) {
  if (rows <= 0) return hipSuccess;
  const int64_t threads = rows * 8;
  norms_kernel<float, __bf16><<<(unsigned)((threads + 255) / 256), 256, 0, s>>>(
      (const __bf16 *)a, rows, d, ld, squared, out, inv);
  return hipGetLastError();
}

// s_waitcnt vmcnt(N) as one instruction with a compile-time N; the memory
// clobber keeps the compiler from moving LDS reads across it.
template <int N>
__device__ __forceinline__ void wait_vm() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// ===========================================================================
// Fused bf16 GEMM + metric + per-row top-k.  KS = padded D / 128 (K-steps).
//
// Work units as in the f32 kernel (query block x corpus split, pulled from an
// atomic counter, split-major so co-resident workgroups stream the same
// corpus tiles through their XCD's L2).  Per unit a wave loads its 32 query
// rows into registers once (af[]: lane (r, h) holds row r, columns
// 128*ks + 8*(8h + sub) .. +8 for K-step ks, MFMA substep sub), then streams
// the unit's corpus tiles.  Corpus K-step g lives in ring slot g % 3; step
// g + 2 is issued behind the first MFMA group of step g, and step g waits
// only for its own DMAs (vmcnt = the DMA count of step g + 1, still in
// flight).  Epilogue: the f32 kernel's two-pass filter / exact queue.
// ===========================================================================
template <int KS, int METRIC>  // KS = padded D / 128
__global__ __launch_bounds__(NW * 64, 1) void gemm_bf16_kernel(GemmF32Args a) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  u64 *thr_l = (u64 *)(smem + OFF_THR);
  unsigned *cnt_l = (unsigned *)(smem + OFF_CNT);
  float *qex_l = (float *)(smem + OFF_QEX);
  float *lo_l = (float *)(smem + OFF_LO);
  float *cv_l = (float *)(smem + OFF_CV);
  int *unit_l = (int *)(smem + OFF_UNIT);

  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int r32 = lane & 31, h = lane >> 5;
  u64 *scr = (u64 *)(smem + OFF_SCR) + (size_t)wid * a.capg;
  u64 *thr_w = thr_l + wid * 32;
  unsigned *cnt_w = cnt_l + wid * 32;
  float *qex_w = qex_l + wid * 32;
  float *lo_w = lo_l + wid * 32;
  constexpr bool XFORM = (METRIC != kMetricDot);

  // Loop-invariant per-lane byte offsets of this wave's corpus DMA pieces:
  // piece i = 4 corpus rows x 256 B; 16-byte chunk c of row r lands in LDS
  // chunk c ^ (r & 15), so the fragment reads (32 rows, one chunk each) hit
  // 16 distinct bank groups per 16 lanes.
  uint32_t b_voff[BPIECES];
#pragma unroll
  for (int i = 0; i < BPIECES; i++) {
    const int col = (i * NW + wid) * 4 + (lane >> 4);
    const int ch = (lane & 15) ^ (col & 15);
    b_voff[i] = (uint32_t)(col * a.ldc * 2 + ch * 16);
  }
  const int swz = r32 & 15;
  const int b_rd = r32 * KB;

  for (;;) {
    if (tid == 0) *unit_l = (int)atomicAdd(a.counter, 1u);
    __syncthreads();
    const int unit = *unit_l;
    __syncthreads();
    if (unit >= a.units) break;
    const int s = unit / a.QB;
    const int qb = unit - s * a.QB;
    const int t0 = s * a.tps;
    const int t1 = min(t0 + a.tps, a.ntiles);
    const int wrow0 = qb * BM + wid * 32;

    if (lane < 32) {
      const int grow = wrow0 + lane;
      const float qv = (XFORM && grow < a.M) ? a.qn[grow] : 0.0f;
      qex_w[lane] = qv;
      const u64 t = (grow < a.M)
                        ? __hip_atomic_load(a.gthr + grow, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                        : ~0ull;
      thr_w[lane] = t;
      lo_w[lane] = prefilter_bound<METRIC>(t, qv);
      cnt_w[lane] = 0u;
    }

    // This wave's query rows, register-resident for the whole unit: lane
    // (r, h) holds row r, columns 128*ks + 8*(8h + sub) .. +8 in af[KSUB*ks + sub].
    bf16x8 af[KSUB * KS];
    {
      const int row = wrow0 + r32;
      const bool ok = row < a.M;
      const uint16_t *qa = a.qb + (int64_t)(ok ? row : 0) * a.ldq + 64 * h;
      const bf16x8 z = {};
#pragma unroll
      for (int i = 0; i < KSUB * KS; i++) {
        const bf16x8 v = *(const bf16x8 *)(qa + (i / KSUB) * 128 + (i % KSUB) * 8);
        af[i] = ok ? v : z;
      }
    }
    wave_sync();

    auto rsrc_b = [&](int tile) {
      const int col0 = tile * BN;
      return make_rsrc(a.cb + (int64_t)col0 * a.ldc, (int64_t)max(0, min(BN, a.N - col0)) * a.ldc * 2);
    };
    auto stage = [&](int slot, __amdgpu_buffer_rsrc_t rb, int ks, int tile) {
      char *st = smem + slot * STAGE;
      const uint32_t soff = (uint32_t)ks * (uint32_t)KB;
#pragma unroll
      for (int i = 0; i < BPIECES; i++) dma16(rb, st + (i * NW + wid) * 1024, b_voff[i], soff);
      if (XFORM && ks == 0) {
        // the tile's pre-filter column factors ride with its first K-step,
        // BN / NW per wave (one 4-byte DMA per lane)
        const int col0 = tile * BN + wid * CV_PER_WAVE;
        const __amdgpu_buffer_rsrc_t rc =
            make_rsrc(a.cpre + col0, (int64_t)max(0, min(CV_PER_WAVE, a.N - col0)) * 4);
        char *dst = (char *)(cv_l + (tile & 1) * BN + wid * CV_PER_WAVE);
        // lanes past CV_PER_WAVE stay masked (an LDS-DMA writes one dword per
        // ACTIVE lane); vmcnt still counts one instruction per wave
        if (lane < CV_PER_WAVE)
          __builtin_amdgcn_raw_ptr_buffer_load_lds(rc, (LDS_AS void *)dst, 4, (uint32_t)(lane * 4),
                                                   0, 0, 0);
      }
    };

    {
      const __amdgpu_buffer_rsrc_t rb0 = rsrc_b(t0);
      stage(0, rb0, 0, t0);
      if (KS > 1) stage(1, rb0, 1, t0);
      else stage(1, rsrc_b(t0 + 1), 0, t0 + 1);
    }
    int sl = 0;  // ring slot of the current K-step
    for (int tile = t0; tile < t1; tile++) {
      const __amdgpu_buffer_rsrc_t rb = rsrc_b(tile);
      const __amdgpu_buffer_rsrc_t rbn = rsrc_b(tile + 1);
      const __amdgpu_buffer_rsrc_t rbnn = (KS == 1) ? rsrc_b(tile + 2) : rbn;
      f32x16 acc[NB];
#pragma unroll
      for (int c = 0; c < NB; c++) acc[c] = (f32x16){};
#pragma unroll
      for (int ks = 0; ks < KS; ks++) {
        // step (tile, ks) landed: only step + 1's DMAs may still be in flight
        if (XFORM && (ks + 1) % KS == 0) wait_vm<BPIECES + 1>();
        else wait_vm<BPIECES>();
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
        const char *st = smem + sl * STAGE;
        // B fragments are double-buffered across substeps: the reads for
        // substep sub + 1 go out between the MFMAs of substep sub
        bf16x8 bq[2][NB];
#pragma unroll
        for (int c = 0; c < NB; c++)
          bq[0][c] = *(const bf16x8 *)(st + b_rd + c * 32 * KB + 16 * ((8 * h) ^ swz));
#pragma unroll
        for (int sub = 0; sub < KSUB; sub++) {
          const int cur = sub & 1;
          if (sub + 1 < KSUB) {
            const int co = 16 * ((8 * h + sub + 1) ^ swz);
#pragma unroll
            for (int c = 0; c < NB; c++) bq[cur ^ 1][c] = *(const bf16x8 *)(st + b_rd + c * 32 * KB + co);
          }
#pragma unroll
          for (int c = 0; c < NB; c++)
            acc[c] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[KSUB * ks + sub], bq[cur][c], acc[c], 0, 0, 0);
          if (sub + 1 < KSUB) {
#pragma unroll
            for (int c = 0; c < NB; c++) {
              __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);  // one LDS read
              __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);  // one MFMA
            }
          }
          if (sub == 0) {
            // step + 2 goes out behind the first MFMA group, into the slot
            // every wave finished reading before this step's barrier; past
            // the unit's last tile it is a harmless extra read (drained below)
            __builtin_amdgcn_sched_barrier(0);
            const int sl2 = (sl == 0) ? 2 : sl - 1;
            const int adv = (ks + 2) / KS;  // tiles ahead of this one (0..2)
            stage(sl2, adv == 0 ? rb : adv == 1 ? rbn : rbnn, (ks + 2) % KS, tile + adv);
            __builtin_amdgcn_sched_barrier(0);
          }
        }
        sl = (sl == NST - 1) ? 0 : sl + 1;
      }

      const int col0 = tile * BN;
      if (a.ablate == 1) {
        float sink = 0.0f;
#pragma unroll
        for (int c = 0; c < NB; c++)
#pragma unroll
          for (int e = 0; e < 16; e++) sink += acc[c][e];
        asm volatile("" ::"v"(sink));
        continue;
      }
      float lo[16];
#pragma unroll
      for (int e = 0; e < 16; e++) lo[e] = lo_w[acc_row(e, h)];
      // ---- fused top-k epilogue (as gemm_f32_kernel): pass 1 filters with
      // one op + compare per score and queues survivors (ballot + mbcnt);
      // pass 2 re-scores them exactly and appends to the candidate buffers.
      const float *cvt = cv_l + (tile & 1) * BN;
      u64 *gq = a.wq + ((size_t)blockIdx.x * NW + wid) * (size_t)(32 * BN);
      int qlen = 0;
      uint32_t opaque0;
      asm volatile("v_mov_b32 %0, 0" : "=v"(opaque0));
      const uint32_t lane_hi = opaque0 + 4u * (uint32_t)h + ((uint32_t)r32 << 5);
#pragma unroll
      for (int c = 0; c < NB; c++) {
        const int gcol = col0 + 32 * c + r32;
        const bool cvalid = gcol < a.N;
        const float cv = XFORM ? cvt[32 * c + r32] : 0.0f;
#pragma unroll
        for (int e = 0; e < 16; e++) {
          const float v = acc[c][e];
          float pv;
          if (METRIC == kMetricDot) pv = v;
          else if (METRIC == kMetricCosine) pv = v * cv;
          else pv = fmaf(2.0f, v, -cv);
          const bool p = cvalid && !(pv < lo[e]);
          const u64 m = __ballot(p);
          if (m == 0ull) continue;
          if (p && a.ablate != 2) {
            const uint32_t hi = lane_hi + (uint32_t)((e & 3) + 8 * (e >> 2) + ((32 * c) << 5));
            gq[qlen + lanes_below(m)] = (u64)__float_as_uint(v) | ((u64)hi << 32);
          }
          qlen += __popcll(m);
        }
      }
      if (a.ablate == 2) qlen = 0;
      if (qlen) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        for (int base = 0; base < qlen; base += 64) {
          const int i = base + lane;
          if (i < qlen) {
            const u64 it = __hip_atomic_load(gq + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            const float v = __uint_as_float((uint32_t)it);
            const int rl = (int)((it >> 32) & 31u);
            const int gcol = col0 + (int)(it >> 37);
            const float sc =
                exact_score<METRIC>(v, XFORM ? qex_w[rl] : 0.0f, XFORM ? a.cn[gcol] : 0.0f);
            const uint32_t key = okey32(METRIC == kMetricEuclidean ? -sc : sc);
            const u64 comp = ((u64)key << 32) | (u64)(~(uint32_t)gcol);
            if (comp > thr_w[rl]) {
              const unsigned pos = atomicAdd(&cnt_w[rl], 1u);
              a.cand[((int64_t)(wrow0 + rl) * a.S + s) * a.capg + pos] = comp;
            }
          }
          wave_sync();
          const unsigned cval = (lane < 32) ? cnt_w[lane] : 0u;
          u64 need = __ballot(lane < 32 && cval > (unsigned)(a.capg - 64));
          if (need) {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            while (need) {
              const int r = __builtin_ctzll(need);
              need &= need - 1;
              compact_row(a, s, wrow0 + r, thr_w + r, cnt_w + r, scr, lane);
            }
            if (lane < 32) lo_w[lane] = prefilter_bound<METRIC>(thr_w[lane], qex_w[lane]);
            wave_sync();
          }
        }
      }
    }
    // the two K-steps issued past the unit's last tile land before the ring
    // is reused by the next unit
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (lane < 32) {
      const int grow = wrow0 + lane;
      if (grow < a.M) a.cnt[(int64_t)grow * a.S + s] = cnt_w[lane];
    }
  }
}

template <int KS, int METRIC>
static hipError_t launch_bf16_t(const GemmF32Args &a, int grid, size_t lds, hipStream_t s) {
  static bool attr_set = false;
  if (!attr_set) {
    hipError_t e = hipFuncSetAttribute((const void *)gemm_bf16_kernel<KS, METRIC>,
                                       hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    if (e != hipSuccess) return e;
    attr_set = true;
  }
  gemm_bf16_kernel<KS, METRIC><<<dim3(grid), dim3(NW * 64), lds, s>>>(a);
  return hipGetLastError();
}

template <int KS>
static hipError_t launch_bf16_m(const GemmF32Args &a, int grid, size_t lds, hipStream_t s) {
  if (a.metric == kMetricCosine) return launch_bf16_t<KS, kMetricCosine>(a, grid, lds, s);
  if (a.metric == kMetricDot) return launch_bf16_t<KS, kMetricDot>(a, grid, lds, s);
  return launch_bf16_t<KS, kMetricEuclidean>(a, grid, lds, s);
}

hipError_t launch_gemm_bf16(const GemmF32Args &a, int grid, hipStream_t s) {
  const size_t lds = gemm_bf16_lds_bytes(a.capg);
  if (lds > 160 * 1024 || a.D % kBf16DAlign != 0) return hipErrorInvalidValue;
  switch (a.D / 128) {
    case 1: return launch_bf16_m<1>(a, grid, lds, s);
    case 2: return launch_bf16_m<2>(a, grid, lds, s);
    case 3: return launch_bf16_m<3>(a, grid, lds, s);
    case 4: return launch_bf16_m<4>(a, grid, lds, s);
    case 5: return launch_bf16_m<5>(a, grid, lds, s);
    case 6: return launch_bf16_m<6>(a, grid, lds, s);
    default: return hipErrorInvalidValue;
  }
}

}  // namespace pmm
