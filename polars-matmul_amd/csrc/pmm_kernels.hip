// pmm_kernels.hip -- gfx950 (MI355X / CDNA4) kernels of the similarity-search
// engine behind `.pmm.topk` / `.pmm.matmul`.
//
// Replaces, in one device pipeline, the reference's CPU chain
//   compute_norms_f32 (src/metrics.rs:382-393) ->
//   matmul_f32 via faer (src/metrics.rs:204-255) ->
//   cosine / euclidean epilogue over the full M x N matrix (src/metrics.rs:314-365) ->
//   select_topk_with_scores_f32 (src/topk.rs:42-75)
// with: an ndarray-order norm kernel, an f32 MFMA GEMM whose epilogue applies
// the metric and runs a threshold-pruned per-row top-k (the M x N score matrix
// never reaches HBM), and a merge kernel.  The same GEMM main loop in "store"
// mode is `.pmm.matmul` (src/metrics.rs:160-202).  f64 inputs use an f64 MFMA
// GEMM plus a row-select kernel (src/metrics.rs:258-311, src/topk.rs:6-39).
//
// Built with -ffp-contract=off: every FMA here is an explicit fmaf()/MFMA, so
// the epilogue arithmetic follows the reference's operation order.
#include "pmm_device.h"

#include <algorithm>

#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>

#include <type_traits>

namespace pmm {

hipError_t launch_norms_f32(const float *a, int64_t rows, int64_t d, int64_t ld, int squared,
                            float *out, float *inv, hipStream_t s) {
  if (rows <= 0) return hipSuccess;
  const int64_t threads = rows * 8;
  const unsigned grid = (unsigned)((threads + 255) / 256);
  norms_kernel<float><<<grid, 256, 0, s>>>(a, rows, d, ld, squared, out, inv);
  return hipGetLastError();
}
hipError_t launch_norms_pair_f32(const float *q, int64_t m, int64_t ldq, float *qout, const float *c,
                                 int64_t n, int64_t ldc, float *cout, float *cinv, int64_t d, int squared,
                                 hipStream_t s, void *zero, size_t zero_bytes) {
  const unsigned gq = (unsigned)((m * 8 + 255) / 256), gc = (unsigned)((n * 8 + 255) / 256);
  if (zero_bytes % 16 != 0 || ((uintptr_t)zero & 15)) return hipErrorInvalidValue;
  const int64_t zn = (int64_t)(zero_bytes / 16);
  const unsigned gz = (unsigned)std::min<int64_t>((zn + 255) / 256, 64);
  if (gq + gc + gz == 0) return hipSuccess;
  norms_pair_kernel<float><<<gq + gc + gz, 256, 0, s>>>(q, m, ldq, qout, c, n, ldc, cout, cinv, d, squared, gq,
                                                        gq + gc, (uint4 *)zero, zn);
  return hipGetLastError();
}
hipError_t launch_norms_f64(const double *a, int64_t rows, int64_t d, int64_t ld, int squared,
                            double *out, hipStream_t s) {
  if (rows <= 0) return hipSuccess;
  const int64_t threads = rows * 8;
  const unsigned grid = (unsigned)((threads + 255) / 256);
  norms_kernel<double><<<grid, 256, 0, s>>>(a, rows, d, ld, squared, out, nullptr);
  return hipGetLastError();
}


// ===========================================================================
// f32 MFMA GEMM: S = Q * C^T on v_mfma_f32_32x32x2_f32 (exact f32 FMA chain).
//
// Work unit = (query block of BM rows) x (corpus split of tps tiles of BN
// columns); persistent workgroups pull units from a counter, split-major, so
// the workgroups running together stream the same corpus tiles through the
// XCD L2s.  Workgroup = NW waves; wave w owns query rows [32w, 32w+32) of the
// block and all BN columns (NB 32x32 accumulators in AGPRs), so every per-row
// top-k state has exactly one owning wave and needs no cross-wave sync.
//
// K loop (BK = 32 floats = one 128-byte row piece per operand row): both the
// wave's query rows and the shared corpus tile are staged HBM -> LDS by
// buffer_load ... lds (LDS-DMA, 16 B per lane, double-buffered, one barrier
// per step).  The buffer resources carry the row range, so rows past M / N
// read as zeros with no clamping, and each lane's byte offset is loop
// invariant (the step advances only the scalar soffset).  The 16-byte chunks
// of every 128-byte row are XOR-swizzled on the SOURCE address (chunk ^
// ((row>>1)&7)) so the ds_read_b128 fragment reads hit 16 distinct bank slots.
// Fragments are fed in natural K order (substep t pairs k = 2t and 2t+1, see
// the K loop), so each output is the k-ordered fmaf chain of the oracle
// bit for bit (v_mfma_f32_32x32x2_f32 is an exact f32 FMA chain).
// ===========================================================================
#ifndef PMM_F32_DEFER
#define PMM_F32_DEFER 1
#endif

// The K-step ring is double-buffered.  (A deeper ring for the small
// variants -- step g + NS - 1 issued from asm behind step g, counted vmcnt
// waits -- measured slower at c1 with 3-5 stages: 0.080 vs 0.074 ms per
// fused launch, profiles/r4_c1/deep_ring_ab.txt; round 3 found the same for
// 128 x 128.  The loop does not wait on the corpus stream.)
constexpr int kF32Stages = 2;

// AK (query rows resident): the unit's query block stays in LDS for all its
// K steps (loaded once at unit start, after the carve below), and the ring
// stages hold corpus pieces only -- every tile after the first re-streamed
// the block from L2 (two thirds of a 128 x 64 tile's DMA at D = 256).
template <int NB, int NW, bool AK = false>
struct GemmShape {
  static constexpr int NS = kF32Stages;
  // CSP (column split; variant 5): 8 waves, 2 per SIMD, in pairs -- waves w
  // and w + 4 own the same 32 query rows (row group w & 3) and one 32-column
  // half of the tile each, with separate top-k state (candidate segments
  // 2 s + half).  One wave per SIMD left the K step's LDS latency and the
  // tile epilogue uncovered at the reference's own size; a partner wave on
  // the SIMD issues MFMAs meanwhile.
  static constexpr bool CSP = NB == 2 && NW == 8;
  static constexpr int RG = CSP ? NW / 2 : NW;      // row groups of 32
  static constexpr int NBW = CSP ? NB / 2 : NB;     // 32-column blocks per wave
  static constexpr int BN = 32 * NB;                // corpus columns per tile
  static constexpr int BM = 32 * RG;                // query rows per workgroup
  static constexpr int RS = 32 * NW;                // per-wave row-state slots
  static constexpr int A_BYTES = RG * 4096;         // RG row groups x 32 rows x 128 B
  static constexpr int B_BYTES = BN * 128;          // BN rows x 128 B
  static constexpr int A_IN_STAGE = AK ? 0 : A_BYTES;
  static constexpr int STAGE = A_IN_STAGE + B_BYTES;
  static constexpr int BPIECES = B_BYTES / 1024 / NW;  // 1 KiB LDS-DMA pieces per wave
  static constexpr int OFF_THR = NS * STAGE;
  static constexpr int OFF_CNT = OFF_THR + RS * 8;
  static constexpr int OFF_QEX = OFF_CNT + RS * 4;   // exact row norm (epilogue)
  static constexpr int OFF_LO = OFF_QEX + RS * 4;    // pre-filter bound per row
  static constexpr int OFF_CV = OFF_LO + RS * 4;     // column factors, NS tiles
  // column norms of the exact re-scores, NS tiles, and the survivor queue in
  // LDS: the small variants only (the 256 x 256 one's carve has no room left
  // at k = 100; its survivors are rare after a unit's first tiles)
  static constexpr bool CNL = NB <= 4 && (NW == 4 || CSP);
  static constexpr int OFF_CN = OFF_CV + NS * BN * 4;
  static constexpr int OFF_UNIT = OFF_CN + (CNL ? NS * BN * 4 : 0);
  static constexpr int OFF_SCR = OFF_UNIT + 16;
  static_assert(B_BYTES % (1024 * NW) == 0, "corpus tile must split into 1 KiB pieces per wave");
  static_assert(OFF_SCR % 16 == 0, "LDS carve must stay 16-byte aligned");
};

// Tile-shape variants compiled in (index = GemmVariant id).
//   0: NB=4 NW=4 (128 x 128, 1 wave/SIMD)   1: NB=8 NW=4 (128 x 256)
//   2: NB=4 NW=8 (256 x 128, 2 waves/SIMD)  3: NB=8 NW=8 (256 x 256)
//   4: NB=2 NW=4 (128 x 64, 1 wave/SIMD: finer units for small problems)
//   5: NB=2 NW=8 (128 x 64, 2 waves/SIMD splitting the columns: GemmShape::CSP)
constexpr int kGemmVariants = 6;
constexpr int kVarNB[kGemmVariants] = {4, 8, 4, 8, 2, 2};
constexpr int kVarNW[kGemmVariants] = {4, 4, 8, 8, 4, 8};
constexpr int kVarRG[kGemmVariants] = {4, 4, 8, 8, 4, 4};  // row groups of 32

int gemm_f32_bm(int variant) { return 32 * kVarRG[variant]; }
int gemm_f32_bn(int variant) { return 32 * kVarNB[variant]; }
int gemm_f32_nw(int variant) { return kVarNW[variant]; }
int gemm_f32_segs(int variant) { return variant == 5 ? 2 : 1; }

// bytes at ns LDS stages; the fit checks use the double-buffered carve
// (ks_resident > 0: the AK carve, query rows of ks_resident K steps after it)
static size_t gemm_f32_lds_bytes_ak(int variant, int mode, int capg, int ks_resident) {
  const int ns = kF32Stages;
  const int nb = kVarNB[variant], nw = kVarNW[variant];
  const bool csp = variant == 5;  // GemmShape::CSP: no compaction scratch (capg <= 512)
  const size_t a_bytes = (size_t)kVarRG[variant] * 4096;
  const size_t stage = (ks_resident ? 0 : a_bytes) + (size_t)32 * nb * 128;
  const bool cnl = nb <= 4 && (nw == 4 || csp);  // GemmShape::CNL
  const size_t fixed = ns * stage + (size_t)32 * nw * 20 + (size_t)(cnl ? 2 : 1) * ns * 32 * nb * 4 + 16;
  if (csp && capg > 512) return size_t(1) << 30;  // (its compactions select: capg <= 512 only)
  return fixed + (mode == 0 && !csp ? (size_t)nw * capg * 8 : 0) + (size_t)ks_resident * a_bytes;
}
size_t gemm_f32_lds_bytes(int variant, int mode, int capg) { return gemm_f32_lds_bytes_ak(variant, mode, capg, 0); }


// K order of the f32 MFMA chain (A/B builds: -DPMM_F32_KORDER=n):
//   2 (default): natural order; the LDS image of every 32-float K step is laid
//      out by 4-byte LDS-DMA gathers so that lane half h's 16-byte fragment
//      read of chunk 2qd+h holds k = 8qd+h, +2, +4, +6: MFMA substep t = 4qd+j
//      pairs k = 2t (h = 0) with 2t+1 (h = 1) straight from one ds_read_b128;
//   3: natural order, corpus image gathered, query image by 16-byte DMA with
//      two v_permlane32_swap per query fragment;
//   1: natural order from 16-byte DMA + two v_permlane32_swap per fragment;
//   0: round-1 permuted order (substep pairs k = 4qd+j with 16+4qd+j; NOT
//      bit-exact vs the oracle's k-ordered chain).
#ifndef PMM_F32_KORDER
#define PMM_F32_KORDER 2
#endif
// The small variants (128 x 128 and 128 x 64, 1 wave per SIMD) use order 3:
// at c1 order 2's 4-byte DMA issues for the query rows (32 per wave per K
// step) were not hidden behind another wave's MFMAs (round 2, 128 x 128:
// order 1/3 0.148 ms per call, order 2 0.153); with the 128 x 64 tile order 3
// (corpus gathered, query 16-byte + swaps) beats order 1: c1 fused kernel
// 73-74 vs 75-76 us, c2 71 vs 74 (profiles/r3_c1/korder_small_ab.txt).
// Every order here but 0 is natural, so all variants return the same bits.
#ifndef PMM_F32_KORDER_SMALL
#define PMM_F32_KORDER_SMALL 3
#endif

template <int NB, int NW, int MODE, int METRIC, bool AK>
__global__ __launch_bounds__(NW * 64, NW / 4) void gemm_f32_kernel(GemmF32Args a) {
  using G = GemmShape<NB, NW, AK>;
  constexpr int NS = G::NS;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  u64 *thr_l = (u64 *)(smem + G::OFF_THR);
  unsigned *cnt_l = (unsigned *)(smem + G::OFF_CNT);
  float *qex_l = (float *)(smem + G::OFF_QEX);
  float *lo_l = (float *)(smem + G::OFF_LO);
  float *cv_l = (float *)(smem + G::OFF_CV);
  float *cn_l = (float *)(smem + G::OFF_CN);
  int *unit_l = (int *)(smem + G::OFF_UNIT);

  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  constexpr bool CSP = G::CSP;
  constexpr int NBW = G::NBW;
  const int rg = CSP ? (wid & (G::RG - 1)) : wid;  // this wave's row group
  const int half = CSP ? (wid / G::RG) : 0;        // CSP: this wave's column half of the tile
  const int r32 = lane & 31, h = lane >> 5;
  const int KS = a.D >> 5;
  // (CSP: no compaction scratch -- capg <= 512 selects in registers)
  u64 *scr = CSP ? nullptr : (u64 *)(smem + G::OFF_SCR) + (size_t)wid * a.capg;
  // AK: the resident query rows, [KS][RG row groups][32 rows x 128 B]
  char *a_res = smem + G::OFF_SCR + (MODE == 0 && !CSP ? (size_t)NW * a.capg * 8 : 0);
  // the survivor queue's first a.qcap entries per wave (the rest: a.wq)
  u64 *lq = (u64 *)(a_res + (AK ? (size_t)KS * G::A_BYTES : 0)) + (size_t)wid * a.qcap;
  u64 *thr_w = thr_l + wid * 32;
  unsigned *cnt_w = cnt_l + wid * 32;
  float *qex_w = qex_l + wid * 32;  // per-row constants live in LDS, not in VGPRs
  float *lo_w = lo_l + wid * 32;    // across the K loop (keeps 256x256 spill-free)
  constexpr bool XFORM = (METRIC != kMetricDot);
  // (lab build with -DPMM_F32_STATS and PMM_STATS=1: per-wave phase cycles,
  // summed over waves -- s_memtime reads, one vector atomic per counter at
  // the end)
#ifdef PMM_F32_STATS
  const bool timing = a.stats != nullptr;
#else
  constexpr bool timing = false;
#endif
  auto stamp = [&]() __attribute__((always_inline)) { return timing ? __builtin_amdgcn_s_memtime() : 0ull; };
  const uint64_t t_start = stamp();
  uint64_t cy_bar = 0, cy_loop = 0, cy_epi = 0, cy_unit = 0, n_tiles = 0, cy_pf = 0, cy_comp = 0, n_surv = 0, cy_flags = 0;

  // Loop-invariant per-lane byte offsets of this wave's LDS-DMA pieces.
  // Gathered image (4-byte pieces of 256 LDS bytes = 2 rows): LDS dword p of
  // a row (physical chunk p>>2, element j = p&3) holds logical chunk
  // ch = (p>>2) ^ swizzle, i.e. k = 8*(ch>>1) + (ch&1) + 2j.  Plain image
  // (16-byte pieces of 1 KiB = 8 rows): chunk ch of a row at ch ^ swizzle.
  constexpr int KO = (NB <= 4 && (NW == 4 || CSP)) ? PMM_F32_KORDER_SMALL : PMM_F32_KORDER;
  constexpr bool A_GATHER = KO == 2;
  constexpr bool B_GATHER = KO == 2 || KO == 3;
  constexpr int AP = A_GATHER ? 16 : 4, APIECE = A_GATHER ? 256 : 1024, ADW = A_GATHER ? 4 : 16;
  constexpr int BP = B_GATHER ? 4 * G::BPIECES : G::BPIECES, BPIECE = B_GATHER ? 256 : 1024,
                BDW = B_GATHER ? 4 : 16;
  auto kofs = [&](int row) __attribute__((always_inline)) {
    const int p = lane & 31;
    const int ch = (p >> 2) ^ ((row >> 1) & 7);
    return 4 * (8 * (ch >> 1) + (ch & 1) + 2 * (p & 3));
  };
  uint32_t a_voff[AP], b_voff[BP];
#pragma unroll
  for (int i = 0; i < AP; i++) {
    if (A_GATHER) {
      const int row = 2 * i + (lane >> 5);
      a_voff[i] = (uint32_t)(row * a.ldq * 4 + kofs(row));
    } else {
      const int row = 8 * i + (lane >> 3);
      const int ch = (lane & 7) ^ ((row >> 1) & 7);
      a_voff[i] = (uint32_t)(row * a.ldq * 4 + ch * 16);
    }
  }
#pragma unroll
  for (int i = 0; i < BP; i++) {
    if (B_GATHER) {
      const int col = 2 * (i * NW + wid) + (lane >> 5);
      b_voff[i] = (uint32_t)(col * a.ldc * 4 + kofs(col));
    } else {
      const int col = (i * NW + wid) * 8 + (lane >> 3);
      const int ch = (lane & 7) ^ ((col >> 1) & 7);
      b_voff[i] = (uint32_t)(col * a.ldc * 4 + ch * 16);
    }
  }
  // Per-lane LDS read offsets (within a stage).
  const int swz = (r32 >> 1) & 7;
  const int a_rd = rg * 4096 + r32 * 128;
  const int b_rd = G::A_IN_STAGE + r32 * 128;

  int buf = 0;
  for (;;) {
    const uint64_t tu0 = stamp();
    if (tid == 0) *unit_l = (int)atomicAdd(a.counter, 1u);
    __syncthreads();
    const int unit = *unit_l;
    __syncthreads();
    if (unit >= a.units) break;
    // units [0, qb_full): whole query blocks (every tile, candidate segment
    // 0: a row's threshold and buffer carry over the whole corpus); then the
    // remaining blocks as (split, block) units, split-major
    int s, qb, t0, t1;
    if (MODE == 0 && unit < a.qb_full) {
      qb = unit;
      s = 0;
      t0 = 0;
      t1 = a.ntiles;
    } else {
      const int u2 = MODE == 0 ? unit - a.qb_full : unit;
      const int qbb = MODE == 0 ? a.QB - a.qb_full : a.QB;
      s = u2 / qbb;
      qb = (MODE == 0 ? a.qb_full : 0) + (u2 - s * qbb);
      t0 = s * a.tps;
      t1 = min(t0 + a.tps, a.ntiles);
    }
    const int wrow0 = qb * G::BM + rg * 32;
    const int seg = CSP ? 2 * s + half : s;  // this wave's candidate segment
    const __amdgpu_buffer_rsrc_t ra =
        make_rsrc(a.q + (int64_t)wrow0 * a.ldq, (int64_t)min(32, a.M - wrow0) * a.ldq * 4);

    // Per-lane row constants for the 16 accumulator rows this lane holds.
    if (lane < 32) {
      const int grow = wrow0 + lane;
      const float qv = (XFORM && grow < a.M) ? a.qn[grow] : 0.0f;
      qex_w[lane] = qv;
      if (MODE == 0) {
        const u64 t = (grow < a.M) ? __hip_atomic_load(a.gthr + grow, __ATOMIC_RELAXED,
                                                        __HIP_MEMORY_SCOPE_AGENT)
                                   : ~0ull;
        thr_w[lane] = t;
        lo_w[lane] = prefilter_bound<METRIC>(t, qv);
        cnt_w[lane] = 0u;
      }
    }
    wave_sync();

    auto rsrc_b = [&](int tile) {
      const int col0 = tile * G::BN;
      return make_rsrc(a.c + (int64_t)col0 * a.ldc, (int64_t)min(G::BN, a.N - col0) * a.ldc * 4);
    };
    // DMA pieces [lo, hi) of one K step (A pieces first, then B pieces)
    auto stage = [&](int sb, __amdgpu_buffer_rsrc_t rb, int ks, int tile, int lo, int hi) {
      char *st = smem + sb * G::STAGE;
      const uint32_t soff = (uint32_t)ks * 128u;
      // (the 16-byte form stays behind the dma16 helper: used directly in a
      // kernel body, the gfx950-only size silently drops the kernel's host stub)
      auto dma = [&](__amdgpu_buffer_rsrc_t r, char *dst, uint32_t voff, int dw) __attribute__((always_inline)) {
        if (dw == 4) __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (LDS_AS void *)dst, 4, voff, soff, 0, 0);
        else dma16(r, dst, voff, soff);
      };
      // (ablation build, PMM_ABLATE=3 / 4: the query rows load only in the
      // unit's first tile -- later tiles read stale rows, results wrong)
      const bool skip_a = (PMM_ABL(a.ablate) == 3 || PMM_ABL(a.ablate) == 4) && tile != t0;
      constexpr int AS = AK ? 0 : AP;  // A pieces per step in the ring
#pragma unroll
      for (int i = 0; i < AS; i++)
        if (i >= lo && i < hi && !skip_a && half == 0) dma(ra, st + rg * 4096 + i * APIECE, a_voff[i], ADW);
#pragma unroll
      for (int i = 0; i < BP; i++)
        if (AS + i >= lo && AS + i < hi) dma(rb, st + G::A_IN_STAGE + (i * NW + wid) * BPIECE, b_voff[i], BDW);
      if (MODE == 0 && XFORM && ks == 0 && wid == 0 && lo == 0) {
        // the tile's pre-filter column factors ride with its first K step
        const int col0 = tile * G::BN;
        const __amdgpu_buffer_rsrc_t rc =
            make_rsrc(a.cpre + col0, (int64_t)min(G::BN, a.N - col0) * 4);
        // (and, small variants, the column norms of its exact re-scores)
        const __amdgpu_buffer_rsrc_t rn = make_rsrc(a.cn + col0, (int64_t)min(G::BN, a.N - col0) * 4);
        char *dst = (char *)(cv_l + ((unsigned)tile % NS) * G::BN);
        char *dsn = (char *)(cn_l + ((unsigned)tile % NS) * G::BN);
#pragma unroll
        for (int i = 0; i < G::BN / 64; i++) {
          __builtin_amdgcn_raw_ptr_buffer_load_lds(rc, (LDS_AS void *)(dst + i * 256), 4,
                                                   (uint32_t)(lane * 4 + i * 256), 0, 0, 0);
          if (G::CNL)
            __builtin_amdgcn_raw_ptr_buffer_load_lds(rn, (LDS_AS void *)(dsn + i * 256), 4,
                                                     (uint32_t)(lane * 4 + i * 256), 0, 0, 0);
        }
      }
    };

    // the next K step's DMA goes out behind MFMA groups 0 .. NPART-1 of this
    // one, TP / NPART pieces each (the natural-order image takes 4x the
    // pieces of the 16-byte form; spread, they do not stall one group)
    constexpr int TP = (AK ? 0 : AP) + BP;
#ifndef PMM_F32_DMA_PARTS
#define PMM_F32_DMA_PARTS 1  // (A/B at c3: 4 measured 7% slower, 2 1.1% slower)
#endif
#ifndef PMM_F32_DMA_PARTS_SMALL
#define PMM_F32_DMA_PARTS_SMALL 2
#endif
    // (the 128 x 128 variant runs one wave per SIMD: no second wave's MFMAs
    // cover this wave's DMA issue; its 8 pieces per step go out 4 behind each
    // of the first two MFMA groups: c1 0.141 vs 0.143 ms, c2 0.134 vs 0.136;
    // 2 behind each of four groups 0.146 / 0.139)
    constexpr int NPART = (NB <= 4 && (NW == 4 || CSP)) ? PMM_F32_DMA_PARTS_SMALL : PMM_F32_DMA_PARTS;
// The large variants' pre-filter in two passes: per-lane survivor flags with
// no branches, their OR over the wave, then ballot + append at the flagged
// positions only (wave-uniform element index).  The one-pass form ran a
// compare -> ballot -> branch chain per score (~50 cycles each, MFMA idle):
// c3 1053.7 / 1055.1 vs 1063.1 / 1063.6 ms, alternated on one box
// (profiles/r5_pf2/ab.txt); the queue order and so the results are unchanged.
#ifndef PMM_F32_PF2
#define PMM_F32_PF2 1
#endif
#ifndef PMM_F32_FLAT_QUEUE
#define PMM_F32_FLAT_QUEUE 1
#endif
#ifndef PMM_F32_FRAG_PREFETCH
#define PMM_F32_FRAG_PREFETCH 1  // (A/B: 0 off, 1 the 128 x 128 variant only, 2 every variant)
#endif
    constexpr bool FPF = PMM_F32_FRAG_PREFETCH == 2 || (PMM_F32_FRAG_PREFETCH == 1 && NB <= 4 && (NW == 4 || CSP));
    // (one ballot per 32 x 32 block before the per-score ones -- the max of
    // the pre-filter differences -- measured flat at c3 in round 2 and slower
    // at c1 in round 3: 0.083-0.085 vs 0.082 ms,
    // profiles/r3_c1/block_prefilter_ab.txt)
    static_assert(TP % NPART == 0 && NPART <= 4, "DMA pieces split evenly over the MFMA groups");
    __amdgpu_buffer_rsrc_t rb = rsrc_b(t0);
    if (AK) {
      // the unit's query rows, every K step, once (the unit-start barriers
      // above: every wave is done with the previous unit's rows)
      for (int ks = 0; ks < KS && half == 0; ks++)
#pragma unroll
        for (int i = 0; i < AP; i++) {
          char *dst = a_res + ks * G::A_BYTES + rg * 4096 + i * APIECE;
          if (ADW == 4)
            __builtin_amdgcn_raw_ptr_buffer_load_lds(ra, (LDS_AS void *)dst, 4, a_voff[i], (uint32_t)ks * 128u, 0, 0);
          else
            dma16(ra, dst, a_voff[i], (uint32_t)ks * 128u);
        }
    }
    stage(buf, rb, 0, t0, 0, TP);
    if (timing) cy_unit += stamp() - tu0;
    for (int tile = t0; tile < t1; tile++) {
      const uint64_t tl0 = stamp();
      const bool last_tile = (tile + 1) >= t1;
      const __amdgpu_buffer_rsrc_t rbn = last_tile ? rb : rsrc_b(tile + 1);
      f32x16 acc[NBW];
#pragma unroll
      for (int c = 0; c < NBW; c++) acc[c] = (f32x16){};
      // PMM_F32_DEFER: the last substep(s) of a K step (NB MFMAs each, their
      // operands one A and NB B values) run after the next step's barrier,
      // behind the next step's first fragment reads -- the same MFMA order
      // per accumulator, so the same bits
      constexpr int DN = PMM_F32_DEFER;  // substeps deferred (1 or 2)
      static_assert(DN >= 0 && DN <= 2, "PMM_F32_DEFER: 0, 1 or 2 substeps");
      float dA[DN > 0 ? DN : 1], dB[DN > 0 ? DN : 1][NBW];
      // one K step; DEF: defer its last substep, PREV: run the previous
      // step's deferred substep first (compile-time, so no per-substep branch)
      auto kstep = [&](int ks, auto DEF, auto PREV) __attribute__((always_inline)) {
        const uint64_t tb0 = stamp();
        __syncthreads();  // stage `buf` landed (vmcnt(0) + barrier); buf^1 free
        if (timing) cy_bar += stamp() - tb0;
        const char *st = smem + buf * G::STAGE;
        // KORDER 0: lane half h covers k = 16h..16h+15 (substep j of group
        // qd pairs k = 4qd+j with 16+4qd+j).  Otherwise half h reads chunk
        // 2qd+h: from a gathered image element j is k = 8qd+h+2j, so
        // substep t = 4qd+j pairs k = 2t (h = 0) with 2t+1 (h = 1) -- every
        // output is the k-ordered fmaf chain of the oracle bit for bit; from
        // a plain image (k = 8qd+4h..+3) two v_permlane32_swap trade the
        // lower half's odd k for the upper half's even k, leaving registers
        // {0,2,1,3} = k pairs (8qd,+1) (8qd+2,+3) (8qd+4,+5) (8qd+6,+7).
        auto rd_frag = [&](int qd, f32x4 &av, f32x4 (&b)[NBW]) __attribute__((always_inline)) {
          const int co = KO == 0 ? 16 * ((4 * h + qd) ^ swz) : 16 * ((2 * qd + h) ^ swz);
          av = *(const f32x4 *)((AK ? a_res + ks * G::A_BYTES : st) + a_rd + co);
#pragma unroll
          for (int c = 0; c < NBW; c++) b[c] = *(const f32x4 *)(st + b_rd + (half * NBW + c) * 4096 + co);
        };
        // FPF: group qd + 1's fragments are read before group qd's MFMAs, so
        // only a K step's first group waits on a fresh LDS read (one wave per
        // SIMD has no partner wave to cover that latency)
        f32x4 avs[FPF ? 2 : 1], bs[FPF ? 2 : 1][NBW];
        if (FPF) rd_frag(0, avs[0], bs[0]);
#pragma unroll
        for (int qd = 0; qd < 4; qd++) {
          if (FPF && qd < 3) {
            rd_frag(qd + 1, avs[(qd + 1) & 1], bs[(qd + 1) & 1]);
            __builtin_amdgcn_sched_barrier(0);  // (hipcc would sink the reads to the group's end)
          }
          if (!FPF) rd_frag(qd, avs[0], bs[0]);
          f32x4 &av = avs[FPF ? (qd & 1) : 0];
          f32x4(&b)[NBW] = bs[FPF ? (qd & 1) : 0];
          constexpr bool A_SWAP = KO == 1 || KO == 3;
          constexpr bool B_SWAP = KO == 1;
          auto kpair = [](f32x4 &x) __attribute__((always_inline)) {
            auto r0 = __builtin_amdgcn_permlane32_swap(__float_as_uint(x[0]), __float_as_uint(x[1]), false, false);
            auto r1 = __builtin_amdgcn_permlane32_swap(__float_as_uint(x[2]), __float_as_uint(x[3]), false, false);
            x[0] = __uint_as_float(r0[0]);
            x[1] = __uint_as_float(r0[1]);
            x[2] = __uint_as_float(r1[0]);
            x[3] = __uint_as_float(r1[1]);
          };
          if (decltype(PREV)::value && qd == 0) {
            // the previous step's deferred substeps, behind this step's reads
#pragma unroll
            for (int j = 0; j < DN; j++)
#pragma unroll
              for (int c = 0; c < NBW; c++)
                acc[c] = __builtin_amdgcn_mfma_f32_32x32x2f32(dA[j], dB[j][c], acc[c], 0, 0, 0);
          }
          if (A_SWAP) kpair(av);
#pragma unroll
          for (int c = 0; c < NBW; c++)
            if (B_SWAP) kpair(b[c]);
#pragma unroll
          for (int jj = 0; jj < 4; jj++) {
            const int js = ((jj & 1) << 1) | (jj >> 1);  // swapped registers: {0, 2, 1, 3}
            const int ja = A_SWAP ? js : jj, jb = B_SWAP ? js : jj;
            if (decltype(DEF)::value && qd == 3 && jj >= 4 - DN) {
              dA[jj - (4 - DN)] = av[ja];
#pragma unroll
              for (int c = 0; c < NBW; c++) dB[jj - (4 - DN)][c] = b[c][jb];
            } else {
#pragma unroll
              for (int c = 0; c < NBW; c++)
                acc[c] = __builtin_amdgcn_mfma_f32_32x32x2f32(av[ja], b[c][jb], acc[c], 0, 0, 0);
            }
          }
          if (qd < NPART) {
            // next step's LDS-DMA goes out behind the MFMA groups, so the
            // matrix pipe restarts right after the barrier
            __builtin_amdgcn_sched_barrier(0);
            constexpr int PER = TP / NPART;
            if (ks + 1 < KS) {
              stage(buf ^ 1, rb, ks + 1, tile, qd * PER, qd * PER + PER);
            } else if (!last_tile) {
              stage(buf ^ 1, rbn, 0, tile + 1, qd * PER, qd * PER + PER);
            }
            __builtin_amdgcn_sched_barrier(0);
          }
        }
        buf = buf + 1 == NS ? 0 : buf + 1;
      };
      using Yes = std::integral_constant<bool, true>;
      using No = std::integral_constant<bool, false>;
      if (!PMM_F32_DEFER || KS == 1) {
        for (int ks = 0; ks < KS; ks++) kstep(ks, No{}, No{});
      } else {
        kstep(0, Yes{}, No{});
        for (int ks = 1; ks + 1 < KS; ks++) kstep(ks, Yes{}, Yes{});
        kstep(KS - 1, No{}, Yes{});
      }
      rb = rbn;
      const uint64_t te0 = stamp();
      if (timing) {
        cy_loop += te0 - tl0;
        n_tiles++;
      }

      const int col0 = tile * G::BN;
      if (PMM_ABL(a.ablate) == 1 || PMM_ABL(a.ablate) == 4) {
        // ablation build path: keep the accumulators live, skip the epilogue
        float sink = 0.0f;
#pragma unroll
        for (int c = 0; c < NBW; c++)
#pragma unroll
          for (int e = 0; e < 16; e++) sink += acc[c][e];
        asm volatile("" ::"v"(sink));
        continue;
      }
      float rv[16], lo[16];
#pragma unroll
      for (int e = 0; e < 16; e++) {
        rv[e] = qex_w[acc_row(e, h)];
        lo[e] = (MODE == 0) ? lo_w[acc_row(e, h)] : 0.0f;
      }
      if (MODE == 1) {
        // ---- store epilogue (.pmm.matmul, or materialised scores) ----
#pragma unroll
        for (int c = 0; c < NBW; c++) {
          const int gcol = col0 + 32 * (half * NBW + c) + r32;
          if (gcol < a.N) {
            const float cv = XFORM ? a.cn[gcol] : 0.0f;
#pragma unroll
            for (int e = 0; e < 16; e++) {
              const int grow = wrow0 + acc_row(e, h);
              if (grow < a.M) {
                const float v = acc[c][e];
                a.out[(int64_t)grow * a.ldo + gcol] =
                    (XFORM && a.store_metric) ? exact_score<METRIC>(v, rv[e], cv) : v;
              }
            }
          }
        }
      } else {
        // ---- fused top-k epilogue ----
        // Pass 1 (accumulators live): one pre-filter op + compare per score;
        // survivors (rare after a unit's first tiles) are appended to this
        // wave's queue with ballot + mbcnt slots (no atomics).  Pass 2
        // (accumulators dead): re-score the queue exactly, 64 items at a time
        // (one per lane), and append to the rows' candidate buffers.  The
        // queue lives in global memory (L2): a tile can produce up to
        // 32 x BN survivors per wave (a unit's first tile).
        const float *cvt = cv_l + ((unsigned)tile % NS) * G::BN;
        const float *cnt_t = cn_l + ((unsigned)tile % NS) * G::BN;
        u64 *gq = a.wq + ((size_t)blockIdx.x * NW + wid) * (size_t)(32 * G::BN);
        int qlen = 0;  // wave-uniform
        // queue item high word = row-in-wave | col-in-tile << 5 = lane part +
        // a per-(c, e) constant; the opaque zero keeps the compiler from
        // hoisting all 16*NB constants out of the tile loop into registers
        uint32_t opaque0;
        asm volatile("v_mov_b32 %0, 0" : "=v"(opaque0));
        const uint32_t lane_hi = opaque0 + 4u * (uint32_t)h + ((uint32_t)r32 << 5);
        auto prefilter = [&](float v, float cv) __attribute__((always_inline)) {
          if (METRIC == kMetricDot) return v;
          if (METRIC == kMetricCosine) return v * cv;
          return fmaf(2.0f, v, -cv);
        };
        if (G::CNL) {
          // small variants (16 NB <= 64 scores per lane): every score's flag
          // first (VALU only), one wave prefix sum of the lanes' counts, then
          // each lane appends its own survivors at consecutive slots.  (A
          // ballot + branch + slot per score serialised the 16 NB compares
          // on scalar round trips: ~7 us of the c1 kernel's 74.)  The queue
          // order changes; the results do not (any order of appends keeps a
          // row's buffer a superset of its top-k above the threshold).
          u64 bits = 0ull;
#pragma unroll
          for (int c = 0; c < NBW; c++) {
            const int tb = half * NBW + c;  // the 32-column block of the tile
            const bool cvalid = col0 + 32 * tb + r32 < a.N;
            const float cv = XFORM ? cvt[32 * tb + r32] : 0.0f;
#pragma unroll
            for (int e = 0; e < 16; e++)
              if (cvalid && !(prefilter(acc[c][e], cv) < lo[e])) bits |= 1ull << (16 * c + e);
          }
          const int nl = __popcll(bits);  // <= 64: 7 bits
          int excl = 0, tot = 0;
#pragma unroll
          for (int j = 0; j < 7; j++) {
            const u64 m = __ballot((nl >> j) & 1);
            excl += lanes_below(m) << j;
            tot += __popcll(m) << j;
          }
          if (timing) cy_flags += stamp() - te0;
          if (bits && PMM_ABL(a.ablate) != 2) {
            int qi = qlen + excl;
#pragma unroll
            for (int c = 0; c < NBW; c++)
#pragma unroll
              for (int e = 0; e < 16; e++)
                if ((bits >> (16 * c + e)) & 1ull) {
                  const uint32_t hi =
                      lane_hi + (uint32_t)((e & 3) + 8 * (e >> 2) + ((32 * (half * NBW + c)) << 5));
                  const u64 item = (u64)__float_as_uint(acc[c][e]) | ((u64)hi << 32);
#if PMM_F32_FLAT_QUEUE
                  // one generic (flat) store, LDS or global by address: no
                  // second divergent branch per position
                  u64 *dst = qi < a.qcap ? lq + qi : gq + qi;
                  *dst = item;
#else
                  if (qi < a.qcap) lq[qi] = item;
                  else gq[qi] = item;
#endif
                  qi++;
                }
          }
          qlen += tot;
        } else {
#if PMM_F32_PF2
          // pass 1, no branches: each lane's survivor flags (16 per column
          // block c, two blocks per word), then their OR over the wave -- the
          // positions (c, e) where some lane holds a survivor; only those
          // take the ballot + append below
          uint32_t fl[(NBW + 1) / 2], U[(NBW + 1) / 2];
#pragma unroll
          for (int i = 0; i < (NBW + 1) / 2; i++) fl[i] = 0u;
#pragma unroll
          for (int c = 0; c < NBW; c++) {
            const float cv = XFORM ? cvt[32 * c + r32] : 0.0f;
            uint32_t f = 0u;
#pragma unroll
            for (int e = 0; e < 16; e++) f |= (prefilter(acc[c][e], cv) < lo[e]) ? 0u : (1u << e);
            if (col0 + 32 * c + r32 >= a.N) f = 0u;
            fl[c >> 1] |= f << (16 * (c & 1));
          }
#pragma unroll
          for (int i = 0; i < (NBW + 1) / 2; i++) {
            uint32_t x = fl[i];
#pragma unroll
            for (int off = 32; off; off >>= 1) x |= (uint32_t)__shfl_xor((int)x, off);
            U[i] = __builtin_amdgcn_readfirstlane(x);
          }
          // pass 2: the flagged positions only, block by block (e is
          // wave-uniform: the accumulator element is read by index)
#pragma unroll
          for (int c = 0; c < NBW; c++) {
            uint32_t uc = (U[c >> 1] >> (16 * (c & 1))) & 0xFFFFu;
            while (uc) {
              const int e = __builtin_ctz(uc);
              uc &= uc - 1u;
              const bool p = (fl[c >> 1] >> (16 * (c & 1) + e)) & 1u;
              const u64 m = __ballot(p);
              if (p && PMM_ABL(a.ablate) != 2) {
                const uint32_t hi = lane_hi + (uint32_t)((e & 3) + 8 * (e >> 2) + ((32 * c) << 5));
                gq[qlen + lanes_below(m)] = (u64)__float_as_uint(acc[c][e]) | ((u64)hi << 32);
              }
              qlen += __popcll(m);
            }
          }
        }
#else
#pragma unroll
          for (int c = 0; c < NBW; c++) {
            const int gcol = col0 + 32 * c + r32;
            const bool cvalid = gcol < a.N;
            const float cv = XFORM ? cvt[32 * c + r32] : 0.0f;
#pragma unroll
            for (int e = 0; e < 16; e++) {
              const float v = acc[c][e];
              const float pv = prefilter(v, cv);
              const bool p = cvalid && !(pv < lo[e]);
              const u64 m = __ballot(p);
              if (m == 0ull) continue;
              if (p && PMM_ABL(a.ablate) != 2) {
                const uint32_t hi = lane_hi + (uint32_t)((e & 3) + 8 * (e >> 2) + ((32 * c) << 5));
                gq[qlen + lanes_below(m)] = (u64)__float_as_uint(v) | ((u64)hi << 32);
              }
              qlen += __popcll(m);
            }
          }
        }
#endif
        if (timing) {
          cy_pf += stamp() - te0;
          n_surv += (uint64_t)qlen;
        }
        if (PMM_ABL(a.ablate) == 2) qlen = 0;  // ablation: pre-filter only
        if (qlen) {
          // queue entries past the LDS part: their stores reached L2
          if (!G::CNL || qlen > a.qcap) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
          if (G::CNL) wave_sync();  // every lane's LDS queue entries written
          for (int base = 0; base < qlen; base += 64) {
            const int i = base + lane;
            if (i < qlen) {
              // (global part: an sc1 load bypasses this CU's L1, reads what
              // the stores left in L2)
              const u64 it = (G::CNL && i < a.qcap) ? lq[i]
                                                    : __hip_atomic_load(gq + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
              const float v = __uint_as_float((uint32_t)it);
              const int rl = (int)((it >> 32) & 31u);
              const int tc = (int)(it >> 37);
              const int gcol = col0 + tc;
              const float sc =
                  exact_score<METRIC>(v, XFORM ? qex_w[rl] : 0.0f, XFORM ? (G::CNL ? cnt_t[tc] : a.cn[gcol]) : 0.0f);
              const uint32_t key = okey32(METRIC == kMetricEuclidean ? -sc : sc);
              const u64 comp = ((u64)key << 32) | (u64)(~(uint32_t)gcol);
              if (comp > thr_w[rl]) {
                const unsigned pos = atomicAdd(&cnt_w[rl], 1u);
                a.cand[((int64_t)(wrow0 + rl) * a.S + seg) * a.capg + pos] = comp;
              }
            }
            // compact every row whose buffer could overflow on the next 64 appends
            wave_sync();
            const unsigned cval = (lane < 32) ? cnt_w[lane] : 0u;
            u64 need = __ballot(lane < 32 && cval > (unsigned)a.ctrig);
            if (need) {
              const uint64_t tc0 = stamp();
              asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
              while (need) {
                const int r = __builtin_ctzll(need);
                need &= need - 1;
                compact_row(a, seg, wrow0 + r, thr_w + r, cnt_w + r, scr, lane);
              }
              if (lane < 32) lo_w[lane] = prefilter_bound<METRIC>(thr_w[lane], qex_w[lane]);
              wave_sync();
              if (timing) cy_comp += stamp() - tc0;
            }
          }
        }
      }
      if (timing) cy_epi += stamp() - te0;
    }

    if (MODE == 0) {
      if (lane < 32) {
        const int grow = wrow0 + lane;
        if (grow < a.M) a.cnt[(int64_t)grow * a.S + seg] = cnt_w[lane];
      }
    }
  }
  if (timing && lane == 0) {
    atomicAdd(a.stats + 0, (u64)(stamp() - t_start));
    atomicAdd(a.stats + 1, (u64)cy_bar);
    atomicAdd(a.stats + 2, (u64)cy_loop);
    atomicAdd(a.stats + 3, (u64)cy_epi);
    atomicAdd(a.stats + 4, (u64)cy_unit);
    atomicAdd(a.stats + 5, (u64)n_tiles);
    atomicAdd(a.stats + 6, (u64)cy_pf);
    atomicAdd(a.stats + 7, (u64)cy_comp);
    atomicAdd(a.stats + 8, (u64)n_surv);
    atomicAdd(a.stats + 9, (u64)cy_flags);
  }
}

// (top-k mode: the survivor queue's LDS part takes what the carve leaves of
// the CU's 160 KiB, up to a tile's 32 x BN entries per wave, in 64-entry
// steps; PMM_F32_QCAP=0: the global queue only, for A/B runs)
template <int NB, int NW, int MODE, int METRIC, bool AK>
static hipError_t launch_gemm_f32_t(const GemmF32Args &a_in, int grid, size_t lds, hipStream_t s) {
  GemmF32Args a = a_in;
  a.qcap = 0;
  static const bool lq_on = !(getenv("PMM_F32_QCAP") && atoi(getenv("PMM_F32_QCAP")) == 0);
  if (MODE == 0 && GemmShape<NB, NW, AK>::CNL && lq_on && lds < 160 * 1024) {
    const size_t per = (160 * 1024 - lds) / (NW * 8);
    a.qcap = (int)(std::min<size_t>(per, 32 * 32 * NB) / 64 * 64);
    lds += (size_t)NW * a.qcap * 8;
  }
  static bool attr_set = false;  // opt in to > 64 KiB dynamic LDS
  if (!attr_set) {
    hipError_t e = hipFuncSetAttribute((const void *)gemm_f32_kernel<NB, NW, MODE, METRIC, AK>,
                                       hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    if (e != hipSuccess) return e;
    attr_set = true;
  }
  gemm_f32_kernel<NB, NW, MODE, METRIC, AK><<<dim3(grid), dim3(NW * 64), lds, s>>>(a);
  return hipGetLastError();
}

template <int NB, int NW, bool AK = false>
static hipError_t launch_gemm_f32_v(const GemmF32Args &a, int mode, int grid, size_t lds, hipStream_t s) {
  if (mode == 0) {
    if (a.metric == kMetricCosine) return launch_gemm_f32_t<NB, NW, 0, kMetricCosine, AK>(a, grid, lds, s);
    if (a.metric == kMetricDot) return launch_gemm_f32_t<NB, NW, 0, kMetricDot, AK>(a, grid, lds, s);
    return launch_gemm_f32_t<NB, NW, 0, kMetricEuclidean, AK>(a, grid, lds, s);
  }
  if (!a.store_metric || a.metric == kMetricDot)
    return launch_gemm_f32_t<NB, NW, 1, kMetricDot, AK>(a, grid, lds, s);
  if (a.metric == kMetricCosine) return launch_gemm_f32_t<NB, NW, 1, kMetricCosine, AK>(a, grid, lds, s);
  return launch_gemm_f32_t<NB, NW, 1, kMetricEuclidean, AK>(a, grid, lds, s);
}

// Small variants: resident query rows (PMM_F32_AK, default on) when the unit
// spans more than one tile and the carve fits (c1: 128 rows x D 256 = 128 KiB
// of the 160), else the rows re-stream with every tile.
#ifndef PMM_F32_AK
#define PMM_F32_AK 1
#endif
template <int NB, int NW>
static hipError_t launch_gemm_f32_small(const GemmF32Args &a, int variant, int mode, int grid, hipStream_t s) {
  const size_t ak = gemm_f32_lds_bytes_ak(variant, mode, a.capg, a.D >> 5);
  static const int ak_env = getenv("PMM_F32_AK") ? atoi(getenv("PMM_F32_AK")) : PMM_F32_AK;
  if (ak_env && a.tps > 1 && ak <= 160 * 1024) return launch_gemm_f32_v<NB, NW, true>(a, mode, grid, ak, s);
  return launch_gemm_f32_v<NB, NW>(a, mode, grid, gemm_f32_lds_bytes(variant, mode, a.capg), s);
}

hipError_t launch_gemm_f32(const GemmF32Args &a, int variant, int mode, int grid, hipStream_t s) {
  const size_t lds = gemm_f32_lds_bytes(variant, mode, a.capg);
  if (lds > 160 * 1024) return hipErrorInvalidValue;
  switch (variant) {
    case 0: return launch_gemm_f32_small<4, 4>(a, variant, mode, grid, s);
    case 1: return launch_gemm_f32_v<8, 4>(a, mode, grid, lds, s);
    case 2: return launch_gemm_f32_v<4, 8>(a, mode, grid, lds, s);
    case 3: return launch_gemm_f32_v<8, 8>(a, mode, grid, lds, s);
    case 4: return launch_gemm_f32_small<2, 4>(a, variant, mode, grid, s);
    case 5: return mode == 0 ? launch_gemm_f32_small<2, 8>(a, variant, mode, grid, s) : hipErrorInvalidValue;
    default: return hipErrorInvalidValue;
  }
}

// ===========================================================================
// Merge: one wave per query row streams candidate entries, keeps those at or
// above the row threshold in an LDS scratch of P slots, compacts (sort, keep
// k) when the scratch fills, and writes the final best-first k_out.
//   loader 0: the fused kernel's per-(row, split) candidate buffers; the
//             shared threshold gthr[row] is a lower bound of the final k-th
//             composite, so everything below it is dropped on load.
//   loader 1: gathered per-shard (idx, score) lists [M][S][k_in] (multi-GPU).
// ===========================================================================
// Merge scratch layout (PMM_MERGE_SWZ; MP maps a slot to its LDS position,
// MPN is the slots allocated per wave).  A ds_read_b64 / ds_write_b64 is
// served in two 32-lane groups, conflict-free when a group's 32 slots are
// distinct mod 32.  The bitonic partners of strides 1..16 hit slots e and
// e + 32 in one group (2-way conflicts at every such step):
//   0: plain slots (default);
//   1: one u64 of padding every 32 slots (slot + slot / 32): fixes stride 1
//      only;
//   2: slots 32..63 of every 64 XOR 31 (bits 0-4 flipped when bit 5 is set):
//      every bitonic step conflict-free, no extra LDS.
// Measured at c3 (alternated, tools/experiments/merge_swz.sh): 0.378-0.381
// ms plain, 0.427-0.428 padded, 0.443-0.445 swizzled; c1 equal.  The merge
// is issue- and latency-bound: the index arithmetic costs more than the
// conflict cycles it removes.
#ifndef PMM_MERGE_SWZ
#define PMM_MERGE_SWZ 0
#endif
#if PMM_MERGE_SWZ == 1
#define MP(i) ((i) + ((i) >> 5))
#define MPN(P) MP(P)
#elif PMM_MERGE_SWZ == 2
#define MP(i) ((i) ^ ((((i) >> 5) & 1) * 31))
#define MPN(P) (P)
#else
#define MP(i) (i)
#define MPN(P) (P)
#endif
#ifndef PMM_MERGE_SEL_E
#define PMM_MERGE_SEL_E 1
#endif
// Chunk loads per batch (two batches in flight when pipelined) and the
// merge kernels' occupancy floor.  The merge is bound by each wave's
// dependent chain (counts -> chunks -> select -> sort -> write), so waves per
// SIMD count: at 4 chunks per batch merge_kernel<0> took 80 VGPRs (6 waves);
// 2 per batch and a 7-wave floor fit it in 72 with no scratch.  Round 6,
// alternated on one box (profiles/r6_merge/occupancy_ab.txt): c3 0.424 ->
// 0.401 ms, c4 0.288 -> 0.262, c5_rank 2.55 -> 2.33, c1 equal; 3 per batch
// the same.  (A floor of 8 spills; a 64-VGPR lab build measured alike.)
#ifndef PMM_MERGE_MU
#define PMM_MERGE_MU 2
#endif
__device__ inline void wave_sort_desc_u64_pad(u64 *s, int P, int lane) {
  for (int size = 2; size <= P; size <<= 1) {
    for (int stride = size >> 1; stride > 0; stride >>= 1) {
      for (int i = lane; i < (P >> 1); i += 64) {
        const int x0 = ((i & ~(stride - 1)) << 1) | (i & (stride - 1));
        const int x1 = x0 + stride;
        const u64 a = s[MP(x0)], b = s[MP(x1)];
        const bool desc = (x0 & size) == 0;
        if (desc ? (a < b) : (a > b)) {
          s[MP(x0)] = b;
          s[MP(x1)] = a;
        }
      }
      wave_sync();
    }
  }
}

// Ranks of the n (<= 128) distinct keys a wave holds in slots lane (y0) and
// 64 + lane (y1): r = the number of keys above it, by broadcasting each key
// with v_readlane (no LDS round trips; see launch_merge for when it pays).
__device__ inline u64 readlane_u64(u64 v, int j) {
  return ((u64)(uint32_t)__builtin_amdgcn_readlane((uint32_t)(v >> 32), j) << 32) |
         (u64)(uint32_t)__builtin_amdgcn_readlane((uint32_t)v, j);
}
__device__ inline void wave_rank2(u64 y0, u64 y1, int n, int &r0, int &r1) {
  r0 = 0;
  r1 = 0;
  const int n0 = n < 64 ? n : 64;
  for (int j = 0; j < n0; j++) {
    const u64 v = readlane_u64(y0, j);
    r0 += v > y0;
    r1 += v > y1;
  }
  for (int j = 64; j < n; j++) {
    const u64 v = readlane_u64(y1, j - 64);
    r0 += v > y0;
    r1 += v > y1;
  }
}
// Bitonic sort, best first, of 128 keys held two per lane in registers (key
// i: lane i & 63, y0 for i < 64, y1 above).  Partners at lane distance 1, 2,
// 4, 8 by DPP (quad_perm, and 4 / 8 as two mirrors: row_half_mirror then
// quad reverse = lane ^ 4, row_mirror then row_half_mirror = lane ^ 8), 16
// by ds_bpermute, 32 by v_permlane32_swap, 64 inside the lane: no LDS round
// trip per stage, against the LDS network's 28 read -> compare -> write
// stages (wave_sort_desc_u64_pad).  Round 6, alternated on one box
// (profiles/r6_merge/sort128_ab.txt): merge c3 0.402 -> 0.375 ms, c4 0.267
// -> 0.231, c5_rank 2.33 -> 2.19; the whole GPU suite passed with every
// merge forced onto it (PMM_MERGE_RANK=0).  The compare-exchange as a lane
// mask (below) and bound_ctrl moves: 0.377 -> 0.329 at c3, 0.222 -> 0.178
// at c4, 2.13 -> 1.61 at c5_rank (profiles/r6_merge/sort128_mask_ab.txt).
#ifndef PMM_MERGE_SORT128
#define PMM_MERGE_SORT128 1
#endif
// (every permutation used here gives every lane a valid source, so
// bound_ctrl costs nothing and spares update_dpp's copy of an old value:
// kway_merge_kernel 85 -> 78 VGPRs)
template <int CTRL>
__device__ __forceinline__ uint32_t dpp_mov(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, CTRL, 0xF, 0xF, true);
}
template <int S>
__device__ __forceinline__ uint32_t lane_xor_u32(uint32_t v, int lane) {
  if constexpr (S == 1) return dpp_mov<0xB1>(v);                    // quad_perm [1,0,3,2]
  else if constexpr (S == 2) return dpp_mov<0x4E>(v);               // quad_perm [2,3,0,1]
  else if constexpr (S == 4) return dpp_mov<0x1B>(dpp_mov<0x141>(v));  // half mirror, quad reverse
  else if constexpr (S == 8) return dpp_mov<0x141>(dpp_mov<0x140>(v)); // row mirror, half mirror
  else if constexpr (S == 16) return (uint32_t)__shfl_xor((int)v, 16);
  else {
    // lanes 32-63 of the first operand swap with lanes 0-31 of the second:
    // r[0] = both halves' low half, r[1] = both halves' high half
    const auto r = __builtin_amdgcn_permlane32_swap(v, v, false, false);
    return lane < 32 ? r[1] : r[0];
  }
}
// element i keeps the larger of (i, i ^ S) iff (i is the pair's lower) ==
// (i's SIZE-block sorts descending: i & SIZE == 0); i = lane + 64 r.  As a
// compile-time lane mask per register: one compare into a lane mask, one
// scalar xor with it, two selects per key (against two selects per max and
// per min and a third pair to choose between them).
template <int SIZE, int S, int R>
constexpr unsigned long long sort128_keepmax() {
  unsigned long long m = 0;
  for (int l = 0; l < 64; l++) {
    const bool lower = (l & S) == 0;
    const bool d = SIZE > 64 ? true : (SIZE == 64 ? R == 0 : (l & SIZE) == 0);
    if (lower == d) m |= 1ull << l;
  }
  return m;
}
template <int SIZE, int S>
__device__ __forceinline__ void sort128_step(u64 &y0, u64 &y1, int lane) {
  auto px = [&](u64 v) __attribute__((always_inline)) {
    return ((u64)lane_xor_u32<S>((uint32_t)(v >> 32), lane) << 32) | (u64)lane_xor_u32<S>((uint32_t)v, lane);
  };
  const u64 p0 = px(y0), p1 = px(y1);
  // take the partner's key where (mine is larger) != (I keep the larger)
  const u64 t0 = __ballot(y0 > p0) ^ sort128_keepmax<SIZE, S, 0>();
  const u64 t1 = __ballot(y1 > p1) ^ sort128_keepmax<SIZE, S, 1>();
  y0 = __builtin_amdgcn_inverse_ballot_w64(t0) ? p0 : y0;
  y1 = __builtin_amdgcn_inverse_ballot_w64(t1) ? p1 : y1;
}
template <int SIZE, int S>
__device__ __forceinline__ void sort128_merge(u64 &y0, u64 &y1, int lane) {
  sort128_step<SIZE, S>(y0, y1, lane);
  if constexpr (S > 1) sort128_merge<SIZE, S / 2>(y0, y1, lane);
}
__device__ inline void wave_sort128_desc(u64 &y0, u64 &y1, int lane) {
  sort128_merge<2, 1>(y0, y1, lane);
  sort128_merge<4, 2>(y0, y1, lane);
  sort128_merge<8, 4>(y0, y1, lane);
  sort128_merge<16, 8>(y0, y1, lane);
  sort128_merge<32, 16>(y0, y1, lane);
  sort128_merge<64, 32>(y0, y1, lane);
  // size 128: (i, i + 64) inside the lane, then distances 32 .. 1, all descending
  const u64 mx = y0 > y1 ? y0 : y1, mn = y0 > y1 ? y1 : y0;
  y0 = mx;
  y1 = mn;
  sort128_merge<128, 32>(y0, y1, lane);
}

// the k best of the cnt (<= 64 E) keys in scr, unordered, to its front.
// The raised threshold comes back by value with the count: a threshold the
// callee wrote through a pointer lived in scratch memory, and every scratch
// read of it (one per taken batch) waited for the batch loads in flight
// (scratch counts in vmcnt).
struct CompactOut {
  int cnt;
  u64 T;
};
template <int E>
__device__ inline CompactOut merge_select(u64 *scr, int cnt, int k, u64 T, int lane) {
  u64 x[E];
#pragma unroll
  for (int e = 0; e < E; e++) x[e] = (lane + 64 * e < cnt) ? scr[MP(lane + 64 * e)] : 0ull;
  wave_sync();  // every lane has read before any rewrites
  const u64 t = wave_kth_u64<E>(x, k);
  if (t > T) T = t;
  cnt = wave_keep_ge<E>(x, t, [&](int pos, u64 v) __attribute__((always_inline)) { scr[MP(pos)] = v; }, lane);
  wave_sync();
  return {cnt, T};
}

__device__ CompactOut merge_compact(u64 *scr, int cnt, int k, int P, u64 T, int lane) {
  if (P <= 512 && cnt > k) {
    // select the k best (wave_kth_u64) over as few key slots per lane as
    // hold cnt: its cost is a compare per slot per bit
#if PMM_MERGE_SEL_E
    if (cnt <= 128) return merge_select<2>(scr, cnt, k, T, lane);
    if (cnt <= 256) return merge_select<4>(scr, cnt, k, T, lane);
#endif
    return merge_select<8>(scr, cnt, k, T, lane);
  }
  for (int i = cnt + lane; i < P; i += 64) scr[MP(i)] = 0ull;
  wave_sync();
  wave_sort_desc_u64_pad(scr, P, lane);
  if (cnt >= k) {
    const u64 t = scr[MP(k - 1)];
    if (t > T) T = t;
    cnt = k;
  }
  wave_sync();
  return {cnt, T};
}

template <int LOADER, bool SPLIT, bool SORTED>
__device__ __forceinline__ void merge_row(const MergeArgs &a, const int rpos, const int wid, const int lane,
                                          char *smem) {
  // kMergeSplitRow (few rows, many lists, k <= 64): the block's 4 waves take
  // one row, wave w merging lists [S w / 4, S (w + 1) / 4) down to its k best;
  // wave 0 then selects the row's k best of those 4 lists.  Otherwise one
  // wave per row; the only block-wide barrier is the split mode's, where
  // every wave of the block has a row (grid = M).
  // (a template parameter: the one-wave-per-row instantiation keeps its
  // registers -- a runtime flag cost it an occupancy step, c3 0.57 vs 0.44 ms)
  constexpr bool split = SPLIT;
  // kMergeReverse: the split units' rows (many segments each) sit after the
  // whole query blocks' rows (one segment); started first, the long rows no
  // longer form the launch's tail
  const int row = (a.flags & kMergeReverse) ? a.M - 1 - rpos : rpos;
  const int s_lo = split ? a.S * wid / 4 : 0, s_hi = split ? a.S * (wid + 1) / 4 : a.S;
  u64 *scr = (u64 *)smem + (size_t)wid * MPN(a.P);
  u64 T = (LOADER == 0) ? a.gthr[row] : 0ull;
  int cnt = 0;
  // candidate i of list s as a composite key (0 = empty)
  auto load_x = [&](int s, int i) __attribute__((always_inline)) -> u64 {
    if (LOADER == 0) return a.cand[((int64_t)row * a.S + s) * a.capg + i];
    const int64_t off = (int64_t)row * a.row_stride + (int64_t)s * a.list_stride + i;
    const uint32_t id = a.in_idx[off];
    const float sc = a.in_score[off];
    const u64 key = ((u64)okey32(a.metric == kMetricEuclidean ? -sc : sc) << 32) | (u64)(~id);
    return id != 0xFFFFFFFFu ? key : 0ull;
  };
  auto take = [&](u64 x) __attribute__((always_inline)) {
    const bool keep = x >= (T ? T : 1ull);  // (x != 0 and x >= T in one compare)
    const u64 m = __ballot(keep);
    const int pos = cnt + lanes_below(m);
    if (keep) scr[MP(pos)] = x;
    cnt += __popcll(m);
    if (cnt > a.P - 64) {
      wave_sync();
      {
        const CompactOut o = merge_compact(scr, cnt, a.k_out, a.P, T, lane);
        cnt = o.cnt;
        T = o.T;
      }
    }
  };
  bool done = false;
  if (SORTED) {
    const int c = min(a.k_in, 256 / a.S);  // prefix read per list (launch_merge: S <= 64)
    const int n = a.S * c;
    u64 x[4];
    u64 ul = 0ull;  // this lane's last-read entries of lists not read to the end
    // (loads unconditional from clamped positions, keys selected: no load
    // under a branch, so the four are in flight together)
#pragma unroll
    for (int j = 0; j < 4; j++) {
      const int f = j * 64 + lane;
      const bool valid = f < n;
      const int g = valid ? f / c : 0, i = valid ? f - g * c : 0;
      const u64 v = load_x(g, i);
      x[j] = valid ? v : 0ull;
      if (valid && i == c - 1 && c < a.k_in && v > ul) ul = v;
    }
    const u64 U = wave_max_u64(ul);
    int nge = 0, nz = 0;
#pragma unroll
    for (int j = 0; j < 4; j++) {
      nge += __popcll(__ballot(x[j] != 0ull && x[j] >= U));
      nz += __popcll(__ballot(x[j] != 0ull));
    }
    if (nge >= a.k_out || (U == 0ull)) {
      // (U == 0: every list read to its end, or its unread part empty slots)
      const u64 t = nz > a.k_out ? wave_kth_u64<4>(x, a.k_out) : 1ull;
      cnt = wave_keep_ge<4>(x, t, [&](int pos, u64 v) __attribute__((always_inline)) { scr[MP(pos)] = v; }, lane);
      done = true;
    }
  }
  if (done || PMM_ABL(a.ablate) == 2) {
    // (ablate 2, benchmarking only: no candidate loads)
  } else if (a.S <= 64) {
    // All list lengths in one load (lane s holds list s's), then the lists'
    // 64-entry chunks as one flat sequence, MU chunk loads in flight at a
    // time: the row's reads no longer wait on one another (HBM latency, not
    // bandwidth, bounded the per-list loop).  (A flat per-slot loader -- prefix
    // sums + a binary search per slot -- measured the same at c1 and 29%
    // slower at c3.)
    constexpr int MU = PMM_MERGE_MU;  // (see PMM_MERGE_MU; at c1's split rows 2, 4 and 8 measured alike)
    // (lists [s_lo, s_hi): lane j holds list s_lo + j's length)
    const int nl = (s_lo + lane < s_hi)
                       ? ((LOADER == 0) ? (int)a.cnt[(int64_t)row * a.S + s_lo + lane] : a.k_in)
                       : 0;
    int s = s_lo, c = 0;
    int ns = __builtin_amdgcn_readlane(nl, 0);  // (0 when the wave has no list)
    while (s < s_hi && c >= ns) {  // first non-empty list
      s++;
      ns = (s < s_hi) ? __builtin_amdgcn_readlane(nl, s - s_lo) : 0;
    }
    // A batch: the positions of its MU chunks first (scalar bookkeeping),
    // then MU loads with no branch around them, each from its position or,
    // past the lists, from a valid dummy one, flagged invalid; the flag is
    // applied where the key is taken.  (A load under a branch, or a register
    // a load is still filling copied at a branch join, waits for the load
    // there: round 5's batches did both, so each batch paid a full memory
    // latency before the next went out.)
    auto fetch = [&](u64(&x)[MU], bool(&vx)[MU]) __attribute__((always_inline)) {
      int ps[MU], pc[MU], pn[MU];
#pragma unroll
      for (int u = 0; u < MU; u++) {
        ps[u] = s;
        pc[u] = c;
        pn[u] = (s < s_hi) ? ns : 0;
        if (s < s_hi) {
          c += 64;
          while (s < s_hi && c >= ns) {
            s++;
            c = 0;
            ns = (s < s_hi) ? __builtin_amdgcn_readlane(nl, s - s_lo) : 0;
          }
        }
      }
#pragma unroll
      for (int u = 0; u < MU; u++) {
        const int i = pc[u] + lane;
        vx[u] = i < pn[u];
        x[u] = load_x(vx[u] ? ps[u] : s_lo, vx[u] ? i : 0);
      }
    };
    if (a.flags & kMergePipelined) {
      // the next batch's loads go out before this one is taken (a row's
      // batches no longer pay one memory latency each); two register sets
      // in turn, never copied into each other
      if (s < s_hi) {
        u64 x[MU], y[MU];
        bool vx[MU], vy[MU];
        fetch(x, vx);
        for (;;) {
          bool more = s < s_hi;
          if (more) fetch(y, vy);
#pragma unroll
          for (int u = 0; u < MU; u++) take(vx[u] ? x[u] : 0ull);
          if (!more) break;
          more = s < s_hi;
          if (more) fetch(x, vx);
#pragma unroll
          for (int u = 0; u < MU; u++) take(vy[u] ? y[u] : 0ull);
          if (!more) break;
        }
      }
    } else {
      while (s < s_hi) {
        u64 x[MU];
        bool vx[MU];
        fetch(x, vx);
#pragma unroll
        for (int u = 0; u < MU; u++) take(vx[u] ? x[u] : 0ull);
      }
    }
  } else {
    for (int s = s_lo; s < s_hi; s++) {
      const int n_s = (LOADER == 0) ? (int)a.cnt[(int64_t)row * a.S + s] : a.k_in;
      for (int i0 = 0; i0 < n_s; i0 += 64) {
        const int i = i0 + lane;
        take(i < n_s ? load_x(s, i) : 0ull);
      }
    }
  }
  wave_sync();
  auto put = [&](int j, u64 x) __attribute__((always_inline)) {
    uint32_t id = 0xFFFFFFFFu;
    float sc = __uint_as_float(0x7FC00000u);
    if (x != 0ull) {
      id = (~(uint32_t)x) + (LOADER == 0 ? a.index_base : 0u);
      const float v = dekey32((uint32_t)(x >> 32));
      // euclidean keys rank -distance; 0 - v (not -v) returns a zero
      // distance as +0.0, the oracle's sqrt(max(., 0))
      sc = (a.metric == kMetricEuclidean) ? 0.0f - v : v;
    }
    a.out_idx[(int64_t)row * a.k_out + j] = id;
    a.out_score[(int64_t)row * a.k_out + j] = sc;
  };
  if (split) {
    // each wave's k best (k <= 64: one slot per lane), then wave 0 takes the
    // row's k best of the four lists into its own scratch
    if (cnt > a.k_out) {
        const CompactOut o = merge_compact(scr, cnt, a.k_out, a.P, T, lane);
        cnt = o.cnt;
        T = o.T;
      }
    int *cnts = (int *)((u64 *)smem + (size_t)4 * MPN(a.P));
    if (lane == 0) cnts[wid] = cnt;
    __syncthreads();
    if (wid != 0) return;
    u64 x[4];
    int tot = 0;
#pragma unroll
    for (int e = 0; e < 4; e++) {
      const int ce = cnts[e];
      x[e] = lane < ce ? ((const u64 *)smem + (size_t)e * MPN(a.P))[MP(lane)] : 0ull;
      tot += ce;
    }
    wave_sync();  // every lane has read before wave 0's scratch is rewritten
    const u64 t = tot > a.k_out ? wave_kth_u64<4>(x, a.k_out) : 1ull;
    cnt = wave_keep_ge<4>(x, t, [&](int pos, u64 v) __attribute__((always_inline)) { scr[MP(pos)] = v; }, lane);
    wave_sync();
  }
  if (PMM_ABL(a.ablate) != 1) {
    // (lab ablate 4: no selection, the first k_out kept; 5: no ranking, slot
    // order; 6: neither -- benchmarking only, results wrong)
    if ((PMM_ABL(a.ablate) == 4 || PMM_ABL(a.ablate) == 6) && cnt > a.k_out) cnt = a.k_out;
    if (cnt > a.k_out && a.P <= 512) {
        const CompactOut o = merge_compact(scr, cnt, a.k_out, a.P, T, lane);
        cnt = o.cnt;
        T = o.T;
      }
    if (PMM_ABL(a.ablate) == 5 || PMM_ABL(a.ablate) == 6) {
      for (int j = lane; j < a.k_out; j += 64) put(j, (j < cnt) ? scr[MP(j)] : 0ull);
      return;
    }
    if (PMM_MERGE_SORT128 && a.k_out <= 128 && cnt <= 128 && a.no_rank) {
      u64 y0 = lane < cnt ? scr[MP(lane)] : 0ull;
      u64 y1 = 64 + lane < cnt ? scr[MP(64 + lane)] : 0ull;
      wave_sort128_desc(y0, y1, lane);  // (empty slots, 0, sort last)
      if (lane < a.k_out) put(lane, y0);
      if (64 + lane < a.k_out) put(64 + lane, y1);
      return;
    }
    if (a.k_out <= 128 && cnt <= a.k_out && !a.no_rank) {
      // best-first by rank counting, no sort: each kept key goes to the
      // position = the number of kept keys above it (keys are distinct)
      const u64 y0 = lane < cnt ? scr[MP(lane)] : 0ull;
      const u64 y1 = 64 + lane < cnt ? scr[MP(64 + lane)] : 0ull;
      int r0, r1;
      wave_rank2(y0, y1, cnt, r0, r1);
      if (lane < cnt) put(r0, y0);
      if (64 + lane < cnt) put(r1, y1);
      for (int j = cnt + lane; j < a.k_out; j += 64) put(j, 0ull);
      return;
    }
    const int P2 = min(a.P, next_pow2_dev(cnt));
    for (int i = cnt + lane; i < P2; i += 64) scr[MP(i)] = 0ull;
    wave_sync();
    wave_sort_desc_u64_pad(scr, P2, lane);
  }
  for (int j = lane; j < a.k_out; j += 64) put(j, (j < cnt) ? scr[MP(j)] : 0ull);
}

#ifndef PMM_MERGE_WAVES
#define PMM_MERGE_WAVES 7  // (min waves per SIMD: the register budget, see PMM_MERGE_MU)
#endif
template <int LOADER, bool SPLIT, bool SORTED = false>
__global__ __launch_bounds__(256, PMM_MERGE_WAVES) void merge_kernel(MergeArgs a) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int wpb = blockDim.x >> 6;
  const int rpos = SPLIT ? (int)blockIdx.x : (int)blockIdx.x * wpb + wid;
  if (rpos >= a.M) return;  // whole wave exits
  merge_row<LOADER, SPLIT, SORTED>(a, rpos, wid, lane, smem);
}

// ===========================================================================
// k-way merge of 5..8 sorted lists per row (loader 1, MergeArgs::sorted: the
// root merge of the corpus-sharded path, configs[4]).  Eight rows per wave,
// eight lanes per row, lane g of a row holding list g: the first kKwayP
// entries of every list are staged in LDS as composite keys (coalesced: 32
// lanes read one list's 128 contiguous bytes per plane), then k_out steps of
// a true merge -- the row's largest head by three DPP max steps inside the
// 8-lane group, its list advances, the group's first lane writes the entry.
// A list that would need entries past its staged prefix (its share of the
// answer exceeds kKwayP: skewed shards) marks its row, which the wave then
// merges again by the general path (merge_row) over every entry.  ~30 vector
// instructions per step for 8 rows at once, no selection and no sort: the
// lists' order is the merge's order.
// ===========================================================================
__device__ __forceinline__ u64 dpp_u64(u64 v, int ctrl_sel) {
  uint32_t lo = (uint32_t)v, hi = (uint32_t)(v >> 32);
  if (ctrl_sel == 0) {  // row_half_mirror: lane i of each 8 <- lane 7 - i
    lo = dpp_mov<0x141>(lo);
    hi = dpp_mov<0x141>(hi);
  } else if (ctrl_sel == 1) {  // quad_perm [2,3,0,1]: lane xor 2
    lo = dpp_mov<0x4E>(lo);
    hi = dpp_mov<0x4E>(hi);
  } else {  // quad_perm [1,0,3,2]: lane xor 1
    lo = dpp_mov<0xB1>(lo);
    hi = dpp_mov<0xB1>(hi);
  }
  return ((u64)hi << 32) | lo;
}
template <int KP>
__global__ __launch_bounds__(256) void kway_merge_kernel(MergeArgs a) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  constexpr int kKwayP = KP;
  u64 *st = (u64 *)smem + (size_t)wid * 64 * kKwayP;  // [segment 8 r + g][kKwayP]
  const int row0 = ((int)blockIdx.x * (int)(blockDim.x >> 6) + wid) * 8;
  if (row0 >= a.M) return;  // whole wave exits
  const int lim = min(kKwayP, a.k_in);
  // stage: iteration t, lanes 32 h .. 32 h + 31 take entries 0..31 of
  // segment 2 t + h (row row0 + s / 8, list s % 8)
  // (loads unconditional, from a clamped offset, and the key selected: a
  // load under a branch waits for its data before the next is issued)
  // (all of a batch's loads first, then its LDS stores: the LDS pointer is
  // generic, so a load may not pass an earlier store)
  static_assert(KP <= 32, "staged prefix: one lane per entry");
  for (int t0 = 0; t0 < 32; t0 += 8) {  // (64 segments, two per iteration)
    uint32_t id[8];
    float sc[8];
#pragma unroll
    for (int u = 0; u < 8; u++) {
      const int sg = 2 * (t0 + u) + (lane >> 5), e = lane & 31;
      const int r = sg >> 3, g = sg & 7, row = row0 + r;
      const bool valid = row < a.M && g < a.S && e < lim;  // (e >= KP: lim <= KP)
      const int64_t off = valid ? (int64_t)row * a.row_stride + (int64_t)g * a.list_stride + e : 0;
      id[u] = a.in_idx[off];
      sc[u] = a.in_score[off];
      if (!valid) id[u] = 0xFFFFFFFFu;
    }
#pragma unroll
    for (int u = 0; u < 8; u++) {
      const int sg = 2 * (t0 + u) + (lane >> 5), e = lane & 31;
      const u64 key = ((u64)okey32(a.metric == kMetricEuclidean ? -sc[u] : sc[u]) << 32) | (u64)(~id[u]);
      if (e < KP) st[sg * kKwayP + e] = id[u] != 0xFFFFFFFFu ? key : 0ull;
    }
  }
  wave_sync();
  const int r = lane >> 3, row = row0 + r;
  const u64 *mine = st + lane * kKwayP;
  int ptr = 0;
  u64 h = mine[0];
  bool fail = false;
  const bool writer = (lane & 7) == 0 && row < a.M;
  uint32_t *oi = a.out_idx + (int64_t)row * a.k_out;
  float *os = a.out_score + (int64_t)row * a.k_out;
  for (int j = 0; j < a.k_out; j++) {
    u64 m = h, o;
    o = dpp_u64(m, 0);
    m = o > m ? o : m;
    o = dpp_u64(m, 1);
    m = o > m ? o : m;
    o = dpp_u64(m, 2);
    m = o > m ? o : m;
    // the group's winner: its lowest lane holding the maximum (equal keys,
    // which distinct shard indices never give, would come from the lower list first)
    const u64 eq = __ballot(m != 0ull && h == m);
    const uint32_t grp = (uint32_t)(eq >> (lane & ~7)) & 0xFFu;
    if (grp != 0u && (lane & 7) == __builtin_ctz(grp)) {
      ptr++;
      if (ptr >= lim && ptr < a.k_in) fail = true;  // the next entry is past the staged prefix
      h = ptr < lim ? mine[ptr] : 0ull;
    }
    if (writer) {
      uint32_t id = 0xFFFFFFFFu;
      float sc = __uint_as_float(0x7FC00000u);
      if (m != 0ull) {
        id = ~(uint32_t)m;
        const float v = dekey32((uint32_t)(m >> 32));
        sc = (a.metric == kMetricEuclidean) ? 0.0f - v : v;
      }
      oi[j] = id;
      os[j] = sc;
    }
  }
  // rows a skewed list made fail: the general path over every entry (the
  // staging area is the scratch now; its stores land after the ones above)
  u64 fm = __ballot(fail);
  if (fm) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    wave_sync();
    MergeArgs b = a;
    b.flags &= ~kMergeReverse;  // (merge_row's rpos is the row itself)
    while (fm) {
      const int rr = __builtin_ctzll(fm) >> 3;
      fm &= ~(0xFFull << (8 * rr));
      merge_row<1, false, false>(b, row0 + rr, wid, lane, (char *)st - (size_t)wid * MPN(a.P) * 8);
      wave_sync();
    }
  }
}

size_t merge_lds_bytes_per_wave(int P) { return (size_t)MPN(P) * 8; }

// ===========================================================================
// Threshold seeding (topk_f32_device_impl): one wave per query row reads the
// row's ns exact scores of the corpus sample (materialised by the store-mode
// GEMM), forms the composite keys (okey(score) << 32 | ~column, the fused
// kernel's keys) and selects the k-th largest by ballots (wave_kth_u64);
// gthr[row] = that key - 1, an exact lower bound of the row's final k-th.
// ===========================================================================
template <int E>
__global__ __launch_bounds__(256) void seed_select_kernel(const float *__restrict__ S, int64_t lds, int m,
                                                          int ns, int k, int metric, u64 *__restrict__ gthr) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= m) return;
  const float *src = S + (int64_t)row * lds;
  u64 x[E];
#pragma unroll
  for (int e = 0; e < E; e++) {
    const int j = lane + 64 * e;
    x[e] = 0ull;
    if (j < ns) {
      const float v = src[j];
      x[e] = ((u64)okey32(metric == kMetricEuclidean ? -v : v) << 32) | (u64)(~(uint32_t)j);
    }
  }
  const u64 t = wave_kth_u64<E>(x, k);
  if (lane == 0 && t != 0ull) gthr[row] = t - 1;
}

hipError_t launch_seed_select(const float *S, int64_t lds, int m, int ns, int k, int metric,
                              unsigned long long *gthr, hipStream_t s) {
  if (m <= 0) return hipSuccess;
  // (up to 4096: the bf16 seed sample and the fire-and-forget kernel's guess)
  if (ns > 4096 || k > ns) return hipErrorInvalidValue;
  const unsigned grid = (unsigned)((m + 3) / 4);
  if (ns <= 256) seed_select_kernel<4><<<grid, 256, 0, s>>>(S, lds, m, ns, k, metric, gthr);
  else if (ns <= 512) seed_select_kernel<8><<<grid, 256, 0, s>>>(S, lds, m, ns, k, metric, gthr);
  else if (ns <= 1024) seed_select_kernel<16><<<grid, 256, 0, s>>>(S, lds, m, ns, k, metric, gthr);
  else if (ns <= 2048) seed_select_kernel<32><<<grid, 256, 0, s>>>(S, lds, m, ns, k, metric, gthr);
  else seed_select_kernel<64><<<grid, 256, 0, s>>>(S, lds, m, ns, k, metric, gthr);
  return hipGetLastError();
}

// The fused top-k's prologue in one launch (small problems, with threshold
// seeding): seed blocks first, then the query and corpus norms blocks, then
// blocks zeroing the work counters and candidate counts.
//
// A seed block takes 4 query rows (staged in LDS) and all ns sample columns,
// thread t columns t, t + 256, ...; each thread runs its 4 dot products as
// fmaf chains in natural K order over the padded dimension -- the fused
// kernel's v_mfma_f32_32x32x2_f32 chain bit for bit -- and, for the
// normalising metrics, its column's norm in ndarray's unrolled order from the
// same loaded values (norms_rows' arithmetic bit for bit); the 4 row norms
// come from norms_rows over the staged rows.  exact_score gives the scores;
// their composite keys go to LDS and wave w writes row w's threshold
// (k-th key - 1).  So the seed needs nothing from the norms blocks and shares
// their launch.  (Round 1: a store-mode pass of the fused kernel + a select
// launch, 32 + 8 us at c1, on 32 workgroups.)  Its per-lane row reads thrash
// the vector L1 (64 rows per load instruction); an LDS-staged variant with
// coalesced loads measured slower (87 us: its load and compute phases
// serialise), as did batching each lane's loads 8 deep (39 us against 28).
namespace seedk {
#ifndef PMM_SEED_RQ
#define PMM_SEED_RQ 4
#endif
// query rows per seed block (a multiple of 4: the block's 4 waves select RQ / 4
// rows each).  Every lane streams its sample column's row once per block, so
// RQ rows share each corpus load.
constexpr int RQ = PMM_SEED_RQ;
static_assert(RQ % 4 == 0 && RQ <= 16, "seed rows per block");
}  // namespace seedk
struct PrologueArgs {
  const float *q;
  int64_t ldq;
  int m;
  const float *c;
  int64_t ldc;
  int64_t n;
  int d, dp, ns, k, squared;
  float *qn, *cn, *cinv;       // norms outputs (cn / cinv unused when cblocks = 0)
  unsigned long long *gthr;    // seed outputs: every row's threshold
  uint4 *z0, *z1;              // zeroed ranges (16-byte words)
  int64_t z0n, z1n;
  unsigned sblocks, qblocks, cblocks, zblocks;
  int lds_seed;                // LDS-staged seed blocks (seed_lds_block)
  int64_t cper;                // LDS-staged launch: corpus norm rows per block
  int ablate;                  // lab build only (PMM_PROLOGUE_ABLATE): 1 no seed blocks' work,
                               // 2 seed without the k-th selection, 4 no norm / fill blocks' work
  int mfma_seed;               // seed blocks on v_mfma_f32_16x16x4_f32 (prologue_mfma_kernel)
};

// LDS-staged seed block (ns <= 256 sample columns, padded D <= 1024): the
// arithmetic of the fmaf-chain block below, bit for bit (the same chains in
// the same K order, the same norm accumulators), but the sample rows reach
// the lanes through LDS.  The fmaf-chain block streams each lane's own 1 KiB
// row: every load instruction touches 64 rows, so the vector cache's tag
// lookups, not the bytes, set its 19-21 us at c1.  Here the block's 256
// columns come in K chunks of 32 floats by LDS-DMA (one instruction: 8
// columns x 128 contiguous bytes), through a 4-chunk ring with 3 chunks in
// flight (asm DMA with counted vmcnt waits: hipcc would wait for the whole
// ring at every LDS read), and each lane reads its column's chunk as eight
// ds_read_b128 of 16-byte pieces XOR-swizzled by column (piece j of column c
// in slot j ^ ((c >> 1) & 7): 16 lanes hit 16 distinct bank groups).
// The block also writes its rows' query norms, and every block of the launch
// takes a slice of the corpus norms and of the zero fill, so the launch has
// no other block kinds (its 152 KiB of LDS admits one block per CU).
namespace seedk {
constexpr int KC = 32;               // K floats per ring chunk
constexpr int NB = 4;                // ring chunks (NB - 1 in flight)
constexpr int CHUNK = 256 * KC * 4;  // 256 columns: 32 KiB
constexpr int kLdsMaxDp = 1024;
__device__ __forceinline__ void wait_vm(int n) {
  switch (n) {
#define PMM_SEED_W(N) \
  case N: asm volatile("s_waitcnt vmcnt(" #N ")" ::: "memory"); break;
    PMM_SEED_W(0) PMM_SEED_W(8) PMM_SEED_W(16) PMM_SEED_W(24)
#undef PMM_SEED_W
    default: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
  }
}
// LDS-DMA of one 16-byte piece per lane into M0 + 16 lane (s_nop 4: M0's one
// state, and five for any descriptor / offset SGPR fresh from a VALU write --
// tests/test_asm_hazards.py)
__device__ __forceinline__ void dma_b128(__amdgpu_buffer_rsrc_t r, uint32_t lds, uint32_t voff, uint32_t soff) {
  asm volatile("s_mov_b32 m0, %0\n\ts_nop 4\n\tbuffer_load_dwordx4 %1, %2, %3 offen lds" ::"s"(lds), "v"(voff),
               "s"(r), "s"(soff)
               : "memory");
}
}  // namespace seedk

template <int METRIC>
__device__ __forceinline__ void seed_lds_block(const PrologueArgs &a, unsigned b, char *smem) {
  using namespace seedk;
  constexpr bool XFORM = METRIC != kMetricDot;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int dp = a.dp, d = a.d, ns = a.ns, m = a.m;
  u64 *keys = (u64 *)(smem + NB * CHUNK);         // [RQ][256]
  float *qs = (float *)(keys + RQ * 256);         // [RQ][dp]
  float *qn_s = qs + RQ * dp;                     // [RQ]
  const uint32_t ring_lds = (uint32_t)(size_t)(LDS_AS char *)smem;
  const int row0 = b * RQ;
  const int G = dp / KC;
  // rows past the sample read as zeros (their keys are never used)
  const __amdgpu_buffer_rsrc_t rc = make_rsrc(a.c, (int64_t)ns * a.ldc * 4);
  // DMA instruction i of wave w fills slots (i 256 + tid): column 32 i +
  // (tid >> 3), slot tid & 7, which holds K piece (tid & 7) ^ ((tid >> 4) & 7)
  uint32_t voff = (uint32_t)((tid >> 3) * a.ldc * 4 + 16 * ((tid & 7) ^ ((tid >> 4) & 7)));
  asm volatile("" : "+v"(voff));
  const uint32_t colstep = (uint32_t)(32 * a.ldc * 4);
  auto issue = [&](int g) __attribute__((always_inline)) {
    const uint32_t dst = ring_lds + (uint32_t)((g % NB) * CHUNK + w * 64 * 16);
#pragma unroll
    for (int i = 0; i < 8; i++)
      dma_b128(rc, __builtin_amdgcn_readfirstlane(dst + (uint32_t)(i * 256 * 16)), voff,
               __builtin_amdgcn_readfirstlane((uint32_t)i * colstep + (uint32_t)(g * KC * 4)));
  };
  for (int g = 0; g < NB - 1 && g < G; g++) issue(g);
  // the query rows, all loads in flight at once (dp / 4 <= 256: one piece
  // per thread and row; the compiler's vmcnt wait for them also retires the
  // ring's first chunks)
  {
    f32x4 v[RQ];
    const bool on = tid < dp / 4;
#pragma unroll
    for (int r = 0; r < RQ; r++) {
      v[r] = (f32x4){0.0f, 0.0f, 0.0f, 0.0f};
      if (on && row0 + r < m) v[r] = *(const f32x4 *)(a.q + (int64_t)(row0 + r) * a.ldq + 4 * tid);
    }
#pragma unroll
    for (int r = 0; r < RQ; r++)
      if (on) *(f32x4 *)(qs + r * dp + 4 * tid) = v[r];
  }
  __syncthreads();
  if (XFORM && w < (RQ + 7) / 8) norms_rows<float, float>(qs, RQ, d, dp, a.squared, qn_s, nullptr, tid);
  __syncthreads();
  const int col = tid, d8 = d & ~7;
  float acc[RQ];
#pragma unroll
  for (int r = 0; r < RQ; r++) acc[r] = 0.0f;
  float p[8];
#pragma unroll
  for (int j = 0; j < 8; j++) p[j] = 0.0f;
  const uint32_t rd0 = ring_lds + (uint32_t)(col * KC * 4);
  const int swz = (col >> 1) & 7;
  for (int g = 0; g < G; g++) {
    // this wave's pieces of chunk g landed (younger: chunks g + 1 .. g + NB - 2)
    wait_vm(8 * (min(G - 1, g + NB - 2) - g));
    __builtin_amdgcn_s_barrier();  // everyone's pieces landed; everyone is past chunk g - 1
    asm volatile("" ::: "memory");
    if (g + NB - 1 < G) issue(g + NB - 1);  // into chunk g - 1's slot
    const uint32_t rb = rd0 + (uint32_t)((g % NB) * CHUNK);
#pragma unroll
    for (int j = 0; j < KC / 4; j++) {
      const f32x4 cv = *(const LDS_AS f32x4 *)(size_t)(rb + (uint32_t)(16 * (j ^ swz)));
      const int j4 = g * (KC / 4) + j;
#pragma unroll
      for (int r = 0; r < RQ; r++) {
        const f32x4 q4 = *(const f32x4 *)(qs + r * dp + 4 * j4);  // broadcast
        acc[r] = fmaf(q4[0], cv[0], acc[r]);
        acc[r] = fmaf(q4[1], cv[1], acc[r]);
        acc[r] = fmaf(q4[2], cv[2], acc[r]);
        acc[r] = fmaf(q4[3], cv[3], acc[r]);
      }
      if (XFORM && 4 * j4 < d8) {
        // ndarray order: accumulator j sums x[8t + j]^2 over t
        const int o = (j & 1) * 4;
#pragma unroll
        for (int e = 0; e < 4; e++) p[o + e] = p[o + e] + cv[e] * cv[e];
      }
    }
  }
  float cnv = 0.0f;
  if (XFORM && col < ns) {
    float sum = 0.0f;
    sum = sum + (p[0] + p[4]);
    sum = sum + (p[1] + p[5]);
    sum = sum + (p[2] + p[6]);
    sum = sum + (p[3] + p[7]);
    const float *crow = a.c + (int64_t)col * a.ldc;
    for (int i = d8; i < d; i++) {
      const float x = crow[i];
      sum = sum + x * x;
    }
    cnv = a.squared ? sum : sqrt_rn<float>(sum);
  }
#pragma unroll
  for (int r = 0; r < RQ; r++) {
    u64 key = 0ull;
    if (col < ns && row0 + r < m) {
      const float sc = exact_score<METRIC>(acc[r], XFORM ? qn_s[r] : 0.0f, cnv);
      key = ((u64)okey32(METRIC == kMetricEuclidean ? -sc : sc) << 32) | (u64)(~(uint32_t)col);
    }
    keys[r * 256 + col] = key;
  }
  __syncthreads();
  if (XFORM && tid < RQ && row0 + tid < m) a.qn[row0 + tid] = qn_s[tid];
  for (int rr = w; rr < RQ; rr += 4) {
    const int row = row0 + rr;
    if (row >= m) return;
    u64 x[4];
#pragma unroll
    for (int e = 0; e < 4; e++) x[e] = keys[rr * 256 + lane + 64 * e];
    const u64 th = seed_threshold<4>(x, a.k);  // a lower bound of the row's final k-th
    if (lane == 0) a.gthr[row] = th;
  }
}

template <int E, int METRIC, int LDSK>
__global__ __launch_bounds__(256) void prologue_kernel(PrologueArgs a) {
  using namespace seedk;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  unsigned b = blockIdx.x;
  if (LDSK) {
    // every block: a slice of the zero fill (stores only, issued first), the
    // seed (blocks < sblocks: one per 4 query rows), then a slice of the
    // corpus norms (cper rows)
    {
      const int64_t tot = a.z0n + a.z1n, per = (tot + gridDim.x - 1) / gridDim.x;
      const int64_t lo = (int64_t)b * per, hi = lo + per < tot ? lo + per : tot;
      for (int64_t i = lo + tid; i < hi; i += 256) {
        if (i < a.z0n) a.z0[i] = make_uint4(0u, 0u, 0u, 0u);
        else a.z1[i - a.z0n] = make_uint4(0u, 0u, 0u, 0u);
      }
    }
    if (b < a.sblocks) seed_lds_block<METRIC>(a, b, smem);
    if (a.cblocks) {
      const int64_t lo = (int64_t)b * a.cper;
      const int64_t rows = lo + a.cper < a.n ? a.cper : a.n - lo;
      for (int64_t g0 = 0; g0 < rows * 8; g0 += 256)
        norms_rows<float, float>(a.c + lo * a.ldc, rows, a.d, a.ldc, a.squared, a.cn + lo, a.cinv + lo, g0 + tid);
    }
    return;
  }
  if (b >= a.sblocks) {
    if (PMM_ABL(a.ablate & 4)) return;  // (lab: phase removal, results wrong)
    b -= a.sblocks;
    if (b < a.qblocks) {
      norms_rows<float, float>(a.q, a.m, a.d, a.ldq, a.squared, a.qn, nullptr, (int64_t)b * 256 + tid);
      return;
    }
    b -= a.qblocks;
    if (b < a.cblocks) {
      norms_rows<float, float>(a.c, a.n, a.d, a.ldc, a.squared, a.cn, a.cinv, (int64_t)b * 256 + tid);
      return;
    }
    b -= a.cblocks;
    const int64_t stride = (int64_t)a.zblocks * 256;
    for (int64_t i = (int64_t)b * 256 + tid; i < a.z0n + a.z1n; i += stride) {
      if (i < a.z0n) a.z0[i] = make_uint4(0u, 0u, 0u, 0u);
      else a.z1[i - a.z0n] = make_uint4(0u, 0u, 0u, 0u);
    }
    return;
  }
  if (PMM_ABL(a.ablate & 1)) return;  // (lab: phase removal, results wrong)
  constexpr bool XFORM = METRIC != kMetricDot;
  const int dp = a.dp, d = a.d, ns = a.ns, m = a.m;
  u64 *keys = (u64 *)smem;                        // [RQ][64 E]
  float *qs = (float *)(smem + RQ * 64 * E * 8);  // [RQ][dp]
  float *qn_s = qs + RQ * dp;                     // [RQ]
  const int row0 = b * RQ;
  for (int r = 0; r < RQ; r++)
    for (int j4 = tid; j4 < dp / 4; j4 += 256) {
      f32x4 v = {0.0f, 0.0f, 0.0f, 0.0f};
      if (row0 + r < m) v = *(const f32x4 *)(a.q + (int64_t)(row0 + r) * a.ldq + 4 * j4);
      *(f32x4 *)(qs + r * dp + 4 * j4) = v;
    }
  __syncthreads();
  if (XFORM && w < (RQ + 7) / 8) norms_rows<float, float>(qs, RQ, d, dp, a.squared, qn_s, nullptr, tid);
  __syncthreads();
  const int d8 = d & ~7;
  for (int col = tid; col < 64 * E; col += 256) {
    float acc[RQ];
#pragma unroll
    for (int r = 0; r < RQ; r++) acc[r] = 0.0f;
    float p[8];
#pragma unroll
    for (int j = 0; j < 8; j++) p[j] = 0.0f;
    float cnv = 0.0f;
    if (col < ns) {
      const float *crow = a.c + (int64_t)col * a.ldc;
      const f32x4 *cr = (const f32x4 *)crow;
      // the row's 16-byte pieces stream through a ring of PD loads in flight
      // (one at a time, each load's latency was exposed: 64 per row at D =
      // 256); the arithmetic and its order are unchanged
      // (dp is a multiple of 32, so nj a multiple of PD; loads past the row's
      // end re-read its last piece, so every load is unconditional and the
      // compiler counts its waits)
      constexpr int PD = 8;  // (measured at c1: 16 and 2-row blocks both slower)
      const int nj = dp / 4;
      f32x4 ring[PD];
#pragma unroll
      for (int q = 0; q < PD; q++) ring[q] = cr[min(q, nj - 1)];
      for (int j0 = 0; j0 < nj; j0 += PD) {
#pragma unroll
        for (int q = 0; q < PD; q++) {
          const int j4 = j0 + q;
          {
            const f32x4 cv = ring[q];
            ring[q] = cr[min(j4 + PD, nj - 1)];
#pragma unroll
            for (int r = 0; r < RQ; r++) {
              const f32x4 q4 = *(const f32x4 *)(qs + r * dp + 4 * j4);  // broadcast
              acc[r] = fmaf(q4[0], cv[0], acc[r]);
              acc[r] = fmaf(q4[1], cv[1], acc[r]);
              acc[r] = fmaf(q4[2], cv[2], acc[r]);
              acc[r] = fmaf(q4[3], cv[3], acc[r]);
            }
            if (XFORM && 4 * j4 < d8) {
              // ndarray order: accumulator j sums x[8t + j]^2 over t
              const int o = (j4 & 1) * 4;
#pragma unroll
              for (int e = 0; e < 4; e++) p[o + e] = p[o + e] + cv[e] * cv[e];
            }
          }
        }
      }
      if (XFORM) {
        float sum = 0.0f;
        sum = sum + (p[0] + p[4]);
        sum = sum + (p[1] + p[5]);
        sum = sum + (p[2] + p[6]);
        sum = sum + (p[3] + p[7]);
        for (int i = d8; i < d; i++) {
          const float x = crow[i];
          sum = sum + x * x;
        }
        cnv = a.squared ? sum : sqrt_rn<float>(sum);
      }
    }
#pragma unroll
    for (int r = 0; r < RQ; r++) {
      u64 key = 0ull;
      if (col < ns && row0 + r < m) {
        const float sc = exact_score<METRIC>(acc[r], XFORM ? qn_s[r] : 0.0f, cnv);
        key = ((u64)okey32(METRIC == kMetricEuclidean ? -sc : sc) << 32) | (u64)(~(uint32_t)col);
      }
      keys[r * 64 * E + col] = key;
    }
  }
  __syncthreads();
  for (int rr = w; rr < RQ; rr += 4) {
    const int row = row0 + rr;
    if (row >= m) return;
    u64 x[E];
#pragma unroll
    for (int e = 0; e < E; e++) x[e] = keys[rr * 64 * E + lane + 64 * e];
    if (PMM_ABL(a.ablate & 2)) {  // (lab: no selection; the keys stay live)
      u64 t = 0ull;
#pragma unroll
      for (int e = 0; e < E; e++) t ^= x[e];
      if (lane == 0) a.gthr[row] = (t == 0x0123456789abcdefull) ? t : 0ull;
      continue;
    }
    const u64 th = seed_threshold<E>(x, a.k);  // a lower bound of the row's final k-th
    if (lane == 0) a.gthr[row] = th;
  }
}

// ===========================================================================
// The prologue with MFMA seed blocks (ns = 256 sample columns, padded D <=
// 1024).  The row-streaming seed block above spends ~13 of the c1
// prologue's ~17 us streaming each lane's own 1 KiB sample row (every load
// instruction touches 64 rows) for 4 query rows at a time.  Here a seed block
// takes 16 query rows and the whole sample on v_mfma_f32_16x16x4_f32: each
// MFMA is bitwise a k-ordered fmaf chain over its 4 k (MI355X_MICROARCH.md,
// FP32-input MFMA), and step s feeds k = 4s + (lane >> 4), so every score is
// the chain over k = 0 .. dp-1 in natural order -- the main pass's and the
// fmaf-chain seed block's value, bit for bit.  The sample streams through LDS
// in K chunks of 32 floats (8 threads per column row piece: 128-byte runs),
// double-buffered, one barrier per chunk; the query rows stay in LDS.  8
// waves, 32 sample columns each (two accumulator chains per wave: the
// 16x16x4's dependent latency is 40 cycles against a 32-cycle issue).  The
// sample columns' norms come from the same chunks in ndarray order (thread c
// owns column c's 8 partial sums), the query rows' from the staged rows.
// Other block kinds (query / corpus norms, fills) as in prologue_kernel, at
// 512 threads per block.
// ===========================================================================
namespace seedm {
constexpr int RM = 16;          // query rows per seed block (the MFMA's M)
#ifndef PMM_SEEDM_NT
#define PMM_SEEDM_NT 1024
#endif
constexpr int NT = PMM_SEEDM_NT;  // threads per block: 16 waves, one query row each for the selection
constexpr int NCH = 256 / (NT / 64) / 16;  // 16-column accumulator chains per wave
constexpr int NSM = 256;        // sample columns
constexpr int KC = 32;          // K floats per corpus chunk
constexpr int CS = KC + 4;      // LDS row stride of a chunk (floats): conflict-free B reads
constexpr int kMaxDp = 1024;
__host__ __device__ constexpr size_t lds_bytes(int dp) {
  return (size_t)RM * (dp + 4) * 4 + (size_t)2 * NSM * CS * 4 + RM * 4 + NSM * 4;
}
static_assert((size_t)RM * NSM * 8 <= (size_t)2 * NSM * CS * 4, "keys alias the chunk buffers");
}  // namespace seedm

#ifdef PMM_SEED_STAMPS
// (lab only: per-block phase clocks of the MFMA seed blocks, read back by
// pmm_lab_seed_stamps; divergent lane-0 vector stores)
__device__ unsigned long long g_seed_st[1024][8];
#define SEED_ST(i)                                                          \
  do {                                                                     \
    const unsigned long long t_ = __builtin_amdgcn_s_memtime();            \
    if (threadIdx.x == 0 && b < 1024) g_seed_st[b][i] = t_;                \
  } while (0)
#else
#define SEED_ST(i) \
  do {             \
  } while (0)
#endif
template <int METRIC>
__device__ __forceinline__ void seed_mfma_block(const PrologueArgs &a, unsigned b, char *smem) {
  using namespace seedm;
  SEED_ST(0);
  constexpr bool XFORM = METRIC != kMetricDot;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int dp = a.dp, d = a.d, m = a.m;
  const int QS = dp + 4;                 // query row stride in LDS: conflict-free A reads
  float *qs = (float *)smem;             // [RM][QS]
  float *cbuf = qs + RM * QS;            // [2][NSM][CS]
  float *qn_s = cbuf + 2 * NSM * CS;     // [RM]
  float *cn_s = qn_s + RM;               // [NSM]
  u64 *keys = (u64 *)cbuf;               // [RM][NSM], after the K loop
  const int row0 = (int)b * RM;
  const int G = dp / KC;
  // the corpus chunk's pieces of this thread: piece p = tid + NT u -> column
  // p >> 3, 16-byte part p & 7 (8 consecutive threads read one 128-byte run).
  // Chunks stream through PFC register sets: chunk t + PFC - 1's loads are
  // issued while chunk t is computed (with one set, each chunk's L2 / HBM
  // latency was exposed: the MFMA blocks took as long as the fmaf-chain ones)
  constexpr int PFC = 4;
  constexpr int NPC = NSM * 8 / NT;  // 16-byte pieces per thread per chunk
  f32x4 v[PFC][NPC];
  auto load_chunk = [&](int t, f32x4 (&r)[NPC]) __attribute__((always_inline)) {
#pragma unroll
    for (int u = 0; u < NPC; u++) {
      const int pc = tid + NT * u, col = pc >> 3, part = pc & 7;
      r[u] = *(const f32x4 *)(a.c + (int64_t)col * a.ldc + t * KC + 4 * part);
    }
  };
  auto store_chunk = [&](int buf, const f32x4 (&r)[NPC]) __attribute__((always_inline)) {
#pragma unroll
    for (int u = 0; u < NPC; u++) {
      const int pc = tid + NT * u, col = pc >> 3, part = pc & 7;
      *(f32x4 *)(cbuf + buf * NSM * CS + col * CS + 4 * part) = r[u];
    }
  };
#pragma unroll
  for (int j = 0; j < PFC; j++) load_chunk(min(j, G - 1), v[j]);  // (clamped: every load unconditional)
  for (int i = tid; i < RM * (dp / 4); i += NT) {
    const int r = i / (dp / 4), j4 = i - r * (dp / 4);
    f32x4 x = {0.0f, 0.0f, 0.0f, 0.0f};
    if (row0 + r < m) x = *(const f32x4 *)(a.q + (int64_t)(row0 + r) * a.ldq + 4 * j4);
    *(f32x4 *)(qs + r * QS + 4 * j4) = x;
  }
  store_chunk(0, v[0]);
  __syncthreads();
  SEED_ST(1);
  const int g4 = lane >> 4, l16 = lane & 15;
  const int col0 = 16 * NCH * w + l16;  // chain c: column col0 + 16 c
  const int d8 = d & ~7;
  f32x4 acc[NCH];
#pragma unroll
  for (int c = 0; c < NCH; c++) acc[c] = (f32x4){0.0f, 0.0f, 0.0f, 0.0f};
  float p[8];
#pragma unroll
  for (int j = 0; j < 8; j++) p[j] = 0.0f;
  // (every load and LDS store unconditional, past the last chunk on clamped
  // or unused data: the compiler then counts the loads in flight instead of
  // waiting for all of them at each branch)
  for (int t0 = 0; t0 < (PMM_ABL(a.ablate & 8) ? 0 : G); t0 += PFC) {  // (lab 8: no K loop)
#pragma unroll
    for (int j = 0; j < PFC; j++) {
      const int t = t0 + j;
      if (t < G) {
      const float *cb = cbuf + (t & 1) * NSM * CS;
      const float *qa = qs + l16 * QS + t * KC + g4;
#pragma unroll
      for (int s4 = 0; s4 < KC / 4; s4++) {
        const float av = qa[4 * s4];
#pragma unroll
        for (int c = 0; c < NCH; c++)
          acc[c] = __builtin_amdgcn_mfma_f32_16x16x4f32(av, cb[(col0 + 16 * c) * CS + 4 * s4 + g4], acc[c], 0, 0, 0);
      }
      if (XFORM && tid < NSM) {
        // column tid's norm partials in ndarray order: accumulator j sums
        // x[8t + j]^2 over t (the chunk's float4 j4 holds k = 4 j4 .. 4 j4 + 3)
        const float *cc = cb + tid * CS;
#pragma unroll
        for (int j4 = 0; j4 < KC / 4; j4++) {
          if (t * KC + 4 * j4 < d8) {
            const f32x4 x = *(const f32x4 *)(cc + 4 * j4);
            const int o = (j4 & 1) * 4;
#pragma unroll
            for (int e = 0; e < 4; e++) p[o + e] = p[o + e] + x[e] * x[e];
          }
        }
      }
      }
      // chunk t + 1 into the other buffer (its last readers, chunk t - 1,
      // passed the previous barrier); chunk t + PFC into chunk t's registers
      store_chunk((t + 1) & 1, v[(j + 1) % PFC]);
      load_chunk(min(t + PFC, G - 1), v[j]);
      __syncthreads();
    }
  }
  SEED_ST(2);
  if (XFORM && tid < NSM) {
    float sum = 0.0f;
    sum = sum + (p[0] + p[4]);
    sum = sum + (p[1] + p[5]);
    sum = sum + (p[2] + p[6]);
    sum = sum + (p[3] + p[7]);
    const float *crow = a.c + (int64_t)tid * a.ldc;
    for (int i = d8; i < d; i++) {
      const float x = crow[i];
      sum = sum + x * x;
    }
    cn_s[tid] = a.squared ? sum : sqrt_rn<float>(sum);
  }
  if (XFORM && w < RM / 8) norms_rows<float, float>(qs, RM, d, QS, a.squared, qn_s, nullptr, tid);
  __syncthreads();
  SEED_ST(3);
  // D of the 16x16x4: lane holds rows 4 (lane >> 4) + i of its column
#pragma unroll
  for (int i = 0; i < 4; i++) {
    const int r = 4 * g4 + i;
    const bool ok = row0 + r < m;
    const float qv = XFORM ? qn_s[r] : 0.0f;
#pragma unroll
    for (int c = 0; c < NCH; c++) {
      const int col = col0 + 16 * c;
      const float sc = exact_score<METRIC>(acc[c][i], qv, XFORM ? cn_s[col] : 0.0f);
      keys[r * NSM + col] =
          ok ? (((u64)okey32(METRIC == kMetricEuclidean ? -sc : sc) << 32) | (u64)(~(uint32_t)col)) : 0ull;
    }
  }
  __syncthreads();
  SEED_ST(4);
  for (int rr = w; rr < RM; rr += NT / 64) {
    const int row = row0 + rr;
    if (row >= m) return;
    u64 x[4];
#pragma unroll
    for (int e = 0; e < 4; e++) x[e] = keys[rr * NSM + lane + 64 * e];
    if (PMM_ABL(a.ablate & 16)) {  // (lab: no selection; the keys stay live)
      u64 t = 0ull;
#pragma unroll
      for (int e = 0; e < 4; e++) t ^= x[e];
      if (lane == 0) a.gthr[row] = (t == 0x0123456789abcdefull) ? t : 0ull;
      continue;
    }
    const u64 th = seed_threshold<4>(x, a.k);  // a lower bound of the row's final k-th
    if (lane == 0) a.gthr[row] = th;
  }
  SEED_ST(5);
}

template <int METRIC>
__global__ __launch_bounds__(seedm::NT) void prologue_mfma_kernel(PrologueArgs a) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x;
  unsigned b = blockIdx.x;
  if (b < a.sblocks) {
    if (PMM_ABL(a.ablate & 1)) return;  // (lab: phase removal, results wrong)
    seed_mfma_block<METRIC>(a, b, smem);
    return;
  }
  if (PMM_ABL(a.ablate & 4)) return;
  b -= a.sblocks;
  if (b < a.qblocks) {
    norms_rows<float, float>(a.q, a.m, a.d, a.ldq, a.squared, a.qn, nullptr, (int64_t)b * seedm::NT + tid);
    return;
  }
  b -= a.qblocks;
  if (b < a.cblocks) {
    norms_rows<float, float>(a.c, a.n, a.d, a.ldc, a.squared, a.cn, a.cinv, (int64_t)b * seedm::NT + tid);
    return;
  }
  b -= a.cblocks;
  const int64_t stride = (int64_t)a.zblocks * seedm::NT;
  for (int64_t i = (int64_t)b * seedm::NT + tid; i < a.z0n + a.z1n; i += stride) {
    if (i < a.z0n) a.z0[i] = make_uint4(0u, 0u, 0u, 0u);
    else a.z1[i - a.z0n] = make_uint4(0u, 0u, 0u, 0u);
  }
}

#ifdef PMM_SEED_STAMPS
extern "C" int pmm_lab_seed_stamps(unsigned long long *out, int n) {
  return (int)hipMemcpyFromSymbol(out, HIP_SYMBOL(g_seed_st), (size_t)n * 8 * sizeof(unsigned long long));
}
#endif
template <int METRIC>
static hipError_t launch_prologue_mfma_t(const PrologueArgs &a, unsigned grid, hipStream_t s) {
  static bool attr = false;
  if (!attr) {
    hipError_t e = hipFuncSetAttribute((const void *)prologue_mfma_kernel<METRIC>,
                                       hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    if (e != hipSuccess) return e;
    attr = true;
  }
  prologue_mfma_kernel<METRIC><<<grid, seedm::NT, seedm::lds_bytes(a.dp), s>>>(a);
  return hipGetLastError();
}

template <int METRIC, int LDSK>
static hipError_t launch_prologue_t2(const PrologueArgs &a, unsigned grid, hipStream_t s) {
  using namespace seedk;
  const size_t lds_base = (size_t)RQ * a.dp * 4 + RQ * 4;
  static bool attr = false;
  if (!attr) {
    hipError_t e = hipFuncSetAttribute((const void *)prologue_kernel<4, METRIC, LDSK>,
                                       hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    if (e == hipSuccess && !LDSK)
      e = hipFuncSetAttribute((const void *)prologue_kernel<8, METRIC, LDSK>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    if (e == hipSuccess && !LDSK)
      e = hipFuncSetAttribute((const void *)prologue_kernel<16, METRIC, LDSK>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    if (e != hipSuccess) return e;
    attr = true;
  }
  if (LDSK) {  // (ns <= 256, dp <= kLdsMaxDp: checked by the caller)
    prologue_kernel<4, METRIC, LDSK><<<grid, 256, (size_t)NB * CHUNK + RQ * 256 * 8 + lds_base, s>>>(a);
    return hipGetLastError();
  }
  auto lds = [&](int nsp) { return lds_base + RQ * nsp * 8; };
  if (a.ns <= 256) prologue_kernel<4, METRIC, LDSK><<<grid, 256, lds(256), s>>>(a);
  else if (a.ns <= 512) prologue_kernel<8, METRIC, LDSK><<<grid, 256, lds(512), s>>>(a);
  else prologue_kernel<16, METRIC, LDSK><<<grid, 256, lds(1024), s>>>(a);
  return hipGetLastError();
}
template <int METRIC>
static hipError_t launch_prologue_t(const PrologueArgs &a, unsigned grid, hipStream_t s) {
  return a.lds_seed ? launch_prologue_t2<METRIC, 1>(a, grid, s) : launch_prologue_t2<METRIC, 0>(a, grid, s);
}

#ifndef PMM_SEED_MFMA_DEFAULT
// MFMA seed blocks by default: c1 step 0.099 vs 0.100 ms, prologue 18 vs
// 19-20 us (bench events), c2 0.096 vs 0.097 (profiles/r5_c1/seed_ab.txt)
#define PMM_SEED_MFMA_DEFAULT 1
#endif
hipError_t launch_seeded_prologue(const float *q, int64_t ldq, int m, const float *c, int64_t ldc, int64_t n,
                                  int d, int dp, int ns, int k, int metric, float *qn, float *cn, bool corpus_norms,
                                  unsigned long long *gthr, void *z0, size_t z0_bytes, void *z1, size_t z1_bytes,
                                  hipStream_t s) {
  if (m <= 0) return hipSuccess;
  // the kernel's shapes: whole float4 groups of padded rows, a sample its LDS
  // holds, 16-byte aligned rows and zeroed ranges
  if (ns > kSeedMaxNs || k > ns || ns > n || dp % 32 != 0 || dp > kSeedDotsMaxD || d > dp || ldq % 4 != 0 ||
      ldc % 4 != 0 || (((uintptr_t)q | (uintptr_t)c | (uintptr_t)z0 | (uintptr_t)z1) & 15) || z0_bytes % 16 ||
      z1_bytes % 16)
    return hipErrorInvalidValue;
  PrologueArgs a{};
  a.q = q;
  a.ldq = ldq;
  a.m = m;
  a.c = c;
  a.ldc = ldc;
  a.n = n;
  a.d = d;
  a.dp = dp;
  a.ns = ns;
  a.k = k;
  a.squared = metric == kMetricEuclidean;
  a.qn = qn;
  a.cn = cn;
  a.cinv = cn + n;
  a.gthr = gthr;
  a.z0 = (uint4 *)z0;
  a.z1 = (uint4 *)z1;
  a.z0n = (int64_t)(z0_bytes / 16);
  a.z1n = (int64_t)(z1_bytes / 16);
  // The fmaf-chain blocks that stream their own rows by default; PMM_SEED_LDS=1
  // (read per call) takes the LDS-staged seed blocks (seed_lds_block) where
  // they apply.  A/B on one box, two alternations (profiles/r4_seed/): c1 step
  // 0.104 ms with the LDS-staged blocks against 0.099 ms (prologue 24 vs
  // 20 us), c2 0.096 vs 0.095 ms; bit-identical either way.
#ifdef PMM_LAB
  a.ablate = getenv("PMM_PROLOGUE_ABLATE") ? atoi(getenv("PMM_PROLOGUE_ABLATE")) : 0;
#endif
  const char *le = getenv("PMM_SEED_LDS");
  a.lds_seed = (ns <= 256 && dp <= seedk::kLdsMaxDp && le && atoi(le) == 1) ? 1 : 0;
  const bool xf = metric != kMetricDot;
  // MFMA seed blocks (prologue_mfma_kernel) for a 256-column sample; PMM_SEED_MFMA
  // (read per call) 0 / 1 forces the fmaf-chain blocks / the MFMA blocks
  const char *me = getenv("PMM_SEED_MFMA");
  const bool mfma_ok = ns == seedm::NSM && dp <= seedm::kMaxDp && !a.lds_seed && n >= seedm::NSM;
  a.mfma_seed = (mfma_ok && (me ? atoi(me) != 0 : PMM_SEED_MFMA_DEFAULT != 0)) ? 1 : 0;
  if (a.mfma_seed) {
    a.sblocks = (unsigned)((m + seedm::RM - 1) / seedm::RM);
    constexpr int T = seedm::NT;
    a.qblocks = xf ? (unsigned)((m * 8 + T - 1) / T) : 0u;
    a.cblocks = (xf && corpus_norms) ? (unsigned)((n * 8 + T - 1) / T) : 0u;
    a.zblocks = (unsigned)std::max<int64_t>(1, std::min<int64_t>((a.z0n + a.z1n + T - 1) / T, 16));
    const unsigned grid = a.sblocks + a.qblocks + a.cblocks + a.zblocks;
    if (metric == kMetricCosine) return launch_prologue_mfma_t<kMetricCosine>(a, grid, s);
    if (metric == kMetricDot) return launch_prologue_mfma_t<kMetricDot>(a, grid, s);
    return launch_prologue_mfma_t<kMetricEuclidean>(a, grid, s);
  }
  a.sblocks = (unsigned)((m + seedk::RQ - 1) / seedk::RQ);
  unsigned grid;
  if (a.lds_seed) {
    // one block kind: seed blocks, plus norms-only blocks so that no block
    // takes more than 64 corpus norm rows
    a.qblocks = 0u;
    grid = std::max<unsigned>(a.sblocks, (xf && corpus_norms) ? (unsigned)((n + 63) / 64) : 1u);
    a.cper = (n + grid - 1) / grid;
    a.cblocks = (xf && corpus_norms) ? 1u : 0u;  // (a flag here)
    a.zblocks = 0u;
  } else {
    a.qblocks = xf ? (unsigned)((m * 8 + 255) / 256) : 0u;
    a.cblocks = (xf && corpus_norms) ? (unsigned)((n * 8 + 255) / 256) : 0u;
    a.zblocks = (unsigned)std::max<int64_t>(1, std::min<int64_t>((a.z0n + a.z1n + 255) / 256, 64));
    grid = a.sblocks + a.qblocks + a.cblocks + a.zblocks;
  }
  if (metric == kMetricCosine) return launch_prologue_t<kMetricCosine>(a, grid, s);
  if (metric == kMetricDot) return launch_prologue_t<kMetricDot>(a, grid, s);
  return launch_prologue_t<kMetricEuclidean>(a, grid, s);
}

constexpr int kMergeRankMaxRows = 16384;
hipError_t launch_merge(const MergeArgs &a0, int loader, hipStream_t s) {
  if (a0.M <= 0) return hipSuccess;
  MergeArgs a = a0;
  // Final order by rank counting when few rows run (their waves wait on the
  // sort's dependent LDS round trips: c1, 1000 rows, 18 vs 21 us), by the
  // bitonic sort otherwise (rank counting's ~8 vector instructions per kept
  // key and lane cost more issue than the sort when every SIMD holds several
  // rows: c3, 100k rows, 0.423 vs 0.403 ms; tools/experiments/merge_rank_ab.sh).
  // PMM_MERGE_RANK: 0 never, 1 always, unset by row count.  Same output.
  static const int rank_env = getenv("PMM_MERGE_RANK") ? atoi(getenv("PMM_MERGE_RANK")) : -1;
  a.no_rank = rank_env == 0 || (rank_env < 0 && a.M > kMergeRankMaxRows);
  // Rows last to first and the next candidate batch in flight while one is
  // taken: c3 0.439 ms against 0.523 (reverse alone 0.506, pipelined alone
  // 0.450; alternated on one box, profiles/r3_merge/flags_ab.txt).  Same
  // output.  PMM_MERGE_FLAGS (read per call) overrides, for A/Bs.
  a.flags = getenv("PMM_MERGE_FLAGS") ? atoi(getenv("PMM_MERGE_FLAGS"))
                                     : (kMergeReverse | kMergePipelined | kMergeSplitRow);
  // four waves per row where rows are few and each has many lists to merge
  // (c1: 1000 rows x 27 lists, one wave per SIMD otherwise) and the per-wave
  // lists fit one slot per lane (k <= 64)
  // sorted input lists (loader 1, MergeArgs::sorted): the prefix fast path
  // when the prefixes can hold the answer (c = 256 / S >= 1 entries per list
  // and k_out <= 256); one wave per row
  const bool sorted = loader == 1 && a.sorted && a.S <= 64 && a.k_out <= 256 && a.P <= 512 &&
                      !(getenv("PMM_MERGE_SORTED") && atoi(getenv("PMM_MERGE_SORTED")) == 0);
  // 5..8 sorted lists (the 8-GPU root merge): the k-way kernel, 8 rows per
  // wave (PMM_MERGE_KWAY=0: the prefix fast path instead)
  // Staged prefix 24 entries per list, 4 waves per block (12 waves per CU by
  // LDS): at configs[4]'s root merge (8 x 1M x 100, alternated on one box,
  // profiles/r6_merge/kway_ab.txt) 1.725 ms against 1.793 (24, 2 waves),
  // 1.933-1.939 (32 entries) and 2.070 for the prefix fast path alone.  A
  // list past 24 of a row's answer sends that row to the general path.
  // (PMM_KWAY_P = 32 / PMM_KWAY_WPB = 2: the A/B alternatives.)
  static const int kp = getenv("PMM_KWAY_P") ? atoi(getenv("PMM_KWAY_P")) : 24;
  if (sorted && a.S >= 5 && a.S <= 8 && a.k_out <= 8 * (kp == 32 ? 32 : 24) &&
      !(getenv("PMM_MERGE_KWAY") && atoi(getenv("PMM_MERGE_KWAY")) == 0) &&
      (size_t)MPN(a.P) * 8 <= (size_t)64 * (kp == 32 ? 32 : 24) * 8) {
    static const int wpb = getenv("PMM_KWAY_WPB") ? atoi(getenv("PMM_KWAY_WPB")) : 4;
    const int rows_per_block = 8 * wpb;
    const unsigned grid = (unsigned)((a.M + rows_per_block - 1) / rows_per_block);
    if (kp != 32) {
      if (wpb == 4) (void)hipFuncSetAttribute((const void *)kway_merge_kernel<24>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
      kway_merge_kernel<24><<<grid, 64 * wpb, (size_t)wpb * 64 * 24 * 8, s>>>(a);
    } else {
      if (wpb == 4) (void)hipFuncSetAttribute((const void *)kway_merge_kernel<32>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
      kway_merge_kernel<32><<<grid, 64 * wpb, (size_t)wpb * 64 * 32 * 8, s>>>(a);
    }
    return hipGetLastError();
  }
  if (!(a.S >= 8 && a.k_out <= 64 && a.P <= 512 && !a.no_rank && a.ablate == 0) || sorted) a.flags &= ~kMergeSplitRow;
  const bool split = (a.flags & kMergeSplitRow) != 0;
  int wpb = (int)(65536 / merge_lds_bytes_per_wave(a.P));
  wpb = split ? 4 : (wpb < 1 ? 1 : (wpb > 4 ? 4 : wpb));
  const size_t lds = (size_t)wpb * merge_lds_bytes_per_wave(a.P) + (split ? 16 : 0);
  const unsigned grid = split ? (unsigned)a.M : (unsigned)((a.M + wpb - 1) / wpb);
  if (lds > 65536) {  // (P = 8192 with the padding: 66 KiB; never in split mode)
    static bool attr_set[2] = {false, false};
    if (!attr_set[loader]) {
      const void *fn = loader == 0 ? (const void *)merge_kernel<0, false> : (const void *)merge_kernel<1, false>;
      hipError_t e = hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
      if (e != hipSuccess) return e;
      attr_set[loader] = true;
    }
  }
  if (sorted) {
    merge_kernel<1, false, true><<<grid, wpb * 64, lds, s>>>(a);
  } else if (split) {
    if (loader == 0) merge_kernel<0, true><<<grid, wpb * 64, lds, s>>>(a);
    else merge_kernel<1, true><<<grid, wpb * 64, lds, s>>>(a);
  } else {
    if (loader == 0) merge_kernel<0, false><<<grid, wpb * 64, lds, s>>>(a);
    else merge_kernel<1, false><<<grid, wpb * 64, lds, s>>>(a);
  }
  return hipGetLastError();
}

// (the f64 GEMM, store mode and fused top-k: pmm_f64.hip)

// ===========================================================================
// Row-select over materialised (metric-transformed) scores: one wave per row
// streams N scores, keeps entries better than the running k-th in LDS,
// compacts when full.  src/topk.rs:6-75 semantics with the total order above.
// ===========================================================================
template <typename T>
__device__ __forceinline__ u64 score_key(T v, int metric);
template <>
__device__ __forceinline__ u64 score_key<float>(float v, int metric) {
  return (u64)okey32(metric == kMetricEuclidean ? -v : v);
}
template <>
__device__ __forceinline__ u64 score_key<double>(double v, int metric) {
  return okey64(metric == kMetricEuclidean ? -v : v);
}
template <typename T>
__device__ __forceinline__ T key_score(u64 k, int metric);
template <>
__device__ __forceinline__ float key_score<float>(u64 k, int metric) {
  const float v = dekey32((uint32_t)k);
  return metric == kMetricEuclidean ? 0.0f - v : v;  // +0.0 for a zero distance
}
template <>
__device__ __forceinline__ double key_score<double>(u64 k, int metric) {
  const double v = dekey64(k);
  return metric == kMetricEuclidean ? 0.0 - v : v;
}

__device__ int ent_compact(Ent *scr, int cnt, int k, int P, Ent *Tv, bool *tfull, int lane) {
  for (int i = cnt + lane; i < P; i += 64) scr[i] = Ent{0ull, 0xFFFFFFFFu, 0u};
  wave_sync();
  wave_sort_desc_ent(scr, P, lane);
  if (cnt >= k) {
    *Tv = scr[k - 1];
    *tfull = true;
    cnt = k;
  }
  wave_sync();
  return cnt;
}

template <typename T>
__global__ __launch_bounds__(256) void rowselect_kernel(RowSelArgs a) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int wpb = blockDim.x >> 6;
  const int row = blockIdx.x * wpb + wid;
  if (row >= a.rows) return;
  Ent *scr = (Ent *)smem + (size_t)wid * a.P;
  const T *src = (const T *)a.scores + (int64_t)row * a.lds;
  Ent Tv{0ull, 0xFFFFFFFFu, 0u};
  bool tfull = false;
  int cnt = 0;
  for (int i0 = 0; i0 < a.N; i0 += 64) {
    const int j = i0 + lane;
    Ent x{0ull, 0xFFFFFFFFu, 0u};
    bool keep = false;
    if (j < a.N) {
      x.key = score_key<T>(src[j], a.metric);
      x.idx = (uint32_t)j;
      keep = !tfull || ent_better(x, Tv);
    }
    const u64 m = __ballot(keep);
    const int pos = cnt + lanes_below(m);
    if (keep) scr[pos] = x;
    cnt += __popcll(m);
    if (cnt > a.P - 64) {
      wave_sync();
      cnt = ent_compact(scr, cnt, a.k, a.P, &Tv, &tfull, lane);
    }
  }
  wave_sync();
  const int P2 = min(a.P, next_pow2_dev(cnt));
  for (int i = cnt + lane; i < P2; i += 64) scr[i] = Ent{0ull, 0xFFFFFFFFu, 0u};
  wave_sync();
  wave_sort_desc_ent(scr, P2, lane);
  T *os = (T *)a.out_score;
  for (int j = lane; j < a.k; j += 64) {
    const Ent x = scr[j];
    a.out_idx[(int64_t)row * a.k + j] = x.idx + a.index_base;
    os[(int64_t)row * a.k + j] = key_score<T>(x.key, a.metric);
  }
}

hipError_t launch_rowselect(const RowSelArgs &a, hipStream_t s) {
  if (a.rows <= 0) return hipSuccess;
  const size_t per_wave = (size_t)a.P * sizeof(Ent);
  int wpb = (int)(65536 / per_wave);
  wpb = wpb < 1 ? 1 : (wpb > 4 ? 4 : wpb);
  const size_t lds = (size_t)wpb * per_wave;
  const unsigned grid = (unsigned)((a.rows + wpb - 1) / wpb);
  if (a.is_f64) rowselect_kernel<double><<<grid, wpb * 64, lds, s>>>(a);
  else rowselect_kernel<float><<<grid, wpb * 64, lds, s>>>(a);
  return hipGetLastError();
}

// ===========================================================================
// Full-row global bitonic sort (k too large for the LDS row-select):
// build entries, log^2 stage launches, extract the best k.
// ===========================================================================
template <typename T>
__global__ void rowsort_build(const T *__restrict__ scores, int64_t lds, int rows, int N, int P2,
                              int metric, Ent *__restrict__ keys) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= (int64_t)rows * P2) return;
  const int r = (int)(t / P2), j = (int)(t % P2);
  Ent e{0ull, 0xFFFFFFFFu, 0u};
  if (j < N) {
    e.key = score_key<T>(scores[(int64_t)r * lds + j], metric);
    e.idx = (uint32_t)j;
  }
  keys[t] = e;
}
__global__ void rowsort_step(Ent *keys, int rows, int P2, int size, int stride) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t half = (int64_t)P2 >> 1;
  if (t >= (int64_t)rows * half) return;
  const int r = (int)(t / half), i = (int)(t % half);
  const int x0 = ((i & ~(stride - 1)) << 1) | (i & (stride - 1));
  const int x1 = x0 + stride;
  Ent *base = keys + (int64_t)r * P2;
  const Ent a = base[x0], b = base[x1];
  const bool desc = (x0 & size) == 0;
  if (desc ? ent_better(b, a) : ent_better(a, b)) {
    base[x0] = b;
    base[x1] = a;
  }
}
template <typename T>
__global__ void rowsort_extract(const Ent *__restrict__ keys, int rows, int P2, int k, int metric,
                                uint32_t index_base, uint32_t *__restrict__ out_idx,
                                T *__restrict__ out_score) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= (int64_t)rows * k) return;
  const int r = (int)(t / k), j = (int)(t % k);
  const Ent e = keys[(int64_t)r * P2 + j];
  out_idx[t] = e.idx + index_base;
  out_score[t] = key_score<T>(e.key, metric);
}

hipError_t launch_rowsort_global(const void *scores, int64_t lds, int rows, int N, int is_f64,
                                 int metric, void *keys_ws, int P2, int k, uint32_t index_base,
                                 uint32_t *out_idx, void *out_score, hipStream_t s) {
  if (rows <= 0) return hipSuccess;
  Ent *keys = (Ent *)keys_ws;
  const int64_t tot = (int64_t)rows * P2;
  const unsigned gb = (unsigned)((tot + 255) / 256);
  if (is_f64) rowsort_build<double><<<gb, 256, 0, s>>>((const double *)scores, lds, rows, N, P2, metric, keys);
  else rowsort_build<float><<<gb, 256, 0, s>>>((const float *)scores, lds, rows, N, P2, metric, keys);
  const unsigned gs = (unsigned)((tot / 2 + 255) / 256);
  for (int size = 2; size <= P2; size <<= 1)
    for (int stride = size >> 1; stride > 0; stride >>= 1)
      rowsort_step<<<gs, 256, 0, s>>>(keys, rows, P2, size, stride);
  const int64_t tk = (int64_t)rows * k;
  const unsigned ge = (unsigned)((tk + 255) / 256);
  if (is_f64) rowsort_extract<double><<<ge, 256, 0, s>>>(keys, rows, P2, k, metric, index_base, out_idx, (double *)out_score);
  else rowsort_extract<float><<<ge, 256, 0, s>>>(keys, rows, P2, k, metric, index_base, out_idx, (float *)out_score);
  return hipGetLastError();
}

}  // namespace pmm
