// pmm_bf16_wide_kernel.h -- bf16 fused GEMM + top-k holding 256 query rows per
// CU (PMM_COMPUTE_BF16; BASELINE configs[3]: 100k x 1M x 768 bf16 cosine
// k=100).  Instantiated per padded-D step count by pmm_bf16_wide_ks.hip; host
// side in pmm_bf16_wide.hip.  Same arithmetic and results as the other bf16
// kernels (bf16 operands, f32 accumulation on v_mfma_f32_32x32x16_bf16, the f32
// path's metric epilogue, pre-filter, candidate buffers and merge).
//
// Why: the wave-specialised kernel (pmm_bf16_ws_kernel.h) holds 128 query rows
// per CU, so every corpus byte streamed from L2 into LDS feeds 128 rows.  Its
// loop without the epilogue ran at ~1250 TFLOP/s, capped by that stream
// (~9.7 TB/s into LDS chip-wide).  Here 8 waves (2 per SIMD) each hold 32
// query rows x D in registers -- 256 rows per CU, half the corpus bytes per flop --
// and every wave computes AND runs its own top-k epilogue; no role split, the
// partner wave on the SIMD keeps the matrix pipe busy while one filters.
//
//   * Operands swapped relative to the other kernels: the corpus fragment is
//     the MFMA's A operand (32 corpus columns x 16 K, from LDS) and the query
//     fragment its B operand (32 query rows x 16 K, registers).  Lane l's 16
//     accumulators are then ONE query row (l & 31) against 16 corpus columns
//     (acc_row(e, l >> 5)): one pre-filter bound per lane instead of 16.
//   * Tile = 32 corpus columns x 256 query rows; K-step = 128 bf16 (8 KiB of
//     corpus per step, one 1 KiB LDS-DMA piece per wave), AHEAD steps in
//     flight, XOR-swizzled slots (conflict-free ds_read_b128 fragments).
//   * Waves 4..7 (the second wave of each SIMD: a workgroup's waves go to the
//     SIMDs cyclically) run LAG = KS / 2 K-steps behind waves 0..3, so the
//     two waves of a SIMD reach their tile epilogues at different barriers and
//     one of them always has MFMAs to issue.  The ring keeps LAG extra slots.
//   * The pre-filter factors and column norms of a tile ride into an LDS ring
//     with the tile's K-steps (one 32-byte DMA per wave per step, the same
//     bytes each step of a tile: every wave issues the same DMAs every step,
//     so every vmcnt wait is one compile-time count).
//   * Epilogue: a tile's accumulators go to LDS after its last K-step; its
//     four score groups are pre-filtered during the next tile's first K-steps
//     (while those MFMAs run), survivors re-scored exactly in-lane (the lane's
//     own row) and appended; candidate buffers are compacted at tile
//     boundaries, where no accumulators are live.
//
// Synchronisation: one s_barrier per K-step, every wave the same number per
// unit (lagging waves idle LAG barriers at a unit's start, leading waves LAG
// at its end), plus one at the unit's end.  Barrier j: every wave has waited
// (counted vmcnt) for its own pieces of stream step j and retired its LDS
// reads of its previous step, so after it stream step j + AHEAD may be DMA'd
// into the slot of step j + AHEAD - NST = j - LAG - 1.
//
// Measured (c4, 100k x 1M x 768 cosine k=100): 374 ms per launch against the
// wave-specialised kernel's 148 ms, so it is opt-in (PMM_BF16_WIDE=1).  With
// 192 of a wave's 256 registers holding query rows, each wave has one MFMA per
// substep and registers for one fragment of prefetch: the loop alone (no
// epilogue, no corpus DMA) ran at 121 ms, against 81 ms for the
// wave-specialised kernel's MFMA waves, and the epilogue's LDS round trips
// stall every wave at the per-step barrier.  DESIGN.md 3c.
//
// Hot-path LDS accesses are inline asm with explicit lgkmcnt waits: hipcc
// cannot tell the DMA ring from the rest of LDS and would otherwise wait for
// every in-flight DMA (vmcnt(0)) before them.
#pragma once
#include "pmm_bf16_ws_kernel.h"

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>
#include <utility>

namespace pmm {

namespace wd {
using ws::bf16x8;
constexpr int NW = 8;                    // waves, 2 per SIMD
constexpr int NTH = NW * 64;
constexpr int BM = 32 * NW;              // query rows per workgroup
constexpr int BN = kBf16WideBN;          // corpus columns per tile
constexpr int KB = 256;                  // bytes of a row per K-step (128 bf16)
constexpr int KSUB = KB / 32;            // MFMA substeps (K = 16) per K-step
constexpr int PF = 1;                    // corpus fragments read PF substeps ahead
constexpr int STAGE = BN * KB;           // one K-step of one tile
static_assert(STAGE == NW * 1024, "one 1 KiB corpus piece per wave per K-step");
constexpr int AHEAD = kBf16WideAhead;    // K-steps in flight beyond the one in use
constexpr int CAPE = kBf16WideMaxCapg / 64;  // candidate-buffer keys per lane in a compaction
constexpr int CVT = 32;                  // tiles in the factor / norm ring
constexpr int CVS = BN * 2;              // floats per tile: [wave][4 factors | 4 norms]
constexpr int ACCB = 16 * 64 * 4;        // a wave's staged accumulators
// LDS carve
constexpr int OFF_THR = 0;
constexpr int OFF_CNT = OFF_THR + BM * 8;
constexpr int OFF_QEX = OFF_CNT + BM * 4;
constexpr int OFF_LO = OFF_QEX + BM * 4;
constexpr int OFF_UNIT = OFF_LO + BM * 4;
constexpr int OFF_CV = (OFF_UNIT + 16 + 255) & ~255;
constexpr int OFF_ACC = OFF_CV + CVT * CVS * 4;
constexpr int OFF_QST = OFF_ACC + NW * ACCB;
// At D = 768 the last QST query fragments of a wave live in LDS instead of
// registers (the 48 fragments + accumulators + the epilogue exceed the 256
// registers of two waves per SIMD by a few): [wave][fragment][lane] x 16 B
constexpr int QST_MAX = 4;
constexpr int OFF_RING = OFF_QST + NW * QST_MAX * 1024;
template <int KS>
struct Carve {
  static constexpr int NQ = KSUB * KS;                   // query fragments per wave
  static constexpr int QST = NQ > 44 ? NQ - 44 : 0;     // of them stashed in LDS
  static constexpr int LAG = KS / 2;               // K-steps waves 4..7 trail 0..3
  static constexpr int NST = AHEAD + LAG + 1;      // ring slots
  static constexpr int BYTES = OFF_RING + NST * STAGE;
  static_assert(OFF_RING % 256 == 0 && QST <= QST_MAX, "LDS carve alignment");
  // the factor ring holds every tile from the oldest undrained survivor to
  // the newest staged one
  static_assert(3 + (KS - 1 + LAG + AHEAD) / KS <= CVT, "factor ring too short");
};

__device__ __forceinline__ void frag_read(bf16x8 &f, uint32_t addr) {
  asm volatile("ds_read_b128 %0, %1" : "=v"(f) : "v"(addr) : "memory");
}
template <int N>
__device__ __forceinline__ void wait_lgkm() {
  asm volatile("s_waitcnt lgkmcnt(%0)" ::"n"(N) : "memory");
}
__device__ __forceinline__ float lds_f32(uint32_t addr) {
  float v;
  asm volatile("ds_read_b32 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=v"(v) : "v"(addr) : "memory");
  return v;
}
__device__ __forceinline__ uint32_t lds_u32(uint32_t addr) {
  uint32_t v;
  asm volatile("ds_read_b32 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=v"(v) : "v"(addr) : "memory");
  return v;
}
__device__ __forceinline__ u64 lds_u64(uint32_t addr) {
  u64 v;
  asm volatile("ds_read_b64 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=v"(v) : "v"(addr) : "memory");
  return v;
}
__device__ __forceinline__ void lds_st32(uint32_t addr, uint32_t v) {
  asm volatile("ds_write_b32 %0, %1" ::"v"(addr), "v"(v) : "memory");
}
__device__ __forceinline__ void lds_st64(uint32_t addr, u64 v) {
  asm volatile("ds_write_b64 %0, %1" ::"v"(addr), "v"(v) : "memory");
}
__device__ __forceinline__ uint32_t lds_addr(const void *p) {
  return (uint32_t)(size_t)(const LDS_AS char *)p;
}
// A = corpus fragment (VGPRs), B = query fragment (AGPRs), accumulator VGPRs
// (hazards: pmm_bf16_kernel.h; drain_acc pads an accumulator before reads)
__device__ __forceinline__ void mfma_acc(f32x16 &c, const bf16x8 &cf, const bf16x8 &qf) {
  asm volatile("v_mfma_f32_32x32x16_bf16 %0, %1, %2, %0" : "+v"(c) : "v"(cf), "v"(qf) : "memory");
}
__device__ __forceinline__ void mfma_first(f32x16 &c, const bf16x8 &cf, const bf16x8 &qf) {
  asm volatile("v_mfma_f32_32x32x16_bf16 %0, %1, %2, 0" : "=&v"(c) : "v"(cf), "v"(qf) : "memory");
}
__device__ __forceinline__ void drain_acc(f32x16 &c) { asm volatile("s_nop 7\n\ts_nop 4" : "+v"(c)); }
// f(std::integral_constant<int, 0>{}) ... f(std::integral_constant<int, N - 1>{})
template <typename F, int... I>
__device__ __forceinline__ void static_for_impl(F &&f, std::integer_sequence<int, I...>) {
  (f(std::integral_constant<int, I>{}), ...);
}
template <int N, typename F>
__device__ __forceinline__ void static_for(F &&f) {
  static_for_impl(f, std::make_integer_sequence<int, N>{});
}
}  // namespace wd

// ===========================================================================
// KS = padded D / 128 (K-steps per tile).
// ===========================================================================
template <int KS, int METRIC>
__global__ __launch_bounds__(wd::NTH, 1) void gemm_bf16_wide_kernel(GemmF32Args a) {
  using namespace wd;
  using C = Carve<KS>;
  constexpr int NST = C::NST, LAG = C::LAG;
  constexpr bool XFORM = METRIC != kMetricDot;
  constexpr int NDMA = XFORM ? 2 : 1;  // DMA instructions per wave per K-step
  constexpr int WAITN = NDMA * (AHEAD - 1);
  constexpr int GSTEPS = KS < 4 ? KS : 4;  // K-steps over which a tile's 4 score groups are filtered
  extern __shared__ __attribute__((aligned(16))) char smem[];
  int *unit_l = (int *)(smem + OFF_UNIT);
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int lag = wid >= NW / 2 ? LAG : 0;
  const int r32 = lane & 31, h = lane >> 5;
  u64 *thr_w = (u64 *)(smem + OFF_THR) + wid * 32;
  unsigned *cnt_w = (unsigned *)(smem + OFF_CNT) + wid * 32;
  float *qex_w = (float *)(smem + OFF_QEX) + wid * 32;
  float *lo_w = (float *)(smem + OFF_LO) + wid * 32;
  float *cvl = (float *)(smem + OFF_CV);
  char *ring = smem + OFF_RING;
  const uint32_t ring_lds = lds_addr(ring);
  const uint32_t thr_lds = lds_addr(thr_w), qex_lds = lds_addr(qex_w), cv_lds = lds_addr(cvl);
  const uint32_t cnt_lds = lds_addr(cnt_w);
  // fragment chunk of lane (col r32, half h), substep sub: chunk 8h + sub of
  // column r32, stored at chunk (8h + sub) ^ (r32 & 15) = lane_off ^ (sub << 4)
  const uint32_t lane_off = (uint32_t)(r32 * KB + 16 * ((8 * h) ^ (r32 & 15)));
  const uint32_t acc_lds = lds_addr(smem + OFF_ACC) + (uint32_t)(wid * ACCB) + (uint32_t)lane * 16u;
  // this wave's corpus piece of every K-step: tile columns 4 wid .. 4 wid + 3,
  // chunk ch of column col stored at chunk ch ^ (col & 15)
  const int pcol = 4 * wid + (lane >> 4);
  const uint32_t b_voff = (uint32_t)(pcol * a.ldc * 2 + (((lane & 15) ^ (pcol & 15)) * 16));
  // [n norms | n pre-filter factors] (a.cn, a.cpre = a.cn + N)
  const __amdgpu_buffer_rsrc_t rcv = make_rsrc(a.cn, XFORM ? (int64_t)a.N * 8 : 0);
  bool sync_on = a.round_sync != 0;
  constexpr int QST = C::QST, NQR = C::NQ - C::QST;  // stashed / register-resident fragments
  bf16x8 qf[NQR];  // this wave's query rows, kept across a run's units
  const uint32_t qst_lds = lds_addr(smem + OFF_QST) + (uint32_t)(wid * QST_MAX * 1024) + (uint32_t)lane * 16u;

  for (int round = 0;; round++) {
    UnitPos u;
    if (!unit_at(a, round, u)) break;
    round_sync(a, u.target, tid, sync_on, unit_l);
    const int s = u.seg;
    const int t0 = u.s * a.tps;
    const int t1 = min(t0 + a.tps, a.ntiles);
    const int wrow0 = u.qb * BM + wid * 32;
    if (u.first) {
      // rows past M read as zeros (buffer range); asm loads, invisible to
      // hipcc's waitcnt bookkeeping: drained right here
      const __amdgpu_buffer_rsrc_t rq = make_rsrc(
          a.qb + (int64_t)wrow0 * a.ldq, (int64_t)max(0, min(32, a.M - wrow0)) * a.ldq * 2);
      const uint32_t qoff = (uint32_t)(r32 * a.ldq * 2 + 128 * h);
      asm volatile("s_nop 4" ::"s"(rq));
      // one K-step (8 fragments) per statement, loads and their wait
      // together: hipcc never sees an output before its data has landed
#define PMM_QLOAD(k)                                                                                  \
  if (KS > k)                                                                                         \
    asm volatile(                                                                                     \
        "buffer_load_dwordx4 %0, %8, %9, 0 offen offset:" #k "*256+0\n\t"                            \
        "buffer_load_dwordx4 %1, %8, %9, 0 offen offset:" #k "*256+16\n\t"                           \
        "buffer_load_dwordx4 %2, %8, %9, 0 offen offset:" #k "*256+32\n\t"                           \
        "buffer_load_dwordx4 %3, %8, %9, 0 offen offset:" #k "*256+48\n\t"                           \
        "buffer_load_dwordx4 %4, %8, %9, 0 offen offset:" #k "*256+64\n\t"                           \
        "buffer_load_dwordx4 %5, %8, %9, 0 offen offset:" #k "*256+80\n\t"                           \
        "buffer_load_dwordx4 %6, %8, %9, 0 offen offset:" #k "*256+96\n\t"                           \
        "buffer_load_dwordx4 %7, %8, %9, 0 offen offset:" #k "*256+112\n\t"                          \
        "s_waitcnt vmcnt(0)"                                                                          \
        : "=&v"(QF(8 * k)), "=&v"(QF(8 * k + 1)), "=&v"(QF(8 * k + 2)), "=&v"(QF(8 * k + 3)),        \
          "=&v"(QF(8 * k + 4)), "=&v"(QF(8 * k + 5)), "=&v"(QF(8 * k + 6)), "=&v"(QF(8 * k + 7))     \
        : "v"(qoff), "s"(rq)                                                                          \
        : "memory");
      // fragment i: register qf[i] below NQR, else a temporary stored to LDS
      bf16x8 qtmp[QST_MAX];
#define QF(i) (*((i) < NQR ? &qf[(i) < NQR ? (i) : 0] : &qtmp[(i) >= NQR ? (i) - NQR : 0]))
      PMM_QLOAD(0) PMM_QLOAD(1) PMM_QLOAD(2) PMM_QLOAD(3) PMM_QLOAD(4) PMM_QLOAD(5)
#undef QF
#undef PMM_QLOAD
#pragma unroll
      for (int i = 0; i < QST; i++)
        asm volatile("ds_write_b128 %0, %1 offset:%2" ::"v"(qst_lds), "v"(qtmp[i]), "i"(i * 1024) : "memory");
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
    }
    wave_sync();
    float lo = lo_w[r32];

    // ---- the unit's corpus stream: step j + AHEAD is issued after barrier j
    int st_tile = t0, st_ks = 0, st_cv = t0 & (CVT - 1);
    uint32_t st_slot = 0;  // byte offset of the ring slot
    auto stage_next = [&]() __attribute__((always_inline)) {
      const int col0 = st_tile * BN;
      const __amdgpu_buffer_rsrc_t rb =
          make_rsrc(a.cb + (int64_t)col0 * a.ldc, (int64_t)max(0, min(BN, a.N - col0)) * a.ldc * 2);
      // PMM_ABLATE (benchmarking only): bit 0 = no epilogue, bit 1 = no corpus DMA
      if (!(a.ablate & 2)) dma16(rb, ring + st_slot + wid * 1024, b_voff, (uint32_t)(st_ks * KB));
      if (XFORM) {
        // lanes 0-3: pre-filter factors of columns col0 + 4 wid + 0..3,
        // lanes 4-7: their norms (the same bytes on every step of the tile)
        const int c = col0 + 4 * wid + (lane & 3);
        const uint32_t off = (c < a.N) ? (uint32_t)((lane < 4 ? a.N + c : c) * 4) : 0x7FFFFFF0u;
        if (lane < 8)
          __builtin_amdgcn_raw_ptr_buffer_load_lds(rcv, (LDS_AS void *)(cvl + st_cv * CVS + wid * 8), 4, off, 0,
                                                   0, 0);
      }
      st_slot += STAGE;
      if (st_slot == (uint32_t)(NST * STAGE)) st_slot = 0;
      if (++st_ks == KS) {
        st_ks = 0;
        st_tile++;
        st_cv = (st_cv + 1) & (CVT - 1);
      }
    };

    // ---- compaction of row r's candidate buffer (compact_row's selection,
    // its LDS state through asm): keep the best k, raise the row threshold
    // to the k-th composite and publish it for later units of the row
    auto compact = [&](int r) __attribute__((always_inline)) {
      const int grow = wrow0 + r;
      u64 *base = a.cand + ((int64_t)grow * a.S + s) * a.capg;
      const int n = (int)lds_u32(cnt_lds + (uint32_t)r * 4u);  // > capg - 64 >= k
      u64 x[CAPE];
#pragma unroll
      for (int e = 0; e < CAPE; e++) {
        const int i = lane + 64 * e;
        x[e] = (i < n) ? __hip_atomic_load(base + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0ull;
      }
      const u64 nt = wave_kth_u64<CAPE>(x, a.k);
      wave_keep_ge<CAPE>(x, nt, [&](int pos, u64 v) __attribute__((always_inline)) { base[pos] = v; }, lane);
      if (lane == 0) {
        lds_st32(cnt_lds + (uint32_t)r * 4u, (uint32_t)a.k);
        const u64 t = lds_u64(thr_lds + (uint32_t)r * 8u);
        lds_st64(thr_lds + (uint32_t)r * 8u, nt > t ? nt : t);
        atomicMax(a.gthr + grow, nt);
      }
      wait_lgkm<0>();
    };

    // ---- row state of this lane's query row r32, in registers: its
    // threshold composite, pre-filter bound and norm (refreshed by compaction)
    // compact every row whose buffer could overflow during one tile's
    // epilogue (<= 32 appends per row), at a tile boundary (no live
    // accumulators: the registers compaction needs are free)
    auto compact_rows = [&]() __attribute__((always_inline)) {
      const unsigned cval = lds_u32(cnt_lds + (uint32_t)r32 * 4u);
      u64 need = __ballot(lane < 32 && cval > (unsigned)(a.capg - 32));
      if (need) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the appends are visible
        while (need) {
          const int r = __builtin_ctzll(need);
          need &= need - 1;
          compact(r);
        }
        lo = prefilter_bound<METRIC>(lds_u64(thr_lds + (uint32_t)r32 * 8u),
                                     XFORM ? lds_f32(qex_lds + (uint32_t)r32 * 4u) : 0.0f);
      }
    };

    // ---- epilogue work for tile ptile (accumulators staged in LDS): score
    // groups [glo, ghi) -- group g = accumulators 4g..4g+3 of every lane (its
    // row r32 against columns 8g + 4h + 0..3) -- pre-filtered; survivors
    // re-scored exactly in-lane (reference operation order) and appended to
    // the row's candidate buffer
    auto epi = [&](int ptile, int glo, int ghi) __attribute__((always_inline)) {
      const uint32_t cvb = cv_lds + (uint32_t)((ptile & (CVT - 1)) * CVS * 4 + h * 32);
      const int nvalid = a.N - ptile * BN;  // the corpus's last tile: columns past N never survive
      for (int g = glo; g < ghi; g++) {
        // reads and their wait in one statement: hipcc would otherwise hoist
        // the (register-only) arithmetic on v4 / cv4 above a separate wait
        f32x4 v4, cv4 = {0.0f, 0.0f, 0.0f, 0.0f};
        if (XFORM)
          asm volatile("ds_read_b128 %0, %2\n\tds_read_b128 %1, %3\n\ts_waitcnt lgkmcnt(0)"
                       : "=&v"(v4), "=&v"(cv4)
                       : "v"(acc_lds + (uint32_t)(g * 1024)), "v"(cvb + (uint32_t)(g * 64))
                       : "memory");
        else
          asm volatile("ds_read_b128 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=&v"(v4) : "v"(acc_lds + (uint32_t)(g * 1024))
                       : "memory");
        uint32_t bits = 0u;
#pragma unroll
        for (int i = 0; i < 4; i++) {
          float d = prefilter_diff<METRIC>(v4[i], cv4[i], lo);
          if (nvalid < BN && 8 * g + 4 * h + i >= nvalid) d = -1.0f;
          bits |= (uint32_t)!(d < 0.0f) << i;
        }
        while (__ballot(bits != 0u) != 0ull) {
          if (bits != 0u) {
            const int i = __builtin_ctz(bits);
            bits &= bits - 1u;
            const float v = i == 0 ? v4[0] : i == 1 ? v4[1] : i == 2 ? v4[2] : v4[3];
            const int col = 8 * g + 4 * h + i;  // column of the tile
            const int gcol = ptile * BN + col;
            // (row state from LDS: survivors are rare once the row fills)
            const float cnv = XFORM ? lds_f32(cvb + (uint32_t)(g * 64 + 16 + i * 4)) : 0.0f;
            const float qex = XFORM ? lds_f32(qex_lds + (uint32_t)r32 * 4u) : 0.0f;
            const float sc = exact_score<METRIC>(v, qex, cnv);
            const uint32_t key = okey32(METRIC == kMetricEuclidean ? -sc : sc);
            const u64 comp = ((u64)key << 32) | (u64)(~(uint32_t)gcol);
            if (comp > lds_u64(thr_lds + (uint32_t)r32 * 8u))
              a.cand[((int64_t)(wrow0 + r32) * a.S + s) * a.capg + ws::lds_inc(&cnt_w[r32])] = comp;
          }
        }
      }
    };

    // ---- one K-step of MFMAs (compile-time KSI: the query fragment indices).
    // Corpus fragments alternate between cf[0] and cf[1] (read one substep
    // ahead); unless the step ends the tile, its last MFMA (fragment in
    // cf[1]) is held back past the next barrier, where it covers the latency
    // of that step's first read.  Only acc and cf[1] live across steps.
    f32x16 acc;
    bf16x8 cf[2], qt;  // qt: a stashed query fragment, read one substep ahead
    auto kstep = [&](auto I, uint32_t sb) __attribute__((always_inline)) {
      constexpr int KSI = decltype(I)::value;
      constexpr int g0 = KSI * KSUB;
      static_assert(PF == 1 && KSUB % 2 == 0, "fragment rotation");
      frag_read(cf[0], sb);
      if constexpr (KSI > 0) mfma_acc(acc, cf[1], qf[g0 - 1]);
#pragma unroll
      for (int sub = 0; sub < KSUB; sub++) {
        const int gs = g0 + sub;
        if (sub + 1 < KSUB) frag_read(cf[(sub + 1) & 1], sb ^ (uint32_t)((sub + 1) << 4));
        // a stashed query fragment is read one substep before its use: the
        // first one here, the others right after the MFMA that read qt
        const bool q_first = gs + 1 == NQR && QST > 0;
        if (q_first) asm volatile("ds_read_b128 %0, %1" : "=v"(qt) : "v"(qst_lds) : "memory");
        if (sub == KSUB - 1 && KSI < KS - 1) break;  // deferred to the next step
        // wait for this substep's operands; the reads issued after them may
        // stay in flight.  The wait names the registers it releases ("+v"),
        // so nothing reading them is scheduled above it.
        bf16x8 &fc = cf[sub & 1];
        const int younger = (sub + 1 < KSUB ? 1 : 0) + (q_first ? 1 : 0);
        if (gs >= NQR) {
          if (younger == 1) asm volatile("s_waitcnt lgkmcnt(1)" : "+v"(fc), "+v"(qt)::"memory");
          else asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(fc), "+v"(qt)::"memory");
          mfma_acc(acc, fc, qt);
          if (gs + 1 < NQR + QST)
            asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(qt) : "v"(qst_lds), "i"((gs + 1 - NQR) * 1024)
                         : "memory");
        } else {
          if (younger == 2) asm volatile("s_waitcnt lgkmcnt(2)" : "+v"(fc)::"memory");
          else if (younger == 1) asm volatile("s_waitcnt lgkmcnt(1)" : "+v"(fc)::"memory");
          else asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(fc)::"memory");
          if (gs == 0) mfma_first(acc, fc, qf[0]);
          else mfma_acc(acc, fc, qf[gs]);
        }
      }
    };
    auto stage_acc = [&]() __attribute__((always_inline)) {
      // the tile's accumulators into LDS for the next tile's epilogue steps
      drain_acc(acc);
      // one dword per statement: a 4-register tuple operand would make hipcc
      // copy the accumulators (the layout is the same as 4 x ds_write_b128)
#pragma unroll
      for (int e = 0; e < 16; e++)
        asm volatile("ds_write_b32 %0, %1 offset:%2" ::"v"(acc_lds), "v"(acc[e]), "i"((e >> 2) * 1024 + (e & 3) * 4)
                     : "memory");
    };
    auto idle_step = [&]() __attribute__((always_inline)) {
      wait_lgkm<0>();
      ws::barrier();
      stage_next();
      ws::wait_vm<WAITN>();
    };

    // ---- the unit.  Per K-step: barrier, (tile boundary: compactions), the
    // step's MFMAs, the DMA of stream step j + AHEAD, the previous tile's
    // score groups for this step (filtered while the MFMAs run), and on the
    // tile's last step the accumulators into LDS.  After the last tile, KS
    // epilogue-only steps.  Every wave: nsteps + KS + LAG barriers.
    const bool epi_on = !(a.ablate & 1);
#pragma unroll
    for (int j = 0; j < AHEAD; j++) stage_next();  // stream steps 0 .. AHEAD-1
    ws::wait_vm<WAITN>();                           // step 0 landed
    for (int j = 0; j < lag; j++) idle_step();
    uint32_t rd_slot = 0;
    for (int tile = t0; tile < t1; tile++) {
      static_for<KS>([&](auto KSC) __attribute__((always_inline)) {
        constexpr int ks = decltype(KSC)::value;
        wait_lgkm<0>();  // this wave's reads of its previous slot retired
        ws::barrier();
        if (ks == 0 && tile > t0) compact_rows();
        uint32_t sb = ring_lds + rd_slot + lane_off;
        asm volatile("" : "+v"(sb));  // keep the per-substep XORs in the loop
        kstep(KSC, sb);
        rd_slot += STAGE;
        if (rd_slot == (uint32_t)(NST * STAGE)) rd_slot = 0;
        stage_next();
        if (ks < GSTEPS && tile > t0 && epi_on) epi(tile - 1, ks * 4 / GSTEPS, (ks + 1) * 4 / GSTEPS);
        if (ks == KS - 1) stage_acc();
        ws::wait_vm<WAITN>();  // this wave's pieces of stream step j + 1 landed
      });
    }
    // the last tile's epilogue steps
    for (int k = 0; k < KS; k++) {
      wait_lgkm<0>();
      ws::barrier();
      if (k == 0) compact_rows();
      stage_next();
      if (k < GSTEPS && epi_on) epi(t1 - 1, k * 4 / GSTEPS, (k + 1) * 4 / GSTEPS);
      ws::wait_vm<WAITN>();
    }
    for (int j = lag; j < LAG; j++) idle_step();
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // stream steps past the unit's end
    if (lane < 32) {
      const int grow = wrow0 + lane;
      if (u.last && grow < a.M) a.cnt[(int64_t)grow * a.S + s] = lds_u32(cnt_lds + (uint32_t)lane * 4u);
    }
    wait_lgkm<0>();
    ws::barrier();  // every wave done with the ring and the factor ring
  }
}

template <int KS, int METRIC>
static hipError_t launch_bf16_wide_t(const GemmF32Args &a, int grid, size_t lds, hipStream_t s) {
  static bool attr_set = false;
  if (!attr_set) {
    hipError_t e = hipFuncSetAttribute((const void *)gemm_bf16_wide_kernel<KS, METRIC>,
                                       hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    if (e != hipSuccess) return e;
    attr_set = true;
  }
  gemm_bf16_wide_kernel<KS, METRIC><<<dim3(grid), dim3(wd::NTH), lds, s>>>(a);
  return hipGetLastError();
}

}  // namespace pmm
