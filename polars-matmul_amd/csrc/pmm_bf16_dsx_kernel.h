// pmm_bf16_dsx_kernel.h -- bf16 fused GEMM + top-k with 256 query rows per
// CU (PMM_COMPUTE_BF16; BASELINE configs[3]: 100k x 1M x 768 bf16 cosine
// k=100).  Instantiated per padded-D step count by pmm_bf16_dsx_ks.hip; host
// side in pmm_bf16_dsx.hip.  Same contract as pmm_bf16_ws_kernel.h (bf16
// operands, f32 accumulation, the f32 path's metric epilogue, pre-filter,
// candidate buffers, compaction and merge); a different MFMA shape and
// summation split, so its scores may differ from the other bf16 kernels' in
// the last f32 bits (its seed kernel below reproduces its own sums).
//
// Why: the wave-specialised kernel holds 128 query rows per CU and streams
// every corpus byte through LDS once per 128 rows; its loop is capped by that
// stream (~1250 TFLOP/s at c4) and its epilogue waves (LDS-DMA issue +
// pre-filter + survivors) are slower still.  A wave's register file holds at
// most ~192 registers of query rows, so 256 rows per CU need every register
// of every wave: here each wave keeps 64 query rows x HALF of D (the D split,
// "dsx"), and two waves on different SIMDs that hold the same 64 rows' two
// K-halves form a pair whose partial sums are added in the epilogue.  Per
// streamed corpus byte the CU does twice the work, and one corpus fragment
// read from LDS feeds four MFMAs (4 row blocks of 16).
//
//   * 8 waves, 512 threads, one workgroup per CU.  Waves 0-3 form group X,
//     waves 4-7 group Y (wave w and w + 4 share a SIMD).  In a group, waves
//     (0, 1) hold rows 0-63 of the group's 128, waves (2, 3) rows 64-127; the
//     even wave of a pair holds K in [0, D/2), the odd one [D/2, D).
//   * A tile is 16 corpus columns x D (16x16x32 MFMAs: per substep of 32 K a
//     wave reads ONE 16-byte fragment per lane and issues 4 MFMAs, one per
//     16-row block).  Tiles stream through an NT-slot LDS ring filled by
//     LDS-DMA; every wave issues its share of the pieces.
//   * Group Y runs half a tile behind group X.  Two barriers per tile: Bx(t)
//     opens tile t for X (Y is half way through tile t - 1), By(t) opens it
//     for Y.  So on every SIMD one wave is at a tile boundary (epilogue work:
//     VALU and LDS round trips) while its partner is mid-tile issuing MFMAs,
//     which keep the matrix pipe busy meanwhile.
//   * End of a wave's tile: it writes its partial sums (64 rows x 16 columns,
//     4 KiB) to its LDS region E.  At its next boundary it reads the two
//     partials of its OWN 32 rows (its own and its partner's region), adds
//     them (final = p_lo + p_hi), and runs the f32 path's pre-filter,
//     survivor queue and exact re-score on its 32 rows x 16 columns.  Row
//     state has a single owner.  (Every register is spoken for by the query
//     fragments: nothing of a tile's sums stays in registers across it.)
//
// Ring slot reuse: the DMA into slot (t - 1) % NT (tile t + NT - 1) is issued
// after By(t), when both groups are done with tile t - 1; before Bx(t + 1)
// every wave has waited (counted vmcnt) for its pieces of tile t + 1.  E is
// single-buffered per wave: a wave reads E(t - 1) (its region and its
// partner's) right after its boundary barrier and before the next barrier,
// while both write E(t) only after that next barrier.
#pragma once
#include "pmm_device.h"
#include "pmm_bf16_ws_kernel.h"  // round_sync, unit_at (the same unit schedule)

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace pmm {

#ifndef PMM_DSX_SEL
#define PMM_DSX_SEL 1  // survivor values selected from registers, not re-read from LDS
#endif
#if !defined(PMM_LAB) || !defined(PMM_DSX_ABL)
#undef PMM_DSX_ABL
#define PMM_DSX_ABL 0
#endif

namespace dsx {
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

constexpr int NW = 8;              // waves per workgroup
constexpr int NTH = NW * 64;
constexpr int BM = 256;            // query rows per workgroup
constexpr int BN = kBf16DsxBN;     // corpus columns per tile (16)
constexpr int CVT = 16;            // tiles in the column-factor / column-norm ring
#ifndef PMM_DSX_QCAP
#define PMM_DSX_QCAP 128
#endif
constexpr int QCAP = PMM_DSX_QCAP;  // survivor queue entries per wave
#ifndef PMM_DSX_PF
#define PMM_DSX_PF 3
#endif
constexpr int PF = PMM_DSX_PF;     // corpus fragments read PF substeps ahead
#ifndef PMM_DSX_DRAIN_TILES
#define PMM_DSX_DRAIN_TILES 4      // periodic survivor drain (column norms stay in the CVT ring)
#endif
constexpr int DRAIN = PMM_DSX_DRAIN_TILES;
// LDS carve (bytes)
constexpr int OFF_THR = 0;                        // u64 [BM] row thresholds
constexpr int OFF_CNT = OFF_THR + BM * 8;         // u32 [BM] candidate counts
constexpr int OFF_QEX = OFF_CNT + BM * 4;         // f32 [BM] row norms (exact re-score)
constexpr int OFF_LO = OFF_QEX + BM * 4;          // f32 [BM] pre-filter bounds
constexpr int OFF_UNIT = OFF_LO + BM * 4;         // round-barrier flag
constexpr int OFF_CVR = (OFF_UNIT + 16 + 255) & ~255;  // f32 [CVT][BN] pre-filter column factors
constexpr int OFF_CNR = OFF_CVR + CVT * BN * 4;         // f32 [CVT][BN] column norms
constexpr int EW = 4 * 64 * 16;                   // a wave's partial sums of a tile: 4 row blocks
constexpr int OFF_E = OFF_CNR + CVT * BN * 4;     // [NW][EW]
constexpr int OFF_QUEUE = OFF_E + NW * EW;        // u64 [NW][QCAP]
constexpr int OFF_RING = (OFF_QUEUE + NW * QCAP * 8 + 255) & ~255;
static_assert(DRAIN >= 1 && DRAIN + 8 <= CVT, "queued survivors' column norms must stay in the ring");

template <int KS>  // KS = padded D / 128
struct Carve {
  static constexpr int D = 128 * KS;
  static constexpr int G2 = 2 * KS;                 // 32-K substeps per wave (half of D)
  static constexpr int STAGE = BN * D * 2;          // one tile: 16 columns x D bf16
  static constexpr int PT = STAGE / 1024;           // 1 KiB DMA pieces per tile
  static constexpr int PW = PT / NW;                // pieces per wave per tile
  static constexpr int NT_FIT = (160 * 1024 - OFF_RING) / STAGE;
  static constexpr int NT = NT_FIT > 8 ? 8 : NT_FIT;  // ring slots
  static constexpr int BYTES = OFF_RING + NT * STAGE;
  static_assert(PT % NW == 0, "whole pieces per wave (KS even)");
  static_assert(NT >= 3 && BYTES <= 160 * 1024, "LDS carve");
  static_assert(G2 % 4 == 0 && PF < G2, "half-tiles of whole substeps; kh G2 a multiple of 4 (fragment XOR)");
};

__device__ __forceinline__ void barrier() {
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}
// LDS stores in asm: hipcc waits vmcnt(0) before every LDS store it sees
// while an LDS-DMA is in flight (it cannot tell the ring from the rest of
// the carve), and every wave here keeps ring DMAs in flight.
__device__ __forceinline__ void lds_st128(uint32_t ad, f32x4 v) {
  asm volatile("ds_write_b128 %0, %1" ::"v"(ad), "v"(v) : "memory");
}
__device__ __forceinline__ void lds_st64(uint32_t ad, u64 v) {
  asm volatile("ds_write_b64 %0, %1" ::"v"(ad), "v"(v) : "memory");
}
__device__ __forceinline__ void lds_st32(uint32_t ad, uint32_t v) {
  asm volatile("ds_write_b32 %0, %1" ::"v"(ad), "v"(v) : "memory");
}
__device__ __forceinline__ unsigned lds_inc(uint32_t ad) {
  unsigned r;
  asm volatile("ds_add_rtn_u32 %0, %1, %2\n\ts_waitcnt lgkmcnt(0)" : "=v"(r) : "v"(ad), "v"(1u) : "memory");
  return r;
}
__device__ __forceinline__ void wait_lgkm0() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }
// LDS loads in asm too: hipcc also puts a vmcnt(0) in front of every LDS load
// that may alias an in-flight LDS-DMA, which would drain the ring's
// look-ahead at every read.  The result of an asm load is valid only after a
// covering s_waitcnt lgkmcnt; `ready` ties such a wait to the values it
// covers (they cannot be used, moved or copied before it).
__device__ __forceinline__ f32x4 lds_ld128(uint32_t ad) {
  f32x4 r;
  asm volatile("ds_read_b128 %0, %1" : "=v"(r) : "v"(ad) : "memory");
  return r;
}
__device__ __forceinline__ uint32_t lds_ld32(uint32_t ad) {
  uint32_t r;
  asm volatile("ds_read_b32 %0, %1" : "=v"(r) : "v"(ad) : "memory");
  return r;
}
__device__ __forceinline__ u64 lds_ld64(uint32_t ad) {
  u64 r;
  asm volatile("ds_read_b64 %0, %1" : "=v"(r) : "v"(ad) : "memory");
  return r;
}
template <typename T>
__device__ __forceinline__ int launder(T &v) {
  asm volatile("" : "+v"(v));
  return 0;
}
template <typename... T>
__device__ __forceinline__ void ready(T &...v) {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  (void)(launder(v) + ... + 0);
}
// LDS-DMA in asm: hipcc's wait-count pass treats every LDS-DMA it sees as a
// pending write to all of LDS (and to the DMA's address register) and puts
// vmcnt(0) waits in front of later LDS and register accesses -- in a loop
// that keeps DMAs in flight, at nearly every step.  Issued from asm they are
// invisible to it; the kernel's own counted vmcnt waits cover them, and a
// compiler-counted wait for its own loads only waits longer for them.
// (M0 = the wave-uniform LDS destination; one wait state before the DMA.  M0
// is a reserved register that asm cannot list as clobbered; the compiler
// emits no M0 use in these kernels -- no other LDS-DMA, no indexed register
// moves -- which tests/test_kernel_resources.py checks in the ISA.)
__device__ __forceinline__ void dma_b128(__amdgpu_buffer_rsrc_t r, uint32_t lds, uint32_t voff) {
  asm volatile("s_mov_b32 m0, %0\n\ts_nop 0\n\tbuffer_load_dwordx4 %1, %2, 0 offen lds"
               ::"s"(lds), "v"(voff), "s"(r) : "memory");
}
__device__ __forceinline__ void dma_b32(__amdgpu_buffer_rsrc_t r, uint32_t lds, uint32_t voff) {
  asm volatile("s_mov_b32 m0, %0\n\ts_nop 0\n\tbuffer_load_dword %1, %2, 0 offen lds"
               ::"s"(lds), "v"(voff), "s"(r) : "memory");
}
// vmcnt with a wave-uniform count (the waves issue different numbers of DMAs)
__device__ __forceinline__ void wait_vm(int n) {
  switch (n) {
#define PMM_DSX_W(N) \
  case N: asm volatile("s_waitcnt vmcnt(" #N ")" ::: "memory"); break;
    PMM_DSX_W(0) PMM_DSX_W(1) PMM_DSX_W(2) PMM_DSX_W(3) PMM_DSX_W(4) PMM_DSX_W(5) PMM_DSX_W(6)
    PMM_DSX_W(7) PMM_DSX_W(8) PMM_DSX_W(9) PMM_DSX_W(10) PMM_DSX_W(11) PMM_DSX_W(12) PMM_DSX_W(13)
    PMM_DSX_W(14) PMM_DSX_W(15) PMM_DSX_W(16) PMM_DSX_W(17) PMM_DSX_W(18) PMM_DSX_W(19) PMM_DSX_W(20)
    PMM_DSX_W(21) PMM_DSX_W(22) PMM_DSX_W(23) PMM_DSX_W(24) PMM_DSX_W(25) PMM_DSX_W(26) PMM_DSX_W(27)
    PMM_DSX_W(28) PMM_DSX_W(29) PMM_DSX_W(30)
#undef PMM_DSX_W
    default: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
  }
}
// The lane id, opaque to the optimiser: per-lane addresses derived from it
// are recomputed where used (a few VALU) instead of being hoisted to the
// kernel entry, where the query fragments leave no registers to hold them.
__device__ __forceinline__ int lane_id() {
  int l = (int)__lane_id();
  asm volatile("" : "+v"(l));
  return l;
}
__device__ __forceinline__ f32x4 mfma(const bf16x8 &a, const bf16x8 &b, const f32x4 &c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}
}  // namespace dsx

// Compaction of one row's candidate buffer (compact_row's selection path,
// capg <= 64 E): its loads in asm, so the compiler tracks no load it could
// later mistake for one still pending (it would then wait for every
// in-flight ring DMA at every step of the tile loop), and its keys in E
// registers per lane.
template <int E>
__device__ __forceinline__ void dsx_compact_row_(u64 *base, int n, int k, uint32_t thr_lds, uint32_t cnt_lds,
                                                unsigned long long *gthr_row) {
  using namespace dsx;
  const int lane = lane_id();
  u64 x[E];
#pragma unroll
  for (int e = 0; e < E; e++) {
    const int i = lane + 64 * e;
    const u64 *p = base + (i < n ? i : 0);
    asm volatile("global_load_dwordx2 %0, %1, off sc1" : "=v"(x[e]) : "v"(p) : "memory");
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
  for (int e = 0; e < E; e++) {
    launder(x[e]);
    if (lane + 64 * e >= n) x[e] = 0ull;
  }
  const u64 nt = wave_kth_u64<E>(x, k);
  wave_keep_ge<E>(x, nt, [&](int pos, u64 v) __attribute__((always_inline)) { base[pos] = v; }, lane);
  if (lane == 0) {
    u64 th = lds_ld64(thr_lds);
    ready(th);
    lds_st32(cnt_lds, (uint32_t)k);
    if (nt > th) lds_st64(thr_lds, nt);
    atomicMax(gthr_row, nt);
  }
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
}

// ===========================================================================
// Main kernel.  KS = padded D / 128 (even).
// ===========================================================================
template <int KS, int METRIC>
__global__ __launch_bounds__(dsx::NTH, 1) void gemm_bf16_dsx_kernel(GemmF32Args a) {
  using namespace dsx;
  using C = Carve<KS>;
  constexpr int G2 = C::G2, NT = C::NT, STAGE = C::STAGE, PW = C::PW;
  constexpr int H1 = G2 / 2;  // substeps in the first half of a tile
  constexpr bool XFORM = (METRIC != kMetricDot);
  extern __shared__ __attribute__((aligned(16))) char smem[];
  int *unit_l = (int *)(smem + OFF_UNIT);
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int grp = wid >> 2;            // 0 = X, 1 = Y (half a tile behind)
  const int kh = wid & 1;              // K half of this wave
  const int pr = (wid >> 1) & 1;       // pair inside the group
  const int prow = grp * 128 + pr * 64;      // the pair's 64 rows in the block
  const int orow = prow + kh * 32;           // this wave's own 32 rows (epilogue)
  const int c16 = lane & 15, q4 = lane >> 4;
  const uint32_t smem_lds = (uint32_t)(size_t)(LDS_AS char *)smem;
  const uint32_t ring_lds = smem_lds + OFF_RING;
  // DMA ops this wave issues per tile: its corpus pieces, plus for the
  // normalising metrics one column-factor load (wave 0) or column-norm load
  // (wave 1)
  const int opt = PW + ((XFORM && wid < 2) ? 1 : 0);

  // ---- per-wave LDS state of its 32 own rows ----
  const unsigned *cnt_w = (const unsigned *)(smem + OFF_CNT) + orow;
  const uint32_t cnt_lds = smem_lds + OFF_CNT + orow * 4;
  const uint32_t lo_lds = smem_lds + OFF_LO + orow * 4;
  const uint32_t thr_lds = smem_lds + OFF_THR + orow * 8;
  const uint32_t e_mine = smem_lds + OFF_E + wid * EW;          // written by this wave
  const uint32_t lq_lds = smem_lds + OFF_QUEUE + wid * QCAP * 8;

  // per-lane DMA source offsets (loop-invariant): piece p of a tile = 64
  // 16-byte chunks in LDS order; LDS chunk cs of column col holds global
  // chunk cs ^ (col & 15) of that column (conflict-free fragment reads)
  // (recomputed per tile from the lane id: no registers live across the
  // MFMA loop)
  auto b_voff = [&](int i) __attribute__((always_inline)) {
    const int ln = lane_id();
    const int li = (i * NW + wid) * 64 + ln;    // linear chunk index in the tile
    const int col = li / (2 * KS * 8);          // chunks per column = D * 2 / 16
    const int cs = li % (2 * KS * 8);
    const int ch = cs ^ (col & 15);
    return (uint32_t)(col * a.ldc * 2 + ch * 16);
  };
  // fragment address of substep gs (global over D) for this lane: column
  // c16, global chunk 4 gs + q4, stored at (4 gs + q4) ^ c16 within its
  // 256-byte block: base + 256 (gs >> 2) + ((lane part) ^ (64 (gs & 3)))
  auto frag_lane = [&]() __attribute__((always_inline)) {
    const int ln = lane_id(), l16 = ln & 15, l4 = ln >> 4;
    return (uint32_t)(l16 * (2 * 128 * KS) + 16 * ((l4 ^ l16) & 3) + 16 * (l16 & 12));
  };

  bool sync_on = a.round_sync != 0;
  // lab builds only (`make lab LAB=-DPMM_DSX_ABL=n`, results wrong; a
  // compile-time constant: a runtime flag changes the register allocation):
  // 1 = no epilogue, 2 = no corpus DMA, 4 = no MFMAs (fragment reads stay),
  // 8 = no fragment reads, 16 = pre-filter only (no survivors queued)
  constexpr int abl = PMM_DSX_ABL;
  bf16x8 af[4][G2];  // the pair's 64 rows x this wave's K half: kept across a run's units
  for (int round = 0;; round++) {
    UnitPos u;
    if (!unit_at(a, round, u)) break;
    round_sync(a, u.target, tid, sync_on, unit_l);
    const int s = u.seg;
    const int t0 = u.s * a.tps;
    const int t1 = min(t0 + a.tps, a.ntiles);
    const int blk0 = u.qb * BM;
    const int wrow0 = blk0 + orow;  // global row of own row 0
    if (u.first) {
      // query fragments: row block rb, substep j: rows blk0 + prow + 16 rb +
      // (lane & 15), K = (kh G2 + j) * 32 + 8 q4 .. + 8
      // (one resource per row block and one lane offset, the substep in the
      // instruction's immediate: nothing per load stays live across units)
      uint32_t qoff = (uint32_t)(c16 * a.ldq * 2 + kh * G2 * 64 + 16 * q4);
      asm volatile("" : "+v"(qoff));
#pragma unroll
      for (int rb = 0; rb < 4; rb++) {
        const int r0 = blk0 + prow + 16 * rb;
        const __amdgpu_buffer_rsrc_t rq =
            make_rsrc(a.qb + (int64_t)r0 * a.ldq, (int64_t)max(0, min(16, a.M - r0)) * a.ldq * 2);
#pragma unroll
        for (int j = 0; j < G2; j++)
          asm volatile("buffer_load_dwordx4 %0, %1, %2, 0 offen offset:%3"
                       : "=v"(af[rb][j]) : "v"(qoff), "s"(rq), "i"(64 * j) : "memory");
      }
      if (lane < 32) {
        const int grow = wrow0 + lane;
        const float qv = (XFORM && grow < a.M) ? a.qn[grow] : 0.0f;
        const u64 t = (grow < a.M) ? __hip_atomic_load(a.gthr + grow, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                                   : ~0ull;
        lds_st32(smem_lds + OFF_QEX + (orow + lane) * 4, __float_as_uint(qv));
        lds_st64(thr_lds + lane * 8, t);
        lds_st32(lo_lds + lane * 4, __float_as_uint(prefilter_bound<METRIC>(t, qv)));
        lds_st32(cnt_lds + lane * 4, 0u);
      }
      asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
      // (the fragments were loaded in asm, invisible to the compiler's wait
      // counting: tie every one of them to the wait above)
#pragma unroll
      for (int rb = 0; rb < 4; rb++)
#pragma unroll
        for (int j = 0; j < G2; j++) launder(af[rb][j]);
    }

    // one tile's DMA into its ring slot (tiles past the unit: no memory
    // traffic, zeros into a slot nobody reads, so the counts stay fixed)
    auto stage = [&](int tile) __attribute__((always_inline)) {
      const int col0 = tile * BN;
      const int nrow = tile < t1 ? max(0, min(BN, a.N - col0)) : 0;
      const __amdgpu_buffer_rsrc_t rb = make_rsrc(a.cb + (int64_t)col0 * a.ldc, (int64_t)nrow * a.ldc * 2);
      const int slot = (tile - t0) % NT;
      const uint32_t st = ring_lds + (uint32_t)(slot * STAGE);
      if (abl & 2) return;
#pragma unroll
      for (int i = 0; i < PW; i++)
        dma_b128(rb, __builtin_amdgcn_readfirstlane(st + (uint32_t)((i * NW + wid) * 1024)), b_voff(i));
      if (XFORM && wid < 2) {
        // one dword per lane, lanes 0-15 (an exec-masked DMA still counts once)
        const __amdgpu_buffer_rsrc_t rc = make_rsrc((wid == 0 ? a.cpre : a.cn) + col0, (int64_t)nrow * 4);
        const uint32_t dst = smem_lds + (uint32_t)((wid == 0 ? OFF_CVR : OFF_CNR) + (tile & (CVT - 1)) * BN * 4);
        const int ln = lane_id();
        if (ln < BN) dma_b32(rc, __builtin_amdgcn_readfirstlane(dst), (uint32_t)(ln * 4));
      }
    };

    // ---- survivors: queue drain (exact re-score, append, compaction) ----
    int qlen = 0;  // wave-uniform
    const uint32_t qex_lds = smem_lds + OFF_QEX + orow * 4;
    const uint32_t cnr_lds = smem_lds + OFF_CNR;
    auto drain = [&]() __attribute__((always_inline)) {
      const int lane = lane_id();
      for (int base = 0; base < qlen; base += 64) {
        const int i = base + lane;
        if (i < qlen) {
          u64 it = lds_ld64(lq_lds + (uint32_t)i * 8u);
          ready(it);
          const int rl = (int)((it >> 32) & 31u);
          const int gcol = (int)(it >> 37);
          uint32_t cnv = XFORM ? lds_ld32(cnr_lds + (uint32_t)((((gcol / BN) & (CVT - 1)) * BN + (gcol % BN)) * 4)) : 0u;
          uint32_t qv = XFORM ? lds_ld32(qex_lds + (uint32_t)rl * 4u) : 0u;
          u64 th = lds_ld64(thr_lds + (uint32_t)rl * 8u);
          ready(cnv, qv, th);
          const float sc = exact_score<METRIC>(__uint_as_float((uint32_t)it), __uint_as_float(qv), __uint_as_float(cnv));
          const uint32_t key = okey32(METRIC == kMetricEuclidean ? -sc : sc);
          const u64 comp = ((u64)key << 32) | (u64)(~(uint32_t)gcol);
          if (comp > th) {
            const unsigned pos = lds_inc(cnt_lds + rl * 4);
            a.cand[((int64_t)(wrow0 + rl) * a.S + s) * a.capg + pos] = comp;
          }
        }
        // a round adds at most 64 per row: compact every row that could
        // overflow on the next round
        uint32_t cval = lds_ld32(cnt_lds + (uint32_t)(lane & 31) * 4u);
        ready(cval);
        u64 need = __ballot(lane < 32 && cval > (unsigned)(a.capg - 64));
        if (need) {
          asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the appends landed
          while (need) {
            const int r = __builtin_ctzll(need);
            need &= need - 1;
            u64 *base = a.cand + ((int64_t)(wrow0 + r) * a.S + s) * a.capg;
            uint32_t nr = lds_ld32(cnt_lds + (uint32_t)r * 4u);
            ready(nr);
            if (a.capg <= 384)
              dsx_compact_row_<6>(base, (int)nr, a.k, thr_lds + r * 8, cnt_lds + r * 4, a.gthr + wrow0 + r);
            else
              dsx_compact_row_<8>(base, (int)nr, a.k, thr_lds + r * 8, cnt_lds + r * 4, a.gthr + wrow0 + r);
          }
          // the compacted rows' pre-filter bounds from their new thresholds
          if (lane < 32) {
            u64 th = lds_ld64(thr_lds + (uint32_t)lane * 8u);
            uint32_t qv = lds_ld32(qex_lds + (uint32_t)lane * 4u);
            ready(th, qv);
            lds_st32(lo_lds + (uint32_t)lane * 4u, __float_as_uint(prefilter_bound<METRIC>(th, __uint_as_float(qv))));
          }
          wait_lgkm0();
        }
      }
      qlen = 0;
    };

    // ---- epilogue of tile pt: final = the pair's two partials of this
    // wave's own 32 rows, then the pre-filter of its 32 rows x 16 columns and
    // the survivor queue.  Register-light (the query fragments take 192
    // registers): the finals go back to LDS (over this wave's own partials of
    // its rows, which nobody else reads) and the survivor loop reads them
    // from there.
    const uint32_t e_own_lds = e_mine + 2 * kh * 1024;
    const uint32_t e_part_lds = smem_lds + OFF_E + (wid ^ 1) * EW + 2 * kh * 1024;
    const uint32_t cvr_lds = smem_lds + OFF_CVR;
    auto epilogue = [&](int pt) __attribute__((always_inline)) {
      if (abl & 1) return;
      const int lane = lane_id(), c16 = lane & 15, q4 = lane >> 4;
      const uint32_t lo16 = (uint32_t)lane * 16u;
      f32x4 f0 = lds_ld128(e_part_lds + lo16);
      f32x4 f1 = lds_ld128(e_part_lds + 1024 + lo16);
      f32x4 k0 = lds_ld128(e_own_lds + lo16);
      f32x4 k1 = lds_ld128(e_own_lds + 1024 + lo16);
      f32x4 l0 = lds_ld128(lo_lds + (uint32_t)q4 * 16u);
      f32x4 l1 = lds_ld128(lo_lds + 64 + (uint32_t)q4 * 16u);
      uint32_t cvu = XFORM ? lds_ld32(cvr_lds + (uint32_t)(((pt & (CVT - 1)) * BN + c16) * 4)) : 0u;
      ready(f0, f1, k0, k1, l0, l1, cvu);
      const float cv = __uint_as_float(cvu);
#pragma unroll
      for (int i = 0; i < 4; i++) {
        f0[i] = k0[i] + f0[i];
        f1[i] = k1[i] + f1[i];
      }
      const int gcol = pt * BN + c16;
      // survivor bits: bit 7 - e <-> score e (NaN differences pass)
      uint32_t bits = 0u;
#pragma unroll
      for (int i = 0; i < 4; i++) bits = (bits << 1) | (uint32_t)!(prefilter_diff<METRIC>(f0[i], cv, l0[i]) < 0.0f);
#pragma unroll
      for (int i = 0; i < 4; i++) bits = (bits << 1) | (uint32_t)!(prefilter_diff<METRIC>(f1[i], cv, l1[i]) < 0.0f);
      if (gcol >= a.N) bits = 0u;
      if (__ballot(bits != 0u) == 0ull || (abl & 16)) return;
#if !PMM_DSX_SEL
      lds_st128(e_own_lds + lo16, f0);
      lds_st128(e_own_lds + 1024 + lo16, f1);
      wait_lgkm0();
#endif
      for (;;) {
        const bool act = bits != 0u;
        const u64 mk = __ballot(act);
        if (mk == 0ull) break;
        if (act) {
          const int j = 31 - __builtin_clz(bits);  // bit j <-> e = 7 - j
          bits &= ~(1u << j);
          const int e = 7 - j;
#if PMM_DSX_SEL
          // the value by selects over the finals (no LDS round trip)
          const float s01 = (e & 1) ? f0[1] : f0[0], s23 = (e & 1) ? f0[3] : f0[2];
          const float s45 = (e & 1) ? f1[1] : f1[0], s67 = (e & 1) ? f1[3] : f1[2];
          const float slo = (e & 2) ? s23 : s01, shi = (e & 2) ? s67 : s45;
          const uint32_t v = __float_as_uint((e & 4) ? shi : slo);
#else
          uint32_t v = lds_ld32(e_own_lds + (uint32_t)((e >> 2) * 1024 + (e & 3) * 4) + lo16);
          ready(v);
#endif
          const uint32_t rl = (uint32_t)((e >> 2) * 16 + q4 * 4 + (e & 3));
          const u64 item = (u64)v | ((u64)(rl | ((uint32_t)gcol << 5)) << 32);
          lds_st64(lq_lds + (uint32_t)(qlen + lanes_below(mk)) * 8u, item);
        }
        qlen += __popcll(mk);
        if (qlen > QCAP - 64) {
          wait_lgkm0();
          drain();
        }
      }
      wait_lgkm0();
    };

    // drain turns: X waves on tiles 0, 4, ..; Y waves two tiles later
    auto drain_turn = [&](int pt) __attribute__((always_inline)) {
      return ((pt - t0) % DRAIN) == (grp ? DRAIN / 2 : 0) && qlen > 0;
    };

    // prologue: tiles t0 .. t0 + NT - 2 of the unit in flight; t0 landed
#pragma unroll
    for (int j = 0; j < NT - 1; j++) stage(t0 + j);
    wait_vm((NT - 2) * opt);

    f32x4 acc[4];
    bf16x8 bq[PF + 1];
    // fragment base of a tile (slot + this lane's column/chunk part), made
    // opaque so the per-substep XOR stays in the loop instead of G2 hoisted
    // addresses
    auto fbase = [&](int tile) __attribute__((always_inline)) {
      return (uint32_t)(((tile - t0) % NT) * STAGE) + frag_lane() + (uint32_t)(kh * G2 * 64);
    };
    auto rdfrag = [&](uint32_t fb, int j, int set) __attribute__((always_inline)) {
      if (abl & 8) return;
      // kh G2 is a multiple of 4: substep j's XOR is (j & 3), its block j >> 2
      const uint32_t ad = ring_lds + ((fb ^ (uint32_t)(64 * (j & 3))) + (uint32_t)(256 * (j >> 2)));
      asm volatile("ds_read_b128 %0, %1" : "=v"(bq[set]) : "v"(ad) : "memory");
    };
    // waits for fragment j: min(PF, G2 - 1 - j) younger reads may be pending
    auto wait_frag = [&](int j, bf16x8 &f) __attribute__((always_inline)) {
      const int young = (G2 - 1 - j) < PF ? (G2 - 1 - j) : PF;
      switch (young) {
        case 0: asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(f)::"memory"); break;
        case 1: asm volatile("s_waitcnt lgkmcnt(1)" : "+v"(f)::"memory"); break;
        case 2: asm volatile("s_waitcnt lgkmcnt(2)" : "+v"(f)::"memory"); break;
        case 3: asm volatile("s_waitcnt lgkmcnt(3)" : "+v"(f)::"memory"); break;
        default: asm volatile("s_waitcnt lgkmcnt(4)" : "+v"(f)::"memory"); break;
      }
    };
    // substeps [j0, j1) of tile `tile` (fragments of substeps < j0 + PF
    // already requested)
    auto mfmas = [&](int tile, int j0, int j1) __attribute__((always_inline)) {
      const uint32_t fb = fbase(tile);
#pragma unroll
      for (int j = j0; j < j1; j++) {
        if (j + PF < G2) rdfrag(fb, j + PF, (j + PF) % (PF + 1));
        // fragment j landed: the reads younger than it (LDS returns in
        // order) may stay in flight; the wait is tied to the fragment
        wait_frag(j, bq[j % (PF + 1)]);
        if (!(abl & 4))
#pragma unroll
        for (int rb = 0; rb < 4; rb++)
          acc[rb] = mfma(af[rb][j], bq[j % (PF + 1)], j == 0 ? (f32x4){0.f, 0.f, 0.f, 0.f} : acc[rb]);
        __builtin_amdgcn_sched_barrier(0);
      }
    };
    // end of a tile: the partial sums to E
    auto end_tile = [&]() __attribute__((always_inline)) {
      // the last MFMAs' results -> the asm stores reading them: 4-pass XDL,
      // 8 wait states (hipcc pads nothing in front of an asm statement)
      asm volatile("s_nop 7" : "+v"(acc[0]), "+v"(acc[1]), "+v"(acc[2]), "+v"(acc[3]));
      const uint32_t ad = e_mine + (uint32_t)lane_id() * 16;
#pragma unroll
      for (int rb = 0; rb < 4; rb++) lds_st128(ad + rb * 1024, acc[rb]);
    };
    auto start_tile = [&](int tile) __attribute__((always_inline)) {
      const uint32_t fb = fbase(tile);
#pragma unroll
      for (int p = 0; p < PF; p++) rdfrag(fb, p, p);
    };

    // One loop for both groups (one code path: the register allocator sees
    // one set of live ranges).  Per tile, barriers A and B: for X, A = Bx(t)
    // and B = By(t); for Y, A = By(t) and B = Bx(t + 1) (Y executes Bx(t0)
    // before the loop).  Only the DMA issue and the landed-wait move:
    //   X: A | epilogue(t-1) | first half | B | DMA(t+NT-1) | second half | end | wait(t+1)
    //   Y: A | DMA(t+NT-1) | epilogue(t-1) | first half | wait(t+1) | B | second half | end
    if (grp) barrier();  // Bx(t0)
    for (int tile = t0; tile < t1; tile++) {
      barrier();  // A
      if (grp) stage(tile + NT - 1);
      if (tile > t0) {
        epilogue(tile - 1);
        if (drain_turn(tile - 1)) {
          wait_lgkm0();
          drain();
        }
      }
      start_tile(tile);
      mfmas(tile, 0, H1);
      if (grp) wait_vm((NT - 2) * opt);  // tile + 1 landed before Bx(tile + 1)
      barrier();  // B
      if (!grp) stage(tile + NT - 1);
      mfmas(tile, H1, G2);
      end_tile();
      if (!grp) wait_vm((NT - 2) * opt);  // tile + 1 landed before Bx(tile + 1)
      wait_lgkm0();                       // E written before the next barrier
    }
    barrier();  // X: Bx(t1); Y: By(t1)
    epilogue(t1 - 1);
    if (!grp) barrier();  // By(t1)
    wait_lgkm0();
    drain();
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // ring DMAs past the unit's end
    if (lane < 32) {
      const int grow = wrow0 + lane;
      if (u.last && grow < a.M) a.cnt[(int64_t)grow * a.S + s] = cnt_w[lane];
    }
    barrier();
  }
}

// ===========================================================================
// Threshold seed for the dsx kernel: S[row][col] for the first ns corpus
// rows, computed exactly as the main pass computes them -- the same
// v_mfma_f32_16x16x32_bf16 chains from zero over each K half (the same
// fragment per lane and substep), the same f32 sum of the two halves, the
// same exact_score -- so each sample score is bit for bit the main pass's and
// (k-th best sample composite) - 1 is an exact lower bound of the row's final
// k-th best.  One wave per 16 query rows; corpus fragments straight from
// global memory (the sample is a few MB, L2-resident).
// ===========================================================================
template <int KS, int METRIC>
__global__ __launch_bounds__(256) void seed_bf16_dsx_kernel(GemmF32Args a, float *__restrict__ S, int ns) {
  using namespace dsx;
  constexpr int G2 = 2 * KS;
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
  const int c16 = lane & 15, q4 = lane >> 4;
  const int r0 = (int)blockIdx.x * 64 + w * 16;
  if (r0 >= a.M) return;  // (wave-uniform)
  bf16x8 af[2 * G2];
  {
    const __amdgpu_buffer_rsrc_t rq = make_rsrc(a.qb + (int64_t)r0 * a.ldq, (int64_t)min(16, a.M - r0) * a.ldq * 2);
#pragma unroll
    for (int gs = 0; gs < 2 * G2; gs++)
      af[gs] = __builtin_bit_cast(
          bf16x8, __builtin_amdgcn_raw_buffer_load_b128(rq, (int)(c16 * a.ldq * 2 + (gs * 32 + 8 * q4) * 2), 0, 0));
  }
  constexpr bool XFORM = METRIC != kMetricDot;
  float qv[4];
#pragma unroll
  for (int i = 0; i < 4; i++) {
    const int row = r0 + q4 * 4 + i;
    qv[i] = (XFORM && row < a.M) ? a.qn[row] : 0.0f;
  }
  const __amdgpu_buffer_rsrc_t rc = make_rsrc(a.cb, (int64_t)ns * a.ldc * 2);
  for (int t = 0; t < ns / 16; t++) {
    const int col = t * 16 + c16;
    const uint32_t boff = (uint32_t)(col * a.ldc * 2 + 16 * q4);
    f32x4 p[2];
#pragma unroll
    for (int h = 0; h < 2; h++) {
      bf16x8 b[G2];
#pragma unroll
      for (int j = 0; j < G2; j++)
        b[j] = __builtin_bit_cast(
            bf16x8, __builtin_amdgcn_raw_buffer_load_b128(rc, (int)(boff + (h * G2 + j) * 64), 0, 0));
      f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int j = 0; j < G2; j++) acc = mfma(af[h * G2 + j], b[j], acc);
      p[h] = acc;
    }
    const float cv = XFORM ? a.cn[col] : 0.0f;
#pragma unroll
    for (int i = 0; i < 4; i++) {
      const int row = r0 + q4 * 4 + i;
      if (row < a.M) S[(int64_t)row * ns + col] = exact_score<METRIC>(p[0][i] + p[1][i], qv[i], cv);
    }
  }
}

template <int KS, int METRIC>
static hipError_t launch_seed_bf16_dsx_t(const GemmF32Args &a, float *S, int ns, hipStream_t s) {
  seed_bf16_dsx_kernel<KS, METRIC><<<dim3((unsigned)((a.M + 63) / 64)), dim3(256), 0, s>>>(a, S, ns);
  return hipGetLastError();
}

template <int KS, int METRIC>
static hipError_t launch_bf16_dsx_t(const GemmF32Args &a, int grid, size_t lds, hipStream_t s) {
  static bool attr_set = false;
  if (!attr_set) {
    hipError_t e = hipFuncSetAttribute((const void *)gemm_bf16_dsx_kernel<KS, METRIC>,
                                       hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    if (e != hipSuccess) return e;
    attr_set = true;
  }
  gemm_bf16_dsx_kernel<KS, METRIC><<<dim3(grid), dim3(dsx::NTH), lds, s>>>(a);
  return hipGetLastError();
}

}  // namespace pmm
