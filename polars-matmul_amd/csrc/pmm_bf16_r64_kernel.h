// pmm_bf16_r64_kernel.h -- bf16 fused GEMM + top-k with 256 query rows per CU
// held by ONE wave per SIMD (PMM_COMPUTE_BF16; BASELINE configs[3]: 100k x 1M
// x 768 bf16 cosine k=100).  Instantiated per padded-D step count by
// pmm_bf16_r64_ks.hip; host side in pmm_bf16_r64.hip.
//
// Why: the wave-specialised kernel (pmm_bf16_ws_kernel.h) holds 128 query
// rows per CU, and its loop is capped by the corpus stream it needs for them
// (LDS-DMA at ~17 B/clk per CU).  Here each of the four
// waves holds 64 query rows x D for a whole run of units -- rows 0-31 of the
// wave in AGPRs, rows 32-63 in VGPRs (192 + 192 registers at D = 768) -- so
// every corpus byte streamed through LDS feeds twice the MFMA work.
//
//   * A tile is 32 corpus columns x D; per 16-K substep a wave reads ONE
//     16-byte corpus fragment per lane from LDS and issues two
//     v_mfma_f32_32x32x16_bf16 (its two 32-row blocks).  Tiles stream through
//     an NS-slot LDS ring filled by LDS-DMA, every wave issuing its share.
//   * The same arithmetic as the wave-specialised kernel, bit for bit: the
//     same query and corpus K-chunks per lane and substep, the same chain of
//     MFMAs from the inline constant 0 in the same K order, the same
//     pre-filter, exact_score, composite keys, candidate buffers, compaction
//     and merge.  So its lists equal that kernel's, and its threshold seed
//     (seed_bf16_ws_kernel) is exact here too.
//   * No epilogue waves: the top-k epilogue runs on the MFMA wave.  Two
//     accumulator sets (in AGPRs) alternate between tiles: while tile t's
//     MFMAs run, the pre-filter of tile t - 1 is interleaved between them
//     (one score per substep), so the matrix pipe is not idle during it.
//     Survivors are queued in LDS after the tile's MFMAs and re-scored
//     exactly in 64-wide rounds every DRAIN tiles (or when the queue fills).
//
// Synchronisation: one s_barrier per tile.  Before it every wave has waited
// (counted vmcnt) for its own DMA pieces of the tile; after it the slot of
// tile t - 1 (read by every wave before the barrier) takes tile t + NS - 1.
// Every DMA, the fragment loads of the query rows and the queue stores are
// inline asm (hipcc would otherwise wait for the in-flight ring at every LDS
// access); the kernel's counted waits cover them.
#pragma once
#include "pmm_device.h"
#include "pmm_bf16_ws_kernel.h"  // round_sync, unit_at (the same unit schedule)

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>

namespace pmm {

namespace r64 {
typedef __attribute__((__vector_size__(8 * sizeof(__bf16)))) __bf16 bf16x8;

constexpr int NW = 4;                 // waves (1 per SIMD)
constexpr int NTH = NW * 64;
constexpr int BM = kBf16R64BM;        // query rows per workgroup (256)
constexpr int RW = BM / NW;           // rows per wave (64)
constexpr int BN = kBf16R64BN;        // corpus columns per tile (32)
constexpr int CVT = 16;               // tiles in the column-factor / column-norm ring
#ifndef PMM_R64_QCAP
#define PMM_R64_QCAP 128
#endif
constexpr int QCAP = PMM_R64_QCAP;    // survivor queue entries per wave
#ifndef PMM_R64_DRAIN_TILES
#define PMM_R64_DRAIN_TILES 8
#endif
constexpr int DRAIN = PMM_R64_DRAIN_TILES;
#ifndef R64_NOQUEUE
#define R64_NOQUEUE 0
#endif
#ifndef R64_NOPRE
#define R64_NOPRE 0
#endif
#ifndef PMM_R64_NA
#define PMM_R64_NA 8  // block-1 query fragments held in AGPRs
#endif
#ifndef PMM_R64_PF
#define PMM_R64_PF 1
#endif
constexpr int PF = PMM_R64_PF;        // corpus fragments read PF substeps ahead
// LDS carve (bytes)
constexpr int OFF_THR = 0;                     // u64 [BM] row thresholds
constexpr int OFF_CNT = OFF_THR + BM * 8;      // u32 [BM] candidate counts
constexpr int OFF_QEX = OFF_CNT + BM * 4;      // f32 [BM] row norms (exact re-score)
constexpr int OFF_LO = OFF_QEX + BM * 4;       // f32 [BM] pre-filter bounds
constexpr int OFF_UNIT = OFF_LO + BM * 4;      // round-barrier flag
constexpr int OFF_CVR = (OFF_UNIT + 16 + 255) & ~255;  // f32 [CVT][BN] pre-filter column factors
constexpr int OFF_CNR = OFF_CVR + CVT * BN * 4;         // f32 [CVT][BN] column norms
constexpr int OFF_QUEUE = OFF_CNR + CVT * BN * 4;       // u64 [NW][QCAP]
constexpr int OFF_RING = (OFF_QUEUE + NW * QCAP * 8 + 1023) & ~1023;
static_assert(DRAIN >= 1 && DRAIN + 3 < CVT, "queued survivors' column norms must stay in the ring");

template <int KS>  // KS = padded D / 128
struct Carve {
  static constexpr int G = 8 * KS;               // 16-K substeps per tile
  static constexpr int ROWB = KS * 256;          // bytes of one column's row in a tile
  static constexpr int TILE = BN * ROWB;         // one tile: 32 columns x D bf16
  static constexpr int PW = TILE / 1024 / NW;    // 1 KiB DMA pieces per wave per tile
  static constexpr int NS_FIT = (160 * 1024 - OFF_RING) / TILE;
  static constexpr int NS = NS_FIT > 4 ? 4 : NS_FIT;  // ring slots
  static constexpr int BYTES = OFF_RING + NS * TILE;
  static_assert(PW * NW * 1024 == TILE, "whole 1 KiB pieces per wave");
  static_assert(NS >= 3 && BYTES <= 160 * 1024, "LDS carve");
  static_assert(DRAIN + NS < CVT, "queued survivors' column norms must stay in the ring");
};

__device__ __forceinline__ void barrier() {
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}
__device__ __forceinline__ void wait_lgkm0() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }
// vmcnt with a wave-uniform count known at compile time after unrolling
__device__ __forceinline__ void wait_vm(int n) {
  switch (n) {
#define PMM_R64_W(N) \
  case N: asm volatile("s_waitcnt vmcnt(" #N ")" ::: "memory"); break;
    PMM_R64_W(0) PMM_R64_W(1) PMM_R64_W(2) PMM_R64_W(3) PMM_R64_W(4) PMM_R64_W(5) PMM_R64_W(6)
    PMM_R64_W(7) PMM_R64_W(8) PMM_R64_W(9) PMM_R64_W(10) PMM_R64_W(11) PMM_R64_W(12) PMM_R64_W(13)
    PMM_R64_W(14) PMM_R64_W(15) PMM_R64_W(16) PMM_R64_W(17) PMM_R64_W(18) PMM_R64_W(19) PMM_R64_W(20)
    PMM_R64_W(21) PMM_R64_W(22) PMM_R64_W(23) PMM_R64_W(24) PMM_R64_W(25) PMM_R64_W(26) PMM_R64_W(27)
    PMM_R64_W(28) PMM_R64_W(29) PMM_R64_W(30)
#undef PMM_R64_W
    default: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
  }
}
// LDS-DMA from asm (M0 = the wave-uniform LDS destination; one wait state
// before the load; the descriptor's SGPRs get their 5 states from the s_nop 4
// when they may be fresh from a VALU write -- see tests/test_asm_hazards.py)
__device__ __forceinline__ void dma_b128(__amdgpu_buffer_rsrc_t r, uint32_t lds, uint32_t voff) {
  asm volatile("s_mov_b32 m0, %0\n\ts_nop 0\n\tbuffer_load_dwordx4 %1, %2, 0 offen lds" ::"s"(lds), "v"(voff),
               "s"(r)
               : "memory");
}
__device__ __forceinline__ void dma_b32(__amdgpu_buffer_rsrc_t r, uint32_t lds, uint32_t voff) {
  asm volatile("s_mov_b32 m0, %0\n\ts_nop 0\n\tbuffer_load_dword %1, %2, 0 offen lds" ::"s"(lds), "v"(voff),
               "s"(r)
               : "memory");
}
__device__ __forceinline__ int lane_id() {
  int l = (int)__lane_id();
  asm volatile("" : "+v"(l));
  return l;
}
// MFMA: query rows (A) from AGPRs or VGPRs, the accumulator in AGPRs
__device__ __forceinline__ void mfma_aa(f32x16 &c, const bf16x8 &a, const bf16x8 &b) {
  asm volatile("v_mfma_f32_32x32x16_bf16 %0, %1, %2, %0" : "+a"(c) : "a"(a), "v"(b));
}
__device__ __forceinline__ void mfma_av(f32x16 &c, const bf16x8 &a, const bf16x8 &b) {
  asm volatile("v_mfma_f32_32x32x16_bf16 %0, %1, %2, %0" : "+a"(c) : "v"(a), "v"(b));
}
__device__ __forceinline__ void mfma_aa0(f32x16 &c, const bf16x8 &a, const bf16x8 &b) {
  asm volatile("v_mfma_f32_32x32x16_bf16 %0, %1, %2, 0" : "=&a"(c) : "a"(a), "v"(b));
}
__device__ __forceinline__ void mfma_av0(f32x16 &c, const bf16x8 &a, const bf16x8 &b) {
  asm volatile("v_mfma_f32_32x32x16_bf16 %0, %1, %2, 0" : "=&a"(c) : "v"(a), "v"(b));
}
}  // namespace r64

// Compaction of one row's candidate buffer (capg <= 64 E: E keys per lane):
// keep its best k, raise the row threshold to the k-th and publish it
// (compact_row's selection path with a small E: the query rows leave few
// registers for it).
template <int E>
__device__ __forceinline__ void r64_compact_row(const GemmF32Args &a, int s, int grow, u64 *thr_slot,
                                                unsigned *cnt_slot, int lane) {
  u64 *base = a.cand + ((int64_t)grow * a.S + s) * a.capg;
  const int n = (int)*cnt_slot;
  if (n <= a.k) return;
  u64 x[E];
#pragma unroll
  for (int e = 0; e < E; e++) {
    const int i = lane + 64 * e;
    x[e] = (i < n) ? __hip_atomic_load(base + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0ull;
  }
  const u64 nt = wave_kth_u64<E>(x, a.k);
  wave_keep_ge<E>(x, nt, [&](int pos, u64 v) __attribute__((always_inline)) { base[pos] = v; }, lane);
  wave_sync();
  if (lane == 0) {
    *cnt_slot = (unsigned)a.k;
    if (nt > *thr_slot) *thr_slot = nt;
    atomicMax(a.gthr + grow, nt);
  }
  wave_sync();
}

// ===========================================================================
// Main kernel.  KS = padded D / 128.
// ===========================================================================
template <int KS, int METRIC>
__global__ __launch_bounds__(r64::NTH, 1) void gemm_bf16_r64_kernel(GemmF32Args a) {
  using namespace r64;
  using C = Carve<KS>;
  constexpr int G = C::G, NS = C::NS, TILE = C::TILE, PW = C::PW, ROWB = C::ROWB;
  constexpr bool XFORM = (METRIC != kMetricDot);
  extern __shared__ __attribute__((aligned(16))) char smem[];
  int *unit_l = (int *)(smem + OFF_UNIT);
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int r32 = lane & 31, h = lane >> 5;
  const uint32_t smem_lds = (uint32_t)(size_t)(LDS_AS char *)smem;
  const uint32_t ring_lds = smem_lds + OFF_RING;
  // DMA ops this wave issues per tile: its corpus pieces, plus for the
  // normalising metrics one column-factor load (wave 0) or column-norm load
  // (wave 1)
  const int opt = PW + ((XFORM && wid < 2) ? 1 : 0);

  // per-wave row state (64 rows: lane r owns row r for the row-wide updates)
  u64 *thr_w = (u64 *)(smem + OFF_THR) + wid * RW;
  unsigned *cnt_w = (unsigned *)(smem + OFF_CNT) + wid * RW;
  float *qex_w = (float *)(smem + OFF_QEX) + wid * RW;
  float *lo_w = (float *)(smem + OFF_LO) + wid * RW;
  const float *cvr = (const float *)(smem + OFF_CVR);
  const float *cnr = (const float *)(smem + OFF_CNR);
  const uint32_t lq_lds = smem_lds + OFF_QUEUE + wid * QCAP * 8;
  const u64 *lq = (const u64 *)(smem + OFF_QUEUE) + wid * QCAP;

  bool sync_on = a.round_sync != 0;
  // rows 0-31 of the wave x D in AGPRs (qa); rows 32-63: the first NA
  // substeps' fragments in AGPRs too (qva, the AGPRs the one accumulator set
  // leaves), the rest in VGPRs (qv): kept across a run's units
  constexpr int NA = G >= 16 ? PMM_R64_NA : 0;
  bf16x8 qa[G], qva[NA > 0 ? NA : 1], qv[G - NA];
  for (int round = 0;; round++) {
    UnitPos u;
    if (!unit_at(a, round, u)) break;
    round_sync(a, u.target, tid, sync_on, unit_l);
    const int s = u.seg;
    const int t0 = u.s * a.tps;
    const int t1 = min(t0 + a.tps, a.ntiles);
    const int wrow0 = u.qb * BM + wid * RW;  // global row of the wave's row 0
    if (u.first) {
      // query fragments, the ws kernel's layout: substep gs = 8 ks + sub takes
      // k = 128 ks + 64 h + 8 sub .. + 8 for row r32 of each 32-row block
      const __amdgpu_buffer_rsrc_t ra =
          make_rsrc(a.qb + (int64_t)wrow0 * a.ldq, (int64_t)max(0, min(32, a.M - wrow0)) * a.ldq * 2);
      const __amdgpu_buffer_rsrc_t rv = make_rsrc(a.qb + (int64_t)(wrow0 + 32) * a.ldq,
                                                  (int64_t)max(0, min(32, a.M - wrow0 - 32)) * a.ldq * 2);
      uint32_t qoff = (uint32_t)(r32 * a.ldq * 2 + 128 * h);
      asm volatile("" : "+v"(qoff));
      asm volatile("s_nop 4" ::"s"(ra), "s"(rv));
#pragma unroll
      for (int i = 0; i < G; i++) {
        asm volatile("buffer_load_dwordx4 %0, %1, %2, 0 offen offset:%3"
                     : "=a"(qa[i])
                     : "v"(qoff), "s"(ra), "i"(((i / 8) * 128 + (i % 8) * 8) * 2)
                     : "memory");
        if (i < NA)
          asm volatile("buffer_load_dwordx4 %0, %1, %2, 0 offen offset:%3"
                       : "=a"(qva[i < NA ? i : 0])
                       : "v"(qoff), "s"(rv), "i"(((i / 8) * 128 + (i % 8) * 8) * 2)
                       : "memory");
        else
          asm volatile("buffer_load_dwordx4 %0, %1, %2, 0 offen offset:%3"
                       : "=v"(qv[i >= NA ? i - NA : 0])
                       : "v"(qoff), "s"(rv), "i"(((i / 8) * 128 + (i % 8) * 8) * 2)
                       : "memory");
      }
      {
        const int grow = wrow0 + lane;
        const float qv0 = (XFORM && grow < a.M) ? a.qn[grow] : 0.0f;
        const u64 t = (grow < a.M) ? __hip_atomic_load(a.gthr + grow, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                                   : ~0ull;
        qex_w[lane] = qv0;
        thr_w[lane] = t;
        lo_w[lane] = prefilter_bound<METRIC>(t, qv0);
        cnt_w[lane] = 0u;
      }
      asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
#pragma unroll
      for (int i = 0; i < G; i++) {
        asm volatile("" : "+a"(qa[i]));
        if (i < NA) asm volatile("" : "+a"(qva[i < NA ? i : 0]));
        else asm volatile("" : "+v"(qv[i >= NA ? i - NA : 0]));
      }
    }
    wave_sync();

    // one tile's DMA into its ring slot (tiles past the unit: no memory
    // traffic, zeros into a slot nobody reads, so the counts stay fixed)
    auto stage = [&](int tile) __attribute__((always_inline)) {
      const int col0 = tile * BN;
      const int nrow = tile < t1 ? max(0, min(BN, a.N - col0)) : 0;
      const __amdgpu_buffer_rsrc_t rb = make_rsrc(a.cb + (int64_t)col0 * a.ldc, (int64_t)nrow * a.ldc * 2);
      const uint32_t st = ring_lds + (uint32_t)(((tile - t0) % NS) * TILE);
      const int ln = lane_id();
#pragma unroll
      for (int i = 0; i < PW; i++) {
        // piece p: LDS bytes [p KiB, +1 KiB) of the tile: column col, 16-byte
        // slot sl of its row; chunk ch of a column is stored at slot
        // ch ^ (col & 15) within each 256-byte group (conflict-free reads)
        const int p = i * NW + wid;
        const int o = p * 1024 + ln * 16;
        const int col = o / ROWB, sl = (o % ROWB) >> 4;
        const int ch = (sl & ~15) | ((sl & 15) ^ (col & 15));
        dma_b128(rb, __builtin_amdgcn_readfirstlane(st + (uint32_t)(p * 1024)),
                 (uint32_t)(col * a.ldc * 2 + ch * 16));
      }
      if (XFORM && wid < 2) {
        // one dword per lane, lanes 0-31 (an exec-masked DMA still counts once)
        const __amdgpu_buffer_rsrc_t rc = make_rsrc((wid == 0 ? a.cpre : a.cn) + col0, (int64_t)nrow * 4);
        const uint32_t dst = smem_lds + (uint32_t)((wid == 0 ? OFF_CVR : OFF_CNR) + (tile & (CVT - 1)) * BN * 4);
        if (ln < BN) dma_b32(rc, __builtin_amdgcn_readfirstlane(dst), (uint32_t)(ln * 4));
      }
    };

    // ---- survivors: queue drain (exact re-score, append, compaction) ----
    int qlen = 0;  // wave-uniform
    unsigned long long *cand_w = a.cand + ((int64_t)wrow0 * a.S + s) * a.capg;
    auto drain = [&]() __attribute__((always_inline)) {
#ifdef R64_NODRAIN
      qlen = 0;
      return;
#endif
      for (int base = 0; base < qlen; base += 64) {
        const int i = base + lane;
        if (i < qlen) {
          const u64 it = lq[i];
          const float v = __uint_as_float((uint32_t)it);
          const int rl = (int)((it >> 32) & 63u);
          const int gcol = (int)(it >> 38);
          const float cnv = XFORM ? cnr[((gcol / BN) & (CVT - 1)) * BN + (gcol % BN)] : 0.0f;
          const float sc = exact_score<METRIC>(v, XFORM ? qex_w[rl] : 0.0f, cnv);
          const uint32_t key = okey32(METRIC == kMetricEuclidean ? -sc : sc);
          const u64 comp = ((u64)key << 32) | (u64)(~(uint32_t)gcol);
          if (comp > thr_w[rl]) {
            const unsigned pos = atomicAdd(&cnt_w[rl], 1u);
            // (a wave-uniform 64-bit base and a 32-bit lane offset: the
            // candidate rows of the wave's 64 rows span well under 4 GiB)
            cand_w[(uint32_t)rl * (uint32_t)(a.S * a.capg) + pos] = comp;
          }
        }
        // a round adds at most 64 per row: compact every row that could
        // overflow on the next round
        wave_sync();
        u64 need = __ballot(cnt_w[lane] > (unsigned)(a.capg - 64));
        if (need) {
          asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the appends landed
          while (need) {
            const int r = __builtin_ctzll(need);
            need &= need - 1;
#ifndef R64_NOCOMPACT
            r64_compact_row<kBf16R64MaxCapg / 64>(a, s, wrow0 + r, thr_w + r, cnt_w + r, lane);
#endif
          }
          lo_w[lane] = prefilter_bound<METRIC>(thr_w[lane], qex_w[lane]);
          wave_sync();
        }
      }
      qlen = 0;
    };

    // ---- one accumulator set, in AGPRs: c0 (rows 0-31), c1 (rows 32-63).
    // A tile runs in two halves over the same fragments: half A is block 0's
    // MFMA chain, half B block 1's.  Half A pre-filters block 1 of the
    // previous tile (c1 still holds it) between its MFMAs, half B block 0 of
    // this tile (done in half A).  So each block is pre-filtered while the
    // other block's MFMAs run, with no second accumulator set.
    f32x16 c0, c1;
#pragma unroll
    for (int e = 0; e < 16; e++) c0[e] = c1[e] = 0.0f;
    // pre-filter bounds of 4 rows of the block being pre-filtered, its column factor
    f32x4 lo4 = {0.0f, 0.0f, 0.0f, 0.0f};
    float cv = 0.0f;
    // Survivors go straight into the LDS queue as the pre-filter finds them
    // (one ballot per score; the value is at hand).  Inside an MFMA stream the
    // queue cannot drain: when a score would overflow it, queueing stops there
    // (e_over = its index) and the block's scores from e_over on are
    // pre-filtered again after the half ("catch-up"), draining first.  Early
    // tiles of a unit with a cold threshold do this; later ones queue a few
    // scores per tile.
    int e_over = 16;  // wave-uniform
    // per block: this lane's column is inside the corpus; the queue item's
    // high word without the row (global column << 6 | 4 h)
    bool colok = false;
    uint32_t hib = 0u;
    auto set_tile = [&](int pt) __attribute__((always_inline)) {
      const int gcol = pt * BN + r32;
      cv = XFORM ? cvr[(pt & (CVT - 1)) * BN + r32] : 0.0f;
      colok = gcol < a.N;
      hib = ((uint32_t)gcol << 6) | (uint32_t)(4 * h);
    };
    // bounds of elements 4q .. 4q + 3 of block rb: rows 32 rb + 8 q + 4 h + (0..3)
    auto load_lo = [&](int rb, int q) __attribute__((always_inline)) {
      lo4 = *(const f32x4 *)(lo_w + 32 * rb + 8 * q + 4 * h);
    };
    // pre-filter of score e of block rb (accumulator p), queued if it passes
    // and the queue has room (else queueing stops at e: e_over)
    auto pre = [&](const f32x16 &p, int rb, int e) __attribute__((always_inline)) {
      const float v = p[e];
      const bool pass = !(prefilter_diff<METRIC>(v, cv, lo4[e & 3]) < 0.0f) && colok && !R64_NOQUEUE;
      const u64 mk = __ballot(pass);
      if (mk == 0ull || e_over < 16) return;
      if (qlen + __popcll(mk) > QCAP) {
        e_over = e;
        return;
      }
      if (pass) {
        // item = value | (row in wave | global column << 6) << 32, as two dwords
        const uint32_t hi = hib | (uint32_t)(32 * rb + (e & 3) + 8 * (e >> 2));
        asm volatile("ds_write2_b32 %0, %1, %2 offset1:1" ::"v"(lq_lds + (uint32_t)(qlen + lanes_below(mk)) * 8u),
                     "v"(__float_as_uint(v)), "v"(hi)
                     : "memory");
      }
      qlen += __popcll(mk);
    };
    // fragment of substep gs = 8 ks + sub for this lane (column r32, half
    // h): chunk 16 ks + 8 h + sub, stored at slot 16 ks + ((8 h + sub) ^ (r32
    // & 15)); since 8 h + sub = 8 h ^ sub (sub < 8) that is the sub-0 slot
    // XOR sub: one v_xor per substep off a per-tile base
    auto frag = [&](uint32_t tb0, int gs) __attribute__((always_inline)) -> bf16x8 {
      const int ks = gs >> 3, sub = gs & 7;
      // (opaque per read: hipcc otherwise keeps the 8 XORed bases live across
      // the loop, 8 of the ~60 registers the query rows leave)
      uint32_t t = tb0;
      asm volatile("" : "+v"(t));
      const uint32_t ad = (t ^ (uint32_t)(sub << 4)) + (uint32_t)(ks * 256);
      return *(const LDS_AS bf16x8 *)(size_t)ad;
    };
    // one half: block RB's MFMA chain over the tile (fragments re-read from
    // LDS), block PB's pre-filter (accumulator p) between the MFMAs
    auto half = [&](auto RBc, uint32_t tbase, f32x16 &c, const f32x16 &p, int pb) __attribute__((always_inline)) {
      constexpr int RB = decltype(RBc)::value;
      bf16x8 fb[PF + 1];
#pragma unroll
      for (int j = 0; j < PF; j++) fb[j] = frag(tbase, j);
      constexpr int SPAN = G - 3;  // substeps with scores (from substep 3)
      constexpr int PER = (16 + SPAN - 1) / SPAN;
#pragma unroll
      for (int gs = 0; gs < G; gs++) {
        if (gs + PF < G) fb[(gs + PF) % (PF + 1)] = frag(tbase, gs + PF);
        const bf16x8 b = fb[gs % (PF + 1)];
        if (RB == 0) {
          if (gs == 0) mfma_aa0(c, qa[0], b);
          else mfma_aa(c, qa[gs], b);
        } else if (gs < NA) {
          if (gs == 0) mfma_aa0(c, qva[0], b);
          else mfma_aa(c, qva[gs < NA ? gs : 0], b);
        } else {
          if (gs == 0) mfma_av0(c, qv[0], b);
          else mfma_av(c, qv[gs >= NA ? gs - NA : 0], b);
        }
#pragma unroll
        for (int q = 0; q < PER; q++) {
          const int e = (gs - 3) * PER + q;
          if (gs >= 3 && e < 16 && !R64_NOPRE) {
            if ((e & 3) == 0) load_lo(pb, e >> 2);
            pre(p, pb, e);
          }
        }
        __builtin_amdgcn_sched_barrier(0);
      }
    };
    // after block pb's pre-filter: its scores from e_over on (queueing
    // stopped there) after a drain
    auto settle = [&](const f32x16 &p, int pb) __attribute__((always_inline)) {
      while (e_over < 16) {
        const int from = e_over;
        e_over = 16;
        wait_lgkm0();
        drain();
#pragma unroll
        for (int e = 0; e < 16; e++) {
          if (e >= from) {
            load_lo(pb, e >> 2);
            pre(p, pb, e);
          }
        }
      }
    };

    // prologue: tiles t0 .. t0 + NS - 2 of the unit in flight
#pragma unroll
    for (int j = 0; j < NS - 1; j++) stage(t0 + j);

    for (int tile = t0; tile < t1; tile++) {
      // own pieces of this tile landed (the next NS - 2 tiles may stay in flight)
      wait_vm((NS - 2) * opt);
      barrier();
      stage(tile + NS - 1);  // into the slot of tile - 1: every wave is past it
      uint32_t tbase = ring_lds + (uint32_t)(((tile - t0) % NS) * TILE) + (uint32_t)(r32 * ROWB) +
                       (uint32_t)(((8 * h) ^ (r32 & 15)) << 4);
      asm volatile("" : "+v"(tbase));
      // half A: block 0 of this tile; block 1 of the previous tile pre-filtered
      // (the unit's first tile has none: nothing queued)
      set_tile(tile - 1);
      e_over = tile > t0 ? 16 : 0;
      half(std::integral_constant<int, 0>{}, tbase, c0, c1, 1);
      if (tile > t0) settle(c1, 1);
      // half B: block 1 of this tile; block 0 of this tile pre-filtered
      // (its last MFMA retired: half B's first three substeps pass first)
      set_tile(tile);
      e_over = 16;
      half(std::integral_constant<int, 1>{}, tbase, c1, c0, 0);
      settle(c0, 0);
      if (((tile - t0) % DRAIN) == DRAIN - 1 && qlen > 0) {
        wait_lgkm0();
        drain();
      }
    }
    // the unit's last tile, block 1: its MFMAs retire (8-pass XDL results ->
    // VALU reads: 12 wait states and more), then its pre-filter and survivors
    asm volatile("s_nop 7\n\ts_nop 7" : "+a"(c1));
    set_tile(t1 - 1);
    e_over = 0;
    settle(c1, 1);
    wait_lgkm0();
    drain();
    wait_lgkm0();
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // ring DMAs past the unit's end, appends
    {
      const int grow = wrow0 + lane;
      if (u.last && grow < a.M) a.cnt[(int64_t)grow * a.S + s] = cnt_w[lane];
    }
    barrier();
  }
}

template <int KS, int METRIC>
static hipError_t launch_bf16_r64_t(const GemmF32Args &a, int grid, size_t lds, hipStream_t s) {
  static bool attr_set = false;
  if (!attr_set) {
    hipError_t e = hipFuncSetAttribute((const void *)gemm_bf16_r64_kernel<KS, METRIC>,
                                       hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    if (e != hipSuccess) return e;
    attr_set = true;
  }
  gemm_bf16_r64_kernel<KS, METRIC><<<dim3(grid), dim3(r64::NTH), lds, s>>>(a);
  return hipGetLastError();
}

}  // namespace pmm
