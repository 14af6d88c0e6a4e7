// pmm_bf16_ff_kernel.h -- bf16 fused GEMM + top-k with 256 query rows per CU
// on v_mfma_f32_16x16x32_bf16, survivors stored fire-and-forget
// (PMM_COMPUTE_BF16; BASELINE configs[3]: 100k x 1M x 768 bf16 cosine k=100).
// Instantiated per padded-D step count by pmm_bf16_ff_ks.hip; host side in
// pmm_bf16_ff.hip and pmm_capi.hip (topk_bf16_ff).
//
// Why: the wave-specialised kernel streams every corpus byte
// through LDS once per 128 query rows, which caps its loop near half the bf16
// peak; holding 256 rows per CU halves the stream, but then only one wave per
// SIMD fits (64 rows x D = 384 registers) and every epilogue instruction runs
// on the MFMA waves.  The 256-row loop measured 0.51 of the peak on N(0,1)
// data with 32x32x16 MFMAs and 0.56 with 16x16x32 (the chip holds a higher
// clock on the smaller shape; tools/experiments/bf16_rows64_probe*.hip), so
// this kernel takes the 16x16x32 form and keeps its per-tile work to a
// pre-filter interleaved between the MFMAs:
//   * a STATIC per-row threshold for the whole pass: the row's j-th best of
//     an exact sample (seed_bf16_ws_kernel over the first ns corpus rows),
//     chosen so that about N j / ns scores per row pass -- a guess, checked
//     afterwards: the pass is exact for every row that keeps at least k
//     scores >= its threshold; the rest are re-run on the wave-specialised
//     kernel;
//   * survivors appended fire-and-forget to a per-(unit, wave) region in HBM
//     (raw dot, row, column; one ballot + mbcnt per 64 scores, no atomics, no
//     LDS queue, no exact re-score, no compaction on the MFMA waves);
//   * ff_bucket_kernel re-scores them exactly (the reference's operation
//     order), drops those below the threshold and buckets them into the
//     per-(row, split) candidate lists merge_kernel reads.
// Two accumulator sets alternate between tiles: tile t's MFMAs run while
// tile t - 1's scores are pre-filtered between them.
#pragma once
#include "pmm_device.h"
#include "pmm_bf16_ws_kernel.h"  // round_sync, unit_at

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace pmm {

namespace ff {
typedef __attribute__((__vector_size__(8 * sizeof(__bf16)))) __bf16 bf16x8;

constexpr int NW = 4;             // waves (1 per SIMD)
constexpr int NTH = NW * 64;
constexpr int BM = kBf16FfBM;     // query rows per workgroup (256)
constexpr int RW = BM / NW;       // rows per wave (64): 4 blocks of 16
constexpr int BN = kBf16FfBN;     // corpus columns per tile (32): 2 blocks of 16
constexpr int CVT = 8;            // tiles in the column-factor ring
// LDS carve (bytes)
constexpr int OFF_LO = 0;                               // f32 [BM] pre-filter bounds
constexpr int OFF_UNIT = OFF_LO + BM * 4;               // round-barrier flag
constexpr int OFF_CVR = (OFF_UNIT + 16 + 255) & ~255;   // f32 [CVT][BN] column factors
constexpr int OFF_RING = (OFF_CVR + CVT * BN * 4 + 1023) & ~1023;

template <int KS>  // KS = padded D / 128
struct Carve {
  static constexpr int G = 4 * KS;               // 32-K steps per tile
  static constexpr int ROWB = KS * 256;          // bytes of one column's row in a tile
  static constexpr int TILE = BN * ROWB;         // one tile: 32 columns x D bf16
  static constexpr int PW = TILE / 1024 / NW;    // 1 KiB DMA pieces per wave per tile
  static constexpr int NS_FIT = (160 * 1024 - OFF_RING) / TILE;
  static constexpr int NS = NS_FIT > 4 ? 4 : NS_FIT;  // ring slots
  static constexpr int BYTES = OFF_RING + NS * TILE;
  // query fragments: (block b, step j) flat index b G + j; the first NAF in
  // AGPRs (all 256), the rest in VGPRs
  static constexpr int NF = 4 * G;
  static constexpr int NAF = NF < 64 ? NF : 64;
  static constexpr int NVF = NF - NAF;
  static_assert(PW * NW * 1024 == TILE, "whole 1 KiB pieces per wave");
  static_assert(NS >= 3 && BYTES <= 160 * 1024, "LDS carve");
  static_assert(CVT >= NS + 2, "a tile's column factors stay in the ring until its pre-filter");
};

__device__ __forceinline__ void barrier() {
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}
// vmcnt with a wave-uniform count (0..63)
__device__ __forceinline__ void wait_vm(int n) {
  switch (n < 0 ? 0 : (n > 63 ? 63 : n)) {
#define PMM_FF_W(N) \
  case N: asm volatile("s_waitcnt vmcnt(" #N ")" ::: "memory"); break;
    PMM_FF_W(0) PMM_FF_W(1) PMM_FF_W(2) PMM_FF_W(3) PMM_FF_W(4) PMM_FF_W(5) PMM_FF_W(6) PMM_FF_W(7)
    PMM_FF_W(8) PMM_FF_W(9) PMM_FF_W(10) PMM_FF_W(11) PMM_FF_W(12) PMM_FF_W(13) PMM_FF_W(14) PMM_FF_W(15)
    PMM_FF_W(16) PMM_FF_W(17) PMM_FF_W(18) PMM_FF_W(19) PMM_FF_W(20) PMM_FF_W(21) PMM_FF_W(22) PMM_FF_W(23)
    PMM_FF_W(24) PMM_FF_W(25) PMM_FF_W(26) PMM_FF_W(27) PMM_FF_W(28) PMM_FF_W(29) PMM_FF_W(30) PMM_FF_W(31)
    PMM_FF_W(32) PMM_FF_W(33) PMM_FF_W(34) PMM_FF_W(35) PMM_FF_W(36) PMM_FF_W(37) PMM_FF_W(38) PMM_FF_W(39)
    PMM_FF_W(40) PMM_FF_W(41) PMM_FF_W(42) PMM_FF_W(43) PMM_FF_W(44) PMM_FF_W(45) PMM_FF_W(46) PMM_FF_W(47)
    PMM_FF_W(48) PMM_FF_W(49) PMM_FF_W(50) PMM_FF_W(51) PMM_FF_W(52) PMM_FF_W(53) PMM_FF_W(54) PMM_FF_W(55)
    PMM_FF_W(56) PMM_FF_W(57) PMM_FF_W(58) PMM_FF_W(59) PMM_FF_W(60) PMM_FF_W(61) PMM_FF_W(62) PMM_FF_W(63)
#undef PMM_FF_W
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
// v_mfma_f32_16x16x32_bf16: A (16 query rows x 32 K) from AGPRs or VGPRs, B
// (16 corpus columns x 32 K) from VGPRs, the accumulator in VGPRs; the "0"
// forms start the chain from zero
__device__ __forceinline__ void mma_a(f32x4 &c, const bf16x8 &a, const bf16x8 &b) {
  asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+v"(c) : "a"(a), "v"(b));
}
__device__ __forceinline__ void mma_v(f32x4 &c, const bf16x8 &a, const bf16x8 &b) {
  asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+v"(c) : "v"(a), "v"(b));
}
__device__ __forceinline__ void mma_a0(f32x4 &c, const bf16x8 &a, const bf16x8 &b) {
  asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, 0" : "=&v"(c) : "a"(a), "v"(b));
}
__device__ __forceinline__ void mma_v0(f32x4 &c, const bf16x8 &a, const bf16x8 &b) {
  asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, 0" : "=&v"(c) : "v"(a), "v"(b));
}
typedef f32x4 AccSet[4][2];  // [row block][column block]
}  // namespace ff

// ===========================================================================
// Main kernel.  KS = padded D / 128.
// ===========================================================================
template <int KS, int METRIC>
__global__ __launch_bounds__(ff::NTH, 1) void gemm_bf16_ff_kernel(GemmF32Args a) {
  using namespace ff;
  using C = Carve<KS>;
  constexpr int G = C::G, NS = C::NS, TILE = C::TILE, PW = C::PW, ROWB = C::ROWB;
  constexpr int NAF = C::NAF, NVF = C::NVF;
  constexpr bool XFORM = (METRIC != kMetricDot);
  extern __shared__ __attribute__((aligned(16))) char smem[];
  int *unit_l = (int *)(smem + OFF_UNIT);
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int c16 = lane & 15, grp = lane >> 4;
  const uint32_t smem_lds = (uint32_t)(size_t)(LDS_AS char *)smem;
  const uint32_t ring_lds = smem_lds + OFF_RING;
  // DMA ops this wave issues per tile: its corpus pieces, plus for the
  // normalising metrics the column-factor dword load (wave 0)
  const int opt = PW + ((XFORM && wid == 0) ? 1 : 0);
  float *lo_w = (float *)(smem + OFF_LO) + wid * RW;
  const float *cvr = (const float *)(smem + OFF_CVR);

  bool sync_on = a.round_sync != 0;
  bf16x8 qa[NAF], qv[NVF > 0 ? NVF : 1];
  for (int round = 0;; round++) {
    UnitPos u;
    if (!unit_at(a, round, u)) break;
    round_sync(a, u.target, tid, sync_on, unit_l);
    const int t0 = u.s * a.tps;
    const int t1 = min(t0 + a.tps, a.ntiles);
    const int wrow0 = u.qb * BM + wid * RW;  // global row of the wave's row 0
    const int unit_id = u.s * a.QB + u.qb;
    {
      // query fragments: block b (rows 16 b .. 16 b + 15 of the wave), step j:
      // lane (c16, grp) holds row 16 b + c16, k = 32 j + 8 grp .. + 8
      const __amdgpu_buffer_rsrc_t rq =
          make_rsrc(a.qb + (int64_t)wrow0 * a.ldq, (int64_t)max(0, min(RW, a.M - wrow0)) * a.ldq * 2);
      // one per-lane offset (row c16, k 8 grp), the block in the scalar
      // offset, the step in the immediate (64 j < 4096): no per-fragment
      // address registers (hipcc hoisted 96 of them out of the unit loop)
      uint32_t qoff = (uint32_t)((c16 * a.ldq + 8 * grp) * 2);
      asm volatile("" : "+v"(qoff));
      asm volatile("s_nop 4" ::"s"(rq));
#pragma unroll
      for (int f = 0; f < C::NF; f++) {
        const int b = f / G, j = f % G;
        const uint32_t sof = __builtin_amdgcn_readfirstlane((uint32_t)(16 * b * a.ldq * 2));
        if (f < NAF)
          asm volatile("buffer_load_dwordx4 %0, %1, %2, %3 offen offset:%4"
                       : "=a"(qa[f < NAF ? f : 0])
                       : "v"(qoff), "s"(rq), "s"(sof), "i"(64 * j)
                       : "memory");
        else
          asm volatile("buffer_load_dwordx4 %0, %1, %2, %3 offen offset:%4"
                       : "=v"(qv[f >= NAF ? f - NAF : 0])
                       : "v"(qoff), "s"(rq), "s"(sof), "i"(64 * j)
                       : "memory");
      }
      {
        const int grow = wrow0 + lane;
        const float qn0 = (XFORM && grow < a.M) ? a.qn[grow] : 0.0f;
        const u64 t = grow < a.M ? a.gthr[grow] : ~0ull;
        lo_w[lane] = prefilter_bound<METRIC>(t, qn0);
      }
      asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
#pragma unroll
      for (int f = 0; f < C::NF; f++) {
        if (f < NAF) asm volatile("" : "+a"(qa[f < NAF ? f : 0]));
        else asm volatile("" : "+v"(qv[f >= NAF ? f - NAF : 0]));
      }
    }
    // this (unit, wave)'s survivor region: count in an SGPR (wave-uniform)
    unsigned long long *reg = a.ffreg + ((int64_t)unit_id * NW + wid) * a.ffcap;
    unsigned nreg = 0;
    // store instructions issued this tile and the two before (the counted
    // vmcnt waits must know every VMEM op younger than a tile's DMA)
    int st_cur = 0, st_p1 = 0, st_p2 = 0;
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
        dma_b128(rb, __builtin_amdgcn_readfirstlane(st + (uint32_t)(p * 1024)), (uint32_t)(col * a.ldc * 2 + ch * 16));
      }
      if (XFORM && wid == 0) {
        const __amdgpu_buffer_rsrc_t rc = make_rsrc(a.cpre + col0, (int64_t)nrow * 4);
        const uint32_t dst = smem_lds + (uint32_t)(OFF_CVR + (tile & (CVT - 1)) * BN * 4);
        if (ln < BN) dma_b32(rc, __builtin_amdgcn_readfirstlane(dst), (uint32_t)(ln * 4));
      }
    };

    // fragment of column block cb at step j for this lane (column col =
    // 16 cb + c16, chunk 4 j + grp, stored at slot chunk ^ (col & 15) of its
    // 256-byte group): from a per-tile base tb[cb] holding the step-0 slot,
    // slot (4 (j & 3) + grp) ^ (col & 15) is that base XOR (j & 3) << 6 bytes
    // (grp < 4), plus 256 (j >> 2): one v_xor per read, the rest immediate
    auto frag = [&](uint32_t tbase, int j) __attribute__((always_inline)) -> bf16x8 {
      uint32_t t = tbase;
      asm volatile("" : "+v"(t));  // (keeps hipcc from hoisting G addresses per tile)
      const uint32_t ad = (t ^ (uint32_t)((j & 3) << 6)) + (uint32_t)(256 * (j >> 2));
      return *(const LDS_AS bf16x8 *)(size_t)ad;
    };

    // pre-filter of the previous tile's scores (set P), item e of 32:
    // row block b = e / 8, column block cb = (e / 4) & 1, register i = e & 3:
    // lane (c16, grp) holds row 16 b + 4 grp + i, column 16 cb + c16.  The
    // lane-derived values are rebuilt per tile from an opaque lane id (kept
    // live across the unit loop they were spilled, and every reload waited
    // on the whole DMA ring)
    f32x4 lo4 = {0.0f, 0.0f, 0.0f, 0.0f};
    float cv0 = 0.0f, cv1 = 0.0f;
    bool ok0 = false, ok1 = false;
    uint32_t hib0 = 0u, hib1 = 0u;  // item high word: (4 grp) << 26 | global column
    uint32_t lo_base = 0u;          // LDS address of lo_w[4 grp]
    auto set_prev = [&](int pt) __attribute__((always_inline)) {
      const int ln = lane_id();
      const int cl = ln & 15, gp = ln >> 4;
      const int g0 = pt * BN + cl, g1 = g0 + 16;
      ok0 = pt >= t0 && g0 < a.N;
      ok1 = pt >= t0 && g1 < a.N;
      cv0 = XFORM ? cvr[(pt & (CVT - 1)) * BN + cl] : 0.0f;
      cv1 = XFORM ? cvr[(pt & (CVT - 1)) * BN + 16 + cl] : 0.0f;
      hib0 = ((uint32_t)(4 * gp) << 26) | (uint32_t)g0;
      hib1 = ((uint32_t)(4 * gp) << 26) | (uint32_t)g1;
      lo_base = (uint32_t)(size_t)(LDS_AS float *)(lo_w + 4 * gp);
    };
    auto pre = [&](const AccSet &P, int e) __attribute__((always_inline)) {
      if (PMM_ABL(a.ablate & 1)) return;  // (lab: no pre-filter at all)
      const int b = e >> 3, cb = (e >> 2) & 1, i = e & 3;
      if ((e & 7) == 0) lo4 = *(const LDS_AS f32x4 *)(size_t)(lo_base + 64u * (uint32_t)b);
      const float v = P[b][cb][i];
      const bool pass = !(prefilter_diff<METRIC>(v, cb ? cv1 : cv0, lo4[i]) < 0.0f) && (cb ? ok1 : ok0);
      const u64 mk = __ballot(pass);
      if (mk == 0ull) return;
      // fire-and-forget append: no atomics (the region is this wave's), the
      // count stays in an SGPR; past the region's capacity nothing is stored
      // but the count runs on (the bucket pass then re-runs the region's rows)
      const unsigned slot = nreg + (unsigned)lanes_below(mk);
      const bool put = pass && slot < (unsigned)a.ffcap && !PMM_ABL(a.ablate & 2);  // (lab: no stores)
      if (put) {
        const uint32_t hi = (cb ? hib1 : hib0) + ((uint32_t)(16 * b + i) << 26);
        reg[slot] = ((u64)hi << 32) | (u64)__float_as_uint(v);
      }
      nreg += (unsigned)__popcll(mk);
      // (counted only when some lane stores: a count for a store that was
      // never issued would let a wait miss a DMA piece; an uncounted one
      // only makes the wait longer)
      st_cur += __ballot(put) != 0ull ? 1 : 0;
    };

    // one tile: its 8 G MFMAs on set A (from zero), set P's pre-filter
    // (the previous tile) spread between them
    auto tile_body = [&](int tile, AccSet &A, const AccSet &P) __attribute__((always_inline)) {
      // own pieces of this tile landed: everything younger than them may stay
      // in flight (the next NS - 2 tiles' DMA and the survivor stores issued
      // since this tile's DMA went out)
      wait_vm((NS - 2) * opt + st_cur + (NS >= 3 ? st_p1 : 0) + (NS >= 4 ? st_p2 : 0));
      barrier();
      stage(tile + NS - 1);  // into the slot of tile - 1: every wave is past it
      st_p2 = st_p1;
      st_p1 = st_cur;
      st_cur = 0;
      set_prev(tile - 1);
      const uint32_t sb = ring_lds + (uint32_t)(((tile - t0) % NS) * TILE);
      uint32_t tb0, tb1;
      {
        const int ln = lane_id();
        const int col = ln & 15, gp = ln >> 4;  // column block 0; block 1 is col + 16, the same swizzle
        tb0 = sb + (uint32_t)(col * ROWB + 16 * (gp ^ (col & 15)));
        tb1 = tb0 + (uint32_t)(16 * ROWB);
      }
      // fragments ping-pong by step parity (no register moves between the
      // reads and the MFMAs that consume them)
      bf16x8 fr[2][2];
      fr[0][0] = frag(tb0, 0);
      fr[0][1] = frag(tb1, 0);
      constexpr int SPAN = G > 1 ? G - 1 : 1;  // steps carrying pre-filter items (from step 1)
      constexpr int PER = (32 + SPAN - 1) / SPAN;
#pragma unroll
      for (int j = 0; j < G; j++) {
        if (j + 1 < G) {
          fr[(j + 1) & 1][0] = frag(tb0, j + 1);
          fr[(j + 1) & 1][1] = frag(tb1, j + 1);
        }
#pragma unroll
        for (int b = 0; b < 4; b++) {
          const int f = b * G + j;
#pragma unroll
          for (int cb = 0; cb < 2; cb++) {
            const bf16x8 &fb = fr[j & 1][cb];
            if (f < NAF) {
              if (j == 0) mma_a0(A[b][cb], qa[f < NAF ? f : 0], fb);
              else mma_a(A[b][cb], qa[f < NAF ? f : 0], fb);
            } else {
              if (j == 0) mma_v0(A[b][cb], qv[f >= NAF ? f - NAF : 0], fb);
              else mma_v(A[b][cb], qv[f >= NAF ? f - NAF : 0], fb);
            }
          }
        }
        if (j >= 1 || G == 1) {
#pragma unroll
          for (int q = 0; q < PER; q++) {
            const int e = (G > 1 ? (j - 1) : 0) * PER + q;
            if (e < 32) pre(P, e);
          }
        }
        __builtin_amdgcn_sched_barrier(0);
      }
    };

    // prologue: tiles t0 .. t0 + NS - 2 of the unit in flight
#pragma unroll
    for (int j = 0; j < NS - 1; j++) stage(t0 + j);
    AccSet X, Y;
#pragma unroll
    for (int b = 0; b < 4; b++)
#pragma unroll
      for (int cb = 0; cb < 2; cb++) X[b][cb] = Y[b][cb] = (f32x4){0.0f, 0.0f, 0.0f, 0.0f};
    int tile = t0;
    for (; tile + 1 < t1; tile += 2) {
      tile_body(tile, X, Y);
      tile_body(tile + 1, Y, X);
    }
    if (tile < t1) tile_body(tile, X, Y);
    // the unit's last tile: its MFMAs retire, then its pre-filter
    asm volatile("s_nop 7\n\ts_nop 7" ::: "memory");
    set_prev(t1 - 1);
    {
      const bool in_x = ((t1 - 1 - t0) & 1) == 0;  // wave-uniform
      if (in_x) {
#pragma unroll
        for (int e = 0; e < 32; e++) pre(X, e);
      } else {
#pragma unroll
        for (int e = 0; e < 32; e++) pre(Y, e);
      }
    }
    if (lane == 0) a.ffcnt[(int64_t)unit_id * NW + wid] = nreg;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // ring DMAs past the unit's end, appends
    barrier();
  }
}

template <int KS, int METRIC>
static hipError_t launch_bf16_ff_t(const GemmF32Args &a, int grid, size_t lds, hipStream_t s) {
  static bool attr_set = false;
  if (!attr_set) {
    hipError_t e = hipFuncSetAttribute((const void *)gemm_bf16_ff_kernel<KS, METRIC>,
                                       hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    if (e != hipSuccess) return e;
    attr_set = true;
  }
  gemm_bf16_ff_kernel<KS, METRIC><<<dim3(grid), dim3(ff::NTH), lds, s>>>(a);
  return hipGetLastError();
}

}  // namespace pmm
