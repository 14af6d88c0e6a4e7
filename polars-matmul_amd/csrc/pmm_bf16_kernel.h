// pmm_bf16_kernel.h -- the bf16 fused GEMM + top-k kernel template, instantiated
// per padded-D step count by pmm_bf16_ks.hip; host side in pmm_bf16.hip.
//
// bf16 compute path of the fused top-k (PMM_COMPUTE_BF16;
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
#pragma once
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
constexpr int KB = 256;                      // bytes of a row per K-step (128 bf16)
constexpr int KSUB = KB / 32;                // MFMA substeps (K = 16) per K-step
constexpr int STAGE = BN * KB;               // BN corpus rows x 128 bf16
constexpr int BPIECES = STAGE / 1024 / NW;   // 1 KiB LDS-DMA pieces per wave per step
constexpr int QCAP = 256;                    // LDS survivor queue per wave (items)
// LDS carve: per-row state, per-tile column data, the survivor queues, then
// the corpus ring (a.nst slots), then the per-wave compaction scratch.
constexpr int OFF_THR = 0;
constexpr int OFF_CNT = OFF_THR + BM * 8;
constexpr int OFF_QEX = OFF_CNT + BM * 4;
constexpr int OFF_LO = OFF_QEX + BM * 4;
constexpr int OFF_CV = OFF_LO + BM * 4;      // pre-filter column factors, 4 tiles
constexpr int OFF_QUEUE = OFF_CV + 4 * BN * 4;
constexpr int OFF_STAGE = OFF_QUEUE + NW * QCAP * 8;  // survivor staging [wave][lane][16]
constexpr int OFF_UNIT = OFF_STAGE + NW * 64 * 16 * 4;
constexpr int OFF_RING = (OFF_UNIT + 16 + 255) & ~255;
static_assert(OFF_RING % 256 == 0 && STAGE % 256 == 0, "LDS carve alignment");
constexpr int CV_PER_WAVE = BN / NW;          // pre-filter factors DMA'd per wave per tile
static_assert(CV_PER_WAVE <= 64, "one 4-byte DMA per lane covers a wave's factors");
}  // namespace

// s_waitcnt vmcnt(N) as one instruction with a compile-time N; the memory
// clobber keeps the compiler from moving LDS reads across it.
template <int N>
__device__ __forceinline__ void wait_vm() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// ---------------------------------------------------------------------------
// MFMA through inline asm so the query fragment (A) is read straight from the
// accumulator register file ("a") and the accumulator lives in VGPRs ("v"):
// the 192 registers of a wave's query rows (D = 768) then sit in AGPRs, and
// the VGPRs hold two accumulator sets, the corpus fragments in flight and the
// epilogue.  Hazards hipcc does not pad inside asm (cdna_hip_programming.md
// 5.7): the accumulate chain (D -> next MFMA's C, same registers) needs no
// wait states; an MFMA's D read by anything else needs 12 (8-pass XDL):
// mfma_drain() pads them after a tile's last MFMAs.  The A registers are
// written once per unit, long before the first MFMA reads them.
// ---------------------------------------------------------------------------
// (volatile + "memory": the LDS fragment reads written ahead of an MFMA in
// the source stay ahead of it, so the prefetch distance is the source's.)
__device__ __forceinline__ void mfma_acc(f32x16 &c, const bf16x8 &a, const bf16x8 &b) {
  asm volatile("v_mfma_f32_32x32x16_bf16 %0, %1, %2, %0" : "+v"(c) : "a"(a), "v"(b) : "memory");
}
__device__ __forceinline__ void mfma_first(f32x16 &c, const bf16x8 &a, const bf16x8 &b) {
  asm volatile("v_mfma_f32_32x32x16_bf16 %0, %1, %2, 0" : "=&v"(c) : "a"(a), "v"(b) : "memory");
}
template <int NBX>
__device__ __forceinline__ void mfma_drain(f32x16 (&acc)[NBX]) {
  // 12 wait states between the last MFMAs and any other access of their D;
  // the "+v" operands keep every reader below this point
  asm volatile("s_nop 7\n\ts_nop 4" : "+v"(acc[0]), "+v"(acc[NBX - 1]));
#pragma unroll
  for (int c = 1; c < NBX - 1; c++) asm volatile("" : "+v"(acc[c]));
}

// Wave-wide OR / sum in DPP steps (quad perms, row half-mirror, row mirror,
// row_bcast:15, row_bcast:31), a few cycles each, instead of ds_bpermute
// shuffles (an LDS round trip each); the result is uniform (lane 63's).
#define PMM_DPP(x, ctrl, rmask) \
  __builtin_amdgcn_update_dpp(0u, (x), (ctrl), (rmask), 0xf, false)
__device__ __forceinline__ uint32_t wave_or(uint32_t x) {
  x |= PMM_DPP(x, 0xb1, 0xf);   // quad_perm [1,0,3,2]
  x |= PMM_DPP(x, 0x4e, 0xf);   // quad_perm [2,3,0,1]
  x |= PMM_DPP(x, 0x141, 0xf);  // row_half_mirror
  x |= PMM_DPP(x, 0x140, 0xf);  // row_mirror
  x |= PMM_DPP(x, 0x142, 0xa);  // row_bcast:15 -> rows 1, 3
  x |= PMM_DPP(x, 0x143, 0xc);  // row_bcast:31 -> rows 2, 3
  return __builtin_amdgcn_readlane(x, 63);
}
__device__ __forceinline__ uint32_t wave_sum(uint32_t x) {
  x += PMM_DPP(x, 0xb1, 0xf);
  x += PMM_DPP(x, 0x4e, 0xf);
  x += PMM_DPP(x, 0x141, 0xf);
  x += PMM_DPP(x, 0x140, 0xf);
  x += PMM_DPP(x, 0x142, 0xa);
  x += PMM_DPP(x, 0x143, 0xc);
  return __builtin_amdgcn_readlane(x, 63);
}
#undef PMM_DPP

// ===========================================================================
// Fused bf16 GEMM + metric + per-row top-k.  KS = padded D / 128 (K-steps).
//
// Work units as in the f32 kernel (query block x corpus split, pulled from an
// atomic counter, split-major so co-resident workgroups stream the same
// corpus tiles through their XCD's L2).  Per unit a wave loads its 32 query
// rows into AGPRs once (af[]: lane (r, h) holds row r, columns
// 128*ks + 8*(8h + sub) .. +8 for K-step ks, MFMA substep sub), then streams
// the unit's corpus tiles.  Corpus K-step g lives in ring slot g % NST; step
// g + NST - 1 is issued behind the first MFMA group of step g, and step g
// waits only for its own DMAs (counted vmcnt).
//
// Epilogue, software-pipelined by one tile (one wave per SIMD: the VALU work
// must hide inside the MFMA stream): tile t accumulates into set t & 1 while
// its MFMA substeps also run the pre-filter of tile t - 1 (set (t - 1) & 1):
// per score one difference, one compare and a shift into a per-lane
// survivor word (bit 15 - e of word c = row e, column group c).  After tile
// t's K-loop the survivors of tile t - 1 (a few per tile once the row
// thresholds settle) are found from the wave-OR of the words (uniform bit
// tests over the 64 (c, e) pairs, compile-time register indices), queued in
// LDS, and re-scored exactly (pass 2: reference order, norms from LDS) into
// the rows' candidate buffers.  A tile with more survivors than the LDS queue
// holds (a unit's first tiles) takes the per-score path through a global
// queue instead.
// ===========================================================================
// KS = padded D / 128; NST = ring slots; PF = fragment prefetch depth (substeps);
// DEF = hold each K-step's last MFMA group back to after the next barrier
template <int KS, int METRIC, int NST, int PF, int DEF>
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
  constexpr int nst = NST;
  char *ring = smem + OFF_RING;
  u64 *scr = (u64 *)(ring + nst * STAGE) + (size_t)wid * a.capg;
  u64 *thr_w = thr_l + wid * 32;
  unsigned *cnt_w = cnt_l + wid * 32;
  float *qex_w = qex_l + wid * 32;
  float *lo_w = lo_l + wid * 32;
  u64 *lq = (u64 *)(smem + OFF_QUEUE) + (size_t)wid * QCAP;
  float *sbuf = (float *)(smem + OFF_STAGE) + ((size_t)wid * 64 + lane) * 16;
  constexpr bool XFORM = (METRIC != kMetricDot);
  constexpr int G = KS * KSUB;  // MFMA substeps per tile
  // PIPE: compute tile t-1's survivor bits between tile t's MFMAs (two
  // accumulator sets; the asm pins keep LLVM from sinking the work below
  // the loop).  Measured no faster than computing them right after each
  // tile's own K-loop (the loop grew by what the epilogue lost), so it is
  // off and the kernel runs one accumulator set.
  constexpr bool PIPE = false;
  constexpr bool DEFER = DEF != 0;

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

  uint32_t st_q = 0, st_g = 0, st_c = 0;  // PMM_STATS counters (wave-uniform)
  uint64_t cy_loop = 0, cy_ext = 0, cy_drain = 0;  // PMM_STATS: shader cycles per phase
  const bool timing = a.stats != nullptr;

  // Static round-robin schedule with a round barrier.  Round r runs units
  // r * grid + blockIdx.x: a round is (almost) one corpus split, and the 32
  // workgroups of an XCD (blocks b, b + 8, ...) stream its tiles together,
  // so the XCD's L2 serves each tile once.  Without re-alignment their uneven
  // epilogues let them drift apart across rounds until every tile comes from
  // MALL / HBM (measured: L2 hit rate 17%, 1 TB per launch at 100k x 1M).
  // The barrier is for speed only: spins are bounded, and a workgroup that
  // times out (e.g. a grid not fully resident) stops syncing; the schedule
  // itself does not depend on it.
  bool sync_on = a.round_sync != 0;
  unsigned *round_bar = a.counter + 32;  // own 128-byte line, zeroed per call
  for (int round = 0;; round++) {
    const int unit = round * (int)gridDim.x + (int)blockIdx.x;
    if (unit >= a.units) break;
    if (sync_on) {
      if (tid == 0) {
        const int parts = min((int)gridDim.x, a.units - round * (int)gridDim.x);
        const unsigned target = (unsigned)(round * (int)gridDim.x + parts);
        atomicAdd(round_bar, 1u);
        const uint64_t tstart = wall_clock64();
        int ok = 1;
        // an atomic read (RMW of 0) is served at the coherence point
        while (__hip_atomic_fetch_add(round_bar, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) <
               target) {
          __builtin_amdgcn_s_sleep(8);
          if (wall_clock64() - tstart > (uint64_t)a.sync_timeout) {  // 100 MHz wall clock
            ok = 0;
            break;
          }
        }
        if (!ok && a.stats) atomicAdd(a.stats + 2, 1ull);
        *unit_l = ok;
      }
      __syncthreads();
      sync_on = *unit_l != 0;
      __syncthreads();
    }
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

    // This wave's query rows, register-resident in AGPRs for the whole unit:
    // loaded by asm straight into AGPRs ("=a"), so the compiler never stages
    // them through VGPRs; rows past M read as zeros (buffer range).  These
    // loads are invisible to hipcc's waitcnt bookkeeping: they are issued
    // before the unit's first corpus DMAs, so the first K-step's counted
    // vmcnt wait (which leaves only younger DMAs outstanding) covers them.
    bf16x8 af[KSUB * KS];
    {
      const __amdgpu_buffer_rsrc_t rq = make_rsrc(
          a.qb + (int64_t)wrow0 * a.ldq, (int64_t)max(0, min(32, a.M - wrow0)) * a.ldq * 2);
      const uint32_t qoff = (uint32_t)(r32 * a.ldq * 2 + 128 * h);
#pragma unroll
      for (int i = 0; i < KSUB * KS; i++)
        asm volatile("buffer_load_dwordx4 %0, %1, %2, 0 offen offset:%3"
                     : "=a"(af[i])
                     : "v"(qoff), "s"(rq), "i"(((i / KSUB) * 128 + (i % KSUB) * 8) * 2)
                     : "memory");
    }
    wave_sync();

    auto rsrc_b = [&](int tile) {
      const int col0 = tile * BN;
      return make_rsrc(a.cb + (int64_t)col0 * a.ldc, (int64_t)max(0, min(BN, a.N - col0)) * a.ldc * 2);
    };
    // one K-step's DMA: this wave's BPIECES pieces, plus (on a tile's first
    // step) its share of the tile's pre-filter factors
    auto stage = [&](int slot, __amdgpu_buffer_rsrc_t rb, int ks, int tile) {
      char *st = ring + slot * STAGE;
      const uint32_t soff = (uint32_t)ks * (uint32_t)KB;
#pragma unroll
      for (int i = 0; i < BPIECES; i++) dma16(rb, st + (i * NW + wid) * 1024, b_voff[i], soff);
      if (XFORM && ks == 0) {
        // 4 tile buffers: tile t - 1's columns are read until the end of
        // tile t, and tile t + 3's may already be in flight (KS == 1)
        const int col0 = tile * BN + wid * CV_PER_WAVE;
        const int64_t nb = (int64_t)max(0, min(CV_PER_WAVE, a.N - col0)) * 4;
        const __amdgpu_buffer_rsrc_t rc = make_rsrc(a.cpre + col0, nb);
        const int o = (tile & 3) * BN + wid * CV_PER_WAVE;
        // lanes past CV_PER_WAVE stay masked (an LDS-DMA writes one dword per
        // ACTIVE lane); vmcnt still counts one instruction per wave
        if (lane < CV_PER_WAVE)
          __builtin_amdgcn_raw_ptr_buffer_load_lds(rc, (LDS_AS void *)(cv_l + o), 4,
                                                   (uint32_t)(lane * 4), 0, 0, 0);
      }
    };

    // prologue: K-steps 0 .. nst-2 of the unit
    for (int j = 0; j < nst - 1; j++) stage(j, rsrc_b(t0 + j / KS), j % KS, t0 + j / KS);
    int sl = 0;  // ring slot of the current K-step

    // ---- pass 2: exact re-score of the LDS-queued survivors ----
    // Deferred: the queue (item = accumulator bits | (row-in-wave | global
    // column << 5) << 32) collects survivors across tiles and drains only when
    // it could overflow or at the unit's end, in full 64-item rounds; the
    // exact column norms come from global memory, one load per item.
    int qlen = 0;  // this wave's queued items (wave-uniform)
    auto drain = [&]() {
      st_q += (uint32_t)qlen;
      if (PMM_ABL(a.ablate) == 2 || qlen == 0) {
        qlen = 0;
        return;
      }
      const uint64_t tdr = timing ? __builtin_amdgcn_s_memtime() : 0;
      wave_sync();
      for (int base = 0; base < qlen; base += 64) {
        const int i = base + lane;
        if (i < qlen) {
          const u64 it = lq[i];
          const float v = __uint_as_float((uint32_t)it);
          const int rl = (int)((it >> 32) & 31u);
          const int gcol = (int)(it >> 37);
          const float sc =
              exact_score<METRIC>(v, XFORM ? qex_w[rl] : 0.0f, XFORM ? a.cn[gcol] : 0.0f);
          const uint32_t key = okey32(METRIC == kMetricEuclidean ? -sc : sc);
          const u64 comp = ((u64)key << 32) | (u64)(~(uint32_t)gcol);
          if (comp > thr_w[rl]) {
            const unsigned pos = atomicAdd(&cnt_w[rl], 1u);
            a.cand[((int64_t)(wrow0 + rl) * a.S + s) * a.capg + pos] = comp;
          }
        }
        // compact every row whose buffer could overflow on the next 64 appends
        wave_sync();
        const unsigned cval = (lane < 32) ? cnt_w[lane] : 0u;
        u64 need = __ballot(lane < 32 && cval > (unsigned)a.ctrig);
        if (need) {
          asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
          st_c += (uint32_t)__popcll(need);
          while (need) {
            const int r = __builtin_ctzll(need);
            need &= need - 1;
            compact_row(a, s, wrow0 + r, thr_w + r, cnt_w + r, scr, lane);
          }
          if (lane < 32) lo_w[lane] = prefilter_bound<METRIC>(thr_w[lane], qex_w[lane]);
          wave_sync();
        }
      }
      qlen = 0;
      if (timing) cy_drain += __builtin_amdgcn_s_memtime() - tdr;
    };

    // ---- survivors of tile pt (set pv, survivor words bits[]) -> pass 2 ----
    // Per column group with any survivor: the lanes holding one stage their
    // 16 accumulator values in LDS (a per-lane dynamic index into registers
    // would go through scratch), then every lane walks its own survivor bits
    // (bit 15 - e = row e) in a divergent loop, queueing one survivor per
    // round with ballot + mbcnt slots; the LDS queue drains whenever it could
    // overflow (a unit's first tiles).
    auto extract = [&](const f32x16 (&pv)[NB], int pt, uint32_t (&bits)[NB])
        __attribute__((always_inline)) {
#pragma unroll
      for (int c = 0; c < NB; c++) {
        uint32_t b = (pt * BN + 32 * c + r32 < a.N) ? bits[c] : 0u;  // columns past N
        if (__ballot(b != 0u) == 0ull) continue;
        if (b) {
#pragma unroll
          for (int q = 0; q < 4; q++)
            *(f32x4 *)(sbuf + 4 * q) =
                (f32x4){pv[c][4 * q], pv[c][4 * q + 1], pv[c][4 * q + 2], pv[c][4 * q + 3]};
        }
        for (;;) {
          const bool act = b != 0u;
          const u64 m = __ballot(act);
          if (m == 0ull) break;
          if (act && PMM_ABL(a.ablate) != 2) {
            const int j = 31 - __builtin_clz(b);  // bit j <-> row e = 15 - j
            b &= ~(1u << j);
            const int e = 15 - j;
            const float v = sbuf[e];
            const uint32_t hi = (uint32_t)(4 * h + (e & 3) + 8 * (e >> 2)) |
                                ((uint32_t)(pt * BN + 32 * c + r32) << 5);
            lq[qlen + lanes_below(m)] = (u64)__float_as_uint(v) | ((u64)hi << 32);
          } else if (act) {
            b &= b - 1u;
          }
          qlen += __popcll(m);
          if (qlen > QCAP - 64) drain();
        }
      }
      st_g++;
    };

    auto tile_consts = [&](int pt, float (&cv)[NB], float (&nlo)[16]) __attribute__((always_inline)) {
#pragma unroll
      for (int e = 0; e < 16; e++) nlo[e] = lo_w[acc_row(e, h)];
#pragma unroll
      for (int c = 0; c < NB; c++) cv[c] = XFORM ? cv_l[(pt & 3) * BN + 32 * c + r32] : 0.0f;
    };

    // One tile: K-loop into `acc`; its substeps also compute the survivor
    // words of the previous tile (set `pv`), extracted after the loop.
    auto tile_step = [&](f32x16 (&acc)[NB], const f32x16 (&pv)[NB], int tile, bool has_prev)
        __attribute__((always_inline)) {
      const uint64_t tts = timing ? __builtin_amdgcn_s_memtime() : 0;
      const int pt = tile - 1;
      float cv[NB], nlo[16];
      if (PIPE) tile_consts(pt, cv, nlo);  // (garbage for a unit's first tile: unused)
      uint32_t bits[NB];
#pragma unroll
      for (int c = 0; c < NB; c++) bits[c] = 0u;
      constexpr int NBQ = PF + 2;
      bf16x8 bq[NBQ][NB];
#pragma unroll
      for (int ks = 0; ks < KS; ks++) {
        // step (tile, ks) landed: only the DMAs of the nst - 2 younger steps
        // may still be in flight (a step's count: BPIECES, +1 on a tile's
        // first step for the pre-filter factors); ks is a constant after
        // unrolling, so the branches fold away
        const int x1 = (XFORM && (ks + 1) % KS == 0) ? 1 : 0;
        const int x2 = (XFORM && (ks + 2) % KS == 0) ? 1 : 0;
        if (nst == 4) {
          if (x1 + x2 == 2) wait_vm<2 * BPIECES + 2>();
          else if (x1 + x2 == 1) wait_vm<2 * BPIECES + 1>();
          else wait_vm<2 * BPIECES>();
        } else {
          if (x1) wait_vm<BPIECES + 1>();
          else wait_vm<BPIECES>();
        }
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
        const char *st = ring + sl * STAGE;
        // corpus fragments read PF substeps ahead of their MFMAs, into a
        // rotation of PF + 2 buffers indexed by the tile's substep number
#pragma unroll
        for (int p = 0; p < PF; p++)
#pragma unroll
          for (int c = 0; c < NB; c++)
            bq[(KSUB * ks + p) % NBQ][c] =
                *(const bf16x8 *)(st + b_rd + c * 32 * KB + 16 * ((8 * h + p) ^ swz));
        // the previous step's last MFMA group, held back from before the
        // barrier (its fragments are in registers): it covers the latency of
        // the reads just issued instead of the MFMA pipe idling behind them
        if (DEFER && ks > 0) {
#pragma unroll
          for (int c = 0; c < NB; c++)
            mfma_acc(acc[c], af[KSUB * ks - 1], bq[(KSUB * ks - 1) % NBQ][c]);
        }
#pragma unroll
        for (int sub = 0; sub < KSUB; sub++) {
          const int gs = KSUB * ks + sub;
          if (sub + PF < KSUB) {
            const int co = 16 * ((8 * h + sub + PF) ^ swz);
#pragma unroll
            for (int c = 0; c < NB; c++)
              bq[(gs + PF) % NBQ][c] = *(const bf16x8 *)(st + b_rd + c * 32 * KB + co);
          }
          if (!(DEFER && sub == KSUB - 1 && ks < KS - 1)) {
#pragma unroll
            for (int c = 0; c < NB; c++) {
              if (gs == 0) mfma_first(acc[c], af[0], bq[0][c]);
              else mfma_acc(acc[c], af[gs], bq[gs % NBQ][c]);
            }
          }
          if (sub == 0) {
            // step + nst - 1 goes out behind the first MFMA group, in one
            // burst (one DMA per substep measured 30% slower), into the slot
            // every wave finished reading before this step's barrier; past
            // the unit's last tile it is a harmless extra read (drained at
            // the unit's end)
            const int slj = (sl == 0) ? nst - 1 : sl - 1;
            constexpr int jj = nst - 1;
            const int adv = (ks + jj) / KS;  // tiles ahead of this one
            stage(slj, rsrc_b(tile + adv), (ks + jj) % KS, tile + adv);
          }
          // this substep's share of the previous tile's survivor test
          if constexpr (PIPE) {
            const int gidx = ks * KSUB + sub;
#pragma unroll
            for (int pidx = 0; pidx < 64; pidx++) {
              if (pidx < gidx * 64 / G || pidx >= (gidx + 1) * 64 / G) continue;
              const int c = pidx >> 4, e = pidx & 15;
              const float d = prefilter_diff<METRIC>(pv[c][e], cv[c], nlo[e]);
              bits[c] = (bits[c] << 1) | (uint32_t)!(d < 0.0f);
              // opaque use in place: without it LLVM sinks this loop-invariant
              // work below the K-loop (sched_barrier acts too late to stop it)
              asm volatile("" : "+v"(bits[c]));
            }
          }
          __builtin_amdgcn_sched_barrier(0);
        }
        sl = (sl == nst - 1) ? 0 : sl + 1;
      }
      mfma_drain(acc);
      const uint64_t tte = timing ? __builtin_amdgcn_s_memtime() : 0;
      if (timing) cy_loop += tte - tts;
      if (PIPE && has_prev && PMM_ABL(a.ablate) != 1) extract(pv, pt, bits);
      if (timing) cy_ext += __builtin_amdgcn_s_memtime() - tte;
    };

    // The unit's last tile: survivor words computed after its K-loop.
    auto tile_last = [&](const f32x16 (&pv)[NB], int pt) __attribute__((always_inline)) {
      float cv[NB], nlo[16];
      tile_consts(pt, cv, nlo);
      uint32_t bits[NB];
#pragma unroll
      for (int c = 0; c < NB; c++) {
        bits[c] = 0u;
#pragma unroll
        for (int e = 0; e < 16; e++) {
          const float d = prefilter_diff<METRIC>(pv[c][e], cv[c], nlo[e]);
          bits[c] = (bits[c] << 1) | (uint32_t)!(d < 0.0f);
        }
      }
      extract(pv, pt, bits);
    };

    if constexpr (PIPE) {
      f32x16 accA[NB], accB[NB];
#pragma unroll
      for (int c = 0; c < NB; c++) accB[c] = (f32x16){};
      for (int tile = t0; tile < t1; tile += 2) {
        tile_step(accA, accB, tile, tile > t0);
        if (tile + 1 < t1) tile_step(accB, accA, tile + 1, true);
      }
      if (PMM_ABL(a.ablate) != 1) {
        if (((t1 - 1 - t0) & 1) == 0) tile_last(accA, t1 - 1);
        else tile_last(accB, t1 - 1);
      }
    } else {
      f32x16 acc[NB];
      for (int tile = t0; tile < t1; tile++) {
        tile_step(acc, acc, tile, false);
        if (PMM_ABL(a.ablate) != 1) {
          const uint64_t tx = timing ? __builtin_amdgcn_s_memtime() : 0;
          tile_last(acc, tile);
          if (timing) cy_ext += __builtin_amdgcn_s_memtime() - tx;
        }
      }
    }
    drain();  // the unit's remaining survivors
    // the K-steps issued past the unit's last tile land before the ring is
    // reused by the next unit
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (lane < 32) {
      const int grow = wrow0 + lane;
      if (grow < a.M) a.cnt[(int64_t)grow * a.S + s] = cnt_w[lane];
    }
  }
  if (a.stats && lane == 0) {
    atomicAdd(a.stats + 0, (u64)st_q);
    atomicAdd(a.stats + 1, (u64)st_g);
    atomicAdd(a.stats + 3, (u64)st_c);
    atomicAdd(a.stats + 4, (u64)cy_loop);
    atomicAdd(a.stats + 5, (u64)(cy_ext - cy_drain));
    atomicAdd(a.stats + 6, (u64)cy_drain);
  }
}

template <int KS, int METRIC, int NST, int PF, int DEF>
static hipError_t launch_bf16_n(const GemmF32Args &a, int grid, size_t lds, hipStream_t s) {
  static bool attr_set = false;
  if (!attr_set) {
    hipError_t e = hipFuncSetAttribute((const void *)gemm_bf16_kernel<KS, METRIC, NST, PF, DEF>,
                                       hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    if (e != hipSuccess) return e;
    attr_set = true;
  }
  gemm_bf16_kernel<KS, METRIC, NST, PF, DEF><<<dim3(grid), dim3(NW * 64), lds, s>>>(a);
  return hipGetLastError();
}
template <int KS, int METRIC>
static hipError_t launch_bf16_t(const GemmF32Args &a, int grid, size_t lds, hipStream_t s) {
  // three ring slots: a fourth (measured at D = 768) gained nothing
  // fragment prefetch one substep ahead: two (measured on the same box) was
  // 0.6% slower
  if (a.defer) return launch_bf16_n<KS, METRIC, 3, 1, 1>(a, grid, lds, s);
  return launch_bf16_n<KS, METRIC, 3, 1, 0>(a, grid, lds, s);
}

template <int KS>
static hipError_t launch_bf16_m(const GemmF32Args &a, int grid, size_t lds, hipStream_t s) {
  if (a.metric == kMetricCosine) return launch_bf16_t<KS, kMetricCosine>(a, grid, lds, s);
  if (a.metric == kMetricDot) return launch_bf16_t<KS, kMetricDot>(a, grid, lds, s);
  return launch_bf16_t<KS, kMetricEuclidean>(a, grid, lds, s);
}


}  // namespace pmm
