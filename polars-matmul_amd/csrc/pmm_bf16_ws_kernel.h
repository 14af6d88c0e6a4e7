// pmm_bf16_ws_kernel.h -- wave-specialised bf16 fused GEMM + top-k kernel
// (PMM_COMPUTE_BF16; BASELINE configs[3]: 100k x 1M x 768 bf16 cosine k=100).
// Instantiated per padded-D step count by pmm_bf16_ks.hip; host side in
// pmm_bf16.hip.  bf16 operands, f32 accumulation on v_mfma_f32_16x16x32_bf16
// with K in natural order (PMM_WS_MFMA16, below; the fire-and-forget kernel
// runs the same chain and returns the same lists bit for bit), the f32
// path's metric epilogue, pre-filter, candidate buffers and merge.
//
// Why a second bf16 kernel: at one wave per SIMD (pmm_bf16_kernel.h) every
// latency of the top-k epilogue (LDS round trips, the survivors' exact
// re-score, candidate stores, compactions) stalls the matrix pipe: measured
// at 100k x 1M x 768 the epilogue adds 50% to the K-loop's time.  Here the
// work is split by role, two waves per SIMD:
//
//   * 4 MFMA waves (one per SIMD).  Wave w keeps its 32 query rows x D in
//     registers for a whole work unit (192 registers at D = 768) and streams
//     the corpus: per 64-column tile, KS K-steps of 128 bf16, each 8 substeps
//     of four v_mfma_f32_16x16x32_bf16 (two row blocks x two 16-column
//     blocks; 32x32x16 pairs before round 4) with the corpus fragments read
//     from LDS two substeps ahead (across K-step boundaries within a tile).
//     After a tile's K-loop it hands its 32 x 64 f32 accumulators to LDS (8
//     ds_write_b128, in the 32x32 accumulator layout the epilogue reads) and
//     starts the next tile.
//     No global memory traffic and no epilogue in this role.
//   * 4 epilogue waves (one per SIMD).  Wave 4 + w owns wave w's 32 rows:
//     their top-k state (threshold, candidate counts, LDS) has one owner.
//     It issues the corpus LDS-DMA for the ring (taking the DMA issue cost off
//     the MFMA waves) and, while the MFMA waves compute tile t, runs the
//     pre-filter, the exact re-score of the survivors, the candidate appends
//     and compactions of tile t - 1.
//
// Synchronisation: every wave of the workgroup executes the same number of
// s_barriers (the two roles run separate loops with equal trip counts; the
// per-unit barriers are outside the role branches).  Barrier B_g opens corpus
// K-step g (ring slot g % NST): before it the epilogue waves have waited
// (counted vmcnt) for the DMA of steps g and g + 1, and the MFMA waves have
// retired their LDS reads of step g - 1 (counted lgkmcnt: the reads of step
// g's first substeps, issued during step g - 1, may stay in flight), so after
// it step g + NST - 1 may be DMA'd into step g - 1's slot.  A tile's
// accumulators are written before the barrier opening the next tile and read
// by the epilogue waves after it (double-buffered: tile t + 2 reuses tile t's
// buffer, written after the epilogue waves have passed the barriers of tile t
// + 1, by which point they finished with tile t).  The pre-filter column
// factors and column norms of a tile ride with the tile's first K-step into
// an 8-tile LDS ring.
#pragma once
#include "pmm_device.h"

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace pmm {

namespace ws {
typedef __attribute__((__vector_size__(8 * sizeof(__bf16)))) __bf16 bf16x8;

constexpr int NWM = 4;                       // MFMA waves (1 per SIMD)
constexpr int NWE = 4;                       // epilogue waves (1 per SIMD)
constexpr int NTH = (NWM + NWE) * 64;
constexpr int BM = 32 * NWM;                 // query rows per workgroup
constexpr int BN = kBf16WsBN;                // corpus columns per tile
constexpr int NB = BN / 32;                  // 32x32 accumulators per MFMA wave
constexpr int KB = 256;                      // bytes of a row per K-step (128 bf16)
constexpr int KSUB = KB / 32;                // MFMA substeps (K = 16) per K-step
constexpr int PF = 2;                        // corpus fragments read PF substeps ahead
constexpr int STAGE = BN * KB;               // one K-step of one tile
constexpr int P = STAGE / 1024 / NWE;        // 1 KiB DMA pieces per epilogue wave per step
constexpr int CVT = 8;                       // tiles in the column-factor ring
constexpr int HAND = 32 * BN * 4;            // accumulator hand-off per wave per tile
// LDS carve
constexpr int OFF_THR = 0;
constexpr int OFF_CNT = OFF_THR + BM * 8;
constexpr int OFF_QEX = OFF_CNT + BM * 4;
constexpr int OFF_LO = OFF_QEX + BM * 4;
constexpr int OFF_UNIT = OFF_LO + BM * 4;
constexpr int OFF_CVR = (OFF_UNIT + 16 + 255) & ~255;   // pre-filter factors [CVT][BN]
constexpr int OFF_CNR = OFF_CVR + CVT * BN * 4;          // column norms [CVT][BN]
constexpr int OFF_HAND = (OFF_CNR + CVT * BN * 4 + 255) & ~255;  // [NHB][NWM][HAND]
#ifndef PMM_WS_QCAP
#define PMM_WS_QCAP 256
#endif
constexpr int QCAP = PMM_WS_QCAP;            // survivor queue per epilogue wave
// The rest of the carve depends on the K-steps per tile.  With KS >= 3 the
// epilogue waves are done with tile t's accumulators (read in the first two
// intervals of tile t + 1) before the MFMA waves write tile t + 1's (after
// the last barrier of tile t + 1), so one hand-off buffer suffices and its
// 32 KiB go to the corpus ring: 7 slots = the step being read, the next
// (landed: its first fragments are read ahead) and 4 K-steps (64 KiB) in
// flight per CU, which the L2 / MALL latency needs at ~55 GB/s per CU.
// (Measured at c4 before the cross-step fragment reads: 5 steps in flight
// instead of 4 changed nothing, so the stream is bound by bandwidth, not by
// the bytes in flight.)  The selection-based compaction (capg <=
// kBf16WsMaxCapg) needs no LDS scratch, which leaves room for the 7th slot.
#ifndef PMM_WS_EPI_SPACING
#define PMM_WS_EPI_SPACING 2  // (A/B: intervals between the epilogue's column groups, KS >= 6)
#endif
#ifndef PMM_WS_DRAIN_INTERVAL
#define PMM_WS_DRAIN_INTERVAL -1  // (A/B: interval of the periodic drain; -1 = the schedule's)
#endif
#ifndef PMM_WS_EPI_OFFSET
#define PMM_WS_EPI_OFFSET -1  // (A/B: -1 = by K steps (2 at KS >= 6, else 1); 0 = from the first interval)
#endif
#ifndef PMM_WS_DRAIN_TILES
#define PMM_WS_DRAIN_TILES 4  // (the survivor drain period; see drain_tiles below)
#endif
static_assert(PMM_WS_DRAIN_TILES >= 1, "survivor drain period");
// A survivor of tile x is queued during tile x + 1 and re-scored with its
// column norm from the CVT-tile ring, whose slot x is overwritten by the DMA
// of tile x + CVT.  By the drain interval of tile D the DMA has reached tile
// D + lead, lead = (drain interval + NST - 1) / KS: 2 or 3 tiles at KS >= 2,
// but 4 at KS = 1 (one K-step per tile).  So the drain period P needs
// P + lead < CVT: at KS = 1 the period 4 let the ring overwrite queued
// survivors' norms (wrong cosine / euclidean scores at padded D = 128; found
// by the bit-equality tests against the 256-row kernel) -- 2 there.
template <int KS>
constexpr int drain_tiles() { return KS == 1 ? (PMM_WS_DRAIN_TILES < 2 ? PMM_WS_DRAIN_TILES : 2) : PMM_WS_DRAIN_TILES; }
#ifndef PMM_WS_NST
#define PMM_WS_NST 7  // (A/B override: -DPMM_WS_NST=n)
#endif
#ifndef PMM_WS_QPS
// 1: survivors queued by a per-group wave prefix sum of the lanes' counts
// (see the epilogue); 0 (default): one ballot round per survivor per lane.
// Measured at c4 (round 5, lab builds alternated twice on one box,
// profiles/r5_c4/qps_ab.txt): 173.3 / 173.4 ms per launch against 137.3 /
// 137.4.  The sixteen per-score appends compile to sixteen VALU compare ->
// exec mask -> branch chains per group (the pattern round 4 measured in
// another form), while a group's survivors are few: the ballot loop runs
// one or two rounds.  Kept as an A/B switch (make lab LAB=-DPMM_WS_QPS=1).
#define PMM_WS_QPS 0
#endif
#ifndef PMM_WS_MFMA16
// 1: the MFMA waves (and the seed) on v_mfma_f32_16x16x32_bf16 (default);
// 0: on v_mfma_f32_32x32x16_bf16 with the K permuted inside each 128-wide
// step (rounds 1-3).  c4 A/B, alternated on one box (profiles/r4_ws16/):
// 143.0 / 142.9 vs 150.5 / 151.1 ms per kernel launch.
#define PMM_WS_MFMA16 1
#endif
template <int KS>
struct Carve {
  static constexpr int NHB = KS >= 3 ? 1 : 2;              // hand-off buffers
  static constexpr int NST = KS >= 3 ? PMM_WS_NST : 5;     // corpus ring slots
  static constexpr int OFF_RING = OFF_HAND + NHB * NWM * HAND;
  static constexpr int QC = KS >= 3 ? QCAP : 256;          // survivor queue entries per wave
  static constexpr int OFF_QUEUE = OFF_RING + NST * STAGE;  // [NWE][QC] u64
  static constexpr int BYTES = OFF_QUEUE + NWE * QC * 8;
  static_assert(BYTES <= 160 * 1024, "LDS carve");
  // When NST divides KS the slot sequence repeats every tile, so the slot at
  // a tile's start is loop-invariant; left visible, hipcc hoisted every
  // K-step's ring addresses out of the tile loop, ran out of VGPRs and
  // spilled inside the MFMA loop (592 B per lane at NST = KS = 6).  Its spill
  // and reload code is not padded for the inline-asm MFMAs it cannot see
  // (stale accumulators and fragments: wrong scores, 2.6x slower).  The
  // kernel makes the slot opaque per tile in that case (SLOT_REPEATS);
  // tests/test_kernel_resources.py keeps spill code out of the MFMA loops.
  static constexpr bool SLOT_REPEATS = KS % NST == 0;
  static_assert(OFF_RING % 256 == 0 && STAGE % 1024 == 0, "LDS carve alignment");
};
static_assert(P * NWE * 1024 == STAGE, "a K-step splits into whole 1 KiB pieces per wave");
static_assert(BN / NWE <= 64, "one column-factor DMA per epilogue wave covers its share");

// DMA instructions an epilogue wave issues for one K-step (corpus pieces, plus
// the pre-filter factors and norms of the tile on its first step)
template <bool XFORM>
constexpr int step_dmas(int ks) { return P + ((XFORM && ks == 0) ? 2 : 0); }

template <int N>
__device__ __forceinline__ void wait_vm() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}
// the same with a count that is constant after unrolling (folds to one wait)
__device__ __forceinline__ void wait_vm_n(int n) {
  switch (n) {
#define PMM_WCASE(N) \
  case N: wait_vm<N>(); break;
    PMM_WCASE(2) PMM_WCASE(4) PMM_WCASE(6) PMM_WCASE(8) PMM_WCASE(10) PMM_WCASE(12)
    PMM_WCASE(14) PMM_WCASE(16) PMM_WCASE(18) PMM_WCASE(20) PMM_WCASE(22) PMM_WCASE(24)
    PMM_WCASE(26) PMM_WCASE(28) PMM_WCASE(30)
#undef PMM_WCASE
    default: wait_vm<0>(); break;  // (never taken; safe)
  }
}
__device__ __forceinline__ void wait_lgkm0() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }
template <int N>
__device__ __forceinline__ void wait_lgkm() {
  asm volatile("s_waitcnt lgkmcnt(%0)" ::"n"(N) : "memory");
}
// LDS fetch-and-increment in asm: hipcc waits vmcnt(0) before any LDS write
// it sees while an LDS-DMA is in flight (it cannot tell the ring from the
// counters), which would stall the epilogue wave on the ring's next K-steps
__device__ __forceinline__ unsigned lds_inc(unsigned *p) {
  unsigned r;
  const uint32_t ad = (uint32_t)(size_t)(LDS_AS unsigned *)p;
  asm volatile("ds_add_rtn_u32 %0, %1, %2\n\ts_waitcnt lgkmcnt(0)" : "=v"(r) : "v"(ad), "v"(1u) : "memory");
  return r;
}
__device__ __forceinline__ void barrier() {
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

// MFMA with A (query fragment) from AGPRs and the accumulator in VGPRs (see
// pmm_bf16_kernel.h for the hazard rules hipcc does not apply inside asm).
__device__ __forceinline__ void mfma_acc(f32x16 &c, const bf16x8 &a, const bf16x8 &b) {
  asm volatile("v_mfma_f32_32x32x16_bf16 %0, %1, %2, %0" : "+v"(c) : "v"(a), "v"(b) : "memory");
}
__device__ __forceinline__ void mfma_first(f32x16 &c, const bf16x8 &a, const bf16x8 &b) {
  asm volatile("v_mfma_f32_32x32x16_bf16 %0, %1, %2, 0" : "=&v"(c) : "v"(a), "v"(b) : "memory");
}
__device__ __forceinline__ void mfma_drain(f32x16 (&acc)[NB]) {
  asm volatile("s_nop 7\n\ts_nop 4" : "+v"(acc[0]), "+v"(acc[NB - 1]));
#pragma unroll
  for (int c = 1; c < NB - 1; c++) asm volatile("" : "+v"(acc[c]));
}
// The 16x16x32 form (PMM_WS_MFMA16): the MFMA waves' 32 x 64 block as 2 x 4
// accumulators of 16 x 16, each K step of 32 in natural order (lane group g
// of 16 lanes carries k 8g .. 8g + 7).  Same cycles per flop as 32x32x16 on
// one SIMD; MI355X_MICROARCH.md measured bare loops of this shape at ~1.15x
// the FLOP/s of the 32x32x16 form on random data (the chip holds a higher
// clock on it).
__device__ __forceinline__ void mfma16_acc(f32x4 &c, const bf16x8 &a, const bf16x8 &b) {
  asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+v"(c) : "v"(a), "v"(b) : "memory");
}
__device__ __forceinline__ void mfma16_first(f32x4 &c, const bf16x8 &a, const bf16x8 &b) {
  asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, 0" : "=&v"(c) : "v"(a), "v"(b) : "memory");
}
__device__ __forceinline__ void mfma16_drain(f32x4 (&acc)[2][2 * NB]) {
  asm volatile("s_nop 7\n\ts_nop 4" : "+v"(acc[0][0]), "+v"(acc[1][2 * NB - 1]));
#pragma unroll
  for (int i = 1; i < 4 * NB - 1; i++) asm volatile("" : "+v"(acc[i / (2 * NB)][i % (2 * NB)]));
}
}  // namespace ws

// Round barrier across the grid (speed only, bounded spin): the workgroups
// of an XCD stream the same corpus tiles together.  Two __syncthreads, in
// every wave of the workgroup; thread 0 (an MFMA wave) spins.
__device__ __forceinline__ void round_sync(const GemmF32Args &a, unsigned target, int tid,
                                           bool &sync_on, int *unit_l) {
  if (!sync_on) return;
  if (tid == 0) {
    unsigned *round_bar = a.counter + 32;
    atomicAdd(round_bar, 1u);
    const uint64_t tstart = wall_clock64();
    int ok = 1;
    while (__hip_atomic_fetch_add(round_bar, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) <
           target) {
      __builtin_amdgcn_s_sleep(8);
      if (wall_clock64() - tstart > (uint64_t)a.sync_timeout) {
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

// Unit schedule.  Phase A: the first qb_full query blocks (a multiple of the
// grid) are processed whole by one workgroup each, split by split in rounds
// (round r: block (r / S) * grid + blockIdx.x, split r % S), so a row's
// threshold and candidate buffer carry over from split to split (one
// continuous top-k stream per row: about k ln(N / k) survivors instead of ~k
// per split on top of a cold first split), while every workgroup of a round
// still streams the same split (shared through the XCD's L2).  Phase B: the
// remaining query blocks as independent (block, split) units, split-major,
// each with its own candidate segment, seeded from the shared thresholds.
struct UnitPos {
  int qb, s, seg;     // query block, corpus split, candidate segment
  bool first, last;   // first / last unit of the row state's run
  unsigned target;    // round-barrier arrivals through this round
};
__device__ __forceinline__ bool unit_at(const GemmF32Args &a, int round, UnitPos &u) {
  const int G = (int)gridDim.x;
  const int rA = a.qb_full / G * a.S;
  if (round < rA) {
    u.qb = (round / a.S) * G + (int)blockIdx.x;
    u.s = round % a.S;
    u.seg = 0;
    u.first = u.s == 0;
    u.last = u.s == a.S - 1;
    u.target = (unsigned)((round + 1) * G);
    return true;
  }
  const int qbb = a.QB - a.qb_full;
  const int nb = qbb * a.S;
  const int idx = (round - rA) * G + (int)blockIdx.x;
  if (idx >= nb) return false;
  u.s = idx / qbb;
  u.qb = a.qb_full + (idx - u.s * qbb);
  u.seg = u.s;
  u.first = u.last = true;
  u.target = (unsigned)(rA * G + min((round - rA + 1) * G, nb));
  return true;
}

// ===========================================================================
// KS = padded D / 128 (K-steps per tile).
// ===========================================================================
template <int KS, int METRIC>
__global__ __launch_bounds__(ws::NTH, 1) void gemm_bf16_ws_kernel(GemmF32Args a) {
  using namespace ws;
  using C = Carve<KS>;
  constexpr int NST = C::NST, NHB = C::NHB;
  static_assert(drain_tiles<KS>() + (KS == 1 ? 4 : 3) < CVT, "queued survivors' column norms must stay in the ring");
  extern __shared__ __attribute__((aligned(16))) char smem[];
  int *unit_l = (int *)(smem + OFF_UNIT);
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const bool is_mfma = wid < NWM;
  const int rw = is_mfma ? wid : wid - NWM;  // row group (32 rows) of this wave
  const int r32 = lane & 31, h = lane >> 5;
  constexpr bool XFORM = (METRIC != kMetricDot);
  char *ring = smem + C::OFF_RING;

  // The two roles run separate unit loops (identical trip counts and barrier
  // sequences), so each role's loop-invariant values stay out of the other's
  // registers.
  bool sync_on = a.round_sync != 0;
  // PMM_STATS: shader cycles per phase, per wave (a diagnostic build path;
  // off, the memtime reads are skipped on a wave-uniform branch)
#ifdef PMM_WS_STATS
  const bool timing = a.stats != nullptr;
#else
  constexpr bool timing = false;  // (build with -DPMM_WS_STATS for the cycle stats)
#endif
  const uint64_t t_start = timing ? __builtin_amdgcn_s_memtime() : 0;
  uint64_t cy0 = 0, cy1 = 0, cy2 = 0, cy3 = 0, nq = 0, cy4 = 0, cy5 = 0, cy6 = 0, ncomp = 0;
  auto stamp = [&]() __attribute__((always_inline)) { return timing ? __builtin_amdgcn_s_memtime() : 0; };
  if (is_mfma) {
  bf16x8 af[KSUB * KS];  // this wave's query rows, kept across a run's units
  for (int round = 0;; round++) {
    UnitPos u;
    if (!unit_at(a, round, u)) break;
    round_sync(a, u.target, tid, sync_on, unit_l);
    const int t0 = u.s * a.tps;
    const int t1 = min(t0 + a.tps, a.ntiles);
    const int wrow0 = u.qb * BM + rw * 32;
      // ================= MFMA role =================
      if (u.first) {
        const __amdgpu_buffer_rsrc_t rq = make_rsrc(
            a.qb + (int64_t)wrow0 * a.ldq, (int64_t)max(0, min(32, a.M - wrow0)) * a.ldq * 2);
        const uint32_t qoff = (uint32_t)(r32 * a.ldq * 2 + 128 * h);
        // the descriptor may be fresh from a VALU write (readfirstlane):
        // 5 wait states before a VMEM instruction reads it (hipcc pads
        // nothing in front of an asm statement)
#if PMM_WS_MFMA16
        // fragment i = 8 ks + 2 j + rb: rows 16 rb + (lane & 15), k 128 ks +
        // 32 j + 8 (lane >> 4) .. + 7 (the row block in the scalar offset,
        // which gets the same 5 wait states as the descriptor)
        const uint32_t qoff16 = (uint32_t)((lane & 15) * a.ldq * 2 + 16 * (lane >> 4));
        const uint32_t rbo = __builtin_amdgcn_readfirstlane((uint32_t)(16 * a.ldq * 2));
        asm volatile("s_nop 4" ::"s"(rq), "s"(rbo));
#pragma unroll
        for (int i = 0; i < KSUB * KS; i++)
          asm volatile("buffer_load_dwordx4 %0, %1, %2, %3 offen offset:%4"
                       : "=v"(af[i])
                       : "v"(qoff16), "s"(rq), "s"((i & 1) ? rbo : 0u), "i"(((i / KSUB) * 128 + ((i % KSUB) / 2) * 32) * 2)
                       : "memory");
        (void)qoff;
#else
        asm volatile("s_nop 4" ::"s"(rq));
#pragma unroll
        for (int i = 0; i < KSUB * KS; i++)
          asm volatile("buffer_load_dwordx4 %0, %1, %2, 0 offen offset:%3"
                       : "=v"(af[i])
                       : "v"(qoff), "s"(rq), "i"(((i / KSUB) * 128 + (i % KSUB) * 8) * 2)
                       : "memory");
#endif
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
      // LDS byte address of this lane's fragment chunk: column r32 of a group
      // at r32 * KB, chunk (8h + sub) stored at chunk (8h + sub) ^ (r32 & 15);
      // since 8h + sub = 8h ^ sub (sub < 8), substep sub's address is the
      // sub-0 address XOR (sub << 4): one v_xor per substep, no per-substep
      // address registers (the A rows leave ~60 VGPRs for everything else)
#if PMM_WS_MFMA16
      // 16x16x32 form: substep sub = half-step (j = sub / 2: k 32 j .. 32 j +
      // 31 of the K-step; half = sub % 2: column blocks 2 half, 2 half + 1);
      // lane (c16, g) reads chunk 4 j + g of column 16 cb + c16, stored at
      // chunk (4 j + g) ^ c16 = (g ^ c16) ^ 4 j: the lane's sub-0 address
      // XOR (j << 6), plus 16 cb columns
      const int c16 = lane & 15, g4 = lane >> 4;
      const uint32_t lane_off = (uint32_t)(c16 * KB + 16 * (g4 ^ c16));
#else
      const uint32_t lane_off = (uint32_t)(r32 * KB + 16 * ((8 * h) ^ (r32 & 15)));
#endif
      const uint32_t ring_lds = (uint32_t)(size_t)(LDS_AS char *)ring;
      int sl = 0;
      for (int tile = t0; tile < t1; tile++) {
        if constexpr (C::SLOT_REPEATS) asm volatile("" : "+s"(sl));  // (see Carve)
#if PMM_WS_MFMA16
        f32x4 acc[2][2 * NB];  // [row block][column block of 16]
#else
        f32x16 acc[NB];
#endif
        bf16x8 bq[PF + 1][NB];  // fragment sets: PF in flight + the one in use
#pragma unroll
        for (int ks = 0; ks < KS; ks++) {
          const int g0 = KSUB * ks;
          const int sn = (sl == NST - 1) ? 0 : sl + 1;
          // reads of the previous slot (and the hand-off writes) retired; the
          // PF groups prefetched from this slot may stay in flight
          if (ks == 0) wait_lgkm0();
          else wait_lgkm<PF * NB>();
          barrier();     // B_g: steps g and g + 1 landed
          uint32_t sbase = ring_lds + (uint32_t)(sl * STAGE) + lane_off;
          asm volatile("" : "+v"(sbase));  // keep the per-substep XORs in the loop
          auto rd = [&](uint32_t base, int sub, int set) __attribute__((always_inline)) {
#ifdef PMM_WS_NOFRAG
            return;  // diagnostic build only: MFMAs on stale fragments, no LDS reads
#endif
#if PMM_WS_MFMA16
            const uint32_t ad = (base ^ (uint32_t)((sub >> 1) << 6)) + (uint32_t)((sub & 1) * 2 * 16 * KB);
#pragma unroll
            for (int c = 0; c < NB; c++) bq[set][c] = *(const LDS_AS bf16x8 *)(size_t)(ad + c * 16 * KB);
#else
            const uint32_t ad = base ^ (uint32_t)(sub << 4);
#pragma unroll
            for (int c = 0; c < NB; c++) bq[set][c] = *(const LDS_AS bf16x8 *)(size_t)(ad + c * 32 * KB);
#endif
          };
          // fragments stream PF substeps ahead across the K-steps of a tile:
          // step g + 1's slot landed before B_g, so its first PF substeps are
          // read during step g and the barrier costs no read latency
          uint32_t nbase = ring_lds + (uint32_t)(sn * STAGE) + lane_off;
          asm volatile("" : "+v"(nbase));
          if (ks == 0) {
#pragma unroll
            for (int p = 0; p < PF; p++) rd(sbase, p, p % (PF + 1));
          }
#pragma unroll
          for (int sub = 0; sub < KSUB; sub++) {
            const int gs = g0 + sub;
            if (sub + PF < KSUB) rd(sbase, sub + PF, (gs + PF) % (PF + 1));
            else if (ks < KS - 1) rd(nbase, sub + PF - KSUB, (gs + PF) % (PF + 1));
#if PMM_WS_MFMA16
            {
              const int j = sub >> 1, half = sub & 1;
#pragma unroll
              for (int rb = 0; rb < 2; rb++)
#pragma unroll
                for (int c = 0; c < NB; c++) {
                  const bf16x8 &A = af[KSUB * ks + 2 * j + rb];
                  if (ks == 0 && j == 0) mfma16_first(acc[rb][2 * half + c], A, bq[gs % (PF + 1)][c]);
                  else mfma16_acc(acc[rb][2 * half + c], A, bq[gs % (PF + 1)][c]);
                }
            }
#else
#pragma unroll
            for (int c = 0; c < NB; c++) {
              if (gs == 0) mfma_first(acc[c], af[0], bq[0][c]);
              else mfma_acc(acc[c], af[gs], bq[gs % (PF + 1)][c]);
            }
#endif
            __builtin_amdgcn_sched_barrier(0);
          }
          sl = sn;
        }
        // hand the tile to the epilogue wave of these rows
        char *hb = smem + OFF_HAND + ((tile % NHB) * NWM + rw) * HAND;
#if PMM_WS_MFMA16
        mfma16_drain(acc);
        // in the 32x32 accumulator layout the epilogue reads: the 4-row group
        // 16 rb + 4 g of column 16 cb + c16 is f32x4 (column block cb / 2,
        // q = 2 rb + g / 2) of lane 16 (cb % 2) + c16 + 32 (g % 2)
        // (one lane address, the rest immediate offsets; kept opaque so hipcc
        // does not hoist eight addresses out of the tile loop)
        uint32_t hl = (uint32_t)(size_t)(LDS_AS char *)hb + (uint32_t)(((g4 >> 1) * 64 + c16 + 32 * (g4 & 1)) * 16);
        asm volatile("" : "+v"(hl));
#pragma unroll
        for (int rb = 0; rb < 2; rb++)
#pragma unroll
          for (int cb = 0; cb < 2 * NB; cb++)
            *(LDS_AS f32x4 *)(size_t)(hl + (uint32_t)((((cb >> 1) * 4 + 2 * rb) * 64 + 16 * (cb & 1)) * 16)) =
                acc[rb][cb];
#else
        mfma_drain(acc);
#pragma unroll
        for (int c = 0; c < NB; c++)
#pragma unroll
          for (int q = 0; q < 4; q++)
            *(f32x4 *)(hb + ((c * 4 + q) * 64 + lane) * 16) =
                (f32x4){acc[c][4 * q], acc[c][4 * q + 1], acc[c][4 * q + 2], acc[c][4 * q + 3]};
#endif
      }
      // the epilogue waves' last tile: two more barriers
      wait_lgkm0();
      barrier();
      barrier();
    }
  } else {
  for (int round = 0;; round++) {
    UnitPos u;
    if (!unit_at(a, round, u)) break;
    round_sync(a, u.target, tid, sync_on, unit_l);
    const int s = u.seg;  // candidate segment of this unit's rows
    const int t0 = u.s * a.tps;
    const int t1 = min(t0 + a.tps, a.ntiles);
    const int wrow0 = u.qb * BM + rw * 32;
      // ================= epilogue role =================
      u64 *thr_w = (u64 *)(smem + OFF_THR) + rw * 32;
      unsigned *cnt_w = (unsigned *)(smem + OFF_CNT) + rw * 32;
      float *qex_w = (float *)(smem + OFF_QEX) + rw * 32;
      float *lo_w = (float *)(smem + OFF_LO) + rw * 32;
      float *cvr = (float *)(smem + OFF_CVR);
      float *cnr = (float *)(smem + OFF_CNR);
      if (u.first && lane < 32) {
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
      wave_sync();
      float lo[16];
      auto load_lo = [&]() __attribute__((always_inline)) {
#pragma unroll
        for (int e = 0; e < 16; e++) lo[e] = lo_w[acc_row(e, h)];
      };
      load_lo();

      // loop-invariant per-lane source offsets of this wave's corpus pieces:
      // piece i = 4 tile columns x 256 B; chunk ch of column col lands in LDS
      // chunk ch ^ (col & 15) (conflict-free ds_read_b128 fragment reads)
      uint32_t b_voff[P];
#pragma unroll
      for (int i = 0; i < P; i++) {
        const int col = (i * NWE + rw) * 4 + (lane >> 4);
        const int ch = (lane & 15) ^ (col & 15);
        b_voff[i] = (uint32_t)(col * a.ldc * 2 + ch * 16);
      }
      // one K-step's DMA: corpus pieces into ring slot `slot`, plus on a
      // tile's first step this wave's share of its column factors / norms
      auto stage = [&](int slot, int tile, int ks) __attribute__((always_inline)) {
        if (PMM_ABL(a.ablate) == 3) return;  // benchmarking only: no corpus traffic at all
        const int col0 = tile * BN;
        const __amdgpu_buffer_rsrc_t rb =
            make_rsrc(a.cb + (int64_t)col0 * a.ldc, (int64_t)max(0, min(BN, a.N - col0)) * a.ldc * 2);
        char *st = ring + slot * STAGE;
        const uint32_t soff = (uint32_t)ks * (uint32_t)KB;
#pragma unroll
        for (int i = 0; i < P; i++) dma16(rb, st + (i * NWE + rw) * 1024, b_voff[i], soff);
        if (XFORM && ks == 0) {
          constexpr int PER = BN / NWE;
          const int c0 = col0 + rw * PER;
          const int64_t nb = (int64_t)max(0, min(PER, a.N - c0)) * 4;
          const __amdgpu_buffer_rsrc_t rc = make_rsrc(a.cpre + c0, nb);
          const __amdgpu_buffer_rsrc_t rn = make_rsrc(a.cn + c0, nb);
          const int o = (tile & (CVT - 1)) * BN + rw * PER;
          if (lane < PER) {
            __builtin_amdgcn_raw_ptr_buffer_load_lds(rc, (LDS_AS void *)(cvr + o), 4,
                                                     (uint32_t)(lane * 4), 0, 0, 0);
            __builtin_amdgcn_raw_ptr_buffer_load_lds(rn, (LDS_AS void *)(cnr + o), 4,
                                                     (uint32_t)(lane * 4), 0, 0, 0);
          }
        }
      };

      // Survivor queue (LDS, per wave): item = accumulator bits | (row in
      // wave | global column << 5) << 32.  Survivors are re-scored exactly
      // in 64-wide rounds (one item per lane) when the queue could overflow,
      // every 4 tiles (the column-norm ring holds the last 8) and at the
      // unit's end.  Queue writes are asm: hipcc would wait for the in-flight
      // ring DMAs before every LDS store it sees.
      constexpr int QCAP = C::QC;
      const uint32_t lq_lds = (uint32_t)(size_t)(LDS_AS char *)(smem + C::OFF_QUEUE) + rw * QCAP * 8;
      const u64 *lq = (const u64 *)(smem + C::OFF_QUEUE) + rw * QCAP;
      int qlen = 0;  // wave-uniform
      // A split unit (phase B) shares its rows with the other splits' units:
      // their compactions raise the rows' shared thresholds (gthr) while this
      // unit runs, so every drain re-reads them (relaxed, agent scope: any
      // value read is some unit's k-th best of its own segment, a lower bound
      // of the row's final k-th) and prunes with the larger bound.  The load
      // is issued at the drain's start and consumed at its end.
      const bool split_unit = u.first && u.last && a.S > 1;
      auto drain = [&]() __attribute__((always_inline)) {
        const uint64_t td0 = stamp();
        if (timing) nq += (uint64_t)qlen;
        u64 gt = 0ull;
        if (split_unit && lane < 32 && wrow0 + lane < a.M)
          gt = __hip_atomic_load(a.gthr + wrow0 + lane, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        for (int base = 0; base < qlen; base += 64) {
          const int i = base + lane;
          if (i < qlen) {
            const u64 it = lq[i];
            const float v = __uint_as_float((uint32_t)it);
            const int rl = (int)((it >> 32) & 31u);
            const int gcol = (int)(it >> 37);
            const float cnv = XFORM ? cnr[((gcol / BN) & (CVT - 1)) * BN + (gcol % BN)] : 0.0f;
            const float sc = exact_score<METRIC>(v, XFORM ? qex_w[rl] : 0.0f, cnv);
            const uint32_t key = okey32(METRIC == kMetricEuclidean ? -sc : sc);
            const u64 comp = ((u64)key << 32) | (u64)(~(uint32_t)gcol);
            if (comp > thr_w[rl]) {
              const unsigned pos = lds_inc(&cnt_w[rl]);
              a.cand[((int64_t)(wrow0 + rl) * a.S + s) * a.capg + pos] = comp;
            }
          }
          // a round adds at most 64 per row: compact every row that could
          // overflow on the next round
          wave_sync();
          const unsigned cval = (lane < 32) ? cnt_w[lane] : 0u;
          u64 need = __ballot(lane < 32 && cval > (unsigned)a.ctrig);
          if (need) {
            const uint64_t tc0 = stamp();
            if (timing) ncomp += (uint64_t)__popcll(need);
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            while (need) {
              const int r = __builtin_ctzll(need);
              need &= need - 1;
              // (capg <= 512: compact_row's selection path, no LDS scratch)
              compact_row(a, s, wrow0 + r, thr_w + r, cnt_w + r, nullptr, lane);
            }
            if (lane < 32) lo_w[lane] = prefilter_bound<METRIC>(thr_w[lane], qex_w[lane]);
            wave_sync();
            load_lo();
            if (timing) cy4 += stamp() - tc0;
          }
        }
        if (split_unit) {
          if (lane < 32 && gt > thr_w[lane]) {
            thr_w[lane] = gt;
            lo_w[lane] = prefilter_bound<METRIC>(gt, qex_w[lane]);
          }
          wave_sync();
          load_lo();
        }
        qlen = 0;
        if (timing) cy6 += stamp() - td0;
      };

      // epilogue of column group c of tile pt (accumulators in hand-off
      // buffer pt & 1): the pre-filter difference of every score, their
      // NaN-propagating max per lane, and only if some lane's max passes,
      // the per-score survivor bits and their queueing
      auto epilogue = [&](int pt, int c) __attribute__((always_inline)) {
        const char *hb = smem + OFF_HAND + ((pt % NHB) * NWM + rw) * HAND;
        f32x4 v4[4];
#pragma unroll
        for (int q = 0; q < 4; q++) v4[q] = *(const f32x4 *)(hb + ((c * 4 + q) * 64 + lane) * 16);
        const int tc = 32 * c + r32;
        const int gcol = pt * BN + tc;
        if (PMM_ABL(a.ablate) & 32) {  // benchmarking only: the hand-off reads, nothing else
          asm volatile("" ::"v"(v4[0]), "v"(v4[1]), "v"(v4[2]), "v"(v4[3]));
          return;
        }
        const float cv = XFORM ? cvr[(pt & (CVT - 1)) * BN + tc] : 0.0f;
        float d[16];
#pragma unroll
        for (int e = 0; e < 16; e++) d[e] = prefilter_diff<METRIC>(v4[e >> 2][e & 3], cv, lo[e]);
        float dm = d[0];
#pragma unroll
        for (int e = 1; e < 16; e++) dm = __builtin_elementwise_maximum(dm, d[e]);
        const bool any = !(dm < 0.0f) && gcol < a.N;
        if (__ballot(any) == 0ull || (PMM_ABL(a.ablate) & 8)) return;  // (8: benchmarking, pre-filter only)
        const uint64_t tq0 = stamp();
        uint32_t bits = 0u;
#pragma unroll
        for (int e = 0; e < 16; e++) bits = (bits << 1) | (uint32_t)!(d[e] < 0.0f);
        if (!any) bits = 0u;
#if PMM_WS_QPS
        // every lane's survivor count, one wave prefix sum (5 ballots: a lane
        // has <= 16), then each lane appends its own survivors at consecutive
        // queue slots straight from the hand-off registers: no per-survivor
        // ballot / branch / LDS re-read round.  One capacity check per group,
        // before the appends.  (The queue order changes, the results do not:
        // the drain's exact re-score and threshold compare see the same set.)
        const int nl = __popc(bits);
        int excl = 0, tot = 0;
#pragma unroll
        for (int j = 0; j < 5; j++) {
          const u64 m = __ballot((nl >> j) & 1);
          excl += lanes_below(m) << j;
          tot += __popcll(m) << j;
        }
        if (qlen + tot > QCAP) {
          wait_lgkm0();
          drain();
        }
        if (tot <= QCAP) {
          uint32_t qa = lq_lds + (uint32_t)(qlen + excl) * 8u;
          const uint32_t hi0 = (uint32_t)(4 * h) | ((uint32_t)gcol << 5);
#pragma unroll
          for (int e = 0; e < 16; e++) {
            if ((bits >> (15 - e)) & 1u) {
              const uint32_t hi = hi0 + (uint32_t)((e & 3) + 8 * (e >> 2));  // acc_row(e, h) | gcol << 5
              const u64 item = (u64)__float_as_uint(v4[e >> 2][e & 3]) | ((u64)hi << 32);
              asm volatile("ds_write_b64 %0, %1" ::"v"(qa), "v"(item) : "memory");
              qa += 8u;
            }
          }
          qlen += tot;
          if (timing) cy5 += stamp() - tq0;
          return;
        }
        // (more survivors in this group than the queue holds: a row's first
        // tiles against an unseeded threshold; the per-round loop below)
#endif
        const float *hf = (const float *)(hb + ((c * 4) * 64 + lane) * 16);
        for (;;) {
          const bool act = bits != 0u;
          const u64 mk = __ballot(act);
          if (mk == 0ull) break;
          if (act) {
            const int j = 31 - __builtin_clz(bits);  // bit j <-> e = 15 - j
            bits &= ~(1u << j);
            const int e = 15 - j;
            const float v = hf[(e >> 2) * 256 + (e & 3)];
            const uint32_t hi = (uint32_t)acc_row(e, h) | ((uint32_t)gcol << 5);
            const u64 item = (u64)__float_as_uint(v) | ((u64)hi << 32);
            asm volatile("ds_write_b64 %0, %1" ::"v"(lq_lds + (uint32_t)(qlen + lanes_below(mk)) * 8u),
                         "v"(item)
                         : "memory");
          }
          qlen += __popcll(mk);
          if (qlen > QCAP - 64) {
            wait_lgkm0();
            drain();
          }
        }
        if (timing) cy5 += stamp() - tq0;
      };

      // prologue: K-steps 0 .. NST-2 of the unit; steps 0 and 1 landed
      // before B_0 (the MFMA waves read step g + 1's first fragments in step g)
      constexpr int LEAD = 1;
#pragma unroll
      for (int j = 0; j < NST - 1; j++) stage(j, t0 + j / KS, j % KS);
      {
        int n = 0;
#pragma unroll
        for (int j = 1 + LEAD; j < NST - 1; j++) n += step_dmas<XFORM>(j % KS);
        wait_vm_n(n);
      }
      int sl = 0;
      for (int tile = t0; tile < t1; tile++) {
        if constexpr (C::SLOT_REPEATS) asm volatile("" : "+s"(sl));  // (see Carve)
        // unrolled: compile-time slot / count arithmetic (a runtime K-step
        // loop, 40% less code, measured 12% slower at c4: the epilogue waves'
        // per-interval instructions are on the critical path)
#pragma unroll
        for (int ks = 0; ks < KS; ks++) {
          uint64_t tt = stamp();
          barrier();  // B_g
          if (timing) {
            const uint64_t t2 = stamp();
            cy3 += t2 - tt;
            tt = t2;
          }
          {
            // step g + NST - 1 into the slot of step g - 1 (read by every
            // MFMA wave before B_g); past the unit's end a harmless read
            constexpr int ahead = NST - 1;
            const int slj = (sl == 0) ? NST - 1 : sl - 1;
            stage(slj, tile + (ks + ahead) / KS, (ks + ahead) % KS);
          }
          if (timing) {
            const uint64_t t2 = stamp();
            cy0 += t2 - tt;
            tt = t2;
          }
          if (tile > t0 && PMM_ABL(a.ablate) != 1 && PMM_ABL(a.ablate) != 3) {
            // column group c in interval ES * c + EO, the drain in interval
            // dks (all of tile - 1's hand-off reads done before interval KS -
            // 1, where the MFMA waves rewrite the hand-off); every other
            // interval when there are enough (KS >= 5): the DMA-only intervals
            // between let the MFMA waves catch up (+0.6% at c4; PMM_ABLATE bit
            // 6 = consecutive intervals), starting one or two intervals into
            // the tile (the MFMA waves' hand-off writes and the tile's first
            // fragment reads go first: c4 147.1-147.3 vs 148.5-149.0 ms for one;
            // groups three intervals apart 148.2; drain in interval 0 worse)
            constexpr bool STR2 = KS >= 2 * NB + 1;
            constexpr int ES2 = KS >= 6 ? PMM_WS_EPI_SPACING : 2;
            // (offset 2 where the K steps allow: c4 151.1-151.4 vs 151.6-151.9
            // ms with offset 1, alternated)
            constexpr int EO2 = PMM_WS_EPI_OFFSET >= 0 ? PMM_WS_EPI_OFFSET : (KS >= 6 ? 2 : 1);
            // every group's hand-off reads end before interval KS - 1
            static_assert(!STR2 || EO2 + ES2 * (NB - 1) <= KS - 2, "epilogue schedule overlaps the hand-off");
            const bool str2 = STR2 && !(PMM_ABL(a.ablate) & 64);
            const int ES = str2 ? ES2 : 1;
            const int EO = str2 ? EO2 : 0;
            const int dks = KS == 1 ? 0 : (str2 ? (PMM_WS_DRAIN_INTERVAL >= 0 ? PMM_WS_DRAIN_INTERVAL % KS
                                                   : (EO ? KS - 1 : 2 * NB)) : NB - 1);
            if (KS == 1) {
#pragma unroll
              for (int c = 0; c < NB; c++) epilogue(tile - 1, c);
            } else if (ks >= EO && (ks - EO) % ES == 0 && (ks - EO) / ES < NB) {
              epilogue(tile - 1, (ks - EO) / ES);
            }
            if (ks == dks && ((tile - t0) % drain_tiles<KS>()) == 0 && qlen > 0) {
              wait_lgkm0();
              drain();
            }
          }
          if (timing) {
            const uint64_t t2 = stamp();
            cy1 += t2 - tt;
            tt = t2;
          }
          // step g + 1 + LEAD landed; later steps may stay in flight
          {
            int n = 0;
#pragma unroll
            for (int j = 2 + LEAD; j < NST; j++) n += step_dmas<XFORM>((ks + j) % KS);
            wait_vm_n(n);
          }
          if (timing) cy2 += stamp() - tt;
          sl = (sl == NST - 1) ? 0 : sl + 1;
        }
      }
      barrier();  // the last tile's accumulators are in LDS
      if (PMM_ABL(a.ablate) != 1 && PMM_ABL(a.ablate) != 3) {
#pragma unroll
        for (int c = 0; c < NB; c++) epilogue(t1 - 1, c);
        wait_lgkm0();
        drain();
      }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // ring DMAs past the unit's end
      if (lane < 32) {
        const int grow = wrow0 + lane;
        if (u.last && grow < a.M) a.cnt[(int64_t)grow * a.S + s] = cnt_w[lane];
      }
      barrier();
    }
  }
  if (timing && lane == 0) {
    // MFMA waves: [1] all; epilogue waves: [0] survivors queued, [3] DMA
    // issue, [4] epilogue, [5] vmcnt waits, [6] barriers, [7] all, [8]
    // compactions, [9] rows compacted, [10] survivor queueing (incl. drains
    // it triggers), [11] drains (incl. compactions)
    const uint64_t all = __builtin_amdgcn_s_memtime() - t_start;
    if (is_mfma) {
      atomicAdd(a.stats + 1, (u64)all);  // (no per-phase stamps: the role has no spare registers)
    } else {
      atomicAdd(a.stats + 0, (u64)nq);
      atomicAdd(a.stats + 3, (u64)cy0);
      atomicAdd(a.stats + 4, (u64)cy1);
      atomicAdd(a.stats + 5, (u64)cy2);
      atomicAdd(a.stats + 6, (u64)cy3);
      atomicAdd(a.stats + 7, (u64)all);
      atomicAdd(a.stats + 8, (u64)cy4);
      atomicAdd(a.stats + 9, (u64)ncomp);
      atomicAdd(a.stats + 10, (u64)cy5);
      atomicAdd(a.stats + 11, (u64)cy6);
    }
  }
}

// ===========================================================================
// Threshold seed for the wave-specialised kernel.  The scores of the first ns
// corpus rows, computed the way the main pass computes them -- the same query
// fragments (registers), the same corpus K-chunk per lane and step, the
// same MFMA chain per accumulator block (16x16x32, or 32x32x16 with
// PMM_WS_MFMA16=0), the same exact_score on the same norms -- so each is bit for
// bit the score the main pass gives that (row, column).  Stored S[row][col]
// (the main pass's candidate buffers, unused until it starts) for
// seed_select_kernel, which sets gthr[row] = (k-th best composite) - 1: an
// exact lower bound of the row's final k-th best.  One wave per 32 query
// rows, one workgroup per 128; the corpus sample streams through LDS in
// 32-column blocks (double-buffered, the next block's global loads in flight
// during this block's MFMAs), staged once per workgroup: round 2 loaded every
// wave's fragments from global memory, four times the L2 traffic, 1.1 ms at
// c4 (ns = 1024).  (The first MFMA accumulates onto zeros where the main
// pass's uses the inline constant 0: the same sums.)
// ===========================================================================
template <int KS>
struct SeedCarve {
  static constexpr int RB = KS * 256;      // bytes of a sample row's padded K range
  static constexpr int RS = RB + 16;       // LDS row stride (16 B pad spreads the 32 rows over the banks)
  static constexpr int CH = RB / 16;       // 16-byte chunks per row
  static constexpr int NCH = 32 * CH / 256;  // chunks per thread per 32-row block
  static constexpr int BYTES = 2 * 32 * RS;
  static_assert((32 * CH) % 256 == 0, "a block's chunks split evenly over 256 threads");
};
template <int KS, int METRIC>
__global__ __launch_bounds__(256, 1) void seed_bf16_ws_kernel(GemmF32Args a, float *__restrict__ S, int ns) {
  using namespace ws;
  using SC = SeedCarve<KS>;
  constexpr int G = KSUB * KS;  // K substeps of 16
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
#if !PMM_WS_MFMA16
  const int r32 = lane & 31, h = lane >> 5;
#endif
  const int wrow0 = (int)blockIdx.x * BM + w * 32;
  // (wave-uniform; a wave past the last query row still stages and syncs)
  const bool active = wrow0 < a.M;
  bf16x8 af[G];
  if (active) {
    const __amdgpu_buffer_rsrc_t rq =
        make_rsrc(a.qb + (int64_t)wrow0 * a.ldq, (int64_t)min(32, a.M - wrow0) * a.ldq * 2);
    // (compiler-visible loads: these registers may be moved before use, and
    // an asm load's destination must not be read before its wait)
#if PMM_WS_MFMA16
    const uint32_t qoff = (uint32_t)((lane & 15) * a.ldq * 2 + 16 * (lane >> 4));
#pragma unroll
    for (int i = 0; i < G; i++)
      af[i] = __builtin_bit_cast(
          bf16x8, __builtin_amdgcn_raw_buffer_load_b128(
                      rq, (int)(qoff + (i & 1) * 16 * a.ldq * 2 + ((i / KSUB) * 128 + ((i % KSUB) / 2) * 32) * 2), 0, 0));
#else
    const uint32_t qoff = (uint32_t)(r32 * a.ldq * 2 + 128 * h);
#pragma unroll
    for (int i = 0; i < G; i++)
      af[i] = __builtin_bit_cast(
          bf16x8, __builtin_amdgcn_raw_buffer_load_b128(rq, (int)(qoff + ((i / KSUB) * 128 + (i % KSUB) * 8) * 2), 0, 0));
#endif
  }
  constexpr bool XFORM = METRIC != kMetricDot;
  float qv[16];
#pragma unroll
  for (int e = 0; e < 16; e++) {
#if PMM_WS_MFMA16
    const int row = wrow0 + 16 * (e >> 2) + 4 * (lane >> 4) + (e & 3);  // e = 4 rb + i
#else
    const int row = wrow0 + acc_row(e, h);
#endif
    qv[e] = (XFORM && row < a.M) ? a.qn[row] : 0.0f;
  }
  const __amdgpu_buffer_rsrc_t rc = make_rsrc(a.cb, (int64_t)ns * a.ldc * 2);
  // block t's rows t*32 .. t*32+31: thread tid carries chunks tid + 256 j
  typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
  u32x4 pf[SC::NCH];
  auto fetch = [&](int t) __attribute__((always_inline)) {
#pragma unroll
    for (int j = 0; j < SC::NCH; j++) {
      const int c = tid + 256 * j, r = c / SC::CH, q = c - r * SC::CH;
      pf[j] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(
                                            rc, (int)((t * 32 + r) * a.ldc * 2 + q * 16), 0, 0));
    }
  };
  auto put = [&](int buf) __attribute__((always_inline)) {
#pragma unroll
    for (int j = 0; j < SC::NCH; j++) {
      const int c = tid + 256 * j, r = c / SC::CH, q = c - r * SC::CH;
      *(u32x4 *)(smem + buf * 32 * SC::RS + r * SC::RS + q * 16) = pf[j];
    }
  };
  const int nt = ns / 32;
  if (nt > 0) {
    fetch(0);
    put(0);
  }
  __syncthreads();
  for (int t = 0; t < nt; t++) {
    if (t + 1 < nt) fetch(t + 1);
#if PMM_WS_MFMA16
    if (active) {
      // lane (c16, g): column block cb of 16, K-step ks, step j: column
      // t 32 + 16 cb + c16, k 128 ks + 32 j + 8 g .. + 7 -- the main pass's
      // chain per 16 x 16 block, K in natural order
      typedef __bf16 bf16v8 __attribute__((ext_vector_type(8)));
      const int c16 = lane & 15, g4 = lane >> 4;
#pragma unroll
      for (int cb = 0; cb < 2; cb++) {
        const int col = t * 32 + 16 * cb + c16;
        const char *base = smem + (t & 1) * 32 * SC::RS + (16 * cb + c16) * SC::RS + 16 * g4;
        f32x4 acc[2] = {{}, {}};
#pragma unroll
        for (int ks = 0; ks < KS; ks++)
#pragma unroll
          for (int j = 0; j < 4; j++) {
            const bf16x8 b = *(const bf16x8 *)(base + (ks * 128 + 32 * j) * 2);
#pragma unroll
            for (int rb = 0; rb < 2; rb++)
              acc[rb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(
                  __builtin_bit_cast(bf16v8, af[KSUB * ks + 2 * j + rb]), __builtin_bit_cast(bf16v8, b), acc[rb], 0,
                  0, 0);
          }
        const float cv = XFORM ? a.cn[col] : 0.0f;
#pragma unroll
        for (int e = 0; e < 8; e++) {
          const int row = wrow0 + 16 * (e >> 2) + 4 * g4 + (e & 3);
          if (row < a.M) S[(int64_t)row * ns + col] = exact_score<METRIC>(acc[e >> 2][e & 3], qv[e], cv);
        }
      }
    }
#else
    if (active) {
      const int col = t * 32 + r32;
      // lane (r32, h), substep gs: column col, K-step gs / 8, chunk 8h + gs % 8
      const char *base = smem + (t & 1) * 32 * SC::RS + r32 * SC::RS + 128 * h;
      // the compiler's MFMA builtin (the same instruction as the main pass's
      // asm, so the same bits): here hipcc allocates the operands freely and
      // must see the instruction to pad its register hazards
      typedef __bf16 bf16v8 __attribute__((ext_vector_type(8)));
      f32x16 acc = {};
#pragma unroll
      for (int gs = 0; gs < G; gs++) {
        const bf16x8 b = *(const bf16x8 *)(base + ((gs / KSUB) * 128 + (gs % KSUB) * 8) * 2);
        acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16v8, af[gs]),
                                                      __builtin_bit_cast(bf16v8, b), acc, 0, 0, 0);
      }
      const float cv = XFORM ? a.cn[col] : 0.0f;
#pragma unroll
      for (int e = 0; e < 16; e++) {
        const int row = wrow0 + acc_row(e, h);
        if (row < a.M) S[(int64_t)row * ns + col] = exact_score<METRIC>(acc[e], qv[e], cv);
      }
    }
#endif
    // block t + 1 into the buffer block t - 1 used (every wave left it at
    // the previous barrier); visible to all after this one
    if (t + 1 < nt) put((t + 1) & 1);
    __syncthreads();
  }
}

template <int KS, int METRIC>
static hipError_t launch_seed_bf16_ws_t(const GemmF32Args &a, float *S, int ns, hipStream_t s) {
  static bool attr_set = false;
  if (!attr_set) {
    hipError_t e = hipFuncSetAttribute((const void *)seed_bf16_ws_kernel<KS, METRIC>,
                                       hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    if (e != hipSuccess) return e;
    attr_set = true;
  }
  seed_bf16_ws_kernel<KS, METRIC><<<dim3((unsigned)((a.M + ws::BM - 1) / ws::BM)), dim3(256),
                                    SeedCarve<KS>::BYTES, s>>>(a, S, ns);
  return hipGetLastError();
}

template <int KS, int METRIC>
static hipError_t launch_bf16_ws_t(const GemmF32Args &a, int grid, size_t lds, hipStream_t s) {
  static bool attr_set = false;
  if (!attr_set) {
    hipError_t e = hipFuncSetAttribute((const void *)gemm_bf16_ws_kernel<KS, METRIC>,
                                       hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    if (e != hipSuccess) return e;
    attr_set = true;
  }
  gemm_bf16_ws_kernel<KS, METRIC><<<dim3(grid), dim3(ws::NTH), lds, s>>>(a);
  return hipGetLastError();
}

}  // namespace pmm
