// bf16_gemm_probe.hip -- feasibility probe (not product code): how fast does
// a conventional LDS-tiled bf16 GEMM loop run at the c4 shape on gfx950,
// both operands streamed through LDS, 256 x 256 output tiles, 4 waves of
// 128 x 128 (16 accumulators of v_mfma_f32_32x32x16_bf16), a 4-stage LDS-DMA
// ring of K = 32 stages, XCD-grouped tile order?  The "epilogue" is one fmax
// per score (a stand-in for the top-k pre-filter's per-score cost).
//
// Build: hipcc --offload-arch=gfx950 -O3 -o bf16_gemm_probe bf16_gemm_probe.hip
// Run:   ./bf16_gemm_probe [reps]
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstdint>
#include <vector>

#define CHECK(x)                                                                 \
  do {                                                                           \
    hipError_t e_ = (x);                                                         \
    if (e_ != hipSuccess) {                                                      \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                                   \
    }                                                                            \
  } while (0)

#define LDS_AS __attribute__((address_space(3)))
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

constexpr int D = 768;
constexpr int BM = 256, BN = 256, KST = 32;  // tile, K per stage
constexpr int NSTG = D / KST;                // stages per tile (24)
constexpr int NS = 4;                        // ring slots
constexpr int STAGE = (BM + BN) * KST * 2;   // 32 KiB
constexpr int GQ = 4, GC = 8;
#ifndef PROBE_ABL
#define PROBE_ABL 0  // 1: no DMA (stale LDS), 2: no fragment reads
#endif                // per-XCD group: 4 query blocks x 8 corpus tiles

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void *p, int64_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void *>(p), (short)0, (int)bytes, 0x00020000);
}
// LDS-DMA from asm (hipcc would otherwise wait vmcnt(0) before every LDS read)
__device__ __forceinline__ void dma(__amdgpu_buffer_rsrc_t r, uint32_t lds, uint32_t voff) {
  asm volatile("s_mov_b32 m0, %0\n\ts_nop 0\n\tbuffer_load_dwordx4 %1, %2, 0 offen lds" ::"s"(lds), "v"(voff),
               "s"(r)
               : "memory");
}

struct Args {
  const uint16_t *q, *c;
  int QB, CT;  // query blocks, corpus tiles (multiples of GQ, GC)
  float *out;
};

__global__ __launch_bounds__(256, 1) void probe(Args a) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wid >> 1, wc = wid & 1;
  const uint32_t lds0 = (uint32_t)(size_t)(LDS_AS char *)smem;
  // XCD-aware work split: workgroup b runs on XCD b % 8, slot j = b / 8 of 32
  const int xcd = blockIdx.x & 7, j = blockIdx.x >> 3;
  const int groups = a.QB / GQ, chunks = a.CT / GC;
  const int my_groups = (groups - xcd + 7) / 8;
  const int ntiles = my_groups * chunks;  // tiles of this workgroup
  auto tile_at = [&](int t, int &qb, int &ct) {
    const int g = xcd + 8 * (t / chunks), ch = t % chunks;
    qb = g * GQ + (j & 3);
    ct = ch * GC + (j >> 2);
  };
  // DMA pieces of one stage: 32 KiB = 32 pieces of 1 KiB, 8 per wave
  // (pieces 0-15 = A rows, 16-31 = B rows; 64 B per row; chunk c of row r at
  // slot c ^ ((r >> 2) & 3))
  auto issue = [&](int gs) {
    if (gs >= ntiles * NSTG || (PROBE_ABL & 1)) return;
    int qb, ct;
    tile_at(gs / NSTG, qb, ct);
    const int ks = gs % NSTG;
    const uint32_t st = lds0 + (uint32_t)((gs % NS) * STAGE);
    const __amdgpu_buffer_rsrc_t ra = rsrc(a.q + (int64_t)qb * BM * D, (int64_t)BM * D * 2);
    const __amdgpu_buffer_rsrc_t rb = rsrc(a.c + (int64_t)ct * BN * D, (int64_t)BN * D * 2);
    // (the lane id opaque: per-lane offsets recomputed here, not hoisted and
    // spilled across the loop)
    int ln = (int)__lane_id();
    asm volatile("" : "+v"(ln));
#pragma unroll
    for (int i = 0; i < 8; i++) {
      const int lane = ln;
      const int p = wid * 8 + i;       // piece 0..31
      const int pr = p & 15;           // piece within the operand
      const int row = pr * 16 + (lane >> 2), slot = lane & 3;
      const int ch = slot ^ ((row >> 2) & 3);
      const uint32_t voff = (uint32_t)(row * D * 2 + ks * KST * 2 + ch * 16);
      dma(p < 16 ? ra : rb, __builtin_amdgcn_readfirstlane(st + (uint32_t)(p * 1024)), voff);
    }
  };
  // the stand-in epilogue's running max lives in LDS (a register for it
  // spills, and the reload's vmcnt(0) would drain the DMA ring every tile)
  float *keep_l = (float *)(smem + NS * STAGE);
  keep_l[tid] = 0.0f;
  const int total = ntiles * NSTG;
  for (int s = 0; s < 3; s++) issue(s);
  for (int t = 0; t < ntiles; t++) {
    f32x16 acc[4][4];
#pragma unroll
    for (int rb = 0; rb < 4; rb++)
#pragma unroll
      for (int cb = 0; cb < 4; cb++) acc[rb][cb] = (f32x16){};
    for (int ks = 0; ks < NSTG; ks++) {
      const int gs = t * NSTG + ks;
      // own pieces of stage gs landed (stages gs+1, gs+2 may still be in flight)
      if (gs + 2 < total) asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
      else if (gs + 1 < total) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
      else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
      issue(gs + 3);  // slot of stage gs - 1: every wave is past it
      const char *st = smem + (gs % NS) * STAGE;
      int ln = (int)__lane_id();
      asm volatile("" : "+v"(ln));
#pragma unroll
      for (int kh = 0; kh < 2; kh++) {
        bf16x8 fa[4], fb[4];
        const int chunk = kh * 2 + (ln >> 5);
#pragma unroll
        for (int rb = 0; rb < 4; rb++) {
          const int row = wr * 128 + rb * 32 + (ln & 31);
          if (PROBE_ABL & 2) { fa[rb] = (bf16x8){}; asm volatile("" : "+v"(fa[rb])); }
          else fa[rb] = *(const bf16x8 *)(st + row * 64 + ((chunk ^ ((row >> 2) & 3)) * 16));
        }
#pragma unroll
        for (int cb = 0; cb < 4; cb++) {
          const int row = wc * 128 + cb * 32 + (ln & 31);
          if (PROBE_ABL & 2) { fb[cb] = (bf16x8){}; asm volatile("" : "+v"(fb[cb])); }
          else fb[cb] = *(const bf16x8 *)(st + BM * 64 + row * 64 + ((chunk ^ ((row >> 2) & 3)) * 16));
        }
#pragma unroll
        for (int rb = 0; rb < 4; rb++)
#pragma unroll
          for (int cb = 0; cb < 4; cb++)
            acc[rb][cb] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[rb], fb[cb], acc[rb][cb], 0, 0, 0);
      }
    }
    // stand-in epilogue: one op per score
    float keep = keep_l[tid];
#pragma unroll
    for (int rb = 0; rb < 4; rb++)
#pragma unroll
      for (int cb = 0; cb < 4; cb++)
#pragma unroll
        for (int e = 0; e < 16; e++) keep = fmaxf(keep, acc[rb][cb][e]);
    keep_l[tid] = keep;
  }
  const float keep = keep_l[tid];
  a.out[blockIdx.x * 256 + tid] = keep;
}

int main(int argc, char **argv) {
  const int reps = argc > 1 ? atoi(argv[1]) : 3;
  const int QB = 392, CT = 3904;  // 100352 x 999424
  const int64_t M = (int64_t)QB * BM, N = (int64_t)CT * BN;
  uint16_t *q, *c;
  float *out;
  CHECK(hipMalloc(&q, M * D * 2));
  CHECK(hipMalloc(&c, N * D * 2));
  CHECK(hipMalloc(&out, 256 * 256 * 4));
  {
    std::vector<uint16_t> h(1 << 20);
    for (size_t i = 0; i < h.size(); i++) h[i] = (uint16_t)(0x3c00 + (i * 2654435761u >> 22) % 0x200);
    for (int64_t o = 0; o < M * D; o += (int64_t)h.size())
      CHECK(hipMemcpy(q + o, h.data(), std::min<int64_t>(h.size(), M * D - o) * 2, hipMemcpyHostToDevice));
    for (int64_t o = 0; o < N * D; o += (int64_t)h.size())
      CHECK(hipMemcpy(c + o, h.data(), std::min<int64_t>(h.size(), N * D - o) * 2, hipMemcpyHostToDevice));
  }
  CHECK(hipFuncSetAttribute((const void *)probe, hipFuncAttributeMaxDynamicSharedMemorySize, NS * STAGE + 1024));
  Args a{q, c, QB, CT, out};
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  for (int r = 0; r < reps + 1; r++) {
    CHECK(hipEventRecord(e0));
    probe<<<256, 256, NS * STAGE + 1024>>>(a);
    CHECK(hipGetLastError());
    CHECK(hipEventRecord(e1));
    CHECK(hipEventSynchronize(e1));
    float ms;
    CHECK(hipEventElapsedTime(&ms, e0, e1));
    const double tf = 2.0 * M * N * D / (ms * 1e-3) / 1e12;
    printf("{\"rep\": %d, \"ms\": %.3f, \"tflops\": %.1f, \"frac\": %.4f}\n", r, ms, tf, tf / 2516.6);
  }
  return 0;
}
