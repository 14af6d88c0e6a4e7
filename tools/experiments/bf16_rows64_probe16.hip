// bf16_rows64_probe16.hip -- feasibility probe (not product code): the
// rows64 probe's loop (256 query rows per CU, one wave per SIMD holding 64
// rows x D = 768 in registers, 32-column corpus tiles through a 3-slot
// LDS-DMA ring, one fmax per score as the stand-in epilogue) on
// v_mfma_f32_16x16x32_bf16 instead of 32x32x16: 4 row blocks x 2 column
// blocks per 32-K step, 8 MFMAs of 16 cycles per two 16-byte fragment reads.
// MI355X_MICROARCH.md (DVFS give-back item 7): on random data the 16x16x32
// loop delivers 1.12-1.15x the FLOP/s of the 32x32x16 one at equal cycles.
// Does that hold for this loop?
//
// Build: hipcc --offload-arch=gfx950 -O3 [-DPROBE_ABL=n] -o bf16_rows64_probe16 bf16_rows64_probe16.hip
// Run:   ./bf16_rows64_probe16 <reps> <mode: 0 pattern data, 1 N(0,1) bf16>
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstdint>
#include <cstring>
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
typedef float f32x4 __attribute__((ext_vector_type(4)));

#ifndef PROBE_ABL
#define PROBE_ABL 0  // 1: no DMA, 2: no fragment reads
#endif
constexpr int D = 768, KS32 = D / 32;     // 24 K32 steps
constexpr int BM = 256, BN = 32;
constexpr int TILE = BN * D * 2;          // 48 KiB
constexpr int NS = 3;
constexpr int PIECES = TILE / 1024 / 4;   // 12 per wave

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void *p, int64_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void *>(p), (short)0, (int)bytes, 0x00020000);
}
__device__ __forceinline__ void dma(__amdgpu_buffer_rsrc_t r, uint32_t lds, uint32_t voff) {
  asm volatile("s_mov_b32 m0, %0\n\ts_nop 0\n\tbuffer_load_dwordx4 %1, %2, 0 offen lds" ::"s"(lds), "v"(voff),
               "s"(r)
               : "memory");
}
__device__ __forceinline__ void mfma_a(f32x4 &c, const bf16x8 &a, const bf16x8 &b) {
  asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+v"(c) : "a"(a), "v"(b));
}
__device__ __forceinline__ void mfma_v(f32x4 &c, const bf16x8 &a, const bf16x8 &b) {
  asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+v"(c) : "v"(a), "v"(b));
}

struct Args {
  const uint16_t *q, *c;
  int QB, CT;
  float *out;
};

__global__ __launch_bounds__(256, 1) void probe(Args a) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const uint32_t lds0 = (uint32_t)(size_t)(LDS_AS char *)smem;
  float *keep_l = (float *)(smem + NS * TILE);
  keep_l[tid] = 0.0f;
  for (int qb = blockIdx.x; qb < a.QB; qb += gridDim.x) {
    // blocks 0,1 (rows 0-31 of the wave) in AGPRs, blocks 2,3 in VGPRs:
    // row (lane & 15) of block b, k = 32 j + 8 (lane >> 4) .. + 8
    bf16x8 qa[2][KS32], qv[2][KS32];
    {
      int ln = (int)__lane_id();
      asm volatile("" : "+v"(ln));
      const int64_t r0 = (int64_t)qb * BM + 64 * wid;
      const uint32_t off = (uint32_t)((ln & 15) * D * 2 + (ln >> 4) * 16);
#pragma unroll
      for (int b = 0; b < 2; b++) {
        const __amdgpu_buffer_rsrc_t ra = rsrc(a.q + (r0 + 16 * b) * D, 16 * D * 2);
        const __amdgpu_buffer_rsrc_t rv = rsrc(a.q + (r0 + 32 + 16 * b) * D, 16 * D * 2);
        asm volatile("s_nop 4" ::"s"(ra), "s"(rv));
#pragma unroll
        for (int j = 0; j < KS32; j++) {
          asm volatile("buffer_load_dwordx4 %0, %1, %2, 0 offen offset:%3" : "=a"(qa[b][j]) : "v"(off), "s"(ra), "i"(64 * j) : "memory");
          asm volatile("buffer_load_dwordx4 %0, %1, %2, 0 offen offset:%3" : "=v"(qv[b][j]) : "v"(off), "s"(rv), "i"(64 * j) : "memory");
        }
      }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
      for (int b = 0; b < 2; b++)
#pragma unroll
        for (int j = 0; j < KS32; j++) {
          asm volatile("" : "+a"(qa[b][j]));
          asm volatile("" : "+v"(qv[b][j]));
        }
    }
    auto issue = [&](int t) {
      if (t >= a.CT || (PROBE_ABL & 1)) return;
      int ln = (int)__lane_id();
      asm volatile("" : "+v"(ln));
      const __amdgpu_buffer_rsrc_t rb = rsrc(a.c + (int64_t)t * BN * D, (int64_t)BN * D * 2);
      const uint32_t st = lds0 + (uint32_t)((t % NS) * TILE);
#pragma unroll
      for (int i = 0; i < PIECES; i++) {
        const int p = wid * PIECES + i;
        const int o = p * 1024 + ln * 16;
        const int col = o / (D * 2), chs = (o % (D * 2)) / 16;
        const int ch = chs ^ (col & 15);
        dma(rb, __builtin_amdgcn_readfirstlane(st + (uint32_t)(p * 1024)), (uint32_t)(col * D * 2 + ch * 16));
      }
    };
    issue(0);
    issue(1);
    for (int t = 0; t < a.CT; t++) {
      if (t + 1 < a.CT) asm volatile("s_waitcnt vmcnt(12)" ::: "memory");
      else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
      issue(t + 2);
      int ln = (int)__lane_id();
      asm volatile("" : "+v"(ln));
      const int c16 = ln & 15, kg = ln >> 4;
      f32x4 acc[4][2];
#pragma unroll
      for (int b = 0; b < 4; b++) acc[b][0] = acc[b][1] = (f32x4){0.f, 0.f, 0.f, 0.f};
      // fragment of column block cb at K32 step j: column cb*16 + c16, chunk 4 j + kg
      auto rd = [&](int cb, int j) -> bf16x8 {
        if (PROBE_ABL & 2) {
          bf16x8 z = {};
          asm volatile("" : "+v"(z));
          return z;
        }
        const int col = cb * 16 + c16;
        return *(const bf16x8 *)(smem + (t % NS) * TILE + col * D * 2 + (((4 * j + kg) ^ (col & 15)) * 16));
      };
      bf16x8 f0 = rd(0, 0), f1 = rd(1, 0);
#pragma unroll
      for (int j = 0; j < KS32; j++) {
        bf16x8 n0, n1;
        if (j + 1 < KS32) {
          n0 = rd(0, j + 1);
          n1 = rd(1, j + 1);
        }
        mfma_a(acc[0][0], qa[0][j], f0);
        mfma_a(acc[0][1], qa[0][j], f1);
        mfma_a(acc[1][0], qa[1][j], f0);
        mfma_a(acc[1][1], qa[1][j], f1);
        mfma_v(acc[2][0], qv[0][j], f0);
        mfma_v(acc[2][1], qv[0][j], f1);
        mfma_v(acc[3][0], qv[1][j], f0);
        mfma_v(acc[3][1], qv[1][j], f1);
        if (j + 1 < KS32) {
          f0 = n0;
          f1 = n1;
        }
      }
      asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 3" : "+v"(acc[0][0]), "+v"(acc[0][1]), "+v"(acc[1][0]), "+v"(acc[1][1]),
                   "+v"(acc[2][0]), "+v"(acc[2][1]), "+v"(acc[3][0]), "+v"(acc[3][1]));
      float keep = keep_l[tid];
#pragma unroll
      for (int b = 0; b < 4; b++)
#pragma unroll
        for (int e = 0; e < 4; e++) keep = fmaxf(keep, fmaxf(acc[b][0][e], acc[b][1][e]));
      keep_l[tid] = keep;
    }
    __syncthreads();
  }
  a.out[blockIdx.x * 256 + tid] = keep_l[tid];
}

static uint16_t f2bf(float f) {
  uint32_t u;
  memcpy(&u, &f, 4);
  return (uint16_t)((u + 0x7FFFu + ((u >> 16) & 1u)) >> 16);
}

int main(int argc, char **argv) {
  const int reps = argc > 1 ? atoi(argv[1]) : 3;
  const int mode = argc > 2 ? atoi(argv[2]) : 1;
  const int QB = 256, CT = 31250;  // 65536 x 1000000 (one query block per workgroup)
  const int64_t M = (int64_t)QB * BM, N = (int64_t)CT * BN;
  uint16_t *q, *c;
  float *out;
  CHECK(hipMalloc(&q, M * D * 2));
  CHECK(hipMalloc(&c, N * D * 2));
  CHECK(hipMalloc(&out, 256 * 256 * 4));
  {
    std::vector<uint16_t> hb((1 << 20) + 17);
    uint64_t st = 0x9E3779B97F4A7C15ull;
    auto u01 = [&]() {
      st ^= st << 13;
      st ^= st >> 7;
      st ^= st << 17;
      return ((st >> 11) + 0.5) * (1.0 / 9007199254740992.0);
    };
    for (size_t i = 0; i < hb.size(); i++)
      hb[i] = mode == 0 ? (uint16_t)(0x3c00 + (i * 2654435761u >> 22) % 0x200)
                        : f2bf((float)(sqrt(-2.0 * log(u01())) * cos(6.283185307179586 * u01())));
    for (int64_t o = 0; o < M * D; o += (int64_t)hb.size())
      CHECK(hipMemcpy(q + o, hb.data(), std::min<int64_t>(hb.size(), M * D - o) * 2, hipMemcpyHostToDevice));
    for (int64_t o = 0; o < N * D; o += (int64_t)hb.size())
      CHECK(hipMemcpy(c + o, hb.data(), std::min<int64_t>(hb.size(), N * D - o) * 2, hipMemcpyHostToDevice));
  }
  const size_t lds = NS * TILE + 1024;
  CHECK(hipFuncSetAttribute((const void *)probe, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  Args a{q, c, QB, CT, out};
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  for (int r = 0; r < reps + 1; r++) {
    CHECK(hipEventRecord(e0));
    probe<<<256, 256, lds>>>(a);
    CHECK(hipGetLastError());
    CHECK(hipEventRecord(e1));
    CHECK(hipEventSynchronize(e1));
    float ms;
    CHECK(hipEventElapsedTime(&ms, e0, e1));
    const double tf = 2.0 * M * N * D / (ms * 1e-3) / 1e12;
    printf("{\"mfma\": \"16x16x32\", \"mode\": %d, \"abl\": %d, \"rep\": %d, \"ms\": %.3f, \"tflops\": %.1f, \"frac\": %.4f}\n",
           mode, PROBE_ABL, r, ms, tf, tf / 2516.6);
  }
  return 0;
}
