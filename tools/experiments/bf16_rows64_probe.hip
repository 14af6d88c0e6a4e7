// bf16_rows64_probe.hip -- feasibility probe (not product code): 256 query
// rows resident per CU with ONE wave per SIMD (64 rows x D = 768 each: 192
// AGPRs + 192 VGPRs of query fragments), corpus tiles of 32 columns streamed
// through a 3-slot LDS-DMA ring, 96 v_mfma_f32_32x32x16_bf16 per tile per
// wave, one fmax per score as the stand-in epilogue.  Half the streamed bytes
// per flop of the wave-specialised kernel; how fast is the bare loop at the
// c4 shape?
//
// Build: hipcc --offload-arch=gfx950 -O3 -o bf16_rows64_probe bf16_rows64_probe.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstdint>
#include <vector>
#include <cmath>
#include <cstring>

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

#ifndef PROBE_ABL
#define PROBE_ABL 0  // 1: no DMA, 2: no fragment reads
#endif
#ifndef PF
#define PF 4  // fragments read ahead
#endif
constexpr int D = 768, KSTEPS = D / 16;   // 48 K16 steps
constexpr int BM = 256, BN = 32;          // rows per workgroup, columns per tile
constexpr int TILE = BN * D * 2;          // 48 KiB
constexpr int NS = 3;                     // ring slots
constexpr int PIECES = TILE / 1024 / 4;   // 12 per wave

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void *p, int64_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void *>(p), (short)0, (int)bytes, 0x00020000);
}
__device__ __forceinline__ void dma(__amdgpu_buffer_rsrc_t r, uint32_t lds, uint32_t voff) {
  asm volatile("s_mov_b32 m0, %0\n\ts_nop 0\n\tbuffer_load_dwordx4 %1, %2, 0 offen lds" ::"s"(lds), "v"(voff),
               "s"(r)
               : "memory");
}
__device__ __forceinline__ void mfma_a(f32x16 &c, const bf16x8 &a, const bf16x8 &b) {
  asm volatile("v_mfma_f32_32x32x16_bf16 %0, %1, %2, %0" : "+v"(c) : "a"(a), "v"(b));
}
__device__ __forceinline__ void mfma_v(f32x16 &c, const bf16x8 &a, const bf16x8 &b) {
  asm volatile("v_mfma_f32_32x32x16_bf16 %0, %1, %2, %0" : "+v"(c) : "v"(a), "v"(b));
}

struct Args {
  const uint16_t *q, *c;
  int QB, CT;  // query blocks of 256 rows, corpus tiles of 32 columns
  float *out;
};

__global__ __launch_bounds__(256, 1) void probe(Args a) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const uint32_t lds0 = (uint32_t)(size_t)(LDS_AS char *)smem;
  float *keep_l = (float *)(smem + NS * TILE);
  keep_l[tid] = 0.0f;
  // work: workgroup b takes query blocks b, b + grid, ...; all corpus tiles
  // each (the workgroups of an XCD stream the same tiles together)
  for (int qb = blockIdx.x; qb < a.QB; qb += gridDim.x) {
    // query fragments: rows qb*256 + 64 wid + 32 rb + (lane & 31), K16 step j:
    // k = 16 j + 8 (lane >> 5) .. + 8
    bf16x8 qa[KSTEPS], qv[KSTEPS];
    {
      int ln = (int)__lane_id();
      asm volatile("" : "+v"(ln));
      const int64_t r0 = (int64_t)qb * BM + 64 * wid;
      const __amdgpu_buffer_rsrc_t ra = rsrc(a.q + r0 * D, 32 * D * 2);
      const __amdgpu_buffer_rsrc_t rv = rsrc(a.q + (r0 + 32) * D, 32 * D * 2);
      const uint32_t off = (uint32_t)((ln & 31) * D * 2 + (ln >> 5) * 16);
      asm volatile("s_nop 4" ::"s"(ra), "s"(rv));
#pragma unroll
      for (int j = 0; j < KSTEPS; j++) {
        asm volatile("buffer_load_dwordx4 %0, %1, %2, 0 offen offset:%3" : "=a"(qa[j]) : "v"(off), "s"(ra), "i"(32 * j) : "memory");
        asm volatile("buffer_load_dwordx4 %0, %1, %2, 0 offen offset:%3" : "=v"(qv[j]) : "v"(off), "s"(rv), "i"(32 * j) : "memory");
      }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
      for (int j = 0; j < KSTEPS; j++) {
        asm volatile("" : "+a"(qa[j]));
        asm volatile("" : "+v"(qv[j]));
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
      const int col = ln & 31, h = ln >> 5;
      const char *st = smem + (t % NS) * TILE + col * D * 2;
      f32x16 acc0 = {}, acc1 = {};
      bf16x8 fb[PF];
      auto rd = [&](int j) -> bf16x8 {
        if (PROBE_ABL & 2) {
          bf16x8 z = {};
          asm volatile("" : "+v"(z));
          return z;
        }
        return *(const bf16x8 *)(st + (((2 * j + h) ^ (col & 15)) * 16));
      };
#pragma unroll
      for (int j = 0; j < PF; j++) fb[j] = rd(j);
#pragma unroll
      for (int j = 0; j < KSTEPS; j++) {
        const bf16x8 b = fb[j % PF];
        if (j + PF < KSTEPS) fb[j % PF] = rd(j + PF);
        mfma_a(acc0, qa[j], b);
        mfma_v(acc1, qv[j], b);
      }
      asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 3" : "+v"(acc0), "+v"(acc1));
      float keep = keep_l[tid];
#pragma unroll
      for (int e = 0; e < 16; e++) keep = fmaxf(keep, fmaxf(acc0[e], acc1[e]));
      keep_l[tid] = keep;
    }
    __syncthreads();
  }
  a.out[blockIdx.x * 256 + tid] = keep_l[tid];
}

// Input data: mode 0 (round 3) fills both operands with one repeating
// pattern of positive bf16 values in [2^-7, 2^-6); mode 1 with N(0, 1) bf16
// (the c4 bench's data: torch.randn rounded to bf16).  The chip's clock under
// an MFMA-dense load depends on the operands (MI355X_MICROARCH.md, DVFS
// give-back), so the loop's ceiling is only meaningful on the real data.
static uint16_t f2bf(float f) {
  uint32_t u;
  memcpy(&u, &f, 4);
  return (uint16_t)((u + 0x7FFFu + ((u >> 16) & 1u)) >> 16);
}

int main(int argc, char **argv) {
  const int reps = argc > 1 ? atoi(argv[1]) : 3;
  const int mode = argc > 2 ? atoi(argv[2]) : 0;
  const int QB = 256, CT = 31250;  // 65536 x 1000000 (one query block per workgroup)
  const int64_t M = (int64_t)QB * BM, N = (int64_t)CT * BN;
  uint16_t *q, *c;
  float *out;
  CHECK(hipMalloc(&q, M * D * 2));
  CHECK(hipMalloc(&c, N * D * 2));
  CHECK(hipMalloc(&out, 256 * 256 * 4));
  {
    std::vector<uint16_t> hb((1 << 20) + 17);  // (17: the rows do not repeat with the 768-wide stride)
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
    printf("{\"mode\": %d, \"abl\": %d, \"rep\": %d, \"ms\": %.3f, \"tflops\": %.1f, \"frac\": %.4f}\n", mode,
           PROBE_ABL, r, ms, tf, tf / 2516.6);
  }
  return 0;
}
