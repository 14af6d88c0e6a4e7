// dma_fetch_calib.hip -- calibrates rocprofv3's FETCH_SIZE for the access
// patterns the fused top-k kernels stream the corpus with (MI355X_MICROARCH.md:
// FETCH_SIZE is only calibrated for 16-byte-per-lane streaming reads).
//
// Each pattern reads a 3 GB row-major "corpus" (1,000,000 rows x 768 f32, the
// c3 corpus; far past the 256 MiB Infinity Cache) exactly once into LDS, so
// the algorithmic byte count is known: FETCH_SIZE x 1024 / bytes is the
// counter's factor for that pattern.
//   pattern 0 "dma4_rows": the f32 kernel's corpus stage (pmm_kernels.hip
//     stage()): per K step of 32 floats, 4-byte buffer_load ... lds, lanes
//     0-31 one row's 128 B, lanes 32-63 the next row's;
//   pattern 1 "dma16_rows": the bf16 kernels' stage: 16-byte buffer_load ...
//     lds, 8 lanes per row's 128-B run, 8 rows per instruction;
//   pattern 2 "dma16_contig": a contiguous 16-byte-per-lane stream (the
//     guide's calibrated case: expect 0.5).
// Build: hipcc --offload-arch=gfx950 -O3 -o dma_fetch_calib dma_fetch_calib.hip
// Run:   rocprofv3 --kernel-trace --pmc FETCH_SIZE -- ./dma_fetch_calib
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

#define CHECK(x)                                                                    \
  do {                                                                              \
    hipError_t e_ = (x);                                                            \
    if (e_ != hipSuccess) {                                                         \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));    \
      exit(1);                                                                      \
    }                                                                               \
  } while (0)

#define LDS_AS __attribute__((address_space(3)))

constexpr int kRows = 1000000, kLd = 768, kRowsPerBlock = 64, kThreads = 256;

__device__ inline __amdgpu_buffer_rsrc_t rsrc(const void *p, int64_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void *>(p), (short)0, (int)bytes, 0x00020000);
}

__device__ __attribute__((always_inline)) inline void dma16(__amdgpu_buffer_rsrc_t r, char *dst,
                                                            uint32_t voff) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (LDS_AS void *)dst, 16, voff, 0, 0, 0);
}

// one workgroup per 64-row block; 4 waves, 16 rows each, all K steps
template <int PAT>
__global__ __launch_bounds__(kThreads) void calib(const float *c, unsigned *sink) {
  __shared__ __attribute__((aligned(16))) char lds[4 * 64 * 16 * 2];
  const int wid = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int64_t row0 = (int64_t)blockIdx.x * kRowsPerBlock;
  const int rows = (int)min<int64_t>(kRowsPerBlock, kRows - row0);
  if (PAT == 2) {
    // contiguous: the block's rows as one byte range, 16 B per lane
    const int64_t bytes = (int64_t)rows * kLd * 4;
    const __amdgpu_buffer_rsrc_t r = rsrc(c + row0 * kLd, bytes);
    for (int64_t o = (int64_t)wid * 1024 + lane * 16; o < bytes; o += 4 * 1024)
      dma16(r, lds + wid * 1024, (uint32_t)o);
  } else {
    const __amdgpu_buffer_rsrc_t r = rsrc(c + row0 * kLd, (int64_t)rows * kLd * 4);
    for (int ks = 0; ks < kLd / 32; ks++) {
      if (PAT == 0) {
#pragma unroll
        for (int i = 0; i < 8; i++) {
          const int row = wid * 16 + 2 * i + (lane >> 5);
          const uint32_t voff = (uint32_t)(row * kLd * 4 + ks * 128 + (lane & 31) * 4);
          __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (LDS_AS void *)(lds + wid * 1024 + i * 256), 4, voff, 0,
                                                   0, 0);
        }
      } else {
#pragma unroll
        for (int i = 0; i < 2; i++) {
          const int row = wid * 16 + 8 * i + (lane >> 3);
          const uint32_t voff = (uint32_t)(row * kLd * 4 + ks * 128 + (lane & 7) * 16);
          dma16(r, lds + wid * 2048 + i * 1024, voff);
        }
      }
    }
  }
  __syncthreads();
  if (threadIdx.x == 0) sink[blockIdx.x] = *(volatile unsigned *)lds;
}

int main() {
  const size_t bytes = (size_t)kRows * kLd * 4;
  float *c;
  unsigned *sink;
  const int blocks = (kRows + kRowsPerBlock - 1) / kRowsPerBlock;
  CHECK(hipMalloc(&c, bytes));
  CHECK(hipMalloc(&sink, blocks * 4));
  CHECK(hipMemset(c, 0x3c, bytes));
  // a 512 MiB buffer written between patterns evicts the Infinity Cache
  char *flush;
  const size_t fbytes = 512ull << 20;
  CHECK(hipMalloc(&flush, fbytes));
  hipEvent_t a, b;
  CHECK(hipEventCreate(&a));
  CHECK(hipEventCreate(&b));
  const char *names[3] = {"dma4_rows", "dma16_rows", "dma16_contig"};
  for (int rep = 0; rep < 2; rep++)
    for (int pat = 0; pat < 3; pat++) {
      CHECK(hipMemset(flush, rep + pat, fbytes));
      CHECK(hipEventRecord(a));
      if (pat == 0) calib<0><<<blocks, kThreads>>>(c, sink);
      if (pat == 1) calib<1><<<blocks, kThreads>>>(c, sink);
      if (pat == 2) calib<2><<<blocks, kThreads>>>(c, sink);
      CHECK(hipGetLastError());
      CHECK(hipEventRecord(b));
      CHECK(hipEventSynchronize(b));
      float ms = 0;
      CHECK(hipEventElapsedTime(&ms, a, b));
      printf("{\"pattern\": \"%s\", \"kernel\": \"calib<%d>\", \"bytes\": %zu, \"ms\": %.3f, \"GBps\": %.1f}\n",
             names[pat], pat, bytes, ms, bytes / (ms * 1e6));
    }
  CHECK(hipDeviceSynchronize());
  return 0;
}
