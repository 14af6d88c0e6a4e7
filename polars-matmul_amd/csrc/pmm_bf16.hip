// pmm_bf16.hip -- bf16 compute path of the fused top-k (PMM_COMPUTE_BF16;
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
#include "pmm_bf16_kernel.h"

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace pmm {

size_t gemm_bf16_lds_bytes(int capg, int nst) {
  return (size_t)OFF_RING + (size_t)nst * STAGE + (size_t)NW * capg * 8;
}

// ---------------------------------------------------------------------------
// f32 -> bf16 with zero padding: one thread per 8 output elements.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void f32_to_bf16_kernel(const float *__restrict__ src,
                                                          int64_t rows, int64_t d, int64_t lds,
                                                          uint16_t *__restrict__ dst, int64_t ldd) {
  const int64_t per_row = ldd >> 3;
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= rows * per_row) return;
  const int64_t r = t / per_row;
  const int64_t c0 = (t - r * per_row) * 8;
  bf16x8 v;
#pragma unroll
  for (int j = 0; j < 8; j++) {
    const int64_t c = c0 + j;
    // plain cast: v_cvt_pk_bf16_f32, round to nearest even, NaN stays NaN
    v[j] = (c < d) ? (__bf16)src[r * lds + c] : (__bf16)0.0f;
  }
  *(bf16x8 *)(dst + r * ldd + c0) = v;
}

hipError_t launch_f32_to_bf16(const float *src, int64_t rows, int64_t d, int64_t lds, uint16_t *dst,
                              int64_t ldd, hipStream_t s) {
  if (rows <= 0) return hipSuccess;
  const int64_t threads = rows * (ldd >> 3);
  f32_to_bf16_kernel<<<(unsigned)((threads + 255) / 256), 256, 0, s>>>(src, rows, d, lds, dst, ldd);
  return hipGetLastError();
}

// bf16 -> f32 (exact widening) with zero padding to ldd: one thread per element
__global__ __launch_bounds__(256) void bf16_to_f32_kernel(const uint16_t *__restrict__ src, int64_t rows,
                                                          int64_t d, int64_t lds, float *__restrict__ dst,
                                                          int64_t ldd) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= rows * ldd) return;
  const int64_t r = t / ldd, c = t - r * ldd;
  dst[t] = (c < d) ? __uint_as_float((uint32_t)src[r * lds + c] << 16) : 0.0f;
}

hipError_t launch_bf16_to_f32(const uint16_t *src, int64_t rows, int64_t d, int64_t lds, float *dst, int64_t ldd,
                              hipStream_t s) {
  if (rows <= 0) return hipSuccess;
  const int64_t threads = rows * ldd;
  bf16_to_f32_kernel<<<(unsigned)((threads + 255) / 256), 256, 0, s>>>(src, rows, d, lds, dst, ldd);
  return hipGetLastError();
}

hipError_t launch_norms_bf16(const uint16_t *a, int64_t rows, int64_t d, int64_t ld, int squared,
                             float *out, float *inv, hipStream_t s) {
  if (rows <= 0) return hipSuccess;
  const int64_t threads = rows * 8;
  norms_kernel<float, __bf16><<<(unsigned)((threads + 255) / 256), 256, 0, s>>>(
      (const __bf16 *)a, rows, d, ld, squared, out, inv);
  return hipGetLastError();
}

// per-KS instantiations (pmm_bf16_ks.hip)
hipError_t launch_bf16_ks1(const GemmF32Args &a, int grid, size_t lds, hipStream_t s);
hipError_t launch_bf16_ks2(const GemmF32Args &a, int grid, size_t lds, hipStream_t s);
hipError_t launch_bf16_ks3(const GemmF32Args &a, int grid, size_t lds, hipStream_t s);
hipError_t launch_bf16_ks4(const GemmF32Args &a, int grid, size_t lds, hipStream_t s);
hipError_t launch_bf16_ks5(const GemmF32Args &a, int grid, size_t lds, hipStream_t s);
hipError_t launch_bf16_ks6(const GemmF32Args &a, int grid, size_t lds, hipStream_t s);

hipError_t launch_gemm_bf16(const GemmF32Args &a, int grid, hipStream_t s) {
  const size_t lds = gemm_bf16_lds_bytes(a.capg, a.nst);
  if (lds > 160 * 1024 || a.D % kBf16DAlign != 0) return hipErrorInvalidValue;
  switch (a.D / 128) {
    case 1: return launch_bf16_ks1(a, grid, lds, s);
    case 2: return launch_bf16_ks2(a, grid, lds, s);
    case 3: return launch_bf16_ks3(a, grid, lds, s);
    case 4: return launch_bf16_ks4(a, grid, lds, s);
    case 5: return launch_bf16_ks5(a, grid, lds, s);
    case 6: return launch_bf16_ks6(a, grid, lds, s);
    default: return hipErrorInvalidValue;
  }
}

}  // namespace pmm
