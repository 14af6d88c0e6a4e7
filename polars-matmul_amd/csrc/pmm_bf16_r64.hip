// pmm_bf16_r64.hip -- host side of the one-wave-per-SIMD 256-row bf16 kernel
// (pmm_bf16_r64_kernel.h; one instantiation per padded-D step count in
// pmm_bf16_r64_ks.hip).
#include "pmm_bf16_r64_kernel.h"

#include <hip/hip_runtime.h>

namespace pmm {

size_t gemm_bf16_r64_lds_bytes(int D) {
  switch (D / 128) {
    case 1: return r64::Carve<1>::BYTES;
    case 2: return r64::Carve<2>::BYTES;
    case 3: return r64::Carve<3>::BYTES;
    case 4: return r64::Carve<4>::BYTES;
    case 5: return r64::Carve<5>::BYTES;
    case 6: return r64::Carve<6>::BYTES;
    default: return 0;
  }
}

hipError_t launch_bf16_r64_ks1(const GemmF32Args &a, int grid, size_t lds, hipStream_t s);
hipError_t launch_bf16_r64_ks2(const GemmF32Args &a, int grid, size_t lds, hipStream_t s);
hipError_t launch_bf16_r64_ks3(const GemmF32Args &a, int grid, size_t lds, hipStream_t s);
hipError_t launch_bf16_r64_ks4(const GemmF32Args &a, int grid, size_t lds, hipStream_t s);
hipError_t launch_bf16_r64_ks5(const GemmF32Args &a, int grid, size_t lds, hipStream_t s);
hipError_t launch_bf16_r64_ks6(const GemmF32Args &a, int grid, size_t lds, hipStream_t s);

hipError_t launch_gemm_bf16_r64(const GemmF32Args &a, int grid, hipStream_t s) {
  const size_t lds = (a.D % 128 == 0) ? gemm_bf16_r64_lds_bytes(a.D) : 0;
  // the kernel's shapes: whole 128-wide K steps, its compaction's keys per
  // lane (capg <= kBf16R64MaxCapg), every unit's tiles inside the corpus, every
  // query block inside QB, and a global column that fits the queue item's
  // 26 bits
  if (lds == 0 || lds > 160 * 1024 || a.capg > kBf16R64MaxCapg || a.capg < a.k + 64 || a.tps < 1 ||
      (int64_t)a.ntiles * r64::BN < a.N || (int64_t)(a.ntiles - 1) * r64::BN >= a.N ||
      (int64_t)a.QB * r64::BM < a.M || grid < 1 || a.N >= (1 << 26))
    return hipErrorInvalidValue;
  switch (a.D / 128) {
    case 1: return launch_bf16_r64_ks1(a, grid, lds, s);
    case 2: return launch_bf16_r64_ks2(a, grid, lds, s);
    case 3: return launch_bf16_r64_ks3(a, grid, lds, s);
    case 4: return launch_bf16_r64_ks4(a, grid, lds, s);
    case 5: return launch_bf16_r64_ks5(a, grid, lds, s);
    case 6: return launch_bf16_r64_ks6(a, grid, lds, s);
    default: return hipErrorInvalidValue;
  }
}

}  // namespace pmm
