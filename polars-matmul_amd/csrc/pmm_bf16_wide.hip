// pmm_bf16_wide.hip -- host side of the 256-query-row bf16 kernel
// (pmm_bf16_wide_kernel.h; per-D instantiations in pmm_bf16_wide_ks.hip).
#include "pmm_bf16_wide_kernel.h"

#include <hip/hip_runtime.h>

namespace pmm {

size_t gemm_bf16_wide_lds_bytes(int D) {
  switch (D / 128) {
    case 1: return wd::Carve<1>::BYTES;
    case 2: return wd::Carve<2>::BYTES;
    case 3: return wd::Carve<3>::BYTES;
    case 4: return wd::Carve<4>::BYTES;
    case 5: return wd::Carve<5>::BYTES;
    default: return wd::Carve<6>::BYTES;
  }
}

hipError_t launch_bf16_wide_ks1(const GemmF32Args &a, int grid, size_t lds, hipStream_t s);
hipError_t launch_bf16_wide_ks2(const GemmF32Args &a, int grid, size_t lds, hipStream_t s);
hipError_t launch_bf16_wide_ks3(const GemmF32Args &a, int grid, size_t lds, hipStream_t s);
hipError_t launch_bf16_wide_ks4(const GemmF32Args &a, int grid, size_t lds, hipStream_t s);
hipError_t launch_bf16_wide_ks5(const GemmF32Args &a, int grid, size_t lds, hipStream_t s);
hipError_t launch_bf16_wide_ks6(const GemmF32Args &a, int grid, size_t lds, hipStream_t s);

hipError_t launch_gemm_bf16_wide(const GemmF32Args &a, int grid, hipStream_t s) {
  const size_t lds = gemm_bf16_wide_lds_bytes(a.D);
  // the kernel's grid and tile shapes assume: whole 128-wide K-steps, the
  // selection-based compaction (no LDS scratch), every unit's tiles inside
  // the corpus, and every query block inside QB
  if (lds > 160 * 1024 || a.D % kBf16DAlign != 0 || a.D > kBf16MaxD || a.capg > kBf16WideMaxCapg ||
      a.capg < a.k + 64 || a.tps < 1 || (int64_t)a.ntiles * wd::BN < a.N ||
      (int64_t)(a.ntiles - 1) * wd::BN >= a.N || (int64_t)a.QB * wd::BM < a.M || grid < 1)
    return hipErrorInvalidValue;
  switch (a.D / 128) {
    case 1: return launch_bf16_wide_ks1(a, grid, lds, s);
    case 2: return launch_bf16_wide_ks2(a, grid, lds, s);
    case 3: return launch_bf16_wide_ks3(a, grid, lds, s);
    case 4: return launch_bf16_wide_ks4(a, grid, lds, s);
    case 5: return launch_bf16_wide_ks5(a, grid, lds, s);
    case 6: return launch_bf16_wide_ks6(a, grid, lds, s);
    default: return hipErrorInvalidValue;
  }
}

}  // namespace pmm
