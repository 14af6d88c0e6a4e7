// pmm_bf16_dsx.hip -- host side of the 256-row (D-split) bf16 kernel
// (pmm_bf16_dsx_kernel.h; instantiations for padded D = 256, 512, 768 in
// pmm_bf16_dsx_ks.hip).
#include "pmm_bf16_dsx_kernel.h"

#include <hip/hip_runtime.h>

namespace pmm {

bool bf16_dsx_supported(int D) { return D % 256 == 0 && D >= 256 && D <= kBf16MaxD; }

size_t gemm_bf16_dsx_lds_bytes(int D) {
  switch (D / 128) {
    case 2: return dsx::Carve<2>::BYTES;
    case 4: return dsx::Carve<4>::BYTES;
    case 6: return dsx::Carve<6>::BYTES;
    default: return 0;
  }
}

hipError_t launch_bf16_dsx_ks2(const GemmF32Args &a, int grid, size_t lds, hipStream_t s);
hipError_t launch_bf16_dsx_ks4(const GemmF32Args &a, int grid, size_t lds, hipStream_t s);
hipError_t launch_bf16_dsx_ks6(const GemmF32Args &a, int grid, size_t lds, hipStream_t s);
hipError_t launch_seed_bf16_dsx_ks2(const GemmF32Args &a, float *S, int ns, hipStream_t s);
hipError_t launch_seed_bf16_dsx_ks4(const GemmF32Args &a, float *S, int ns, hipStream_t s);
hipError_t launch_seed_bf16_dsx_ks6(const GemmF32Args &a, float *S, int ns, hipStream_t s);

hipError_t launch_seed_bf16_dsx(const GemmF32Args &a, float *S, int ns, hipStream_t s) {
  // whole 16-column sample tiles inside the corpus
  if (ns < 16 || ns % 16 != 0 || ns > a.N || !bf16_dsx_supported(a.D) || a.M <= 0) return hipErrorInvalidValue;
  switch (a.D / 128) {
    case 2: return launch_seed_bf16_dsx_ks2(a, S, ns, s);
    case 4: return launch_seed_bf16_dsx_ks4(a, S, ns, s);
    case 6: return launch_seed_bf16_dsx_ks6(a, S, ns, s);
    default: return hipErrorInvalidValue;
  }
}

hipError_t launch_gemm_bf16_dsx(const GemmF32Args &a, int grid, hipStream_t s) {
  const size_t lds = gemm_bf16_dsx_lds_bytes(a.D);
  // the kernel's grid and tile shapes assume: an even number of 128-wide K
  // steps, the selection-based compaction (no LDS scratch), every unit's
  // tiles inside the corpus and every query block inside QB
  if (!bf16_dsx_supported(a.D) || lds == 0 || lds > 160 * 1024 || a.capg > kBf16WsMaxCapg ||
      a.capg < a.k + 64 || a.tps < 1 || (int64_t)a.ntiles * dsx::BN < a.N ||
      (int64_t)(a.ntiles - 1) * dsx::BN >= a.N || (int64_t)a.QB * dsx::BM < a.M || grid < 1 || a.N >= (1 << 27))
    return hipErrorInvalidValue;
  switch (a.D / 128) {
    case 2: return launch_bf16_dsx_ks2(a, grid, lds, s);
    case 4: return launch_bf16_dsx_ks4(a, grid, lds, s);
    case 6: return launch_bf16_dsx_ks6(a, grid, lds, s);
    default: return hipErrorInvalidValue;
  }
}

}  // namespace pmm
