// pmm_bf16_ws.hip -- host side of the wave-specialised bf16 kernel
// (pmm_bf16_ws_kernel.h; per-D instantiations in pmm_bf16_ws_ks.hip).
#include "pmm_bf16_ws_kernel.h"

#include <hip/hip_runtime.h>

namespace pmm {

size_t gemm_bf16_ws_lds_bytes(int capg, int D) {
  (void)capg;  // capg <= kBf16WsMaxCapg: compactions select in registers
  switch (D / 128) {
    case 1: return ws::Carve<1>::BYTES;
    case 2: return ws::Carve<2>::BYTES;
    case 3: return ws::Carve<3>::BYTES;
    case 4: return ws::Carve<4>::BYTES;
    case 5: return ws::Carve<5>::BYTES;
    default: return ws::Carve<6>::BYTES;
  }
}

hipError_t launch_bf16_ws_ks1(const GemmF32Args &a, int grid, size_t lds, hipStream_t s);
hipError_t launch_bf16_ws_ks2(const GemmF32Args &a, int grid, size_t lds, hipStream_t s);
hipError_t launch_bf16_ws_ks3(const GemmF32Args &a, int grid, size_t lds, hipStream_t s);
hipError_t launch_bf16_ws_ks4(const GemmF32Args &a, int grid, size_t lds, hipStream_t s);
hipError_t launch_bf16_ws_ks5(const GemmF32Args &a, int grid, size_t lds, hipStream_t s);
hipError_t launch_bf16_ws_ks6(const GemmF32Args &a, int grid, size_t lds, hipStream_t s);

hipError_t launch_seed_bf16_ws_ks1(const GemmF32Args &a, float *S, int ns, hipStream_t s);
hipError_t launch_seed_bf16_ws_ks2(const GemmF32Args &a, float *S, int ns, hipStream_t s);
hipError_t launch_seed_bf16_ws_ks3(const GemmF32Args &a, float *S, int ns, hipStream_t s);
hipError_t launch_seed_bf16_ws_ks4(const GemmF32Args &a, float *S, int ns, hipStream_t s);
hipError_t launch_seed_bf16_ws_ks5(const GemmF32Args &a, float *S, int ns, hipStream_t s);
hipError_t launch_seed_bf16_ws_ks6(const GemmF32Args &a, float *S, int ns, hipStream_t s);

hipError_t launch_seed_bf16_ws(const GemmF32Args &a, float *S, int ns, hipStream_t s) {
  // whole 32-column sample tiles inside the corpus, whole K-steps
  if (ns < 32 || ns % 32 != 0 || ns > a.N || a.D % kBf16DAlign != 0 || a.M <= 0) return hipErrorInvalidValue;
  switch (a.D / 128) {
    case 1: return launch_seed_bf16_ws_ks1(a, S, ns, s);
    case 2: return launch_seed_bf16_ws_ks2(a, S, ns, s);
    case 3: return launch_seed_bf16_ws_ks3(a, S, ns, s);
    case 4: return launch_seed_bf16_ws_ks4(a, S, ns, s);
    case 5: return launch_seed_bf16_ws_ks5(a, S, ns, s);
    case 6: return launch_seed_bf16_ws_ks6(a, S, ns, s);
    default: return hipErrorInvalidValue;
  }
}

hipError_t launch_gemm_bf16_ws(const GemmF32Args &a, int grid, hipStream_t s) {
  const size_t lds = gemm_bf16_ws_lds_bytes(a.capg, a.D);
  // the kernel's grid and tile shapes assume: whole 128-wide K-steps, a
  // capacity the LDS carve holds, and every unit's tiles inside the corpus
  if (lds > 160 * 1024 || a.D % kBf16DAlign != 0 || a.capg > kBf16WsMaxCapg || a.tps < 1 ||
      (int64_t)a.ntiles * ws::BN < a.N || (int64_t)a.QB * ws::BM < a.M)
    return hipErrorInvalidValue;
  switch (a.D / 128) {
    case 1: return launch_bf16_ws_ks1(a, grid, lds, s);
    case 2: return launch_bf16_ws_ks2(a, grid, lds, s);
    case 3: return launch_bf16_ws_ks3(a, grid, lds, s);
    case 4: return launch_bf16_ws_ks4(a, grid, lds, s);
    case 5: return launch_bf16_ws_ks5(a, grid, lds, s);
    case 6: return launch_bf16_ws_ks6(a, grid, lds, s);
    default: return hipErrorInvalidValue;
  }
}

}  // namespace pmm
