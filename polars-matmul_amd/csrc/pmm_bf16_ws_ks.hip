// pmm_bf16_ws_ks.hip -- one instantiation of the wave-specialised bf16 kernel
// (compiled once per padded-D step count: -DPMM_BF16_KS=1..6, in parallel).
#include "pmm_bf16_ws_kernel.h"

#ifndef PMM_BF16_KS
#error "compile with -DPMM_BF16_KS=<padded D / 128>"
#endif

namespace pmm {

#define PMM_CAT2(a, b) a##b
#define PMM_CAT(a, b) PMM_CAT2(a, b)
hipError_t PMM_CAT(launch_bf16_ws_ks, PMM_BF16_KS)(const GemmF32Args &a, int grid, size_t lds,
                                                  hipStream_t s) {
  if (a.metric == kMetricCosine) return launch_bf16_ws_t<PMM_BF16_KS, kMetricCosine>(a, grid, lds, s);
  if (a.metric == kMetricDot) return launch_bf16_ws_t<PMM_BF16_KS, kMetricDot>(a, grid, lds, s);
  return launch_bf16_ws_t<PMM_BF16_KS, kMetricEuclidean>(a, grid, lds, s);
}

hipError_t PMM_CAT(launch_seed_bf16_ws_ks, PMM_BF16_KS)(const GemmF32Args &a, float *S, int ns,
                                                       hipStream_t s) {
  if (a.metric == kMetricCosine) return launch_seed_bf16_ws_t<PMM_BF16_KS, kMetricCosine>(a, S, ns, s);
  if (a.metric == kMetricDot) return launch_seed_bf16_ws_t<PMM_BF16_KS, kMetricDot>(a, S, ns, s);
  return launch_seed_bf16_ws_t<PMM_BF16_KS, kMetricEuclidean>(a, S, ns, s);
}

}  // namespace pmm
