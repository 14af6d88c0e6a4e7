// Probe: in which order does v_mfma_f32_32x32x2_f32 accumulate its two K
// products (lanes 0-31 carry k=0, lanes 32-63 k=1)?  Prints the result of
// c + p0 + p1 for two crafted cases; see DESIGN.md §2 (bit-exact GEMM order).
#include <hip/hip_runtime.h>
#include <cstdio>
typedef float f32x16 __attribute__((ext_vector_type(16)));
__global__ void probe(const float *p, float c, float *out) {
  const int lane = threadIdx.x;
  const float a = (lane < 32) ? p[0] : p[1];
  f32x16 acc;
  for (int e = 0; e < 16; e++) acc[e] = c;
  acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a, 1.0f, acc, 0, 0, 0);
  out[lane] = acc[0];
}
int main() {
  const float t = 5.9604645e-08f;  // 2^-24
  float cases[2][2] = {{1.0f, t}, {t, 1.0f}};
  float *dp, *dout, h[64];
  hipMalloc(&dp, 8);
  hipMalloc(&dout, 256);
  for (int i = 0; i < 2; i++) {
    hipMemcpy(dp, cases[i], 8, hipMemcpyHostToDevice);
    probe<<<1, 64>>>(dp, t, dout);
    hipMemcpy(h, dout, 256, hipMemcpyDeviceToHost);
    printf("case %d (p0=%g p1=%g c=2^-24): %.9g (1 + %g ulp)\n", i, cases[i][0], cases[i][1], h[0],
           (h[0] - 1.0f) / 1.1920929e-07f);
  }
  printf("k0-first chain => case0 1.0, case1 1+1ulp; k1-first => case0 1+1ulp, case1 1.0; single rounding => both 1+1ulp\n");
  return 0;
}
