// Micro-benchmark: dependent-chain latency of f64 VALU ops (one wave).
#include <hip/hip_runtime.h>
#include <cstdio>

template <int MODE>
__global__ void k(double* out, double x, int iters) {
  double v = x + threadIdx.x * 1e-9;
  const uint64_t c0 = clock64();
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int u = 0; u < 16; ++u) {
      if (MODE == 0) v = __builtin_fma(v, 0.999999, 1e-7);
      if (MODE == 1) v = __builtin_amdgcn_rcp(v);
      if (MODE == 2) v = v * 1.0000001;
      if (MODE == 3) v = __builtin_fmaf((float)v, 0.999f, 1e-3f);
    }
  }
  const uint64_t c1 = clock64();
  if (threadIdx.x == 0) out[MODE] = (double)(c1 - c0) / (iters * 16.0);
  out[8 + threadIdx.x] = v;
}

int main() {
  double* d;
  (void)hipMalloc(&d, 1024 * sizeof(double));
  double h[4];
  for (int rep = 0; rep < 2; ++rep) {
    k<0><<<1, 64>>>(d, 1.0, 1000);
    k<1><<<1, 64>>>(d, 1.5, 1000);
    k<2><<<1, 64>>>(d, 1.0, 1000);
    k<3><<<1, 64>>>(d, 1.0, 1000);
    (void)hipMemcpy(h, d, 32, hipMemcpyDeviceToHost);
    printf("dep latency (clk): fma_f64 %.1f  rcp_f64 %.1f  mul_f64 %.1f  fma_f32 %.1f\n", h[0], h[1],
           h[2], h[3]);
  }
  return 0;
}
