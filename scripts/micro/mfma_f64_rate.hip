// Issue rate and dependent latency of v_mfma_f64_16x16x4_f64 on gfx950 vs a
// v_fma_f64 chain: cycles per instruction per wave, 1 and 2 waves per SIMD.
#include <hip/hip_runtime.h>
#include <cstdio>
typedef double d4 __attribute__((ext_vector_type(4)));

template <int NACC>
__global__ void k_mfma(double* out, int iters, unsigned long long* cyc) {
  d4 acc[NACC];
  for (int s = 0; s < NACC; ++s) acc[s] = d4{0, 0, 0, 0};
  double a = threadIdx.x * 1e-3, b = 1.0 + threadIdx.x * 1e-4;
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int s = 0; s < NACC; ++s) acc[s] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc[s], 0, 0, 0);
  }
  double v = 0;
  for (int s = 0; s < NACC; ++s) v += acc[s][0] + acc[s][1] + acc[s][2] + acc[s][3];
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  out[blockIdx.x * blockDim.x + threadIdx.x] = v;
  if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

__global__ void k_fma(double* out, int iters, unsigned long long* cyc) {
  double x[8];
  for (int s = 0; s < 8; ++s) x[s] = threadIdx.x + s;
  const double a = 1.0000001, b = 1e-9;
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int s = 0; s < 8; ++s) x[s] = __builtin_fma(x[s], a, b);
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  double v = 0;
  for (int s = 0; s < 8; ++s) v += x[s];
  out[blockIdx.x * blockDim.x + threadIdx.x] = v;
  if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

int main() {
  double* out;
  unsigned long long* cyc;
  hipMalloc(&out, 1 << 24);
  hipMalloc(&cyc, 1 << 16);
  unsigned long long h[1024];
  const int iters = 2000;
  for (int wpb : {64, 256, 512}) {  // 1 wave; 4 waves (1/SIMD); 8 waves (2/SIMD)
    k_mfma<1><<<1, wpb>>>(out, iters, cyc);
    hipMemcpy(h, cyc, 8, hipMemcpyDeviceToHost);
    printf("mfma f64 16x16x4, 1 acc (dependent), %d waves/WG: %.1f clk/mfma/wave\n", wpb / 64, (double)h[0] / iters);
    k_mfma<4><<<1, wpb>>>(out, iters, cyc);
    hipMemcpy(h, cyc, 8, hipMemcpyDeviceToHost);
    printf("mfma f64 16x16x4, 4 acc, %d waves/WG: %.1f clk/mfma/wave\n", wpb / 64, (double)h[0] / (4.0 * iters));
    k_fma<<<1, wpb>>>(out, iters, cyc);
    hipMemcpy(h, cyc, 8, hipMemcpyDeviceToHost);
    printf("v_fma_f64, 8 chains, %d waves/WG: %.2f clk/fma/wave\n", wpb / 64, (double)h[0] / (8.0 * iters));
  }
  return 0;
}
