// Micro-benchmark: per-step latency of the k_solve_reg step skeleton pieces
// (single 512-thread workgroup): barrier only, LDS write+barrier+read,
// + f64 divide.  Prints ns/step and core cycles/step.
#include <hip/hip_runtime.h>
#include <cstdio>

template <int MODE>
__global__ __launch_bounds__(512) void k(double* out, int steps) {
  __shared__ double buf[2][128];
  const int t = threadIdx.x;
  if (t < 128) buf[0][t] = 1.0 + t;
  __syncthreads();
  double v = 1.0 + t * 1e-3;
  const uint64_t w0 = wall_clock64();
  const uint64_t c0 = clock64();
  for (int s = 0; s < steps; ++s) {
    if (MODE >= 1) {
      const double a = buf[s & 1][(t * 7) & 127];
      const double b = buf[s & 1][(t * 13 + s) & 127];
      double inv = 1.0;
      if (MODE >= 2) inv = 1.0 / buf[s & 1][s & 127];
      v -= a * b * inv * 1e-9;
      if (t < 128) buf[(s + 1) & 1][t] = v;
    }
    __syncthreads();
  }
  const uint64_t c1 = clock64();
  const uint64_t w1 = wall_clock64();
  if (t == 0) {
    out[0] = 10.0 * (double)(w1 - w0) / steps;
    out[1] = (double)(c1 - c0) / steps;
  }
  out[2 + t] = v;
}

int main() {
  double* d;
  hipMalloc(&d, 1024 * sizeof(double));
  double h[2];
  const int steps = 10000;
  for (int rep = 0; rep < 2; ++rep) {
    k<0><<<1, 512>>>(d, steps);
    hipMemcpy(h, d, 16, hipMemcpyDeviceToHost);
    printf("barrier only        : %.1f ns/step  %.0f clk/step\n", h[0], h[1]);
    k<1><<<1, 512>>>(d, steps);
    hipMemcpy(h, d, 16, hipMemcpyDeviceToHost);
    printf("lds r/w + barrier   : %.1f ns/step  %.0f clk/step\n", h[0], h[1]);
    k<2><<<1, 512>>>(d, steps);
    hipMemcpy(h, d, 16, hipMemcpyDeviceToHost);
    printf("+ f64 divide        : %.1f ns/step  %.0f clk/step\n", h[0], h[1]);
  }
  return 0;
}
