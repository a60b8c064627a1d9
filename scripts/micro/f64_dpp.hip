// Micro-benchmark: one wave's f64 VALU / DPP costs on gfx950 (clk per op):
// dependent-chain latency and independent issue cost of v_fma_f64,
// v_mov_b64_dpp, v_fmac_f64_dpp (row_newbcast), v_rsq_f64.
#include <hip/hip_runtime.h>
#include <cstdio>

__device__ __forceinline__ double bc3(double v) {
  return __builtin_amdgcn_update_dpp(0.0, v, 0x153, 0xf, 0xf, true);
}

template <int MODE>
__global__ void k(double* out, double x, int iters) {
  double v[8];
#pragma unroll
  for (int u = 0; u < 8; ++u) v[u] = x + (threadIdx.x + u) * 1e-9;
  const double c = 0.999999, d = 1e-7;
  const uint64_t c0 = clock64();
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int u = 0; u < 16; ++u) {
      if (MODE == 0) v[0] = __builtin_fma(v[0], c, d);                 // dep fma
      if (MODE == 1) v[0] = __builtin_amdgcn_rsq(v[0]);                 // dep rsq
      if (MODE == 2) {                                                  // 8 independent fma
#pragma unroll
        for (int w = 0; w < 8; ++w) v[w] = __builtin_fma(v[w], c, d);
      }
      if (MODE == 3) v[0] = __builtin_fma(bc3(v[0]), c, d);            // dep dpp mov + fma
      if (MODE == 4) {                                                  // 8 independent fmac_dpp
        asm volatile("s_nop 1\n"
                     "v_fmac_f64_dpp %0, %8, %9 row_newbcast:3 row_mask:0xf bank_mask:0xf\n"
                     "v_fmac_f64_dpp %1, %8, %9 row_newbcast:4 row_mask:0xf bank_mask:0xf\n"
                     "v_fmac_f64_dpp %2, %8, %9 row_newbcast:5 row_mask:0xf bank_mask:0xf\n"
                     "v_fmac_f64_dpp %3, %8, %9 row_newbcast:6 row_mask:0xf bank_mask:0xf\n"
                     "v_fmac_f64_dpp %4, %8, %9 row_newbcast:7 row_mask:0xf bank_mask:0xf\n"
                     "v_fmac_f64_dpp %5, %8, %9 row_newbcast:8 row_mask:0xf bank_mask:0xf\n"
                     "v_fmac_f64_dpp %6, %8, %9 row_newbcast:9 row_mask:0xf bank_mask:0xf\n"
                     "v_fmac_f64_dpp %7, %8, %9 row_newbcast:10 row_mask:0xf bank_mask:0xf\n"
                     : "+v"(v[0]), "+v"(v[1]), "+v"(v[2]), "+v"(v[3]), "+v"(v[4]), "+v"(v[5]),
                       "+v"(v[6]), "+v"(v[7])
                     : "v"(c), "v"(d));
      }
      if (MODE == 5) {                                                  // 8 independent dpp movs
#pragma unroll
        for (int w = 0; w < 8; ++w) v[w] = bc3(v[w]);
      }
      if (MODE == 6) {                                                  // 8 independent fma (asm, no dpp)
        asm volatile("v_fmac_f64 %0, %8, %9\n v_fmac_f64 %1, %8, %9\n v_fmac_f64 %2, %8, %9\n"
                     "v_fmac_f64 %3, %8, %9\n v_fmac_f64 %4, %8, %9\n v_fmac_f64 %5, %8, %9\n"
                     "v_fmac_f64 %6, %8, %9\n v_fmac_f64 %7, %8, %9\n"
                     : "+v"(v[0]), "+v"(v[1]), "+v"(v[2]), "+v"(v[3]), "+v"(v[4]), "+v"(v[5]),
                       "+v"(v[6]), "+v"(v[7])
                     : "v"(c), "v"(d));
      }
      if (MODE == 7) v[0] = v[0] * c;                                   // dep mul
    }
  }
  const uint64_t c1 = clock64();
  const double per = (MODE == 2 || MODE == 4 || MODE == 5 || MODE == 6) ? 128.0 : 16.0;
  if (threadIdx.x == 0) out[MODE] = (double)(c1 - c0) / (iters * per);
  double s = 0;
#pragma unroll
  for (int u = 0; u < 8; ++u) s += v[u];
  out[16 + threadIdx.x] = s;
}

int main() {
  double* d;
  (void)hipMalloc(&d, 1024 * sizeof(double));
  double h[8];
  for (int rep = 0; rep < 3; ++rep) {
    k<0><<<1, 64>>>(d, 1.0, 2000);
    k<1><<<1, 64>>>(d, 1.5, 2000);
    k<2><<<1, 64>>>(d, 1.0, 2000);
    k<3><<<1, 64>>>(d, 1.0, 2000);
    k<4><<<1, 64>>>(d, 1.0, 2000);
    k<5><<<1, 64>>>(d, 1.0, 2000);
    k<6><<<1, 64>>>(d, 1.0, 2000);
    k<7><<<1, 64>>>(d, 1.0, 2000);
    (void)hipMemcpy(h, d, 64, hipMemcpyDeviceToHost);
    printf("clk/op: dep fma %.1f | dep rsq %.1f | indep fma %.1f | dep dppmov+fma %.1f | indep fmac_dpp %.1f | "
           "indep dppmov %.1f | indep fmac %.1f | dep mul %.1f\n",
           h[0], h[1], h[2], h[3], h[4], h[5], h[6], h[7]);
  }
  return 0;
}
