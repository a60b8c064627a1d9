// Micro-benchmark: cost of cold code after the caches were flushed by other
// work (a 1 GiB memset between launches, like the LM kernels between two
// solves).  One wave runs a straight-line block three times (pass 0 cold,
// passes 1-2 warm), with and without the memset before the launch.
#include <hip/hip_runtime.h>
#include <cstdio>

template <int MODE>
__global__ void k(unsigned long long* out) {
#pragma unroll 1
  for (int it = 0; it < 3; ++it) {
    const unsigned long long w0 = wall_clock64();
    if (MODE == 0) asm volatile(".rept 128\n v_add_f64 v[2:3], v[4:5], v[6:7]\n .endr" ::: "v2", "v3");
    if (MODE == 1) asm volatile(".rept 1024\n v_add_f64 v[2:3], v[4:5], v[6:7]\n .endr" ::: "v2", "v3");
    if (MODE == 2) asm volatile(".rept 4096\n v_add_f64 v[2:3], v[4:5], v[6:7]\n .endr" ::: "v2", "v3");
    const unsigned long long w1 = wall_clock64();
    if (threadIdx.x == 0) out[it] = w1 - w0;
  }
}

int main() {
  unsigned long long* d;
  void* big;
  const size_t nbig = size_t(1) << 30;
  (void)hipMalloc(&d, 3 * sizeof(unsigned long long));
  (void)hipMalloc(&big, nbig);
  const char* names[3] = {"128 x v_add_f64 (1 KB)", "1024 x v_add_f64 (8 KB)", "4096 x v_add_f64 (32 KB)"};
  for (int rep = 0; rep < 3; ++rep)
    for (int flush = 0; flush < 2; ++flush)
      for (int m = 0; m < 3; ++m) {
        if (flush) (void)hipMemsetAsync(big, rep + m, nbig);
        if (m == 0) k<0><<<1, 64>>>(d);
        if (m == 1) k<1><<<1, 64>>>(d);
        if (m == 2) k<2><<<1, 64>>>(d);
        unsigned long long h[3];
        (void)hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
        printf("rep %d %-8s %-26s pass0 %6.2f us | pass1 %6.2f us | pass2 %6.2f us\n", rep,
               flush ? "flushed" : "warm", names[m], h[0] * 0.01, h[1] * 0.01, h[2] * 0.01);
      }
  return 0;
}
