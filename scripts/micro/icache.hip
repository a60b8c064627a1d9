// Micro-benchmark: cost of running cold code on gfx950.  One wave runs the
// same straight-line block three times in a loop (pass 0 cold, passes 1-2
// warm); the wall-clock (100 MHz) and shader-clock time of each pass.
//   blocks: 4096 x v_add_f64 (VOP3, 8 B: 32 KB), 4096 x v_mov_b32 (VOP1, 4 B: 16 KB),
//   1024 x v_add_f64 (8 KB)
#include <hip/hip_runtime.h>
#include <cstdio>

template <int MODE>
__global__ void k(unsigned long long* out) {
#pragma unroll 1
  for (int it = 0; it < 3; ++it) {
    const unsigned long long w0 = wall_clock64(), c0 = clock64();
    if (MODE == 0) asm volatile(".rept 4096\n v_add_f64 v[2:3], v[4:5], v[6:7]\n .endr" ::: "v2", "v3");
    if (MODE == 1) asm volatile(".rept 4096\n v_mov_b32 v2, v4\n .endr" ::: "v2");
    if (MODE == 2) asm volatile(".rept 1024\n v_add_f64 v[2:3], v[4:5], v[6:7]\n .endr" ::: "v2", "v3");
    const unsigned long long c1 = clock64(), w1 = wall_clock64();
    if (threadIdx.x == 0) {
      out[2 * it] = w1 - w0;
      out[2 * it + 1] = c1 - c0;
    }
  }
}

int main() {
  unsigned long long* d;
  hipMalloc(&d, 6 * sizeof(unsigned long long));
  const char* names[3] = {"4096 x v_add_f64 (32 KB)", "4096 x v_mov_b32 (16 KB)", "1024 x v_add_f64 (8 KB)"};
  for (int rep = 0; rep < 2; ++rep)
    for (int m = 0; m < 3; ++m) {
      if (m == 0) k<0><<<1, 64>>>(d);
      if (m == 1) k<1><<<1, 64>>>(d);
      if (m == 2) k<2><<<1, 64>>>(d);
      unsigned long long h[6];
      hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
      printf("launch %d %-26s pass0 %7.2f us %6llu clk | pass1 %7.2f us %6llu clk | pass2 %7.2f us %6llu clk\n",
             rep, names[m], h[0] * 0.01, h[1], h[2] * 0.01, h[3], h[4] * 0.01, h[5]);
    }
  return 0;
}
