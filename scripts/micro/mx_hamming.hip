// Micro-check of the Hamming-on-matrix-cores idea before it goes into
// csrc/hamming.hip: one v_mfma_scale_f32_16x16x128_f8f6f4 pair (fp4 e2m1
// operands, K = 256 bits) computes, for 16 queries x 16 train rows,
//   key(i, j) = ((pt_j - 2 popcount(q_i & t_j) + 256) << 14) + j
// exactly in f32 (integers < 2^24), with query bits as fp4 +1.0 (0x2), train
// bits as fp4 -2.0 (0xC) scaled by 2^14 (E8M0 141), and the accumulator
// initialised to (pt_j + 256) * 2^14 + j.  Assumed operand map (any k
// permutation shared by A and B is harmless): lane l holds row / column l & 15
// and bits [32 (l >> 4), +32) of each 128-bit half as 32 nibbles, low nibble
// first; C/D: row 4 (l >> 4) + r, column l & 15.  Prints mismatches vs the CPU.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>

typedef int v8i __attribute__((ext_vector_type(8)));
typedef float v4f __attribute__((ext_vector_type(4)));

__device__ uint32_t spread8(uint32_t b, uint32_t nib) {  // 8 bits -> 8 nibbles (nib per set bit)
  uint32_t x = b & 0xFFu;
  x = (x | (x << 12)) & 0x000F000Fu;
  x = (x | (x << 6)) & 0x03030303u;
  x = (x | (x << 3)) & 0x11111111u;
  return x * nib;
}

__global__ void k(const uint32_t* q, const uint32_t* t, const int* pt, float* out) {
  const int l = threadIdx.x, r = l & 15, g = l >> 4;
  v4f acc;
  const float init = (float)((pt[r] + 256) * 16384 + r);
  acc[0] = acc[1] = acc[2] = acc[3] = init;  // column l & 15 of every row
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const uint32_t qa = q[r * 8 + 4 * h + g], tb = t[r * 8 + 4 * h + g];
    v8i A = {0, 0, 0, 0, 0, 0, 0, 0}, B = A;
    for (int d = 0; d < 4; ++d) {
      A[d] = (int)spread8(qa >> (8 * d), 0x2u);
      B[d] = (int)spread8(tb >> (8 * d), 0xCu);
    }
    acc = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(A, B, acc, 4, 4, 0, 127, 0, 141);
  }
  for (int i = 0; i < 4; ++i) out[(4 * g + i) * 16 + r] = acc[i];
}

int main() {
  uint32_t hq[128], ht[128];
  int hpt[16];
  srand(7);
  for (int i = 0; i < 128; ++i) {
    hq[i] = (uint32_t)rand() ^ ((uint32_t)rand() << 16);
    ht[i] = (uint32_t)rand() ^ ((uint32_t)rand() << 16);
  }
  for (int j = 0; j < 16; ++j) {
    hpt[j] = 0;
    for (int w = 0; w < 8; ++w) hpt[j] += __builtin_popcount(ht[j * 8 + w]);
  }
  uint32_t *dq, *dt;
  int* dpt;
  float* dout;
  hipMalloc(&dq, sizeof(hq));
  hipMalloc(&dt, sizeof(ht));
  hipMalloc(&dpt, sizeof(hpt));
  hipMalloc(&dout, 256 * sizeof(float));
  hipMemcpy(dq, hq, sizeof(hq), hipMemcpyHostToDevice);
  hipMemcpy(dt, ht, sizeof(ht), hipMemcpyHostToDevice);
  hipMemcpy(dpt, hpt, sizeof(hpt), hipMemcpyHostToDevice);
  k<<<1, 64>>>(dq, dt, dpt, dout);
  float h[256];
  hipMemcpy(h, dout, sizeof(h), hipMemcpyDeviceToHost);
  int bad = 0;
  for (int i = 0; i < 16; ++i)
    for (int j = 0; j < 16; ++j) {
      int pa = 0;
      for (int w = 0; w < 8; ++w) pa += __builtin_popcount(hq[i * 8 + w] & ht[j * 8 + w]);
      const double want = (double)(hpt[j] - 2 * pa + 256) * 16384.0 + j;
      if ((double)h[i * 16 + j] != want) {
        if (bad < 8) printf("mismatch q%d t%d: got %.1f want %.1f\n", i, j, h[i * 16 + j], want);
        ++bad;
      }
    }
  printf("mx_hamming: %d mismatches of 256\n", bad);
  return bad != 0;
}
