// Brute-force Hamming kNN-2 matcher + Lowe ratio test, gfx950.
//
// Replaces cv2.FlannBasedMatcher(LSH).knnMatch(k=2) + the 0.7 ratio loop of
// /root/reference/keypoint.py:40-51, Point3D.py:35-49, tracking.py:14-30.
//
// Design (integer-VALU bound, see DESIGN.md "Hamming matcher"):
//   * one workgroup = 8 waves x 64 lanes x QPL queries of ONE batch item; every
//     wave holds the same 64 x QPL query descriptors in VGPRs (8 dwords each)
//     and takes every 8th train row, so a 2000-row train set keeps 8 waves busy
//     per 128 queries; the 8 partial top-2 lists are merged through LDS;
//   * a train row is uniform across the wave: it is read with s_load_dwordx8
//     (scalar cache, 8 rows in flight) straight into SGPR operands -- no LDS
//     staging and no per-lane vector traffic for the train set;
//   * per (query, train) pair: 8 v_xor + 8 v_bcnt (popcount with accumulate)
//     + 1 v_lshl_or to form key = dist<<16 | train_idx, then the running top-2
//     is k2 = med3(k1, k2, key), k1 = min(k1, key): branch-free, and the
//     packed key breaks distance ties by the lower train index (BFMatcher rule).
#include "common.hpp"

namespace {

constexpr int kWG = 512;
constexpr int kWaves = kWG / kWave;     // 8: the train rows of a chunk are split over the waves
constexpr int kQPL = 2;                 // queries per lane
constexpr int kQPerWG = kWave * kQPL;   // 128 queries per workgroup (every wave holds all of them)
constexpr uint32_t kNone = 0xFFFFFFFFu;
int g_knn2_valu = 0;  // slam_hamming_force_valu

// popcount-accumulate: v_bcnt_u32_b32 d, x, acc (one VALU op per dword; the
// compiler would otherwise split the sum into v_add3 trees)
__device__ __forceinline__ uint32_t bcnt_acc(uint32_t x, uint32_t acc) {
  uint32_t d;
  asm("v_bcnt_u32_b32 %0, %1, %2" : "=v"(d) : "v"(x), "v"(acc));
  return d;
}

__device__ __forceinline__ uint32_t hd8(const uint32_t (&a)[8], const uint4& x,
                                        const uint4& y) {
  uint32_t d = bcnt_acc(a[0] ^ x.x, 0u);
  d = bcnt_acc(a[1] ^ x.y, d);
  d = bcnt_acc(a[2] ^ x.z, d);
  d = bcnt_acc(a[3] ^ x.w, d);
  d = bcnt_acc(a[4] ^ y.x, d);
  d = bcnt_acc(a[5] ^ y.y, d);
  d = bcnt_acc(a[6] ^ y.z, d);
  d = bcnt_acc(a[7] ^ y.w, d);
  return d;
}

__device__ __forceinline__ uint32_t umed3(uint32_t a, uint32_t b, uint32_t c) {
  // LLVM folds this min/max pattern into a single v_med3_u32.
  return max(min(a, b), min(max(a, b), c));
}

// Top-2 keys (k1 <= k2) merged with another top-2 (a1 <= a2).
__device__ __forceinline__ void merge2(uint32_t& k1, uint32_t& k2, uint32_t a1, uint32_t a2) {
  const uint32_t n1 = min(k1, a1);
  const uint32_t n2 = min(max(k1, a1), min(k2, a2));
  k1 = n1;
  k2 = n2;
}

// Workgroup = 128 queries of one batch item; its 8 waves each take every 8th
// train row of the LDS chunk (so a 2000-row train set keeps 8 waves busy per
// 128 queries and a C2 batch fills the chip), then the wave partials are
// merged through LDS.  Keys dist << 16 | train_idx make the result
// independent of the processing order (ties -> lower train index).
__global__ __launch_bounds__(kWG) void knn2_kernel(
    const uint4* __restrict__ q, const int32_t* __restrict__ nq_arr, int q_cap,
    const uint4* __restrict__ t, const int32_t* __restrict__ nt_arr, int t_cap,
    int tiles_per_item, int2* __restrict__ idx2, int2* __restrict__ dist2,
    uint8_t* __restrict__ good) {
  __shared__ uint32_t part[kWaves][2][kQPerWG];
  const int item = blockIdx.x / tiles_per_item;
  const int tile = blockIdx.x - item * tiles_per_item;
  const int nq = min(max(nq_arr[item], 0), q_cap);
  const int nt = min(max(nt_arr[item], 0), t_cap);
  const int q0 = tile * kQPerWG;
  if (q0 >= nq) return;  // uniform over the workgroup
  const int lane = threadIdx.x & (kWave - 1);
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x / kWave);  // uniform: scalar loop

  const uint4* qb = q + (size_t)item * q_cap * 2;
  const uint4* tb = t + (size_t)item * t_cap * 2;

  uint32_t qa[kQPL][8];
  uint32_t k1[kQPL], k2[kQPL];
#pragma unroll
  for (int s = 0; s < kQPL; ++s) {
    const int qi = q0 + s * kWave + lane;
    uint4 a = make_uint4(0, 0, 0, 0), b = a;
    if (qi < nq) {
      a = qb[2 * qi];
      b = qb[2 * qi + 1];
    }
    qa[s][0] = a.x; qa[s][1] = a.y; qa[s][2] = a.z; qa[s][3] = a.w;
    qa[s][4] = b.x; qa[s][5] = b.y; qa[s][6] = b.z; qa[s][7] = b.w;
    k1[s] = kNone;
    k2[s] = kNone;
  }

  // Train rows are uniform across the wave: read them with scalar loads
  // (s_load_dwordx8 through the scalar cache) straight into SGPR operands of
  // the VALU xors -- no LDS staging and no per-lane vector traffic.
  // kRowsAhead rows per step, all loads issued before the first use, so the
  // scalar-cache latency overlaps the previous rows' VALU work.
  constexpr int kRowsAhead = 8;
  int j = wid;
  for (; j + (kRowsAhead - 1) * kWaves < nt; j += kRowsAhead * kWaves) {
    uint4 x[kRowsAhead], y[kRowsAhead];
#pragma unroll
    for (int u = 0; u < kRowsAhead; ++u) {
      x[u] = tb[2 * (j + u * kWaves)];
      y[u] = tb[2 * (j + u * kWaves) + 1];
    }
#pragma unroll
    for (int u = 0; u < kRowsAhead; ++u) {
      const uint32_t jj = (uint32_t)(j + u * kWaves);
#pragma unroll
      for (int s = 0; s < kQPL; ++s) {
        const uint32_t key = (hd8(qa[s], x[u], y[u]) << 16) | jj;
        k2[s] = umed3(k1[s], k2[s], key);
        k1[s] = min(k1[s], key);
      }
    }
  }
  for (; j < nt; j += kWaves) {
    const uint4 x = tb[2 * j];
    const uint4 y = tb[2 * j + 1];
    const uint32_t jj = (uint32_t)j;
#pragma unroll
    for (int s = 0; s < kQPL; ++s) {
      const uint32_t key = (hd8(qa[s], x, y) << 16) | jj;
      k2[s] = umed3(k1[s], k2[s], key);
      k1[s] = min(k1[s], key);
    }
  }
  // merge the wave partials
#pragma unroll
  for (int s = 0; s < kQPL; ++s) {
    part[wid][0][s * kWave + lane] = k1[s];
    part[wid][1][s * kWave + lane] = k2[s];
  }
  __syncthreads();
  if (threadIdx.x >= kQPerWG) return;
  const int ql = threadIdx.x;  // local query of this workgroup
  uint32_t m1 = part[0][0][ql], m2 = part[0][1][ql];
#pragma unroll
  for (int w = 1; w < kWaves; ++w) merge2(m1, m2, part[w][0][ql], part[w][1][ql]);
  const int qi = q0 + ql;
  if (qi >= nq) return;
  const size_t o = (size_t)item * q_cap + qi;
  int2 id, ds;
  id.x = m1 == kNone ? -1 : (int)(m1 & 0xFFFFu);
  ds.x = m1 == kNone ? -1 : (int)(m1 >> 16);
  id.y = m2 == kNone ? -1 : (int)(m2 & 0xFFFFu);
  ds.y = m2 == kNone ? -1 : (int)(m2 >> 16);
  idx2[o] = id;
  dist2[o] = ds;
  good[o] = (m2 != kNone && 10 * ds.x < 7 * ds.y) ? 1 : 0;
}

// ---------------------------------------------------------------- matrix-core matcher
// The same kNN-2 on the fp4 matrix cores (v_mfma_scale_f32_16x16x128_f8f6f4,
// e2m1 operands, K = 128 bits per instruction, two per 256-bit descriptor).
// With query bits as +1.0 and train bits as -2.0 x 2^14 (E8M0 block scale
// 141), and the accumulator of column j initialised to (pt_j + 256) 2^14 + j
// (pt_j = popcount of train row j), one 16 x 16 tile of the product is
//   key(i, j) = (pt_j - 2 popcount(q_i & t_j) + 256) 2^14 + j
//             = (H(q_i, t_j) - pq_i + 256) 2^14 + j,
// every term an integer below 2^24, so the f32 accumulation is exact and its
// order immaterial.  For a fixed query the key orders train rows exactly as
// the VALU kernel's dist << 16 | j (Hamming distance, ties to the lower
// index); the running top-2 is v_min_f32 / v_med3_f32 on the keys.
//   * one workgroup = 64 queries (4 blocks of 16) x the whole train set; its
//     4 waves hold the same query fragments in registers and take every 4th
//     step of 16 train rows (4 waves per SIMD at the C2 batch: the MFMA /
//     load latency of one wave hides behind the others), each lane loading
//     its column's whole 32-byte row 2 steps ahead (popcount in-lane); the
//     wave partials are merged over the 16 column-lanes (shuffles), then over
//     the 4 waves through LDS in wave order (keys are unique: the order is
//     immaterial anyway);
//   * bits -> fp4 nibbles in registers, no tables: operand dword d of a
//     32-bit descriptor word w is ((w >> d) & 0x11111111) times the nibble
//     (+1.0 = 0x2, -2.0 = 0xC), i.e. nibble k of dword d is bit 4k + d -- a
//     permutation of K shared by A and B, so every product pairs the same bit
//     of query and train row (2-3 VALU ops per dword; the round-3 byte tables
//     cost 2.8 LDS bank-conflict cycles per lookup);
//   * operand map (scripts/micro/mx_hamming.hip, exact on the GPU): lane l
//     holds row / column l & 15 and bits [32 (l >> 4), +32) of each 128-bit
//     half as 32 nibbles (any k order shared by A and B is harmless); C/D:
//     row 4 (l >> 4) + r, column l & 15 -- each lane keeps a partial top-2 of
//     4 queries per block over the columns = l mod 16;
//   * XCD-aware block order: the workgroups of one batch item are dealt to ONE
//     XCD (blocks b and b + 8 share an XCD), so each item's train set is
//     fetched into one L2 instead of all eight.
// Train row index < 2^14 (t_cap <= 16383; larger sets take knn2_kernel).
#ifndef SLAM_MX_WG
#define SLAM_MX_WG 256
#endif
constexpr int kMxWG = SLAM_MX_WG;          // 4 waves: train steps dealt round-robin
constexpr int kMxWaves = kMxWG / kWave;
// Query blocks of 16 per workgroup: 8 is the fastest alone (C2 micro-bench
// 2897 vs 2429 Gpairs/s at batch 32), 6 inside the tracking pipeline (192
// instead of 248 VGPRs, so its waves find room beside the local-BA and tail
// kernels on the CUs ORB leaves: 19.4-19.7k vs 19.0-19.1k frames/s in
// alternating runs, profiles/r3_sweeps/mxqb_pipe_v1/ in git history before 1bfa753) -- the pipeline wins.
#ifndef SLAM_MX_QB
#define SLAM_MX_QB 6
#endif
constexpr int kMxQB = SLAM_MX_QB;          // (4 per step measured 10 % slower than 8 alone)
constexpr int kMxQWG = 16 * kMxQB;         // queries per workgroup
// the kernel merges one query per thread: the -D tunables must keep
// every query of the workgroup within it
static_assert(kMxWG >= kMxQWG && kMxWG % 64 == 0,
              "knn2_mx_kernel: SLAM_MX_WG must cover 16 * SLAM_MX_QB queries");
#ifndef SLAM_MX_XCD
#define SLAM_MX_XCD 1  // XCD-aware block order (0: blocks in launch order, for A/B)
#endif
constexpr int kMxAhead = 2;                // train steps loaded ahead
constexpr float kMxNone = 16777215.0f;     // > every valid key (< 2^23 + 2^14)
typedef int mx_v8i __attribute__((ext_vector_type(8)));
typedef float mx_v4f __attribute__((ext_vector_type(4)));

// operand dword d (0..3) of a descriptor word: nibble k = bit 4k + d of w, as
// fp4 +1.0 (0x2, query) or -2.0 (0xC, train)
template <int D>
__device__ __forceinline__ int nib_q(uint32_t w) {
  return (int)(((w >> D) & 0x11111111u) << 1);
}
template <int D>
__device__ __forceinline__ int nib_t(uint32_t w) {
  const uint32_t x = (w >> D) & 0x11111111u;
  return (int)((x << 3) | (x << 2));
}

// Blocks are dealt round-robin over the 8 XCDs (b and b + 8 share one): the
// bijection that gives XCD x the contiguous virtual range of its blocks.
__device__ __forceinline__ int xcd_block(int b, int nb) {
  const int x = b & 7, per = nb >> 3, rem = nb & 7;
  return x * per + min(x, rem) + (b >> 3);
}

__global__ __launch_bounds__(kMxWG) void knn2_mx_kernel(
    const uint32_t* __restrict__ q, const int32_t* __restrict__ nq_arr, int q_cap,
    const uint32_t* __restrict__ t, const int32_t* __restrict__ nt_arr, int t_cap,
    int tiles_per_item, int2* __restrict__ idx2, int2* __restrict__ dist2,
    uint8_t* __restrict__ good) {
  __shared__ uint32_t part[kMxWaves][kMxQWG][2];
#if SLAM_MX_XCD
  const int vb = xcd_block((int)blockIdx.x, (int)gridDim.x);
#else
  const int vb = (int)blockIdx.x;
#endif
  const int item = vb / tiles_per_item;
  const int tile = vb - item * tiles_per_item;
  const int nq = min(max(nq_arr[item], 0), q_cap);
  const int nt = min(max(nt_arr[item], 0), t_cap);
  const int q0 = tile * kMxQWG;
  if (q0 >= nq) return;  // uniform over the workgroup
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x / kWave);
  const int l = threadIdx.x & (kWave - 1), r = l & 15, g = l >> 4;
  const uint32_t* qb = q + (size_t)item * q_cap * 8;
  const uint4* tb = reinterpret_cast<const uint4*>(t + (size_t)item * t_cap * 8);
  // query fragments: block b, half h = dword 4 h + g of query q0 + 16 b + r
  mx_v8i A[kMxQB][2];
#pragma unroll
  for (int b = 0; b < kMxQB; ++b) {
    const int qi = q0 + 16 * b + r;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const uint32_t w = qi < nq ? qb[(size_t)qi * 8 + 4 * h + g] : 0u;
      A[b][h] = mx_v8i{nib_q<0>(w), nib_q<1>(w), nib_q<2>(w), nib_q<3>(w), 0, 0, 0, 0};
    }
  }
  uint32_t k1[kMxQB][4], k2[kMxQB][4];  // key bit patterns (non-negative floats)
#pragma unroll
  for (int b = 0; b < kMxQB; ++b)
#pragma unroll
    for (int i = 0; i < 4; ++i) k1[b][i] = k2[b][i] = __float_as_uint(kMxNone);
  // this wave's steps: train rows 16 (wid + 4 s) + r; whole rows, kMxAhead
  // ahead.  Software pipeline: while the MFMAs of step s run, the operands of
  // step s + 1 are formed (popcount, bits -> nibbles) and the keys of
  // step s - 1 are folded into the top-2 (the loop is unrolled twice so the
  // two accumulator sets alternate by name).
  const int nsteps = (nt + 15) >> 4;
  const int nmine = nsteps > wid ? (nsteps - wid + kMxWaves - 1) / kMxWaves : 0;  // uniform
  uint4 ra[kMxAhead][2];
  auto ld = [&](int s, uint4 (&o)[2]) {
    const int j = 16 * (wid + kMxWaves * s) + r;
    const size_t row = (size_t)min(j, max(nt - 1, 0));
    const bool ok = nt > 0 && s < nmine;
    o[0] = ok ? tb[2 * row] : make_uint4(0, 0, 0, 0);
    o[1] = ok ? tb[2 * row + 1] : make_uint4(0, 0, 0, 0);
  };
  // operands of step s from its row (ra[0]): B halves and the accumulator seed
  struct Ops {
    mx_v8i B0, B1;
    float init;
  };
  auto form = [&](int s) {
    const uint4 x = ra[0][0], y = ra[0][1];
#pragma unroll
    for (int a = 0; a + 1 < kMxAhead; ++a) {
      ra[a][0] = ra[a + 1][0];
      ra[a][1] = ra[a + 1][1];
    }
    ld(s + kMxAhead, ra[kMxAhead - 1]);
    const int j = 16 * (wid + kMxWaves * s) + r;
    const bool valid = j < nt && s < nmine;
    const int pc = __builtin_popcount(x.x) + __builtin_popcount(x.y) + __builtin_popcount(x.z) +
                   __builtin_popcount(x.w) + __builtin_popcount(y.x) + __builtin_popcount(y.y) +
                   __builtin_popcount(y.z) + __builtin_popcount(y.w);
    Ops o;
    o.init = valid ? (float)((pc + 256) * 16384 + j) : kMxNone;
    // dwords g and 4 + g of the row (zero past the train set: B = 0, the
    // accumulator keeps kMxNone)
    uint32_t w0 = g == 0 ? x.x : g == 1 ? x.y : g == 2 ? x.z : x.w;
    uint32_t w1 = g == 0 ? y.x : g == 1 ? y.y : g == 2 ? y.z : y.w;
    w0 = valid ? w0 : 0u;
    w1 = valid ? w1 : 0u;
    o.B0 = mx_v8i{nib_t<0>(w0), nib_t<1>(w0), nib_t<2>(w0), nib_t<3>(w0), 0, 0, 0, 0};
    o.B1 = mx_v8i{nib_t<0>(w1), nib_t<1>(w1), nib_t<2>(w1), nib_t<3>(w1), 0, 0, 0, 0};
    return o;
  };
  // all first halves, then all second halves (independent accumulators
  // between the dependent pairs)
  auto issue = [&](const Ops& o, mx_v4f (&acc)[kMxQB]) {
#pragma unroll
    for (int b = 0; b < kMxQB; ++b) {
      acc[b] = mx_v4f{o.init, o.init, o.init, o.init};
      acc[b] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(A[b][0], o.B0, acc[b], 4, 4, 0, 127, 0, 141);
    }
#pragma unroll
    for (int b = 0; b < kMxQB; ++b)
      acc[b] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(A[b][1], o.B1, acc[b], 4, 4, 0, 127, 0, 141);
  };
  // the keys are non-negative floats: their bit patterns order as unsigned
  // integers (v_min_u32 / v_med3_u32, no NaN canonicalisation)
  auto fold = [&](const mx_v4f (&acc)[kMxQB]) {
#pragma unroll
    for (int b = 0; b < kMxQB; ++b)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const uint32_t key = __float_as_uint(acc[b][i]);
        k2[b][i] = umed3(k1[b][i], k2[b][i], key);
        k1[b][i] = min(k1[b][i], key);
      }
  };
#pragma unroll
  for (int a = 0; a < kMxAhead; ++a) ld(a, ra[a]);
  mx_v4f accA[kMxQB], accB[kMxQB];
  if (nmine > 0) {
    Ops o = form(0);
    issue(o, accA);
    int s = 1;
    for (; s + 1 < nmine; s += 2) {
      o = form(s);
      issue(o, accB);
      fold(accA);
      o = form(s + 1);
      issue(o, accA);
      fold(accB);
    }
    if (s < nmine) {
      o = form(s);
      issue(o, accB);
      fold(accA);
      fold(accB);
    } else {
      fold(accA);
    }
  }
  // merge the 16 column-lanes of each query row (lanes 16 g .. 16 g + 15)
#pragma unroll
  for (int off = 1; off < 16; off <<= 1)
#pragma unroll
    for (int b = 0; b < kMxQB; ++b)
#pragma unroll
      for (int i = 0; i < 4; ++i)
        merge2(k1[b][i], k2[b][i], __shfl_xor(k1[b][i], off, kWave), __shfl_xor(k2[b][i], off, kWave));
  // lane (g, r < 4) holds query 16 b + 4 g + r of this wave's partial
  if (r < 4) {
#pragma unroll
    for (int b = 0; b < kMxQB; ++b) {
      uint32_t m1 = k1[b][0], m2 = k2[b][0];
#pragma unroll
      for (int i = 1; i < 4; ++i) {
        m1 = r == i ? k1[b][i] : m1;
        m2 = r == i ? k2[b][i] : m2;
      }
      part[wid][16 * b + 4 * g + r][0] = m1;
      part[wid][16 * b + 4 * g + r][1] = m2;
    }
  }
  __syncthreads();
  const int ql = threadIdx.x;  // one thread per query of the workgroup
  if (ql >= kMxQWG) return;
  const int qi = q0 + ql;
  if (qi >= nq) return;
  uint32_t b1 = part[0][ql][0], b2 = part[0][ql][1];
#pragma unroll
  for (int w = 1; w < kMxWaves; ++w) merge2(b1, b2, part[w][ql][0], part[w][ql][1]);
  const float m1 = __uint_as_float(b1), m2 = __uint_as_float(b2);
  int pq = 0;
#pragma unroll
  for (int w = 0; w < 8; ++w) pq += __builtin_popcount(qb[(size_t)qi * 8 + w]);
  const bool h1 = m1 < kMxNone, h2 = m2 < kMxNone;
  const uint32_t u1 = (uint32_t)m1, u2 = (uint32_t)m2;
  int2 id, ds;
  id.x = h1 ? (int)(u1 & 16383u) : -1;
  ds.x = h1 ? (int)(u1 >> 14) - 256 + pq : -1;
  id.y = h2 ? (int)(u2 & 16383u) : -1;
  ds.y = h2 ? (int)(u2 >> 14) - 256 + pq : -1;
  const size_t o = (size_t)item * q_cap + qi;
  idx2[o] = id;
  dist2[o] = ds;
  good[o] = (h2 && 10 * ds.x < 7 * ds.y) ? 1 : 0;
}

// One workgroup per batch item: order-preserving compaction of good rows.
#ifndef SLAM_CWG
#define SLAM_CWG 1024
#endif
constexpr int kCWG = SLAM_CWG;

__global__ __launch_bounds__(kCWG) void compact_kernel(
    const int2* __restrict__ idx2, const uint8_t* __restrict__ good,
    const int32_t* __restrict__ nq_arr, int q_cap, const double* __restrict__ gate_xyz,
    double gate, int2* __restrict__ pairs, int32_t* __restrict__ count) {
  __shared__ int wave_tot[kCWG / kWave];
  __shared__ int carry;
  const int item = blockIdx.x;
  const int nq = min(max(nq_arr[item], 0), q_cap);
  const int lane = threadIdx.x & (kWave - 1);
  const int wid = threadIdx.x / kWave;
  if (threadIdx.x == 0) carry = 0;
  __syncthreads();
  for (int base = 0; base < nq; base += kCWG) {
    const int qi = base + threadIdx.x;
    bool keep = false;
    if (qi < nq) {
      const size_t o = (size_t)item * q_cap + qi;
      keep = good[o] != 0;
      if (keep && gate_xyz != nullptr) {
        const double* X = gate_xyz + o * 3;
        keep = fabs(X[0]) < gate && fabs(X[1]) < gate && fabs(X[2]) < gate;
      }
    }
    const unsigned long long m = __ballot(keep);
    const int before = __popcll(m & ((1ull << lane) - 1ull));
    if (lane == 0) wave_tot[wid] = __popcll(m);
    __syncthreads();
    int off = carry;
    for (int w = 0; w < wid; ++w) off += wave_tot[w];
    if (keep) {
      const size_t o = (size_t)item * q_cap + qi;
      pairs[(size_t)item * q_cap + off + before] = make_int2(qi, idx2[o].x);
    }
    __syncthreads();
    if (threadIdx.x == 0) {
      int tot = 0;
      for (int w = 0; w < kCWG / kWave; ++w) tot += wave_tot[w];
      carry += tot;
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) count[item] = carry;
}

}  // namespace

extern "C" int slam_hamming_knn2(const uint8_t* d_q, const int32_t* d_nq, int q_cap,
                                 const uint8_t* d_t, const int32_t* d_nt, int t_cap,
                                 int batch, int32_t* d_idx2, int32_t* d_dist2,
                                 uint8_t* d_good, void* stream) {
  SLAM_REQUIRE(batch >= 0, "slam_hamming_knn2: batch < 0");
  SLAM_REQUIRE(q_cap >= 0 && t_cap >= 0, "slam_hamming_knn2: negative capacity");
  SLAM_REQUIRE(t_cap <= 65535, "slam_hamming_knn2: t_cap %d > 65535", t_cap);
  if (batch == 0 || q_cap == 0) return SLAM_OK;
  SLAM_REQUIRE(d_q && d_nq && d_t && d_nt && d_idx2 && d_dist2 && d_good,
               "slam_hamming_knn2: null pointer");
  SLAM_REQUIRE(((uintptr_t)d_q & 15) == 0 && ((uintptr_t)d_t & 15) == 0,
               "slam_hamming_knn2: descriptor buffers must be 16-byte aligned");
  if (t_cap <= 16383 && !g_knn2_valu) {  // matrix-core form (train index in 14 bits)
    const int tiles = (q_cap + kMxQWG - 1) / kMxQWG;
    const long long grid = (long long)tiles * batch;
    SLAM_REQUIRE(grid < (1ll << 31), "slam_hamming_knn2: grid too large");
    knn2_mx_kernel<<<dim3((unsigned)grid), dim3(kMxWG), 0, slam::as_stream(stream)>>>(
        reinterpret_cast<const uint32_t*>(d_q), d_nq, q_cap, reinterpret_cast<const uint32_t*>(d_t),
        d_nt, t_cap, tiles, reinterpret_cast<int2*>(d_idx2), reinterpret_cast<int2*>(d_dist2),
        d_good);
    SLAM_LAUNCHED("knn2_mx_kernel");
    return SLAM_OK;
  }
  const int tiles = (q_cap + kQPerWG - 1) / kQPerWG;
  const long long grid = (long long)tiles * batch;
  SLAM_REQUIRE(grid < (1ll << 31), "slam_hamming_knn2: grid too large");
  knn2_kernel<<<dim3((unsigned)grid), dim3(kWG), 0, slam::as_stream(stream)>>>(
      reinterpret_cast<const uint4*>(d_q), d_nq, q_cap, reinterpret_cast<const uint4*>(d_t),
      d_nt, t_cap, tiles, reinterpret_cast<int2*>(d_idx2), reinterpret_cast<int2*>(d_dist2),
      d_good);
  SLAM_LAUNCHED("knn2_kernel");
  return SLAM_OK;
}

extern "C" int slam_hamming_force_valu(int valu) {
  const int prev = g_knn2_valu;
  g_knn2_valu = valu != 0;
  return prev;
}

extern "C" int slam_compact_matches(const int32_t* d_idx2, const uint8_t* d_good,
                                    const int32_t* d_nq, int q_cap, int batch,
                                    const double* d_gate_xyz, double gate,
                                    int32_t* d_pairs, int32_t* d_count, void* stream) {
  SLAM_REQUIRE(batch >= 0 && q_cap >= 0, "slam_compact_matches: bad shape");
  if (batch == 0) return SLAM_OK;
  SLAM_REQUIRE(d_idx2 && d_good && d_nq && d_pairs && d_count,
               "slam_compact_matches: null pointer");
  compact_kernel<<<dim3(batch), dim3(kCWG), 0, slam::as_stream(stream)>>>(
      reinterpret_cast<const int2*>(d_idx2), d_good, d_nq, q_cap, d_gate_xyz, gate,
      reinterpret_cast<int2*>(d_pairs), d_count);
  SLAM_LAUNCHED("compact_kernel");
  return SLAM_OK;
}
