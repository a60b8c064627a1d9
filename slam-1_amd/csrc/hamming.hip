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

// One workgroup per batch item: order-preserving compaction of good rows.
constexpr int kCWG = 1024;

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
