// Fundamental-matrix LMedS outlier mask for gfx950, batched over frame pairs.
//
// Replaces cv2.findFundamentalMat(pts_left, pts_right, cv2.FM_LMEDS) and the
// mask application of /root/reference/keypoint.py:59-66, following the
// deterministic spec of oracle/fundamental.c (300 seeded 7-point hypotheses,
// Hartley-normalised Gauss-Jordan null space, cubic roots, float errors,
// min-median selection, OpenCV's robust sigma for the final inlier mask).
//
// k_fm_hyp: kSplit workgroups (8 waves) per frame pair, each a contiguous
// range of the hypotheses:
//   phase 1: one hypothesis per lane -> up to 3 candidate F in LDS;
//   phase 2: wave w owns hypotheses h = w mod 8 of the range.  Per candidate the
//            wave counts errors below its best median so far (exact reject: the
//            median improves iff more than M/2 errors are below it); only
//            improving candidates pay an exact radix-select median (4 x 8-bit
//            passes, errors recomputed per pass instead of stored);
//   phase 3: the workgroup's best (min median, lowest candidate index);
// k_fm_finish: one workgroup per pair merges the kSplit bests by the same rule,
//   recomputes the winner and writes the inlier mask.
#include "common.hpp"

#include <cmath>

namespace {

#ifndef SLAM_FMH_WG
#define SLAM_FMH_WG 256
#endif
// k_fm_hyp workgroup: its ~254-VGPR waves need a whole SIMD's register file two
// at a time, so the size decides which CUs (next to ORB's waves or idle) take it
constexpr int kHWG = SLAM_FMH_WG, kHWaves = kHWG / 64;
constexpr int kFWG = 64;  // k_fm_finish: one wave (lane 0 recomputes the winner, then the mask)
constexpr int kS = 7;

__device__ inline uint64_t splitmix64(uint64_t& s) {
  s += 0x9E3779B97F4A7C15ull;
  uint64_t z = s;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

// 7 distinct indices in [0, M) from the hypothesis' splitmix64 stream
// (rejection of repeats, as oracle/fundamental.c); unrolled so idx stays in
// registers
__device__ __forceinline__ void draw_sample(uint64_t& s, int M, int idx[kS]) {
#pragma unroll
  for (int k = 0; k < kS; ++k) {
    int v;
    bool dup;
    do {
      v = (int)((splitmix64(s) >> 32) % (uint64_t)M);
      dup = false;
#pragma unroll
      for (int j = 0; j < k; ++j) dup |= idx[j] == v;
    } while (dup);
    idx[k] = v;
  }
}

__device__ inline double det3(const double* F) {
  return F[0] * (F[4] * F[8] - F[5] * F[7]) - F[1] * (F[3] * F[8] - F[5] * F[6]) +
         F[2] * (F[3] * F[7] - F[4] * F[6]);
}

__device__ inline double detmix(const double* F1, const double* F2, double a) {
  double F[9];
  for (int i = 0; i < 9; ++i) F[i] = a * F1[i] + (1.0 - a) * F2[i];
  return det3(F);
}

// Real roots of c3 x^3 + c2 x^2 + c1 x + c0, polished by two Newton steps and
// sorted ascending (oracle/fundamental.c states the same arithmetic).  The
// roots live in three fixed registers (every index is a compile-time
// constant, so nothing spills to scratch); unused slots hold +inf.
__device__ int cubic_roots(double c3, double c2, double c1, double c0, double r[3]) {
  r[0] = r[1] = r[2] = INFINITY;
  const double mx = fmax(fmax(fabs(c3), fabs(c2)), fmax(fabs(c1), fabs(c0)));
  if (mx == 0.0) return 0;
  int n = 0;
  if (fabs(c3) <= 1e-12 * mx) {
    if (fabs(c2) <= 1e-12 * mx) {
      if (fabs(c1) <= 1e-12 * mx) return 0;
      r[0] = -c0 / c1;
      return 1;
    }
    const double d = c1 * c1 - 4.0 * c2 * c0;
    if (d < 0) return 0;
    const double sq = sqrt(d);
    const double q = -0.5 * (c1 + (c1 >= 0 ? sq : -sq));
    r[0] = q / c2;
    n = 1;
    if (q != 0.0) {
      r[1] = c0 / q;
      n = 2;
    }
  } else {
    const double a = c2 / c3, b = c1 / c3, c = c0 / c3;
    const double p = b - a * a / 3.0;
    const double q = 2.0 * a * a * a / 27.0 - a * b / 3.0 + c;
    const double disc = q * q / 4.0 + p * p * p / 27.0;
    if (disc > 0) {
      const double sd = sqrt(disc);
      const double u = cbrt(-q / 2.0 + sd), v = cbrt(-q / 2.0 - sd);
      r[0] = u + v - a / 3.0;
      n = 1;
    } else {
      const double rr = sqrt(fmax(-p / 3.0, 0.0));
      double ca = rr > 0 ? -q / (2.0 * rr * rr * rr) : 0.0;
      ca = fmin(fmax(ca, -1.0), 1.0);
      const double phi = acos(ca);
#pragma unroll
      for (int k = 0; k < 3; ++k)
        r[k] = 2.0 * rr * cos((phi + 2.0 * 3.14159265358979323846 * k) / 3.0) - a / 3.0;
      n = 3;
    }
  }
#pragma unroll
  for (int i = 0; i < 3; ++i)
    if (i < n)
#pragma unroll
      for (int it = 0; it < 2; ++it) {
        const double x = r[i];
        const double f = ((c3 * x + c2) * x + c1) * x + c0;
        const double df = (3.0 * c3 * x + 2.0 * c2) * x + c1;
        if (df != 0.0) r[i] = x - f / df;
      }
  // insertion sort of the first n (the +inf slots stay behind)
  if (n > 1 && r[1] < r[0]) { const double t = r[0]; r[0] = r[1]; r[1] = t; }
  if (n > 2 && r[2] < r[1]) {
    const double t = r[1]; r[1] = r[2]; r[2] = t;
    if (r[1] < r[0]) { const double u = r[0]; r[0] = r[1]; r[1] = u; }
  }
  return n;
}

// The 7-point algorithm on Hartley-normalised points: Gauss-Jordan with full
// pivoting on the 7x9 system, the two-dimensional null space (F1, F2), the
// cubic det(a F1 + (1 - a) F2) = 0, de-normalisation and unit Frobenius norm.
// Writes up to 3 candidates to out (LDS) and returns their number.  Pivot rows,
// pivot columns and the free columns are data-dependent, so they are applied
// as selects over fully unrolled loops: the 7x9 matrix stays in registers.
__device__ int seven_point(const double* m1, const double* m2, const int* idx, double (*out)[9]) {
  double P1[kS][2], P2[kS][2];
#pragma unroll
  for (int i = 0; i < kS; ++i) {
    P1[i][0] = m1[2 * idx[i]]; P1[i][1] = m1[2 * idx[i] + 1];
    P2[i][0] = m2[2 * idx[i]]; P2[i][1] = m2[2 * idx[i] + 1];
  }
  double c1x = 0, c1y = 0, c2x = 0, c2y = 0;
#pragma unroll
  for (int i = 0; i < kS; ++i) {
    c1x += P1[i][0]; c1y += P1[i][1];
    c2x += P2[i][0]; c2y += P2[i][1];
  }
  c1x /= kS; c1y /= kS; c2x /= kS; c2y /= kS;
  double d1 = 0, d2 = 0;
#pragma unroll
  for (int i = 0; i < kS; ++i) {
    d1 += sqrt((P1[i][0] - c1x) * (P1[i][0] - c1x) + (P1[i][1] - c1y) * (P1[i][1] - c1y));
    d2 += sqrt((P2[i][0] - c2x) * (P2[i][0] - c2x) + (P2[i][1] - c2y) * (P2[i][1] - c2y));
  }
  d1 /= kS; d2 /= kS;
  if (!(d1 > 1e-12) || !(d2 > 1e-12)) return 0;
  const double s1 = sqrt(2.0) / d1, s2 = sqrt(2.0) / d2;
  double A[7][9];
#pragma unroll
  for (int i = 0; i < kS; ++i) {
    const double x1 = (P1[i][0] - c1x) * s1, y1 = (P1[i][1] - c1y) * s1;
    const double x2 = (P2[i][0] - c2x) * s2, y2 = (P2[i][1] - c2y) * s2;
    A[i][0] = x2 * x1; A[i][1] = x2 * y1; A[i][2] = x2;
    A[i][3] = y2 * x1; A[i][4] = y2 * y1; A[i][5] = y2;
    A[i][6] = x1; A[i][7] = y1; A[i][8] = 1.0;
  }
  int pc[7];
  unsigned used = 0;
#pragma unroll
  for (int r = 0; r < 7; ++r) {
    int bi = -1, bj = -1;
    double bv = 0.0;
#pragma unroll
    for (int i = r; i < 7; ++i)
#pragma unroll
      for (int j = 0; j < 9; ++j)
        if (!((used >> j) & 1u) && fabs(A[i][j]) > bv) {
          bv = fabs(A[i][j]);
          bi = i;
          bj = j;
        }
    if (bv < 1e-10) return 0;
#pragma unroll
    for (int i = r + 1; i < 7; ++i) {
      const bool sw = i == bi;
#pragma unroll
      for (int j = 0; j < 9; ++j) {
        const double t = A[r][j];
        A[r][j] = sw ? A[i][j] : t;
        A[i][j] = sw ? t : A[i][j];
      }
    }
    used |= 1u << bj;
    pc[r] = bj;
    double piv = 0.0;
#pragma unroll
    for (int j = 0; j < 9; ++j) piv = j == bj ? A[r][j] : piv;
    const double inv = 1.0 / piv;
#pragma unroll
    for (int j = 0; j < 9; ++j) A[r][j] *= inv;
#pragma unroll
    for (int i = 0; i < 7; ++i) {
      if (i == r) continue;
      double f = 0.0;
#pragma unroll
      for (int j = 0; j < 9; ++j) f = j == bj ? A[i][j] : f;
#pragma unroll
      for (int j = 0; j < 9; ++j) A[i][j] = f != 0.0 ? A[i][j] - f * A[r][j] : A[i][j];
    }
  }
  // the first two unused columns span the null space
  int fr0 = -1, fr1 = -1;
#pragma unroll
  for (int j = 0; j < 9; ++j)
    if (!((used >> j) & 1u)) {
      if (fr0 < 0) fr0 = j;
      else if (fr1 < 0) fr1 = j;
    }
  double F1[9], F2[9];
#pragma unroll
  for (int j = 0; j < 9; ++j) {
    F1[j] = j == fr0 ? 1.0 : 0.0;
    F2[j] = j == fr1 ? 1.0 : 0.0;
  }
#pragma unroll
  for (int r = 0; r < 7; ++r) {
    double a1 = 0.0, a2 = 0.0;  // A[r][fr0], A[r][fr1]
#pragma unroll
    for (int j = 0; j < 9; ++j) {
      a1 = j == fr0 ? A[r][j] : a1;
      a2 = j == fr1 ? A[r][j] : a2;
    }
#pragma unroll
    for (int j = 0; j < 9; ++j) {
      F1[j] = j == pc[r] ? -a1 : F1[j];
      F2[j] = j == pc[r] ? -a2 : F2[j];
    }
  }
  const double v0 = detmix(F1, F2, 0.0), v1 = detmix(F1, F2, 1.0);
  const double vm = detmix(F1, F2, -1.0), v2 = detmix(F1, F2, 2.0);
  const double cc0 = v0;
  const double cc2 = (v1 + vm) / 2.0 - cc0;
  const double s = (v1 - vm) / 2.0;
  const double u = v2 - 4.0 * cc2 - cc0;
  const double cc3 = (u - 2.0 * s) / 6.0;
  const double cc1 = s - cc3;
  double roots[3];
  const int nr = cubic_roots(cc3, cc2, cc1, cc0, roots);
  const double T1[9] = {s1, 0, -s1 * c1x, 0, s1, -s1 * c1y, 0, 0, 1};
  const double T2[9] = {s2, 0, -s2 * c2x, 0, s2, -s2 * c2y, 0, 0, 1};
  int n = 0;
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    if (k >= nr) break;
    double Fn[9], tmp[9], F[9];
#pragma unroll
    for (int i = 0; i < 9; ++i) Fn[i] = roots[k] * F1[i] + (1.0 - roots[k]) * F2[i];
#pragma unroll
    for (int i = 0; i < 3; ++i)
#pragma unroll
      for (int j = 0; j < 3; ++j)
        tmp[3 * i + j] = Fn[3 * i] * T1[j] + Fn[3 * i + 1] * T1[3 + j] + Fn[3 * i + 2] * T1[6 + j];
#pragma unroll
    for (int i = 0; i < 3; ++i)
#pragma unroll
      for (int j = 0; j < 3; ++j)
        F[3 * i + j] = T2[i] * tmp[j] + T2[3 + i] * tmp[3 + j] + T2[6 + i] * tmp[6 + j];
    double nrm = 0.0;
#pragma unroll
    for (int i = 0; i < 9; ++i) nrm += F[i] * F[i];
    nrm = sqrt(nrm);
    if (!(nrm > 0.0) || !isfinite(nrm)) continue;
#pragma unroll
    for (int i = 0; i < 9; ++i) out[n][i] = F[i] / nrm;
    ++n;
  }
  return n;
}

__device__ __forceinline__ float fm_error(const double* F, const double* p1, const double* p2) {
  double a = F[0] * p1[0] + F[1] * p1[1] + F[2];
  double b = F[3] * p1[0] + F[4] * p1[1] + F[5];
  double c = F[6] * p1[0] + F[7] * p1[1] + F[8];
  const double s2 = 1.0 / (a * a + b * b);
  const double d2 = p2[0] * a + p2[1] * b + c;
  a = F[0] * p2[0] + F[3] * p2[1] + F[6];
  b = F[1] * p2[0] + F[4] * p2[1] + F[7];
  c = F[2] * p2[0] + F[5] * p2[1] + F[8];
  const double s1 = 1.0 / (a * a + b * b);
  const double d1 = p1[0] * a + p1[1] * b + c;
  const float e = (float)fmax(d1 * d1 * s1, d2 * d2 * s2);
  return isnan(e) ? INFINITY : e;
}

// Hypotheses of one frame pair are spread over kSplit workgroups (a
// contiguous hypothesis range each), so a batch of B pairs fills B * kSplit
// workgroups; each reports its best (median, candidate index) and k_fm_finish
// merges them (min median, lowest index: the order-independent rule of the
// single-workgroup form) and computes the mask.  The per-split bests travel in
// F's own slot (72 B per pair), which k_fm_finish then overwrites.
constexpr int kSplit = 8;
constexpr int kRound = 64;  // hypotheses per round (one per lane of wave 0)
constexpr int kEv = 12;     // points per lane cached in registers (M <= 768 fully)
static_assert(kSplit * 8 <= 9 * 8, "per-split bests must fit F[b]");
#ifdef SLAM_FMH_TRACE
__device__ unsigned long long g_fmh[8];
#define FMH_T(i) do { if (threadIdx.x == 0 && blockIdx.x == 3 && blockIdx.y == 5) g_fmh[i] = __builtin_amdgcn_s_memtime(); } while (0)
#else
#define FMH_T(i) (void)0
#endif

__global__ __launch_bounds__(kHWG) void k_fm_hyp(const double* __restrict__ m1all,
                                                const double* __restrict__ m2all,
                                                const int32_t* __restrict__ count, int cap,
                                                uint64_t seed, int item0, int n_hyp,
                                                double* __restrict__ Fout) {
  __shared__ double cand[kRound][3][9];  // hypotheses processed in rounds of kRound
  __shared__ int ncand[kRound];
  __shared__ int hist[kHWaves][256];
  __shared__ float wbest[kHWaves];
  __shared__ int wbidx[kHWaves];
  const int b = blockIdx.x, sp = blockIdx.y, t = threadIdx.x;
  const int lane = t & 63, w = t >> 6;
  const int M = min(max(count[b], 0), cap);
  if (M < 8) return;  // k_fm_finish writes the empty mask
  const double* m1 = m1all + (size_t)b * cap * 2;
  const double* m2 = m2all + (size_t)b * cap * 2;
  const int hb = (int)((long long)n_hyp * sp / kSplit), he = (int)((long long)n_hyp * (sp + 1) / kSplit);
  float my_best = INFINITY;
  int my_idx = 0x7FFFFFFF;
  const int need = M / 2 + 1;  // #errors below a value for the median to be below it
  FMH_T(0);
#ifdef SLAM_FMH_TRACE
  int n_sel = 0, n_cand = 0;
#endif
  for (int h0 = hb; h0 < he; h0 += kRound) {
    const int nh = min(kRound, he - h0);
    __syncthreads();
    if (t < nh) {
      const int h = h0 + t;
      uint64_t s = seed ^ ((uint64_t)(item0 + b) * 0xD1B54A32D192ED03ull) ^
                   ((uint64_t)h * 0x9FB21C651E98DF25ull);
      int idx[kS];
      draw_sample(s, M, idx);
      ncand[t] = seven_point(m1, m2, idx, cand[t]);
    }
    __syncthreads();
    FMH_T(1);
    // the candidates' errors at the lane's points i = lane + 64 j (j < kEv) are
    // kept in registers for the median select (points past 64 kEv: recomputed);
    // ln is opaque so that their addresses are not hoisted (live) across the
    // seven-point solves, which need the whole register file
    int ln = lane;
    asm volatile("" : "+v"(ln));
    double pc[kEv][4];  // the points themselves, read once per round
#pragma unroll
    for (int j = 0; j < kEv; ++j) {
      const int i = min(ln + 64 * j, M - 1);
      pc[j][0] = m1[2 * i];
      pc[j][1] = m1[2 * i + 1];
      pc[j][2] = m2[2 * i];
      pc[j][3] = m2[2 * i + 1];
    }
    for (int hl = w; hl < nh; hl += kHWaves) {
      for (int k = 0; k < ncand[hl]; ++k) {
        const double* F = cand[hl][k];
        int below = 0;
        float ev[kEv];
#pragma unroll
        for (int j = 0; j < kEv; ++j) {
          ev[j] = INFINITY;
          if (ln + 64 * j < M) {
            ev[j] = fm_error(F, pc[j], pc[j] + 2);
            below += ev[j] < my_best ? 1 : 0;
          }
        }
        for (int i = ln + 64 * kEv; i < M; i += 64)
          below += fm_error(F, m1 + 2 * i, m2 + 2 * i) < my_best ? 1 : 0;
        for (int off = 32; off > 0; off >>= 1) below += __shfl_xor(below, off, 64);
#ifdef SLAM_FMH_TRACE
        ++n_cand;
#endif
        if (below < need) continue;  // median >= my_best: cannot improve (uniform)
#ifdef SLAM_FMH_TRACE
        ++n_sel;
#endif
        // exact median = (M/2)-th smallest error, radix select on the float bits
        uint32_t prefix = 0, pmask = 0;
        int krank = M / 2;
        for (int shift = 24; shift >= 0; shift -= 8) {
          for (int j = lane; j < 256; j += 64) hist[w][j] = 0;
          __builtin_amdgcn_wave_barrier();
#pragma unroll
          for (int j = 0; j < kEv; ++j) {
            const uint32_t bits = __float_as_uint(ev[j]);
            if (ln + 64 * j < M && (bits & pmask) == prefix)
              atomicAdd(&hist[w][(bits >> shift) & 255u], 1);
          }
          for (int i = ln + 64 * kEv; i < M; i += 64) {
            const uint32_t bits = __float_as_uint(fm_error(F, m1 + 2 * i, m2 + 2 * i));
            if ((bits & pmask) == prefix) atomicAdd(&hist[w][(bits >> shift) & 255u], 1);
          }
          __builtin_amdgcn_wave_barrier();
          __builtin_amdgcn_s_waitcnt(0xC07F);
          // prefix sums over 256 bins, 4 per lane
          const int c0 = hist[w][4 * lane], c1 = hist[w][4 * lane + 1];
          const int c2 = hist[w][4 * lane + 2], c3 = hist[w][4 * lane + 3];
          const int sm = c0 + c1 + c2 + c3;
          int inc = sm;
          for (int off = 1; off < 64; off <<= 1) {
            const int o = __shfl_up(inc, off, 64);
            if (lane >= off) inc += o;
          }
          const int exc = inc - sm;
          int bin = -1, before = 0;
          if (krank >= exc && krank < inc) {
            int acc = exc;
            if (krank < acc + c0) { bin = 4 * lane; before = acc; }
            else if (krank < acc + c0 + c1) { bin = 4 * lane + 1; before = acc + c0; }
            else if (krank < acc + c0 + c1 + c2) { bin = 4 * lane + 2; before = acc + c0 + c1; }
            else { bin = 4 * lane + 3; before = acc + c0 + c1 + c2; }
          }
          const unsigned long long bal = __ballot(bin >= 0);
          const int src = __ffsll((long long)bal) - 1;
          bin = __shfl(bin, src, 64);
          before = __shfl(before, src, 64);
          krank -= before;
          prefix |= (uint32_t)bin << shift;
          pmask |= 255u << shift;
        }
        const float med = __uint_as_float(prefix);
        if (med < my_best) {
          my_best = med;
          my_idx = (h0 + hl) * 3 + k;
        }
      }
    }
  }
  FMH_T(2);
#ifdef SLAM_FMH_TRACE
  if (threadIdx.x == 0 && blockIdx.x == 3 && blockIdx.y == 5) { g_fmh[5] = n_cand; g_fmh[6] = n_sel; g_fmh[7] = M; }
#endif
  if (lane == 0) {
    wbest[w] = my_best;
    wbidx[w] = my_idx;
  }
  __syncthreads();
  FMH_T(3);
  if (t == 0) {
    float bm = INFINITY;
    int bi = 0x7FFFFFFF;
    for (int i = 0; i < kHWaves; ++i)
      if (wbest[i] < bm || (wbest[i] == bm && wbidx[i] < bi)) {
        bm = wbest[i];
        bi = wbidx[i];
      }
    float* slot = reinterpret_cast<float*>(Fout + 9 * (size_t)b) + 2 * sp;
    slot[0] = bm;
    reinterpret_cast<int*>(slot)[1] = bi;
  }
}

__global__ __launch_bounds__(kFWG) void k_fm_finish(const double* __restrict__ m1all,
                                                   const double* __restrict__ m2all,
                                                   const int32_t* __restrict__ count, int cap,
                                                   uint64_t seed, int item0,
                                                   uint8_t* __restrict__ mask,
                                                   double* __restrict__ Fout,
                                                   int32_t* __restrict__ ninl) {
  __shared__ double Fb[9];
  __shared__ double Fw[3][9];  // the winner's candidates, recomputed
  __shared__ float best_s;
  __shared__ int found_s, cnt_s;
  const int b = blockIdx.x, t = threadIdx.x;
  const int lane = t & 63;
  const int M = min(max(count[b], 0), cap);
  const double* m1 = m1all + (size_t)b * cap * 2;
  const double* m2 = m2all + (size_t)b * cap * 2;
  uint8_t* mk = mask + (size_t)b * cap;
  if (M < 8) {  // no hypothesis: empty mask, F = 0
    for (int i = t; i < M; i += kFWG) mk[i] = 0;
    if (t < 9) Fout[9 * b + t] = 0.0;
    if (t == 0) ninl[b] = -1;
    return;
  }
  if (t == 0) {
    const float* slots = reinterpret_cast<const float*>(Fout + 9 * (size_t)b);
    float bm = INFINITY;
    int bi = 0x7FFFFFFF;
    for (int i = 0; i < kSplit; ++i) {
      const float v = slots[2 * i];
      const int ix = reinterpret_cast<const int*>(slots)[2 * i + 1];
      if (v < bm || (v == bm && ix < bi)) {
        bm = v;
        bi = ix;
      }
    }
    best_s = bm;
    found_s = bi != 0x7FFFFFFF && bm < INFINITY;
    cnt_s = 0;
    if (found_s) {
      // recompute the winner
      const int h = bi / 3, k = bi % 3;
      uint64_t s = seed ^ ((uint64_t)(item0 + b) * 0xD1B54A32D192ED03ull) ^
                   ((uint64_t)h * 0x9FB21C651E98DF25ull);
      int idx[kS];
      draw_sample(s, M, idx);
      seven_point(m1, m2, idx, Fw);
      for (int i = 0; i < 9; ++i) Fb[i] = Fw[k][i];
    }
  }
  __syncthreads();
  if (!found_s) {  // F[b] still holds k_fm_hyp's per-split slots: overwrite with 0
    for (int i = t; i < M; i += kFWG) mk[i] = 0;
    if (t < 9) Fout[9 * b + t] = 0.0;
    if (t == 0) ninl[b] = -1;
    return;
  }
  double sigma = 2.5 * 1.4826 * (1 + 5.0 / (M - kS)) * sqrt((double)best_s);
  sigma = fmax(sigma, 0.001);
  const double thr = sigma * sigma;
  double F[9];
  for (int i = 0; i < 9; ++i) F[i] = Fb[i];
  int c = 0;
  for (int i = t; i < M; i += kFWG) {
    const uint8_t in = (double)fm_error(F, m1 + 2 * i, m2 + 2 * i) <= thr ? 1 : 0;
    mk[i] = in;
    c += in;
  }
  for (int off = 32; off > 0; off >>= 1) c += __shfl_xor(c, off, 64);
  if (lane == 0) atomicAdd(&cnt_s, c);
  __syncthreads();
  if (t < 9) Fout[9 * b + t] = F[t];
  if (t == 0) ninl[b] = cnt_s;
}

// Order-preserving compaction of pairs[b][k] (k < count[b]) by mask[b][k].
#ifndef SLAM_CWG
#define SLAM_CWG 1024
#endif
constexpr int kCWG = SLAM_CWG;
__global__ __launch_bounds__(kCWG) void k_filter_pairs(const int2* __restrict__ pairs,
                                                       const int32_t* __restrict__ count,
                                                       const uint8_t* __restrict__ mask, int cap,
                                                       int2* __restrict__ out,
                                                       int32_t* __restrict__ out_count) {
  __shared__ int wave_tot[kCWG / 64];
  __shared__ int carry;
  const int b = blockIdx.x;
  const int n = min(max(count[b], 0), cap);
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  if (threadIdx.x == 0) carry = 0;
  __syncthreads();
  for (int base = 0; base < n; base += kCWG) {
    const int k = base + threadIdx.x;
    const bool keep = k < n && mask[(size_t)b * cap + k] != 0;
    const unsigned long long m = __ballot(keep);
    const int before = __popcll(m & ((1ull << lane) - 1ull));
    if (lane == 0) wave_tot[wid] = __popcll(m);
    __syncthreads();
    int off = carry;
    for (int i = 0; i < wid; ++i) off += wave_tot[i];
    if (keep) out[(size_t)b * cap + off + before] = pairs[(size_t)b * cap + k];
    __syncthreads();
    if (threadIdx.x == 0) {
      int tot = 0;
      for (int i = 0; i < kCWG / 64; ++i) tot += wave_tot[i];
      carry += tot;
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) out_count[b] = carry;
}

}  // namespace

extern "C" int slam_fundamental_lmeds(const double* d_m1, const double* d_m2,
                                      const int32_t* d_count, int cap, int batch, uint64_t seed,
                                      int item0, int n_hyp, uint8_t* d_mask, double* d_F,
                                      int32_t* d_ninliers, void* stream) {
  SLAM_REQUIRE(batch >= 0 && cap >= 0, "slam_fundamental_lmeds: bad shape");
  SLAM_REQUIRE(n_hyp >= 1 && n_hyp <= 4096, "slam_fundamental_lmeds: n_hyp in [1, 4096]");
  if (batch == 0) return SLAM_OK;
  SLAM_REQUIRE(d_m1 && d_m2 && d_count && d_mask && d_F && d_ninliers,
               "slam_fundamental_lmeds: null pointer");
  hipStream_t s = slam::as_stream(stream);
  k_fm_hyp<<<dim3(batch, kSplit), kHWG, 0, s>>>(d_m1, d_m2, d_count, cap, seed, item0, n_hyp, d_F);
  SLAM_LAUNCHED("k_fm_hyp");
  k_fm_finish<<<batch, kFWG, 0, s>>>(d_m1, d_m2, d_count, cap, seed, item0, d_mask, d_F,
                                    d_ninliers);
  SLAM_LAUNCHED("k_fm_finish");
  return SLAM_OK;
}

extern "C" int slam_filter_pairs(const int32_t* d_pairs, const int32_t* d_count,
                                 const uint8_t* d_mask, int cap, int batch, int32_t* d_out,
                                 int32_t* d_out_count, void* stream) {
  SLAM_REQUIRE(batch >= 0 && cap >= 0, "slam_filter_pairs: bad shape");
  if (batch == 0) return SLAM_OK;
  SLAM_REQUIRE(d_pairs && d_count && d_mask && d_out && d_out_count,
               "slam_filter_pairs: null pointer");
  SLAM_REQUIRE(d_out != d_pairs, "slam_filter_pairs: in-place filtering is not supported");
  k_filter_pairs<<<batch, kCWG, 0, slam::as_stream(stream)>>>(
      reinterpret_cast<const int2*>(d_pairs), d_count, d_mask, cap, reinterpret_cast<int2*>(d_out),
      d_out_count);
  SLAM_LAUNCHED("k_filter_pairs");
  return SLAM_OK;
}

#ifdef SLAM_FMH_TRACE
extern "C" int slam_fmh_trace(unsigned long long* out) {
  SLAM_HIP(hipDeviceSynchronize());
  SLAM_HIP(hipMemcpyFromSymbol(out, HIP_SYMBOL(g_fmh), 8 * sizeof(unsigned long long)));
  return SLAM_OK;
}
#endif
