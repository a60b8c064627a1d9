// Matched-point gather, DLT triangulation and RANSAC + LM PnP for gfx950.
//
// Replaces, per frame pair of the tracking loop (/root/reference/main.py:82-97):
//   keypoint.py:53-57        gather of matched points (f64) and descriptors
//   Point3D.py:14-19          cv2.triangulatePoints (per-point 4x4 SVD null vector)
//   transformation.py:5-19    cv2.solvePnPRansac(Q, q, K, 0) (ITERATIVE flavour:
//                             minimal 5-point LM hypotheses, 8 px reprojection
//                             threshold, LM refinement on the inliers)
// RANSAC sampling is a counter-based splitmix64 stream keyed by (seed, frame,
// hypothesis) so the CPU oracle draws the same subsets (OpenCV's own RNG
// sequence is not reproducible here).
#include "common.hpp"
#include "epnp.hpp"
#include "dlt.hpp"

#include <climits>

#include <cmath>

namespace {

constexpr int kBS = 256;

// --------------------------------------------------------------- gather
__global__ __launch_bounds__(kBS) void k_gather(const float* __restrict__ kpq, int kq_cap,
                                                const float* __restrict__ kpt, int kt_cap,
                                                const uint8_t* __restrict__ dq_in,
                                                const uint8_t* __restrict__ dt_in,
                                                const int2* __restrict__ pairs,
                                                const int32_t* __restrict__ count, int p_cap,
                                                double* __restrict__ ptq, double* __restrict__ ptt,
                                                uint8_t* __restrict__ dq, uint8_t* __restrict__ dt) {
  const int b = blockIdx.y;
  const int n = min(max(count[b], 0), p_cap);
  const int k = blockIdx.x * kBS + threadIdx.x;
  if (k >= n) return;
  const size_t o = (size_t)b * p_cap + k;
  const int2 pr = pairs[o];
  const float* a = kpq + ((size_t)b * kq_cap + pr.x) * 5;
  const float* c = kpt + ((size_t)b * kt_cap + pr.y) * 5;
  ptq[2 * o] = (double)a[0];
  ptq[2 * o + 1] = (double)a[1];
  ptt[2 * o] = (double)c[0];
  ptt[2 * o + 1] = (double)c[1];
  if (dq) {
    const uint4* s0 = reinterpret_cast<const uint4*>(dq_in + ((size_t)b * kq_cap + pr.x) * 32);
    const uint4* s1 = reinterpret_cast<const uint4*>(dt_in + ((size_t)b * kt_cap + pr.y) * 32);
    uint4* d0 = reinterpret_cast<uint4*>(dq + o * 32);
    uint4* d1 = reinterpret_cast<uint4*>(dt + o * 32);
    d0[0] = s0[0];
    d0[1] = s0[1];
    d1[0] = s1[0];
    d1[1] = s1[1];
  }
}

// 2D-3D correspondences of find_2D_and_3D_correspondenses (Point3D.py:50-52):
// Q1 = X[qi], q1 = ptl[qi] (tracked left points at t), q2 = kp_next[ti].xy.
__global__ __launch_bounds__(kBS) void k_gather_temporal(
    const double* __restrict__ X, const double* __restrict__ ptl, int xcap,
    const float* __restrict__ kpn, int kcap, const int2* __restrict__ pairs,
    const int32_t* __restrict__ count, int pcap, double* __restrict__ Q1,
    double* __restrict__ q2, double* __restrict__ q1) {
  const int b = blockIdx.y;
  const int n = min(max(count[b], 0), pcap);
  const int k = blockIdx.x * kBS + threadIdx.x;
  if (k >= n) return;
  const size_t o = (size_t)b * pcap + k;
  const int2 pr = pairs[o];
  const size_t xi = (size_t)b * xcap + pr.x;
  Q1[3 * o] = X[3 * xi];
  Q1[3 * o + 1] = X[3 * xi + 1];
  Q1[3 * o + 2] = X[3 * xi + 2];
  q1[2 * o] = ptl[2 * xi];
  q1[2 * o + 1] = ptl[2 * xi + 1];
  const float* c = kpn + ((size_t)b * kcap + pr.y) * 5;
  q2[2 * o] = (double)c[0];
  q2[2 * o + 1] = (double)c[1];
}

// --------------------------------------------------------------- triangulation
__global__ __launch_bounds__(kBS) void k_triangulate(const double* __restrict__ pl,
                                                     const double* __restrict__ pr,
                                                     const int32_t* __restrict__ count, int cap,
                                                     const double* __restrict__ Pl,
                                                     const double* __restrict__ Pr, int pstride,
                                                     double* __restrict__ X) {
  const int b = blockIdx.y;
  const int n = min(max(count[b], 0), cap);
  const int k = blockIdx.x * kBS + threadIdx.x;
  if (k >= n) return;
  const double* P[2] = {Pl + (size_t)b * pstride, Pr + (size_t)b * pstride};
  const size_t o = (size_t)b * cap + k;
  const double xy[2][2] = {{pl[2 * o], pl[2 * o + 1]}, {pr[2 * o], pr[2 * o + 1]}};
  double A[4][4];
#pragma unroll
  for (int j = 0; j < 2; ++j)
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      A[2 * j][c] = xy[j][0] * P[j][8 + c] - P[j][c];
      A[2 * j + 1][c] = xy[j][1] * P[j][8 + c] - P[j][4 + c];
    }
  double v[4];
  null_vector4(A, v);
  X[3 * o] = v[0] / v[3];
  X[3 * o + 1] = v[1] / v[3];
  X[3 * o + 2] = v[2] / v[3];
}

// --------------------------------------------------------------- PnP
__device__ __host__ inline uint64_t splitmix64(uint64_t& s) {
  s += 0x9E3779B97F4A7C15ull;
  uint64_t z = s;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

// cv::Rodrigues (rotation vector -> matrix)
__device__ inline void rodrigues(const double r[3], double R[9]) {
  const double th = sqrt(r[0] * r[0] + r[1] * r[1] + r[2] * r[2]);
  if (th < 2.220446049250313e-16) {
    R[0] = 1; R[1] = 0; R[2] = 0; R[3] = 0; R[4] = 1; R[5] = 0; R[6] = 0; R[7] = 0; R[8] = 1;
    return;
  }
  const double c = cos(th), s = sin(th), c1 = 1.0 - c, it = 1.0 / th;
  const double x = r[0] * it, y = r[1] * it, z = r[2] * it;
  R[0] = c + c1 * x * x; R[1] = c1 * x * y - s * z; R[2] = c1 * x * z + s * y;
  R[3] = c1 * x * y + s * z; R[4] = c + c1 * y * y; R[5] = c1 * y * z - s * x;
  R[6] = c1 * x * z - s * y; R[7] = c1 * y * z + s * x; R[8] = c + c1 * z * z;
}

struct Cam {
  double fx, fy, cx, cy;
};

// reprojection residual of one point and (optionally) its 2x6 Jacobian wrt (r, t)
template <bool JAC>
__device__ inline void pnp_residual(const double p[6], const double R[9], const double* Q,
                                    const double* q, const Cam& K, double r[2], double J[2][6]) {
  const double X0 = Q[0], X1 = Q[1], X2 = Q[2];
  const double RX0 = R[0] * X0 + R[1] * X1 + R[2] * X2;
  const double RX1 = R[3] * X0 + R[4] * X1 + R[5] * X2;
  const double RX2 = R[6] * X0 + R[7] * X1 + R[8] * X2;
  const double Xc = RX0 + p[3], Yc = RX1 + p[4], Zc = RX2 + p[5];
  const double iz = 1.0 / Zc;
  r[0] = K.fx * (Xc * iz) + K.cx - q[0];
  r[1] = K.fy * (Yc * iz) + K.cy - q[1];
  if constexpr (JAC) {
    const double du[3] = {K.fx * iz, 0.0, -K.fx * Xc * iz * iz};
    const double dv[3] = {0.0, K.fy * iz, -K.fy * Yc * iz * iz};
    // dRX/dr: Gallego & Yezzi, -[RX]x at r = 0
    double D[3][3];
    const double w0 = p[0], w1 = p[1], w2 = p[2];
    const double th2 = w0 * w0 + w1 * w1 + w2 * w2;
    if (th2 < 1e-24) {
      D[0][0] = 0; D[0][1] = RX2; D[0][2] = -RX1;
      D[1][0] = -RX2; D[1][1] = 0; D[1][2] = RX0;
      D[2][0] = RX1; D[2][1] = -RX0; D[2][2] = 0;
    } else {
      const double W[3][3] = {{0.0, -w2, w1}, {w2, 0.0, -w0}, {-w1, w0, 0.0}};
      const double w[3] = {w0, w1, w2};
      double Am[3][3];
      for (int i = 0; i < 3; ++i)
        for (int k = 0; k < 3; ++k) {
          double acc = w[i] * w[k];
          for (int j = 0; j < 3; ++j) acc += R[3 * j + i] * W[j][k];
          Am[i][k] = acc - W[i][k];
        }
      const double Xs[3][3] = {{0.0, -X2, X1}, {X2, 0.0, -X0}, {-X1, X0, 0.0}};
      double B[3][3];
      for (int i = 0; i < 3; ++i)
        for (int k = 0; k < 3; ++k)
          B[i][k] = Xs[i][0] * Am[0][k] + Xs[i][1] * Am[1][k] + Xs[i][2] * Am[2][k];
      const double inv = -1.0 / th2;
      for (int i = 0; i < 3; ++i)
        for (int k = 0; k < 3; ++k)
          D[i][k] = (R[3 * i] * B[0][k] + R[3 * i + 1] * B[1][k] + R[3 * i + 2] * B[2][k]) * inv;
    }
    for (int k = 0; k < 3; ++k) {
      J[0][k] = du[0] * D[0][k] + du[1] * D[1][k] + du[2] * D[2][k];
      J[1][k] = dv[0] * D[0][k] + dv[1] * D[1][k] + dv[2] * D[2][k];
      J[0][3 + k] = du[k];
      J[1][3 + k] = dv[k];
    }
  }
}

// Solve (H + lam diag(H)) d = -g for the 6x6 SPD system (Cholesky); false on failure.
__device__ inline bool solve6(const double H[21], const double g[6], double lam, double d[6]) {
  double A[6][6];
  int k = 0;
  for (int i = 0; i < 6; ++i)
    for (int j = 0; j <= i; ++j) {
      A[i][j] = H[k];
      A[j][i] = H[k];
      ++k;
    }
  for (int i = 0; i < 6; ++i) A[i][i] += lam * fmax(A[i][i], 1e-12);
  for (int j = 0; j < 6; ++j) {
    double s = A[j][j];
    for (int p = 0; p < j; ++p) s -= A[j][p] * A[j][p];
    if (!(s > 0.0)) return false;
    A[j][j] = sqrt(s);
    for (int i = j + 1; i < 6; ++i) {
      double t = A[i][j];
      for (int p = 0; p < j; ++p) t -= A[i][p] * A[j][p];
      A[i][j] = t / A[j][j];
    }
  }
  double y[6];
  for (int i = 0; i < 6; ++i) {
    double t = -g[i];
    for (int p = 0; p < i; ++p) t -= A[i][p] * y[p];
    y[i] = t / A[i][i];
  }
  for (int i = 5; i >= 0; --i) {
    double t = y[i];
    for (int p = i + 1; p < 6; ++p) t -= A[p][i] * d[p];
    d[i] = t / A[i][i];
  }
  return true;
}

constexpr int kMinSample = 5;
constexpr int kPnPWG = 256;
constexpr int kMaxHyp = 256;
constexpr int kRc = 4;  // refinement points per lane held in registers (L <= 256 fully)

// Levenberg-Marquardt on a hypothesis' sample (oracle/geometry.c lm with idx)
// on a 16-lane group (lane k = lane & 15): lanes s < n evaluate
// point s (residual, Jacobian) and publish its per-(s, a) terms; lane j < 28
// sums term j over (s, a) in the oracle's order (H, g, cost), every lane then
// reads the 28 sums and runs the identical 6x6 solve and decision, so p and
// lam stay replicated.  Bitwise the operations of oracle lm.
// t: LDS [2 * kMinSample][kLmT], sums: LDS [28 + kMinSample].  Every lane of
// the group's wave must call it (wave-level __syncthreads inside).
// Row stride 29 doubles: the five point lanes' term stores (16-lane groups of
// ds_write_b64, bank = dword mod 32) fall on distinct banks (at 28 lanes 0, 2
// and 4 shared one: 3.3 conflict cycles per LDS instruction).
constexpr int kLmT = 29;
// per-group block of t: 10 rows of 29 doubles padded to 304 (608 dwords = 32
// mod 64), so the sum reads of groups g and g+1 (one 32-lane half of a
// ds_read_b64, bank = dword mod 64) use the two bank halves
constexpr int kLmGroup = 304;
static_assert(kLmGroup >= 2 * kMinSample * kLmT && (2 * kLmGroup) % 64 == 32, "lm_group LDS layout");
__device__ void lm_group(const double* Q, const double* q, int n, const Cam& K, int iters,
                         double p[6], int k, double (*t)[kLmT], double* sums) {
  double lam = 1e-3;
  double R[9];  // rotation of p: carried over from the trial pose when a step is accepted
  rodrigues(p, R);
  for (int it = 0; it < iters; ++it) {
    if (k < n) {
      double r[2], J[2][6];
      pnp_residual<true>(p, R, Q + 3 * k, q + 2 * k, K, r, J);
#pragma unroll
      for (int a = 0; a < 2; ++a) {
        double* o = t[2 * k + a];
        int m = 0;
#pragma unroll
        for (int u = 0; u < 6; ++u) {
#pragma unroll
          for (int v = 0; v <= u; ++v) o[m++] = J[a][u] * J[a][v];
          o[21 + u] = J[a][u] * r[a];
        }
        o[27] = r[a] * r[a];
      }
    }
    __syncthreads();
    // lane k sums terms k and k + 16 (< 28)
#pragma unroll
    for (int e = 0; e < 2; ++e) {
      const int j = k + 16 * e;
      if (j < 28) {
        double acc = 0.0;
        for (int sa = 0; sa < 2 * n; ++sa) acc += t[sa][j];
        sums[j] = acc;
      }
    }
    __syncthreads();
    double H[21], g[6];
#pragma unroll
    for (int i = 0; i < 21; ++i) H[i] = sums[i];
#pragma unroll
    for (int i = 0; i < 6; ++i) g[i] = sums[21 + i];
    const double cost = sums[27];
    double d[6], pn[6];
    const bool ok = solve6(H, g, lam, d);
    if (!ok) {
      lam = fmin(lam * 10.0, 1e12);
      __syncthreads();  // sums are rewritten next iteration
      continue;
    }
    for (int i = 0; i < 6; ++i) pn[i] = p[i] + d[i];
    double Rn[9];
    rodrigues(pn, Rn);
    __syncthreads();  // every lane has read sums
    if (k < n) {
      double r[2], J[2][6];
      pnp_residual<false>(pn, Rn, Q + 3 * k, q + 2 * k, K, r, J);
      sums[k] = r[0] * r[0] + r[1] * r[1];
    }
    __syncthreads();
    double cn = 0.0;
    for (int s2 = 0; s2 < n; ++s2) cn += sums[s2];
    __syncthreads();
    if (cn < cost) {
      for (int i = 0; i < 6; ++i) p[i] = pn[i];
      for (int i = 0; i < 9; ++i) R[i] = Rn[i];
      lam = fmax(lam * 0.1, 1e-12);
    } else {
      lam = fmin(lam * 10.0, 1e12);
    }
  }
}

// Sum over the 64 lanes of a wave, every lane ends with the total (xor butterfly).
__device__ __forceinline__ double wave_allsum(double v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
  return v;
}

// Sums of 32 values over the 64 lanes of a wave, every lane ends with all 32
// totals (v[k] = total k).  Reduce-scatter by halving: at offset 32, 16, .., 2
// a lane keeps the half of its values its partner does not (one shuffle per
// kept value: 16 + 8 + 4 + 2 + 1, then one at offset 1), so total j ends on
// lanes 2j and 2j+1 and is broadcast by v_readlane -- 32 double shuffles
// instead of 6 per value of the xor butterfly.
__device__ __forceinline__ double readlane_d(double x, int l) {
  const unsigned long long u = __double_as_longlong(x);
  const unsigned lo = __builtin_amdgcn_readlane((unsigned)u, l);
  const unsigned hi = __builtin_amdgcn_readlane((unsigned)(u >> 32), l);
  return __longlong_as_double((long long)(((unsigned long long)hi << 32) | lo));
}
template <int OFF>
__device__ __forceinline__ void allsum_halve(double (&v)[32], int lane) {
  constexpr int half = OFF / 2;
  const bool hi = (lane & OFF) != 0;
#pragma unroll
  for (int k = 0; k < half; ++k) {
    const double send = hi ? v[k] : v[k + half];
    const double keep = hi ? v[k + half] : v[k];
    v[k] = keep + __shfl_xor(send, OFF, 64);
  }
}
__device__ __forceinline__ void wave_allsum32(double (&v)[32]) {
  const int lane = threadIdx.x & 63;
  allsum_halve<32>(v, lane);
  allsum_halve<16>(v, lane);
  allsum_halve<8>(v, lane);
  allsum_halve<4>(v, lane);
  allsum_halve<2>(v, lane);
  const double tot = v[0] + __shfl_xor(v[0], 1, 64);
#pragma unroll
  for (int j = 0; j < 32; ++j) v[j] = readlane_d(tot, 2 * j);
}

// PnP-RANSAC hypotheses: kHypGroups per one-wave workgroup, a 16-lane group
// each.  Sample h of pair b: 5 distinct indices from splitmix64(seed,
// item0 + b, h); EPnP on the sample (OpenCV's RANSAC kernel for
// SOLVEPNP_ITERATIVE; csrc/epnp.hpp group form: M^T M rows and the 12x12
// Jacobi on 12 lanes, the three beta approximations on 3 lanes), then
// hyp_iters LM steps on the same 5 points from that pose (a degenerate sample
// starts LM at r = t = 0).  Poses -> ws [b][h][6].
constexpr int kHypGroups = 4;  // hypotheses per one-wave workgroup (16 lanes each)
#ifdef SLAM_PNPH_TRACE
__device__ unsigned long long g_pnph[8];
#define PNPH_T(i) do { if (threadIdx.x == 0 && blockIdx.x == 3 && blockIdx.y == 5) g_pnph[i] = __builtin_amdgcn_s_memtime(); } while (0)
#else
#define PNPH_T(i) (void)0
#endif
// Sample h of pair b (lane 0 of its group): 5 distinct indices from
// splitmix64(seed, item, h); Q[idx], q[idx] in draw order into pw / uv.
__device__ void pnp_sample(uint64_t seed, int item, int h, int L, const double* Q, const double* q,
                           double* pw, double* uv, int* sidx) {
  uint64_t s = seed ^ ((uint64_t)item * 0xD1B54A32D192ED03ull) ^
               ((uint64_t)h * 0x8CB92BA72F3D8DD7ull);
  int idx[kMinSample];
  for (int kk = 0; kk < kMinSample; ++kk) {
    int v;
    bool dup;
    do {
      v = (int)((splitmix64(s) >> 32) % (uint64_t)L);
      dup = false;
      for (int j = 0; j < kk; ++j) dup |= idx[j] == v;
    } while (dup);
    idx[kk] = v;
    sidx[kk] = v;
    for (int d = 0; d < 3; ++d) pw[3 * kk + d] = Q[3 * v + d];
    for (int d = 0; d < 2; ++d) uv[2 * kk + d] = q[2 * v + d];
  }
}

__global__ __launch_bounds__(64) void k_pnp_hyp(const double* __restrict__ Qall,
                                                const double* __restrict__ qall,
                                                const int32_t* __restrict__ count, int cap,
                                                const double* __restrict__ Kp, uint64_t seed,
                                                int item0, int n_hyp, double* __restrict__ ws) {
#ifdef SLAM_PNP_PRIO
  __builtin_amdgcn_s_setprio(SLAM_PNP_PRIO);
#endif
  __shared__ slam_epnp::EpGroup grp[kHypGroups];
  __shared__ double spw[kHypGroups][3 * kMinSample], suv[kHypGroups][2 * kMinSample];
  __shared__ int sidx[kHypGroups][kMinSample];
  const int b = blockIdx.x, t = threadIdx.x;
  const int g = t >> 4, k = t & 15;
  const int h = blockIdx.y * kHypGroups + g;
  const int L = min(max(count[b], 0), cap);
  if (L < kMinSample) return;  // uniform over the workgroup
  const bool live = h < n_hyp;
  const double* Q = Qall + (size_t)b * cap * 3;
  const double* q = qall + (size_t)b * cap * 2;
  const Cam K{Kp[0], Kp[4], Kp[2], Kp[5]};
  slam_epnp::EpGroup& G = grp[g];
  PNPH_T(0);
  if (k == 0 && live) {
    pnp_sample(seed, item0 + b, h, L, Q, q, spw[g], suv[g], sidx[g]);
    G.flag = slam_epnp::ep_bary<kMinSample>(spw[g], G);
  }
  __syncthreads();
  PNPH_T(1);
  bool ok = live && G.flag != 0;
  if (ok && k < 12) slam_epnp::ep_mtm_row<kMinSample>(k, suv[g], K.fx, K.fy, K.cx, K.cy, G);
  __syncthreads();
  PNPH_T(2);
  slam_epnp::ep_jacobi12_group(G, k, ok);
  PNPH_T(3);
#ifdef SLAM_PNPH_TRACE
  if (threadIdx.x == 0 && blockIdx.x == 3 && blockIdx.y == 5) g_pnph[7] = (unsigned long long)G.offdia[1];
#endif
  if (ok && k == 0) slam_epnp::ep_lrho(G);
  __syncthreads();
  PNPH_T(4);
  if (ok && k < 3) slam_epnp::ep_approx<kMinSample>(k, spw[g], suv[g], K.fx, K.fy, K.cx, K.cy, G);
  __syncthreads();
  PNPH_T(5);
  if (k == 0 && live) {  // the EPnP pose (a degenerate sample: r = t = 0) -> ws
    double p[6] = {0, 0, 0, 0, 0, 0};
    if (!(ok && slam_epnp::ep_choose(G, p)))
      for (int i = 0; i < 6; ++i) p[i] = 0.0;
    double* o = ws + ((size_t)b * n_hyp + h) * 6;
    for (int i = 0; i < 6; ++i) o[i] = p[i];
  }
  PNPH_T(6);
}

// Hypothesis LM (the second half of a hypothesis, split from k_pnp_hyp so each
// kernel fits beside ORB's workgroups): hyp_iters LM steps on the same 5
// points from the EPnP pose in ws, the result written back in place.  The
// sample is redrawn (same splitmix64 stream) into LDS.  A dead group
// (h >= n_hyp) runs along on zeros and writes nothing.
__global__ __launch_bounds__(64) void k_pnp_hyp_lm(const double* __restrict__ Qall,
                                                   const double* __restrict__ qall,
                                                   const int32_t* __restrict__ count, int cap,
                                                   const double* __restrict__ Kp, uint64_t seed,
                                                   int item0, int n_hyp, int hyp_iters,
                                                   double* __restrict__ ws) {
#ifdef SLAM_PNP_PRIO
  __builtin_amdgcn_s_setprio(SLAM_PNP_PRIO);
#endif
  __shared__ double spw[kHypGroups][3 * kMinSample], suv[kHypGroups][2 * kMinSample];
  __shared__ int sidx[kHypGroups][kMinSample];
  __shared__ double lmt[kHypGroups * kLmGroup], lms[kHypGroups][28 + kMinSample];
  __shared__ double p0[kHypGroups][6];
  const int b = blockIdx.x, t = threadIdx.x;
  const int g = t >> 4, k = t & 15;
  const int h = blockIdx.y * kHypGroups + g;
  const int L = min(max(count[b], 0), cap);
  if (L < kMinSample) return;  // uniform over the workgroup
  const bool live = h < n_hyp;
  const double* Q = Qall + (size_t)b * cap * 3;
  const double* q = qall + (size_t)b * cap * 2;
  const Cam K{Kp[0], Kp[4], Kp[2], Kp[5]};
  double* o = ws + ((size_t)b * n_hyp + (live ? h : 0)) * 6;
  if (k == 0) {
    if (live) pnp_sample(seed, item0 + b, h, L, Q, q, spw[g], suv[g], sidx[g]);
    else
      for (int i = 0; i < 3 * kMinSample; ++i) spw[g][i] = suv[g][i % (2 * kMinSample)] = 0.0;
  }
  if (k < 6) p0[g][k] = live ? o[k] : 0.0;
  __syncthreads();
  double p[6];
  for (int i = 0; i < 6; ++i) p[i] = p0[g][i];
  lm_group(spw[g], suv[g], kMinSample, K, hyp_iters, p, k,
           reinterpret_cast<double (*)[kLmT]>(lmt + g * kLmGroup), lms[g]);
  if (k == 0 && live)
    for (int i = 0; i < 6; ++i) o[i] = p[i];
}

// One workgroup per frame pair:
//   hypotheses   one per lane: 5 distinct random points, LM from r = t = 0; the
//                pose and its rotation matrix go to LDS;
//   counting     (hypothesis, point) pairs spread over the whole workgroup,
//                inliers tallied with LDS atomics (integer: order-free);
//   selection    max inliers, lowest h; the inlier mask of the winner;
//   refinement   LM over the mask by wave 0 alone: lanes take points, the 28
//                normal-equation sums are wave butterflies (every lane holds
//                them), every lane solves the same 6x6 system — no workgroup
//                barriers inside the iteration loop.
__global__ __launch_bounds__(kPnPWG) void k_pnp(const double* __restrict__ Qall,
                                                const double* __restrict__ qall,
                                                const int32_t* __restrict__ count, int cap,
                                                const double* __restrict__ Kp, uint64_t seed,
                                                int item0, int n_hyp, double thresh,
                                                int hyp_iters, int refine_iters,
                                                double* __restrict__ rvec, double* __restrict__ tvec,
                                                int32_t* __restrict__ ninl,
                                                uint8_t* __restrict__ mask,
                                                const double* __restrict__ hws) {
#ifdef SLAM_PNP_PRIO
  __builtin_amdgcn_s_setprio(SLAM_PNP_PRIO);
#endif
  __shared__ double hp[kMaxHyp][6];
  __shared__ double hR[kMaxHyp][9];
  __shared__ int hcnt[kMaxHyp];
  __shared__ int best_s;
  const int b = blockIdx.x, t = threadIdx.x;
  const int lane = t & 63, wid = t >> 6;
  const int L = min(max(count[b], 0), cap);
  const double* Q = Qall + (size_t)b * cap * 3;
  const double* q = qall + (size_t)b * cap * 2;
  uint8_t* mk = mask + (size_t)b * cap;
  const Cam K{Kp[0], Kp[4], Kp[2], Kp[5]};
  if (L < kMinSample) {
    if (t == 0) {
      ninl[b] = -1;
      for (int i = 0; i < 3; ++i) rvec[3 * b + i] = tvec[3 * b + i] = 0.0;
    }
    for (int i = t; i < L; i += kPnPWG) mk[i] = 0;
    return;
  }
  const double thr2 = thresh * thresh;
#ifdef SLAM_PNP_PROFILE
  const uint64_t pt0 = __builtin_amdgcn_s_memtime();
#endif
  // ---- hypotheses (k_pnp_hyp: EPnP + LM on each sample)
  for (int h = t; h < n_hyp; h += kPnPWG) {
    double p[6], R[9];
    const double* src = hws + ((size_t)b * n_hyp + h) * 6;
    for (int i = 0; i < 6; ++i) p[i] = src[i];
    const bool finite = isfinite(p[0]) && isfinite(p[1]) && isfinite(p[2]) && isfinite(p[3]) &&
                        isfinite(p[4]) && isfinite(p[5]);
    rodrigues(p, R);
    for (int i = 0; i < 6; ++i) hp[h][i] = p[i];
    for (int i = 0; i < 9; ++i) hR[h][i] = R[i];
    hcnt[h] = finite ? 0 : INT_MIN;  // a non-finite pose scores 0 (see below)
  }
  __syncthreads();
#ifdef SLAM_PNP_PROFILE
  const uint64_t pt1 = __builtin_amdgcn_s_memtime();
#endif
  // ---- inlier counts over (hypothesis, point) pairs
  for (int pr = t; pr < n_hyp * L; pr += kPnPWG) {
    const int h = pr / L, i = pr - h * L;
    if (hcnt[h] < 0) continue;
    double r[2], J[2][6];
    pnp_residual<false>(hp[h], hR[h], Q + 3 * i, q + 2 * i, K, r, J);
    if (r[0] * r[0] + r[1] * r[1] <= thr2) atomicAdd(&hcnt[h], 1);
  }
  __syncthreads();
  if (t == 0) {
    int bh = 0, bc = max(hcnt[0], 0);
    for (int h = 1; h < n_hyp; ++h)
      if (max(hcnt[h], 0) > bc) {
        bc = max(hcnt[h], 0);
        bh = h;
      }
    best_s = bh;
  }
  __syncthreads();
  const int bh = best_s;
  for (int i = t; i < L; i += kPnPWG) {
    double r[2], J[2][6];
    pnp_residual<false>(hp[bh], hR[bh], Q + 3 * i, q + 2 * i, K, r, J);
    mk[i] = (r[0] * r[0] + r[1] * r[1] <= thr2) ? 1 : 0;
  }
  __syncthreads();
#ifdef SLAM_PNP_PROFILE
  const uint64_t pt2 = __builtin_amdgcn_s_memtime();
#endif
  if (wid != 0) return;
  // ---- LM refinement over the winner's inliers (fixed set), wave 0
  double p[6];
  for (int i = 0; i < 6; ++i) p[i] = hp[bh][i];
  // the lane's points i = lane + 64 j (j < kRc) and their inlier flags in
  // registers for all refine_iters iterations (points past 64 kRc: re-read)
  double rq[kRc][5];
  bool rin[kRc];
#pragma unroll
  for (int j = 0; j < kRc; ++j) {
    const int i = lane + 64 * j, ic = min(i, L - 1);
    rin[j] = i < L && mk[i] != 0;
    for (int d = 0; d < 3; ++d) rq[j][d] = Q[3 * ic + d];
    for (int d = 0; d < 2; ++d) rq[j][3 + d] = q[2 * ic + d];
  }
  double lam = 1e-3;
  double R[9];  // rotation of p: carried over from the trial pose when a step is accepted
  rodrigues(p, R);
  for (int it = 0; it < refine_iters; ++it) {
    double acc[32];
#pragma unroll
    for (int i = 0; i < 32; ++i) acc[i] = 0.0;
    auto add_terms = [&](const double* Qi, const double* qi) {
      double r[2], J[2][6];
      pnp_residual<true>(p, R, Qi, qi, K, r, J);
#pragma unroll
      for (int a = 0; a < 2; ++a) {
        int k = 0;
#pragma unroll
        for (int u = 0; u < 6; ++u) {
#pragma unroll
          for (int v = 0; v <= u; ++v) acc[k++] += J[a][u] * J[a][v];
          acc[21 + u] += J[a][u] * r[a];
        }
        acc[27] += r[a] * r[a];
      }
    };
#pragma unroll
    for (int j = 0; j < kRc; ++j)
      if (rin[j]) add_terms(rq[j], rq[j] + 3);
    for (int i = lane + 64 * kRc; i < L; i += 64)
      if (mk[i]) add_terms(Q + 3 * i, q + 2 * i);
    wave_allsum32(acc);
    double H[21], g[6];
#pragma unroll
    for (int i = 0; i < 21; ++i) H[i] = acc[i];
#pragma unroll
    for (int i = 0; i < 6; ++i) g[i] = acc[21 + i];
    const double cost = acc[27];
    double d[6], pn[6], Rn[9];
    const bool ok = solve6(H, g, lam, d);
    for (int i = 0; i < 6; ++i) pn[i] = ok ? p[i] + d[i] : p[i];
    rodrigues(pn, Rn);
    double cn = 0.0;
#pragma unroll
    for (int j = 0; j < kRc; ++j)
      if (rin[j]) {
        double r[2], J[2][6];
        pnp_residual<false>(pn, Rn, rq[j], rq[j] + 3, K, r, J);
        cn += r[0] * r[0] + r[1] * r[1];
      }
    for (int i = lane + 64 * kRc; i < L; i += 64) {
      if (!mk[i]) continue;
      double r[2], J[2][6];
      pnp_residual<false>(pn, Rn, Q + 3 * i, q + 2 * i, K, r, J);
      cn += r[0] * r[0] + r[1] * r[1];
    }
    cn = wave_allsum(cn);
    if (ok && cn < cost) {
      for (int i = 0; i < 6; ++i) p[i] = pn[i];
      for (int i = 0; i < 9; ++i) R[i] = Rn[i];
      lam = fmax(lam * 0.1, 1e-12);
    } else {
      lam = fmin(lam * 10.0, 1e12);
    }
  }
  if (lane < 3) {
    rvec[3 * b + lane] = p[lane];
    tvec[3 * b + lane] = p[3 + lane];
  }
  if (lane == 0) ninl[b] = max(hcnt[bh], 0);
#ifdef SLAM_PNP_PROFILE
  const uint64_t pt3 = __builtin_amdgcn_s_memtime();
  if (lane == 0) {  // cycles of hypotheses / counting / refinement in rvec (debug build)
    rvec[3 * b] = (double)(pt1 - pt0);
    rvec[3 * b + 1] = (double)(pt2 - pt1);
    rvec[3 * b + 2] = (double)(pt3 - pt2);
  }
#endif
}

// --------------------------------------------------------------- stereo VO pose
// The reference's second pose estimator (visual_odometry.py:65-81, 135-157):
// dof = (rotvec r, t), T = [R(r) | t];
//   forward  q1_pred = proj(P_l T,      Q2)   vs q1
//   backward q2_pred = proj(P_l T^-1,   Q1)   vs q2
// residual vector f (4N) = [fwd x (N), fwd y (N), bwd x (N), bwd y (N)]
// (np.vstack([q1_pred - q1.T, q2_pred - q2.T]).flatten(), :81).
// estimate_pose: max_iter hypotheses of 6 points drawn WITH replacement
// (np.random.choice(range(n), 6), :139), LM from dof = 0 on the sample (:142),
// error = sum of the norms of CONSECUTIVE PAIRS of f (the reshape((2N, 2)) of
// :144-146 pairs f[2k], f[2k+1]), sequential early termination after 5
// non-improving hypotheses (:147-154).  All hypotheses run in parallel (one per
// lane) and the sequential rule is applied to their errors in order, which
// selects exactly what the sequential loop would.
constexpr int kVoWG = 128;
constexpr int kVoSample = 6;

// X -> (u, v) with P (3x4 row-major); a0/a1: d(u, v)/dX when JAC
template <bool JAC>
__device__ inline void vo_project(const double* P, const double X[3], double uv[2], double a[2][3]) {
  const double x0 = P[0] * X[0] + P[1] * X[1] + P[2] * X[2] + P[3];
  const double x1 = P[4] * X[0] + P[5] * X[1] + P[6] * X[2] + P[7];
  const double x2 = P[8] * X[0] + P[9] * X[1] + P[10] * X[2] + P[11];
  const double iz = 1.0 / x2;
  uv[0] = x0 * iz;
  uv[1] = x1 * iz;
  if constexpr (JAC) {
    for (int k = 0; k < 3; ++k) {
      a[0][k] = (P[k] - uv[0] * P[8 + k]) * iz;
      a[1][k] = (P[4 + k] - uv[1] * P[8 + k]) * iz;
    }
  }
}

// d(R(w) X)/dw (sgn = +1) and d(R(w)^T X)/dw (sgn = -1), Gallego & Yezzi 2015:
//   d(R X)/dw   = -R  [X]x (w w^T + (R^T - I)[w]x) / |w|^2
//   d(R^T X)/dw =  R^T [X]x (w w^T - (R - I)[w]x) / |w|^2
// with the first-order forms -[RX]x and [X]x at w = 0.
__device__ inline void vo_drot(const double w[3], const double R[9], const double X[3], int sgn,
                               double D[3][3]) {
  const double th2 = w[0] * w[0] + w[1] * w[1] + w[2] * w[2];
  if (th2 < 1e-24) {
    // sgn > 0: -[R X]x = -[X]x (R = I); sgn < 0: [X]x
    const double s = sgn > 0 ? -1.0 : 1.0;
    D[0][0] = 0.0; D[0][1] = -s * X[2]; D[0][2] = s * X[1];
    D[1][0] = s * X[2]; D[1][1] = 0.0; D[1][2] = -s * X[0];
    D[2][0] = -s * X[1]; D[2][1] = s * X[0]; D[2][2] = 0.0;
    return;
  }
  const double W[3][3] = {{0.0, -w[2], w[1]}, {w[2], 0.0, -w[0]}, {-w[1], w[0], 0.0}};
  double Am[3][3];
  for (int i = 0; i < 3; ++i)
    for (int k = 0; k < 3; ++k) {
      double acc = w[i] * w[k];
      if (sgn > 0) {
        for (int j = 0; j < 3; ++j) acc += R[3 * j + i] * W[j][k];  // R^T W
        Am[i][k] = acc - W[i][k];
      } else {
        for (int j = 0; j < 3; ++j) acc -= R[3 * i + j] * W[j][k];  // - R W
        Am[i][k] = acc + W[i][k];
      }
    }
  const double Xs[3][3] = {{0.0, -X[2], X[1]}, {X[2], 0.0, -X[0]}, {-X[1], X[0], 0.0}};
  double B[3][3];
  for (int i = 0; i < 3; ++i)
    for (int k = 0; k < 3; ++k)
      B[i][k] = Xs[i][0] * Am[0][k] + Xs[i][1] * Am[1][k] + Xs[i][2] * Am[2][k];
  const double inv = (sgn > 0 ? -1.0 : 1.0) / th2;
  for (int i = 0; i < 3; ++i)
    for (int k = 0; k < 3; ++k) {
      // sgn > 0: R B; sgn < 0: R^T B
      const double m0 = sgn > 0 ? R[3 * i] : R[i], m1 = sgn > 0 ? R[3 * i + 1] : R[3 + i],
                   m2 = sgn > 0 ? R[3 * i + 2] : R[6 + i];
      D[i][k] = (m0 * B[0][k] + m1 * B[1][k] + m2 * B[2][k]) * inv;
    }
}

// the 4 residuals of point pair (Q1, Q2, q1, q2) and optionally the 4x6 Jacobian
template <bool JAC>
__device__ inline void vo_residual(const double p[6], const double R[9], const double* P,
                                   const double* Q1, const double* Q2, const double* q1,
                                   const double* q2, double r[4], double J[4][6]) {
  double X[3], Y[3], Z[3], uv[2], a[2][3];
  for (int i = 0; i < 3; ++i) X[i] = R[3 * i] * Q2[0] + R[3 * i + 1] * Q2[1] + R[3 * i + 2] * Q2[2] + p[3 + i];
  for (int i = 0; i < 3; ++i) Z[i] = Q1[i] - p[3 + i];
  for (int i = 0; i < 3; ++i) Y[i] = R[i] * Z[0] + R[3 + i] * Z[1] + R[6 + i] * Z[2];
  vo_project<JAC>(P, X, uv, a);
  r[0] = uv[0] - q1[0];
  r[1] = uv[1] - q1[1];
  if constexpr (JAC) {
    double D[3][3];
    vo_drot(p, R, Q2, +1, D);
    for (int c = 0; c < 2; ++c)
      for (int k = 0; k < 3; ++k) {
        J[c][k] = a[c][0] * D[0][k] + a[c][1] * D[1][k] + a[c][2] * D[2][k];
        J[c][3 + k] = a[c][k];
      }
  }
  vo_project<JAC>(P, Y, uv, a);
  r[2] = uv[0] - q2[0];
  r[3] = uv[1] - q2[1];
  if constexpr (JAC) {
    double D[3][3];
    vo_drot(p, R, Z, -1, D);
    for (int c = 0; c < 2; ++c)
      for (int k = 0; k < 3; ++k) {
        J[2 + c][k] = a[c][0] * D[0][k] + a[c][1] * D[1][k] + a[c][2] * D[2][k];
        // dY/dt = -R^T
        J[2 + c][3 + k] = -(a[c][0] * R[3 * k] + a[c][1] * R[3 * k + 1] + a[c][2] * R[3 * k + 2]);
      }
  }
}

// element i of the flat residual vector f (one projection)
__device__ inline double vo_elem(const double p[6], const double R[9], const double* P,
                                 const double* Q1, const double* Q2, const double* q1,
                                 const double* q2, int N, int i) {
  const int row = i / N, col = i - row * N;
  double X[3], uv[2], a[2][3];
  if (row < 2) {
    const double* Q = Q2 + 3 * col;
    for (int k = 0; k < 3; ++k) X[k] = R[3 * k] * Q[0] + R[3 * k + 1] * Q[1] + R[3 * k + 2] * Q[2] + p[3 + k];
    vo_project<false>(P, X, uv, a);
    return uv[row] - q1[2 * col + row];
  }
  const double* Q = Q1 + 3 * col;
  const double Z[3] = {Q[0] - p[3], Q[1] - p[4], Q[2] - p[5]};
  for (int k = 0; k < 3; ++k) X[k] = R[k] * Z[0] + R[3 + k] * Z[1] + R[6 + k] * Z[2];
  vo_project<false>(P, X, uv, a);
  return uv[row - 2] - q2[2 * col + row - 2];
}

// Hypothesis h of pair b: LM on its 6-point sample from dof = 0 -> ws_pp[b][h]
__global__ __launch_bounds__(kVoWG) void k_vo_hyp(
    const double* __restrict__ q1a, const double* __restrict__ q2a, const double* __restrict__ Q1a,
    const double* __restrict__ Q2a, const int32_t* __restrict__ count, int cap,
    const double* __restrict__ Pg, uint64_t seed, int item0, int max_iter, int lm_iters,
    double* __restrict__ ws_pp) {
  const int b = blockIdx.x, h = threadIdx.x;
  const int N = min(max(count[b], 0), cap);
  if (N <= 0) return;  // uniform: before the barrier
  const double* q1 = q1a + (size_t)b * cap * 2;
  const double* q2 = q2a + (size_t)b * cap * 2;
  const double* Q1 = Q1a + (size_t)b * cap * 3;
  const double* Q2 = Q2a + (size_t)b * cap * 3;
  // the lane's 6-point sample in LDS ([point][Q1 3, Q2 3, q1 2, q2 2]) and P in
  // LDS: indexed loads there instead of spilled register arrays
  __shared__ double smp[kVoWG][kVoSample][10];
  __shared__ double Ps[12];
  if (h < 12) Ps[h] = Pg[h];
  const double* P = Ps;
  uint64_t s = seed ^ ((uint64_t)(item0 + b) * 0xD1B54A32D192ED03ull) ^
               ((uint64_t)h * 0x8CB92BA72F3D8DD7ull);
  for (int k = 0; k < kVoSample; ++k) {
    const int v = (int)((splitmix64(s) >> 32) % (uint64_t)N);  // with replacement
    double* d = smp[h][k];
    for (int c = 0; c < 3; ++c) {
      d[c] = Q1[3 * v + c];
      d[3 + c] = Q2[3 * v + c];
    }
    for (int c = 0; c < 2; ++c) {
      d[6 + c] = q1[2 * v + c];
      d[8 + c] = q2[2 * v + c];
    }
  }
  __syncthreads();
  // LM on the sample from dof = 0 (Marquardt diagonal, lambda x0.1 / x10)
  double pp[6] = {0, 0, 0, 0, 0, 0}, lam = 1e-3, R[9];
  for (int it = 0; it < lm_iters; ++it) {
    rodrigues(pp, R);
    double H[21] = {0}, g[6] = {0}, cost = 0.0;
    for (int k = 0; k < kVoSample; ++k) {
      double r[4], J[4][6];
      const double* d = smp[h][k];
      vo_residual<true>(pp, R, P, d, d + 3, d + 6, d + 8, r, J);
      for (int a = 0; a < 4; ++a) {
        int m = 0;
        for (int i = 0; i < 6; ++i) {
          for (int j = 0; j <= i; ++j) H[m++] += J[a][i] * J[a][j];
          g[i] += J[a][i] * r[a];
        }
        cost += r[a] * r[a];
      }
    }
    double d[6], pn[6], Rn[9];
    if (!solve6(H, g, lam, d)) {
      lam = fmin(lam * 10.0, 1e12);
      continue;
    }
    for (int i = 0; i < 6; ++i) pn[i] = pp[i] + d[i];
    rodrigues(pn, Rn);
    double cn = 0.0;
    for (int k = 0; k < kVoSample; ++k) {
      double r[4], J[4][6];
      const double* d = smp[h][k];
      vo_residual<false>(pn, Rn, P, d, d + 3, d + 6, d + 8, r, J);
      cn += r[0] * r[0] + r[1] * r[1] + r[2] * r[2] + r[3] * r[3];
    }
    if (cn < cost) {
      for (int i = 0; i < 6; ++i) pp[i] = pn[i];
      lam = fmax(lam * 0.1, 1e-12);
    } else {
      lam = fmin(lam * 10.0, 1e12);
    }
  }
  if (h < max_iter)
    for (int i = 0; i < 6; ++i) ws_pp[((size_t)b * max_iter + h) * 6 + i] = pp[i];
}

// Error of hypothesis h of pair b over all points (:144-146):
// np.sum(np.linalg.norm(f.reshape((2N, 2)), axis=1)) in numpy's order: chunks
// of 8192 norms summed in sequence, each chunk a pairwise sum (leaves of <= 128
// with 8 accumulators; halves split at multiples of 8).  One workgroup: the
// norms of a chunk in LDS (one pass of all lanes), the leaves summed in
// parallel, the tree combined by one lane in the recursion's order.
constexpr int kErrWG = 256;
constexpr int kNpChunk = 8192;
constexpr int kMaxLeaves = 160;

__device__ __forceinline__ double leaf_sum(const double* a, int n) {
  if (n < 8) {
    double r = 0.0;
    for (int i = 0; i < n; ++i) r += a[i];
    return r;
  }
  double r0 = a[0], r1 = a[1], r2 = a[2], r3 = a[3], r4 = a[4], r5 = a[5], r6 = a[6], r7 = a[7];
  int i = 8;
  for (; i < n - (n % 8); i += 8) {
    r0 += a[i]; r1 += a[i + 1]; r2 += a[i + 2]; r3 += a[i + 3];
    r4 += a[i + 4]; r5 += a[i + 5]; r6 += a[i + 6]; r7 += a[i + 7];
  }
  double res = ((r0 + r1) + (r2 + r3)) + ((r4 + r5) + (r6 + r7));
  for (; i < n; ++i) res += a[i];
  return res;
}

__global__ __launch_bounds__(kErrWG) void k_vo_err(
    const double* __restrict__ q1a, const double* __restrict__ q2a, const double* __restrict__ Q1a,
    const double* __restrict__ Q2a, const int32_t* __restrict__ count, int cap,
    const double* __restrict__ Pg, int max_iter, const double* __restrict__ ws_pp,
    double* __restrict__ ws_err) {
  extern __shared__ double nrm[];  // min(2N, kNpChunk) norms of the current chunk
  __shared__ double lsum[kMaxLeaves];
  __shared__ int llo[kMaxLeaves], lnn[kMaxLeaves];
  __shared__ int nleaves;
  // thread 0's recursion stacks live in LDS (dynamically indexed registers
  // would go to scratch)
  __shared__ int st_lo[32], st_n[32], fs[32];
  __shared__ double vals[32];
  const int h = blockIdx.x, b = blockIdx.y, t = threadIdx.x;
  const int N = min(max(count[b], 0), cap);
  if (N <= 0) return;
  const double* q1 = q1a + (size_t)b * cap * 2;
  const double* q2 = q2a + (size_t)b * cap * 2;
  const double* Q1 = Q1a + (size_t)b * cap * 3;
  const double* Q2 = Q2a + (size_t)b * cap * 3;
  double P[12], pp[6], R[9];
  for (int i = 0; i < 12; ++i) P[i] = Pg[i];
  for (int i = 0; i < 6; ++i) pp[i] = ws_pp[((size_t)b * max_iter + h) * 6 + i];
  rodrigues(pp, R);
  const int M = 2 * N;
  double total = 0.0;
  for (int c0 = 0; c0 < M; c0 += kNpChunk) {
    const int n = min(kNpChunk, M - c0);
    for (int k = t; k < n; k += kErrWG) {
      const int kk = c0 + k;
      const double f0 = vo_elem(pp, R, P, Q1, Q2, q1, q2, N, 2 * kk);
      const double f1 = vo_elem(pp, R, P, Q1, Q2, q1, q2, N, 2 * kk + 1);
      nrm[k] = sqrt(f0 * f0 + f1 * f1);
    }
    if (t == 0) {  // leaves of pairwise_sum(nrm, n), left to right
      int sp = 0, nl = 0;
      st_lo[sp] = 0;
      st_n[sp++] = n;
      while (sp > 0) {
        --sp;
        const int lo = st_lo[sp], m = st_n[sp];
        if (m <= 128) {
          llo[nl] = lo;
          lnn[nl++] = m;
        } else {
          int m2 = m / 2;
          m2 -= m2 % 8;
          st_lo[sp] = lo + m2;  // right half below the left one
          st_n[sp++] = m - m2;
          st_lo[sp] = lo;
          st_n[sp++] = m2;
        }
      }
      nleaves = nl;
    }
    __syncthreads();
    for (int i = t; i < nleaves; i += kErrWG) lsum[i] = leaf_sum(nrm + llo[i], lnn[i]);
    __syncthreads();
    if (t == 0) {  // combine in the recursion's order (post-order, explicit stacks)
      int* fn = st_n;  // the leaf stacks are free again
      int fp = 0, next = 0, vp = 0;
      fn[fp] = n;
      fs[fp++] = 0;
      while (fp > 0) {
        const int m = fn[fp - 1];
        if (m <= 128) {
          --fp;
          vals[vp++] = lsum[next++];
          continue;
        }
        int m2 = m / 2;
        m2 -= m2 % 8;
        if (fs[fp - 1] == 0) {
          fs[fp - 1] = 1;
          fn[fp] = m2;
          fs[fp++] = 0;
        } else if (fs[fp - 1] == 1) {
          fs[fp - 1] = 2;
          fn[fp] = m - m2;
          fs[fp++] = 0;
        } else {
          --fp;
          const double r = vals[--vp];
          const double l = vals[--vp];
          vals[vp++] = l + r;
        }
      }
      total += vals[0];
    }
    __syncthreads();
  }
  if (t == 0) ws_err[(size_t)b * max_iter + h] = total;
}

// the sequential loop of :138-154 over the hypotheses' errors in order
__global__ void k_vo_select(const int32_t* __restrict__ count, int cap, int batch, int max_iter,
                            int early_stop, const double* __restrict__ ws_pp,
                            const double* __restrict__ ws_err, double* __restrict__ pose,
                            int32_t* __restrict__ best_out, int32_t* __restrict__ ntried,
                            double* __restrict__ err_out) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= batch) return;
  const int N = min(max(count[b], 0), cap);
  double mn = INFINITY;
  int best = -1, tried = 0, early = 0;
  if (N > 0)
    for (int k = 0; k < max_iter; ++k) {
      tried = k + 1;
      const double e = ws_err[(size_t)b * max_iter + k];
      if (e < mn) {
        mn = e;
        best = k;
        early = 0;
      } else {
        ++early;
      }
      if (early == early_stop) break;
    }
  for (int i = 0; i < 6; ++i)
    pose[6 * b + i] = best >= 0 ? ws_pp[((size_t)b * max_iter + best) * 6 + i] : 0.0;
  best_out[b] = best;
  ntried[b] = tried;
  err_out[b] = mn;
}

// reprojection_residuals(dof, q1, q2, Q1, Q2) (:65-81): f [batch][4 cap], the
// first 4 count[b] entries of item b in the reference's flat order
__global__ __launch_bounds__(kBS) void k_vo_residuals(
    const double* __restrict__ dof, const double* __restrict__ q1a, const double* __restrict__ q2a,
    const double* __restrict__ Q1a, const double* __restrict__ Q2a,
    const int32_t* __restrict__ count, int cap, const double* __restrict__ Pg,
    double* __restrict__ out) {
  const int b = blockIdx.y, i = blockIdx.x * kBS + threadIdx.x;
  const int N = min(max(count[b], 0), cap);
  if (i >= 4 * N) return;
  double p[6], P[12], R[9];
  for (int k = 0; k < 6; ++k) p[k] = dof[6 * b + k];
  for (int k = 0; k < 12; ++k) P[k] = Pg[k];
  rodrigues(p, R);
  out[(size_t)b * 4 * cap + i] =
      vo_elem(p, R, P, Q1a + (size_t)b * cap * 3, Q2a + (size_t)b * cap * 3,
              q1a + (size_t)b * cap * 2, q2a + (size_t)b * cap * 2, N, i);
}
}  // namespace

// --------------------------------------------------------------- pose chain
// main.py:94-98, 120-124 on the device: T_b = [Rodrigues(-rvec_b) | -tvec_b]
// (transformation.py:15-19's sign flip) when PnP ran (ninl >= 0), else the
// previous T is reused (stale); pose_{b+1} = pose_b @ T_b.  state [32] =
// (pose 4x4, T 4x4) row-major carries the chain across calls, so consecutive
// tracking batches chain without a host round trip.  One lane: B 4x4 products.
// Pose chain of a batch (main.py:94-98,120-124): lanes build the pairs' T_b
// (Rodrigues of -rvec, -tvec) in parallel into LDS, then 16 lanes advance
// P <- P T one element each (the same expression as the serial form, so the
// poses are bit-identical), a pair with ninl < 0 keeping the previous T.
// (One lane doing both for every pair was 41 us per 32 pairs.)
__global__ __launch_bounds__(64) void k_pose_chain(const double* __restrict__ rvec,
                                                   const double* __restrict__ tvec,
                                                   const int32_t* __restrict__ ninl, int B,
                                                   double* __restrict__ state,
                                                   double* __restrict__ poses) {
  __shared__ double Tb[64][16];
  __shared__ int val[64];
  __shared__ double P[16], T[16];
  const int t = threadIdx.x;
  if (t < 16) {
    P[t] = state[t];
    T[t] = state[16 + t];
  }
  const int ei = (t & 15) >> 2, ej = t & 3;
  for (int b0 = 0; b0 < B; b0 += 64) {
    const int nb = min(64, B - b0), b = b0 + t;
    if (t < nb) {
      const bool v = ninl[b] >= 0;
      val[t] = v ? 1 : 0;
      if (v) {
        const double r[3] = {-rvec[3 * b], -rvec[3 * b + 1], -rvec[3 * b + 2]};
        double R[9];
        rodrigues(r, R);
        for (int i = 0; i < 3; ++i) {
          for (int j = 0; j < 3; ++j) Tb[t][4 * i + j] = R[3 * i + j];
          Tb[t][4 * i + 3] = -tvec[3 * b + i];
        }
        Tb[t][12] = 0.0; Tb[t][13] = 0.0; Tb[t][14] = 0.0; Tb[t][15] = 1.0;
      }
    }
    __syncthreads();
    for (int k = 0; k < nb; ++k) {
      if (val[k] && t < 16) T[t] = Tb[k][t];
      __syncthreads();
      double n = 0.0;
      if (t < 16)
        n = P[4 * ei] * T[ej] + P[4 * ei + 1] * T[4 + ej] + P[4 * ei + 2] * T[8 + ej] +
            P[4 * ei + 3] * T[12 + ej];
      __syncthreads();
      if (t < 16) {
        P[t] = n;
        poses[16 * (b0 + k) + t] = n;
      }
      __syncthreads();
    }
  }
  if (t < 16) {
    state[t] = P[t];
    state[16 + t] = T[t];
  }
}

extern "C" int slam_gather_matches(const float* d_kpq, int kq_cap, const float* d_kpt, int kt_cap,
                                   const uint8_t* d_desq, const uint8_t* d_dest,
                                   const int32_t* d_pairs, const int32_t* d_count, int p_cap,
                                   int batch, double* d_ptq, double* d_ptt, uint8_t* d_dq,
                                   uint8_t* d_dt, void* stream) {
  SLAM_REQUIRE(batch >= 0 && p_cap >= 0 && kq_cap >= 0 && kt_cap >= 0,
               "slam_gather_matches: bad shape");
  if (batch == 0 || p_cap == 0) return SLAM_OK;
  SLAM_REQUIRE(d_kpq && d_kpt && d_pairs && d_count && d_ptq && d_ptt,
               "slam_gather_matches: null pointer");
  SLAM_REQUIRE((d_dq == nullptr) == (d_dt == nullptr) && (d_dq == nullptr || (d_desq && d_dest)),
               "slam_gather_matches: descriptor pointers must be all set or all null");
  dim3 grid((p_cap + kBS - 1) / kBS, batch);
  k_gather<<<grid, kBS, 0, slam::as_stream(stream)>>>(
      d_kpq, kq_cap, d_kpt, kt_cap, d_desq, d_dest, reinterpret_cast<const int2*>(d_pairs),
      d_count, p_cap, d_ptq, d_ptt, d_dq, d_dt);
  SLAM_LAUNCHED("k_gather");
  return SLAM_OK;
}

extern "C" int slam_gather_temporal(const double* d_X, const double* d_ptl, int xcap,
                                    const float* d_kp_next, int kcap, const int32_t* d_pairs,
                                    const int32_t* d_count, int pcap, int batch, double* d_Q1,
                                    double* d_q2, double* d_q1, void* stream) {
  SLAM_REQUIRE(batch >= 0 && pcap >= 0 && xcap >= 0 && kcap >= 0,
               "slam_gather_temporal: bad shape");
  if (batch == 0 || pcap == 0) return SLAM_OK;
  SLAM_REQUIRE(d_X && d_ptl && d_kp_next && d_pairs && d_count && d_Q1 && d_q2 && d_q1,
               "slam_gather_temporal: null pointer");
  dim3 grid((pcap + kBS - 1) / kBS, batch);
  k_gather_temporal<<<grid, kBS, 0, slam::as_stream(stream)>>>(
      d_X, d_ptl, xcap, d_kp_next, kcap, reinterpret_cast<const int2*>(d_pairs), d_count, pcap,
      d_Q1, d_q2, d_q1);
  SLAM_LAUNCHED("k_gather_temporal");
  return SLAM_OK;
}

extern "C" int slam_triangulate(const double* d_ptl, const double* d_ptr, const int32_t* d_count,
                                int cap, int batch, const double* d_Pl, const double* d_Pr,
                                int proj_stride, double* d_X, void* stream) {
  SLAM_REQUIRE(batch >= 0 && cap >= 0, "slam_triangulate: bad shape");
  SLAM_REQUIRE(proj_stride == 0 || proj_stride == 12, "slam_triangulate: proj_stride 0 or 12");
  if (batch == 0 || cap == 0) return SLAM_OK;
  SLAM_REQUIRE(d_ptl && d_ptr && d_count && d_Pl && d_Pr && d_X, "slam_triangulate: null pointer");
  dim3 grid((cap + kBS - 1) / kBS, batch);
  k_triangulate<<<grid, kBS, 0, slam::as_stream(stream)>>>(d_ptl, d_ptr, d_count, cap, d_Pl, d_Pr,
                                                           proj_stride, d_X);
  SLAM_LAUNCHED("k_triangulate");
  return SLAM_OK;
}

extern "C" long long slam_pnp_workspace_len(int batch, int n_hyp) {
  return (long long)batch * n_hyp * 6;
}

extern "C" int slam_pnp_ransac(const double* d_Q, const double* d_q, const int32_t* d_count,
                               int cap, int batch, const double* d_K, uint64_t seed, int item0,
                               int n_hyp, double reproj_thresh, int hyp_iters, int refine_iters,
                               double* d_rvec, double* d_tvec, int32_t* d_ninliers,
                               uint8_t* d_mask, double* d_ws, long long ws_len, void* stream) {
  SLAM_REQUIRE(batch >= 0 && cap >= 0, "slam_pnp_ransac: bad shape");
  SLAM_REQUIRE(n_hyp >= 1 && n_hyp <= kMaxHyp, "slam_pnp_ransac: n_hyp in [1, %d]", kMaxHyp);
  SLAM_REQUIRE(hyp_iters >= 0 && refine_iters >= 0 && reproj_thresh > 0,
               "slam_pnp_ransac: bad iteration/threshold arguments");
  if (batch == 0) return SLAM_OK;
  SLAM_REQUIRE(d_Q && d_q && d_count && d_K && d_rvec && d_tvec && d_ninliers && d_mask && d_ws,
               "slam_pnp_ransac: null pointer");
  if (ws_len < slam_pnp_workspace_len(batch, n_hyp)) {
    slam::set_error("slam_pnp_ransac: workspace %lld < %lld doubles", ws_len,
                    slam_pnp_workspace_len(batch, n_hyp));
    return SLAM_ERR_WORKSPACE;
  }
  hipStream_t s = slam::as_stream(stream);
  const dim3 hgrid(batch, (n_hyp + kHypGroups - 1) / kHypGroups);
  k_pnp_hyp<<<hgrid, 64, 0, s>>>(d_Q, d_q, d_count, cap, d_K, seed, item0, n_hyp, d_ws);
  SLAM_LAUNCHED("k_pnp_hyp");
  k_pnp_hyp_lm<<<hgrid, 64, 0, s>>>(d_Q, d_q, d_count, cap, d_K, seed, item0, n_hyp, hyp_iters,
                                    d_ws);
  SLAM_LAUNCHED("k_pnp_hyp_lm");
  k_pnp<<<batch, kPnPWG, 0, s>>>(d_Q, d_q, d_count, cap, d_K, seed, item0, n_hyp, reproj_thresh,
                                 hyp_iters, refine_iters, d_rvec, d_tvec, d_ninliers, d_mask,
                                 d_ws);
  SLAM_LAUNCHED("k_pnp");
  return SLAM_OK;
}

extern "C" int slam_vo_pose_workspace_bytes(int batch, int max_iter, size_t* bytes) {
  SLAM_REQUIRE(batch >= 0 && max_iter >= 1 && bytes, "slam_vo_pose_workspace_bytes: bad args");
  *bytes = (size_t)batch * max_iter * 7 * sizeof(double) + 256;
  return SLAM_OK;
}

extern "C" int slam_vo_estimate_pose(const double* d_q1, const double* d_q2, const double* d_Q1,
                                     const double* d_Q2, const int32_t* d_count, int cap,
                                     int batch, const double* d_P, uint64_t seed, int item0,
                                     int max_iter, int lm_iters, int early_stop, double* d_pose,
                                     int32_t* d_best, int32_t* d_ntried, double* d_err,
                                     void* d_ws, size_t ws_bytes, void* stream) {
  SLAM_REQUIRE(batch >= 0 && cap >= 0, "slam_vo_estimate_pose: bad shape");
  SLAM_REQUIRE(max_iter >= 1 && max_iter <= kVoWG, "slam_vo_estimate_pose: max_iter in [1, %d]",
               kVoWG);
  SLAM_REQUIRE(lm_iters >= 0 && early_stop >= 1, "slam_vo_estimate_pose: bad lm_iters/early_stop");
  if (batch == 0) return SLAM_OK;
  SLAM_REQUIRE(d_q1 && d_q2 && d_Q1 && d_Q2 && d_count && d_P && d_pose && d_best && d_ntried &&
                   d_err,
               "slam_vo_estimate_pose: null pointer");
  SLAM_REQUIRE(d_ws != nullptr, "slam_vo_estimate_pose: null workspace");
  size_t need = 0;
  if (int rc = slam_vo_pose_workspace_bytes(batch, max_iter, &need)) return rc;
  if (ws_bytes < need) {
    slam::set_error("slam_vo_estimate_pose: workspace %zu < %zu bytes", ws_bytes, need);
    return SLAM_ERR_WORKSPACE;
  }
  double* ws_pp = static_cast<double*>(d_ws);
  double* ws_err = ws_pp + (size_t)batch * max_iter * 6;
  hipStream_t s = slam::as_stream(stream);
  k_vo_hyp<<<batch, kVoWG, 0, s>>>(d_q1, d_q2, d_Q1, d_Q2, d_count, cap, d_P, seed, item0,
                                   max_iter, lm_iters, ws_pp);
  SLAM_LAUNCHED("k_vo_hyp");
  const size_t lds = sizeof(double) * (size_t)min(2 * cap, kNpChunk);
  k_vo_err<<<dim3(max_iter, batch), kErrWG, lds, s>>>(d_q1, d_q2, d_Q1, d_Q2, d_count, cap, d_P,
                                                      max_iter, ws_pp, ws_err);
  SLAM_LAUNCHED("k_vo_err");
  k_vo_select<<<(batch + 63) / 64, 64, 0, s>>>(d_count, cap, batch, max_iter, early_stop, ws_pp,
                                               ws_err, d_pose, d_best, d_ntried, d_err);
  SLAM_LAUNCHED("k_vo_select");
  return SLAM_OK;
}

extern "C" int slam_vo_residuals(const double* d_dof, const double* d_q1, const double* d_q2,
                                 const double* d_Q1, const double* d_Q2, const int32_t* d_count,
                                 int cap, int batch, const double* d_P, double* d_res,
                                 void* stream) {
  SLAM_REQUIRE(batch >= 0 && cap >= 0, "slam_vo_residuals: bad shape");
  if (batch == 0 || cap == 0) return SLAM_OK;
  SLAM_REQUIRE(d_dof && d_q1 && d_q2 && d_Q1 && d_Q2 && d_count && d_P && d_res,
               "slam_vo_residuals: null pointer");
  dim3 grid((4 * cap + kBS - 1) / kBS, batch);
  k_vo_residuals<<<grid, kBS, 0, slam::as_stream(stream)>>>(d_dof, d_q1, d_q2, d_Q1, d_Q2,
                                                           d_count, cap, d_P, d_res);
  SLAM_LAUNCHED("k_vo_residuals");
  return SLAM_OK;
}

extern "C" int slam_pose_chain(const double* d_rvec, const double* d_tvec,
                               const int32_t* d_ninliers, int batch, double* d_state,
                               double* d_poses, void* stream) {
  SLAM_REQUIRE(batch >= 0, "slam_pose_chain: batch < 0");
  if (batch == 0) return SLAM_OK;
  SLAM_REQUIRE(d_rvec && d_tvec && d_ninliers && d_state && d_poses, "slam_pose_chain: null pointer");
  k_pose_chain<<<1, 64, 0, slam::as_stream(stream)>>>(d_rvec, d_tvec, d_ninliers, batch, d_state,
                                                     d_poses);
  SLAM_LAUNCHED("k_pose_chain");
  return SLAM_OK;
}

#ifdef SLAM_PNPH_TRACE
extern "C" int slam_pnph_trace(unsigned long long* out) {
  SLAM_HIP(hipDeviceSynchronize());
  SLAM_HIP(hipMemcpyFromSymbol(out, HIP_SYMBOL(g_pnph), 8 * sizeof(unsigned long long)));
  return SLAM_OK;
}
#endif
