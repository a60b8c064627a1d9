// Levenberg-Marquardt bundle adjustment (BAL model) for gfx950.
//
// Replaces the reference's BAL block (/root/reference/BundleAdjustment.py:287-402:
// rotate, project, objective with its two >5000 px clamps, the 2x12 sparsity
// and scipy least_squares TRF) with LM on the normal equations, all state on
// the device so a fixed number of iterations runs with no host round trip.
//
// One LM iteration = 4 launches (local BA):
//   k_linearize     point group -> residuals + Jacobians, V*_p, e_p = V*^-1 g_p,
//                                  W_o = Jc^T Jp, u_o = Jp e_p, and the group's
//                                  slot partials of the reduced camera system:
//                                  per camera U - sum Y W^T, Jc^T r, Jc^T u;
//                                  per camera pair sum Y_o1 W_o2^T
//   k_assemble      block  -> S = sum of its slot partials in group order,
//                             b = -Jc^T r - Jc^T u, g, diag U, cost
//   (all-reduce of sys over ranks happens here for multi-GPU)
//   k_solve_blk     1 WG   -> damp, blocked LDL^T (MFMA trailing updates), camera
//                             step, pred_cam, trial cameras (tiled k_tl3_flow / k_tl2_* for 9C > 120)
//   k_back_trial    point group -> point step, trial points, trial |r|^2 and
//                                  pred partials; the last group sums them into
//                                  small (and, single rank, decides)
//   (all-reduce of small over ranks, then k_decide)
//   k_decide        1 lane -> rho, accept/reject, lambda update, buffer swap
#include "common.hpp"

#include <cmath>

namespace {

typedef double d4 __attribute__((ext_vector_type(4)));

// Cross-workgroup hand-off inside one launch (ticket pattern): the partials
// are stored and loaded with agent-scope relaxed atomics, i.e. write-through
// `sc1` stores and `sc1` loads that bypass the per-XCD L2, so no L2-wide
// release/acquire fence is needed (MI355X_MICROARCH.md, correctness table).
__device__ __forceinline__ void st_sc1(double* p, double v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ double ld_sc1(const double* p) {
  return __hip_atomic_load(const_cast<double*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ unsigned ticket_add(uint32_t* p) {
  return __hip_atomic_fetch_add(p, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void ticket_reset(uint32_t* p) {
  __hip_atomic_store(p, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

constexpr double kClamp = 5000.0;
constexpr double kDiagMin = 1e-6, kDiagMax = 1e32;
constexpr double kLamMin = 1e-16, kLamMax = 1e32;
constexpr int kBS = 256;   // block size of the element-wise kernels

// Batched LM: independent problems (local-BA windows) advance through one set
// of launches, one problem per blockIdx.y; each keeps its own buffers and LM
// state, so the iterates of a batched problem equal its solo iterates.  The
// problem descriptors travel by value in the kernel arguments (16 x 392 B).
constexpr int kBaMaxBatch = SLAM_BA_MAX_BATCH;
struct BaBatch {
  slam_ba_problem p[kBaMaxBatch];
};
#define BA_PROB(b) const slam_ba_problem& p = (b).p[blockIdx.y]
// The batched per-observation / per-block launches (grid x = the problem's
// workgroups, y = problem) with 8k problems: workgroups are dealt round-robin
// over the 8 XCDs (for speed only; nothing depends on it), so the linear
// workgroup id is remapped to keep each problem's workgroups on one XCD --
// problem w's observations, points and partial rows stay in that XCD's L2
// from k_lin_mfma through k_assemble to k_back_trial.  The same (x, problem)
// pairs run either way, so results do not change.
#ifndef SLAM_BA_XCD
#define SLAM_BA_XCD 1
#endif
__device__ __forceinline__ int2 ba_xcd_map() {
  const int gx = (int)gridDim.x, n = (int)gridDim.y;
  if (!SLAM_BA_XCD || n < 8 || (n & 7)) return int2{(int)blockIdx.x, (int)blockIdx.y};
  const int lin = (int)blockIdx.y * gx + (int)blockIdx.x;
  const int xcd = lin & 7, slot = lin >> 3;  // n gx / 8 slots per XCD: its n / 8 problems
  const int wi = slot / gx;
  return int2{slot - wi * gx, xcd + 8 * wi};
}
#define BA_PROB_X(b)                 \
  const int2 bw_ = ba_xcd_map();     \
  const int bx = bw_.x;              \
  const slam_ba_problem& p = (b).p[bw_.y]
// the batch travels by value in the kernel arguments: 16 x 392 B,
// beyond the traditional 4 KB; ROCm 7.2 takes it (tests/test_ba.py launches 16)
static_assert(sizeof(slam_ba_problem) <= 392, "slam_ba_problem grew: re-check the kernarg size");
static_assert(sizeof(BaBatch) <= 16 * 392, "BaBatch kernel argument size");

// The LM kernels are short and latency-bound and usually share their CUs with
// the (throughput-bound) ORB workgroups of the concurrent tracking stream: they
// raise their waves' issue priority so their dependent chains are issued first
// and the ORB waves fill the gaps.
__device__ __forceinline__ void lm_wave_priority() { __builtin_amdgcn_s_setprio(3); }

// ---------------------------------------------------------------- projection
// Residual (proj - q) of BundleAdjustment.py:317-337 with the operation order
// of the numpy code, and optionally its analytic 2x12 Jacobian.
// Per-camera part of the projection: everything that depends on the rotation
// vector only (theta, v, cos, sin, R and the Jacobian's A matrix), computed
// once per camera by cam_prep and stored as a 32-double record; the per-
// observation part (reproject_pre) then does no sqrt/sin/cos/division by theta.
// Both halves keep the operation order of the single-function form, so
// results are bit-identical to computing everything per observation.
constexpr int kCamRec = 32;  // c s omc v(3) R(9) A(9) inv small t(3) f k1 k2 pad(0)
__device__ __forceinline__ void cam_prep(const double* __restrict__ cam, double* __restrict__ o) {
  const double w0 = cam[0], w1 = cam[1], w2 = cam[2];
  const double th = sqrt(w0 * w0 + w1 * w1 + w2 * w2);
  double v0 = 0.0, v1 = 0.0, v2 = 0.0;  // nan_to_num(w / 0) == 0  (:292-293)
  if (th > 0.0) {
    v0 = w0 / th;
    v1 = w1 / th;
    v2 = w2 / th;
  }
  const double c = cos(th), s = sin(th);
  const double omc = 1.0 - c;
  // R = c I + s [v]x + (1-c) v v^T
  double R[3][3];
  R[0][0] = c + omc * v0 * v0; R[0][1] = -s * v2 + omc * v0 * v1; R[0][2] = s * v1 + omc * v0 * v2;
  R[1][0] = s * v2 + omc * v1 * v0; R[1][1] = c + omc * v1 * v1; R[1][2] = -s * v0 + omc * v1 * v2;
  R[2][0] = -s * v1 + omc * v2 * v0; R[2][1] = s * v0 + omc * v2 * v1; R[2][2] = c + omc * v2 * v2;
  // dRX/dw (Gallego & Yezzi): -R [X]x A / |w|^2 with A = w w^T + (R^T - I)[w]x
  const double th2 = w0 * w0 + w1 * w1 + w2 * w2;
  const double W[3][3] = {{0.0, -w2, w1}, {w2, 0.0, -w0}, {-w1, w0, 0.0}};
  const double w[3] = {w0, w1, w2};
  double A[3][3];
  for (int i = 0; i < 3; ++i)
    for (int k = 0; k < 3; ++k) {
      double acc = w[i] * w[k];
      for (int j = 0; j < 3; ++j) acc += R[j][i] * W[j][k];
      A[i][k] = acc - W[i][k];
    }
  o[0] = c; o[1] = s; o[2] = omc;
  o[3] = v0; o[4] = v1; o[5] = v2;
  for (int i = 0; i < 9; ++i) o[6 + i] = R[i / 3][i % 3];
  for (int i = 0; i < 9; ++i) o[15 + i] = A[i / 3][i % 3];
  o[24] = th2 < 1e-24 ? 0.0 : -1.0 / th2;
  o[25] = th2 < 1e-24 ? 1.0 : 0.0;
  for (int i = 0; i < 6; ++i) o[26 + i] = cam[3 + i];
}

// Residual (proj - q) of BundleAdjustment.py:317-337 with the operation order
// of the numpy code, and optionally its analytic 2x12 Jacobian, from a camera
// record of cam_prep.
template <bool JAC>
__device__ __forceinline__ void reproject_pre(const double* __restrict__ cr,
                                              const double* __restrict__ X,
                                              const double* __restrict__ q, double r[2],
                                              double J[2][12]) {
  const double c = cr[0], s = cr[1], omc = cr[2];
  const double v0 = cr[3], v1 = cr[4], v2 = cr[5];
  const double X0 = X[0], X1 = X[1], X2 = X[2];
  const double dot = X0 * v0 + X1 * v1 + X2 * v2;
  const double cx0 = v1 * X2 - v2 * X1;
  const double cx1 = v2 * X0 - v0 * X2;
  const double cx2 = v0 * X1 - v1 * X0;
  const double dk = dot * omc;
  const double RX0 = c * X0 + s * cx0 + dk * v0;
  const double RX1 = c * X1 + s * cx1 + dk * v1;
  const double RX2 = c * X2 + s * cx2 + dk * v2;
  const double P0 = RX0 + cr[26], P1 = RX1 + cr[27], P2 = RX2 + cr[28];
  const double p0 = -P0 / P2, p1 = -P1 / P2;
  const double f = cr[29], k1 = cr[30], k2 = cr[31];
  const double n = p0 * p0 + p1 * p1;
  const double rad = 1.0 + k1 * n + k2 * (n * n);
  const double sc = rad * f;
  r[0] = p0 * sc - q[0];
  r[1] = p1 * sc - q[1];
  if constexpr (JAC) {
    double R[3][3], A[3][3];
    for (int i = 0; i < 9; ++i) {
      R[i / 3][i % 3] = cr[6 + i];
      A[i / 3][i % 3] = cr[15 + i];
    }
    double dR[3][3];
    if (cr[25] != 0.0) {  // |w|^2 < 1e-24: -[RX]x
      dR[0][0] = 0.0;  dR[0][1] = RX2;  dR[0][2] = -RX1;
      dR[1][0] = -RX2; dR[1][1] = 0.0;  dR[1][2] = RX0;
      dR[2][0] = RX1;  dR[2][1] = -RX0; dR[2][2] = 0.0;
    } else {
      const double Xs[3][3] = {{0.0, -X2, X1}, {X2, 0.0, -X0}, {-X1, X0, 0.0}};
      double B[3][3];
      for (int i = 0; i < 3; ++i)
        for (int k = 0; k < 3; ++k)
          B[i][k] = Xs[i][0] * A[0][k] + Xs[i][1] * A[1][k] + Xs[i][2] * A[2][k];
      const double inv = cr[24];
      for (int i = 0; i < 3; ++i)
        for (int k = 0; k < 3; ++k)
          dR[i][k] = (R[i][0] * B[0][k] + R[i][1] * B[1][k] + R[i][2] * B[2][k]) * inv;
    }
    // dp/dP
    const double iz = 1.0 / P2;
    const double dpP[2][3] = {{-iz, 0.0, P0 * iz * iz}, {0.0, -iz, P1 * iz * iz}};
    // dproj/dp = sc I + 2 f (k1 + 2 k2 n) p p^T
    const double g2 = 2.0 * f * (k1 + 2.0 * k2 * n);
    const double Dp[2][2] = {{sc + g2 * p0 * p0, g2 * p0 * p1}, {g2 * p1 * p0, sc + g2 * p1 * p1}};
    double D[2][3];
    for (int a = 0; a < 2; ++a)
      for (int k = 0; k < 3; ++k) D[a][k] = Dp[a][0] * dpP[0][k] + Dp[a][1] * dpP[1][k];
    const double pp[2] = {p0, p1};
    for (int a = 0; a < 2; ++a) {
      for (int k = 0; k < 3; ++k) {
        J[a][k] = D[a][0] * dR[0][k] + D[a][1] * dR[1][k] + D[a][2] * dR[2][k];
        J[a][3 + k] = D[a][k];
        J[a][9 + k] = D[a][0] * R[0][k] + D[a][1] * R[1][k] + D[a][2] * R[2][k];
      }
      J[a][6] = pp[a] * rad;
      J[a][7] = pp[a] * (f * n);
      J[a][8] = pp[a] * (f * n * n);
    }
  }
}

// Single-call form (standalone residual / Jacobian entry points).
template <bool JAC>
__device__ __forceinline__ void reproject(const double* __restrict__ cam,
                                          const double* __restrict__ X,
                                          const double* __restrict__ q, double r[2],
                                          double J[2][12]) {
  double cr[kCamRec];
  cam_prep(cam, cr);
  reproject_pre<JAC>(cr, X, q, r, J);
}

// The two clamps of BundleAdjustment.py:339-350 (x first, then y on the
// rescaled row), with the chain rule applied to J when JAC.
template <bool JAC>
__device__ __forceinline__ void clamp_rows(double r[2], double J[2][12]) {
#pragma unroll
  for (int comp = 0; comp < 2; ++comp) {
    const double rc = r[comp];
    if (fabs(rc) > kClamp) {
      const double arc = fabs(rc);
      const double half = comp == 0 ? 613.0 : 185.0;
      if constexpr (JAC) {
        const double a = (half * 2.0) / arc;
        double Jc[12];
        for (int k = 0; k < 12; ++k) Jc[k] = J[comp][k];
        for (int row = 0; row < 2; ++row) {
          const double ratio = r[row] / rc;
          for (int k = 0; k < 12; ++k) J[row][k] = a * (J[row][k] - ratio * Jc[k]);
        }
      }
      r[0] = r[0] / arc * half * 2.0;
      r[1] = r[1] / arc * half * 2.0;
    }
  }
}

// reproject_pre<true> + clamp_rows<true> split over two lanes by Jacobian
// columns: H = 0 the rotation / translation columns 0..5, H = 1 the f, k1, k2
// and point columns 6..11 (Jh[a][k] = J[a][6 H + k]).  Both halves run the
// forward projection; every value is computed with the same operations in
// the same order as the one-lane form (the clamp's chain rule is per column).
template <int H>
__device__ __forceinline__ void reproject_half(const double* __restrict__ cr,
                                               const double* __restrict__ X,
                                               const double* __restrict__ q, double r[2],
                                               double Jh[2][6]) {
  const double c = cr[0], s = cr[1], omc = cr[2];
  const double v0 = cr[3], v1 = cr[4], v2 = cr[5];
  const double X0 = X[0], X1 = X[1], X2 = X[2];
  const double dot = X0 * v0 + X1 * v1 + X2 * v2;
  const double cx0 = v1 * X2 - v2 * X1;
  const double cx1 = v2 * X0 - v0 * X2;
  const double cx2 = v0 * X1 - v1 * X0;
  const double dk = dot * omc;
  const double RX0 = c * X0 + s * cx0 + dk * v0;
  const double RX1 = c * X1 + s * cx1 + dk * v1;
  const double RX2 = c * X2 + s * cx2 + dk * v2;
  const double P0 = RX0 + cr[26], P1 = RX1 + cr[27], P2 = RX2 + cr[28];
  const double p0 = -P0 / P2, p1 = -P1 / P2;
  const double f = cr[29], k1 = cr[30], k2 = cr[31];
  const double n = p0 * p0 + p1 * p1;
  const double rad = 1.0 + k1 * n + k2 * (n * n);
  const double sc = rad * f;
  r[0] = p0 * sc - q[0];
  r[1] = p1 * sc - q[1];
  const double iz = 1.0 / P2;
  const double dpP[2][3] = {{-iz, 0.0, P0 * iz * iz}, {0.0, -iz, P1 * iz * iz}};
  const double g2 = 2.0 * f * (k1 + 2.0 * k2 * n);
  const double Dp[2][2] = {{sc + g2 * p0 * p0, g2 * p0 * p1}, {g2 * p1 * p0, sc + g2 * p1 * p1}};
  double D[2][3];
  for (int a = 0; a < 2; ++a)
    for (int k = 0; k < 3; ++k) D[a][k] = Dp[a][0] * dpP[0][k] + Dp[a][1] * dpP[1][k];
  if constexpr (H == 0) {
    double dR[3][3];
    if (cr[25] != 0.0) {
      dR[0][0] = 0.0;  dR[0][1] = RX2;  dR[0][2] = -RX1;
      dR[1][0] = -RX2; dR[1][1] = 0.0;  dR[1][2] = RX0;
      dR[2][0] = RX1;  dR[2][1] = -RX0; dR[2][2] = 0.0;
    } else {
      double R[3][3], A[3][3];
      for (int i = 0; i < 9; ++i) {
        R[i / 3][i % 3] = cr[6 + i];
        A[i / 3][i % 3] = cr[15 + i];
      }
      const double Xs[3][3] = {{0.0, -X2, X1}, {X2, 0.0, -X0}, {-X1, X0, 0.0}};
      double B[3][3];
      for (int i = 0; i < 3; ++i)
        for (int k = 0; k < 3; ++k)
          B[i][k] = Xs[i][0] * A[0][k] + Xs[i][1] * A[1][k] + Xs[i][2] * A[2][k];
      const double inv = cr[24];
      for (int i = 0; i < 3; ++i)
        for (int k = 0; k < 3; ++k)
          dR[i][k] = (R[i][0] * B[0][k] + R[i][1] * B[1][k] + R[i][2] * B[2][k]) * inv;
    }
    for (int a = 0; a < 2; ++a)
      for (int k = 0; k < 3; ++k) {
        Jh[a][k] = D[a][0] * dR[0][k] + D[a][1] * dR[1][k] + D[a][2] * dR[2][k];
        Jh[a][3 + k] = D[a][k];
      }
  } else {
    double R[3][3];
    for (int i = 0; i < 9; ++i) R[i / 3][i % 3] = cr[6 + i];
    const double pp[2] = {p0, p1};
    for (int a = 0; a < 2; ++a) {
      Jh[a][0] = pp[a] * rad;
      Jh[a][1] = pp[a] * (f * n);
      Jh[a][2] = pp[a] * (f * n * n);
      for (int k = 0; k < 3; ++k) Jh[a][3 + k] = D[a][0] * R[0][k] + D[a][1] * R[1][k] + D[a][2] * R[2][k];
    }
  }
#pragma unroll
  for (int comp = 0; comp < 2; ++comp) {  // clamp_rows<true> on this lane's columns
    const double rc = r[comp];
    if (fabs(rc) > kClamp) {
      const double arc = fabs(rc);
      const double half = comp == 0 ? 613.0 : 185.0;
      const double a = (half * 2.0) / arc;
      double Jc[6];
      for (int k = 0; k < 6; ++k) Jc[k] = Jh[comp][k];
      for (int row = 0; row < 2; ++row) {
        const double ratio = r[row] / rc;
        for (int k = 0; k < 6; ++k) Jh[row][k] = a * (Jh[row][k] - ratio * Jc[k]);
      }
      r[0] = r[0] / arc * half * 2.0;
      r[1] = r[1] / arc * half * 2.0;
    }
  }
}

__device__ __forceinline__ double block_sum(double v, double* lds) {
  // deterministic: fixed shuffle tree then fixed LDS order
  for (int off = 32; off > 0; off >>= 1) v += __shfl_down(v, off, 64);
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  if (lane == 0) lds[wid] = v;
  __syncthreads();
  double s = 0.0;
  if (threadIdx.x == 0) {
    const int nw = (blockDim.x + 63) >> 6;
    for (int w = 0; w < nw; ++w) s += lds[w];
  }
  __syncthreads();
  return s;  // valid on thread 0
}

// ---------------------------------------------------------------- standalone
__global__ __launch_bounds__(kBS) void k_residual(const double* __restrict__ cams,
                                                  const double* __restrict__ pts,
                                                  const int32_t* __restrict__ ci,
                                                  const int32_t* __restrict__ pi,
                                                  const double* __restrict__ qs, int n_obs,
                                                  double* __restrict__ resid,
                                                  double* __restrict__ jac) {
  const int o = blockIdx.x * kBS + threadIdx.x;
  if (o >= n_obs) return;
  double r[2], J[2][12];
  if (jac) {
    reproject<true>(cams + 9 * ci[o], pts + 3 * pi[o], qs + 2 * o, r, J);
    clamp_rows<true>(r, J);
    for (int a = 0; a < 2; ++a)
      for (int k = 0; k < 12; ++k) jac[(size_t)o * 24 + a * 12 + k] = J[a][k];
  } else {
    reproject<false>(cams + 9 * ci[o], pts + 3 * pi[o], qs + 2 * o, r, J);
    clamp_rows<false>(r, J);
  }
  resid[2 * o] = r[0];
  resid[2 * o + 1] = r[1];
}

// ---------------------------------------------------------------- LM kernels
__device__ __forceinline__ int cur_of(const double* state) {
  return state[SLAM_BA_ST_CUR] != 0.0 ? 1 : 0;
}

__device__ __forceinline__ double clampd(double d) { return fmin(fmax(d, kDiagMin), kDiagMax); }

// Layout of sys (the buffer all-reduced across ranks).  Dense (9C <= 120, the
// one-workgroup solver): S [(9C)^2] row-major, all C(C+1)/2 blocks listed.
// Packed (larger systems, tiled solver): only the listed upper blocks
// (diagonal + camera pairs with common points), 81 doubles each, row-major
// (rows of c1, columns of c2).  Then b, g, diag U [9C] each and cost [C].
constexpr int kDenseMaxN = 120;
__host__ __device__ __forceinline__ bool sys_packed(int n_cams) { return 9 * n_cams > kDenseMaxN; }
__host__ __device__ __forceinline__ long long sys_vec_off(int n_cams, int n_blocks) {
  return sys_packed(n_cams) ? 81ll * n_blocks : 81ll * n_cams * n_cams;
}


// Per point: V = sum Jp^T Jp and g = -sum Jp^T r over its observations, in
// observation order (pt_acc per observation row), then V* = V + lam diag(V)
// (diag clamped), V*^-1 by cofactors and e = V*^-1 g (pt_schur).  The
// linearisers and k_back_trial run the same operations in the same order, so
// the back substitution sees bit-identical V*^-1, e, g, diag.
struct PtSchur {
  double V00 = 0, V01 = 0, V02 = 0, V11 = 0, V12 = 0, V22 = 0, g0 = 0, g1 = 0, g2 = 0;
  double d[3], iv[6], e[3];
  __device__ __forceinline__ void acc(double j0, double j1, double j2, double rr) {
    V00 += j0 * j0; V01 += j0 * j1; V02 += j0 * j2;
    V11 += j1 * j1; V12 += j1 * j2; V22 += j2 * j2;
    g0 -= j0 * rr; g1 -= j1 * rr; g2 -= j2 * rr;
  }
  __device__ __forceinline__ void solve(double lam);
};
__device__ __forceinline__ void PtSchur::solve(double lam) {
  d[0] = clampd(V00); d[1] = clampd(V11); d[2] = clampd(V22);
  const double a00 = V00 + lam * d[0], a11 = V11 + lam * d[1], a22 = V22 + lam * d[2];
  const double a01 = V01, a02 = V02, a12 = V12;
  const double c00 = a11 * a22 - a12 * a12;
  const double c01 = a02 * a12 - a01 * a22;
  const double c02 = a01 * a12 - a02 * a11;
  const double c11 = a00 * a22 - a02 * a02;
  const double c12 = a01 * a02 - a00 * a12;
  const double c22 = a00 * a11 - a01 * a01;
  const double det = a00 * c00 + a01 * c01 + a02 * c02;
  const double id = det != 0.0 ? 1.0 / det : 0.0;
  iv[0] = c00 * id; iv[1] = c01 * id; iv[2] = c02 * id;
  iv[3] = c11 * id; iv[4] = c12 * id; iv[5] = c22 * id;
  e[0] = iv[0] * g0 + iv[1] * g1 + iv[2] * g2;
  e[1] = iv[1] * g0 + iv[3] * g1 + iv[4] * g2;
  e[2] = iv[2] * g0 + iv[4] * g1 + iv[5] * g2;
}

constexpr int kCPart = 112;  // per camera slot: U - sum Y W^T (81), Jc^T r, Jc^T u, diag U (9 each), |r|^2, pad
// Point groups: a workgroup owns the contiguous observation range of a group
// of whole points (observations are sorted by point), at most kGrp of them.
constexpr int kGrp = 128;
constexpr int kLinWG = 256;  // k_linearize: obs / point phases use kGrp lanes, slot phase all
constexpr int kSlotLds = 128;  // slot ranges staged in LDS (larger groups read them from memory)
constexpr int kPairLds = 1024; // observation pairs staged in LDS (ditto)

// LDS of k_linearize (65 KB: leaves room for a co-resident ORB workgroup)
struct LinLds {
  double jc[kGrp][18];  // Jc rows (2 x 9)
  double w[kGrp][27];   // W = Jc^T Jp [i][c]; before phase 3: Jp (6), r (2)
  double ru[kGrp][4];   // r0 r1 u0 u1
  double pt[kGrp][9];   // per group point: e (3), V*^-1 (i00 i01 i02 i11 i12 i22)
  int lpt[kGrp];        // group-local point of each observation
  int cobs[kGrp];       // the group's camera-slot observation lists
  int cptr[kSlotLds];   // camera-slot ranges in cobs (when the group has < kSlotLds slots)
  int bptr[kSlotLds];   // block-slot ranges in pairs
  int pairs[kPairLds];  // the group's observation pairs (when <= kPairLds)
};

// Y_o row i (= W_o row i times V*^-1, V*^-1 symmetric) of a group observation
__device__ __forceinline__ void y_row(const double* W, const double* Vi, int i, double y[3]) {
  const double a = W[3 * i], b = W[3 * i + 1], c = W[3 * i + 2];
  y[0] = a * Vi[0] + b * Vi[1] + c * Vi[2];
  y[1] = a * Vi[1] + b * Vi[3] + c * Vi[4];
  y[2] = a * Vi[2] + b * Vi[4] + c * Vi[5];
}

// Linearisation, point elimination and the group's share of the reduced camera
// system, one workgroup per point group:
//   per observation: residual and 2x12 Jacobian (BundleAdjustment.py:317-350
//     + analytic derivative) -> LDS;
//   per point: V = sum Jp^T Jp, g = -sum Jp^T r, V* = V + lam diag(V),
//     V*^-1 (cofactors), e = V*^-1 g;
//   per observation: W = Jc^T Jp, u = Jp e -> LDS;
//   per slot row (a lane owns row i of one slot; slots from the planner):
//     camera slot (c):      U - sum_o Y_o W_o^T, Jc^T r, Jc^T u, diag U, |r|^2
//                           over the group's observations of camera c;
//     block slot (c1 <= c2): sum Y_o1 W_o2^T over the group's observation pairs
//                           o1 < o2 of one point with cameras c1, c2.
// Everything stays in LDS between the phases; only the slot partials (and the
// per-point data the back substitution needs) are written.
// Slot partials of one group (see k_linearize): a lane owns row i of one slot
// (405 lanes' worth at C3: two rounds of the workgroup).
// cptr / bptr: slot ranges (minus coff / boff) into the group's camera-slot
// observations (L.cobs) and observation pairs.
__device__ __forceinline__ void lin_slots(const slam_ba_problem& p, LinLds& L, int cs0, int ncs,
                                          int bs0, int nbs, const int* cptr, int coff,
                                          const int* bptr, int boff, const int* pairs) {
  const int t = threadIdx.x;
  const int* cobs = L.cobs;
  for (int item = t; item < 9 * (ncs + nbs); item += kLinWG) {
    const int sl = item / 9, i = item - 9 * sl;
    double acc[9];
#pragma unroll
    for (int j = 0; j < 9; ++j) acc[j] = 0.0;
    if (sl < ncs) {
      const int s = cs0 + sl;
      double vr = 0.0, vu = 0.0, vd = 0.0, cost = 0.0;
      // the next observation's index and point are fetched one iteration
      // ahead, so each iteration waits on one LDS round trip, not three
      const int qb = cptr[sl] - coff, qe = cptr[sl + 1] - coff;
      int k = cobs[qb < qe ? qb : 0], lk = L.lpt[k];
      for (int q = qb; q < qe; ++q) {
        const int kn = cobs[q + 1 < qe ? q + 1 : q], lkn = L.lpt[kn];
        const double* jc = L.jc[k];
        const double* W = L.w[k];
        double y[3];
        y_row(W, L.pt[lk] + 3, i, y);
        const double a0 = jc[i], a1 = jc[9 + i];
#pragma unroll
        for (int j = 0; j < 9; ++j) {
          const double u = __builtin_fma(a0, jc[j], a1 * jc[9 + j]);
          const double v = __builtin_fma(y[0], W[3 * j], __builtin_fma(y[1], W[3 * j + 1], y[2] * W[3 * j + 2]));
          acc[j] += u - v;
        }
        const double r0 = L.ru[k][0], r1 = L.ru[k][1];
        vr = __builtin_fma(a0, r0, __builtin_fma(a1, r1, vr));
        vu = __builtin_fma(a0, L.ru[k][2], __builtin_fma(a1, L.ru[k][3], vu));
        vd = __builtin_fma(a0, a0, __builtin_fma(a1, a1, vd));
        cost = __builtin_fma(r0, r0, __builtin_fma(r1, r1, cost));
        k = kn;
        lk = lkn;
      }
      double* out = p.cpart + (size_t)p.cslot_row[s] * kCPart;
#pragma unroll
      for (int j = 0; j < 9; ++j) out[9 * i + j] = acc[j];
      out[81 + i] = vr;
      out[90 + i] = vu;
      out[99 + i] = vd;
      if (i == 0) out[108] = cost;
    } else {
      const int sb = sl - ncs, s = bs0 + sb;
      const int qb = bptr[sb] - boff, qe = bptr[sb + 1] - boff;
      int pr = pairs[qb < qe ? qb : 0], lk = L.lpt[pr & 0xffff];
      for (int q = qb; q < qe; ++q) {
        const int prn = pairs[q + 1 < qe ? q + 1 : q], lkn = L.lpt[prn & 0xffff];
        const int k1 = pr & 0xffff, k2 = pr >> 16;
        double y[3];
        y_row(L.w[k1], L.pt[lk] + 3, i, y);
        const double* W2 = L.w[k2];
#pragma unroll
        for (int j = 0; j < 9; ++j)
          acc[j] = __builtin_fma(y[0], W2[3 * j], __builtin_fma(y[1], W2[3 * j + 1], __builtin_fma(y[2], W2[3 * j + 2], acc[j])));
        pr = prn;
        lk = lkn;
      }
      double* out = p.bpart + (size_t)p.bslot_row[s] * 81;
#pragma unroll
      for (int j = 0; j < 9; ++j) out[9 * i + j] = acc[j];
    }
  }
}

#ifdef SLAM_LIN_PROFILE
#define LIN_T(i) const uint64_t lin_t##i = __builtin_amdgcn_s_memtime()
#else
#define LIN_T(i) (void)0
#endif
__global__ __launch_bounds__(kLinWG) void k_linearize(BaBatch bat) {
  BA_PROB_X(bat);
  const int g = bx;
  if (g >= p.n_grps) return;  // batch: grid.x covers the largest problem
  lm_wave_priority();
  __shared__ LinLds L;
  LIN_T(0);
  const int p0 = p.grp_ptr[g], p1 = p.grp_ptr[g + 1];
  const int o0 = p.pt_ptr[p0], o1 = p.pt_ptr[p1];
  const int t = threadIdx.x;
  const int o = o0 + t;
  const bool has = t < kGrp && o < o1;
  const int cur = cur_of(p.state);
  // slot lists of this group -> LDS (their loads overlap the projections)
  const int cs0 = p.grp_cslot[g], ncs = p.grp_cslot[g + 1] - cs0;
  const int bs0 = p.grp_bslot[g], nbs = p.grp_bslot[g + 1] - bs0;
  const int cb0 = p.cslot_obs_ptr[cs0], pb0 = p.bslot_pair_ptr[bs0];
  const int npairs = p.bslot_pair_ptr[bs0 + nbs] - pb0;
  const bool fit_c = ncs < kSlotLds, fit_b = nbs < kSlotLds, fit_p = npairs <= kPairLds;
  if (fit_c && t <= ncs) L.cptr[t] = p.cslot_obs_ptr[cs0 + t] - cb0;
  if (fit_b && t <= nbs) L.bptr[t] = p.bslot_pair_ptr[bs0 + t] - pb0;
  if (t < kGrp && t < o1 - o0) L.cobs[t] = p.cslot_obs[cb0 + t];
  if (fit_p)
    for (int q = t; q < npairs; q += kLinWG) L.pairs[q] = p.bslot_pairs[pb0 + q];
  double r[2], J[2][12];
  if (has) {
    const int pt = p.obs_pt[o];
    reproject_pre<true>(p.camrec[cur] + kCamRec * p.obs_cam[o], p.pts[cur] + 3 * pt,
                        p.obs_q + 2 * o, r, J);
    clamp_rows<true>(r, J);
#pragma unroll
    for (int a = 0; a < 2; ++a) {
#pragma unroll
      for (int i = 0; i < 9; ++i) L.jc[t][9 * a + i] = J[a][i];
#pragma unroll
      for (int c = 0; c < 3; ++c) L.w[t][3 * a + c] = J[a][9 + c];
      L.w[t][6 + a] = r[a];
      L.ru[t][a] = r[a];
    }
    L.lpt[t] = pt - p0;
  }
  __syncthreads();
  LIN_T(1);
  const double lam = p.state[SLAM_BA_ST_LAMBDA];
  if (t < p1 - p0) {
    const int pt = p0 + t;
    PtSchur ps;
    for (int k = p.pt_ptr[pt] - o0; k < p.pt_ptr[pt + 1] - o0; ++k) {
#pragma unroll
      for (int a = 0; a < 2; ++a) ps.acc(L.w[k][3 * a], L.w[k][3 * a + 1], L.w[k][3 * a + 2], L.w[k][6 + a]);
    }
    ps.solve(lam);
#pragma unroll
    for (int k = 0; k < 3; ++k) L.pt[t][k] = ps.e[k];
#pragma unroll
    for (int k = 0; k < 6; ++k) L.pt[t][3 + k] = ps.iv[k];
  }
  __syncthreads();
  if (has) {
    const double* e = L.pt[L.lpt[t]];
#pragma unroll
    for (int i = 0; i < 9; ++i)
#pragma unroll
      for (int c = 0; c < 3; ++c) L.w[t][3 * i + c] = J[0][i] * J[0][9 + c] + J[1][i] * J[1][9 + c];
    L.ru[t][2] = J[0][9] * e[0] + J[0][10] * e[1] + J[0][11] * e[2];
    L.ru[t][3] = J[1][9] * e[0] + J[1][10] * e[1] + J[1][11] * e[2];
  }
  __syncthreads();
  LIN_T(2);
  // the group's slot lists (staged in LDS at kernel start: see below)
  // slot phase: LDS-staged lists when they fit (always at C3), else from memory
  // (two inlined copies, so every list access is a plain ds_read or global load)
  if (fit_c && fit_b && fit_p)
    lin_slots(p, L, cs0, ncs, bs0, nbs, L.cptr, 0, L.bptr, 0, L.pairs);
  else
    lin_slots(p, L, cs0, ncs, bs0, nbs, p.cslot_obs_ptr + cs0, cb0, p.bslot_pair_ptr + bs0, pb0,
              p.bslot_pairs + pb0);
#ifdef SLAM_LIN_PROFILE
  __builtin_amdgcn_s_waitcnt(0);
  __syncthreads();
  LIN_T(3);
  if (g == 7 && t == 0) {
    p.state[12] = (double)(lin_t1 - lin_t0);
    p.state[13] = (double)(lin_t2 - lin_t1);
    p.state[14] = (double)(lin_t3 - lin_t2);
    p.state[15] = (double)(ncs * 100 + nbs);
  }
#endif
}

// ---------------------------------------------------------------- camera-union linearisation
// lin_mode 1 (planner ba.plan_mfma): a workgroup owns a supergroup -- a run of
// chunks (<= kMObs observations, <= kMPts whole points each) whose points
// together see m <= kMCams cameras -- and forms its whole share of the reduced
// camera system as ONE dense (9m x 9m) matrix, on the f64 matrix cores
// (v_mfma_f64_16x16x4_f64):
//   Schur part  T = sum_p Y_p W_p^T: W_p is the point's 9m x 3 column of camera
//               blocks (W~_{p,a} = sum of Jc_o^T Jp_o over its observations by
//               camera a; zero for cameras that do not see p), Y_p = W_p V*_p^-1;
//               one MFMA per point and upper 16x16 tile of T (K = the point's
//               3 coordinates, padded to 4);
//   camera part Z_a = sum over the observation rows of camera a of z^T z with
//               z = [Jc row (9) | r | u | 0]: one 16x16 tile per camera holding
//               U_a = Jc^T Jc, Jc^T r, Jc^T u, diag U and |r|^2 (K = 2 rows of
//               2 observations per MFMA);
// accumulated in registers across the supergroup's chunks and written once:
// per camera a one cpart row (U_a - T_aa, Jc^T r, Jc^T u, diag U, |r|^2), per
// co-observed camera pair a < b one bpart row (T_ab) -- the rows k_assemble
// sums.  Per point: V, g, V*, V*^-1, e (PtSchur, as k_linearize; LDS only).
constexpr int kMObs = 120, kMPts = 16, kMCams = 7, kMRows = 64;
constexpr int kMWG = 256;
constexpr int kSgMeta = 24;  // sg_meta record: ch0 ch1 cs0 m bs0 nb p0 p1 o0 o1 cams[8] pad
constexpr int kMObsS = kMObs + 1;  // odd stride: element-major arrays read across lanes without conflicts
struct alignas(16) MLds {
  // per-observation values stored element-major ([value][obs], stride 121):
  // lanes taking consecutive observations touch consecutive doubles, and the
  // 16 lanes of an MFMA operand group (one observation, 16 values) stride by
  // an odd number of doubles (was [obs][18]: 3 LDS conflict cycles per access)
  double jc[18][kMObsS];         // Jc rows (2 x 9)
  double jp[6][kMObsS];          // Jp rows (2 x 3)
  double ru[4][kMObsS];          // r0 r1 u0 u1
  double vi[kMPts][6];           // V*^-1 (i00 i01 i02 i11 i12 i22)
  double e[kMPts][3];
  double yt[kMPts][3][kMRows];   // Y_p, [point][k][row]: the MFMA A operand
  double wt[kMPts][3][kMRows];   // W_p, [point][k][row]: the MFMA B operand
  double cam[kMCams][kCamRec];   // the supergroup's camera records (live parameters)
  double X[kMPts][3];            // the chunk's points
  double zero;                   // operand of padded MFMA lanes
  int optr[kMPts + 1];           // chunk-local observation range of each point
  int lpt[kMObs];                // chunk-local point of each observation
  int la[kMObs];                 // supergroup-local camera of each observation
  int cobs[kMObs];               // chunk-local observations sorted by camera
  int cptr[8];                   // their per-camera runs
  int crow[kMCams];              // cpart row of each camera slot
  int bab[kMCams * (kMCams - 1) / 2], brow[kMCams * (kMCams - 1) / 2];  // block slots
};
static_assert(sizeof(MLds) <= 80 * 1024, "k_lin_mfma: two workgroups per CU");
static_assert(9 * kMCams <= kMRows, "k_lin_mfma: 9m rows in 4 tile rows");
static_assert(2 * kMPts * 3 * kMRows >= kMRows * kMRows + kMCams * 256, "staging aliases yt/wt");

// -DSLAM_LINM_PROFILE: shader cycles per phase, summed over the workgroup's
// chunks (thread 0, s_memtime): 1 staging (incl. the wait for the prefetched
// loads), 2 projections (A), 3 points (B), 4 W/Y (C), 5 MFMA + U (D),
// 6 write-out (E); slam_linm_stamps reads them (scripts/linm_prof.py).
#ifdef SLAM_LINM_PROFILE
__device__ unsigned long long g_linm_stamp[4096][8];
#define LINM_DECL() unsigned long long linm_prev = __builtin_amdgcn_s_memtime(), linm_acc[7] = {0, 0, 0, 0, 0, 0, 0}
#define LINM_T(i)                                                  \
  do {                                                             \
    if (threadIdx.x == 0) {                                        \
      const unsigned long long linm_now = __builtin_amdgcn_s_memtime(); \
      linm_acc[i] += linm_now - linm_prev;                         \
      linm_prev = linm_now;                                        \
    }                                                              \
  } while (0)
#define LINM_END()                                                               \
  do {                                                                           \
    if (threadIdx.x == 0 && blockIdx.x + 1024 * blockIdx.y < 4096)               \
      for (int linm_i = 0; linm_i < 7; ++linm_i)                                 \
        g_linm_stamp[blockIdx.x + 1024 * blockIdx.y][linm_i] = linm_acc[linm_i]; \
  } while (0)
#else
#define LINM_DECL() (void)0
#define LINM_T(i) (void)0
#define LINM_END() (void)0
#endif

// ---------------------------------------------------------------- folded assembly
// lin_mode 1 with asm_tab (include/slam355.h): k_lin_mfma assembles the reduced
// camera system itself.  Every supergroup adds one to the counter of each block
// it wrote a partial row of, after its (sc1, write-through) row stores have
// drained; the supergroup whose add completes a block (count == need) sums that
// block's rows with sc1 loads -- its add coming last makes it the acquire for
// all the rows (MI355X_MICROARCH.md hand-off table, row 1) -- and writes the
// block into sys; blocks with no partial row here are zeroed by the build.  The
// sums run in a fixed order (rows interleaved over the parts, parts added in
// order), whichever workgroup assembles.  One dependent launch (k_assemble) and
// its wait for CU slots fewer per LM iteration.
struct AsmTab {
  const int32_t* need;
  int32_t* cnt;
  const int32_t* cam_dblk;
  const int32_t* row_blk;
  int n_empty;
  const int32_t* empty;
  __device__ explicit AsmTab(const slam_ba_problem& p) {
    const int nb = p.n_blocks;
    need = p.asm_tab;
    cnt = p.asm_tab + nb;
    cam_dblk = p.asm_tab + 2 * nb;
    row_blk = cam_dblk + p.n_cams;
    n_empty = row_blk[p.n_bslots];
    empty = row_blk + p.n_bslots + 1;
  }
};

// out[e] (e < n) = sum over rows [rb, re) of part[row][e], with kMWG threads:
// nparts = kMWG / n parts (rows rb + k, rb + k + nparts, ...; 4 loads in
// flight), added in part order.  red: LDS [nparts][n].
__device__ void fold_rows_sum(const double* __restrict__ part, int stride, int rb, int re, int n,
                              double* red, double* out) {
  const int t = threadIdx.x;
  const int nparts = kMWG / n, k = t / n, e = t - k * n;
  if (k < nparts) {
    double a[4] = {0.0, 0.0, 0.0, 0.0};
    int r = rb + k;
    for (; r + 3 * nparts < re; r += 4 * nparts) {
      double v[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) v[u] = ld_sc1(part + (size_t)(r + u * nparts) * stride + e);
#pragma unroll
      for (int u = 0; u < 4; ++u) a[u] += v[u];
    }
    for (int u = 0; r < re; r += nparts, ++u) a[u] += ld_sc1(part + (size_t)r * stride + e);
    red[k * n + e] = (a[0] + a[1]) + (a[2] + a[3]);
  }
  __syncthreads();
  if (t < n) {
    double v = 0.0;
    for (int q = 0; q < nparts; ++q) v += red[q * n + t];
    out[t] = v;
  }
  __syncthreads();
}

// sys block blk (+ its camera's vectors when diagonal) from the partial rows;
// the same formulas as k_assemble
__device__ void fold_block(const slam_ba_problem& p, int blk, double* scratch) {
  double* red = scratch;             // [<= 3][112]
  double* sh = scratch + 3 * kCPart;  // [112]
  double* sb = sh + kCPart;           // [81]
  const int c1 = p.blocks[2 * blk], c2 = p.blocks[2 * blk + 1];
  const int C9 = 9 * p.n_cams, t = threadIdx.x;
  double* S = p.sys;
  double* bvec = S + sys_vec_off(p.n_cams, p.n_blocks);
  double* gvec = bvec + C9;
  double* diagU = gvec + C9;
  double* costc = diagU + C9;
  const bool diag = c1 == c2;
  const int bb = p.blk_bslot_ptr[blk], be = p.blk_bslot_ptr[blk + 1];
  if (diag) fold_rows_sum(p.cpart, kCPart, p.cam_cslot_ptr[c1], p.cam_cslot_ptr[c1 + 1], 109, red, sh);
  if (be > bb) {
    fold_rows_sum(p.bpart, 81, bb, be, 81, red, sb);
  } else if (t < 81) {
    sb[t] = 0.0;
  }
  __syncthreads();
  if (sys_packed(p.n_cams)) {
    if (t < 81) S[(size_t)blk * 81 + t] = diag ? sh[t] - (sb[t] + sb[9 * (t % 9) + t / 9]) : -sb[t];
  } else if (t < 81) {
    const int i = t / 9, j = t - 9 * (t / 9);
    if (diag) {
      S[(size_t)(9 * c1 + i) * C9 + 9 * c1 + j] = sh[t] - (sb[t] + sb[9 * j + i]);
    } else {
      S[(size_t)(9 * c1 + i) * C9 + 9 * c2 + j] = -sb[t];
      S[(size_t)(9 * c2 + j) * C9 + 9 * c1 + i] = -sb[t];
    }
  }
  if (diag && t < 9) {
    gvec[9 * c1 + t] = -sh[81 + t];
    bvec[9 * c1 + t] = -sh[81 + t] - sh[90 + t];
    diagU[9 * c1 + t] = sh[99 + t];
  }
  if (diag && t == 0) costc[c1] = sh[108];
  __syncthreads();
}

// a block with no partial row in this problem: zeros (and zero vectors when
// diagonal), every build -- the packed multi-rank sys is all-reduced in place
__device__ void fold_zero_block(const slam_ba_problem& p, int blk, int t0, int nt) {
  const int c1 = p.blocks[2 * blk], c2 = p.blocks[2 * blk + 1];
  const int C9 = 9 * p.n_cams;
  double* S = p.sys;
  double* bvec = S + sys_vec_off(p.n_cams, p.n_blocks);
  for (int e = t0; e < 81; e += nt) {
    const int i = e / 9, j = e - 9 * (e / 9);
    if (sys_packed(p.n_cams)) {
      S[(size_t)blk * 81 + e] = 0.0;
    } else {
      S[(size_t)(9 * c1 + i) * C9 + 9 * c2 + j] = 0.0;
      S[(size_t)(9 * c2 + j) * C9 + 9 * c1 + i] = 0.0;
    }
  }
  if (c1 == c2)
    for (int e = t0; e < 28; e += nt) {  // b, g, diag U (9 each), cost
      if (e < 27) bvec[(size_t)(e / 9) * C9 + 9 * c1 + e % 9] = 0.0;
      else bvec[3 * (size_t)C9 + c1] = 0.0;
    }
}

__device__ void lin_fold_assemble(const slam_ba_problem& p, const int* cams, int m, int nb,
                                  const int* brow, double* scratch) {
  const AsmTab A(p);
  __shared__ int done[kMCams + kMCams * (kMCams - 1) / 2];
  __shared__ int ndone;
  __builtin_amdgcn_s_waitcnt(0);  // this workgroup's partial rows have left (sc1)
  __syncthreads();
  if (threadIdx.x == 0) {
    int n = 0;
    for (int q = 0; q < m + nb; ++q) {
      const int blk = q < m ? A.cam_dblk[cams[q]] : A.row_blk[brow[q - m]];
      const int old = (int)ticket_add(reinterpret_cast<uint32_t*>(A.cnt + blk));
      if (old == A.need[blk] - 1) {
        done[n++] = blk;
        __hip_atomic_store(A.cnt + blk, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // re-armed
      }
    }
    ndone = n;
  }
  __syncthreads();
  for (int q = 0; q < ndone; ++q) fold_block(p, done[q], scratch);
}

__global__ __launch_bounds__(kMWG) void k_lin_mfma(BaBatch bat) {
  BA_PROB_X(bat);
  const int sg = bx;
  if (sg >= p.n_sgrps) return;  // batch: grid.x covers the largest problem
  LINM_DECL();
  lm_wave_priority();
  __shared__ MLds L;
  if (p.asm_tab != nullptr) {  // folded assembly: this supergroup's share of the empty blocks
    const AsmTab A(p);
    for (int q = sg; q < A.n_empty; q += p.n_sgrps) fold_zero_block(p, A.empty[q], threadIdx.x, kMWG);
  }
  const int t = threadIdx.x, lane = t & 63;
  const int wid = __builtin_amdgcn_readfirstlane(t >> 6);
  // the supergroup record (one hop): chunk range, slot ranges, the first
  // chunk's extents, its cameras
  const int* sm = p.sg_meta + kSgMeta * sg;
  const int ch0 = sm[0], ch1 = sm[1], cs0 = sm[2], m = sm[3], bs0 = sm[4], nb = sm[5];
  const int nt = (9 * m + 15) >> 4;  // tile rows of T
  const int cur = cur_of(p.state);
  const double lam = p.state[SLAM_BA_ST_LAMBDA];
  // the supergroup's camera records -> LDS (one load per lane)
  if (t < kMCams * kCamRec) {
    const int a = t / kCamRec, k = t - kCamRec * (t / kCamRec);
    const int c = a < m ? sm[10 + a] : -1;
    if (c >= 0) L.cam[a][k] = p.camrec[cur][(size_t)kCamRec * c + k];
  }
  if (t == 0) L.zero = 0.0;
  // output rows of this supergroup (read at the end; loaded now, off the tail)
  if (t < m) L.crow[t] = p.cslot_row[cs0 + t];
  if (t >= 64 && t - 64 < nb) {
    L.bab[t - 64] = p.bslot_ab[bs0 + t - 64];
    L.brow[t - 64] = p.bslot_row[bs0 + t - 64];
  }
  // this wave's upper tiles of T (I <= J), dealt round-robin: <= 3 per wave;
  // its cameras a = wid, wid + 4 (<= 2)
  int tI[3], tJ[3];
  int ntl = 0;
  {
    int s = 0;
    for (int I = 0; I < nt; ++I)
      for (int J = I; J < nt; ++J, ++s)
        if ((s & 3) == wid && ntl < 3) {
          tI[ntl] = I;
          tJ[ntl] = J;
          ++ntl;
        }
  }
  const int nza = (m > wid) + (m > wid + 4);
  int tRow[3], tCol[3];  // operand rows of this lane for each tile slot
#pragma unroll
  for (int s = 0; s < 3; ++s) {
    tRow[s] = 16 * (s < ntl ? tI[s] : 0) + (lane & 15);
    tCol[s] = 16 * (s < ntl ? tJ[s] : 0) + (lane & 15);
  }
  d4 acc[3], zacc[2];
#pragma unroll
  for (int s = 0; s < 3; ++s) acc[s] = d4{0.0, 0.0, 0.0, 0.0};
#pragma unroll
  for (int s = 0; s < 2; ++s) zacc[s] = d4{0.0, 0.0, 0.0, 0.0};
  const int mi = lane & 15, mk = lane >> 4;

  // chunk extents: the first from the record, the next loaded one chunk ahead;
  // a chunk's inputs are loaded one chunk ahead too (issued after the current
  // chunk is staged, in flight across its phases: barriers wait on LDS only)
  struct ChunkIn {
    double q0, q1, xv;
    int meta, pp, cp;
  };
  auto load_in = [&](int ch, int p0, int p1, int o0, int o1) {
    ChunkIn in{0.0, 0.0, 0.0, 0, 0, 0};
    const int nobs = o1 - o0, npts = p1 - p0;
    const int ko = t & 127;  // (A) splits an observation over lanes t and t + 128
    if (ko < nobs) {
      in.q0 = p.obs_q[2 * (o0 + ko)];
      in.q1 = p.obs_q[2 * (o0 + ko) + 1];
    }
    if (t < nobs) in.meta = p.obs_meta[o0 + t];
    if (t < 3 * npts) in.xv = p.pts[cur][3 * p0 + t];
    if (t >= 128 && t - 128 <= npts) in.pp = p.pt_ptr[p0 + t - 128] - o0;
    if (t < 8) in.cp = p.chk_cptr[8 * ch + t];
    return in;
  };
  int p0 = sm[6], p1 = sm[7], o0 = sm[8], o1 = sm[9];
  int np0 = 0, np1 = 0, no0 = 0, no1 = 0;
  if (ch0 + 1 < ch1) {
    np0 = p.grp_ptr[ch0 + 1];
    np1 = p.grp_ptr[ch0 + 2];
    no0 = p.chk_optr[ch0 + 1];
    no1 = p.chk_optr[ch0 + 2];
  }
  ChunkIn in = load_in(ch0, p0, p1, o0, o1);
  for (int ch = ch0; ch < ch1; ++ch) {
    const int nobs = o1 - o0, npts = p1 - p0;
    const double q0 = in.q0, q1 = in.q1;
    __syncthreads();  // the previous chunk's readers are done with L
    if (t < nobs) {
      L.lpt[t] = in.meta & 255;
      L.la[t] = (in.meta >> 8) & 255;
      L.cobs[t] = in.meta >> 16;
    }
    if (t < 3 * npts) (&L.X[0][0])[t] = in.xv;
    if (t >= 128 && t - 128 <= npts) L.optr[t - 128] = in.pp;
    if (t < 8) L.cptr[t] = in.cp;
    // Y/W operand planes of the chunk's points start at zero (rows of cameras
    // a point is not seen by, rows >= 9m): all 64 rows of each of its 3 npts
    // planes, one contiguous range, 16-byte stores (was: only the 16 nt rows
    // of each plane through the rotation's index math -- 12 % of the kernel)
    {
      typedef double dbl2 __attribute__((ext_vector_type(2)));
      dbl2* y2 = reinterpret_cast<dbl2*>(&L.yt[0][0][0]);
      dbl2* w2 = reinterpret_cast<dbl2*>(&L.wt[0][0][0]);
      const int n2 = npts * 3 * kMRows / 2;
      for (int i = t; i < n2; i += kMWG) {
        y2[i] = dbl2{0.0, 0.0};
        w2[i] = dbl2{0.0, 0.0};
      }
    }
    __syncthreads();
    // prefetch: the next chunk's inputs and the extents of the one after
    int nnp0 = 0, nnp1 = 0, nno0 = 0, nno1 = 0;
    if (ch + 1 < ch1) {
      in = load_in(ch + 1, np0, np1, no0, no1);
      if (ch + 2 < ch1) {
        nnp0 = p.grp_ptr[ch + 2];
        nnp1 = p.grp_ptr[ch + 3];
        nno0 = p.chk_optr[ch + 2];
        nno1 = p.chk_optr[ch + 3];
      }
    }
    LINM_T(1);
    // (A) per observation: residual + Jacobian (BundleAdjustment.py:317-350),
    //     split by Jacobian columns over lanes k and k + 128 (all 4 waves busy;
    //     was lanes 0..119 only)
    {
      const int k = t & 127;
      if (k < nobs) {
        const double q[2] = {q0, q1};
        double r[2], Jh[2][6];
        if (t < 128) {
          reproject_half<0>(L.cam[L.la[k]], L.X[L.lpt[k]], q, r, Jh);
#pragma unroll
          for (int a = 0; a < 2; ++a) {
#pragma unroll
            for (int i = 0; i < 6; ++i) L.jc[9 * a + i][k] = Jh[a][i];
            L.ru[a][k] = r[a];
          }
        } else {
          reproject_half<1>(L.cam[L.la[k]], L.X[L.lpt[k]], q, r, Jh);
#pragma unroll
          for (int a = 0; a < 2; ++a) {
#pragma unroll
            for (int i = 0; i < 3; ++i) L.jc[9 * a + 6 + i][k] = Jh[a][i];
#pragma unroll
            for (int c = 0; c < 3; ++c) L.jp[3 * a + c][k] = Jh[a][3 + c];
          }
        }
      }
    }
    __syncthreads();
    LINM_T(2);
    // (B) per point: V, g, V* = V + lam diag(V), V*^-1 (cofactors), e = V*^-1 g
    if (t < npts) {
      PtSchur ps;
      for (int k = L.optr[t]; k < L.optr[t + 1]; ++k) {
#pragma unroll
        for (int a = 0; a < 2; ++a) ps.acc(L.jp[3 * a][k], L.jp[3 * a + 1][k], L.jp[3 * a + 2][k], L.ru[a][k]);
      }
      ps.solve(lam);
#pragma unroll
      for (int k = 0; k < 3; ++k) L.e[t][k] = ps.e[k];
#pragma unroll
      for (int k = 0; k < 6; ++k) L.vi[t][k] = ps.iv[k];
    }
    __syncthreads();
    LINM_T(3);
    // (C) per observation, rows i of W~ split over two lanes (lane t: rows
    //     0..4, lane t + 128: rows 5..8): W~_{p,a} rows summed over the run of
    //     observations of the same (point, camera) (adjacent: obs are sorted by
    //     point, then camera), Y = W~ V*^-1, into the operand planes; u_o.
    {
      const int h = t >> 7, k0 = t & 127;
      const bool lead = k0 < nobs && (k0 == 0 || L.lpt[k0 - 1] != L.lpt[k0] ||
                                      L.la[k0 - 1] != L.la[k0]);
      if (lead) {
        const int lp = L.lpt[k0], a = L.la[k0];
        const int ib = h ? 5 : 0, ie = h ? 9 : 5;
        double W[5][3];
#pragma unroll
        for (int i = 0; i < 5; ++i)
#pragma unroll
          for (int c = 0; c < 3; ++c) W[i][c] = 0.0;
        for (int k = k0; k < nobs && L.lpt[k] == lp && L.la[k] == a; ++k) {
#pragma unroll
          for (int i = 0; i < 5; ++i) {
            if (ib + i >= ie) break;
#pragma unroll
            for (int c = 0; c < 3; ++c)
              W[i][c] += L.jc[ib + i][k] * L.jp[c][k] + L.jc[9 + ib + i][k] * L.jp[3 + c][k];
          }
        }
        const double* vi = L.vi[lp];
        const double V[3][3] = {{vi[0], vi[1], vi[2]}, {vi[1], vi[3], vi[4]}, {vi[2], vi[4], vi[5]}};
#pragma unroll
        for (int i = 0; i < 5; ++i) {
          if (ib + i >= ie) break;
          const int row = 9 * a + ib + i;
#pragma unroll
          for (int c = 0; c < 3; ++c) {
            const int pos = (row + 16 * ((3 * lp + c) & 3)) & (kMRows - 1);  // see (D)
            L.wt[lp][c][pos] = W[i][c];
            L.yt[lp][c][pos] = W[i][0] * V[0][c] + W[i][1] * V[1][c] + W[i][2] * V[2][c];
          }
        }
      }
      if (h == 0 && k0 < nobs) {
        const double* e = L.e[L.lpt[k0]];
        L.ru[2][k0] = L.jp[0][k0] * e[0] + L.jp[1][k0] * e[1] + L.jp[2][k0] * e[2];
        L.ru[3][k0] = L.jp[3][k0] * e[0] + L.jp[4][k0] * e[1] + L.jp[5][k0] * e[2];
      }
    }
    __syncthreads();
    LINM_T(4);
    // (D) T += sum_p Y_p W_p^T as ONE product over the flat index kk = 3 lp + c
    //     (point lp, coordinate c): K-step s of an MFMA takes kk = 4 s + k
    //     (k = lane >> 4), so the 3 coordinates of consecutive points pack the
    //     K = 4 steps densely -- ceil(3 npts / 4) MFMAs per tile instead of one
    //     per point with K padded 3 -> 4 (-25 %).  Plane kk stores row r at
    //     (r + 16 (kk & 3)) mod 64, so the lane groups k = 0, 1 of an operand
    //     read fall on different LDS banks:
    //     A[i][k] = Y[16I + i][kk], B[k][j] = W[16J + j][kk], kk >= 3 npts -> 0.
    //     Every wave issues 3 tile MFMAs per K-step (a wave with 2 tiles feeds
    //     its third accumulator zeros), so the accumulators stay in their own
    //     AGPRs with no control flow around the MFMAs; operands of 4 K-steps
    //     are loaded before their MFMAs are issued.
    {
      const double* Yf = &L.yt[0][0][0];
      const double* Wf = &L.wt[0][0][0];
      const int nk = 3 * npts;
      for (int k0 = 0; k0 < nk; k0 += 16) {
        double av[4][3], bv[4][3];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const int kk = min(k0 + 4 * u + mk, 3 * kMPts - 1);
#pragma unroll
          for (int s = 0; s < 3; ++s) {
            av[u][s] = Yf[kk * kMRows + ((tRow[s] + 16 * mk) & (kMRows - 1))];
            bv[u][s] = Wf[kk * kMRows + ((tCol[s] + 16 * mk) & (kMRows - 1))];
          }
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const bool on = k0 + 4 * u + mk < nk;
#pragma unroll
          for (int s = 0; s < 3; ++s) {
            const bool o = on && s < ntl;
            acc[s] = __builtin_amdgcn_mfma_f64_16x16x4f64(o ? av[u][s] : 0.0, o ? bv[u][s] : 0.0,
                                                         acc[s], 0, 0, 0);
          }
        }
      }
    }
    //     Z_a += z^T z over camera a's observation rows, 2 observations per MFMA:
    //     lane (i = lane & 15, k = lane >> 4) supplies z[row k & 1 of obs k >> 1][i]
    //     as both operands (A[i][k] and B[k][i] take the same value).  The
    //     wave's two cameras (a = wid, wid + 4) advance together, 4 MFMAs each
    //     per step, operands loaded ahead; missing cameras / observations: zeros.
    {
      const int row = mk & 1;
      int qb[2], qe[2];
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        const int a = wid + 4 * s;
        qb[s] = s < nza ? L.cptr[a] : 0;
        qe[s] = s < nza ? L.cptr[a + 1] : 0;
      }
      const int nsteps = max(qe[0] - qb[0], qe[1] - qb[1]);
      for (int q = 0; q < nsteps; q += 8) {
        double z[2][4];
        bool ok[2][4];
#pragma unroll
        for (int s = 0; s < 2; ++s)
#pragma unroll
          for (int u = 0; u < 4; ++u) {
            const int qq = qb[s] + q + 2 * u + (mk >> 1);
            ok[s][u] = qq < qe[s];
            const int k = L.cobs[ok[s][u] ? qq : 0];
            const double* src = mi < 9 ? &L.jc[9 * row + mi][k]
                                : mi < 11 ? &L.ru[row + 2 * (mi - 9)][k] : &L.zero;
            z[s][u] = *src;
          }
#pragma unroll
        for (int u = 0; u < 4; ++u)
#pragma unroll
          for (int s = 0; s < 2; ++s) {
            const double zv = ok[s][u] ? z[s][u] : 0.0;
            zacc[s] = __builtin_amdgcn_mfma_f64_16x16x4f64(zv, zv, zacc[s], 0, 0, 0);
          }
      }
    }
    p0 = np0; p1 = np1; o0 = no0; o1 = no1;
    np0 = nnp0; np1 = nnp1; no0 = nno0; no1 = nno1;
    LINM_T(5);
  }
  // (E) T and the Z_a tiles -> LDS staging (aliases the operand planes), then
  //     the partial rows
  __syncthreads();
  double* T = &L.yt[0][0][0];
  double* Z = T + kMRows * kMRows;  // [kMCams][16][16]
#pragma unroll
  for (int s = 0; s < 3; ++s) {
    if (s >= ntl) break;
#pragma unroll
    for (int r = 0; r < 4; ++r)
      T[(16 * tI[s] + mk + 4 * r) * kMRows + 16 * tJ[s] + mi] = acc[s][r];
  }
#pragma unroll
  for (int s = 0; s < 2; ++s) {
    if (s >= nza) break;
#pragma unroll
    for (int r = 0; r < 4; ++r) Z[(wid + 4 * s) * 256 + (mk + 4 * r) * 16 + mi] = zacc[s][r];
  }
  __syncthreads();
  const bool fold = p.asm_tab != nullptr;  // uniform
  // camera rows: items (a, 112-wide row entry)
  for (int q = t; q < m * 109; q += kMWG) {
    const int a = q / 109, e = q - 109 * (q / 109);
    const double* Za = Z + a * 256;
    double v;
    if (e < 81) {
      const int i = e / 9, j = e - 9 * (e / 9);
      const int row = 9 * a + i, col = 9 * a + j;  // T is symmetric; upper tiles were formed
      const double tv = (row >> 4) <= (col >> 4) ? T[row * kMRows + col] : T[col * kMRows + row];
      v = Za[i * 16 + j] - tv;
    } else if (e < 90) {
      v = Za[(e - 81) * 16 + 9];   // Jc^T r
    } else if (e < 99) {
      v = Za[(e - 90) * 16 + 10];  // Jc^T u
    } else if (e < 108) {
      v = Za[(e - 99) * 17];       // diag U
    } else {
      v = Za[9 * 16 + 9];          // |r|^2
    }
    // written through (sc1) only for the folded assembly (other CUs read them in
    // this launch); plain stores keep the lines in L2 for k_assemble
    double* cp = p.cpart + (size_t)L.crow[a] * kCPart + e;
    if (fold) st_sc1(cp, v);
    else *cp = v;
  }
  for (int q = t; q < 81 * nb; q += kMWG) {
    const int pr = q / 81, e = q - 81 * (q / 81);
    const int ab = L.bab[pr], a = ab & 255, b = ab >> 8;
    const int i = e / 9, j = e - 9 * (e / 9);
    const double v = T[(9 * a + i) * kMRows + 9 * b + j];
    double* bp = p.bpart + (size_t)L.brow[pr] * 81 + e;
    if (fold) st_sc1(bp, v);
    else *bp = v;
  }
  LINM_T(6);
  if (p.asm_tab != nullptr) lin_fold_assemble(p, sm + 10, m, nb, L.brow, &L.jc[0][0]);
  LINM_END();
}

// Column sums of the n-wide rows [rb, re) of part (row stride `stride`): the
// workgroup's lanes are (part k, column e) pairs; part k takes rows rb + k,
// rb + k + nparts, ... with 8 loads in flight, then the parts are added in
// order k = 0, 1, ... (deterministic).  Result in out[0..n).
#ifndef SLAM_ASM_WG
#define SLAM_ASM_WG 1024  // k_assemble workgroup (>= 128: one lane per element of a 109-double row)
#endif
constexpr int kAsmWG = SLAM_ASM_WG;
static_assert(kAsmWG >= 128 && kAsmWG % 64 == 0, "SLAM_ASM_WG");
__device__ void rows_sum(const double* __restrict__ part, int stride, int rb, int re, int n,
                         double (*red)[kCPart], double* out) {
  const int t = threadIdx.x;
  const int nparts = kAsmWG / n, k = t / n, e = t - k * n;
  if (k < nparts) {
    double a[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    int r = rb + k;
    for (; r + 7 * nparts < re; r += 8 * nparts) {
      double v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) v[u] = part[(size_t)(r + u * nparts) * stride + e];
#pragma unroll
      for (int u = 0; u < 8; ++u) a[u] += v[u];
    }
    for (int u = 0; r < re; r += nparts, ++u) a[u] += part[(size_t)r * stride + e];
    red[k][e] = ((a[0] + a[1]) + (a[2] + a[3])) + ((a[4] + a[5]) + (a[6] + a[7]));
  }
  __syncthreads();
  if (t < n) {
    double v = 0.0;
    for (int q = 0; q < nparts; ++q) v += red[q][t];
    out[t] = v;
  }
  __syncthreads();
}

// One workgroup per upper camera-pair block (c1 <= c2), ALL C(C+1)/2 of them.
// The slot partials of a camera / block are contiguous rows (the planner's
// camera- / block-major row order), summed in group order (deterministic):
//   diagonal block c:  S = sum (U - Y W^T) over the camera rows of c, minus
//                      B + B^T for the block rows of (c, c) (a point observed
//                      twice by c); b = -Jc^T r - Jc^T u, g = -Jc^T r, diag U, cost;
//   block c1 < c2:     S = -sum Y W^T (and its transpose) over the block rows.
// Dense layout: blocks without common points are written as zeros, so sys
// needs no separate clearing.  Packed layout: each listed block is written
// once, full 9x9, at sys + 81 * blk.
__global__ __launch_bounds__(kAsmWG) void k_assemble(BaBatch bat) {
  BA_PROB_X(bat);
  if (bx >= (p.asm_act != nullptr ? p.n_asm_act : p.n_blocks)) return;
  lm_wave_priority();
  __shared__ double red[kAsmWG / 81][kCPart];
  __shared__ double sh[kCPart];
  __shared__ double sb[81];
  const int blk = p.asm_act != nullptr ? p.asm_act[bx] : bx;
  if (p.asm_act != nullptr) {
    // this workgroup's share of the zeros of the unlisted blocks and of the
    // vector entries of the cameras without rows (what the assembly writes for
    // them: S -0.0, b and g -0.0, diag U and cost +0.0), beside the listed
    // blocks that the workgroups write (disjoint addresses, no ordering needed)
    const int32_t* listed = p.asm_act + p.n_asm_act;  // [n_blocks] 0/1
    const int32_t* camrows = listed + p.n_blocks;      // [n_cams] 0/1
    const size_t ns = (size_t)p.n_blocks * 81, c9 = 9 * (size_t)p.n_cams, nv = ns + 3 * c9 + p.n_cams;
    for (size_t i = (size_t)bx * kAsmWG + threadIdx.x; i < nv; i += (size_t)p.n_asm_act * kAsmWG) {
      if (i < ns) {
        if (!listed[i / 81]) p.sys[i] = -0.0;
      } else {
        const size_t j = i - ns;
        const int cam = j < 3 * c9 ? (int)((j % c9) / 9) : (int)(j - 3 * c9);
        if (!camrows[cam]) p.sys[i] = j < 2 * c9 ? -0.0 : 0.0;
      }
    }
  }
  const int c1 = p.blocks[2 * blk], c2 = p.blocks[2 * blk + 1];
  const int C9 = 9 * p.n_cams;
  double* S = p.sys;
  double* bvec = S + sys_vec_off(p.n_cams, p.n_blocks);
  double* gvec = bvec + C9;
  double* diagU = gvec + C9;
  double* costc = diagU + C9;
  const int t = threadIdx.x;
  const bool diag = c1 == c2;
  const int bb = p.blk_bslot_ptr[blk], be = p.blk_bslot_ptr[blk + 1];
  if (!diag && be == bb) {
    // a block without partial rows (most listed blocks of a landmark shard:
    // the global block list, this rank's points): its zeros (-sum of nothing,
    // bit for bit what the sum path writes) without the row sums' barriers
    if (t < 81) {
      if (sys_packed(p.n_cams)) {
        S[(size_t)blk * 81 + t] = -0.0;
      } else {
        const int i = t / 9, j = t - 9 * (t / 9);
        S[(size_t)(9 * c1 + i) * C9 + 9 * c2 + j] = -0.0;
        S[(size_t)(9 * c2 + j) * C9 + 9 * c1 + i] = -0.0;
      }
    }
    return;
  }
  if (diag) rows_sum(p.cpart, kCPart, p.cam_cslot_ptr[c1], p.cam_cslot_ptr[c1 + 1], 109, red, sh);
  if (!diag || be > bb) {
    rows_sum(p.bpart, 81, bb, be, 81, red, sb);
  } else if (t < 81) {
    sb[t] = 0.0;
  }
  __syncthreads();
  if (sys_packed(p.n_cams)) {
    if (t < 81) S[(size_t)blk * 81 + t] = diag ? sh[t] - (sb[t] + sb[9 * (t % 9) + t / 9]) : -sb[t];
  } else if (t < 81) {
    const int i = t / 9, j = t - 9 * (t / 9);
    if (diag) {
      S[(size_t)(9 * c1 + i) * C9 + 9 * c1 + j] = sh[t] - (sb[t] + sb[9 * j + i]);
    } else {
      S[(size_t)(9 * c1 + i) * C9 + 9 * c2 + j] = -sb[t];
      S[(size_t)(9 * c2 + j) * C9 + 9 * c1 + i] = -sb[t];
    }
  }
  if (diag && t < 9) {
    gvec[9 * c1 + t] = -sh[81 + t];
    bvec[9 * c1 + t] = -sh[81 + t] - sh[90 + t];
    diagU[9 * c1 + t] = sh[99 + t];
  }
  if (diag && t == 0) costc[c1] = sh[108];
}

// ---------------------------------------------------------------- solve
// Reduced camera system S x = b, S SPD (damped).  Two solvers: k_solve_blk
// (one workgroup, whole system in LDS/registers) for the local-BA window
// (9C <= kLdsMaxN), and the tiled multi-workgroup Cholesky (k_tl3_flow, k_tl2_*) for
// larger systems.
constexpr int kLdsMaxN = kDenseMaxN;  // k_solve_blk keeps the system in LDS up to 9C = 120
constexpr int kSolveHdr = 32;   // doubles of LDS header in k_solve_blk

// Inputs of the epilogue: camera gradient, Gram diagonal, live cameras and the
// per-camera cost partials (global memory in the tiled solves, LDS copies prefetched at
// kernel start in k_solve_blk so their latency is off the critical path).
struct EpiSrc {
  const double *g, *dU, *cam, *costc;
};
#ifdef SLAM_FLOW_PROFILE
// the dataflow solve's epilogue: start, x staged, pc / cost reduced, cameras prepared
__device__ unsigned long long g_flow_epi[4];
#endif

// Shared epilogue: camera step, trial cameras, predicted reduction of the camera
// part, LM cost at the live parameters.  GLOBAL (the tiled solves, 9C up to
// 8192): the inputs are read from memory, so every thread issues its loads in
// groups of 8 before using them (the per-thread order of the pc sum is the
// same), and the per-camera cost is summed by all threads (strided, then the
// fixed tree of block_sum2) instead of by thread 0 alone -- at C5 the serial
// forms were ~18 dependent memory round trips per thread plus 500 dependent
// loads and adds.
__device__ __forceinline__ void block_sum2(double& a, double& b, double* lds) {
  // deterministic: fixed shuffle tree then fixed LDS order (lds: 2 x 16 doubles)
  for (int off = 32; off > 0; off >>= 1) {
    a += __shfl_down(a, off, 64);
    b += __shfl_down(b, off, 64);
  }
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  if (lane == 0) {
    lds[wid] = a;
    lds[16 + wid] = b;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    const int nw = (blockDim.x + 63) >> 6;
    a = 0.0;
    b = 0.0;
    for (int w = 0; w < nw; ++w) {
      a += lds[w];
      b += lds[16 + w];
    }
  }
  __syncthreads();
}

template <bool GLOBAL = false>
__device__ void solve_epilogue(const slam_ba_problem& p, const double* x, bool ok, double* red,
                               const EpiSrc& e, int fail_code = 1) {
  const int C9 = 9 * p.n_cams, t = threadIdx.x;
  double* state = p.state;
  const double lam = state[SLAM_BA_ST_LAMBDA];
  const int cur = cur_of(state);
  double pc = 0.0, cost = 0.0;
  if constexpr (GLOBAL) {
    const int nt = blockDim.x;
    for (int i0 = t; i0 < C9; i0 += 8 * nt) {
      double xv[8], cv[8], uv[8], gv[8];
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        const int i = min(i0 + q * nt, C9 - 1);
        xv[q] = x[i];
        cv[q] = e.cam[i];
        uv[q] = e.dU[i];
        gv[q] = e.g[i];
      }
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        const int i = i0 + q * nt;
        if (i < C9) {
          const double d = ok ? xv[q] : 0.0;
          p.delta_c[i] = d;
          p.cams[1 - cur][i] = cv[q] + d;
          pc += d * (lam * clampd(uv[q]) * d + gv[q]);
        }
      }
    }
    for (int c = t; c < p.n_cams; c += nt) cost += e.costc[c];
    block_sum2(pc, cost, red);  // (its barriers also publish the trial cameras to the WG)
#ifdef SLAM_FLOW_PROFILE
    if (t == 0) g_flow_epi[2] = wall_clock64();
#endif
  } else {
    for (int i = t; i < C9; i += blockDim.x) {
      const double d = ok ? x[i] : 0.0;
      p.delta_c[i] = d;
      p.cams[1 - cur][i] = e.cam[i] + d;
      pc += d * (lam * clampd(e.dU[i]) * d + e.g[i]);
    }
    pc = block_sum(pc, red);  // (its barriers also publish the trial cameras to the WG)
    if (t == 0)
      for (int c = 0; c < p.n_cams; ++c) cost += e.costc[c];
  }
  for (int c = t; c < p.n_cams; c += blockDim.x)
    cam_prep(p.cams[1 - cur] + 9 * c, p.camrec[1 - cur] + kCamRec * c);
#ifdef SLAM_FLOW_PROFILE
  if (GLOBAL) {
    __builtin_amdgcn_s_waitcnt(0);
    __syncthreads();
    if (t == 0) g_flow_epi[3] = wall_clock64();
  }
#endif
  if (t == 0) {
    state[SLAM_BA_ST_COST] = 0.5 * cost;
    state[SLAM_BA_ST_PRED_CAM] = 0.5 * pc;
    state[SLAM_BA_ST_CHOL_FAIL] = ok ? 0.0 : (double)fail_code;
    if (!ok && fail_code == 2) state[SLAM_BA_ST_SOLVE_FAULT] += 1.0;
  }
}

// -DSLAM_SOLVE_PROFILE: phase timestamps (wall_clock64, 100 MHz) of k_solve_blk
// into the spare LM state slots 12..15 (ns): load, eliminate, back-substitute, epilogue.
#ifdef SLAM_SOLVE_PROFILE
#define SOLVE_PROF_T(i) uint64_t prof_t##i = wall_clock64()
#define SOLVE_PROF_END()                                                        \
  do {                                                                          \
    const uint64_t prof_e = wall_clock64();                                     \
    if (threadIdx.x == 0) {                                                     \
      p.state[12] = 10.0 * (double)(prof_t1 - prof_t0);                         \
      p.state[13] = 10.0 * (double)(prof_t2 - prof_t1);                         \
      p.state[14] = 10.0 * (double)(prof_t3 - prof_t2);                         \
      p.state[15] = 10.0 * (double)(prof_e - prof_t3);                          \
    }                                                                           \
  } while (0)
#else
#define SOLVE_PROF_T(i) (void)0
#define SOLVE_PROF_END() (void)0
#endif

// Small systems (9C <= kLdsMaxN, the local-BA window): blocked LDL^T with the
// trailing updates on the f64 matrix cores.
//
// The augmented matrix [S ; b^T] ((n+1) x n, b carried as row n so the
// elimination also performs the forward substitution) is kept as 16x16 f64
// MFMA accumulator tiles, lower tiles only, spread round-robin over the 4
// waves (<= 36 tiles for n <= 120, <= 9 per wave).  One block step per camera
// (9 columns):
//   (a) the owners of the 9 panel columns copy them to LDS;        barrier
//   (b) wave 0 factors the panel in registers, two rows per lane, pivot rows
//       broadcast with v_readlane (no LDS round trips, no barriers); it writes
//       W = -A_panel and L = A_panel D^-1 for the rows below the panel (zeros
//       elsewhere) and the final factor columns;                    barrier
//   (c) every wave updates its live tiles: T -= W_I L_J^T, 3 MFMAs
//       (v_mfma_f64_16x16x4_f64, K = 9 padded to 12) per tile.
// 2 barriers per camera instead of one per column.  Back substitution runs in
// wave 0 with x in registers (two rows per lane) and x_k broadcast by readlane.
constexpr int kBlkWG = 256;   // 4 waves, one per SIMD; <= 256 registers per lane (2 waves per SIMD)
constexpr int kBlkWaves = kBlkWG / 64;
constexpr int kTileMax = 9;   // lower 16x16 tiles per wave: 4 * 9 >= 36
constexpr int kPanelW = 9;    // columns per block step (one camera)
constexpr int kWLs = 13;      // W/L row stride: K = 9 padded to 3 MFMA steps of 4 (odd: no LDS bank conflicts)
static_assert(kLdsMaxN <= kBlkWG, "k_solve_blk prefetch assumes one element per thread");
static_assert(kBlkWaves * kTileMax >= ((kLdsMaxN + 16) / 16) * ((kLdsMaxN + 16) / 16 + 1) / 2,
              "kTileMax too small");

// 1/d from v_rcp_f64 refined by two Newton steps (full double precision, off
// the v_div_* sequence's long dependent chain)
__device__ __forceinline__ double rcp_f64(double d) {
  double r = __builtin_amdgcn_rcp(d);
  double e = __builtin_fma(-d, r, 1.0);
  r = __builtin_fma(r, e, r);
  e = __builtin_fma(-d, r, 1.0);
  return __builtin_fma(r, e, r);
}

__device__ __forceinline__ double readlane_d(double v, int lane) {
  const unsigned long long u = (unsigned long long)__double_as_longlong(v);
  const unsigned lo = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)u, lane);
  const unsigned hi = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)(u >> 32), lane);
  return __longlong_as_double((long long)(((unsigned long long)hi << 32) | lo));
}

// LDS layout of k_solve_blk (doubles, after the kSolveHdr header)
struct BlkLds {
  int n16;        // rows rounded up to a tile multiple (>= n + 1)
  int pn, wl, ll, lf, dd, yy, xx, ep, total;
  __host__ __device__ explicit BlkLds(int n) {
    n16 = ((n + 1 + 15) / 16) * 16;
    pn = kSolveHdr;                       // [n16][kPanelW] panel copy
    wl = pn + n16 * kPanelW;              // [n16][kWLs] W = -A_panel (rows below the panel)
    ll = wl + n16 * kWLs;                 // [n16][kWLs] L = A_panel D^-1
    lf = ll + n16 * kWLs;                 // [n(n-1)/2] factor L, packed by rows
    dd = lf + ((n * (n - 1) / 2 + 1) & ~1);  // [n] D
    yy = dd + ((n + 1) & ~1);             // [n] y = L^-1 b
    xx = yy + ((n + 1) & ~1);             // [n] solution
    ep = xx + ((n + 1) & ~1);             // [5][n] b, g, diagU, live cameras, cost partials
    total = ep + 5 * ((n + 1) & ~1);
  }
};

#ifdef SLAM_SOLVE_TRACE
__device__ unsigned long long g_solve_trace[20][6];
#define SOLVE_TR(step, i)                                                        \
  do {                                                                           \
    if (threadIdx.x == 0 && blockIdx.y == 0 && (step) < 20)                      \
      g_solve_trace[step][i] = __builtin_amdgcn_s_memtime();                     \
  } while (0)
#else
#define SOLVE_TR(step, i) (void)0
#endif

// k_solve_blk's panel pivots, the same fused form (9-wide panels):
// u[i] += bcast_i(uj) * nl for i = J+2..8 (column J's updates after the next
// pivot's entry, which stays in compiler code)
template <int J> struct PanelRest;
static_assert(kPanelW == 9, "PanelRest is written for 9-wide panels");
template <> struct PanelRest<0> {
  static __device__ __forceinline__ void run(double (&u)[9], double uj, double nl) {
    asm("s_nop 1\n" "v_fmac_f64_dpp %0, %7, %8 row_newbcast:2 row_mask:0xf bank_mask:0xf\n" "v_fmac_f64_dpp %1, %7, %8 row_newbcast:3 row_mask:0xf bank_mask:0xf\n" "v_fmac_f64_dpp %2, %7, %8 row_newbcast:4 row_mask:0xf bank_mask:0xf\n" "v_fmac_f64_dpp %3, %7, %8 row_newbcast:5 row_mask:0xf bank_mask:0xf\n" "v_fmac_f64_dpp %4, %7, %8 row_newbcast:6 row_mask:0xf bank_mask:0xf\n" "v_fmac_f64_dpp %5, %7, %8 row_newbcast:7 row_mask:0xf bank_mask:0xf\n" "v_fmac_f64_dpp %6, %7, %8 row_newbcast:8 row_mask:0xf bank_mask:0xf\n"
        : "+v"(u[2]), "+v"(u[3]), "+v"(u[4]), "+v"(u[5]), "+v"(u[6]), "+v"(u[7]), "+v"(u[8])
        : "v"(uj), "v"(nl));
  }
};
template <> struct PanelRest<1> {
  static __device__ __forceinline__ void run(double (&u)[9], double uj, double nl) {
    asm("s_nop 1\n" "v_fmac_f64_dpp %0, %6, %7 row_newbcast:3 row_mask:0xf bank_mask:0xf\n" "v_fmac_f64_dpp %1, %6, %7 row_newbcast:4 row_mask:0xf bank_mask:0xf\n" "v_fmac_f64_dpp %2, %6, %7 row_newbcast:5 row_mask:0xf bank_mask:0xf\n" "v_fmac_f64_dpp %3, %6, %7 row_newbcast:6 row_mask:0xf bank_mask:0xf\n" "v_fmac_f64_dpp %4, %6, %7 row_newbcast:7 row_mask:0xf bank_mask:0xf\n" "v_fmac_f64_dpp %5, %6, %7 row_newbcast:8 row_mask:0xf bank_mask:0xf\n"
        : "+v"(u[3]), "+v"(u[4]), "+v"(u[5]), "+v"(u[6]), "+v"(u[7]), "+v"(u[8])
        : "v"(uj), "v"(nl));
  }
};
template <> struct PanelRest<2> {
  static __device__ __forceinline__ void run(double (&u)[9], double uj, double nl) {
    asm("s_nop 1\n" "v_fmac_f64_dpp %0, %5, %6 row_newbcast:4 row_mask:0xf bank_mask:0xf\n" "v_fmac_f64_dpp %1, %5, %6 row_newbcast:5 row_mask:0xf bank_mask:0xf\n" "v_fmac_f64_dpp %2, %5, %6 row_newbcast:6 row_mask:0xf bank_mask:0xf\n" "v_fmac_f64_dpp %3, %5, %6 row_newbcast:7 row_mask:0xf bank_mask:0xf\n" "v_fmac_f64_dpp %4, %5, %6 row_newbcast:8 row_mask:0xf bank_mask:0xf\n"
        : "+v"(u[4]), "+v"(u[5]), "+v"(u[6]), "+v"(u[7]), "+v"(u[8])
        : "v"(uj), "v"(nl));
  }
};
template <> struct PanelRest<3> {
  static __device__ __forceinline__ void run(double (&u)[9], double uj, double nl) {
    asm("s_nop 1\n" "v_fmac_f64_dpp %0, %4, %5 row_newbcast:5 row_mask:0xf bank_mask:0xf\n" "v_fmac_f64_dpp %1, %4, %5 row_newbcast:6 row_mask:0xf bank_mask:0xf\n" "v_fmac_f64_dpp %2, %4, %5 row_newbcast:7 row_mask:0xf bank_mask:0xf\n" "v_fmac_f64_dpp %3, %4, %5 row_newbcast:8 row_mask:0xf bank_mask:0xf\n"
        : "+v"(u[5]), "+v"(u[6]), "+v"(u[7]), "+v"(u[8])
        : "v"(uj), "v"(nl));
  }
};
template <> struct PanelRest<4> {
  static __device__ __forceinline__ void run(double (&u)[9], double uj, double nl) {
    asm("s_nop 1\n" "v_fmac_f64_dpp %0, %3, %4 row_newbcast:6 row_mask:0xf bank_mask:0xf\n" "v_fmac_f64_dpp %1, %3, %4 row_newbcast:7 row_mask:0xf bank_mask:0xf\n" "v_fmac_f64_dpp %2, %3, %4 row_newbcast:8 row_mask:0xf bank_mask:0xf\n"
        : "+v"(u[6]), "+v"(u[7]), "+v"(u[8])
        : "v"(uj), "v"(nl));
  }
};
template <> struct PanelRest<5> {
  static __device__ __forceinline__ void run(double (&u)[9], double uj, double nl) {
    asm("s_nop 1\n" "v_fmac_f64_dpp %0, %2, %3 row_newbcast:7 row_mask:0xf bank_mask:0xf\n" "v_fmac_f64_dpp %1, %2, %3 row_newbcast:8 row_mask:0xf bank_mask:0xf\n"
        : "+v"(u[7]), "+v"(u[8])
        : "v"(uj), "v"(nl));
  }
};
template <> struct PanelRest<6> {
  static __device__ __forceinline__ void run(double (&u)[9], double uj, double nl) {
    asm("s_nop 1\n" "v_fmac_f64_dpp %0, %1, %2 row_newbcast:8 row_mask:0xf bank_mask:0xf\n"
        : "+v"(u[8])
        : "v"(uj), "v"(nl));
  }
};
template <> struct PanelRest<7> {
  static __device__ __forceinline__ void run(double (&u)[9], double uj, double nl) {
    (void)u; (void)uj; (void)nl;
  }
};
template <> struct PanelRest<8> {
  static __device__ __forceinline__ void run(double (&u)[9], double uj, double nl) {
    (void)u; (void)uj; (void)nl;
  }
};

__global__ __launch_bounds__(kBlkWG) __attribute__((amdgpu_waves_per_eu(2))) void k_solve_blk(BaBatch bat) {
  BA_PROB(bat);
  lm_wave_priority();
  extern __shared__ __attribute__((aligned(16))) double lds[];
  double* red = lds;
  int* fail_p = reinterpret_cast<int*>(lds + 16);
  const int n = 9 * p.n_cams;
  const BlkLds g(n);
  double* Pn = lds + g.pn;
  double* WL = lds + g.wl;
  double* LL = lds + g.ll;
  double* LF = lds + g.lf;
  double* Dd = lds + g.dd;
  double* Yy = lds + g.yy;
  double* X = lds + g.xx;
  const double* S = p.sys;
  const double* bvec = S + (size_t)n * n;
  const double* diagU = bvec + 2 * n;
  const double lam = p.state[SLAM_BA_ST_LAMBDA];
  const int t = threadIdx.x, lane = t & 63;
  const int wid = __builtin_amdgcn_readfirstlane(t >> 6);
  const int NT = g.n16 / 16, NL = NT * (NT + 1) / 2;
  SOLVE_PROF_T(0);
  SOLVE_TR(19, 1);
  const int n2 = (n + 1) & ~1;
  if (t == 0) *fail_p = 0;
  for (int i = t; i < 2 * g.n16 * kWLs; i += kBlkWG) WL[i] = 0.0;  // WL and LL
  // this wave's tiles: tl = wid + 4 s -> (I, J), I >= J.  All S loads are
  // issued unconditionally (clamped addresses) before any is used.
  int tI[kTileMax], tJ[kTileMax];
  d4 acc[kTileMax];
#pragma unroll
  for (int s = 0; s < kTileMax; ++s) {
    const int tl = wid + kBlkWaves * s;
    int I = 0;
    while ((I + 1) * (I + 2) / 2 <= tl) ++I;
    tI[s] = tl < NL ? I : -1;
    tJ[s] = tl < NL ? tl - I * (I + 1) / 2 : -1;
    const int col = min(max(tJ[s], 0) * 16 + (lane & 15), n - 1);
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int row = min(max(tI[s], 0) * 16 + (lane >> 4) + 4 * q, n - 1);
      acc[s][q] = S[(size_t)row * n + col];
    }
  }
  double* Eb = lds + g.ep;  // prefetch: b, g, diagU, live cameras, cost partials
  {
    const double* src[5] = {bvec, bvec + n, diagU, p.cams[cur_of(p.state)], diagU + n};
    const int len[5] = {n, n, n, n, p.n_cams};
    double v[5];  // n <= kLdsMaxN < kBlkWG: one element per thread, loads issued together
#pragma unroll
    for (int a = 0; a < 5; ++a) v[a] = src[a][min(t, len[a] - 1)];
#pragma unroll
    for (int a = 0; a < 5; ++a)
      if (t < len[a]) Eb[a * n2 + t] = v[a];
  }
  __syncthreads();  // prefetched b and diagU
#pragma unroll
  for (int s = 0; s < kTileMax; ++s) {
    const int col = tJ[s] * 16 + (lane & 15);
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int row = tI[s] * 16 + (lane >> 4) + 4 * q;
      double a = acc[s][q];
      if (row == col) a += lam * clampd(Eb[2 * n2 + col]);
      if (row == n) a = Eb[min(col, n - 1)];
      if (tI[s] < 0 || col >= n || row > n) a = 0.0;
      acc[s][q] = a;
    }
  }
  SOLVE_PROF_T(1);
  bool ok = true;
  SOLVE_TR(19, 0);
  for (int c0 = 0; c0 < n; c0 += kPanelW) {
    SOLVE_TR(c0 / kPanelW, 0);
#ifdef SLAM_SOLVE_PROFILE_STEP
    const uint64_t q0 = __builtin_amdgcn_s_memtime();
#endif
    // (a) panel columns [c0, c0 + 9), rows c0..n -> Pn[row - c0][col - c0]
#pragma unroll
    for (int s = 0; s < kTileMax; ++s) {
      if (tI[s] < 0 || tJ[s] * 16 + 15 < c0 || tJ[s] * 16 >= c0 + kPanelW || tI[s] * 16 + 15 < c0)
        continue;  // uniform per wave
      const int col = tJ[s] * 16 + (lane & 15);
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int row = tI[s] * 16 + (lane >> 4) + 4 * q;
        if (col >= c0 && col < c0 + kPanelW && col <= row && row >= c0 && row <= n)
          Pn[(row - c0) * kPanelW + (col - c0)] = acc[s][q];
      }
    }
    __syncthreads();
    SOLVE_TR(c0 / kPanelW, 1);
#ifdef SLAM_SOLVE_PROFILE_STEP
    const uint64_t q1 = __builtin_amdgcn_s_memtime();
#endif
    // (b) panel factorisation, one panel row per lane: lanes 0..8 of every
    // participating wave hold the 9 pivot rows r = c0 + m (lower entries),
    // lanes 9..63 of wave w the rows c0 + 9 + 55 w + (lane - 9) (the rhs row n
    // included).  Right-looking: at step j the pivot d_j and the column-j
    // entries of the pivot rows are broadcast with v_readlane, and every lane
    // eliminates its own row (u_i -= (u_j / d_j) A(c0+i, c0+j)).  Afterwards
    // u_j is the partially eliminated entry A^{(j)}(r, c0+j), L(r, j) = u_j/d_j.
    // (Was: every lane factored the whole 9x9 block redundantly, ~3x the
    // VALU work of this form.)
    // Every 16-lane DPP row of a participating wave holds a copy of the 9 pivot
    // rows (lanes 0..8 of the row) and 7 rows below the panel (lanes 9..15), so
    // the pivot entries reach the other lanes as DPP row_newbcast operands
    // (no v_readlane -> SGPR hop in the pivot chain).  28 rows below per wave:
    // 4 waves cover 9C + 1 - 9 <= 112 rows.
    constexpr int kRowsBelow = 16 - kPanelW;              // per DPP row
    const int nbelow = n + 1 - c0 - kPanelW;             // rows below the panel, rhs included
    const int nw = max(1, (nbelow + 4 * kRowsBelow - 1) / (4 * kRowsBelow));  // uniform
    if (wid < nw) {
      const int rl = lane & 15, rg = lane >> 4;
      const bool piv = rl < kPanelW;
      const int r = piv ? c0 + rl
                        : c0 + kPanelW + 4 * kRowsBelow * wid + kRowsBelow * rg + (rl - kPanelW);
      const bool valid = r <= n;
      const double* pr = Pn + (r - c0) * kPanelW;
      double u[kPanelW];
#pragma unroll
      for (int j = 0; j < kPanelW; ++j) u[j] = valid && (!piv || j <= rl) ? pr[j] : 0.0;
      double Dinv[kPanelW];
      bool bad = false;
#ifdef SLAM_SOLVE_PROFILE_PANEL
      __builtin_amdgcn_s_waitcnt(0);
      const uint64_t qb1 = __builtin_amdgcn_s_memtime();
#endif
      static_for<0, kPanelW>([&](auto J) {
        constexpr int j = decltype(J)::value;
        const double d = bcast16<j>(u[j]);
        bad |= !(d > 0.0) || !isfinite(d);
        Dinv[j] = rcp_f64(d);
        const double l = u[j] * Dinv[j];
        if constexpr (j + 1 < kPanelW) u[j + 1] = __builtin_fma(-l, bcast16<j + 1>(u[j]), u[j + 1]);
        PanelRest<j>::run(u, u[j], -l);
      });
#ifdef SLAM_SOLVE_PROFILE_PANEL
      {
        double chk = u[kPanelW - 1];
        __asm__ volatile("" : "+v"(chk));
        u[kPanelW - 1] = chk;
      }
      const uint64_t qb2 = __builtin_amdgcn_s_memtime();
      if (t == 0 && c0 == 9 * (n / 18)) {
        p.state[SLAM_BA_ST_SLOTS - 2] = (double)(qb1 - q1);  // replaces barrier / (c)
        p.state[SLAM_BA_ST_SLOTS - 1] = (double)(qb2 - qb1);
      }
#endif
      // stores grouped so that each lane class takes one exec-mask region
      if (valid && ((wid == 0 && rg == 0) || !piv)) {
        double* wl = WL + r * kWLs;
        double* ll = LL + r * kWLs;
        double* lf = LF + r * (r - 1) / 2 + c0;
        double lj[kPanelW];
#pragma unroll
        for (int j = 0; j < kPanelW; ++j) {
          lj[j] = u[j] * Dinv[j];
          wl[j] = -u[j];
          ll[j] = lj[j];
        }
        if (r == n) {
#pragma unroll
          for (int j = 0; j < kPanelW; ++j) Yy[c0 + j] = u[j];
        } else if (!piv) {
#pragma unroll
          for (int j = 0; j < kPanelW; ++j) lf[j] = lj[j];
        } else {
          // pivot row m = lane: D_m and the lower part L(r, c0 + j), j < m
          double dm = u[0];
#pragma unroll
          for (int j = 1; j < kPanelW; ++j) dm = j == rl ? u[j] : dm;
          Dd[r] = dm;
#pragma unroll
          for (int j = 0; j < kPanelW - 1; ++j)
            if (j < rl) lf[j] = lj[j];
        }
      }
      if (wid == 0 && lane == 0 && bad) *fail_p = 1;
    }
#ifdef SLAM_SOLVE_PROFILE_STEP
    const uint64_t q2 = __builtin_amdgcn_s_memtime();
#endif
    SOLVE_TR(c0 / kPanelW, 2);
    __syncthreads();
    SOLVE_TR(c0 / kPanelW, 3);
#ifdef SLAM_SOLVE_PROFILE_STEP
    const uint64_t q3 = __builtin_amdgcn_s_memtime();
#endif
    if (*fail_p) {
      ok = false;
      break;
    }
    // (c) trailing update of the tiles right of / below the panel, tile by
    // tile (6 operand loads, then its 3 MFMAs; each tile's sum in the same kk
    // order).  Loading every live tile's operands first held ~100 more
    // registers (317 per lane: one wave per SIMD, so a solve workgroup waited
    // for a whole idle CU beside ORB); at 210 (two waves per SIMD) the batched
    // local-BA stage in the tracking bench drops 3.1 -> 2.75 ms per step
    // (profiles/r4/solve_lowreg_ab/ at git f26058c)
    const int tr = c0 + kPanelW;
#pragma unroll
    for (int s = 0; s < kTileMax; ++s) {
      if (!(tI[s] >= 0 && tJ[s] * 16 + 15 >= tr)) continue;  // uniform (I >= J)
      const double* wrow = WL + (tI[s] * 16 + (lane & 15)) * kWLs + (lane >> 4);
      const double* lrow = LL + (tJ[s] * 16 + (lane & 15)) * kWLs + (lane >> 4);
      double wa[3], lb[3];
#pragma unroll
      for (int kk = 0; kk < 3; ++kk) {
        wa[kk] = wrow[4 * kk];
        lb[kk] = lrow[4 * kk];
      }
#pragma unroll
      for (int kk = 0; kk < 3; ++kk)
        acc[s] = __builtin_amdgcn_mfma_f64_16x16x4f64(wa[kk], lb[kk], acc[s], 0, 0, 0);
    }
#ifdef SLAM_SOLVE_TRACE
    if (threadIdx.x == 0) {
      double chk = acc[0][0];
      __asm__ volatile("" : "+v"(chk));
      acc[0][0] = chk;
    }
    SOLVE_TR(c0 / kPanelW, 4);
#endif
#ifdef SLAM_SOLVE_PROFILE_STEP
    __builtin_amdgcn_s_waitcnt(0);
    const uint64_t q4 = __builtin_amdgcn_s_memtime();
    if (t == 0 && c0 == 9 * (n / 18)) {
      p.state[12] = (double)(q1 - q0);
      p.state[13] = (double)(q2 - q1);
#ifndef SLAM_SOLVE_PROFILE_PANEL
      p.state[14] = (double)(q3 - q2);
      p.state[15] = (double)(q4 - q3);
#endif
    }
#endif
  }
  SOLVE_PROF_T(2);
  SOLVE_TR(18, 0);
  if (ok && wid == 0) {
    // z = D^-1 y, then L^T x = z from the bottom; lane l holds rows l, l + 64.
    // Step k: x_i -= L(k, i) x_k for i < k, x_k broadcast by v_readlane.  Rows
    // k >= 64 update every x0 (i = lane < 64 <= k, no mask) and the x1 rows
    // below k; rows k < 64 update x0 only.  The L rows of kBackU steps are
    // loaded (clamped, then masked by a select) ahead of the dependent chain.
    double x0 = lane < n ? Yy[lane] / Dd[lane] : 0.0;
    double x1 = lane + 64 < n ? Yy[lane + 64] / Dd[lane + 64] : 0.0;
    constexpr int kBackU = 8;
    int k = n - 1;
    for (; k - kBackU + 1 >= 64; k -= kBackU) {
      double l0[kBackU], l1[kBackU];
#pragma unroll
      for (int u = 0; u < kBackU; ++u) {
        const int kk = k - u;
        const double* Lk = LF + kk * (kk - 1) / 2;
        l0[u] = Lk[lane];
        const double v = Lk[min(lane + 64, kk - 1)];
        l1[u] = lane + 64 < kk ? v : 0.0;
      }
#pragma unroll
      for (int u = 0; u < kBackU; ++u) {
        const double xk = readlane_d(x1, k - u - 64);
        x0 = __builtin_fma(-l0[u], xk, x0);
        x1 = __builtin_fma(-l1[u], xk, x1);
      }
    }
    for (; k >= 64; --k) {
      const double* Lk = LF + k * (k - 1) / 2;
      const double v = Lk[min(lane + 64, k - 1)];
      const double xk = readlane_d(x1, k - 64);
      x0 = __builtin_fma(-Lk[lane], xk, x0);
      x1 = __builtin_fma(-(lane + 64 < k ? v : 0.0), xk, x1);
    }
    for (; k - kBackU + 1 >= 1; k -= kBackU) {
      double l0[kBackU];
#pragma unroll
      for (int u = 0; u < kBackU; ++u) {
        const int kk = k - u;
        const double v = LF[kk * (kk - 1) / 2 + min(lane, kk - 1)];
        l0[u] = lane < kk ? v : 0.0;
      }
#pragma unroll
      for (int u = 0; u < kBackU; ++u) x0 = __builtin_fma(-l0[u], readlane_d(x0, k - u), x0);
    }
    for (; k >= 1; --k) {
      const double v = LF[k * (k - 1) / 2 + min(lane, k - 1)];
      x0 = __builtin_fma(-(lane < k ? v : 0.0), readlane_d(x0, k), x0);
    }
    if (lane < n) X[lane] = x0;
    if (lane + 64 < n) X[lane + 64] = x1;
  }
  __syncthreads();
  SOLVE_PROF_T(3);
  SOLVE_TR(18, 1);
  solve_epilogue(p, X, ok, red, EpiSrc{Eb + n2, Eb + 2 * n2, Eb + 3 * n2, Eb + 4 * n2});
  SOLVE_PROF_END();
  SOLVE_TR(18, 2);
}

// ---------------------------------------------------------------- tiled solve
// Large reduced camera systems (9C > kLdsMaxN: the sharded C4 window, global
// BA): blocked Cholesky LL^T over 64x64 f64 tiles in the nested-dissection
// tile order of ba.tl_schedule (symbolic structure on the host), two forms:
//   k_tl3_flow    one launch, one persistent workgroup per tile column; device
//                 flags replace launch boundaries (the default);
//   k_tl2_*       the same tile operations level by level as separate launches
//                 (when the columns cannot all be resident: more tiles than
//                 the stream's CUs, or tl_mode "levels").
// Both start from k_tl2_load / k_tl2_scatter (damped S -> lower tiles, b) and
// end in solve_epilogue.  The diagonal-tile factor + inverse is
// tile_chol_inv_blk (16x16 diagonal blocks in wave 0's registers, the rest on
// the f64 matrix cores).
#ifndef SLAM_TL_KSKIP
#define SLAM_TL_KSKIP 0    // 1: the flow kernel's products skip a tile's padding k-blocks
#endif
#ifndef SLAM_TL_PADSKIP
#define SLAM_TL_PADSKIP 1  // the tile factor skips the pivot chain of padding blocks
#endif
constexpr int kTB = 64;        // tile edge
constexpr int kTlHdr = 12;     // ints of the tile schedule's header
constexpr int kEpiCams = 16;   // cameras per tile in k_tl3_flow's spread epilogue (ba.EPI_CAMS_MAX)
constexpr int kTlWG = 256;     // 4 waves: wave w owns rows 16w..16w+15 of a tile

struct TlLayout {  // doubles inside p.chol; T = the schedule's tile count (ba.tl_schedule)
  int T, N;
  long long a, dinv, b, y, x, nz, fail, xo, fc, epi, flow, total;
  __host__ __device__ TlLayout(int n, int n_tiles) {
    T = n_tiles;
    N = T * kTB;
    a = 0;
    dinv = a + (long long)N * N;         // T tiles L_kk^-1 (row-major 64x64 each)
    b = dinv + (long long)N * kTB;
    y = b + N;
    x = y + N;
    nz = x + N;                          // T*T bytes
    fail = nz + ((long long)T * T + 7) / 8;
    xo = fail + 8;                       // fail flag + 7 profiling slots (SLAM_TL_PROFILE)
    fc = xo + N;                         // k_tl3_flow: x in camera order; [T][T][64] L_Ik y_k
    epi = fc + (long long)T * T * kTB;   // (forward-substitution terms); [T][2] epilogue partials
    flow = epi + 2 * T;                  // (pc, cost per tile), then ints: flags
    // tile[T][T], y[T], x[T]; ticket, epoch, start ticket (+5 spare); retired row
    // tiles + waiter mark cnt[T]; L_JJ^-1 / y_J published dv[T]
    total = flow + ((long long)T * T + 4 * T + 8 + 1) / 2;
    // then k_tl3_flow's product slots (tl_sched[11] of them, slam_ba_chol_len):
    // [slots][64][64] terms L_Ik L_Jk^T, then one epoch flag (int) per slot
  }
  __host__ __device__ long long prod(int slot) const { return total + (long long)slot * kTB * kTB; }
  __host__ __device__ long long with_slots(int n_slots) const {
    return prod(n_slots) + ((long long)n_slots + 1) / 2;
  }
};

// fragment-ordered LDS image of a 64x64 tile: the MFMA operand of sub-tile s,
// k-step kk is 64 consecutive doubles (lane l: row 16s + (l & 15), col 4kk + (l >> 4))
__device__ __forceinline__ int frag_idx(int r, int c) {
  return ((((r >> 4) << 4) + (c >> 2)) << 6) + (r & 15) + ((c & 3) << 4);
}

__device__ __forceinline__ void tile_to_frag(const double* __restrict__ g, int ld, double* f,
                                             int w = threadIdx.x >> 6, int nw = kTlWG / 64) {
  // wave w of nw writes fragments (s, kk) = w, w + nw, ...: 64 consecutive doubles
  // per fragment (conflict-free LDS stores); the global reads are 16 rows x 32 B
  const int lane = threadIdx.x & 63;
  const int r = lane & 15, c = lane >> 4;
  // 16 loads in flight per lane before their LDS stores
  for (int f0 = w; f0 < 64; f0 += 16 * nw) {
    double tmp[16];
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      const int fi = f0 + q * nw;
      tmp[q] = fi < 64 ? g[(size_t)(16 * (fi >> 4) + r) * ld + 4 * (fi & 15) + c] : 0.0;
    }
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      const int fi = f0 + q * nw;
      if (fi < 64) f[(fi << 6) + lane] = tmp[q];
    }
  }
}

// acc[s] (wave w) = rows 16w.., cols 16s.. of X Y^T with Y LOWER triangular
// (L_kk^-1): column block s takes only the k-steps kk <= 4s + 3 (Y's entries
// past them are exact zeros), 40 of the 64 MFMAs -- the same sums.
__device__ __forceinline__ void gemm_xyT_lowY(const double* Xf, const double* Yf, d4 acc[4]) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
#pragma unroll
  for (int s = 0; s < 4; ++s) acc[s] = d4{0.0, 0.0, 0.0, 0.0};
  static_for<0, 16>([&](auto K) {
    constexpr int kk = decltype(K)::value;
    const double a = Xf[((w * 16 + kk) << 6) + lane];
    static_for<kk / 4, 4>([&](auto S) {
      constexpr int s = decltype(S)::value;
      acc[s] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, Yf[((s * 16 + kk) << 6) + lane], acc[s], 0, 0, 0);
    });
  });
}

// Fragment order with the offset inside each 64-double fragment F rotated by
// (4 * (c & 3) + (F & 3)) mod 16 within its 16-row quarter: the MFMA result
// layout (lanes along a row) then stores without LDS bank conflicts (16-way in
// plain fragment order: a 16-lane group's doubles all sit 32 dwords apart),
// and a fragment still reads back conflict-free (a permutation of each quarter).
__device__ __forceinline__ int frag_swz(int r, int c) {
  const int F = ((r >> 4) << 4) + (c >> 2), hi = c & 3;
  return (F << 6) + (hi << 4) + (((r & 15) + 4 * hi + (F & 3)) & 15);
}
// gemm_xyT_lowY with both operands in frag_swz order (same products, same order);
// only the k-steps kk < kmax (Y's columns past a tile's camera rows are padding:
// X's entries there are exact zeros)
__device__ __forceinline__ void gemm_xyT_lowY_swz(const double* Xf, const double* Yf, d4 acc[4],
                                                  int kmax = 16) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  int so[4];
#pragma unroll
  for (int k3 = 0; k3 < 4; ++k3) so[k3] = ((lane >> 4) << 4) + (((lane & 15) + 4 * (lane >> 4) + k3) & 15);
#pragma unroll
  for (int s = 0; s < 4; ++s) acc[s] = d4{0.0, 0.0, 0.0, 0.0};
  static_for<0, 16>([&](auto K) {
    constexpr int kk = decltype(K)::value;
    if (SLAM_TL_KSKIP && kk >= kmax) return;  // (uniform)
    const double a = Xf[((w * 16 + kk) << 6) + so[kk & 3]];
    static_for<kk / 4, 4>([&](auto S) {
      constexpr int s = decltype(S)::value;
      acc[s] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, Yf[((s * 16 + kk) << 6) + so[kk & 3]], acc[s], 0, 0, 0);
    });
  });
}

__device__ __forceinline__ bool tl_failed(const slam_ba_problem& p, const TlLayout& L) {
  return *reinterpret_cast<const volatile int*>(p.chol + L.fail) != 0;
}

// Blocked factor + inverse of the 64x64 diagonal tile (4 x 4 blocks of 16):
// per block column p, wave 0 factors the 16x16 diagonal block in registers
// (lane i = row i, pivots and column entries broadcast by DPP row_newbcast)
// and inverts it (lane c = column c of L_pp^-1); the panel L_ip = A_ip L_pp^-T
// and the trailing update A_ij -= L_ip L_jp^T run on the f64 matrix cores
// (16x16x4), one block per wave, for p = 0, 1 (workgroup barriers between);
// block columns 2 and 3 (L_32, A_33 and both factors) are wave 0's chain
// alone.  L^-1's off-diagonal blocks X_ip = -X_ii sum_{k=p}^{i-1} L_ik X_kp
// are formed by waves 1-3 beside that chain as their inputs appear (round 5:
// X_10 during block 2's factor, X_21 / X_20 and the sums T_3p during block
// 3's, the last three products X_3p = -X_33 T_3p once X_33 is out), so after
// the last pivot only one 16x16 product per wave is left (the assembly after
// the factor was 2.2 us of 13.0 per tile; 0.44 now).  M: LDS [64][65] (A, then
// L's off-diagonal blocks), Xb: LDS [10][16][17] (lower blocks of L^-1), Tb:
// LDS [3][16][17] scratch + six int flags (the wave-to-wave hand-offs of
// L_10 .. L_32, right after the scratch).  Every wave must call
// it; returns false (uniform) on a non-positive or non-finite pivot.
constexpr int kMS = 65;   // row stride of M (odd: MFMA operand reads spread over banks)
constexpr int kVR = 65;   // row stride of k_tl3_flow's row-major L_JJ^-1
constexpr int kBS17 = 17; // row stride of a 16x16 block
__device__ __forceinline__ int blk_id(int i, int j) { return i * (i + 1) / 2 + j; }

// C (+)= X Y^T (16x16 blocks, strides sx / sy); a_neg negates the product
__device__ __forceinline__ d4 mm16_xyT(const double* X, int sx, const double* Y, int sy, d4 acc,
                                       bool a_neg) {
  const int l = threadIdx.x & 63;
#pragma unroll
  for (int kk = 0; kk < 4; ++kk) {
    const double a = X[(l & 15) * sx + 4 * kk + (l >> 4)];
    const double b = Y[(l & 15) * sy + 4 * kk + (l >> 4)];
    acc = __builtin_amdgcn_mfma_f64_16x16x4f64(a_neg ? -a : a, b, acc, 0, 0, 0);
  }
  return acc;
}
// C (+)= X Y (16x16 blocks)
__device__ __forceinline__ d4 mm16_xy(const double* X, int sx, const double* Y, int sy, d4 acc,
                                      bool a_neg) {
  const int l = threadIdx.x & 63;
#pragma unroll
  for (int kk = 0; kk < 4; ++kk) {
    const double a = X[(l & 15) * sx + 4 * kk + (l >> 4)];
    const double b = Y[(4 * kk + (l >> 4)) * sy + (l & 15)];
    acc = __builtin_amdgcn_mfma_f64_16x16x4f64(a_neg ? -a : a, b, acc, 0, 0, 0);
  }
  return acc;
}
__device__ __forceinline__ void st16(double* C, int sc, d4 acc) {
  const int l = threadIdx.x & 63;
#pragma unroll
  for (int r = 0; r < 4; ++r) C[((l >> 4) + 4 * r) * sc + (l & 15)] = acc[r];
}
__device__ __forceinline__ d4 ld16(const double* C, int sc) {
  const int l = threadIdx.x & 63;
  d4 acc;
#pragma unroll
  for (int r = 0; r < 4; ++r) acc[r] = C[((l >> 4) + 4 * r) * sc + (l & 15)];
  return acc;
}

#ifdef SLAM_TL_PROFILE
__device__ unsigned long long g_tl_stamp[8];
#define TL_STAMP(i) \
  if (blockIdx.x == 1 && threadIdx.x == 0 && tl_prof_on) g_tl_stamp[i] = wall_clock64()
#else
#define TL_STAMP(i) (void)0
#endif
// Akk == nullptr: the tile is already in M (written before the call; the
// first barrier below publishes it).
#ifdef SLAM_FLOW_PROFILE
__device__ unsigned long long g_flow_fac[16];
#define FAC_T(i)                                                    \
  do {                                                              \
    if (blockIdx.x == 0 && threadIdx.x == 0) g_flow_fac[i] = wall_clock64(); \
  } while (0)
#else
#define FAC_T(i) (void)0
#endif
// LDS written by this wave visible to its own later reads (no other wave involved)
__device__ __forceinline__ void wave_lds_fence() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// Fused broadcast-FMA updates of the 16x16 register factor (v_fmac_f64 with a
// DPP row_newbcast source: one instruction per update instead of a
// v_mov_b64_dpp + v_fma_f64 pair -- the compiler does not combine 64-bit DPP
// moves into VOP2).  FacRest<J>: v[m] += bcast_m(nl) * l for m = J+1..15;
// InvRest<K>: s[i] += bcast_i(vk) * xk for i = K+1..15.  The leading s_nop 1
// covers the VALU-write -> DPP-read hazard of the broadcast source; no
// register these blocks write is read by a DPP (compiler or asm) before
// compiler code rewrites it.  Bit for bit the products and sums of the
// two-instruction form.
template <int J> struct FacRest;
template <int K> struct InvRest;
template <> struct FacRest<0> {
  static __device__ __forceinline__ void run(double (&v)[16], double nl, double l) {
    asm("s_nop 1\n" "v_fmac_f64_dpp %0, %15, %16 row_newbcast:1 row_mask:0xf bank_mask:0xf\n" "v_fmac_f64_dpp %1, %15, %16 row_newbcast:2 row_mask:0xf bank_mask:0xf\n" "v_fmac_f64_dpp %2, %15, %16 row_newbcast:3 row_mask:0xf bank_mask:0xf\n" "v_fmac_f64_dpp %3, %15, %16 row_newbcast:4 row_mask:0xf bank_mask:0xf\n" "v_fmac_f64_dpp %4, %15, %16 row_newbcast:5 row_mask:0xf bank_mask:0xf\n" "v_fmac_f64_dpp %5, %15, %16 row_newbcast:6 row_mask:0xf bank_mask:0xf\n" "v_fmac_f64_dpp %6, %15, %16 row_newbcast:7 row_mask:0xf bank_mask:0xf\n" "v_fmac_f64_dpp %7, %15, %16 row_newbcast:8 row_mask:0xf bank_mask:0xf\n" "v_fmac_f64_dpp %8, %15, %16 row_newbcast:9 row_mask:0xf bank_mask:0xf\n" "v_fmac_f64_dpp %9, %15, %16 row_newbcast:10 row_mask:0xf bank_mask:0xf\n" "v_fmac_f64_dpp %10, %15, %16 row_newbcast:11 row_mask:0xf bank_mask:0xf\n" "v_fmac_f64_dpp %11, %15, %16 row_newbcast:12 row_mask:0xf bank_mask:0xf\n" "v_fmac_f64_dpp %12, %15, %16 row_newbcast:13 row_mask:0xf bank_mask:0xf\n" "v_fmac_f64_dpp %13, %15, %16 row_newbcast:14 row_mask:0xf bank_mask:0xf\n" "v_fmac_f64_dpp %14, %15, %16 row_newbcast:15 row_mask:0xf bank_mask:0xf\n"
                 : "+v"(v[1]), "+v"(v[2]), "+v"(v[3]), "+v"(v[4]), "+v"(v[5]), "+v"(v[6]), "+v"(v[7]), "+v"(v[8]), "+v"(v[9]), "+v"(v[10]), "+v"(v[11]), "+v"(v[12]), "+v"(v[13]), "+v"(v[14]), "+v"(v[15])
                 : "v"(nl), "v"(l));
  }
};
template <> struct FacRest<1> {
  static __device__ __forceinline__ void run(double (&v)[16], double nl, double l) {
    asm("s_nop 1\n" "v_fmac_f64_dpp %0, %14, %15 row_newbcast:2 row_mask:0xf bank_mask:0xf\n" "v_fmac_f64_dpp %1, %14, %15 row_newbcast:3 row_mask:0xf bank_mask:0xf\n" "v_fmac_f64_dpp %2, %14, %15 row_newbcast:4 row_mask:0xf bank_mask:0xf\n" "v_fmac_f64_dpp %3, %14, %15 row_newbcast:5 row_mask:0xf bank_mask:0xf\n" "v_fmac_f64_dpp %4, %14, %15 row_newbcast:6 row_mask:0xf bank_mask:0xf\n" "v_fmac_f64_dpp %5, %14, %15 row_newbcast:7 row_mask:0xf bank_mask:0xf\n" "v_fmac_f64_dpp %6, %14, %15 row_newbcast:8 row_mask:0xf bank_mask:0xf\n" "v_fmac_f64_dpp %7, %14, %15 row_newbcast:9 row_mask:0xf bank_mask:0xf\n" "v_fmac_f64_dpp %8, %14, %15 row_newbcast:10 row_mask:0xf bank_mask:0xf\n" "v_fmac_f64_dpp %9, %14, %15 row_newbcast:11 row_mask:0xf bank_mask:0xf\n" "v_fmac_f64_dpp %10, %14, %15 row_newbcast:12 row_mask:0xf bank_mask:0xf\n" "v_fmac_f64_dpp %11, %14, %15 row_newbcast:13 row_mask:0xf bank_mask:0xf\n" "v_fmac_f64_dpp %12, %14, %15 row_newbcast:14 row_mask:0xf bank_mask:0xf\n" "v_fmac_f64_dpp %13, %14, %15 row_newbcast:15 row_mask:0xf bank_mask:0xf\n"
                 : "+v"(v[2]), "+v"(v[3]), "+v"(v[4]), "+v"(v[5]), "+v"(v[6]), "+v"(v[7]), "+v"(v[8]), "+v"(v[9]), "+v"(v[10]), "+v"(v[11]), "+v"(v[12]), "+v"(v[13]), "+v"(v[14]), "+v"(v[15])
                 : "v"(nl), "v"(l));
  }
};
template <> struct FacRest<2> {
  static __device__ __forceinline__ void run(double (&v)[16], double nl, double l) {
    asm("s_nop 1\n" "v_fmac_f64_dpp %0, %13, %14 row_newbcast:3 row_mask:0xf bank_mask:0xf\n" "v_fmac_f64_dpp %1, %13, %14 row_newbcast:4 row_mask:0xf bank_mask:0xf\n" "v_fmac_f64_dpp %2, %13, %14 row_newbcast:5 row_mask:0xf bank_mask:0xf\n" "v_fmac_f64_dpp %3, %13, %14 row_newbcast:6 row_mask:0xf bank_mask:0xf\n" "v_fmac_f64_dpp %4, %13, %14 row_newbcast:7 row_mask:0xf bank_mask:0xf\n" "v_fmac_f64_dpp %5, %13, %14 row_newbcast:8 row_mask:0xf bank_mask:0xf\n" "v_fmac_f64_dpp %6, %13, %14 row_newbcast:9 row_mask:0xf bank_mask:0xf\n" "v_fmac_f64_dpp %7, %13, %14 row_newbcast:10 row_mask:0xf bank_mask:0xf\n" "v_fmac_f64_dpp %8, %13, %14 row_newbcast:11 row_mask:0xf bank_mask:0xf\n" "v_fmac_f64_dpp %9, %13, %14 row_newbcast:12 row_mask:0xf bank_mask:0xf\n" "v_fmac_f64_dpp %10, %13, %14 row_newbcast:13 row_mask:0xf bank_mask:0xf\n" "v_fmac_f64_dpp %11, %13, %14 row_newbcast:14 row_mask:0xf bank_mask:0xf\n" "v_fmac_f64_dpp %12, %13, %14 row_newbcast:15 row_mask:0xf bank_mask:0xf\n"
                 : "+v"(v[3]), "+v"(v[4]), "+v"(v[5]), "+v"(v[6]), "+v"(v[7]), "+v"(v[8]), "+v"(v[9]), "+v"(v[10]), "+v"(v[11]), "+v"(v[12]), "+v"(v[13]), "+v"(v[14]), "+v"(v[15])
                 : "v"(nl), "v"(l));
  }
};
template <> struct FacRest<3> {
  static __device__ __forceinline__ void run(double (&v)[16], double nl, double l) {
    asm("s_nop 1\n" "v_fmac_f64_dpp %0, %12, %13 row_newbcast:4 row_mask:0xf bank_mask:0xf\n" "v_fmac_f64_dpp %1, %12, %13 row_newbcast:5 row_mask:0xf bank_mask:0xf\n" "v_fmac_f64_dpp %2, %12, %13 row_newbcast:6 row_mask:0xf bank_mask:0xf\n" "v_fmac_f64_dpp %3, %12, %13 row_newbcast:7 row_mask:0xf bank_mask:0xf\n" "v_fmac_f64_dpp %4, %12, %13 row_newbcast:8 row_mask:0xf bank_mask:0xf\n" "v_fmac_f64_dpp %5, %12, %13 row_newbcast:9 row_mask:0xf bank_mask:0xf\n" "v_fmac_f64_dpp %6, %12, %13 row_newbcast:10 row_mask:0xf bank_mask:0xf\n" "v_fmac_f64_dpp %7, %12, %13 row_newbcast:11 row_mask:0xf bank_mask:0xf\n" "v_fmac_f64_dpp %8, %12, %13 row_newbcast:12 row_mask:0xf bank_mask:0xf\n" "v_fmac_f64_dpp %9, %12, %13 row_newbcast:13 row_mask:0xf bank_mask:0xf\n" "v_fmac_f64_dpp %10, %12, %13 row_newbcast:14 row_mask:0xf bank_mask:0xf\n" "v_fmac_f64_dpp %11, %12, %13 row_newbcast:15 row_mask:0xf bank_mask:0xf\n"
                 : "+v"(v[4]), "+v"(v[5]), "+v"(v[6]), "+v"(v[7]), "+v"(v[8]), "+v"(v[9]), "+v"(v[10]), "+v"(v[11]), "+v"(v[12]), "+v"(v[13]), "+v"(v[14]), "+v"(v[15])
                 : "v"(nl), "v"(l));
  }
};
template <> struct FacRest<4> {
  static __device__ __forceinline__ void run(double (&v)[16], double nl, double l) {
    asm("s_nop 1\n" "v_fmac_f64_dpp %0, %11, %12 row_newbcast:5 row_mask:0xf bank_mask:0xf\n" "v_fmac_f64_dpp %1, %11, %12 row_newbcast:6 row_mask:0xf bank_mask:0xf\n" "v_fmac_f64_dpp %2, %11, %12 row_newbcast:7 row_mask:0xf bank_mask:0xf\n" "v_fmac_f64_dpp %3, %11, %12 row_newbcast:8 row_mask:0xf bank_mask:0xf\n" "v_fmac_f64_dpp %4, %11, %12 row_newbcast:9 row_mask:0xf bank_mask:0xf\n" "v_fmac_f64_dpp %5, %11, %12 row_newbcast:10 row_mask:0xf bank_mask:0xf\n" "v_fmac_f64_dpp %6, %11, %12 row_newbcast:11 row_mask:0xf bank_mask:0xf\n" "v_fmac_f64_dpp %7, %11, %12 row_newbcast:12 row_mask:0xf bank_mask:0xf\n" "v_fmac_f64_dpp %8, %11, %12 row_newbcast:13 row_mask:0xf bank_mask:0xf\n" "v_fmac_f64_dpp %9, %11, %12 row_newbcast:14 row_mask:0xf bank_mask:0xf\n" "v_fmac_f64_dpp %10, %11, %12 row_newbcast:15 row_mask:0xf bank_mask:0xf\n"
                 : "+v"(v[5]), "+v"(v[6]), "+v"(v[7]), "+v"(v[8]), "+v"(v[9]), "+v"(v[10]), "+v"(v[11]), "+v"(v[12]), "+v"(v[13]), "+v"(v[14]), "+v"(v[15])
                 : "v"(nl), "v"(l));
  }
};
template <> struct FacRest<5> {
  static __device__ __forceinline__ void run(double (&v)[16], double nl, double l) {
    asm("s_nop 1\n" "v_fmac_f64_dpp %0, %10, %11 row_newbcast:6 row_mask:0xf bank_mask:0xf\n" "v_fmac_f64_dpp %1, %10, %11 row_newbcast:7 row_mask:0xf bank_mask:0xf\n" "v_fmac_f64_dpp %2, %10, %11 row_newbcast:8 row_mask:0xf bank_mask:0xf\n" "v_fmac_f64_dpp %3, %10, %11 row_newbcast:9 row_mask:0xf bank_mask:0xf\n" "v_fmac_f64_dpp %4, %10, %11 row_newbcast:10 row_mask:0xf bank_mask:0xf\n" "v_fmac_f64_dpp %5, %10, %11 row_newbcast:11 row_mask:0xf bank_mask:0xf\n" "v_fmac_f64_dpp %6, %10, %11 row_newbcast:12 row_mask:0xf bank_mask:0xf\n" "v_fmac_f64_dpp %7, %10, %11 row_newbcast:13 row_mask:0xf bank_mask:0xf\n" "v_fmac_f64_dpp %8, %10, %11 row_newbcast:14 row_mask:0xf bank_mask:0xf\n" "v_fmac_f64_dpp %9, %10, %11 row_newbcast:15 row_mask:0xf bank_mask:0xf\n"
                 : "+v"(v[6]), "+v"(v[7]), "+v"(v[8]), "+v"(v[9]), "+v"(v[10]), "+v"(v[11]), "+v"(v[12]), "+v"(v[13]), "+v"(v[14]), "+v"(v[15])
                 : "v"(nl), "v"(l));
  }
};
template <> struct FacRest<6> {
  static __device__ __forceinline__ void run(double (&v)[16], double nl, double l) {
    asm("s_nop 1\n" "v_fmac_f64_dpp %0, %9, %10 row_newbcast:7 row_mask:0xf bank_mask:0xf\n" "v_fmac_f64_dpp %1, %9, %10 row_newbcast:8 row_mask:0xf bank_mask:0xf\n" "v_fmac_f64_dpp %2, %9, %10 row_newbcast:9 row_mask:0xf bank_mask:0xf\n" "v_fmac_f64_dpp %3, %9, %10 row_newbcast:10 row_mask:0xf bank_mask:0xf\n" "v_fmac_f64_dpp %4, %9, %10 row_newbcast:11 row_mask:0xf bank_mask:0xf\n" "v_fmac_f64_dpp %5, %9, %10 row_newbcast:12 row_mask:0xf bank_mask:0xf\n" "v_fmac_f64_dpp %6, %9, %10 row_newbcast:13 row_mask:0xf bank_mask:0xf\n" "v_fmac_f64_dpp %7, %9, %10 row_newbcast:14 row_mask:0xf bank_mask:0xf\n" "v_fmac_f64_dpp %8, %9, %10 row_newbcast:15 row_mask:0xf bank_mask:0xf\n"
                 : "+v"(v[7]), "+v"(v[8]), "+v"(v[9]), "+v"(v[10]), "+v"(v[11]), "+v"(v[12]), "+v"(v[13]), "+v"(v[14]), "+v"(v[15])
                 : "v"(nl), "v"(l));
  }
};
template <> struct FacRest<7> {
  static __device__ __forceinline__ void run(double (&v)[16], double nl, double l) {
    asm("s_nop 1\n" "v_fmac_f64_dpp %0, %8, %9 row_newbcast:8 row_mask:0xf bank_mask:0xf\n" "v_fmac_f64_dpp %1, %8, %9 row_newbcast:9 row_mask:0xf bank_mask:0xf\n" "v_fmac_f64_dpp %2, %8, %9 row_newbcast:10 row_mask:0xf bank_mask:0xf\n" "v_fmac_f64_dpp %3, %8, %9 row_newbcast:11 row_mask:0xf bank_mask:0xf\n" "v_fmac_f64_dpp %4, %8, %9 row_newbcast:12 row_mask:0xf bank_mask:0xf\n" "v_fmac_f64_dpp %5, %8, %9 row_newbcast:13 row_mask:0xf bank_mask:0xf\n" "v_fmac_f64_dpp %6, %8, %9 row_newbcast:14 row_mask:0xf bank_mask:0xf\n" "v_fmac_f64_dpp %7, %8, %9 row_newbcast:15 row_mask:0xf bank_mask:0xf\n"
                 : "+v"(v[8]), "+v"(v[9]), "+v"(v[10]), "+v"(v[11]), "+v"(v[12]), "+v"(v[13]), "+v"(v[14]), "+v"(v[15])
                 : "v"(nl), "v"(l));
  }
};
template <> struct FacRest<8> {
  static __device__ __forceinline__ void run(double (&v)[16], double nl, double l) {
    asm("s_nop 1\n" "v_fmac_f64_dpp %0, %7, %8 row_newbcast:9 row_mask:0xf bank_mask:0xf\n" "v_fmac_f64_dpp %1, %7, %8 row_newbcast:10 row_mask:0xf bank_mask:0xf\n" "v_fmac_f64_dpp %2, %7, %8 row_newbcast:11 row_mask:0xf bank_mask:0xf\n" "v_fmac_f64_dpp %3, %7, %8 row_newbcast:12 row_mask:0xf bank_mask:0xf\n" "v_fmac_f64_dpp %4, %7, %8 row_newbcast:13 row_mask:0xf bank_mask:0xf\n" "v_fmac_f64_dpp %5, %7, %8 row_newbcast:14 row_mask:0xf bank_mask:0xf\n" "v_fmac_f64_dpp %6, %7, %8 row_newbcast:15 row_mask:0xf bank_mask:0xf\n"
                 : "+v"(v[9]), "+v"(v[10]), "+v"(v[11]), "+v"(v[12]), "+v"(v[13]), "+v"(v[14]), "+v"(v[15])
                 : "v"(nl), "v"(l));
  }
};
template <> struct FacRest<9> {
  static __device__ __forceinline__ void run(double (&v)[16], double nl, double l) {
    asm("s_nop 1\n" "v_fmac_f64_dpp %0, %6, %7 row_newbcast:10 row_mask:0xf bank_mask:0xf\n" "v_fmac_f64_dpp %1, %6, %7 row_newbcast:11 row_mask:0xf bank_mask:0xf\n" "v_fmac_f64_dpp %2, %6, %7 row_newbcast:12 row_mask:0xf bank_mask:0xf\n" "v_fmac_f64_dpp %3, %6, %7 row_newbcast:13 row_mask:0xf bank_mask:0xf\n" "v_fmac_f64_dpp %4, %6, %7 row_newbcast:14 row_mask:0xf bank_mask:0xf\n" "v_fmac_f64_dpp %5, %6, %7 row_newbcast:15 row_mask:0xf bank_mask:0xf\n"
                 : "+v"(v[10]), "+v"(v[11]), "+v"(v[12]), "+v"(v[13]), "+v"(v[14]), "+v"(v[15])
                 : "v"(nl), "v"(l));
  }
};
template <> struct FacRest<10> {
  static __device__ __forceinline__ void run(double (&v)[16], double nl, double l) {
    asm("s_nop 1\n" "v_fmac_f64_dpp %0, %5, %6 row_newbcast:11 row_mask:0xf bank_mask:0xf\n" "v_fmac_f64_dpp %1, %5, %6 row_newbcast:12 row_mask:0xf bank_mask:0xf\n" "v_fmac_f64_dpp %2, %5, %6 row_newbcast:13 row_mask:0xf bank_mask:0xf\n" "v_fmac_f64_dpp %3, %5, %6 row_newbcast:14 row_mask:0xf bank_mask:0xf\n" "v_fmac_f64_dpp %4, %5, %6 row_newbcast:15 row_mask:0xf bank_mask:0xf\n"
                 : "+v"(v[11]), "+v"(v[12]), "+v"(v[13]), "+v"(v[14]), "+v"(v[15])
                 : "v"(nl), "v"(l));
  }
};
template <> struct FacRest<11> {
  static __device__ __forceinline__ void run(double (&v)[16], double nl, double l) {
    asm("s_nop 1\n" "v_fmac_f64_dpp %0, %4, %5 row_newbcast:12 row_mask:0xf bank_mask:0xf\n" "v_fmac_f64_dpp %1, %4, %5 row_newbcast:13 row_mask:0xf bank_mask:0xf\n" "v_fmac_f64_dpp %2, %4, %5 row_newbcast:14 row_mask:0xf bank_mask:0xf\n" "v_fmac_f64_dpp %3, %4, %5 row_newbcast:15 row_mask:0xf bank_mask:0xf\n"
                 : "+v"(v[12]), "+v"(v[13]), "+v"(v[14]), "+v"(v[15])
                 : "v"(nl), "v"(l));
  }
};
template <> struct FacRest<12> {
  static __device__ __forceinline__ void run(double (&v)[16], double nl, double l) {
    asm("s_nop 1\n" "v_fmac_f64_dpp %0, %3, %4 row_newbcast:13 row_mask:0xf bank_mask:0xf\n" "v_fmac_f64_dpp %1, %3, %4 row_newbcast:14 row_mask:0xf bank_mask:0xf\n" "v_fmac_f64_dpp %2, %3, %4 row_newbcast:15 row_mask:0xf bank_mask:0xf\n"
                 : "+v"(v[13]), "+v"(v[14]), "+v"(v[15])
                 : "v"(nl), "v"(l));
  }
};
template <> struct FacRest<13> {
  static __device__ __forceinline__ void run(double (&v)[16], double nl, double l) {
    asm("s_nop 1\n" "v_fmac_f64_dpp %0, %2, %3 row_newbcast:14 row_mask:0xf bank_mask:0xf\n" "v_fmac_f64_dpp %1, %2, %3 row_newbcast:15 row_mask:0xf bank_mask:0xf\n"
                 : "+v"(v[14]), "+v"(v[15])
                 : "v"(nl), "v"(l));
  }
};
template <> struct FacRest<14> {
  static __device__ __forceinline__ void run(double (&v)[16], double nl, double l) {
    asm("s_nop 1\n" "v_fmac_f64_dpp %0, %1, %2 row_newbcast:15 row_mask:0xf bank_mask:0xf\n"
                 : "+v"(v[15])
                 : "v"(nl), "v"(l));
  }
};
template <> struct FacRest<15> {
  static __device__ __forceinline__ void run(double (&v)[16], double nl, double l) {
    (void)v; (void)nl; (void)l;
  }
};
template <> struct InvRest<0> {
  static __device__ __forceinline__ void run(double (&s)[16], double vk, double xk) {
    asm("s_nop 1\n" "v_fmac_f64_dpp %0, %15, %16 row_newbcast:1 row_mask:0xf bank_mask:0xf\n" "v_fmac_f64_dpp %1, %15, %16 row_newbcast:2 row_mask:0xf bank_mask:0xf\n" "v_fmac_f64_dpp %2, %15, %16 row_newbcast:3 row_mask:0xf bank_mask:0xf\n" "v_fmac_f64_dpp %3, %15, %16 row_newbcast:4 row_mask:0xf bank_mask:0xf\n" "v_fmac_f64_dpp %4, %15, %16 row_newbcast:5 row_mask:0xf bank_mask:0xf\n" "v_fmac_f64_dpp %5, %15, %16 row_newbcast:6 row_mask:0xf bank_mask:0xf\n" "v_fmac_f64_dpp %6, %15, %16 row_newbcast:7 row_mask:0xf bank_mask:0xf\n" "v_fmac_f64_dpp %7, %15, %16 row_newbcast:8 row_mask:0xf bank_mask:0xf\n" "v_fmac_f64_dpp %8, %15, %16 row_newbcast:9 row_mask:0xf bank_mask:0xf\n" "v_fmac_f64_dpp %9, %15, %16 row_newbcast:10 row_mask:0xf bank_mask:0xf\n" "v_fmac_f64_dpp %10, %15, %16 row_newbcast:11 row_mask:0xf bank_mask:0xf\n" "v_fmac_f64_dpp %11, %15, %16 row_newbcast:12 row_mask:0xf bank_mask:0xf\n" "v_fmac_f64_dpp %12, %15, %16 row_newbcast:13 row_mask:0xf bank_mask:0xf\n" "v_fmac_f64_dpp %13, %15, %16 row_newbcast:14 row_mask:0xf bank_mask:0xf\n" "v_fmac_f64_dpp %14, %15, %16 row_newbcast:15 row_mask:0xf bank_mask:0xf\n"
                 : "+v"(s[1]), "+v"(s[2]), "+v"(s[3]), "+v"(s[4]), "+v"(s[5]), "+v"(s[6]), "+v"(s[7]), "+v"(s[8]), "+v"(s[9]), "+v"(s[10]), "+v"(s[11]), "+v"(s[12]), "+v"(s[13]), "+v"(s[14]), "+v"(s[15])
                 : "v"(vk), "v"(xk));
  }
};
template <> struct InvRest<1> {
  static __device__ __forceinline__ void run(double (&s)[16], double vk, double xk) {
    asm("s_nop 1\n" "v_fmac_f64_dpp %0, %14, %15 row_newbcast:2 row_mask:0xf bank_mask:0xf\n" "v_fmac_f64_dpp %1, %14, %15 row_newbcast:3 row_mask:0xf bank_mask:0xf\n" "v_fmac_f64_dpp %2, %14, %15 row_newbcast:4 row_mask:0xf bank_mask:0xf\n" "v_fmac_f64_dpp %3, %14, %15 row_newbcast:5 row_mask:0xf bank_mask:0xf\n" "v_fmac_f64_dpp %4, %14, %15 row_newbcast:6 row_mask:0xf bank_mask:0xf\n" "v_fmac_f64_dpp %5, %14, %15 row_newbcast:7 row_mask:0xf bank_mask:0xf\n" "v_fmac_f64_dpp %6, %14, %15 row_newbcast:8 row_mask:0xf bank_mask:0xf\n" "v_fmac_f64_dpp %7, %14, %15 row_newbcast:9 row_mask:0xf bank_mask:0xf\n" "v_fmac_f64_dpp %8, %14, %15 row_newbcast:10 row_mask:0xf bank_mask:0xf\n" "v_fmac_f64_dpp %9, %14, %15 row_newbcast:11 row_mask:0xf bank_mask:0xf\n" "v_fmac_f64_dpp %10, %14, %15 row_newbcast:12 row_mask:0xf bank_mask:0xf\n" "v_fmac_f64_dpp %11, %14, %15 row_newbcast:13 row_mask:0xf bank_mask:0xf\n" "v_fmac_f64_dpp %12, %14, %15 row_newbcast:14 row_mask:0xf bank_mask:0xf\n" "v_fmac_f64_dpp %13, %14, %15 row_newbcast:15 row_mask:0xf bank_mask:0xf\n"
                 : "+v"(s[2]), "+v"(s[3]), "+v"(s[4]), "+v"(s[5]), "+v"(s[6]), "+v"(s[7]), "+v"(s[8]), "+v"(s[9]), "+v"(s[10]), "+v"(s[11]), "+v"(s[12]), "+v"(s[13]), "+v"(s[14]), "+v"(s[15])
                 : "v"(vk), "v"(xk));
  }
};
template <> struct InvRest<2> {
  static __device__ __forceinline__ void run(double (&s)[16], double vk, double xk) {
    asm("s_nop 1\n" "v_fmac_f64_dpp %0, %13, %14 row_newbcast:3 row_mask:0xf bank_mask:0xf\n" "v_fmac_f64_dpp %1, %13, %14 row_newbcast:4 row_mask:0xf bank_mask:0xf\n" "v_fmac_f64_dpp %2, %13, %14 row_newbcast:5 row_mask:0xf bank_mask:0xf\n" "v_fmac_f64_dpp %3, %13, %14 row_newbcast:6 row_mask:0xf bank_mask:0xf\n" "v_fmac_f64_dpp %4, %13, %14 row_newbcast:7 row_mask:0xf bank_mask:0xf\n" "v_fmac_f64_dpp %5, %13, %14 row_newbcast:8 row_mask:0xf bank_mask:0xf\n" "v_fmac_f64_dpp %6, %13, %14 row_newbcast:9 row_mask:0xf bank_mask:0xf\n" "v_fmac_f64_dpp %7, %13, %14 row_newbcast:10 row_mask:0xf bank_mask:0xf\n" "v_fmac_f64_dpp %8, %13, %14 row_newbcast:11 row_mask:0xf bank_mask:0xf\n" "v_fmac_f64_dpp %9, %13, %14 row_newbcast:12 row_mask:0xf bank_mask:0xf\n" "v_fmac_f64_dpp %10, %13, %14 row_newbcast:13 row_mask:0xf bank_mask:0xf\n" "v_fmac_f64_dpp %11, %13, %14 row_newbcast:14 row_mask:0xf bank_mask:0xf\n" "v_fmac_f64_dpp %12, %13, %14 row_newbcast:15 row_mask:0xf bank_mask:0xf\n"
                 : "+v"(s[3]), "+v"(s[4]), "+v"(s[5]), "+v"(s[6]), "+v"(s[7]), "+v"(s[8]), "+v"(s[9]), "+v"(s[10]), "+v"(s[11]), "+v"(s[12]), "+v"(s[13]), "+v"(s[14]), "+v"(s[15])
                 : "v"(vk), "v"(xk));
  }
};
template <> struct InvRest<3> {
  static __device__ __forceinline__ void run(double (&s)[16], double vk, double xk) {
    asm("s_nop 1\n" "v_fmac_f64_dpp %0, %12, %13 row_newbcast:4 row_mask:0xf bank_mask:0xf\n" "v_fmac_f64_dpp %1, %12, %13 row_newbcast:5 row_mask:0xf bank_mask:0xf\n" "v_fmac_f64_dpp %2, %12, %13 row_newbcast:6 row_mask:0xf bank_mask:0xf\n" "v_fmac_f64_dpp %3, %12, %13 row_newbcast:7 row_mask:0xf bank_mask:0xf\n" "v_fmac_f64_dpp %4, %12, %13 row_newbcast:8 row_mask:0xf bank_mask:0xf\n" "v_fmac_f64_dpp %5, %12, %13 row_newbcast:9 row_mask:0xf bank_mask:0xf\n" "v_fmac_f64_dpp %6, %12, %13 row_newbcast:10 row_mask:0xf bank_mask:0xf\n" "v_fmac_f64_dpp %7, %12, %13 row_newbcast:11 row_mask:0xf bank_mask:0xf\n" "v_fmac_f64_dpp %8, %12, %13 row_newbcast:12 row_mask:0xf bank_mask:0xf\n" "v_fmac_f64_dpp %9, %12, %13 row_newbcast:13 row_mask:0xf bank_mask:0xf\n" "v_fmac_f64_dpp %10, %12, %13 row_newbcast:14 row_mask:0xf bank_mask:0xf\n" "v_fmac_f64_dpp %11, %12, %13 row_newbcast:15 row_mask:0xf bank_mask:0xf\n"
                 : "+v"(s[4]), "+v"(s[5]), "+v"(s[6]), "+v"(s[7]), "+v"(s[8]), "+v"(s[9]), "+v"(s[10]), "+v"(s[11]), "+v"(s[12]), "+v"(s[13]), "+v"(s[14]), "+v"(s[15])
                 : "v"(vk), "v"(xk));
  }
};
template <> struct InvRest<4> {
  static __device__ __forceinline__ void run(double (&s)[16], double vk, double xk) {
    asm("s_nop 1\n" "v_fmac_f64_dpp %0, %11, %12 row_newbcast:5 row_mask:0xf bank_mask:0xf\n" "v_fmac_f64_dpp %1, %11, %12 row_newbcast:6 row_mask:0xf bank_mask:0xf\n" "v_fmac_f64_dpp %2, %11, %12 row_newbcast:7 row_mask:0xf bank_mask:0xf\n" "v_fmac_f64_dpp %3, %11, %12 row_newbcast:8 row_mask:0xf bank_mask:0xf\n" "v_fmac_f64_dpp %4, %11, %12 row_newbcast:9 row_mask:0xf bank_mask:0xf\n" "v_fmac_f64_dpp %5, %11, %12 row_newbcast:10 row_mask:0xf bank_mask:0xf\n" "v_fmac_f64_dpp %6, %11, %12 row_newbcast:11 row_mask:0xf bank_mask:0xf\n" "v_fmac_f64_dpp %7, %11, %12 row_newbcast:12 row_mask:0xf bank_mask:0xf\n" "v_fmac_f64_dpp %8, %11, %12 row_newbcast:13 row_mask:0xf bank_mask:0xf\n" "v_fmac_f64_dpp %9, %11, %12 row_newbcast:14 row_mask:0xf bank_mask:0xf\n" "v_fmac_f64_dpp %10, %11, %12 row_newbcast:15 row_mask:0xf bank_mask:0xf\n"
                 : "+v"(s[5]), "+v"(s[6]), "+v"(s[7]), "+v"(s[8]), "+v"(s[9]), "+v"(s[10]), "+v"(s[11]), "+v"(s[12]), "+v"(s[13]), "+v"(s[14]), "+v"(s[15])
                 : "v"(vk), "v"(xk));
  }
};
template <> struct InvRest<5> {
  static __device__ __forceinline__ void run(double (&s)[16], double vk, double xk) {
    asm("s_nop 1\n" "v_fmac_f64_dpp %0, %10, %11 row_newbcast:6 row_mask:0xf bank_mask:0xf\n" "v_fmac_f64_dpp %1, %10, %11 row_newbcast:7 row_mask:0xf bank_mask:0xf\n" "v_fmac_f64_dpp %2, %10, %11 row_newbcast:8 row_mask:0xf bank_mask:0xf\n" "v_fmac_f64_dpp %3, %10, %11 row_newbcast:9 row_mask:0xf bank_mask:0xf\n" "v_fmac_f64_dpp %4, %10, %11 row_newbcast:10 row_mask:0xf bank_mask:0xf\n" "v_fmac_f64_dpp %5, %10, %11 row_newbcast:11 row_mask:0xf bank_mask:0xf\n" "v_fmac_f64_dpp %6, %10, %11 row_newbcast:12 row_mask:0xf bank_mask:0xf\n" "v_fmac_f64_dpp %7, %10, %11 row_newbcast:13 row_mask:0xf bank_mask:0xf\n" "v_fmac_f64_dpp %8, %10, %11 row_newbcast:14 row_mask:0xf bank_mask:0xf\n" "v_fmac_f64_dpp %9, %10, %11 row_newbcast:15 row_mask:0xf bank_mask:0xf\n"
                 : "+v"(s[6]), "+v"(s[7]), "+v"(s[8]), "+v"(s[9]), "+v"(s[10]), "+v"(s[11]), "+v"(s[12]), "+v"(s[13]), "+v"(s[14]), "+v"(s[15])
                 : "v"(vk), "v"(xk));
  }
};
template <> struct InvRest<6> {
  static __device__ __forceinline__ void run(double (&s)[16], double vk, double xk) {
    asm("s_nop 1\n" "v_fmac_f64_dpp %0, %9, %10 row_newbcast:7 row_mask:0xf bank_mask:0xf\n" "v_fmac_f64_dpp %1, %9, %10 row_newbcast:8 row_mask:0xf bank_mask:0xf\n" "v_fmac_f64_dpp %2, %9, %10 row_newbcast:9 row_mask:0xf bank_mask:0xf\n" "v_fmac_f64_dpp %3, %9, %10 row_newbcast:10 row_mask:0xf bank_mask:0xf\n" "v_fmac_f64_dpp %4, %9, %10 row_newbcast:11 row_mask:0xf bank_mask:0xf\n" "v_fmac_f64_dpp %5, %9, %10 row_newbcast:12 row_mask:0xf bank_mask:0xf\n" "v_fmac_f64_dpp %6, %9, %10 row_newbcast:13 row_mask:0xf bank_mask:0xf\n" "v_fmac_f64_dpp %7, %9, %10 row_newbcast:14 row_mask:0xf bank_mask:0xf\n" "v_fmac_f64_dpp %8, %9, %10 row_newbcast:15 row_mask:0xf bank_mask:0xf\n"
                 : "+v"(s[7]), "+v"(s[8]), "+v"(s[9]), "+v"(s[10]), "+v"(s[11]), "+v"(s[12]), "+v"(s[13]), "+v"(s[14]), "+v"(s[15])
                 : "v"(vk), "v"(xk));
  }
};
template <> struct InvRest<7> {
  static __device__ __forceinline__ void run(double (&s)[16], double vk, double xk) {
    asm("s_nop 1\n" "v_fmac_f64_dpp %0, %8, %9 row_newbcast:8 row_mask:0xf bank_mask:0xf\n" "v_fmac_f64_dpp %1, %8, %9 row_newbcast:9 row_mask:0xf bank_mask:0xf\n" "v_fmac_f64_dpp %2, %8, %9 row_newbcast:10 row_mask:0xf bank_mask:0xf\n" "v_fmac_f64_dpp %3, %8, %9 row_newbcast:11 row_mask:0xf bank_mask:0xf\n" "v_fmac_f64_dpp %4, %8, %9 row_newbcast:12 row_mask:0xf bank_mask:0xf\n" "v_fmac_f64_dpp %5, %8, %9 row_newbcast:13 row_mask:0xf bank_mask:0xf\n" "v_fmac_f64_dpp %6, %8, %9 row_newbcast:14 row_mask:0xf bank_mask:0xf\n" "v_fmac_f64_dpp %7, %8, %9 row_newbcast:15 row_mask:0xf bank_mask:0xf\n"
                 : "+v"(s[8]), "+v"(s[9]), "+v"(s[10]), "+v"(s[11]), "+v"(s[12]), "+v"(s[13]), "+v"(s[14]), "+v"(s[15])
                 : "v"(vk), "v"(xk));
  }
};
template <> struct InvRest<8> {
  static __device__ __forceinline__ void run(double (&s)[16], double vk, double xk) {
    asm("s_nop 1\n" "v_fmac_f64_dpp %0, %7, %8 row_newbcast:9 row_mask:0xf bank_mask:0xf\n" "v_fmac_f64_dpp %1, %7, %8 row_newbcast:10 row_mask:0xf bank_mask:0xf\n" "v_fmac_f64_dpp %2, %7, %8 row_newbcast:11 row_mask:0xf bank_mask:0xf\n" "v_fmac_f64_dpp %3, %7, %8 row_newbcast:12 row_mask:0xf bank_mask:0xf\n" "v_fmac_f64_dpp %4, %7, %8 row_newbcast:13 row_mask:0xf bank_mask:0xf\n" "v_fmac_f64_dpp %5, %7, %8 row_newbcast:14 row_mask:0xf bank_mask:0xf\n" "v_fmac_f64_dpp %6, %7, %8 row_newbcast:15 row_mask:0xf bank_mask:0xf\n"
                 : "+v"(s[9]), "+v"(s[10]), "+v"(s[11]), "+v"(s[12]), "+v"(s[13]), "+v"(s[14]), "+v"(s[15])
                 : "v"(vk), "v"(xk));
  }
};
template <> struct InvRest<9> {
  static __device__ __forceinline__ void run(double (&s)[16], double vk, double xk) {
    asm("s_nop 1\n" "v_fmac_f64_dpp %0, %6, %7 row_newbcast:10 row_mask:0xf bank_mask:0xf\n" "v_fmac_f64_dpp %1, %6, %7 row_newbcast:11 row_mask:0xf bank_mask:0xf\n" "v_fmac_f64_dpp %2, %6, %7 row_newbcast:12 row_mask:0xf bank_mask:0xf\n" "v_fmac_f64_dpp %3, %6, %7 row_newbcast:13 row_mask:0xf bank_mask:0xf\n" "v_fmac_f64_dpp %4, %6, %7 row_newbcast:14 row_mask:0xf bank_mask:0xf\n" "v_fmac_f64_dpp %5, %6, %7 row_newbcast:15 row_mask:0xf bank_mask:0xf\n"
                 : "+v"(s[10]), "+v"(s[11]), "+v"(s[12]), "+v"(s[13]), "+v"(s[14]), "+v"(s[15])
                 : "v"(vk), "v"(xk));
  }
};
template <> struct InvRest<10> {
  static __device__ __forceinline__ void run(double (&s)[16], double vk, double xk) {
    asm("s_nop 1\n" "v_fmac_f64_dpp %0, %5, %6 row_newbcast:11 row_mask:0xf bank_mask:0xf\n" "v_fmac_f64_dpp %1, %5, %6 row_newbcast:12 row_mask:0xf bank_mask:0xf\n" "v_fmac_f64_dpp %2, %5, %6 row_newbcast:13 row_mask:0xf bank_mask:0xf\n" "v_fmac_f64_dpp %3, %5, %6 row_newbcast:14 row_mask:0xf bank_mask:0xf\n" "v_fmac_f64_dpp %4, %5, %6 row_newbcast:15 row_mask:0xf bank_mask:0xf\n"
                 : "+v"(s[11]), "+v"(s[12]), "+v"(s[13]), "+v"(s[14]), "+v"(s[15])
                 : "v"(vk), "v"(xk));
  }
};
template <> struct InvRest<11> {
  static __device__ __forceinline__ void run(double (&s)[16], double vk, double xk) {
    asm("s_nop 1\n" "v_fmac_f64_dpp %0, %4, %5 row_newbcast:12 row_mask:0xf bank_mask:0xf\n" "v_fmac_f64_dpp %1, %4, %5 row_newbcast:13 row_mask:0xf bank_mask:0xf\n" "v_fmac_f64_dpp %2, %4, %5 row_newbcast:14 row_mask:0xf bank_mask:0xf\n" "v_fmac_f64_dpp %3, %4, %5 row_newbcast:15 row_mask:0xf bank_mask:0xf\n"
                 : "+v"(s[12]), "+v"(s[13]), "+v"(s[14]), "+v"(s[15])
                 : "v"(vk), "v"(xk));
  }
};
template <> struct InvRest<12> {
  static __device__ __forceinline__ void run(double (&s)[16], double vk, double xk) {
    asm("s_nop 1\n" "v_fmac_f64_dpp %0, %3, %4 row_newbcast:13 row_mask:0xf bank_mask:0xf\n" "v_fmac_f64_dpp %1, %3, %4 row_newbcast:14 row_mask:0xf bank_mask:0xf\n" "v_fmac_f64_dpp %2, %3, %4 row_newbcast:15 row_mask:0xf bank_mask:0xf\n"
                 : "+v"(s[13]), "+v"(s[14]), "+v"(s[15])
                 : "v"(vk), "v"(xk));
  }
};
template <> struct InvRest<13> {
  static __device__ __forceinline__ void run(double (&s)[16], double vk, double xk) {
    asm("s_nop 1\n" "v_fmac_f64_dpp %0, %2, %3 row_newbcast:14 row_mask:0xf bank_mask:0xf\n" "v_fmac_f64_dpp %1, %2, %3 row_newbcast:15 row_mask:0xf bank_mask:0xf\n"
                 : "+v"(s[14]), "+v"(s[15])
                 : "v"(vk), "v"(xk));
  }
};
template <> struct InvRest<14> {
  static __device__ __forceinline__ void run(double (&s)[16], double vk, double xk) {
    asm("s_nop 1\n" "v_fmac_f64_dpp %0, %1, %2 row_newbcast:15 row_mask:0xf bank_mask:0xf\n"
                 : "+v"(s[15])
                 : "v"(vk), "v"(xk));
  }
};
template <> struct InvRest<15> {
  static __device__ __forceinline__ void run(double (&s)[16], double vk, double xk) {
    (void)s; (void)vk; (void)xk;
  }
};

// Wave 0's part of block column p: the 16x16 diagonal block of M factored in
// registers and inverted (X_pp = L_pp^-1 into Xb); `ok` cleared on a
// non-positive or non-finite pivot.
__device__ __forceinline__ void blk_factor_w0(double* M, double* Xb, int p, bool& ok) {
  const int l = threadIdx.x & 63;
  const int i = l & 15;
  double v[16], rj[16];
#pragma unroll
  for (int c = 0; c < 16; ++c) v[c] = c <= i ? M[(16 * p + i) * kMS + 16 * p + c] : 0.0;
  // Pivot chain: d_j -> rsq + 2 Newton steps -> p = v_j r (row i's L_ij for
  // i > j) -> lane j+1's own update d_{j+1} = v_{j+1} - p^2 -> broadcast.  The
  // broadcasts of column j to the other rows read p from rows m > j only, so
  // they need no select; the whole-row update of column j (fused DPP FMAs)
  // is off the chain.  Same operations as the plain right-looking form.
  double dn = bcast16<0>(v[0]);
  static_for<0, 16>([&](auto J) {
    constexpr int j = decltype(J)::value;
    const double djj = dn;
    ok = ok && djj > 0.0 && djj < INFINITY;
    double r = __builtin_amdgcn_rsq(djj);
    const double h = 0.5 * djj;
    r = r * __builtin_fma(-h * r, r, 1.5);
    r = r * __builtin_fma(-h * r, r, 1.5);
    rj[j] = r;
    const double pj = v[j] * r;
    if constexpr (j + 1 < 16) dn = bcast16<j + 1>(__builtin_fma(-pj, pj, v[j + 1]));
    const double lij = i > j ? pj : (i == j ? djj * r : 0.0);
    v[j] = lij;
    FacRest<j>::run(v, -pj, lij);
  });
  FAC_T(2 + 3 * p);  // (profiling build: wave 0's pivots of block p done)
  // column c = lane of L_pp^-1: x_c = 1 / l_cc, x_i = -(sum_{k<i} l_ik x_k) / l_ii
  // (column-oriented: once x_k is known, every later row's sum takes its
  // term -- the same k order per sum as the row form, a 16-step chain
  // instead of 120 dependent FMAs); l_ik = lane ii's v[k], by row_newbcast.
  // The sum of row c starts at -1 so that x_k = -s_k / l_kk holds for every
  // k >= c with no select on the chain (x_c = 1 / l_cc exactly; the rows
  // above c carry signed zeros, written as 0 below)
  const int c = l & 15;
  double x[16], sacc[16];
#pragma unroll
  for (int ii = 0; ii < 16; ++ii) sacc[ii] = ii == c ? -1.0 : 0.0;
  static_for<0, 16>([&](auto K) {
    constexpr int k = decltype(K)::value;
    x[k] = -sacc[k] * rj[k];
    InvRest<k>::run(sacc, v[k], x[k]);
  });
  if (l < 16) {
    double* X = Xb + blk_id(p, p) * 16 * kBS17;
#pragma unroll
    for (int ii = 0; ii < 16; ++ii) X[ii * kBS17 + c] = ii < c ? 0.0 : x[ii];
  }
}

// nb: the tile's 16-row blocks that hold rows of S (ba.tl_schedule: a tile of
// c whole cameras has 9c rows, the rest padding with a unit diagonal and no
// coupling); wave 0 skips the pivot chain of every block p >= nb, whose factor
// and inverse are the identity (X_pp = I written directly), so a 45-row tile
// runs three 16x16 factors instead of four.  Waves 1-3 still form the blocks of
// L / L^-1 in the padding rows (exact zeros) beside the chain.
__device__ __forceinline__ void blk_identity_w0(double* Xb, int p) {
  const int l = threadIdx.x & 63;
  if (l < 16) {
    double* X = Xb + blk_id(p, p) * 16 * kBS17;
#pragma unroll
    for (int ii = 0; ii < 16; ++ii) X[ii * kBS17 + l] = ii == l ? 1.0 : 0.0;
  }
}

__device__ __forceinline__ bool tile_chol_inv_blk(const double* __restrict__ Akk, int ld,
                                                  double* M, double* Xb, double* Tb, int* okp,
                                                  int nb = 4, bool tl_prof_on = false) {
  const int t = threadIdx.x, l = t & 63, w = t >> 6;
  TL_STAMP(0);
  if (Akk != nullptr) {
    // all 16 loads of a lane in flight before the LDS stores
    double tmp[kTB * kTB / kTlWG];
#pragma unroll
    for (int q = 0; q < kTB * kTB / kTlWG; ++q) {
      const int e = t + kTlWG * q;
      tmp[q] = Akk[(size_t)(e >> 6) * ld + (e & 63)];
    }
#pragma unroll
    for (int q = 0; q < kTB * kTB / kTlWG; ++q) {
      const int e = t + kTlWG * q;
      M[(e >> 6) * kMS + (e & 63)] = tmp[q];
    }
  }
  bool ok = true;
  // wave-to-wave hand-offs inside the tile (LDS flags, raised once per call):
  // 0: L_10, 1: L_20, 2: L_30, 3: L_21, 4: L_31, 5: L_32 stored
  // callers pass M = VX, Xb = VX + kTB * kMS, Tb = Xb + 10 * 16 * kBS17 of a
  // VX[2 * kTB * kTB]: M + Xb + Tb + the six flags (3 doubles) must fit in it
  static_assert(kTB * kMS + 13 * 16 * kBS17 + 3 <= 2 * kTB * kTB, "tile factor LDS layout overflows VX");
  int* fl = reinterpret_cast<int*>(Tb + 3 * 16 * kBS17);
  if (t < 6) fl[t] = 0;
  __syncthreads();
  TL_STAMP(1);
  FAC_T(0);
  // One loop over the block columns with ONE instance of wave 0's 16x16 code
  // (an instance per block column measured 0.4-1.0 us slower per block: the
  // unrolled factor is ~16 KB of code and the copies missed the instruction
  // cache).  Wave 0 runs the critical chain with look-ahead: before block p's
  // factor it forms the panel block L_{p,p-1} and the trailing block A_pp
  // itself, so the only workgroup barrier per block column is the one that
  // publishes X_pp.  Waves 1-3 take the other panel and trailing blocks of
  // block column p-1 beside block p's factor (LDS flags for the blocks one
  // wave forms and another reads) and assemble L^-1 block by block as its
  // inputs appear, so that after block 3's factor only X_3p = -X_33 T_3p is
  // left (one 16x16 product per wave):
  //   X_ip = -X_ii T_ip,  T_ip = sum_{k=p}^{i-1} L_ik X_kp  (k ascending).
  // Every block gets the same updates in the same order as the column-by-column
  // form: bit-identical.
  const d4 z = d4{0.0, 0.0, 0.0, 0.0};
  auto T_of = [&](int i, int p, int k_end) {  // sum_{k=p}^{k_end-1} L_ik X_kp
    d4 acc = z;
    for (int k = p; k < k_end; ++k)
      acc = mm16_xy(M + (16 * i) * kMS + 16 * k, kMS, Xb + blk_id(k, p) * 16 * kBS17, kBS17, acc, false);
    return acc;
  };
  auto X_from = [&](int i, int p, d4 T) {  // X_ip = -X_ii T (T through this wave's Tb block)
    double* Tw = Tb + (w - 1) * 16 * kBS17;
    st16(Tw, kBS17, T);
    wave_lds_fence();
    st16(Xb + blk_id(i, p) * 16 * kBS17, kBS17, mm16_xy(Xb + blk_id(i, i) * 16 * kBS17, kBS17, Tw, kBS17, z, true));
    wave_lds_fence();
  };
  auto Mb = [&](int i, int j) { return M + (16 * i) * kMS + 16 * j; };
  auto panel = [&](int i, int p) {  // L_ip = A_ip X_pp^T, in place
    st16(Mb(i, p), kMS, mm16_xyT(Mb(i, p), kMS, Xb + blk_id(p, p) * 16 * kBS17, kBS17, z, false));
    wave_lds_fence();
  };
  auto trail = [&](int i, int j, int p) {  // A_ij -= L_ip L_jp^T
    st16(Mb(i, j), kMS, mm16_xyT(Mb(i, p), kMS, Mb(j, p), kMS, ld16(Mb(i, j), kMS), true));
    wave_lds_fence();
  };
  auto put = [&](int f) {  // this wave's LDS stores before it, then flag f
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    if (l == 0) __hip_atomic_store(fl + f, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
  };
  auto get = [&](int f) {
    while (__hip_atomic_load(fl + f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) == 0)
      __builtin_amdgcn_s_sleep(1);
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
  };
  d4 T3 = z;
#pragma unroll 1
  for (int p = 0; p < 4; ++p) {
    if (w == 0) {
      if (SLAM_TL_PADSKIP && p >= nb) {  // a padding block: L_{p,p-1} = 0, L_pp = X_pp = I
        put(p == 1 ? 0 : (p == 2 ? 3 : 5));
        blk_identity_w0(Xb, p);
      } else {
        if (p > 0) {  // look-ahead: L_{p,p-1}, then A_pp's last update
          panel(p, p - 1);
          put(p == 1 ? 0 : (p == 2 ? 3 : 5));
          trail(p, p, p - 1);
        }
        FAC_T(1 + 3 * p);  // (profiling build: block p's look-ahead done)
        blk_factor_w0(M, Xb, p, ok);
      }
    } else if (p == 1) {  // block column 0's other panel and trailing blocks
      if (w == 1) {
        panel(2, 0);
        put(1);
        trail(2, 2, 0);
        get(0);
        trail(2, 1, 0);
      } else if (w == 2) {
        panel(3, 0);
        put(2);
        trail(3, 3, 0);
        get(0);
        trail(3, 1, 0);
      } else {
        get(1);
        get(2);
        trail(3, 2, 0);
      }
    } else if (p == 2) {  // block column 1's, and X_10
      if (w == 1) {
        panel(3, 1);
        put(4);
        trail(3, 3, 1);
      } else if (w == 2) {
        get(3);
        get(4);
        trail(3, 2, 1);
      } else {
        X_from(1, 0, T_of(1, 0, 1));  // X_10 (X_00, X_11: published by the barriers)
      }
    } else if (p == 3) {
      if (w == 1) X_from(2, 1, T_of(2, 1, 2));  // X_21
      if (w == 2) X_from(2, 0, T_of(2, 0, 2));  // X_20 (needs X_10: published by the barrier)
      // wave 1: T_31, wave 2: T_30, wave 3: T_32 (each wave reads only the X
      // blocks it formed itself or that the barrier published), after L_32
      get(5);
      T3 = T_of(3, w == 1 ? 1 : (w == 2 ? 0 : 2), 3);
    }
    if (p < 3) {
      __syncthreads();  // X_pp and block column p-1's blocks published
      FAC_T(3 + 3 * p);
    }
  }
  FAC_T(12);
  __syncthreads();  // X_33 published
  if (w > 0) X_from(3, w == 1 ? 1 : (w == 2 ? 0 : 2), T3);
  TL_STAMP(2);
  if (w == 0 && l == 0) *okp = ok ? 1 : 0;
  __syncthreads();
  TL_STAMP(3);
  FAC_T(13);
  return *okp != 0;
}

// ---------------------------------------------------------------- level-scheduled tiled solve
// The same tile factor with the columns grouped by elimination-tree level
// (slam355/ba.py tl_schedule: tiles renumbered by nested dissection of the
// tile graph, symbolic structure on the host).  Per level: k_tl2_panel (WG per
// (k, I) of every column k of the level: the diagonal WG stores L_kk^-1 and
// y_k = L_kk^-1 b_k, the others L_Ik = A_Ik L_kk^-T), then k_tl2_update (WG
// per target tile (I, J) of the level: A_IJ -= sum_k L_Ik L_Jk^T on the f64
// matrix cores, and for I = J also b_I -= sum_k L_Ik y_k -- the sums over the
// level's columns inside one WG, no atomics).  k_tl2_back walks the levels in
// reverse: x_k = L_kk^-T (y_k - sum_I L_Ik^T x_I) over the ancestors I; then
// k_tl2_unperm moves x back to the camera order (into the y region, which the
// epilogue reads).  A banded window of T tiles runs ~log2 T levels instead of
// T panel steps (C4: 4 levels for 9 tiles; C5: 8 for 71).
// The schedule's row maps sit at fixed offsets after its kTlHdr-int header (ba.tl_schedule;
// checked on the host in tl_check_sched), so no lookup waits on a header load:
// row r of S (camera order) -> its row in the tiled system
__device__ __forceinline__ int tl_new_row(const int32_t* sched, int r) { return sched[kTlHdr + r]; }
// row of the tiled system -> row of S, -1 on a tile's padding rows
__device__ __forceinline__ int tl_old_row(const int32_t* sched, int n, int rn) { return sched[kTlHdr + n + rn]; }
// rows of S in tile k (they come first, padding after them)
__device__ __forceinline__ const int32_t* tl_tile_rows(const int32_t* sched, int n, int T) {
  return sched + kTlHdr + n + T * kTB;
}

// Zero the lower tiles (identity on the padded rows' diagonal), b in the new order.
// struct_only: only the tiles the symbolic factor touches -- (J, J) and (I, J)
// for the rows I of column J (column table; grid T x (1 + max rows)); every
// other lower tile is never read by either solve form (C5: 71 diagonal + row
// tiles of 2556 lower tiles).  Otherwise all T (T + 1) / 2 lower tiles.
__global__ __launch_bounds__(kTlWG) void k_tl2_load(slam_ba_problem p, int T_, int struct_only) {
  lm_wave_priority();
  const int n = 9 * p.n_cams;
  const TlLayout L(n, T_);
  const int32_t* S = p.tl_sched;
  int I, J;
  bool first;
  if (struct_only) {
    J = blockIdx.x;
    const int q = blockIdx.y;
    const int32_t* rec = S + S[5] + 5 * J;
    if (q > rec[1]) return;  // uniform; (0, 0) always runs
    I = q == 0 ? J : S[rec[0] + q - 1];
    first = blockIdx.x == 0 && q == 0;
  } else {
    const int idx = blockIdx.x;
    I = (int)((sqrtf(8.0f * (float)idx + 1.0f) - 1.0f) * 0.5f);
    while ((I + 1) * (I + 2) / 2 <= idx) ++I;
    while (I * (I + 1) / 2 > idx) --I;
    J = idx - I * (I + 1) / 2;
    first = idx == 0;
  }
  double* A = p.chol + L.a;
  for (int e = threadIdx.x; e < kTB * kTB; e += kTlWG) {
    const int i = I * kTB + (e >> 6), j = J * kTB + (e & 63);
    A[(size_t)i * L.N + j] = (i == j && tl_old_row(S, n, i) < 0) ? 1.0 : 0.0;  // identity on padding
  }
  if (I == J && threadIdx.x < kTB) {
    const int r = tl_old_row(S, n, I * kTB + threadIdx.x);  // row of S landing at new row I*64 + t
    p.chol[L.b + I * kTB + threadIdx.x] = r >= 0 ? p.sys[sys_vec_off(p.n_cams, p.n_blocks) + r] : 0.0;
  }
  if (first) {
    // k_tl3_flow: a new solve epoch (its flags compare against it); the retire
    // ticket, the start ticket and the per-column parent counters re-armed
    int* fl = reinterpret_cast<int*>(p.chol + L.flow) + L.T * L.T + 2 * L.T;
    for (int i = threadIdx.x; i < L.T; i += blockDim.x) fl[8 + i] = 0;
    if (threadIdx.x == 0) {
      *reinterpret_cast<int*>(p.chol + L.fail) = 0;
      fl[0] = 0;
      fl[1] = fl[1] + 1;
      fl[2] = 0;
    }
  }
}

// One WG per packed block: its values at their renumbered positions (lower
// tiles, full symmetric inside diagonal tiles), camera damping on the diagonal.
__global__ __launch_bounds__(128) void k_tl2_scatter(slam_ba_problem p, int T_) {
  lm_wave_priority();
  const int n = 9 * p.n_cams;
  const TlLayout L(n, T_);
  const int32_t* S = p.tl_sched;
  const int blk = blockIdx.x, t = threadIdx.x;
  if (t >= 81) return;
  const int c1 = p.blocks[2 * blk], c2 = p.blocks[2 * blk + 1];
  const double* vec = p.sys + sys_vec_off(p.n_cams, p.n_blocks);
  const int i = t / 9, j = t - 9 * (t / 9);
  const int r = 9 * c1 + i, c = 9 * c2 + j;  // element (r, c) of S
  double v = p.sys[(size_t)blk * 81 + t];
  if (r == c) v += p.state[SLAM_BA_ST_LAMBDA] * clampd(vec[2 * n + r]);
  double* A = p.chol + L.a;
  const int rn = tl_new_row(S, r), cn = tl_new_row(S, c);
  const int tr = rn / kTB, tc = cn / kTB;
  if (tr >= tc) A[(size_t)rn * L.N + cn] = v;
  if (c1 != c2 && tc >= tr) A[(size_t)cn * L.N + rn] = v;
}

__global__ __launch_bounds__(kTlWG) __attribute__((amdgpu_waves_per_eu(1, 1)))
void k_tl2_panel(slam_ba_problem p, int T_, int eoff) {
  lm_wave_priority();
  const TlLayout L(9 * p.n_cams, T_);
  if (tl_failed(p, L)) return;
  const int32_t* S = p.tl_sched;
  const int k = S[eoff + 2 * blockIdx.x], I = S[eoff + 2 * blockIdx.x + 1];
  __shared__ double VX[2 * kTB * kTB];
  double* Vf = VX;                        // L_kk^-1, fragment order
  __shared__ double Xf[kTB * kTB];        // A_Ik, fragment order
  __shared__ int okf;
  double* A = p.chol + L.a;
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const double* Akk = A + (size_t)k * kTB * L.N + k * kTB;
  double* AIk = A + (size_t)I * kTB * L.N + k * kTB;
  if (I > k && w >= 2) tile_to_frag(AIk, L.N, Xf, w - 2, 2);
  double x[kTB];
  double* Mb = VX;
  double* Xb = VX + kTB * kMS;
  double* Tb = Xb + 10 * 16 * kBS17;
  const bool ok = tile_chol_inv_blk(Akk, L.N, Mb, Xb, Tb, &okf, (tl_tile_rows(S, 9 * p.n_cams, T_)[k] + 15) >> 4);
  if (w == 1) {
    const int cb16 = lane >> 4;
#pragma unroll
    for (int m = 0; m < kTB; ++m)
      x[m] = (m >> 4) >= cb16 ? Xb[blk_id(m >> 4, cb16) * 16 * kBS17 + (m & 15) * kBS17 + (lane & 15)]
                              : 0.0;
  }
  __syncthreads();  // VX is reused below
  if (w == 1) {
    if (I == k) {
      const double bc = p.chol[L.b + k * kTB + lane];
      double* Vkk = p.chol + L.dinv + (size_t)k * kTB * kTB;
#pragma unroll
      for (int m = 0; m < kTB; ++m) Vkk[m * kTB + lane] = x[m];
#pragma unroll
      for (int m = 0; m < kTB; ++m) Vf[m * kTB + lane] = x[m] * bc;
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      double y = 0.0;
      for (int c = 0; c < kTB; ++c) y += Vf[lane * kTB + ((c + lane) & 63)];
      p.chol[L.y + k * kTB + lane] = y;
      if (!ok && lane == 0) *reinterpret_cast<int*>(p.chol + L.fail) = 1;
    } else {
#pragma unroll
      for (int m = 0; m < kTB; ++m) Vf[frag_idx(m, lane)] = x[m];
    }
  }
  if (I == k || !ok) return;
  __syncthreads();
  d4 acc[4];
  gemm_xyT_lowY(Xf, Vf, acc);  // L_Ik = A_Ik (L_kk^-1)^T
#pragma unroll
  for (int s2 = 0; s2 < 4; ++s2)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int row = w * 16 + (lane >> 4) + 4 * r, col = s2 * 16 + (lane & 15);
      AIk[(size_t)row * L.N + col] = acc[s2][r];
    }
}

__global__ __launch_bounds__(kTlWG) void k_tl2_update(slam_ba_problem p, int T_, int eoff) {
  lm_wave_priority();
  const TlLayout L(9 * p.n_cams, T_);
  if (tl_failed(p, L)) return;
  const int32_t* S = p.tl_sched;
  const int32_t* e = S + eoff + 4 * blockIdx.x;
  const int I = e[0], J = e[1], ko = e[2], kc = e[3];
  __shared__ double Xf[kTB * kTB], Yf[kTB * kTB];
  __shared__ double part[4][kTB];
  double* A = p.chol + L.a;
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  d4 acc[4];
#pragma unroll
  for (int s2 = 0; s2 < 4; ++s2) acc[s2] = d4{0.0, 0.0, 0.0, 0.0};
  double bs = 0.0;  // thread (w, lane): sum over k of row lane's part [16w, 16w + 16) of L_Ik y_k
  for (int q = 0; q < kc; ++q) {
    const int k = S[ko + q];
    const double* LIk = A + (size_t)I * kTB * L.N + k * kTB;
    tile_to_frag(LIk, L.N, Xf);
    if (I != J) tile_to_frag(A + (size_t)J * kTB * L.N + k * kTB, L.N, Yf);
    if (I == J) {
      const double* yk = p.chol + L.y + k * kTB;
      for (int m = 16 * w; m < 16 * w + 16; ++m)
        bs = __builtin_fma(LIk[(size_t)lane * L.N + m], yk[m], bs);
    }
    __syncthreads();
    const double* Y = I == J ? Xf : Yf;
#pragma unroll 4
    for (int kk = 0; kk < 16; ++kk) {
      const double a = Xf[((w * 16 + kk) << 6) + lane];
#pragma unroll
      for (int s2 = 0; s2 < 4; ++s2)
        acc[s2] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, Y[((s2 * 16 + kk) << 6) + lane], acc[s2],
                                                       0, 0, 0);
    }
    __syncthreads();  // Xf / Yf reloaded next k
  }
  double* AIJ = A + (size_t)I * kTB * L.N + J * kTB;
#pragma unroll
  for (int s2 = 0; s2 < 4; ++s2)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int row = w * 16 + (lane >> 4) + 4 * r, col = s2 * 16 + (lane & 15);
      AIJ[(size_t)row * L.N + col] -= acc[s2][r];
    }
  if (I == J) {
    part[w][lane] = bs;
    __syncthreads();
    if (t < kTB)
      p.chol[L.b + I * kTB + t] -= ((part[0][t] + part[1][t]) + part[2][t]) + part[3][t];
  }
}

// x_k = L_kk^-T (y_k - sum_I L_Ik^T x_I), I over the column's structure (ancestors).
__global__ __launch_bounds__(kTlWG) void k_tl2_back(slam_ba_problem p, int T_, int eoff) {
  lm_wave_priority();
  const TlLayout L(9 * p.n_cams, T_);
  if (tl_failed(p, L)) return;
  const int32_t* S = p.tl_sched;
  const int32_t* e = S + eoff + 3 * blockIdx.x;
  const int k = e[0], so = e[1], sc = e[2];
  __shared__ double r[kTB];
  __shared__ double part[4][kTB];
  const double* A = p.chol + L.a;
  const int t = threadIdx.x, c = t & 63, q = t >> 6;
  // thread (q, c): rows m in [16q, 16q + 16) of every L_Ik^T x_I, column c
  double s2 = 0.0;
  for (int u = 0; u < sc; ++u) {
    const int I = S[so + u];
    const double* LIk = A + (size_t)I * kTB * L.N + k * kTB;
    const double* xI = p.chol + L.x + I * kTB;
    for (int m = 16 * q; m < 16 * q + 16; ++m) s2 = __builtin_fma(LIk[(size_t)m * L.N + c], xI[m], s2);
  }
  part[q][c] = s2;
  __syncthreads();
  if (t < kTB) r[t] = p.chol[L.y + k * kTB + t] - (((part[0][t] + part[1][t]) + part[2][t]) + part[3][t]);
  __syncthreads();
  const double* Vkk = p.chol + L.dinv + (size_t)k * kTB * kTB;  // L_kk^-1
  double s3 = 0.0;
  for (int m = 16 * q; m < 16 * q + 16; ++m) s3 = __builtin_fma(Vkk[m * kTB + c], r[m], s3);
  part[q][c] = s3;
  __syncthreads();
  if (t < kTB) p.chol[L.x + k * kTB + t] = ((part[0][t] + part[1][t]) + part[2][t]) + part[3][t];
}

// x (new tile order, L.x) -> camera order in the y region (read by the epilogue)
__global__ __launch_bounds__(kTB) void k_tl2_unperm(slam_ba_problem p, int T_) {
  const TlLayout L(9 * p.n_cams, T_);
  const int I = blockIdx.x;  // new tile
  const int r = tl_old_row(p.tl_sched, 9 * p.n_cams, I * kTB + threadIdx.x);
  if (r >= 0) p.chol[L.y + r] = p.chol[L.x + I * kTB + threadIdx.x];
}

__global__ __launch_bounds__(1024) void k_tl2_epilogue(slam_ba_problem p, int T_) {
  lm_wave_priority();
  __shared__ double red[32];
  const int n = 9 * p.n_cams;
  const TlLayout L(n, T_);
  const bool ok = !tl_failed(p, L);
  const double* bvec = p.sys + sys_vec_off(p.n_cams, p.n_blocks);
  const double* gvec = bvec + n;
  solve_epilogue<true>(p, p.chol + L.y, ok, red,
                       EpiSrc{gvec, bvec + 2 * n, p.cams[cur_of(p.state)], gvec + 2 * n});
}

// ---------------------------------------------------------------- dataflow tiled solve
// The same factor as a dataflow graph in ONE launch: workgroup J owns tile
// column J (new numbering) for the whole solve and, from the schedule's column
// table (slam355/ba.py tl_schedule),
//   (1) A_JJ -= sum_{k in rs(J)} L_Jk L_Jk^T  (waits for each L_Jk's flag),
//       factor + inverse of the diagonal tile (tile_chol_inv_blk, from LDS);
//   (2) per row tile I in rows(J), parent first: A_IJ -= sum_k L_Ik L_Jk^T,
//       L_IJ = A_IJ L_JJ^-T, published (tile flag);
//   (3) y_J = L_JJ^-1 (b_J - sum_{k in rs(J)} L_Jk y_k)  (waits for y_k);
//   (4) x_J = L_JJ^-T (y_J - sum_{I in rows(J)} L_IJ^T x_I)  (waits for x_I),
//       stored in the new order and in camera order;
//   (5) the last column to finish (ticket) runs the solve epilogue.
// Launch boundaries become device flags: a column starts as soon as the tiles
// it needs exist, so the factor advances along the elimination tree with no
// per-level launch gaps.  Data crossing workgroups (L tiles, L_JJ^-1, y, x) is
// written with sc1 (write-through) stores and read with sc1 loads; a flag is
// raised after the writer's stores have drained (s_waitcnt + barrier) and
// equals the solve's epoch (bumped by k_tl2_load), so flags never need clearing.
// No residency assumption: a workgroup takes its column from a start
// ticket, so the columns are handed out in the order the workgroups actually
// start, and steps (1)-(3) wait only on lower columns -- workgroups that have
// already started and cannot be descheduled.  The back substitution (4) never
// waits on a later column: x_J is computed by the workgroup that retires the
// LAST of J's row tiles' x (a per-column counter; the roots by their own
// workgroup), so a column whose workgroup finished its forward part long ago,
// or a workgroup that has not started yet, holds nothing up.  The solve is
// therefore correct with any number of its workgroups resident (a CU-masked
// stream, other streams' kernels holding the CUs), and bit-identical whichever
// workgroup computes a column.  Every wait still gives up when the solve failed
// (non-SPD tile) or after kFlowSpinMax polls (a safety net that then marks the
// solve failed: SOLVE_FAULT), and every column is retired exactly once, so the
// retire ticket always reaches T and its last adder runs the epilogue.
constexpr int kFlowSpinMax = 1 << 22;  // ~0.2 s of 128-cycle polls
#ifndef SLAM_FLOW_SLEEP
#define SLAM_FLOW_SLEEP 2  // s_sleep between flag polls (units of 64 clocks)
#endif

#ifdef SLAM_FLOW_PROFILE
// per column: wall clock (100 MHz) at start, diagonal updates done, factor done,
// row tiles published, y published, x inputs in, x published, end
__device__ unsigned long long g_flow_stamp[SLAM_TL_FLOW_MAX_T][8];
// (stamps are kept per COLUMN: the workgroup's own column J, and (5), (6) for
// the column k whose x it formed)
#define FLOW_TC(col, i)                                           \
  do {                                                            \
    if (threadIdx.x == 0) g_flow_stamp[(col)][i] = wall_clock64(); \
  } while (0)
// finer stamps of the same column: first child tile in, last child tile in,
// row 0's deferred folds done, row 0 staged, row 0's product done, row 0 published
__device__ unsigned long long g_flow_sub[SLAM_TL_FLOW_MAX_T][8];
// The own column's stamps go to LDS (flow_lds: 0-4 phases, 8-13 sub-stamps)
// and out to global memory at the end, so that no stamp store is pending at
// the phases' own s_waitcnt vmcnt(0).
#define FLOW_LDS(i)                                               \
  do {                                                            \
    if (threadIdx.x == 0) flow_lds[i] = wall_clock64();           \
  } while (0)
#define FLOW_S(i) FLOW_LDS(8 + (i))
#define FLOW_T(i) FLOW_LDS(i)
#define FLOW_FLUSH()                                                             \
  do {                                                                           \
    if (threadIdx.x == 0) {                                                      \
      for (int i_ = 0; i_ < 5; ++i_) g_flow_stamp[J][i_] = flow_lds[i_];         \
      for (int i_ = 0; i_ < 6; ++i_) g_flow_sub[J][i_] = flow_lds[8 + i_];       \
      g_flow_sub[J][6] = flow_lds[5];                                            \
      g_flow_sub[J][7] = flow_lds[6];                                            \
    }                                                                            \
  } while (0)
#else
#define FLOW_TC(col, i) (void)0
#define FLOW_S(i) (void)0
#define FLOW_T(i) (void)0
#define FLOW_FLUSH() (void)0
#endif

struct FlowPtrs {
  int *tile, *yf, *xf, *ticket, *epoch, *start, *fail, *cnt, *dv, *pf;
  __device__ FlowPtrs(const slam_ba_problem& p, const TlLayout& L) {
    int* base = reinterpret_cast<int*>(p.chol + L.flow);
    tile = base;
    yf = base + L.T * L.T;
    xf = yf + L.T;
    ticket = xf + L.T;
    epoch = ticket + 1;
    start = ticket + 2;
    fail = ticket + 3;  // k_tl3_flow's epoch-tagged fail word
    cnt = ticket + 8;
    dv = cnt + L.T;
    pf = reinterpret_cast<int*>(p.chol + L.prod(p.tl_sched[11]));  // product slot flags
  }
};

__device__ __forceinline__ int ld_flag(const int* f) {
  return __hip_atomic_load(const_cast<int*>(f), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_flag(int* f, int v) {
  __hip_atomic_store(f, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// The dataflow solve's fail word carries its solve: (epoch << 2) | code, code
// 1 a non-SPD tile, 2 a timed-out wait -- so no launch has to clear it
__device__ __forceinline__ int flow_fcode(const int* fail, int epoch) {
  const int v = ld_flag(fail);
  return (v >> 2) == epoch ? (v & 3) : 0;
}
__device__ __forceinline__ void flow_fail(int* fail, int epoch, int code) { st_flag(fail, (epoch << 2) | code); }

// Thread 0 polls until *flag == epoch; false (uniform) when the solve failed or
// the wait timed out (which marks it failed).
__device__ bool flow_wait(const int* flag, int epoch, int* fail, int* sh) {
  if (threadIdx.x == 0) {
    int ok = 1;
    for (int spins = 0; ld_flag(flag) != epoch; ++spins) {
      if (flow_fcode(fail, epoch) != 0) {
        ok = 0;
        break;
      }
      if (spins > kFlowSpinMax) {
        flow_fail(fail, epoch, 2);
        ok = 0;
        break;
      }
      __builtin_amdgcn_s_sleep(SLAM_FLOW_SLEEP);
    }
    *sh = ok;
  }
  __syncthreads();
  const bool ok = *sh != 0;
  __syncthreads();
  return ok;
}

// Wave 0 polls base[idx[i]] == epoch for all i < cnt together (lane i, chunks
// of 64), so flags that are already up cost one round trip, not cnt.
__device__ bool flow_wait_many(const int* base, const int32_t* idx, int cnt, int epoch, int* fail,
                               int* sh) {
  if (threadIdx.x < 64) {
    const int lane = threadIdx.x;
    int ok = 1;
    for (int c0 = 0; c0 < cnt && ok; c0 += 64) {
      const int* f = c0 + lane < cnt ? base + idx[c0 + lane] : nullptr;
      for (int spins = 0;; ++spins) {
        const bool up = f == nullptr || ld_flag(f) == epoch;
        if (__all(up)) break;
        if (flow_fcode(fail, epoch) != 0) {
          ok = 0;
          break;
        }
        if (spins > kFlowSpinMax) {
          if (lane == 0) flow_fail(fail, epoch, 2);
          ok = 0;
          break;
        }
        __builtin_amdgcn_s_sleep(SLAM_FLOW_SLEEP);
      }
    }
    if (lane == 0) *sh = ok;
  }
  __syncthreads();
  const bool ok = *sh != 0;
  __syncthreads();
  return ok;
}

// one flag, the same contract as flow_wait (its definition follows below)
__device__ bool flow_wait(const int* flag, int epoch, int* fail, int* sh);
__device__ __forceinline__ bool flow_wait_one(const int* flag, int epoch, int* fail, int* sh) {
  return flow_wait(flag, epoch, fail, sh);
}

// Thread 0 polls the parent counter of column J until its low half (retired row
// tiles) reaches rc -- the retirers' x stores drained before their adds (the
// counter is the acquire for those bytes); false (uniform) when the solve failed
// or the wait timed out.
__device__ bool flow_wait_count(const int* cnt, int rc, int epoch, int* fail, int* sh) {
  if (threadIdx.x == 0) {
    int ok = 1;
    for (int spins = 0; (ld_flag(cnt) & 0xffff) < rc; ++spins) {
      if (flow_fcode(fail, epoch) != 0) {
        ok = 0;
        break;
      }
      if (spins > kFlowSpinMax) {
        flow_fail(fail, epoch, 2);
        ok = 0;
        break;
      }
      __builtin_amdgcn_s_sleep(SLAM_FLOW_SLEEP);
    }
    *sh = ok;
  }
  __syncthreads();
  const bool ok = *sh != 0;
  __syncthreads();
  return ok;
}

// every thread's (sc1) stores drained, then thread 0 raises the flag
__device__ __forceinline__ void flow_publish(int* flag, int epoch) {
  __builtin_amdgcn_s_waitcnt(0);
  __syncthreads();
  if (threadIdx.x == 0) st_flag(flag, epoch);
}

// tile_to_frag through sc1 loads (the tile was written by another workgroup)
__device__ __forceinline__ void tile_to_frag_sc1(const double* __restrict__ g, int ld, double* f) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int r = lane & 15, c = lane >> 4;
  double tmp[16];
#pragma unroll
  for (int q = 0; q < 16; ++q) {
    const int fi = w + 4 * q;
    tmp[q] = ld_sc1(g + (size_t)(16 * (fi >> 4) + r) * ld + 4 * (fi & 15) + c);
  }
#pragma unroll
  for (int q = 0; q < 16; ++q) f[((w + 4 * q) << 6) + lane] = tmp[q];
}

// two tiles through sc1 loads, all 32 loads of a lane in flight before the LDS stores
__device__ __forceinline__ void tiles2_to_frag_sc1(const double* __restrict__ g0, const double* __restrict__ g1,
                                                   int ld, double* f0, double* f1) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int r = lane & 15, c = lane >> 4;
  double t0[16], t1[16];
#pragma unroll
  for (int q = 0; q < 16; ++q) {
    const int fi = w + 4 * q;
    const size_t o = (size_t)(16 * (fi >> 4) + r) * ld + 4 * (fi & 15) + c;
    t0[q] = ld_sc1(g0 + o);
    t1[q] = ld_sc1(g1 + o);
  }
#pragma unroll
  for (int q = 0; q < 16; ++q) {
    f0[((w + 4 * q) << 6) + lane] = t0[q];
    f1[((w + 4 * q) << 6) + lane] = t1[q];
  }
}

// acc[s] += (rows 16w.., cols 16s.. of X Y^T), X and Y in fragment order, over
// the first nbk 16-column blocks of k (the columns of a child tile past its
// camera rows' blocks are exact zeros in both operands)
__device__ __forceinline__ void gemm_xyT_acc(const double* Xf, const double* Yf, d4 acc[4],
                                             int nbk = 4) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
#if SLAM_TL_KSKIP
  for (int kb = 0; kb < nbk; ++kb) {
#pragma unroll
    for (int k4 = 0; k4 < 4; ++k4) {
      const int kk = 4 * kb + k4;
#else
  (void)nbk;
  {
#pragma unroll 4
    for (int kk = 0; kk < 16; ++kk) {
#endif
      const double a = Xf[((w * 16 + kk) << 6) + lane];
#pragma unroll
      for (int s = 0; s < 4; ++s)
        acc[s] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, Yf[((s * 16 + kk) << 6) + lane], acc[s], 0, 0, 0);
    }
  }
}

// Elements of the damped tiled system gathered straight from the packed S
// (what k_tl2_load + k_tl2_scatter lay out for the level-scheduled solve),
// through the schedule's per-column gather tables (ba.tl_schedule): gt = the
// tile's [64][64] packed-S offsets (-1 zero, -2 a padding row's unit
// diagonal).  Two rounds of independent loads for all N elements (offsets,
// then values); dg: the diagonal tile's rows of S, for lambda clamp(diag U) on
// its diagonal (null for a row tile).
template <int N>
__device__ __forceinline__ void tl_gather(const double* __restrict__ sys, const int32_t* gt,
                                          const int32_t* dg, const double* dU, double lam,
                                          const int (&ri)[N], const int (&ci)[N], double* out) {
  int g[N], r[N];
#pragma unroll
  for (int i = 0; i < N; ++i) {
    g[i] = gt[ri[i] * kTB + ci[i]];
    r[i] = dg != nullptr && ri[i] == ci[i] ? dg[ri[i]] : -1;
  }
  double v[N], d[N];
#pragma unroll
  for (int i = 0; i < N; ++i) {
    v[i] = sys[max(g[i], 0)];
    d[i] = r[i] >= 0 ? dU[r[i]] : 0.0;
  }
#pragma unroll
  for (int i = 0; i < N; ++i) {
    double x = g[i] >= 0 ? v[i] : (g[i] == -2 ? 1.0 : 0.0);
    if (r[i] >= 0) x += lam * clampd(d[i]);
    out[i] = x;
  }
}

// lower 16x16 blocks (row, column) of the diagonal update per wave of k_tl3_flow
__constant__ int kDiagBlk[4][3][2] = {{{0, 0}, {3, 0}, {3, 1}}, {{1, 0}, {1, 1}, {3, 2}},
                                      {{2, 0}, {2, 1}, {2, 0}}, {{2, 2}, {3, 3}, {2, 2}}};

__global__ __launch_bounds__(kTlWG) __attribute__((amdgpu_waves_per_eu(1, 1)))
void k_tl3_flow(slam_ba_problem p, int T_) {
  lm_wave_priority();
  const int n = 9 * p.n_cams;
  const TlLayout L(n, T_);
  const int32_t* S = p.tl_sched;
  const int T = L.T;
  const FlowPtrs F(p, L);
  __shared__ double VX[2 * kTB * kTB];  // factor scratch; then L_JJ^-1 (fragments) | operand Y
  __shared__ double Xf[kTB * kTB];      // operand X
  __shared__ double part[4][kTB];
  __shared__ double yv[kTB];
  __shared__ double rv[kTB];
  __shared__ int shf, okf, col_sh, ep_sh;
  __shared__ double VR[kTB * kVR];        // L_JJ^-1 row-major (stride 65): (3), this column's x
  __shared__ int stk[SLAM_TL_FLOW_MAX_T], sp_sh, cur_sh, last_sh, own_sh;
#ifdef SLAM_FLOW_PROFILE
  __shared__ unsigned long long flow_lds[16];
#endif
  // the column: the start ticket hands them out in the order the workgroups
  // start.  The ticket is never reset: every solve takes exactly T tickets, so
  // ticket v is column v mod T of solve v / T, whose number is the epoch that
  // every flag of this solve carries (no clearing launch before the solve)
  if (threadIdx.x == 0) {
    const unsigned v = ticket_add(reinterpret_cast<uint32_t*>(F.start));
    col_sh = (int)(v % (unsigned)T);
    ep_sh = (int)(v / (unsigned)T) + 1;
  }
  __syncthreads();
  const int J = col_sh;
  const int epoch = ep_sh;
  const int32_t* rec = S + S[5] + 5 * J;
  const int ro = rec[0], rc = rec[1], so = rec[2], sc = rec[3], uo = rec[4];
  // rows of a tile (its rows of S first, padding after them): the 16-row
  // blocks of the factor and of the products over its columns
  const int32_t* trows = tl_tile_rows(S, n, T);
  auto nblk = [&](int k) { return (trows[k] + 15) >> 4; };
  const int nbJ = nblk(J);
  // Product tasks (ba.tl_schedule): the terms L_Ik L_Jk^T of a column J's rows
  // 0 and 1 are formed by column k itself, as soon as both of its tiles exist,
  // into slots that J sums after its factor -- J's diagonal phase never waits
  // for a child's later row tiles, which its children publish after the L_Jk
  // that phase needs.  This column's tasks (a, b, slot), ordered by b.
  const int32_t* tkJ = S + S[S[10] + 2 * J];
  const int n_tk = S[S[10] + 2 * J + 1];
  double* prod = p.chol + L.prod(0);
  // (4b)'s inputs for the cameras this column owns, loaded before any wait:
  // thread t < 9 e_cnt takes row t % 9 of owned camera t / 9
  const double* bvec = p.sys + sys_vec_off(p.n_cams, p.n_blocks);  // b | g | diag U | cost
  const int cur = cur_of(p.state);
  const double lam = p.state[SLAM_BA_ST_LAMBDA];
  const int32_t* erJ = S + S[7] + 2 * J;
  const int e_off = erJ[0], e_cnt = erJ[1];
  int e_row = 0, e_rn = 0;
  double e_cam = 0.0, e_du = 0.0, e_g = 0.0, e_cost = 0.0;
  if (threadIdx.x < 9 * e_cnt) {
    e_row = 9 * S[e_off + threadIdx.x / 9] + threadIdx.x % 9;
    e_rn = tl_new_row(S, e_row);
    e_cam = p.cams[cur][e_row];
    e_g = bvec[n + e_row];
    e_du = bvec[2 * n + e_row];
  }
  if (threadIdx.x < e_cnt) e_cost = bvec[3 * n + S[e_off + threadIdx.x]];
  const int own_orow = threadIdx.x < kTB ? tl_old_row(S, n, J * kTB + threadIdx.x) : -1;
  const double b_own = own_orow >= 0 ? bvec[own_orow] : 0.0;  // b_J in the tiled order (3)
  int* fail = F.fail;
  // this column's parent counter, re-armed before any tile of J is published:
  // no row tile of J can retire before J's tiles exist (x_I needs L_IJ)
  if (threadIdx.x == 0) st_flag(F.cnt + J, 0);
  // this column's gather tables: its diagonal tile, row tile q at 1 + q, the
  // diagonal tile's rows of S after them
  const int32_t* gtJ = S + S[S[9] + J];
  const int32_t* dgJ = gtJ + (1 + rc) * kTB * kTB;
  const double* dU = bvec + 2 * n;
  double* A = p.chol + L.a;
  double* Vf = VX;
  double* Yf = VX + kTB * kTB;
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  bool ok = true;
  FLOW_T(0);
  // The diagonal update is symmetric and the factor reads only lower blocks:
  // the 10 lower 16x16 blocks, three per wave (waves 2 and 3 repeat one block
  // they do not store), so each SIMD's MFMA chain per child tile is 48 steps
  // instead of 64.
  int dR[3], dC[3];
#pragma unroll
  for (int b = 0; b < 3; ++b) {
    dR[b] = kDiagBlk[w][b][0];
    dC[b] = kDiagBlk[w][b][1];
  }
  const int dnb = w < 2 ? 3 : 2;
  // A_JJ's blocks, gathered from the packed system into registers before any
  // wait (no load / scatter launch before the solve)
  double ajj[12];
  {
    int gi[12], gj[12];
#pragma unroll
    for (int b = 0; b < 3; ++b)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        gi[4 * b + r] = dR[b] * 16 + (lane >> 4) + 4 * r;
        gj[4 * b + r] = dC[b] * 16 + (lane & 15);
      }
    tl_gather<12>(p.sys, gtJ, dgJ, dU, lam, gi, gj, ajj);
  }
  // ... and the first two row tiles' A_IJ
  double air[2][16];
#pragma unroll
  for (int q = 0; q < 2; ++q) {
    int gi[16], gj[16];
#pragma unroll
    for (int s2 = 0; s2 < 4; ++s2)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        gi[4 * s2 + r] = w * 16 + (lane >> 4) + 4 * r;
        gj[4 * s2 + r] = s2 * 16 + (lane & 15);
      }
    tl_gather<16>(p.sys, gtJ + (q < rc ? 1 + q : 0) * kTB * kTB, nullptr, dU, lam, gi, gj, air[q]);
  }
  // (1) diagonal tile, child tiles k in rs order: L_Jk operands double-buffered
  // (Xf / VX[4096:]); the next child's tile is fetched before this one's MFMAs
  // when its flag is already up (loads in flight under the MFMAs), after them
  // otherwise (a child that is not ready yet never holds up the MFMAs of the
  // ones that are).  Row tiles 0 and 1 take their updates from the product
  // slots after the factor (2).
  d4 acc[4];
#pragma unroll
  for (int s2 = 0; s2 < 4; ++s2) acc[s2] = d4{0.0, 0.0, 0.0, 0.0};
  // The buffers alternate so that the LAST child's L_Jk lands in Xf.
  if (sc > 0) {
    ok = flow_wait(F.tile + J * T + S[so], epoch, fail, &shf);
    if (ok) tile_to_frag_sc1(A + (size_t)J * kTB * L.N + S[so] * kTB, L.N, ((sc - 1) & 1) ? Yf : Xf);
    FLOW_S(0);
  }
  for (int q = 0; q < sc && ok; ++q) {
    double* cur = ((sc - 1 - q) & 1) ? Yf : Xf;
    double* nxt = ((sc - 1 - q) & 1) ? Xf : Yf;
    __syncthreads();  // cur filled; the previous MFMAs' reads of nxt done
    if (q == sc - 1) FLOW_S(1);
    bool pre = false;
    if (q + 1 < sc) {
      if (t == 0) shf = ld_flag(F.tile + J * T + S[so + q + 1]) == epoch ? 1 : 0;
      __syncthreads();
      pre = shf != 0;
      __syncthreads();
      if (pre) tile_to_frag_sc1(A + (size_t)J * kTB * L.N + S[so + q + 1] * kTB, L.N, nxt);
    }
#if SLAM_TL_KSKIP
    const int kmk = nblk(S[so + q]);  // child k's column blocks past its rows: zeros
    for (int kb = 0; kb < kmk; ++kb)
#pragma unroll
      for (int k4 = 0; k4 < 4; ++k4)
#pragma unroll
        for (int b = 0; b < 3; ++b) {
          const int kk = 4 * kb + k4;
          acc[b] = __builtin_amdgcn_mfma_f64_16x16x4f64(cur[((dR[b] * 16 + kk) << 6) + lane],
                                                        cur[((dC[b] * 16 + kk) << 6) + lane], acc[b], 0, 0, 0);
        }
#else
#pragma unroll 4
    for (int kk = 0; kk < 16; ++kk)
#pragma unroll
      for (int b = 0; b < 3; ++b)
        acc[b] = __builtin_amdgcn_mfma_f64_16x16x4f64(cur[((dR[b] * 16 + kk) << 6) + lane],
                                                      cur[((dC[b] * 16 + kk) << 6) + lane], acc[b], 0, 0, 0);
#endif
    if (q + 1 < sc) {
      if (!pre) {
        ok = flow_wait(F.tile + J * T + S[so + q + 1], epoch, fail, &shf);
        if (ok) tile_to_frag_sc1(A + (size_t)J * kTB * L.N + S[so + q + 1] * kTB, L.N, nxt);
      }
    }
  }
  __syncthreads();
  FLOW_T(1);
  if (ok) {
    double* M = VX;  // lower blocks only (tile_chol_inv_blk reads no others)
#pragma unroll
    for (int b = 0; b < 3; ++b)
      if (b < dnb) {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int row = dR[b] * 16 + (lane >> 4) + 4 * r, col = dC[b] * 16 + (lane & 15);
          M[row * kMS + col] = ajj[4 * b + r] - acc[b][r];
        }
      }
    double* Xb = VX + kTB * kMS;
    ok = tile_chol_inv_blk(nullptr, 0, M, Xb, Xb + 10 * 16 * kBS17, &okf, nbJ);
    // L_JJ^-1 out of the block store into (swizzled) fragment order (Vf) and
    // row-major (VR): wave w takes rows [16w, 16w + 16), lane = column
    double x[16];
    if (ok) {
      const int cb16 = lane >> 4;
#pragma unroll
      for (int m = 0; m < 16; ++m)
        x[m] = w >= cb16 ? Xb[blk_id(w, cb16) * 16 * kBS17 + m * kBS17 + (lane & 15)] : 0.0;
    }
    __syncthreads();  // VX is reused below
    if (!ok) {
      if (t == 0) flow_fail(fail, epoch, 1);
    } else {
#pragma unroll
      for (int m = 0; m < 16; ++m) {
        Vf[frag_swz(16 * w + m, lane)] = x[m];
        VR[(16 * w + m) * kVR + lane] = x[m];
      }
    }
    __syncthreads();
  }
  FLOW_T(2);
  // (2) row tiles, parent first.  Rows 0 and 1 (the children folded in during
  // (1), A_IJ in registers) and the rest are separate straight-line instances:
  // one uniform branch per row tile, not one per element (this code runs once
  // per solve on a CU whose instruction cache the LM kernels have refilled, so
  // every taken branch into cold code costs an L2 fetch).
  double l0[16];  // L_{rows[0]} J, kept for this column's product tasks with a = 0
  auto row_tile = [&](auto QC, int q) {
    constexpr int qc = decltype(QC)::value;  // 0, 1: rows 0 / 1; 2: any later row
    const int I = S[ro + q];
    const int ko = S[uo + 2 * q], kc = S[uo + 2 * q + 1];
#pragma unroll
    for (int s2 = 0; s2 < 4; ++s2) acc[s2] = d4{0.0, 0.0, 0.0, 0.0};
    // Rows 0 and 1: the k list's product slots (after the list), summed in list
    // order, each a 64x64 term in the accumulator layout; the staged A_IJ goes
    // to Yf.  Later rows load both tiles (loads in flight together), MFMA the
    // term here and stage into Xf.
    double* stg = qc < 2 ? Yf : Xf;
    if constexpr (qc < 2) {
      if (kc > 0) ok = flow_wait_many(F.pf, S + ko + kc, kc, epoch, fail, &shf);
#ifdef SLAM_FLOW_PROFILE
      if (q == 0) FLOW_LDS(5);
#endif
      for (int u0 = 0; u0 < kc && ok; u0 += 2) {
        double cv[2][16];
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const double* Cp = prod + (size_t)S[ko + kc + min(u0 + h, kc - 1)] * kTB * kTB;
#pragma unroll
          for (int e = 0; e < 16; ++e) cv[h][e] = ld_sc1(Cp + ((4 * w + (e >> 2)) * 4 + (e & 3)) * 64 + lane);
        }
#pragma unroll
        for (int h = 0; h < 2; ++h)
          if (u0 + h < kc) {
#pragma unroll
            for (int s2 = 0; s2 < 4; ++s2)
#pragma unroll
              for (int r = 0; r < 4; ++r) acc[s2][r] += cv[h][4 * s2 + r];
          }
      }
#ifdef SLAM_FLOW_PROFILE
      if (q == 0) FLOW_LDS(6);
#endif
    } else {
      for (int u = 0; u < kc && ok; ++u) {
        const int k = S[ko + u];
        ok = flow_wait(F.tile + I * T + k, epoch, fail, &shf);  // (J, k) was waited for in (1)
        if (!ok) break;
        tiles2_to_frag_sc1(A + (size_t)I * kTB * L.N + k * kTB, A + (size_t)J * kTB * L.N + k * kTB, L.N,
                           Yf, Xf);
        __syncthreads();
        gemm_xyT_acc(Yf, Xf, acc, nblk(k));
        __syncthreads();
      }
    }
    if (!ok) return;
    if (q == 0) FLOW_S(2);
    double* AIJ = A + (size_t)I * kTB * L.N + J * kTB;
    double a[16];
    if constexpr (qc < 2) {
#pragma unroll
      for (int e = 0; e < 16; ++e) a[e] = air[qc][e];
    } else {
      int gi[16], gj[16];
#pragma unroll
      for (int s2 = 0; s2 < 4; ++s2)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          gi[4 * s2 + r] = w * 16 + (lane >> 4) + 4 * r;
          gj[4 * s2 + r] = s2 * 16 + (lane & 15);
        }
      tl_gather<16>(p.sys, gtJ + (1 + q) * kTB * kTB, nullptr, dU, lam, gi, gj, a);
    }
#pragma unroll
    for (int s2 = 0; s2 < 4; ++s2)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = w * 16 + (lane >> 4) + 4 * r, col = s2 * 16 + (lane & 15);
        stg[frag_swz(row, col)] = a[4 * s2 + r] - acc[s2][r];
      }
    __syncthreads();
    if (q == 0) FLOW_S(3);
    d4 lacc[4];
    gemm_xyT_lowY_swz(stg, Vf, lacc, 4 * nbJ);  // L_IJ = A_IJ (L_JJ^-1)^T
#ifdef SLAM_FLOW_PROFILE
    if (q == 0) {
      __builtin_amdgcn_s_waitcnt(0);
      FLOW_S(4);
    }
#endif
#pragma unroll
    for (int s2 = 0; s2 < 4; ++s2)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = w * 16 + (lane >> 4) + 4 * r, col = s2 * 16 + (lane & 15);
        st_sc1(AIJ + (size_t)row * L.N + col, lacc[s2][r]);
      }
    flow_publish(F.tile + I * T + J, epoch);
    if (q == 0) FLOW_S(5);
    if (q == 0) {
#pragma unroll
      for (int s2 = 0; s2 < 4; ++s2)
#pragma unroll
        for (int r = 0; r < 4; ++r) l0[4 * s2 + r] = lacc[s2][r];
    }
    // this column's product tasks with b = q: L_IJ (this row tile, X operand)
    // times L_{rows[a]} J^T (row 0 from registers, others reloaded), into the
    // slot; the publish's barrier ended every read of Xf / Yf
    bool xs = false;
    for (int e = 0; e < n_tk; ++e) {
      if (tkJ[3 * e + 1] != q) continue;  // (uniform)
      const int ta = tkJ[3 * e], slot = tkJ[3 * e + 2];
      if (!xs) {
#pragma unroll
        for (int s2 = 0; s2 < 4; ++s2)
#pragma unroll
          for (int r = 0; r < 4; ++r)
            Xf[frag_idx(w * 16 + (lane >> 4) + 4 * r, s2 * 16 + (lane & 15))] = lacc[s2][r];
        xs = true;
      }
      if (ta == 0) {
#pragma unroll
        for (int s2 = 0; s2 < 4; ++s2)
#pragma unroll
          for (int r = 0; r < 4; ++r)
            Yf[frag_idx(w * 16 + (lane >> 4) + 4 * r, s2 * 16 + (lane & 15))] = l0[4 * s2 + r];
      } else {
        tile_to_frag_sc1(A + (size_t)S[ro + ta] * kTB * L.N + J * kTB, L.N, Yf);
      }
      __syncthreads();
      d4 pacc[4];
#pragma unroll
      for (int s2 = 0; s2 < 4; ++s2) pacc[s2] = d4{0.0, 0.0, 0.0, 0.0};
      gemm_xyT_acc(Xf, Yf, pacc, nbJ);
      double* Cp = prod + (size_t)slot * kTB * kTB;
#pragma unroll
      for (int s2 = 0; s2 < 4; ++s2)
#pragma unroll
        for (int r = 0; r < 4; ++r) st_sc1(Cp + ((4 * w + s2) * 4 + r) * 64 + lane, pacc[s2][r]);
      flow_publish(F.pf + slot, epoch);  // (its barrier also ends this task's Yf reads)
    }
  };
  if (ok && rc > 0) row_tile(std::integral_constant<int, 0>{}, 0);
  if (ok && rc > 1) row_tile(std::integral_constant<int, 1>{}, 1);
  for (int q = 2; q < rc && ok; ++q) row_tile(std::integral_constant<int, 2>{}, q);
  FLOW_T(3);
  // (3) forward substitution: r = b_J - sum_{k in rs(J)} L_Jk y_k, the terms
  // pushed by the children (fc[J][k]); y_J = L_JJ^-1 r; then this column's
  // own terms L_IJ y_J for its rows I (fc[I][J]), published with the y flag
  if (ok) ok = flow_wait_many(F.yf, S + so, sc, epoch, fail, &shf);
  if (ok) {
    if (t < kTB) {
      double r = b_own;
      for (int q0 = 0; q0 < sc; q0 += 16) {
        double v[16];
#pragma unroll
        for (int u = 0; u < 16; ++u)
          v[u] = q0 + u < sc ? ld_sc1(p.chol + L.fc + ((size_t)J * T + S[so + q0 + u]) * kTB + t) : 0.0;
#pragma unroll
        for (int u = 0; u < 16; ++u)
          if (q0 + u < sc) r -= v[u];
      }
      rv[t] = r;
    }
    __syncthreads();
    // y_J[m] = sum_c L_JJ^-1[m][c] r[c]: thread (w, m) sums c in [16w, 16w + 16)
    double s3 = 0.0;
    for (int c = 16 * w; c < 16 * w + 16; ++c) s3 = __builtin_fma(VR[lane * kVR + c], rv[c], s3);
    part[w][lane] = s3;
    __syncthreads();
    if (t < kTB) yv[t] = ((part[0][t] + part[1][t]) + part[2][t]) + part[3][t];
    __syncthreads();
    for (int q = 0; q < rc; ++q) {
      const int I = S[ro + q];
      const double* LIJ = A + (size_t)(I * kTB + lane) * L.N + J * kTB + 16 * w;
      double la[16];
#pragma unroll
      for (int c = 0; c < 16; ++c) la[c] = ld_sc1(LIJ + c);
      double s4 = 0.0;
#pragma unroll
      for (int c = 0; c < 16; ++c) s4 = __builtin_fma(la[c], yv[16 * w + c], s4);
      part[w][lane] = s4;
      __syncthreads();
      if (t < kTB)
        st_sc1(p.chol + L.fc + ((size_t)I * T + J) * kTB + t,
               ((part[0][t] + part[1][t]) + part[2][t]) + part[3][t]);
      __syncthreads();
    }
    flow_publish(F.yf + J, epoch);
  }
  FLOW_T(4);
  // (4) back substitution: x_k = L_kk^-T (y_k - sum_I L_Ik^T x_I) over the row
  // tiles I of column k (thread (w, c = lane) sums rows [16w, 16w + 16) of every
  // I in row order; the operations and their order do not depend on which
  // workgroup forms x_k).  Who forms x_J:
  //   a root (no row tiles): this workgroup, right away;
  //   otherwise, once every workgroup of the grid has started (the start ticket
  //   reached T: waiting can then hold up no one), this workgroup registers as
  //   the waiter on cnt[J] (+2^16) and forms x_J when its row tiles' x are all
  //   retired -- unless the last of them was retired before it registered;
  //   else the workgroup that retires the last row tile of J (cnt[J] reaches
  //   rows(J) with no waiter registered) pushes J on its own stack.
  // So the columns run in parallel when the grid is resident, and a column whose
  // workgroup cannot wait is still formed.  Every column is retired once: x
  // flag, its children's counters, the retire ticket.
  if (t == 0) {
    sp_sh = 0;
    last_sh = 0;
    own_sh = 0;
    if (rc == 0) {
      own_sh = 1;
    } else if (ld_flag(F.start) >= epoch * T) {  // every workgroup of this solve has started
      const unsigned old = __hip_atomic_fetch_add(reinterpret_cast<unsigned*>(F.cnt + J), 1u << 16,
                                                  __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      own_sh = (int)(old & 0xffffu) < rc ? 2 : 0;
    }
  }
  __syncthreads();
  if (!own_sh) {
    // another workgroup forms x_J: L_JJ^-1 and y_J for it, published by dv[J]
    double* V = p.chol + L.dinv + (size_t)J * kTB * kTB;
    for (int e = t; e < kTB * kTB; e += kTlWG) st_sc1(V + e, VR[(e >> 6) * kVR + (e & 63)]);
    if (t < kTB) st_sc1(p.chol + L.y + J * kTB + t, yv[t]);
    flow_publish(F.dv + J, epoch);
  }
  // the own column's first two L_IJ in flight before its wait (they are this
  // workgroup's own stores of (2)): only x_I is loaded after the counter
  double la_pre[2][16];
  if (own_sh == 2) {
#pragma unroll
    for (int q = 0; q < 2; ++q)
      if (q < rc) {
        const double* LIk = A + (size_t)(S[ro + q] * kTB + 16 * w) * L.N + J * kTB + lane;
#pragma unroll
        for (int m = 0; m < 16; ++m) la_pre[q][m] = ld_sc1(LIk + (size_t)m * L.N);
      }
  }
  for (int it = 0;; ++it) {
    int k;
    bool okk;
    if (it == 0) {  // this workgroup's own column, when it forms it
      if (!own_sh) continue;
      k = J;
      okk = ok && (own_sh == 1 || flow_wait_count(F.cnt + J, rc, epoch, fail, &shf));
    } else {
      if (t == 0) cur_sh = sp_sh > 0 ? stk[--sp_sh] : -1;
      __syncthreads();
      k = cur_sh;
      if (k < 0) break;
      okk = flow_wait_one(F.dv + k, epoch, fail, &shf);
    }
    const bool own = k == J;
    const int32_t* rk = S + S[5] + 5 * k;
    const int kro = rk[0], krc = rk[1], kso = rk[2], ksc = rk[3];
    // x_k's rows in camera order: loaded before the waits below, off the chain
    const int orow = own ? own_orow : (t < kTB ? tl_old_row(S, n, k * kTB + t) : -1);
    if (okk) {
      if (!own && t < kTB) yv[t] = ld_sc1(p.chol + L.y + k * kTB + t);
      double s2 = 0.0;
      for (int q = 0; q < krc; ++q) {
        const int I = S[kro + q];
        const double* LIk = A + (size_t)(I * kTB + 16 * w) * L.N + k * kTB + lane;
        const double* xI = p.chol + L.x + I * kTB + 16 * w;
        double la[16], xa[16];
        const bool pre = it == 0 && own_sh == 2 && q < 2;  // (uniform)
#pragma unroll
        for (int m = 0; m < 16; ++m) {
          la[m] = pre ? (q == 0 ? la_pre[0][m] : la_pre[1][m]) : ld_sc1(LIk + (size_t)m * L.N);
          xa[m] = ld_sc1(xI + m);
        }
#pragma unroll
        for (int m = 0; m < 16; ++m) s2 = __builtin_fma(la[m], xa[m], s2);
      }
      FLOW_TC(k, 5);
      part[w][lane] = s2;
      __syncthreads();
      if (t < kTB) rv[t] = yv[t] - (((part[0][t] + part[1][t]) + part[2][t]) + part[3][t]);
      __syncthreads();
      double s3 = 0.0;  // x_k[c] = sum_m L_kk^-1[m][c] r[m]
      if (own) {
        for (int m = 16 * w; m < 16 * w + 16; ++m) s3 = __builtin_fma(VR[m * kVR + lane], rv[m], s3);
      } else {
        const double* Vk = p.chol + L.dinv + (size_t)k * kTB * kTB;
        for (int m = 16 * w; m < 16 * w + 16; ++m) s3 = __builtin_fma(ld_sc1(Vk + m * kTB + lane), rv[m], s3);
      }
      __syncthreads();  // rv / part reads done before part is rewritten
      part[w][lane] = s3;
      __syncthreads();
      if (t < kTB) {
        const double xv = ((part[0][t] + part[1][t]) + part[2][t]) + part[3][t];
        Xf[t] = xv;  // (4b) (Xf is free after (2))
        st_sc1(p.chol + L.x + k * kTB + t, xv);
        if (orow >= 0) st_sc1(p.chol + L.xo + orow, xv);  // camera order (padding rows dropped)
      }
    }
    // retire column k even when the solve failed (the counters and the ticket
    // still complete; the epilogue sees the fail code)
    flow_publish(F.xf + k, epoch);
    FLOW_TC(k, 6);
    // the parent counters (one lane each) in flight together -- independent,
    // and a chain of returning atomics cost a device round trip each on the
    // back substitution's critical path; the columns this retire completes go
    // on the stack in u order
    if (t < 64) {
      for (int u0 = 0; u0 == 0 || u0 < ksc; u0 += 64) {
        const int u = u0 + t;
        int c = 0, rcc = 0;
        unsigned old = 0;
        if (u < ksc) {
          c = S[kso + u];  // k is a row tile of column c
          rcc = S[S[5] + 5 * c + 1];
          old = ticket_add(reinterpret_cast<uint32_t*>(F.cnt + c));
        }
        const bool push = u < ksc && (int)(old & 0xffffu) == rcc - 1 && (old >> 16) == 0;
        const unsigned long long m = __ballot(push);
        const int base = sp_sh;
        if (push) stk[base + __popcll(m & ((1ull << t) - 1ull))] = c;
        wave_lds_fence();
        if (t == 0) sp_sh = base + __popcll(m);
        wave_lds_fence();
      }
    }
    // (4b) the epilogue of the cameras tile k owns (ba.tl_schedule: those whose
    // lowest tile is k -- every other tile of a camera is a row tile of k, so
    // its x is already out), after the retire so that no child waits on it:
    // delta_c, the trial parameters cams[1-cur] and their projection records,
    // this tile's share of the camera part of the predicted reduction and of
    // the cost (fixed order) into epi[k]; the same operations whichever
    // workgroup forms x_k.  Written through (sc1) and drained before the retire
    // ticket, so that the last retirer's failure path overwrites them safely.
    {
      const bool mine = own && own_sh != 0;
      const int32_t* er = S + S[7] + 2 * k;
      const int eo = mine ? e_off : er[0], ec = mine ? e_cnt : er[1];
      double* ct = Xf + kTB;                  // trial parameters [ec][9]
      double* pv = ct + 9 * kEpiCams;         // pc terms [9 ec]
      double* cv = pv + 9 * kEpiCams;         // cost terms [ec]
      if (t < 9 * ec) {
        int row = e_row, rn = e_rn;
        double cam = e_cam, du = e_du, g = e_g;
        if (!mine) {
          row = 9 * S[eo + t / 9] + t % 9;
          rn = tl_new_row(S, row);
          cam = p.cams[cur][row];
          g = bvec[n + row];
          du = bvec[2 * n + row];
        }
        const double d = (rn >> 6) == k ? Xf[rn & 63] : ld_sc1(p.chol + L.xo + row);
        st_sc1(p.delta_c + row, d);
        const double tr = cam + d;
        st_sc1(p.cams[1 - cur] + row, tr);
        ct[t] = tr;
        pv[t] = d * (lam * clampd(du) * d + g);
      }
      if (t < ec) cv[t] = mine ? e_cost : bvec[3 * n + S[eo + t]];
      __syncthreads();
      if (t < ec) {
        double rec[kCamRec];
        cam_prep(ct + 9 * t, rec);
        double* o = p.camrec[1 - cur] + kCamRec * S[eo + t];
#pragma unroll
        for (int i = 0; i < kCamRec; ++i) st_sc1(o + i, rec[i]);
      }
      if (t == 0) {
        double pc = 0.0, cs = 0.0;
        for (int i = 0; i < 9 * ec; ++i) pc += pv[i];
        for (int q = 0; q < ec; ++q) cs += cv[q];
        st_sc1(p.chol + L.epi + 2 * k, pc);
        st_sc1(p.chol + L.epi + 2 * k + 1, cs);
      }
      __builtin_amdgcn_s_waitcnt(0);
      __syncthreads();
      // (never reset: T retires per solve, the last of each solve is T - 1 mod T)
      if (t == 0 && ticket_add(reinterpret_cast<uint32_t*>(F.ticket)) % (unsigned)T == (unsigned)(T - 1))
        last_sh = 1;
    }
    __syncthreads();
  }
  FLOW_FLUSH();
  // (5) the workgroup that retired the last column (after its epilogue share)
  // sums the per-tile partials in tile order; after a failed solve it redoes
  // the whole epilogue with a zero step instead (its plain stores land after
  // the shares' drained write-through stores)
  if (!last_sh) return;
#ifdef SLAM_FLOW_PROFILE
  if (t == 0) g_flow_epi[0] = wall_clock64();
#endif
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
  const int fcode = flow_fcode(fail, epoch);  // 0 ok, 1 non-SPD tile, 2 a wait timed out
  if (fcode != 0) {
    const double* gvec = bvec + n;
    solve_epilogue<true>(p, p.chol + L.xo, false, &part[0][0],
                         EpiSrc{gvec, bvec + 2 * n, p.cams[cur], gvec + 2 * n}, fcode);
  } else if (t < 64) {
    double pc = 0.0, cs = 0.0;  // lane t: tiles t, t + 64, ...; then a fixed shuffle tree
    for (int k = t; k < T; k += 64) {
      pc += ld_sc1(p.chol + L.epi + 2 * k);
      cs += ld_sc1(p.chol + L.epi + 2 * k + 1);
    }
    for (int off = 32; off > 0; off >>= 1) {
      pc += __shfl_down(pc, off, 64);
      cs += __shfl_down(cs, off, 64);
    }
    if (t == 0) {
      p.state[SLAM_BA_ST_COST] = 0.5 * cs;
      p.state[SLAM_BA_ST_PRED_CAM] = 0.5 * pc;
      p.state[SLAM_BA_ST_CHOL_FAIL] = 0.0;
    }
  }
#ifdef SLAM_FLOW_PROFILE
  __builtin_amdgcn_s_waitcnt(0);
  __syncthreads();
  if (t == 0) g_flow_epi[3] = wall_clock64();
#endif
  FLOW_TC(J, 7);
}

// The dataflow solve makes no residency assumption (k_tl3_flow's comment), so it
// runs on any stream, CU-masked or not, beside any other work.  It needs the
// column count within its LDS stack (SLAM_TL_FLOW_MAX_T, < 2^16 for the parent
// counters) and the camera-order x of the epilogue in its LDS scratch;
// otherwise (or with tl_mode "levels") the level-scheduled launches run.
static bool tl_flow_ok(const slam_ba_problem& p, hipStream_t) {
  if (p.tl_mode != 0 || p.tl_sched_host == nullptr || p.tl_sched_host[5] <= 0) return false;
  const TlLayout L(9 * p.n_cams, p.tl_sched_host[1]);
  return L.T <= SLAM_TL_FLOW_MAX_T && 9 * p.n_cams <= 2 * kTB * kTB;
}

// k_tl2_load over the structural tiles when the schedule carries the column table
static void tl_load(const slam_ba_problem& p, hipStream_t s) {
  const int32_t* h = p.tl_sched_host;
  const int T = h[1];
  if (h[5] > 0) {
    int maxrc = 0;
    for (int J = 0; J < T; ++J) maxrc = std::max(maxrc, (int)h[h[5] + 5 * J + 1]);
    k_tl2_load<<<dim3(T, 1 + maxrc), kTlWG, 0, s>>>(p, T, 1);
  } else {
    k_tl2_load<<<T * (T + 1) / 2, kTlWG, 0, s>>>(p, T, 0);
  }
}

// the layout the kernels assume (row maps at fixed offsets after the header,
// every row of S in some tile)
static int tl_check_sched(const slam_ba_problem& p) {
  const int32_t* h = p.tl_sched_host;
  const int n = 9 * p.n_cams, T = h[1];
  SLAM_REQUIRE(T >= (n + kTB - 1) / kTB && h[2] == kTlHdr && h[3] == kTlHdr + n &&
                   h[6] == kTlHdr + n + T * kTB && h[8] > 0 && h[9] > 0 && h[10] > h[9] && h[11] >= 0,
               "slam_ba: tl_sched layout is not ba.tl_schedule's (T %d, offsets %d %d %d for n %d)", T,
               h[2], h[3], h[6], n);
  return SLAM_OK;
}

static int tl_solve_flow(const slam_ba_problem& p, hipStream_t s) {
  const TlLayout L(9 * p.n_cams, p.tl_sched_host[1]);
  if (int rc = tl_check_sched(p)) return rc;
  k_tl3_flow<<<L.T, kTlWG, 0, s>>>(p, L.T);  // gathers its tiles from the packed system itself
  SLAM_LAUNCHED("k_tl3_flow");
  return SLAM_OK;
}

static int tl_solve_levels(const slam_ba_problem& p, hipStream_t s) {
  const TlLayout L(9 * p.n_cams, p.tl_sched_host[1]);
  const int32_t* h = p.tl_sched_host;
  const int nlev = h[0], T = h[1];
  if (int rc = tl_check_sched(p)) return rc;
  const int32_t* tab = h + h[4];
  tl_load(p, s);
  k_tl2_scatter<<<p.n_blocks, 128, 0, s>>>(p, L.T);
  for (int lv = 0; lv < nlev; ++lv) {
    const int32_t* e = tab + 6 * lv;
    if (e[1] > 0) k_tl2_panel<<<e[1], kTlWG, 0, s>>>(p, T, e[0]);
    if (e[3] > 0) k_tl2_update<<<e[3], kTlWG, 0, s>>>(p, T, e[2]);
  }
  for (int lv = nlev - 1; lv >= 0; --lv) {
    const int32_t* e = tab + 6 * lv;
    if (e[5] > 0) k_tl2_back<<<e[5], kTlWG, 0, s>>>(p, T, e[4]);
  }
  k_tl2_unperm<<<T, kTB, 0, s>>>(p, T);
  k_tl2_epilogue<<<1, 1024, 0, s>>>(p, T);
  SLAM_LAUNCHED("k_tl2_*");
  return SLAM_OK;
}

__device__ void lm_decide(double* __restrict__ state, const double* __restrict__ small);

// Back substitution + trial cost, one workgroup per point group:
//   per observation: Jacobian at the live parameters (the one the lineariser
//     used), Jp and r -> LDS, w_o = W_o^T dc = Jp^T (Jc dc_cam(o))   (-> LDS)
//   per point: V, g, diag, V*^-1, e re-derived in the lineariser's operation
//     order (PtSchur: bit-identical to what it used -- no per-point record
//     written by the lineariser and read back here), dp = e - sum_o V*^-1 w_o,
//     trial point x + dp, predicted-reduction term
//   per observation: trial residual at (cams[next], trial point)   (-> |r|^2)
// Workgroup partial sums go to part[g] (cost) and part[G + g] (pred) as sc1
// stores; the last workgroup to finish (agent-scope ticket) sums them in a
// fixed order into small[0..1] and, when DECIDE (single rank), applies the LM
// decision.
template <bool DECIDE>
__global__ __launch_bounds__(kGrp) void k_back_trial(BaBatch bat) {
  BA_PROB_X(bat);
  const int g = bx, G = p.n_grps;
  if (g >= G) return;  // batch: grid.x covers the largest problem (not in the ticket count)
  double* __restrict__ part = p.red_part;
  lm_wave_priority();
  __shared__ double sjp[6][kGrp + 1], sr[2][kGrp + 1], sw[3][kGrp + 1];  // [value][obs]
  __shared__ double snp[kGrp][3];
  __shared__ double red[kGrp / 64];
  __shared__ int last;
  // group extents in one hop (chk_optr = pt_ptr[grp_ptr])
  const int p0 = p.grp_ptr[g], p1 = p.grp_ptr[g + 1];
  const int o0 = p.chk_optr[g], o1 = p.chk_optr[g + 1];
  const int t = threadIdx.x;
  const int o = o0 + t;
  const bool has = o < o1;
  const int cur = cur_of(p.state);
  const bool fail = p.state[SLAM_BA_ST_CHOL_FAIL] != 0.0;
  // the point lanes' inputs, loaded before the observation phase
  const bool ptl = t < p1 - p0;
  double xv[3];
  int kb = 0, ke = 0;
  if (ptl) {
#pragma unroll
    for (int k = 0; k < 3; ++k) xv[k] = p.pts[cur][3 * (p0 + t) + k];
    kb = p.pt_ptr[p0 + t] - o0;
    ke = p.pt_ptr[p0 + t + 1] - o0;
  }
  if (has) {
    double r[2], J[2][12];
    const int pt = p.obs_pt[o];
    reproject_pre<true>(p.camrec[cur] + kCamRec * p.obs_cam[o], p.pts[cur] + 3 * pt,
                        p.obs_q + 2 * o, r, J);
    clamp_rows<true>(r, J);
    const double* dc = p.delta_c + 9 * p.obs_cam[o];
    double w0 = 0.0, w1 = 0.0, w2 = 0.0;
#pragma unroll
    for (int i = 0; i < 9; ++i) {
      const double c = dc[i];
      w0 += (J[0][i] * J[0][9] + J[1][i] * J[1][9]) * c;
      w1 += (J[0][i] * J[0][10] + J[1][i] * J[1][10]) * c;
      w2 += (J[0][i] * J[0][11] + J[1][i] * J[1][11]) * c;
    }
    sw[0][t] = w0;
    sw[1][t] = w1;
    sw[2][t] = w2;
#pragma unroll
    for (int a = 0; a < 2; ++a) {
#pragma unroll
      for (int c = 0; c < 3; ++c) sjp[3 * a + c][t] = J[a][9 + c];
      sr[a][t] = r[a];
    }
  }
  __syncthreads();
  double pred = 0.0;
  if (ptl) {
    const int pt = p0 + t;
    const double lam = p.state[SLAM_BA_ST_LAMBDA];
    PtSchur ps;
    for (int k = kb; k < ke; ++k) {
#pragma unroll
      for (int a = 0; a < 2; ++a) ps.acc(sjp[3 * a][k], sjp[3 * a + 1][k], sjp[3 * a + 2][k], sr[a][k]);
    }
    ps.solve(lam);
    const double* iv = ps.iv;
    double d0 = ps.e[0], d1 = ps.e[1], d2 = ps.e[2];
    for (int k = kb; k < ke; ++k) {
      const double w0 = sw[0][k], w1 = sw[1][k], w2 = sw[2][k];
      d0 -= iv[0] * w0 + iv[1] * w1 + iv[2] * w2;
      d1 -= iv[1] * w0 + iv[3] * w1 + iv[4] * w2;
      d2 -= iv[2] * w0 + iv[4] * w1 + iv[5] * w2;
    }
    const double* x = xv;
    double* xn = p.pts[1 - cur] + 3 * pt;
    snp[t][0] = xn[0] = x[0] + d0;
    snp[t][1] = xn[1] = x[1] + d1;
    snp[t][2] = xn[2] = x[2] + d2;
    pred = d0 * (lam * ps.d[0] * d0 + ps.g0) + d1 * (lam * ps.d[1] * d1 + ps.g1) +
           d2 * (lam * ps.d[2] * d2 + ps.g2);
    if (fail) pred = 0.0;
  }
  __syncthreads();
  double v = 0.0;
  if (has) {
    double r[2], J[2][12];
    reproject_pre<false>(p.camrec[1 - cur] + kCamRec * p.obs_cam[o], snp[p.obs_pt[o] - p0],
                         p.obs_q + 2 * o, r, J);
    clamp_rows<false>(r, J);
    v = r[0] * r[0] + r[1] * r[1];
  }
  v = block_sum(v, red);
  pred = block_sum(pred, red);
  if (t == 0) {
    st_sc1(part + g, v);
    st_sc1(part + G + g, pred);
    __builtin_amdgcn_s_waitcnt(0);  // drained before the ticket
    last = ticket_add(p.ticket) == (unsigned)(G - 1);
  }
  __syncthreads();
  if (!last) return;
  double a = 0.0, b = 0.0;
  for (int i = t; i < G; i += kGrp) {
    a += ld_sc1(part + i);
    b += ld_sc1(part + G + i);
  }
  a = block_sum(a, red);
  b = block_sum(b, red);
  if (t == 0) {
    p.small[0] = a;
    p.small[1] = b;
    ticket_reset(p.ticket);  // re-arm for the next launch
    if (DECIDE) lm_decide(p.state, p.small);
  }
}

__global__ void k_decide(BaBatch bat) {
  BA_PROB(bat);
  if (threadIdx.x == 0) lm_decide(p.state, p.small);
}

__device__ void lm_decide(double* __restrict__ state, const double* __restrict__ small) {
  const double cost = state[SLAM_BA_ST_COST];
  const double cost_new = 0.5 * small[0];
  const double pred = state[SLAM_BA_ST_PRED_CAM] + 0.5 * small[1];
  const bool fail = state[SLAM_BA_ST_CHOL_FAIL] != 0.0;
  const double rho = (!fail && pred > 0.0) ? (cost - cost_new) / pred : -1.0;
  double lam = state[SLAM_BA_ST_LAMBDA], nu = state[SLAM_BA_ST_NU];
  const bool acc = rho > 0.0 && isfinite(cost_new);
  if (acc) {
    const double t = 2.0 * rho - 1.0;
    lam *= fmax(1.0 / 3.0, 1.0 - t * t * t);
    lam = fmin(fmax(lam, kLamMin), kLamMax);
    nu = 2.0;
    state[SLAM_BA_ST_CUR] = state[SLAM_BA_ST_CUR] != 0.0 ? 0.0 : 1.0;
    state[SLAM_BA_ST_COST] = cost_new;
    state[SLAM_BA_ST_NACCEPT] += 1.0;
  } else {
    lam = fmin(lam * nu, kLamMax);
    nu *= 2.0;
  }
  state[SLAM_BA_ST_LAMBDA] = lam;
  state[SLAM_BA_ST_NU] = nu;
  state[SLAM_BA_ST_COST_NEW] = cost_new;
  state[SLAM_BA_ST_PRED] = pred;
  state[SLAM_BA_ST_RHO] = rho;
  state[SLAM_BA_ST_ACCEPTED] = acc ? 1.0 : 0.0;
  state[SLAM_BA_ST_ITERS] += 1.0;
}

__global__ void k_reset(BaBatch bat, double lam0) {
  BA_PROB(bat);
  const int t = threadIdx.x;
  double* state = p.state;
  if (t < SLAM_BA_ST_SLOTS) state[t] = 0.0;
  if (t == 0) {
    state[SLAM_BA_ST_LAMBDA] = lam0;
    state[SLAM_BA_ST_NU] = 2.0;
  }
  for (int c = t; c < p.n_cams; c += blockDim.x) cam_prep(p.cams[0] + 9 * c, p.camrec[0] + kCamRec * c);
}

inline int nblk(int n, int bs) { return (n + bs - 1) / bs; }

int check_problem(const slam_ba_problem* p) {
  SLAM_REQUIRE(p != nullptr, "slam_ba: null problem");
  SLAM_REQUIRE(p->n_cams > 0 && p->n_pts >= 0 && p->n_obs >= 0, "slam_ba: bad sizes");
  SLAM_REQUIRE(p->cams[0] && p->cams[1] && p->camrec[0] && p->camrec[1] &&
                   p->cpart && p->bpart && p->grp_ptr && p->grp_cslot && p->grp_bslot &&
                   p->cslot_obs_ptr && p->bslot_pair_ptr && p->cam_cslot_ptr && p->cslot_row && p->bslot_row &&
                   p->blk_bslot_ptr && p->blocks && p->ticket && p->sys && p->state &&
                   p->small && p->red_part && p->delta_c,
               "slam_ba: null buffer");
  SLAM_REQUIRE(p->n_grps >= 1, "slam_ba: n_grps must be >= 1 (an empty group for P = 0)");
  SLAM_REQUIRE(p->lin_mode == 0 || p->lin_mode == 1, "slam_ba: lin_mode must be 0 or 1");
  SLAM_REQUIRE(p->chk_optr != nullptr, "slam_ba: chk_optr (= pt_ptr[grp_ptr]) required");
  SLAM_REQUIRE(p->lin_mode == 0 || (p->n_sgrps >= 1 && p->sg_ptr && p->sg_meta && p->obs_meta &&
                                     p->chk_cptr && p->bslot_ab),
               "slam_ba: lin_mode 1 needs n_sgrps >= 1 and the supergroup tables");
  SLAM_REQUIRE(sys_packed(p->n_cams) ? (p->n_blocks >= p->n_cams &&
                                        p->n_blocks <= p->n_cams * (p->n_cams + 1) / 2)
                                     : p->n_blocks == p->n_cams * (p->n_cams + 1) / 2,
               "slam_ba: n_blocks must list all C(C+1)/2 upper blocks (9C <= %d) or the "
               "diagonal and every block with common points (packed)", kDenseMaxN);
  SLAM_REQUIRE(!p->tl_sched == !p->tl_sched_host,
               "slam_ba: tl_sched and tl_sched_host come together");
  SLAM_REQUIRE(p->asm_act == nullptr ||
                   (sys_packed(p->n_cams) && p->asm_tab == nullptr && p->n_asm_act >= 1 &&
                    p->n_asm_act <= p->n_blocks),
               "slam_ba: asm_act (n_asm_act %d of %d blocks) needs a packed system without asm_tab",
               p->n_asm_act, p->n_blocks);
  SLAM_REQUIRE(p->tl_mode == 0 || p->tl_mode == 1, "slam_ba: tl_mode must be 0 or 1");
  SLAM_REQUIRE(!sys_packed(p->n_cams) || p->chol != nullptr,
               "slam_ba: chol workspace (slam_ba_chol_len doubles) required for 9C > %d",
               kLdsMaxN);
  SLAM_REQUIRE(!sys_packed(p->n_cams) || p->tl_sched != nullptr,
               "slam_ba: the tile schedule (tl_sched, ba.tl_schedule) is required for 9C > %d",
               kLdsMaxN);
  return SLAM_OK;
}

}  // namespace

extern "C" int slam_ba_red_slots(int n_grps) { return 2 * n_grps; }

extern "C" long long slam_ba_chol_len(int n_cams, const int32_t* tl_sched_host) {
  // tiled factor workspace (9C > kLdsMaxN) for a schedule of tl_sched_host[1]
  // tiles and tl_sched_host[11] product slots; no schedule: the fewest 64-row
  // tiles that hold 9C rows, no slots
  if (n_cams <= 0) return 0;
  const int n = 9 * n_cams;
  if (tl_sched_host == nullptr) return TlLayout(n, (n + kTB - 1) / kTB).total;
  return TlLayout(n, tl_sched_host[1]).with_slots(tl_sched_host[11]);
}

extern "C" long long slam_ba_sys_len(int n_cams, int n_blocks) {
  const long long c9 = 9ll * n_cams;
  return sys_vec_off(n_cams, n_blocks) + 3 * c9 + n_cams;
}

extern "C" int slam_ba_residual(const double* d_cams, const double* d_pts,
                                const int32_t* d_cam_idx, const int32_t* d_pt_idx,
                                const double* d_qs, int n_obs, double* d_resid, void* stream) {
  SLAM_REQUIRE(n_obs >= 0, "slam_ba_residual: n_obs < 0");
  if (n_obs == 0) return SLAM_OK;
  SLAM_REQUIRE(d_cams && d_pts && d_cam_idx && d_pt_idx && d_qs && d_resid,
               "slam_ba_residual: null pointer");
  k_residual<<<nblk(n_obs, kBS), kBS, 0, slam::as_stream(stream)>>>(
      d_cams, d_pts, d_cam_idx, d_pt_idx, d_qs, n_obs, d_resid, nullptr);
  SLAM_LAUNCHED("k_residual");
  return SLAM_OK;
}

extern "C" int slam_ba_jacobian(const double* d_cams, const double* d_pts,
                                const int32_t* d_cam_idx, const int32_t* d_pt_idx,
                                const double* d_qs, int n_obs, double* d_resid, double* d_jac,
                                void* stream) {
  SLAM_REQUIRE(n_obs >= 0, "slam_ba_jacobian: n_obs < 0");
  if (n_obs == 0) return SLAM_OK;
  SLAM_REQUIRE(d_cams && d_pts && d_cam_idx && d_pt_idx && d_qs && d_resid && d_jac,
               "slam_ba_jacobian: null pointer");
  k_residual<<<nblk(n_obs, kBS), kBS, 0, slam::as_stream(stream)>>>(
      d_cams, d_pts, d_cam_idx, d_pt_idx, d_qs, n_obs, d_resid, d_jac);
  SLAM_LAUNCHED("k_residual(jac)");
  return SLAM_OK;
}

namespace {

// Descriptor batch of problems [i0, i0 + n) (n <= kBaMaxBatch) and the launch
// extents that cover the largest of them.
struct Launch {
  BaBatch b;
  int n, max_grps, max_blocks, max_sgrps, mode;
  size_t solve_lds;
  bool dense;
};

// LDS floor of the one-workgroup camera solve (slam_ba_set_solve_lds_floor): a
// floor above what a co-resident ORB workgroup leaves keeps the latency-bound
// pivot chain off CUs whose SIMDs are busy with ORB waves.
static size_t g_solve_lds_floor = 0;

static int make_launch(const slam_ba_problem* probs, int n, Launch* L) {
  SLAM_REQUIRE(n >= 1 && n <= kBaMaxBatch, "slam_ba: batch of %d problems (1..%d)", n, kBaMaxBatch);
  SLAM_REQUIRE(probs != nullptr, "slam_ba: null problem array");
  L->n = n;
  L->max_grps = L->max_blocks = L->max_sgrps = 0;
  L->mode = probs[0].lin_mode;
  L->solve_lds = 0;
  L->dense = true;
  for (int i = 0; i < n; ++i) {
    if (int rc = check_problem(probs + i)) return rc;
    for (int j = 0; j < i; ++j)
      SLAM_REQUIRE(probs[j].state != probs[i].state && probs[j].sys != probs[i].sys,
                   "slam_ba: problems %d and %d of a batch share buffers", j, i);
    SLAM_REQUIRE(probs[i].lin_mode == L->mode,
                 "slam_ba: problems of one batch must share lin_mode");
    L->b.p[i] = probs[i];
    L->max_grps = max(L->max_grps, probs[i].n_grps);
    L->max_sgrps = max(L->max_sgrps, probs[i].n_sgrps);
    L->max_blocks = max(L->max_blocks, probs[i].asm_act != nullptr ? probs[i].n_asm_act : probs[i].n_blocks);
    L->solve_lds = std::max(L->solve_lds, sizeof(double) * BlkLds(9 * probs[i].n_cams).total);
    L->solve_lds = std::max(L->solve_lds, g_solve_lds_floor);
    L->dense = L->dense && !sys_packed(probs[i].n_cams);
  }
  SLAM_REQUIRE(n == 1 || L->dense,
               "slam_ba: batched problems must use the one-workgroup solver (9C <= %d)", kLdsMaxN);
  return SLAM_OK;
}

static int launch_reset(const Launch& L, double lam0, hipStream_t s) {
  k_reset<<<dim3(1, L.n), 64, 0, s>>>(L.b, lam0);
  SLAM_LAUNCHED("k_reset");
  return SLAM_OK;
}

static int launch_build(const Launch& L, hipStream_t s) {
  // every entry of sys is written by the assembly (all listed blocks), so no clearing
  bool folded = L.mode == 1;
  for (int i = 0; i < L.n; ++i) folded = folded && L.b.p[i].asm_tab != nullptr;
  if (L.mode == 1) {
    k_lin_mfma<<<dim3(L.max_sgrps, L.n), kMWG, 0, s>>>(L.b);
    SLAM_LAUNCHED("k_lin_mfma");
  } else {
    k_linearize<<<dim3(L.max_grps, L.n), kLinWG, 0, s>>>(L.b);
    SLAM_LAUNCHED("k_linearize");
  }
  if (!folded) {  // k_lin_mfma skips the fold of a problem without asm_tab
    k_assemble<<<dim3(L.max_blocks, L.n), kAsmWG, 0, s>>>(L.b);
    SLAM_LAUNCHED("k_assemble");
  }
  return SLAM_OK;
}

static int launch_solve(const Launch& L, bool fuse_decide, hipStream_t s) {
  if (L.dense) {
    k_solve_blk<<<dim3(1, L.n), kBlkWG, L.solve_lds, s>>>(L.b);
    SLAM_LAUNCHED("k_solve_blk");
  } else {
    if (tl_flow_ok(L.b.p[0], s)) {
      if (int rc = tl_solve_flow(L.b.p[0], s)) return rc;
    } else {
      if (int rc = tl_solve_levels(L.b.p[0], s)) return rc;
    }
  }
  if (fuse_decide)
    k_back_trial<true><<<dim3(L.max_grps, L.n), kGrp, 0, s>>>(L.b);
  else
    k_back_trial<false><<<dim3(L.max_grps, L.n), kGrp, 0, s>>>(L.b);
  SLAM_LAUNCHED("k_back_trial");
  return SLAM_OK;
}

}  // namespace

extern "C" int slam_ba_set_solve_lds_floor(int bytes) {
  SLAM_REQUIRE(bytes >= 0 && bytes <= 160 * 1024, "slam_ba_set_solve_lds_floor: %d B", bytes);
  g_solve_lds_floor = (size_t)bytes;
  return SLAM_OK;
}

extern "C" int slam_ba_reset(const slam_ba_problem* prob, double lambda0, void* stream) {
  return slam_ba_reset_batch(prob, 1, lambda0, stream);
}

extern "C" int slam_ba_reset_batch(const slam_ba_problem* probs, int n_probs, double lambda0,
                                   void* stream) {
  SLAM_REQUIRE(n_probs >= 0, "slam_ba_reset_batch: n_probs < 0");
  SLAM_REQUIRE(n_probs == 0 || probs != nullptr, "slam_ba_reset_batch: null problem array");
  for (int i0 = 0; i0 < n_probs; i0 += kBaMaxBatch) {
    Launch L;
    const int n = min(kBaMaxBatch, n_probs - i0);
    for (int i = 0; i < n; ++i)
      if (int rc = check_problem(probs + i0 + i)) return rc;
    L.n = n;
    for (int i = 0; i < n; ++i) L.b.p[i] = probs[i0 + i];
    if (int rc = launch_reset(L, lambda0, slam::as_stream(stream))) return rc;
  }
  return SLAM_OK;
}

extern "C" int slam_ba_build_system(const slam_ba_problem* prob, void* stream) {
  Launch L;
  if (int rc = make_launch(prob, 1, &L)) return rc;
  return launch_build(L, slam::as_stream(stream));
}

extern "C" int slam_ba_solve_step(const slam_ba_problem* prob, void* stream) {
  Launch L;
  if (int rc = make_launch(prob, 1, &L)) return rc;
  return launch_solve(L, false, slam::as_stream(stream));
}

extern "C" int slam_ba_decide(const slam_ba_problem* prob, void* stream) {
  Launch L;
  if (int rc = make_launch(prob, 1, &L)) return rc;
  k_decide<<<dim3(1, 1), 64, 0, slam::as_stream(stream)>>>(L.b);
  SLAM_LAUNCHED("k_decide");
  return SLAM_OK;
}

extern "C" int slam_ba_iterate(const slam_ba_problem* prob, int n_iter, void* stream) {
  return slam_ba_iterate_batch(prob, 1, n_iter, stream);
}

extern "C" int slam_ba_iterate_batch(const slam_ba_problem* probs, int n_probs, int n_iter,
                                     void* stream) {
  SLAM_REQUIRE(n_probs >= 0 && n_iter >= 0, "slam_ba_iterate_batch: negative count");
  SLAM_REQUIRE(n_probs == 0 || probs != nullptr, "slam_ba_iterate_batch: null problem array");
  hipStream_t s = slam::as_stream(stream);
  // dense problems in chunks of kBaMaxBatch share launches; a packed (tiled
  // solver) problem iterates on its own
  int i0 = 0;
  while (i0 < n_probs) {
    int n = 0;
    while (n < kBaMaxBatch && i0 + n < n_probs && (n == 0 || !sys_packed(probs[i0 + n].n_cams)) &&
           !(n > 0 && sys_packed(probs[i0].n_cams)))
      ++n;
    Launch L;
    if (int rc = make_launch(probs + i0, n, &L)) return rc;
    for (int it = 0; it < n_iter; ++it) {
      if (int rc = launch_build(L, s)) return rc;
      if (int rc = launch_solve(L, true, s)) return rc;  // decide fused into the last group
    }
    i0 += n;
  }
  return SLAM_OK;
}

#ifdef SLAM_SOLVE_TRACE
extern "C" int slam_solve_trace(unsigned long long* out) {
  SLAM_HIP(hipDeviceSynchronize());
  SLAM_HIP(hipMemcpyFromSymbol(out, HIP_SYMBOL(g_solve_trace), 20 * 6 * sizeof(unsigned long long)));
  return SLAM_OK;
}
#endif

#ifdef SLAM_LINM_PROFILE
extern "C" int slam_linm_stamps(unsigned long long* out, int n) {
  SLAM_HIP(hipDeviceSynchronize());
  SLAM_HIP(hipMemcpyFromSymbol(out, HIP_SYMBOL(g_linm_stamp), (size_t)n * 8 * sizeof(unsigned long long)));
  return SLAM_OK;
}
#endif

#ifdef SLAM_FLOW_PROFILE
extern "C" int slam_flow_epi_stamps(unsigned long long* out4) {
  SLAM_HIP(hipDeviceSynchronize());
  SLAM_HIP(hipMemcpyFromSymbol(out4, HIP_SYMBOL(g_flow_epi), 4 * sizeof(unsigned long long)));
  return SLAM_OK;
}
extern "C" int slam_flow_sub_stamps(unsigned long long* out, int n_cols) {
  SLAM_HIP(hipDeviceSynchronize());
  SLAM_HIP(hipMemcpyFromSymbol(out, HIP_SYMBOL(g_flow_sub), (size_t)n_cols * 8 * sizeof(unsigned long long)));
  return SLAM_OK;
}
extern "C" int slam_flow_fac_stamps(unsigned long long* out16) {
  SLAM_HIP(hipDeviceSynchronize());
  SLAM_HIP(hipMemcpyFromSymbol(out16, HIP_SYMBOL(g_flow_fac), 16 * sizeof(unsigned long long)));
  return SLAM_OK;
}
extern "C" int slam_flow_stamps(unsigned long long* out, int n_cols) {
  SLAM_HIP(hipDeviceSynchronize());
  SLAM_HIP(hipMemcpyFromSymbol(out, HIP_SYMBOL(g_flow_stamp), (size_t)n_cols * 8 * sizeof(unsigned long long)));
  return SLAM_OK;
}
#endif

#ifdef SLAM_TL_PROFILE
extern "C" int slam_tl_stamps(unsigned long long* out8) {
  SLAM_HIP(hipDeviceSynchronize());
  SLAM_HIP(hipMemcpyFromSymbol(out8, HIP_SYMBOL(g_tl_stamp), 8 * sizeof(unsigned long long)));
  return SLAM_OK;
}
#endif
