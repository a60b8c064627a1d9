// EPnP (Lepetit, Moreno-Noguer, Fua 2009) on a PnP-RANSAC sample, device
// form.  The minimal solver OpenCV's solvePnPRansac runs on each 5-point
// sample for SOLVEPNP_ITERATIVE (the reference's call,
// /root/reference/transformation.py:11-13): the same operations in the same
// order as the CPU restatement oracle/epnp.h (control points from the scatter
// matrix, barycentric weights, the 4 smallest eigenvectors of M^T M by cyclic
// Jacobi, OpenCV's three beta approximations + 5 Gauss-Newton steps, Horn's
// quaternion for the absolute orientation, least mean reprojection error).
// One lane per sample; the 12x12 M^T M and its eigenvectors live in the
// caller's LDS slot (MtM, V12: 144 doubles each; wsl: kEpnpWs doubles for the
// barycentric weights, the 4 null vectors and L).
#pragma once

#include <hip/hip_runtime.h>
#include <cmath>

namespace slam_epnp {

constexpr int EPNP_MAXN = 8;
constexpr int kEpnpWs = 4 * EPNP_MAXN + 48 + 60;

/* cyclic Jacobi on the symmetric n x n matrix A (row-major, destroyed: its
 * diagonal ends as the eigenvalues); V (row-major) gets the eigenvectors as
 * columns.  Fixed rule: sweeps until the off-diagonal mass is below 1e-30 of
 * the diagonal mass, at most 40. */
template <int n>
__device__ __forceinline__ void ep_jacobi(double* A, double* V) {
  #pragma unroll
  for (int i = 0; i < n; ++i)
    #pragma unroll
    for (int j = 0; j < n; ++j) V[i * n + j] = i == j ? 1.0 : 0.0;
  #pragma unroll 1
  for (int sweep = 0; sweep < 40; ++sweep) {
    double off = 0.0, dia = 0.0;
    #pragma unroll
    for (int i = 0; i < n; ++i) {
      dia += A[i * n + i] * A[i * n + i];
      #pragma unroll
      for (int j = i + 1; j < n; ++j) off += A[i * n + j] * A[i * n + j];
    }
    if (!(off > 1e-30 * dia)) break;
    constexpr int kUnroll = n <= 4 ? 4 : 1;
    #pragma unroll kUnroll
    for (int p = 0; p < n - 1; ++p)
      #pragma unroll kUnroll
      for (int q = p + 1; q < n; ++q) {
        const double apq = A[p * n + q];
        if (apq == 0.0) continue;
        const double app = A[p * n + p], aqq = A[q * n + q];
        const double th = (aqq - app) / (2.0 * apq);
        const double t = (th >= 0.0 ? 1.0 : -1.0) / (fabs(th) + sqrt(th * th + 1.0));
        const double c = 1.0 / sqrt(t * t + 1.0), s = t * c;
        #pragma unroll
        for (int k = 0; k < n; ++k) {  /* columns p, q */
          const double akp = A[k * n + p], akq = A[k * n + q];
          A[k * n + p] = c * akp - s * akq;
          A[k * n + q] = s * akp + c * akq;
        }
        #pragma unroll
        for (int k = 0; k < n; ++k) {  /* rows p, q */
          const double apk = A[p * n + k], aqk = A[q * n + k];
          A[p * n + k] = c * apk - s * aqk;
          A[q * n + k] = s * apk + c * aqk;
        }
        #pragma unroll
        for (int k = 0; k < n; ++k) {
          const double vkp = V[k * n + p], vkq = V[k * n + q];
          V[k * n + p] = c * vkp - s * vkq;
          V[k * n + q] = s * vkp + c * vkq;
        }
      }
  }
}

/* least squares x (k <= 5 unknowns) of the 6 x k system A x = b by the
 * normal equations (Cholesky); returns 0 when not positive definite */
template <int k>
__device__ __forceinline__ int ep_lsq6(const double* A, const double* b, double* x) {
  double N[5][5], r[5];
  #pragma unroll
  for (int i = 0; i < k; ++i) {
    #pragma unroll
    for (int j = 0; j <= i; ++j) {
      double s = 0.0;
      #pragma unroll
      for (int m = 0; m < 6; ++m) s += A[m * k + i] * A[m * k + j];
      N[i][j] = s;
    }
    double s = 0.0;
    #pragma unroll
    for (int m = 0; m < 6; ++m) s += A[m * k + i] * b[m];
    r[i] = s;
  }
  #pragma unroll
  for (int j = 0; j < k; ++j) {
    double s = N[j][j];
    #pragma unroll
    for (int p = 0; p < j; ++p) s -= N[j][p] * N[j][p];
    if (!(s > 0.0)) return 0;
    N[j][j] = sqrt(s);
    #pragma unroll
    for (int i = j + 1; i < k; ++i) {
      double t = N[i][j];
      #pragma unroll
      for (int p = 0; p < j; ++p) t -= N[i][p] * N[j][p];
      N[i][j] = t / N[j][j];
    }
  }
  double y[5];
  #pragma unroll
  for (int i = 0; i < k; ++i) {
    double t = r[i];
    #pragma unroll
    for (int p = 0; p < i; ++p) t -= N[i][p] * y[p];
    y[i] = t / N[i][i];
  }
  #pragma unroll
  for (int i = k - 1; i >= 0; --i) {
    double t = y[i];
    #pragma unroll
    for (int p = i + 1; p < k; ++p) t -= N[p][i] * x[p];
    x[i] = t / N[i][i];
  }
  return 1;
}

// ep_lsq6<k> on a 6 x 5 system whose columns >= k are dead (decoupled: unit
// diagonal in the normal equations, zero right-hand side, x = 0): the live
// part performs exactly the operations of ep_lsq6<k>
__device__ __forceinline__ int ep_lsq6_live(const double* A, const double* b, int k, double* x) {
  double N[5][5], r[5];
  #pragma unroll
  for (int i = 0; i < 5; ++i) {
    #pragma unroll
    for (int j = 0; j <= i; ++j) {
      double s = 0.0;
      #pragma unroll
      for (int m = 0; m < 6; ++m) s += A[m * 5 + i] * A[m * 5 + j];
      N[i][j] = i < k ? s : (i == j ? 1.0 : 0.0);
    }
    double s = 0.0;
    #pragma unroll
    for (int m = 0; m < 6; ++m) s += A[m * 5 + i] * b[m];
    r[i] = i < k ? s : 0.0;
  }
  bool ok = true;
  #pragma unroll
  for (int j = 0; j < 5; ++j) {
    double s = N[j][j];
    #pragma unroll
    for (int p = 0; p < j; ++p) s -= N[j][p] * N[j][p];
    ok = ok && s > 0.0;
    N[j][j] = sqrt(s);
    #pragma unroll
    for (int i = j + 1; i < 5; ++i) {
      double t = N[i][j];
      #pragma unroll
      for (int p = 0; p < j; ++p) t -= N[i][p] * N[j][p];
      N[i][j] = t / N[j][j];
    }
  }
  if (!ok) return 0;
  double y[5];
  #pragma unroll
  for (int i = 0; i < 5; ++i) {
    double t = r[i];
    #pragma unroll
    for (int p = 0; p < i; ++p) t -= N[i][p] * y[p];
    y[i] = t / N[i][i];
  }
  #pragma unroll
  for (int i = 4; i >= 0; --i) {
    double t = y[i];
    #pragma unroll
    for (int p = i + 1; p < 5; ++p) t -= N[p][i] * x[p];
    x[i] = t / N[i][i];
  }
  return 1;
}

/* pose from the 4 camera-frame control points ccs (betas applied): R, t and
 * the mean reprojection error over the n points */
template <int n>
__device__ __forceinline__ double ep_pose(const double ccs[4][3], const double* alph, const double* pw,
                             const double* uv, double fx, double fy, double cx, double cy,
                             double R[9], double t[3]) {
  double pc[EPNP_MAXN][3] = {{0.0}};
  double cc[4][3];
  #pragma unroll
  for (int j = 0; j < 4; ++j)
    #pragma unroll
    for (int d = 0; d < 3; ++d) cc[j][d] = ccs[j][d];
  #pragma unroll
  for (int i = 0; i < n; ++i)
    #pragma unroll
    for (int d = 0; d < 3; ++d)
      pc[i][d] = alph[4 * i] * cc[0][d] + alph[4 * i + 1] * cc[1][d] + alph[4 * i + 2] * cc[2][d] +
                 alph[4 * i + 3] * cc[3][d];
  if (pc[0][2] < 0.0)
    #pragma unroll
    for (int i = 0; i < n; ++i)
      #pragma unroll
      for (int d = 0; d < 3; ++d) pc[i][d] = -pc[i][d];
  double c0[3] = {0, 0, 0}, w0[3] = {0, 0, 0};
  #pragma unroll
  for (int i = 0; i < n; ++i)
    #pragma unroll
    for (int d = 0; d < 3; ++d) {
      c0[d] += pc[i][d];
      w0[d] += pw[3 * i + d];
    }
  #pragma unroll
  for (int d = 0; d < 3; ++d) {
    c0[d] /= n;
    w0[d] /= n;
  }
  double S[3][3] = {{0, 0, 0}, {0, 0, 0}, {0, 0, 0}};  /* S[a][b] = sum pw_a pc_b */
  #pragma unroll
  for (int i = 0; i < n; ++i)
    #pragma unroll
    for (int a = 0; a < 3; ++a)
      #pragma unroll
      for (int b = 0; b < 3; ++b) S[a][b] += (pw[3 * i + a] - w0[a]) * (pc[i][b] - c0[b]);
  double N[16] = {S[0][0] + S[1][1] + S[2][2], S[1][2] - S[2][1], S[2][0] - S[0][2], S[0][1] - S[1][0],
                  S[1][2] - S[2][1], S[0][0] - S[1][1] - S[2][2], S[0][1] + S[1][0], S[2][0] + S[0][2],
                  S[2][0] - S[0][2], S[0][1] + S[1][0], -S[0][0] + S[1][1] - S[2][2], S[1][2] + S[2][1],
                  S[0][1] - S[1][0], S[2][0] + S[0][2], S[1][2] + S[2][1], -S[0][0] - S[1][1] + S[2][2]};
  double V[16];
  ep_jacobi<4>(N, V);
  int bi = 0;
  #pragma unroll
  for (int i = 1; i < 4; ++i)
    if (N[i * 4 + i] > N[bi * 4 + bi]) bi = i;
  double q0 = V[0 * 4 + bi], q1 = V[1 * 4 + bi], q2 = V[2 * 4 + bi], q3 = V[3 * 4 + bi];
  if (q0 < 0.0) {
    q0 = -q0; q1 = -q1; q2 = -q2; q3 = -q3;
  }
  R[0] = q0 * q0 + q1 * q1 - q2 * q2 - q3 * q3;
  R[1] = 2.0 * (q1 * q2 - q0 * q3);
  R[2] = 2.0 * (q1 * q3 + q0 * q2);
  R[3] = 2.0 * (q1 * q2 + q0 * q3);
  R[4] = q0 * q0 - q1 * q1 + q2 * q2 - q3 * q3;
  R[5] = 2.0 * (q2 * q3 - q0 * q1);
  R[6] = 2.0 * (q1 * q3 - q0 * q2);
  R[7] = 2.0 * (q2 * q3 + q0 * q1);
  R[8] = q0 * q0 - q1 * q1 - q2 * q2 + q3 * q3;
  #pragma unroll
  for (int d = 0; d < 3; ++d) t[d] = c0[d] - (R[3 * d] * w0[0] + R[3 * d + 1] * w0[1] + R[3 * d + 2] * w0[2]);
  double err = 0.0;
  #pragma unroll
  for (int i = 0; i < n; ++i) {
    const double* X = pw + 3 * i;
    const double Xc = R[0] * X[0] + R[1] * X[1] + R[2] * X[2] + t[0];
    const double Yc = R[3] * X[0] + R[4] * X[1] + R[5] * X[2] + t[1];
    const double Zc = R[6] * X[0] + R[7] * X[1] + R[8] * X[2] + t[2];
    const double du = cx + fx * Xc / Zc - uv[2 * i], dv = cy + fy * Yc / Zc - uv[2 * i + 1];
    err += sqrt(du * du + dv * dv);
  }
  return err / n;
}

/* rotation vector of the unit quaternion of R (R = ep_pose output) */
__device__ inline void ep_rvec(const double R[9], double r[3]) {
  /* quaternion from R (Shepperd, largest-diagonal branch) */
  const double tr = R[0] + R[4] + R[8];
  double q0, q1, q2, q3;
  if (tr > 0.0) {
    const double s = 2.0 * sqrt(tr + 1.0);
    q0 = 0.25 * s; q1 = (R[7] - R[5]) / s; q2 = (R[2] - R[6]) / s; q3 = (R[3] - R[1]) / s;
  } else if (R[0] > R[4] && R[0] > R[8]) {
    const double s = 2.0 * sqrt(1.0 + R[0] - R[4] - R[8]);
    q0 = (R[7] - R[5]) / s; q1 = 0.25 * s; q2 = (R[1] + R[3]) / s; q3 = (R[2] + R[6]) / s;
  } else if (R[4] > R[8]) {
    const double s = 2.0 * sqrt(1.0 + R[4] - R[0] - R[8]);
    q0 = (R[2] - R[6]) / s; q1 = (R[1] + R[3]) / s; q2 = 0.25 * s; q3 = (R[5] + R[7]) / s;
  } else {
    const double s = 2.0 * sqrt(1.0 + R[8] - R[0] - R[4]);
    q0 = (R[3] - R[1]) / s; q1 = (R[2] + R[6]) / s; q2 = (R[5] + R[7]) / s; q3 = 0.25 * s;
  }
  if (q0 < 0.0) {
    q0 = -q0; q1 = -q1; q2 = -q2; q3 = -q3;
  }
  const double vn = sqrt(q1 * q1 + q2 * q2 + q3 * q3);
  const double th = 2.0 * atan2(vn, q0);
  const double k = vn > 0.0 ? th / vn : 2.0;
  r[0] = q1 * k; r[1] = q2 * k; r[2] = q3 * k;
}

// ---------------------------------------------------------------- group form
// One EPnP per 16-lane group of a one-wave workgroup (lane k = lane & 15 of
// group g = lane >> 4); the steps that dominate -- M^T M and its 12x12 Jacobi
// eigen-decomposition -- run with lanes k < 12 owning row k, the three beta
// approximations on lanes 0..2, the rest on lane 0.  Every value is computed
// with the operations of oracle/epnp.h in the same order.  The caller's
// workgroup is one wave, so __syncthreads() is a cheap wave-level fence.
constexpr int kJld = 13;  // row stride of the Jacobi buffers (odd: rows on distinct banks)
struct EpGroup {         // LDS of one group
  double A[144], V[144]; // M^T M (destroyed: eigenvalues on the diagonal), eigenvectors
  double alph[4 * EPNP_MAXN];
  double v[4][12];
  double L[60], rho[6];
  double cw[4][3];
  double res[3][8];      // per approximation: err, p[6], valid
  double offdia[2];
  double B[2][12 * kJld];  // Jacobi: A ping-pong (round r reads B[cur], writes B[cur ^ 1])
  double cs[12];           // Jacobi: the round's (c, s) of the 6 pairs
  double part[24];         // Jacobi: per-row diagonal / off-diagonal squares
  double pad[27];
  int flag;              // 0: degenerate, 1: ok; Jacobi: 1 while sweeping
};
// consecutive groups 32 banks apart, so lanes 0..15 and 16..31 of a wave
// (one ds_read_b64 bank group) never collide on the stride-13 rows
static_assert(sizeof(EpGroup) % 256 == 128, "EpGroup stride must be 128 mod 256 bytes");

// control points and barycentric weights (lane 0); returns 0 when degenerate
template <int n>
__device__ __forceinline__ int ep_bary(const double* pw, EpGroup& G) {
  double cw[4][3] = {{0, 0, 0}};
  for (int i = 0; i < n; ++i)
    for (int d = 0; d < 3; ++d) cw[0][d] += pw[3 * i + d];
  for (int d = 0; d < 3; ++d) cw[0][d] /= n;
  double A3[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0}, V3[9];
  for (int i = 0; i < n; ++i)
    for (int a = 0; a < 3; ++a)
      for (int b = 0; b < 3; ++b) A3[3 * a + b] += (pw[3 * i + a] - cw[0][a]) * (pw[3 * i + b] - cw[0][b]);
  ep_jacobi<3>(A3, V3);
  int ord[3] = {0, 1, 2};
  for (int i = 0; i < 3; ++i)
    for (int j = i + 1; j < 3; ++j)
      if (A3[4 * ord[j]] > A3[4 * ord[i]]) {
        const int tmp = ord[i]; ord[i] = ord[j]; ord[j] = tmp;
      }
  for (int k = 0; k < 3; ++k) {
    const double sc = sqrt(fmax(A3[4 * ord[k]], 0.0) / n);
    for (int d = 0; d < 3; ++d) cw[k + 1][d] = cw[0][d] + sc * V3[3 * d + ord[k]];
  }
  for (int k = 0; k < 4; ++k)
    for (int d = 0; d < 3; ++d) G.cw[k][d] = cw[k][d];
  double C[3][3];
  for (int d = 0; d < 3; ++d)
    for (int k = 0; k < 3; ++k) C[d][k] = cw[k + 1][d] - cw[0][d];
  const double c00 = C[1][1] * C[2][2] - C[1][2] * C[2][1];
  const double c01 = C[0][2] * C[2][1] - C[0][1] * C[2][2];
  const double c02 = C[0][1] * C[1][2] - C[0][2] * C[1][1];
  const double c10 = C[1][2] * C[2][0] - C[1][0] * C[2][2];
  const double c11 = C[0][0] * C[2][2] - C[0][2] * C[2][0];
  const double c12 = C[0][2] * C[1][0] - C[0][0] * C[1][2];
  const double c20 = C[1][0] * C[2][1] - C[1][1] * C[2][0];
  const double c21 = C[0][1] * C[2][0] - C[0][0] * C[2][1];
  const double c22 = C[0][0] * C[1][1] - C[0][1] * C[1][0];
  const double det = C[0][0] * c00 + C[0][1] * c10 + C[0][2] * c20;
  if (!(fabs(det) > 0.0)) return 0;
  const double id = 1.0 / det;
  for (int i = 0; i < n; ++i) {
    const double x = pw[3 * i] - cw[0][0], y = pw[3 * i + 1] - cw[0][1], z = pw[3 * i + 2] - cw[0][2];
    const double a1 = (c00 * x + c01 * y + c02 * z) * id;
    const double a2 = (c10 * x + c11 * y + c12 * z) * id;
    const double a3 = (c20 * x + c21 * y + c22 * z) * id;
    G.alph[4 * i] = 1.0 - a1 - a2 - a3;
    G.alph[4 * i + 1] = a1;
    G.alph[4 * i + 2] = a2;
    G.alph[4 * i + 3] = a3;
  }
  return 1;
}

// row r of M^T M: sum over points i (in order) of m1[r] m1[c] + m2[r] m2[c]
template <int n>
__device__ __forceinline__ void ep_mtm_row(int r, const double* uv, double fx, double fy, double cx,
                                           double cy, EpGroup& G) {
  double acc[12];
#pragma unroll
  for (int c = 0; c < 12; ++c) acc[c] = 0.0;
  const int jr = r / 3, dr = r - 3 * jr;
  for (int i = 0; i < n; ++i) {
    double m1[12], m2[12];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const double a = G.alph[4 * i + j];
      m1[3 * j] = a * fx; m1[3 * j + 1] = 0.0; m1[3 * j + 2] = a * (cx - uv[2 * i]);
      m2[3 * j] = 0.0; m2[3 * j + 1] = a * fy; m2[3 * j + 2] = a * (cy - uv[2 * i + 1]);
    }
    const double ar = G.alph[4 * i + jr];
    const double m1r = dr == 0 ? ar * fx : dr == 1 ? 0.0 : ar * (cx - uv[2 * i]);
    const double m2r = dr == 0 ? 0.0 : dr == 1 ? ar * fy : ar * (cy - uv[2 * i + 1]);
#pragma unroll
    for (int c = 0; c < 12; ++c) acc[c] += m1r * m1[c] + m2r * m2[c];
  }
#pragma unroll
  for (int c = 0; c < 12; ++c) G.A[12 * r + c] = acc[c];
}

// The 12x12 Jacobi of M^T M with the round-robin ordering of
// oracle/epnp.h ep_jacobi12_par: lanes k < 12 of the group own row k of A
// (in LDS, ping-pong B[cur] -> B[cur ^ 1]) and of V (in registers).  Per
// round: lanes 0..5 derive pair k's (c, s) from the round-start matrix and
// publish them; then every lane rotates the column pairs of its own row AND
// of its partner's row (A J, the same operations the partner performs), and
// forms its new row from the two (J^T (A J)) -- one exchange through LDS
// per round, rounds fully unrolled so the pair columns are compile-time
// register indices.  The wave loops until every group has met its own
// stopping rule; a finished group keeps copying its rows.
__device__ __forceinline__ void ep_pairs12(int r, int pp[6], int qq[6]) {
  int a[12];
  a[0] = 0;
#pragma unroll
  for (int i = 1; i < 12; ++i) a[i] = 1 + (i - 1 + r) % 11;
#pragma unroll
  for (int i = 0; i < 6; ++i) {
    const int x = a[i], y = a[11 - i];
    pp[i] = x < y ? x : y;
    qq[i] = x < y ? y : x;
  }
}

// branch-free (the six pairs' chains interleave): a_pq = 0 selects the
// identity (c = 1, s = 0) as the oracle's early return does
__device__ __forceinline__ void ep_rot_cs(double app, double aqq, double apq, double& c, double& s) {
  const bool z = apq == 0.0;
  const double th = (aqq - app) / (2.0 * (z ? 1.0 : apq));
  const double t = (th >= 0.0 ? 1.0 : -1.0) / (fabs(th) + sqrt(th * th + 1.0));
  const double cc = 1.0 / sqrt(t * t + 1.0);
  c = z ? 1.0 : cc;
  s = z ? 0.0 : t * cc;
}

template <int r>
__device__ __forceinline__ void ep_jacobi_round(EpGroup& G, int k, int kr, bool act, int cur,
                                                double (&vr)[12]) {
  constexpr int n = 12, ld = kJld;
  const double* A0 = G.B[cur];
  double* A1 = G.B[cur ^ 1];
  int pp[6], qq[6];
  ep_pairs12(r, pp, qq);
  if (k < 6) {
    // pair k of this round (a[k], a[11 - k] of ep_pairs12)
    const int x = k == 0 ? 0 : 1 + (k - 1 + r) % 11, y = 1 + (10 - k + r) % 11;
    const int p = x < y ? x : y, q = x < y ? y : x;
    double c, s;
    ep_rot_cs(A0[p * ld + p], A0[q * ld + q], A0[p * ld + q], c, s);
    G.cs[2 * k] = c;
    G.cs[2 * k + 1] = s;
  }
  // the pair holding row kr (closed form of ep_pairs12: kr sits at position
  // pos of a[], its partner at 11 - pos) -- no per-pair compare chains
  const int pos = kr == 0 ? 0 : (kr + 10 - r % 11) % 11 + 1;
  const int ppos = 11 - pos;
  const int partner = ppos == 0 ? 0 : 1 + (ppos - 1 + r) % 11;
  const int pi = pos < ppos ? pos : ppos;
  const bool isp = kr < partner;
  double row[n], prow[n];
#pragma unroll
  for (int j = 0; j < n; ++j) {
    row[j] = A0[kr * ld + j];
    prow[j] = A0[partner * ld + j];
  }
  __syncthreads();
  double c[6], s[6];
#pragma unroll
  for (int i = 0; i < 6; ++i) {
    c[i] = G.cs[2 * i];
    s[i] = G.cs[2 * i + 1];
  }
  double ck = c[0], sk = s[0];
#pragma unroll
  for (int i = 1; i < 6; ++i) {
    ck = pi == i ? c[i] : ck;
    sk = pi == i ? s[i] : sk;
  }
  double out[n];
#pragma unroll
  for (int j = 0; j < n; ++j) out[j] = row[j];
  // columns (A J, V J): the pairs are disjoint, any order
#pragma unroll
  for (int i = 0; i < 6; ++i) {
    const int P = pp[i], Q = qq[i];
    const double akp = row[P], akq = row[Q];
    row[P] = c[i] * akp - s[i] * akq;
    row[Q] = s[i] * akp + c[i] * akq;
    const double bkp = prow[P], bkq = prow[Q];
    prow[P] = c[i] * bkp - s[i] * bkq;
    prow[Q] = s[i] * bkp + c[i] * bkq;
    const double vkp = vr[P], vkq = vr[Q];
    const double wp = c[i] * vkp - s[i] * vkq, wq = s[i] * vkp + c[i] * vkq;
    vr[P] = act ? wp : vkp;
    vr[Q] = act ? wq : vkq;
  }
  // pin V's rotated values here: left free, the compiler defers the V chain
  // and keeps every round's (c, s) live across the sweep (22 VGPRs a round)
#pragma unroll
  for (int j = 0; j < n; ++j) asm volatile("" : "+v"(vr[j]));
  // rows (J^T (A J)) of the pair holding k; a finished group copies its row
#pragma unroll
  for (int j = 0; j < n; ++j) {
    const double nv = isp ? ck * row[j] - sk * prow[j] : sk * prow[j] + ck * row[j];
    out[j] = act ? nv : out[j];
  }
  if (k < n) {
#pragma unroll
    for (int j = 0; j < n; ++j) A1[k * ld + j] = out[j];
  }
  __syncthreads();
}

__device__ __forceinline__ void ep_jacobi12_group(EpGroup& G, int k, bool live) {
  constexpr int n = 12, ld = kJld;
  const bool own = k < n;
  const int kr = own ? k : 0;
  double vr[n];
#pragma unroll
  for (int j = 0; j < n; ++j) vr[j] = kr == j ? 1.0 : 0.0;
  if (own) {
#pragma unroll
    for (int j = 0; j < n; ++j) G.B[0][k * ld + j] = G.A[k * n + j];
  }
  if (k == 0) G.flag = live ? 1 : 0;
  __syncthreads();
  int cur = 0;
  for (int sweep = 0; sweep < 40; ++sweep) {
    // off / dia by rows: row k's squares, then lane 0 sums the rows in order
    if (own) {
      const double* Ar = G.B[cur] + k * ld;
      double o = 0.0;
#pragma unroll
      for (int j = 1; j < n; ++j)
        if (j > k) o += Ar[j] * Ar[j];
      G.part[k] = Ar[k] * Ar[k];
      G.part[n + k] = o;
    }
    __syncthreads();
    if (k == 0 && G.flag) {
      double off = 0.0, dia = 0.0;
      for (int i = 0; i < n; ++i) {
        dia += G.part[i];
        off += G.part[n + i];
      }
      if (!(off > 1e-24 * dia)) G.flag = 0;
    }
    __syncthreads();
    const bool act = own && G.flag != 0;
    if (__ballot(G.flag != 0) == 0ull) break;
#ifdef SLAM_PNPH_TRACE
    if (threadIdx.x == 0) G.offdia[1] = sweep + 1;
#endif
    ep_jacobi_round<0>(G, k, kr, act, cur, vr);
    ep_jacobi_round<1>(G, k, kr, act, cur ^ 1, vr);
    ep_jacobi_round<2>(G, k, kr, act, cur, vr);
    ep_jacobi_round<3>(G, k, kr, act, cur ^ 1, vr);
    ep_jacobi_round<4>(G, k, kr, act, cur, vr);
    ep_jacobi_round<5>(G, k, kr, act, cur ^ 1, vr);
    ep_jacobi_round<6>(G, k, kr, act, cur, vr);
    ep_jacobi_round<7>(G, k, kr, act, cur ^ 1, vr);
    ep_jacobi_round<8>(G, k, kr, act, cur, vr);
    ep_jacobi_round<9>(G, k, kr, act, cur ^ 1, vr);
    ep_jacobi_round<10>(G, k, kr, act, cur, vr);
    cur ^= 1;  // 11 rounds: odd
  }
  if (own) {
#pragma unroll
    for (int j = 0; j < n; ++j) {
      G.A[k * n + j] = G.B[cur][k * ld + j];
      G.V[k * n + j] = vr[j];
    }
  }
  __syncthreads();
}

// eigen ordering, the 4 null vectors, L and rho (lane 0)
__device__ __forceinline__ void ep_lrho(EpGroup& G) {
  int o12[12];
  for (int i = 0; i < 12; ++i) o12[i] = i;
  for (int i = 0; i < 4; ++i)
    for (int j = i + 1; j < 12; ++j)
      if (G.A[13 * o12[j]] < G.A[13 * o12[i]]) {
        const int tmp = o12[i]; o12[i] = o12[j]; o12[j] = tmp;
      }
  for (int k = 0; k < 4; ++k)
    for (int r = 0; r < 12; ++r) G.v[k][r] = G.V[12 * r + o12[k]];
  const int pa[6] = {0, 0, 0, 1, 1, 2}, pb[6] = {1, 2, 3, 2, 3, 3};
  for (int j = 0; j < 6; ++j) {
    double dv[4][3];
    for (int k = 0; k < 4; ++k)
      for (int d = 0; d < 3; ++d) dv[k][d] = G.v[k][3 * pa[j] + d] - G.v[k][3 * pb[j] + d];
#define EP_DOT(a, b) (dv[a][0] * dv[b][0] + dv[a][1] * dv[b][1] + dv[a][2] * dv[b][2])
    G.L[10 * j + 0] = EP_DOT(0, 0);
    G.L[10 * j + 1] = 2.0 * EP_DOT(0, 1);
    G.L[10 * j + 2] = EP_DOT(1, 1);
    G.L[10 * j + 3] = 2.0 * EP_DOT(0, 2);
    G.L[10 * j + 4] = 2.0 * EP_DOT(1, 2);
    G.L[10 * j + 5] = EP_DOT(2, 2);
    G.L[10 * j + 6] = 2.0 * EP_DOT(0, 3);
    G.L[10 * j + 7] = 2.0 * EP_DOT(1, 3);
    G.L[10 * j + 8] = 2.0 * EP_DOT(2, 3);
    G.L[10 * j + 9] = EP_DOT(3, 3);
#undef EP_DOT
    double s = 0.0;
    for (int d = 0; d < 3; ++d) {
      const double e = G.cw[pa[j]][d] - G.cw[pb[j]][d];
      s += e * e;
    }
    G.rho[j] = s;
  }
}

// beta approximation `approx` (0, 1, 2), 5 Gauss-Newton steps, pose and its
// reprojection error -> G.res[approx] (lane `approx`)
template <int n>
__device__ __forceinline__ void ep_approx(int approx, const double* pw, const double* uv, double fx,
                                          double fy, double cx, double cy, EpGroup& G) {
  double* res = G.res[approx];
  res[7] = 0.0;
  // columns of L per approximation: {B11 B12 B13 B14}, {B11 B12 B22},
  // {B11 B12 B22 B13 B23}; a fixed 6 x 5 system whose unused columns are
  // decoupled (unit diagonal, zero right-hand side) -- the live k x k part
  // rounds exactly as ep_lsq6<k>, and no register array is indexed by lane
  const int k = approx == 0 ? 4 : approx == 1 ? 3 : 5;
  double As[30], xb[5], rho[6];
#pragma unroll
  for (int j = 0; j < 6; ++j) rho[j] = G.rho[j];
#pragma unroll
  for (int j = 0; j < 6; ++j)
#pragma unroll
    for (int c = 0; c < 5; ++c) {
      const int col = c < 2 ? c : approx == 0 ? (c == 2 ? 3 : 6) : c;
      As[j * 5 + c] = c < k ? G.L[10 * j + col] : 0.0;
    }
  if (!ep_lsq6_live(As, rho, k, xb)) return;
  double be[4] = {0, 0, 0, 0};
  if (approx == 0) {
    if (xb[0] < 0.0) {
      be[0] = sqrt(-xb[0]);
      be[1] = -xb[1] / be[0]; be[2] = -xb[2] / be[0]; be[3] = -xb[3] / be[0];
    } else {
      be[0] = sqrt(xb[0]);
      be[1] = xb[1] / be[0]; be[2] = xb[2] / be[0]; be[3] = xb[3] / be[0];
    }
  } else {
    if (xb[0] < 0.0) {
      be[0] = sqrt(-xb[0]);
      be[1] = xb[2] < 0.0 ? sqrt(-xb[2]) : 0.0;
    } else {
      be[0] = sqrt(xb[0]);
      be[1] = xb[2] > 0.0 ? sqrt(xb[2]) : 0.0;
    }
    if (xb[1] < 0.0) be[0] = -be[0];
    if (approx == 2) be[2] = xb[3] / be[0];
  }
#pragma unroll 1
  for (int it = 0; it < 5; ++it) {
    double Ag[24], bg[6], dx[4];
    // an opaque offset: L is re-read from LDS every iteration (hoisted out of
    // the loop, its 60 values would hold 120 registers)
    int lo = 0;
    asm volatile("" : "+v"(lo));
    for (int j = 0; j < 6; ++j) {
      const double* l = G.L + 10 * j + lo;
      Ag[4 * j + 0] = 2.0 * l[0] * be[0] + l[1] * be[1] + l[3] * be[2] + l[6] * be[3];
      Ag[4 * j + 1] = l[1] * be[0] + 2.0 * l[2] * be[1] + l[4] * be[2] + l[7] * be[3];
      Ag[4 * j + 2] = l[3] * be[0] + l[4] * be[1] + 2.0 * l[5] * be[2] + l[8] * be[3];
      Ag[4 * j + 3] = l[6] * be[0] + l[7] * be[1] + l[8] * be[2] + 2.0 * l[9] * be[3];
      bg[j] = rho[j] - (l[0] * be[0] * be[0] + l[1] * be[0] * be[1] + l[2] * be[1] * be[1] +
                        l[3] * be[0] * be[2] + l[4] * be[1] * be[2] + l[5] * be[2] * be[2] +
                        l[6] * be[0] * be[3] + l[7] * be[1] * be[3] + l[8] * be[2] * be[3] +
                        l[9] * be[3] * be[3]);
    }
    if (!ep_lsq6<4>(Ag, bg, dx)) break;
    for (int c = 0; c < 4; ++c) be[c] += dx[c];
  }
  double ccs[4][3];
  for (int j = 0; j < 4; ++j)
    for (int d = 0; d < 3; ++d)
      ccs[j][d] = be[0] * G.v[0][3 * j + d] + be[1] * G.v[1][3 * j + d] + be[2] * G.v[2][3 * j + d] +
                  be[3] * G.v[3][3 * j + d];
  double R[9], t[3];
  res[0] = ep_pose<n>(ccs, G.alph, pw, uv, fx, fy, cx, cy, R, t);
  double r[3];
  ep_rvec(R, r);
  res[1] = r[0]; res[2] = r[1]; res[3] = r[2];
  res[4] = t[0]; res[5] = t[1]; res[6] = t[2];
  res[7] = 1.0;
}

// the choice of epnp(): least error, first on ties, then the finiteness check
__device__ __forceinline__ int ep_choose(const EpGroup& G, double p[6]) {
  double best_err = INFINITY;
  int ok = 0;
  for (int a = 0; a < 3; ++a) {
    if (G.res[a][7] == 0.0) continue;
    if (G.res[a][0] < best_err) {
      best_err = G.res[a][0];
      for (int i = 0; i < 6; ++i) p[i] = G.res[a][1 + i];
      ok = 1;
    }
  }
  for (int i = 0; i < 6; ++i) ok &= isfinite(p[i]) ? 1 : 0;
  return ok;
}

}  // namespace slam_epnp
