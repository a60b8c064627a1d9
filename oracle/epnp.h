/*
 * ORACLE — test infrastructure only (see oracle/__init__.py).
 *
 * EPnP (Lepetit, Moreno-Noguer, Fua, IJCV 2009) on a small point set: the
 * minimal solver OpenCV's solvePnPRansac runs on each 5-point sample when the
 * caller asks for SOLVEPNP_ITERATIVE (the reference's call,
 * /root/reference/transformation.py:11-13, flags default): model_points = 5,
 * ransac kernel = EPnP.  Written out here with every step explicit, so the HIP
 * kernel (csrc/epnp.hpp) can state the same operations in the same order:
 *   control points  c0 = centroid, c1..c3 = c0 + sqrt(l_k / n) e_k from the
 *                   eigen-decomposition (cyclic Jacobi) of the scatter matrix;
 *   barycentric     alpha = [c1-c0 c2-c0 c3-c0]^-1 (X - c0) (3x3 cofactors);
 *   M (2n x 12)     the projection rows; the 4 eigenvectors of M^T M with the
 *                   smallest eigenvalues (Jacobi, round-robin pair ordering);
 *   betas           OpenCV's three approximations (L columns {B11 B12 B13 B14},
 *                   {B11 B12 B22}, {B11 B12 B22 B13 B23}) by normal equations,
 *                   each refined by 5 Gauss-Newton steps (normal equations);
 *   pose            camera control points, sign fix (z of the first point > 0),
 *                   absolute orientation by Horn's quaternion (4x4 Jacobi,
 *                   always a proper rotation), t = pc0 - R pw0;
 *   choice          the least mean reprojection error, first on ties.
 * PARITY UNPINNED vs OpenCV (absent here; OpenCV's epnp.cpp uses SVD solvers
 * and QR where this restatement uses Jacobi and normal equations): the spec
 * is the algorithm, checked by pose recovery on exact and noisy points.
 * Output: rvec (axis-angle from the quaternion) and t; returns 0 when the
 * sample is degenerate (non-finite result).
 */
#ifndef SLAM_ORACLE_EPNP_H
#define SLAM_ORACLE_EPNP_H
#include <math.h>
#include <string.h>

#define EPNP_MAXN 8

/* cyclic Jacobi on the symmetric n x n matrix A (row-major, destroyed: its
 * diagonal ends as the eigenvalues); V (row-major) gets the eigenvectors as
 * columns.  Fixed rule: sweeps until the off-diagonal mass is below 1e-30 of
 * the diagonal mass, at most 40. */
static inline void ep_jacobi(double* A, int n, double* V) {
  for (int i = 0; i < n; ++i)
    for (int j = 0; j < n; ++j) V[i * n + j] = i == j ? 1.0 : 0.0;
  for (int sweep = 0; sweep < 40; ++sweep) {
    double off = 0.0, dia = 0.0;
    for (int i = 0; i < n; ++i) {
      dia += A[i * n + i] * A[i * n + i];
      for (int j = i + 1; j < n; ++j) off += A[i * n + j] * A[i * n + j];
    }
    if (!(off > 1e-30 * dia)) break;
    for (int p = 0; p < n - 1; ++p)
      for (int q = p + 1; q < n; ++q) {
        const double apq = A[p * n + q];
        if (apq == 0.0) continue;
        const double app = A[p * n + p], aqq = A[q * n + q];
        const double th = (aqq - app) / (2.0 * apq);
        const double t = (th >= 0.0 ? 1.0 : -1.0) / (fabs(th) + sqrt(th * th + 1.0));
        const double c = 1.0 / sqrt(t * t + 1.0), s = t * c;
        for (int k = 0; k < n; ++k) {  /* columns p, q */
          const double akp = A[k * n + p], akq = A[k * n + q];
          A[k * n + p] = c * akp - s * akq;
          A[k * n + q] = s * akp + c * akq;
        }
        for (int k = 0; k < n; ++k) {  /* rows p, q */
          const double apk = A[p * n + k], aqk = A[q * n + k];
          A[p * n + k] = c * apk - s * aqk;
          A[q * n + k] = s * apk + c * aqk;
        }
        for (int k = 0; k < n; ++k) {
          const double vkp = V[k * n + p], vkq = V[k * n + q];
          V[k * n + p] = c * vkp - s * vkq;
          V[k * n + q] = s * vkp + c * vkq;
        }
      }
  }
}

/* the 12x12 eigen-decomposition of M^T M: Jacobi with the round-robin
 * (tournament) ordering -- 11 rounds of 6 disjoint pairs per sweep, the pair
 * (p, q) of slot i in round r being {a[i], a[11 - i]} with a[0] = 0 and
 * a[1..11] = 1..11 rotated by r.  In a round, every pair's (c, s) comes from
 * the matrix at the round start (c = 1, s = 0 when a_pq = 0); then all column
 * rotations (A J), then all row rotations (J^T (A J)), then V J; sweeps stop
 * when the off-diagonal mass is below 1e-24 of the diagonal mass.  The rounds
 * are what a GPU group executes in parallel (csrc/epnp.hpp). */
static inline void ep_pairs12(int r, int pp[6], int qq[6]) {
  int a[12];
  a[0] = 0;
  for (int i = 1; i < 12; ++i) a[i] = 1 + (i - 1 + r) % 11;
  for (int i = 0; i < 6; ++i) {
    const int x = a[i], y = a[11 - i];
    pp[i] = x < y ? x : y;
    qq[i] = x < y ? y : x;
  }
}

static inline void ep_rot_cs(double app, double aqq, double apq, double* c, double* s) {
  if (apq == 0.0) {
    *c = 1.0;
    *s = 0.0;
    return;
  }
  const double th = (aqq - app) / (2.0 * apq);
  const double t = (th >= 0.0 ? 1.0 : -1.0) / (fabs(th) + sqrt(th * th + 1.0));
  *c = 1.0 / sqrt(t * t + 1.0);
  *s = t * *c;
}

static inline void ep_jacobi12_par(double* A, double* V) {
  const int n = 12;
  for (int i = 0; i < n; ++i)
    for (int j = 0; j < n; ++j) V[i * n + j] = i == j ? 1.0 : 0.0;
  for (int sweep = 0; sweep < 40; ++sweep) {
    /* off-diagonal mass summed row by row (row partials, then the rows in order) */
    double off = 0.0, dia = 0.0;
    for (int i = 0; i < n; ++i) {
      dia += A[i * n + i] * A[i * n + i];
      double o = 0.0;
      for (int j = i + 1; j < n; ++j) o += A[i * n + j] * A[i * n + j];
      off += o;
    }
    if (!(off > 1e-24 * dia)) break;
    for (int r = 0; r < 11; ++r) {
      int pp[6], qq[6];
      double c[6], s[6];
      ep_pairs12(r, pp, qq);
      for (int i = 0; i < 6; ++i)
        ep_rot_cs(A[pp[i] * n + pp[i]], A[qq[i] * n + qq[i]], A[pp[i] * n + qq[i]], &c[i], &s[i]);
      for (int i = 0; i < 6; ++i)
        for (int k = 0; k < n; ++k) {  /* columns */
          const double akp = A[k * n + pp[i]], akq = A[k * n + qq[i]];
          A[k * n + pp[i]] = c[i] * akp - s[i] * akq;
          A[k * n + qq[i]] = s[i] * akp + c[i] * akq;
        }
      for (int i = 0; i < 6; ++i)
        for (int k = 0; k < n; ++k) {  /* rows */
          const double apk = A[pp[i] * n + k], aqk = A[qq[i] * n + k];
          A[pp[i] * n + k] = c[i] * apk - s[i] * aqk;
          A[qq[i] * n + k] = s[i] * apk + c[i] * aqk;
        }
      for (int i = 0; i < 6; ++i)
        for (int k = 0; k < n; ++k) {
          const double vkp = V[k * n + pp[i]], vkq = V[k * n + qq[i]];
          V[k * n + pp[i]] = c[i] * vkp - s[i] * vkq;
          V[k * n + qq[i]] = s[i] * vkp + c[i] * vkq;
        }
    }
  }
}

/* least squares x (k <= 5 unknowns) of the 6 x k system A x = b by the
 * normal equations (Cholesky); returns 0 when not positive definite */
static inline int ep_lsq6(const double* A, int k, const double* b, double* x) {
  double N[5][5], r[5];
  for (int i = 0; i < k; ++i) {
    for (int j = 0; j <= i; ++j) {
      double s = 0.0;
      for (int m = 0; m < 6; ++m) s += A[m * k + i] * A[m * k + j];
      N[i][j] = s;
    }
    double s = 0.0;
    for (int m = 0; m < 6; ++m) s += A[m * k + i] * b[m];
    r[i] = s;
  }
  for (int j = 0; j < k; ++j) {
    double s = N[j][j];
    for (int p = 0; p < j; ++p) s -= N[j][p] * N[j][p];
    if (!(s > 0.0)) return 0;
    N[j][j] = sqrt(s);
    for (int i = j + 1; i < k; ++i) {
      double t = N[i][j];
      for (int p = 0; p < j; ++p) t -= N[i][p] * N[j][p];
      N[i][j] = t / N[j][j];
    }
  }
  double y[5];
  for (int i = 0; i < k; ++i) {
    double t = r[i];
    for (int p = 0; p < i; ++p) t -= N[i][p] * y[p];
    y[i] = t / N[i][i];
  }
  for (int i = k - 1; i >= 0; --i) {
    double t = y[i];
    for (int p = i + 1; p < k; ++p) t -= N[p][i] * x[p];
    x[i] = t / N[i][i];
  }
  return 1;
}

/* pose from the 4 camera-frame control points ccs (betas applied): R, t and
 * the mean reprojection error over the n points */
static inline double ep_pose(const double ccs[4][3], const double* alph, const double* pw, int n,
                             const double* uv, double fx, double fy, double cx, double cy,
                             double R[9], double t[3]) {
  double pc[EPNP_MAXN][3] = {{0.0}};
  double cc[4][3];
  memcpy(cc, ccs, sizeof(cc));
  for (int i = 0; i < n; ++i)
    for (int d = 0; d < 3; ++d)
      pc[i][d] = alph[4 * i] * cc[0][d] + alph[4 * i + 1] * cc[1][d] + alph[4 * i + 2] * cc[2][d] +
                 alph[4 * i + 3] * cc[3][d];
  if (pc[0][2] < 0.0)
    for (int i = 0; i < n; ++i)
      for (int d = 0; d < 3; ++d) pc[i][d] = -pc[i][d];
  double c0[3] = {0, 0, 0}, w0[3] = {0, 0, 0};
  for (int i = 0; i < n; ++i)
    for (int d = 0; d < 3; ++d) {
      c0[d] += pc[i][d];
      w0[d] += pw[3 * i + d];
    }
  for (int d = 0; d < 3; ++d) {
    c0[d] /= n;
    w0[d] /= n;
  }
  double S[3][3] = {{0, 0, 0}, {0, 0, 0}, {0, 0, 0}};  /* S[a][b] = sum pw_a pc_b */
  for (int i = 0; i < n; ++i)
    for (int a = 0; a < 3; ++a)
      for (int b = 0; b < 3; ++b) S[a][b] += (pw[3 * i + a] - w0[a]) * (pc[i][b] - c0[b]);
  double N[16] = {S[0][0] + S[1][1] + S[2][2], S[1][2] - S[2][1], S[2][0] - S[0][2], S[0][1] - S[1][0],
                  S[1][2] - S[2][1], S[0][0] - S[1][1] - S[2][2], S[0][1] + S[1][0], S[2][0] + S[0][2],
                  S[2][0] - S[0][2], S[0][1] + S[1][0], -S[0][0] + S[1][1] - S[2][2], S[1][2] + S[2][1],
                  S[0][1] - S[1][0], S[2][0] + S[0][2], S[1][2] + S[2][1], -S[0][0] - S[1][1] + S[2][2]};
  double V[16];
  ep_jacobi(N, 4, V);
  int bi = 0;
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
  for (int d = 0; d < 3; ++d) t[d] = c0[d] - (R[3 * d] * w0[0] + R[3 * d + 1] * w0[1] + R[3 * d + 2] * w0[2]);
  double err = 0.0;
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
static inline void ep_rvec(const double R[9], double r[3]) {
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

/* EPnP on n (4..EPNP_MAXN) points pw [n][3] / uv [n][2] -> p = (rvec, t);
 * returns 1 on a finite pose */
static inline int epnp(const double* pw, const double* uv, int n, double fx, double fy, double cx,
                       double cy, double p[6]) {
  /* control points */
  double cw[4][3] = {{0, 0, 0}};
  for (int i = 0; i < n; ++i)
    for (int d = 0; d < 3; ++d) cw[0][d] += pw[3 * i + d];
  for (int d = 0; d < 3; ++d) cw[0][d] /= n;
  double A3[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0}, V3[9];
  for (int i = 0; i < n; ++i)
    for (int a = 0; a < 3; ++a)
      for (int b = 0; b < 3; ++b) A3[3 * a + b] += (pw[3 * i + a] - cw[0][a]) * (pw[3 * i + b] - cw[0][b]);
  ep_jacobi(A3, 3, V3);
  /* eigenvalues descending */
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
  /* barycentric coordinates: [c1-c0 c2-c0 c3-c0] a = X - c0 */
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
  double alph[4 * EPNP_MAXN];
  for (int i = 0; i < n; ++i) {
    const double x = pw[3 * i] - cw[0][0], y = pw[3 * i + 1] - cw[0][1], z = pw[3 * i + 2] - cw[0][2];
    const double a1 = (c00 * x + c01 * y + c02 * z) * id;
    const double a2 = (c10 * x + c11 * y + c12 * z) * id;
    const double a3 = (c20 * x + c21 * y + c22 * z) * id;
    alph[4 * i] = 1.0 - a1 - a2 - a3;
    alph[4 * i + 1] = a1;
    alph[4 * i + 2] = a2;
    alph[4 * i + 3] = a3;
  }
  /* M^T M (12 x 12) of the 2n projection rows */
  double MtM[144], V12[144];
  memset(MtM, 0, sizeof(MtM));
  for (int i = 0; i < n; ++i) {
    double m1[12], m2[12];
    for (int j = 0; j < 4; ++j) {
      const double a = alph[4 * i + j];
      m1[3 * j] = a * fx; m1[3 * j + 1] = 0.0; m1[3 * j + 2] = a * (cx - uv[2 * i]);
      m2[3 * j] = 0.0; m2[3 * j + 1] = a * fy; m2[3 * j + 2] = a * (cy - uv[2 * i + 1]);
    }
    for (int r = 0; r < 12; ++r)
      for (int c = 0; c < 12; ++c) MtM[12 * r + c] += m1[r] * m1[c] + m2[r] * m2[c];
  }
  ep_jacobi12_par(MtM, V12);
  /* the 4 eigenvectors of the smallest eigenvalues, ascending: v[0] smallest */
  int o12[12];
  for (int i = 0; i < 12; ++i) o12[i] = i;
  for (int i = 0; i < 4; ++i)
    for (int j = i + 1; j < 12; ++j)
      if (MtM[13 * o12[j]] < MtM[13 * o12[i]]) {
        const int tmp = o12[i]; o12[i] = o12[j]; o12[j] = tmp;
      }
  double v[4][12];
  for (int k = 0; k < 4; ++k)
    for (int r = 0; r < 12; ++r) v[k][r] = V12[12 * r + o12[k]];
  /* L (6 x 10) and rho (control point distances) */
  static const int pa[6] = {0, 0, 0, 1, 1, 2}, pb[6] = {1, 2, 3, 2, 3, 3};
  double L[60], rho[6];
  for (int j = 0; j < 6; ++j) {
    double dv[4][3];
    for (int k = 0; k < 4; ++k)
      for (int d = 0; d < 3; ++d) dv[k][d] = v[k][3 * pa[j] + d] - v[k][3 * pb[j] + d];
#define EP_DOT(a, b) (dv[a][0] * dv[b][0] + dv[a][1] * dv[b][1] + dv[a][2] * dv[b][2])
    L[10 * j + 0] = EP_DOT(0, 0);
    L[10 * j + 1] = 2.0 * EP_DOT(0, 1);
    L[10 * j + 2] = EP_DOT(1, 1);
    L[10 * j + 3] = 2.0 * EP_DOT(0, 2);
    L[10 * j + 4] = 2.0 * EP_DOT(1, 2);
    L[10 * j + 5] = EP_DOT(2, 2);
    L[10 * j + 6] = 2.0 * EP_DOT(0, 3);
    L[10 * j + 7] = 2.0 * EP_DOT(1, 3);
    L[10 * j + 8] = 2.0 * EP_DOT(2, 3);
    L[10 * j + 9] = EP_DOT(3, 3);
#undef EP_DOT
    double s = 0.0;
    for (int d = 0; d < 3; ++d) {
      const double e = cw[pa[j]][d] - cw[pb[j]][d];
      s += e * e;
    }
    rho[j] = s;
  }
  double best_err = INFINITY;
  int ok = 0;
  for (int approx = 0; approx < 3; ++approx) {
    static const int cols[3][5] = {{0, 1, 3, 6, 0}, {0, 1, 2, 0, 0}, {0, 1, 2, 3, 4}};
    static const int nk[3] = {4, 3, 5};
    const int k = nk[approx];
    double As[30], xb[5];
    for (int j = 0; j < 6; ++j)
      for (int c = 0; c < k; ++c) As[j * k + c] = L[10 * j + cols[approx][c]];
    if (!ep_lsq6(As, k, rho, xb)) continue;
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
    /* Gauss-Newton on the 4 betas (5 steps) */
    for (int it = 0; it < 5; ++it) {
      double Ag[24], bg[6], dx[4];
      for (int j = 0; j < 6; ++j) {
        const double* l = L + 10 * j;
        Ag[4 * j + 0] = 2.0 * l[0] * be[0] + l[1] * be[1] + l[3] * be[2] + l[6] * be[3];
        Ag[4 * j + 1] = l[1] * be[0] + 2.0 * l[2] * be[1] + l[4] * be[2] + l[7] * be[3];
        Ag[4 * j + 2] = l[3] * be[0] + l[4] * be[1] + 2.0 * l[5] * be[2] + l[8] * be[3];
        Ag[4 * j + 3] = l[6] * be[0] + l[7] * be[1] + l[8] * be[2] + 2.0 * l[9] * be[3];
        bg[j] = rho[j] - (l[0] * be[0] * be[0] + l[1] * be[0] * be[1] + l[2] * be[1] * be[1] +
                          l[3] * be[0] * be[2] + l[4] * be[1] * be[2] + l[5] * be[2] * be[2] +
                          l[6] * be[0] * be[3] + l[7] * be[1] * be[3] + l[8] * be[2] * be[3] +
                          l[9] * be[3] * be[3]);
      }
      if (!ep_lsq6(Ag, 4, bg, dx)) break;
      for (int c = 0; c < 4; ++c) be[c] += dx[c];
    }
    double ccs[4][3];
    for (int j = 0; j < 4; ++j)
      for (int d = 0; d < 3; ++d)
        ccs[j][d] = be[0] * v[0][3 * j + d] + be[1] * v[1][3 * j + d] + be[2] * v[2][3 * j + d] +
                    be[3] * v[3][3 * j + d];
    double R[9], t[3];
    const double err = ep_pose(ccs, alph, pw, n, uv, fx, fy, cx, cy, R, t);
    if (err < best_err) {  /* NaN errors never win */
      best_err = err;
      double r[3];
      ep_rvec(R, r);
      p[0] = r[0]; p[1] = r[1]; p[2] = r[2];
      p[3] = t[0]; p[4] = t[1]; p[5] = t[2];
      ok = 1;
    }
  }
  for (int i = 0; i < 6; ++i) ok &= isfinite(p[i]) != 0;
  return ok;
}

#endif
