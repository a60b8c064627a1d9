/*
 * ORACLE — test infrastructure only (see oracle/__init__.py).
 *
 * CPU restatement of the pose step of the reference's tracking loop:
 *   /root/reference/transformation.py:5-19  cv2.solvePnPRansac(Q, q, K, zeros(5))
 *     (defaults: SOLVEPNP_ITERATIVE, 100 iterations, 8 px, confidence 0.99)
 * OpenCV's RNG sequence and exact EPnP arithmetic are not reproducible here
 * (OpenCV absent; PARITY UNPINNED vs OpenCV), so the deterministic spec both
 * this oracle and the HIP kernel follow is:
 *   - n_hyp hypotheses; hypothesis h draws 5 distinct indices from a
 *     splitmix64 stream seeded with seed ^ (frame * C1) ^ (h * C2);
 *   - each hypothesis: EPnP on its 5 points (epnp.h: OpenCV's RANSAC kernel
 *     for SOLVEPNP_ITERATIVE is EPnP on 5-point samples), then LM (lambda
 *     1e-3, x0.1 / x10, Marquardt diagonal) from that pose on the same points,
 *     hyp_iters iterations (a degenerate sample starts LM from r = t = 0);
 *   - score = #points with squared reprojection error <= thresh^2; best = max
 *     score, lowest h on ties;
 *   - refinement: the same LM from the best hypothesis over its inlier set,
 *     refine_iters iterations (solvePnPRansac re-runs ITERATIVE on the inliers).
 * Returned rvec/tvec follow OpenCV: X_cam = R(rvec) X + tvec.
 */
#include <math.h>
#include <stdint.h>
#include <string.h>

#include "pose_util.h"
#include "epnp.h"

typedef struct { double fx, fy, cx, cy; } camk;

/* residual (projection - observation) and optional 2x6 Jacobian wrt (r, t) */
static void residual(const double p[6], const double R[9], const double* Q, const double* q,
                     const camk* K, double r[2], double J[2][6]) {
  const double X0 = Q[0], X1 = Q[1], X2 = Q[2];
  const double RX0 = R[0] * X0 + R[1] * X1 + R[2] * X2;
  const double RX1 = R[3] * X0 + R[4] * X1 + R[5] * X2;
  const double RX2 = R[6] * X0 + R[7] * X1 + R[8] * X2;
  const double Xc = RX0 + p[3], Yc = RX1 + p[4], Zc = RX2 + p[5];
  const double iz = 1.0 / Zc;
  r[0] = K->fx * (Xc * iz) + K->cx - q[0];
  r[1] = K->fy * (Yc * iz) + K->cy - q[1];
  if (!J) return;
  const double du[3] = {K->fx * iz, 0.0, -K->fx * Xc * iz * iz};
  const double dv[3] = {0.0, K->fy * iz, -K->fy * Yc * iz * iz};
  double D[3][3];
  const double w0 = p[0], w1 = p[1], w2 = p[2];
  const double th2 = w0 * w0 + w1 * w1 + w2 * w2;
  if (th2 < 1e-24) {
    D[0][0] = 0; D[0][1] = RX2; D[0][2] = -RX1;
    D[1][0] = -RX2; D[1][1] = 0; D[1][2] = RX0;
    D[2][0] = RX1; D[2][1] = -RX0; D[2][2] = 0;
  } else {
    /* d(R X)/dw = -R [X]x (w w^T + (R^T - I)[w]x) / |w|^2  (Gallego & Yezzi 2015) */
    const double W[3][3] = {{0.0, -w2, w1}, {w2, 0.0, -w0}, {-w1, w0, 0.0}};
    const double w[3] = {w0, w1, w2};
    double A[3][3], B[3][3];
    for (int i = 0; i < 3; ++i)
      for (int k = 0; k < 3; ++k) {
        double acc = w[i] * w[k];
        for (int j = 0; j < 3; ++j) acc += R[3 * j + i] * W[j][k];
        A[i][k] = acc - W[i][k];
      }
    const double Xs[3][3] = {{0.0, -X2, X1}, {X2, 0.0, -X0}, {-X1, X0, 0.0}};
    for (int i = 0; i < 3; ++i)
      for (int k = 0; k < 3; ++k) B[i][k] = Xs[i][0] * A[0][k] + Xs[i][1] * A[1][k] + Xs[i][2] * A[2][k];
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

/* LM over the points listed in idx (or all with sel[i] != 0 when idx == NULL) */
static void lm(const double* Q, const double* q, const int* idx, int n, const uint8_t* sel, int L,
               const camk* K, int iters, double p[6]) {
  double lam = 1e-3, R[9];
  for (int it = 0; it < iters; ++it) {
    rodrigues(p, R);
    double H[21] = {0}, g[6] = {0}, cost = 0.0;
    const int m = idx ? n : L;
    for (int s = 0; s < m; ++s) {
      const int i = idx ? idx[s] : s;
      if (!idx && !sel[i]) continue;
      double r[2], J[2][6];
      residual(p, R, Q + 3 * i, q + 2 * i, K, r, J);
      for (int a = 0; a < 2; ++a) {
        int k = 0;
        for (int u = 0; u < 6; ++u) {
          for (int v = 0; v <= u; ++v) H[k++] += J[a][u] * J[a][v];
          g[u] += J[a][u] * r[a];
        }
        cost += r[a] * r[a];
      }
    }
    double d[6], pn[6], Rn[9];
    if (!solve6(H, g, lam, d)) { lam = fmin(lam * 10.0, 1e12); continue; }
    for (int i = 0; i < 6; ++i) pn[i] = p[i] + d[i];
    rodrigues(pn, Rn);
    double cn = 0.0;
    for (int s = 0; s < m; ++s) {
      const int i = idx ? idx[s] : s;
      if (!idx && !sel[i]) continue;
      double r[2];
      residual(pn, Rn, Q + 3 * i, q + 2 * i, K, r, NULL);
      cn += r[0] * r[0] + r[1] * r[1];
    }
    if (cn < cost) {
      memcpy(p, pn, sizeof(pn));
      lam = fmax(lam * 0.1, 1e-12);
    } else {
      lam = fmin(lam * 10.0, 1e12);
    }
  }
}

/* EPnP on n (4..8) points: p = (rvec, t), X_cam = R(rvec) X + t; returns 1 if finite */
int oracle_epnp(const double* pw, const double* uv, int n, const double* Kmat, double* p) {
  if (n < 4 || n > EPNP_MAXN) return 0;
  return epnp(pw, uv, n, Kmat[0], Kmat[4], Kmat[2], Kmat[5], p);
}

/* returns #inliers of the chosen hypothesis, -1 if L < 5 */
int oracle_pnp_ransac(const double* Q, const double* q, int L, const double* Kmat, uint64_t seed,
                      int item, int n_hyp, double thresh, int hyp_iters, int refine_iters,
                      double* rvec, double* tvec, uint8_t* mask, double* hyp_out, int* hyp_cnt) {
  const camk K = {Kmat[0], Kmat[4], Kmat[2], Kmat[5]};
  if (L < 5) {
    memset(rvec, 0, 3 * sizeof(double));
    memset(tvec, 0, 3 * sizeof(double));
    memset(mask, 0, (size_t)L);
    return -1;
  }
  const double thr2 = thresh * thresh;
  int best = -1, bestc = -1;
  double bp[6] = {0};
  for (int h = 0; h < n_hyp; ++h) {
    uint64_t s = seed ^ ((uint64_t)item * 0xD1B54A32D192ED03ull) ^ ((uint64_t)h * 0x8CB92BA72F3D8DD7ull);
    int idx[5];
    for (int k = 0; k < 5; ++k) {
      int v, dup;
      do {
        v = (int)((splitmix64(&s) >> 32) % (uint64_t)L);
        dup = 0;
        for (int j = 0; j < k; ++j) dup |= idx[j] == v;
      } while (dup);
      idx[k] = v;
    }
    /* EPnP seed on the sample (OpenCV's RANSAC kernel for ITERATIVE), then LM
       on the same 5 points; a degenerate sample starts LM from r = t = 0 */
    double p[6] = {0, 0, 0, 0, 0, 0}, R[9];
    {
      double pw[15], uv[10];
      for (int k = 0; k < 5; ++k) {
        memcpy(pw + 3 * k, Q + 3 * idx[k], 3 * sizeof(double));
        memcpy(uv + 2 * k, q + 2 * idx[k], 2 * sizeof(double));
      }
      if (!epnp(pw, uv, 5, K.fx, K.fy, K.cx, K.cy, p)) memset(p, 0, sizeof(p));
    }
    lm(Q, q, idx, 5, NULL, L, &K, hyp_iters, p);
    int c = 0;
    int finite = 1;
    for (int i = 0; i < 6; ++i) finite &= isfinite(p[i]) != 0;
    if (finite) {
      rodrigues(p, R);
      for (int i = 0; i < L; ++i) {
        double r[2];
        residual(p, R, Q + 3 * i, q + 2 * i, &K, r, NULL);
        c += (r[0] * r[0] + r[1] * r[1] <= thr2);
      }
    }
    if (hyp_out) memcpy(hyp_out + 6 * h, p, sizeof(p));
    if (hyp_cnt) hyp_cnt[h] = c;
    if (c > bestc) { bestc = c; best = h; memcpy(bp, p, sizeof(p)); }
  }
  double R[9];
  rodrigues(bp, R);
  for (int i = 0; i < L; ++i) {
    double r[2];
    residual(bp, R, Q + 3 * i, q + 2 * i, &K, r, NULL);
    mask[i] = (r[0] * r[0] + r[1] * r[1] <= thr2);
  }
  (void)best;
  lm(Q, q, NULL, 0, mask, L, &K, refine_iters, bp);
  memcpy(rvec, bp, 3 * sizeof(double));
  memcpy(tvec, bp + 3, 3 * sizeof(double));
  return bestc;
}
