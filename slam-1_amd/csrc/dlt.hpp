// DLT triangulation helper shared by geometry.hip (cv2.triangulatePoints,
// Point3D.py:14-19) and vofront.hip (calc_3d, visual_odometry.py:129-134).
#pragma once

#include <hip/hip_runtime.h>

namespace {

// Null vector of the 4x4 DLT matrix by one-sided (Hestenes) Jacobi SVD in f64.
__device__ __forceinline__ void null_vector4(double A[4][4], double v[4]) {
  double V[4][4] = {{1, 0, 0, 0}, {0, 1, 0, 0}, {0, 0, 1, 0}, {0, 0, 0, 1}};
  for (int sweep = 0; sweep < 12; ++sweep) {
    double off = 0.0;
#pragma unroll
    for (int p = 0; p < 3; ++p)
#pragma unroll
      for (int q = p + 1; q < 4; ++q) {
        double al = 0, be = 0, ga = 0;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          al += A[i][p] * A[i][p];
          be += A[i][q] * A[i][q];
          ga += A[i][p] * A[i][q];
        }
        const double den = sqrt(al * be);
        if (den == 0.0 || fabs(ga) <= 1e-15 * den) continue;
        off = fmax(off, fabs(ga) / den);
        const double zeta = (be - al) / (2.0 * ga);
        const double tt = (zeta >= 0 ? 1.0 : -1.0) / (fabs(zeta) + sqrt(1.0 + zeta * zeta));
        const double c = 1.0 / sqrt(1.0 + tt * tt), s = c * tt;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const double ap = A[i][p], aq = A[i][q];
          A[i][p] = c * ap - s * aq;
          A[i][q] = s * ap + c * aq;
          const double vp = V[i][p], vq = V[i][q];
          V[i][p] = c * vp - s * vq;
          V[i][q] = s * vp + c * vq;
        }
      }
    if (off < 1e-15) break;
  }
  int best = 0;
  double bn = 1e300;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    double nn = 0;
#pragma unroll
    for (int i = 0; i < 4; ++i) nn += A[i][j] * A[i][j];
    if (nn < bn) {
      bn = nn;
      best = j;
    }
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    double x = V[i][0];
#pragma unroll
    for (int j = 1; j < 4; ++j) x = best == j ? V[i][j] : x;  // no dynamic register index
    v[i] = x;
  }
}

}  // namespace
