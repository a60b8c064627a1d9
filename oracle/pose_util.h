/*
 * ORACLE — test infrastructure only (see oracle/__init__.py).
 * Helpers shared by the pose oracles (geometry.c: PnP, vo.c: stereo VO pose):
 * the splitmix64 hypothesis stream, cv2.Rodrigues, and the damped 6x6
 * Cholesky solve of the LM steps.  The HIP kernels (csrc/geometry.hip) state
 * the same operations in the same order.
 */
#ifndef SLAM_ORACLE_POSE_UTIL_H
#define SLAM_ORACLE_POSE_UTIL_H
#include <math.h>
#include <stdint.h>
#include <string.h>

static inline uint64_t splitmix64(uint64_t* s) {
  *s += 0x9E3779B97F4A7C15ull;
  uint64_t z = *s;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

static inline void rodrigues(const double r[3], double R[9]) {
  const double th = sqrt(r[0] * r[0] + r[1] * r[1] + r[2] * r[2]);
  if (th < 2.220446049250313e-16) {
    memset(R, 0, 9 * sizeof(double));
    R[0] = R[4] = R[8] = 1.0;
    return;
  }
  const double c = cos(th), s = sin(th), c1 = 1.0 - c, it = 1.0 / th;
  const double x = r[0] * it, y = r[1] * it, z = r[2] * it;
  R[0] = c + c1 * x * x; R[1] = c1 * x * y - s * z; R[2] = c1 * x * z + s * y;
  R[3] = c1 * x * y + s * z; R[4] = c + c1 * y * y; R[5] = c1 * y * z - s * x;
  R[6] = c1 * x * z - s * y; R[7] = c1 * y * z + s * x; R[8] = c + c1 * z * z;
}

static inline int solve6(const double H[21], const double g[6], double lam, double d[6]) {
  double A[6][6];
  int k = 0;
  for (int i = 0; i < 6; ++i)
    for (int j = 0; j <= i; ++j) { A[i][j] = A[j][i] = H[k]; ++k; }
  for (int i = 0; i < 6; ++i) A[i][i] += lam * fmax(A[i][i], 1e-12);
  for (int j = 0; j < 6; ++j) {
    double s = A[j][j];
    for (int p = 0; p < j; ++p) s -= A[j][p] * A[j][p];
    if (!(s > 0.0)) return 0;
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
  return 1;
}

#endif
