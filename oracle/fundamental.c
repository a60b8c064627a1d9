/*
 * ORACLE — test infrastructure only (see oracle/__init__.py).
 *
 * CPU restatement of the stereo outlier filter of the reference:
 *   /root/reference/keypoint.py:59-66
 *     F, mask = cv2.findFundamentalMat(pts_left, pts_right, cv2.FM_LMEDS)
 *     pts_left = pts_left[mask] ...
 * OpenCV (absent here; PARITY UNPINNED vs OpenCV) runs LMeDS over random
 * 7-point samples.  The deterministic spec shared with csrc/fundamental.hip:
 *   - M < 8 matches: no model, empty mask;
 *   - n_hyp = 300 hypotheses (OpenCV's LMeDS count for confidence 0.99 and
 *     outlier ratio 0.45: cvRound(log(0.01) / log(1 - 0.55^7)));
 *   - hypothesis h draws 7 distinct indices from splitmix64 seeded with
 *     seed ^ (frame * C1) ^ (h * C3);
 *   - 7-point algorithm on Hartley-normalised points: 2-D null space of the 7x9
 *     system by Gauss-Jordan with full pivoting, det(a F1 + (1-a) F2) = 0 from
 *     its values at a = 0, 1, -1, 2, real roots ascending (Cardano /
 *     trigonometric + 2 Newton steps), denormalised, scaled to unit Frobenius norm;
 *   - error (OpenCV FMEstimatorCallback::computeError), as float:
 *     max(d1^2 / (a1^2 + b1^2), d2^2 / (a2^2 + b2^2));
 *   - LMedS: median = sorted_err[M/2]; best = min median over candidates in
 *     (h, root) order, first on ties;
 *   - inliers: err <= sigma^2, sigma = max(2.5 * 1.4826 * (1 + 5/(M-7)) * sqrt(median), 0.001).
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#define FM_SAMPLE 7

static uint64_t splitmix64(uint64_t* s) {
  *s += 0x9E3779B97F4A7C15ull;
  uint64_t z = *s;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

static double det3(const double* F) {
  return F[0] * (F[4] * F[8] - F[5] * F[7]) - F[1] * (F[3] * F[8] - F[5] * F[6]) +
         F[2] * (F[3] * F[7] - F[4] * F[6]);
}

static double detmix(const double* F1, const double* F2, double a) {
  double F[9];
  for (int i = 0; i < 9; ++i) F[i] = a * F1[i] + (1.0 - a) * F2[i];
  return det3(F);
}

/* real roots of c3 x^3 + c2 x^2 + c1 x + c0, ascending; returns count */
static int cubic_roots(double c3, double c2, double c1, double c0, double* r) {
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
    r[n++] = q / c2;
    if (q != 0.0) r[n++] = c0 / q;
  } else {
    const double a = c2 / c3, b = c1 / c3, c = c0 / c3;
    const double p = b - a * a / 3.0;
    const double q = 2.0 * a * a * a / 27.0 - a * b / 3.0 + c;
    const double disc = q * q / 4.0 + p * p * p / 27.0;
    if (disc > 0) {
      const double sd = sqrt(disc);
      const double u = cbrt(-q / 2.0 + sd), v = cbrt(-q / 2.0 - sd);
      r[n++] = u + v - a / 3.0;
    } else {
      const double rr = sqrt(fmax(-p / 3.0, 0.0));
      double ca = rr > 0 ? -q / (2.0 * rr * rr * rr) : 0.0;
      ca = fmin(fmax(ca, -1.0), 1.0);
      const double phi = acos(ca);
      for (int k = 0; k < 3; ++k)
        r[n++] = 2.0 * rr * cos((phi + 2.0 * 3.14159265358979323846 * k) / 3.0) - a / 3.0;
    }
  }
  for (int i = 0; i < n; ++i)
    for (int it = 0; it < 2; ++it) {
      const double x = r[i];
      const double f = ((c3 * x + c2) * x + c1) * x + c0;
      const double df = (3.0 * c3 * x + 2.0 * c2) * x + c1;
      if (df != 0.0) r[i] = x - f / df;
    }
  for (int i = 1; i < n; ++i)
    for (int j = i; j > 0 && r[j] < r[j - 1]; --j) {
      const double t = r[j]; r[j] = r[j - 1]; r[j - 1] = t;
    }
  return n;
}

/* 7-point algorithm; returns the number of candidates written to F (9 each) */
int oracle_fm_7point(const double* m1, const double* m2, const int* idx, double* Fout) {
  double c1x = 0, c1y = 0, c2x = 0, c2y = 0;
  for (int i = 0; i < FM_SAMPLE; ++i) {
    c1x += m1[2 * idx[i]]; c1y += m1[2 * idx[i] + 1];
    c2x += m2[2 * idx[i]]; c2y += m2[2 * idx[i] + 1];
  }
  c1x /= FM_SAMPLE; c1y /= FM_SAMPLE; c2x /= FM_SAMPLE; c2y /= FM_SAMPLE;
  double d1 = 0, d2 = 0;
  for (int i = 0; i < FM_SAMPLE; ++i) {
    d1 += sqrt((m1[2 * idx[i]] - c1x) * (m1[2 * idx[i]] - c1x) +
               (m1[2 * idx[i] + 1] - c1y) * (m1[2 * idx[i] + 1] - c1y));
    d2 += sqrt((m2[2 * idx[i]] - c2x) * (m2[2 * idx[i]] - c2x) +
               (m2[2 * idx[i] + 1] - c2y) * (m2[2 * idx[i] + 1] - c2y));
  }
  d1 /= FM_SAMPLE; d2 /= FM_SAMPLE;
  if (!(d1 > 1e-12) || !(d2 > 1e-12)) return 0;
  const double s1 = sqrt(2.0) / d1, s2 = sqrt(2.0) / d2;
  double A[7][9];
  for (int i = 0; i < FM_SAMPLE; ++i) {
    const double x1 = (m1[2 * idx[i]] - c1x) * s1, y1 = (m1[2 * idx[i] + 1] - c1y) * s1;
    const double x2 = (m2[2 * idx[i]] - c2x) * s2, y2 = (m2[2 * idx[i] + 1] - c2y) * s2;
    const double row[9] = {x2 * x1, x2 * y1, x2, y2 * x1, y2 * y1, y2, x1, y1, 1.0};
    memcpy(A[i], row, sizeof(row));
  }
  /* Gauss-Jordan with full pivoting */
  int pc[7], used[9] = {0};
  for (int r = 0; r < 7; ++r) {
    int bi = -1, bj = -1;
    double bv = 0.0;
    for (int i = r; i < 7; ++i)
      for (int j = 0; j < 9; ++j)
        if (!used[j] && fabs(A[i][j]) > bv) { bv = fabs(A[i][j]); bi = i; bj = j; }
    if (bv < 1e-10) return 0;
    if (bi != r)
      for (int j = 0; j < 9; ++j) { const double t = A[r][j]; A[r][j] = A[bi][j]; A[bi][j] = t; }
    used[bj] = 1;
    pc[r] = bj;
    const double inv = 1.0 / A[r][bj];
    for (int j = 0; j < 9; ++j) A[r][j] *= inv;
    for (int i = 0; i < 7; ++i) {
      if (i == r) continue;
      const double f = A[i][bj];
      if (f != 0.0)
        for (int j = 0; j < 9; ++j) A[i][j] -= f * A[r][j];
    }
  }
  int fr[2], nf = 0;
  for (int j = 0; j < 9; ++j)
    if (!used[j]) fr[nf++] = j;
  double F1[9], F2[9];
  for (int k = 0; k < 2; ++k) {
    double* f = k ? F2 : F1;
    for (int j = 0; j < 9; ++j) f[j] = 0.0;
    f[fr[k]] = 1.0;
    for (int r = 0; r < 7; ++r) f[pc[r]] = -A[r][fr[k]];
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
  for (int k = 0; k < nr; ++k) {
    double Fn[9], tmp[9], F[9];
    for (int i = 0; i < 9; ++i) Fn[i] = roots[k] * F1[i] + (1.0 - roots[k]) * F2[i];
    /* F = T2^T Fn T1 */
    for (int i = 0; i < 3; ++i)
      for (int j = 0; j < 3; ++j)
        tmp[3 * i + j] = Fn[3 * i] * T1[j] + Fn[3 * i + 1] * T1[3 + j] + Fn[3 * i + 2] * T1[6 + j];
    for (int i = 0; i < 3; ++i)
      for (int j = 0; j < 3; ++j)
        F[3 * i + j] = T2[i] * tmp[j] + T2[3 + i] * tmp[3 + j] + T2[6 + i] * tmp[6 + j];
    double nrm = 0.0;
    for (int i = 0; i < 9; ++i) nrm += F[i] * F[i];
    nrm = sqrt(nrm);
    if (!(nrm > 0.0) || !isfinite(nrm)) continue;
    for (int i = 0; i < 9; ++i) Fout[9 * n + i] = F[i] / nrm;
    ++n;
  }
  return n;
}

static float fm_error(const double* F, const double* p1, const double* p2) {
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
  return isnan(e) ? INFINITY : e; /* degenerate epipolar line: never an inlier */
}

static int cmp_f(const void* a, const void* b) {
  const float x = *(const float*)a, y = *(const float*)b;
  return (x > y) - (x < y);
}

/* Returns #inliers (-1 if M < 8 or no model); mask [M]; F [9] */
int oracle_fm_lmeds(const double* m1, const double* m2, int M, uint64_t seed, int item, int n_hyp,
                    uint8_t* mask, double* Fbest, float* med_out) {
  memset(mask, 0, (size_t)M);
  if (M < 8) return -1;
  float* err = (float*)malloc(sizeof(float) * M);
  float* srt = (float*)malloc(sizeof(float) * M);
  float best = INFINITY;
  int have = 0;
  for (int h = 0; h < n_hyp; ++h) {
    uint64_t s = seed ^ ((uint64_t)item * 0xD1B54A32D192ED03ull) ^ ((uint64_t)h * 0x9FB21C651E98DF25ull);
    int idx[FM_SAMPLE];
    for (int k = 0; k < FM_SAMPLE; ++k) {
      int v, dup;
      do {
        v = (int)((splitmix64(&s) >> 32) % (uint64_t)M);
        dup = 0;
        for (int j = 0; j < k; ++j) dup |= idx[j] == v;
      } while (dup);
      idx[k] = v;
    }
    double F[27];
    const int nc = oracle_fm_7point(m1, m2, idx, F);
    for (int k = 0; k < nc; ++k) {
      for (int i = 0; i < M; ++i) srt[i] = fm_error(F + 9 * k, m1 + 2 * i, m2 + 2 * i);
      qsort(srt, M, sizeof(float), cmp_f);
      const float med = srt[M / 2];
      if (med < best) {
        best = med;
        have = 1;
        memcpy(Fbest, F + 9 * k, 9 * sizeof(double));
      }
    }
  }
  int n = -1;
  if (have) {
    double sigma = 2.5 * 1.4826 * (1 + 5.0 / (M - FM_SAMPLE)) * sqrt((double)best);
    sigma = fmax(sigma, 0.001);
    const double thr = sigma * sigma;
    n = 0;
    for (int i = 0; i < M; ++i) {
      err[i] = fm_error(Fbest, m1 + 2 * i, m2 + 2 * i);
      mask[i] = (double)err[i] <= thr;
      n += mask[i];
    }
    if (med_out) *med_out = best;
  }
  free(err);
  free(srt);
  return n;
}
