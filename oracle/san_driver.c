/* ORACLE sanitizer driver (test infrastructure only).
 *
 * Built by `make -C oracle san` with -fsanitize=address,undefined and linked
 * directly against the oracle sources (no LD_PRELOAD, no Python), then run.
 * It drives every oracle entry point the parity tests use through ordinary
 * and edge inputs: ORB on textured, flat, tiny and overflowing images; kNN-2
 * on empty / single / duplicate train sets; F-LMedS below and at the 8-point
 * minimum and with an all-duplicate sample; PnP with L < 5, degenerate
 * (coplanar / coincident) samples and large motion; EPnP on 4..8 points and
 * collinear input; VO pose with N = 0 and N = 3; FAST tiles with cap = 0;
 * LK at the borders; SGBM on a narrow image.  Any heap/stack overflow, use
 * after free, leak or UB aborts with a report; the exit status is 0 only when
 * every case ran clean.  tests/test_sanitize.py runs it on the CPU. */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

int oracle_orb_tiles(const uint8_t* img, int H, int W, int stride, int max_kp, int overlap_div,
                     int height_div, int width_div, const int8_t* pattern, float* kp,
                     int32_t* octave, uint8_t* desc, int cap);
void oracle_orb_tiles_batch(const uint8_t* img, int B, int H, int W, int stride, int max_kp,
                            const int8_t* pattern, float* kp, int32_t* octave, uint8_t* desc,
                            int cap, int32_t* counts);
void oracle_hamming_knn2(const uint8_t* q, int nq, const uint8_t* t, int nt, int32_t* idx2,
                         int32_t* dist2, uint8_t* good);
int oracle_fm_lmeds(const double* m1, const double* m2, int M, uint64_t seed, int item, int n_hyp,
                    uint8_t* mask, double* Fbest, float* med_out);
int oracle_epnp(const double* pw, const double* uv, int n, const double* Kmat, double* p);
int oracle_pnp_ransac(const double* Q, const double* q, int L, const double* Kmat, uint64_t seed,
                      int item, int n_hyp, double thresh, int hyp_iters, int refine_iters,
                      double* rvec, double* tvec, uint8_t* mask, double* hyp_out, int* hyp_cnt);
int oracle_vo_estimate_pose(const double* q1, const double* q2, const double* Q1, const double* Q2,
                            int N, const double* P, uint64_t seed, int item, int max_iter,
                            int lm_iters, int early_stop, double* pose, int* ntried, double* err,
                            double* errs);
int oracle_fast_tiles(const uint8_t* img, int H, int W, int stride, int tile_h, int tile_w,
                      int threshold, int per_tile, float* out, int cap);
void oracle_lk_track(const uint8_t* prev, const uint8_t* next, int H, int W, const float* pts,
                     int n, int win, int max_level, int max_count, double eps, float min_eig,
                     float* out, uint8_t* status, float* err);
void oracle_sgbm(const uint8_t* L, const uint8_t* R, int H, int W, int minD, int numD, int block,
                 int P1, int P2, int16_t* disp);

static uint64_t rng = 0x9E3779B97F4A7C15ull;
static uint32_t rnd(void) {
  rng ^= rng << 13;
  rng ^= rng >> 7;
  rng ^= rng << 17;
  return (uint32_t)(rng >> 16);
}
static double urand(void) { return (rnd() & 0xFFFFFF) / (double)0x1000000; }

static int fails = 0;
#define CHECK(c, ...)                                   \
  do {                                                  \
    if (!(c)) {                                         \
      fprintf(stderr, "FAIL %s:%d: ", __FILE__, __LINE__); \
      fprintf(stderr, __VA_ARGS__);                     \
      fputc('\n', stderr);                              \
      ++fails;                                          \
    }                                                   \
  } while (0)

static int load_pattern(const char* path, int8_t* pat) {
  FILE* f = fopen(path, "r");
  if (!f) return 0;
  char line[256];
  int n = 0;
  while (n < 1024 && fgets(line, sizeof line, f)) {
    if (line[0] == '#') continue;
    int a, b, c, d;
    if (sscanf(line, "%d %d %d %d", &a, &b, &c, &d) == 4) {
      pat[n++] = (int8_t)a;
      pat[n++] = (int8_t)b;
      pat[n++] = (int8_t)c;
      pat[n++] = (int8_t)d;
    }
  }
  fclose(f);
  return n == 1024;
}

/* blocky texture plus dots: plenty of FAST corners */
static void texture(uint8_t* im, int H, int W, int stride, int cell) {
  for (int y = 0; y < H; ++y)
    for (int x = 0; x < W; ++x) {
      uint32_t h = (uint32_t)(x / cell) * 73856093u ^ (uint32_t)(y / cell) * 19349663u;
      h ^= h >> 13;
      h *= 0x5bd1e995u;
      im[(size_t)y * stride + x] = (uint8_t)(40 + (h >> 24) % 180);
    }
}

static void case_orb(const int8_t* pat) {
  const int H = 376, W = 1241, stride = 1248, cap = 4096;
  uint8_t* im = (uint8_t*)malloc((size_t)H * stride * 2);
  texture(im, H, W, stride, 5);
  texture(im + (size_t)H * stride, H, W, stride, 9);
  float* kp = (float*)malloc(sizeof(float) * 5 * cap * 2);
  int32_t* oc = (int32_t*)malloc(sizeof(int32_t) * cap * 2);
  uint8_t* desc = (uint8_t*)malloc((size_t)32 * cap * 2);
  int32_t counts[2];
  oracle_orb_tiles_batch(im, 2, H, W, stride, 64, pat, kp, oc, desc, cap, counts);
  CHECK(counts[0] > 100 && counts[1] > 100, "orb batch counts %d %d", counts[0], counts[1]);
  for (int i = 0; i < counts[0]; ++i)
    CHECK(kp[5 * i] >= 0 && kp[5 * i] < W && kp[5 * i + 1] >= 0 && kp[5 * i + 1] < H,
          "orb kp %d out of image", i);
  /* overflow: cap far below the count -> negative return, nothing past cap */
  const int small = 37;
  float* kps = (float*)malloc(sizeof(float) * 5 * small);
  int32_t* ocs = (int32_t*)malloc(sizeof(int32_t) * small);
  uint8_t* ds = (uint8_t*)malloc((size_t)32 * small);
  int n = oracle_orb_tiles(im, H, W, stride, 64, 2, 5, 10, pat, kps, ocs, ds, small);
  CHECK(n < 0 && -n - 1 <= small, "orb overflow returned %d", n);
  n = oracle_orb_tiles(im, H, W, stride, 64, 2, 5, 10, pat, kps, ocs, ds, 0);
  CHECK(n <= 0, "orb cap 0 returned %d", n);
  /* flat image: no corners */
  memset(im, 128, (size_t)H * stride);
  n = oracle_orb_tiles(im, H, W, stride, 64, 2, 5, 10, pat, kp, oc, desc, cap);
  CHECK(n == 0, "orb flat returned %d", n);
  /* tiny image (tiles smaller than the FAST/descriptor border) and whole-image mode */
  texture(im, 40, 64, 64, 3);
  n = oracle_orb_tiles(im, 40, 64, 64, 64, 2, 5, 10, pat, kp, oc, desc, cap);
  CHECK(n >= 0, "orb tiny returned %d", n);
  n = oracle_orb_tiles(im, 40, 64, 64, 500, 2, 0, 0, pat, kp, oc, desc, cap);
  CHECK(n >= 0, "orb whole-image tiny returned %d", n);
  free(kps), free(ocs), free(ds), free(im), free(kp), free(oc), free(desc);
}

static void case_knn(void) {
  const int nq = 300, nt = 257;
  uint8_t* q = (uint8_t*)malloc(32 * nq);
  uint8_t* t = (uint8_t*)malloc(32 * nt);
  for (int i = 0; i < 32 * nq; ++i) q[i] = (uint8_t)rnd();
  for (int i = 0; i < 32 * nt; ++i) t[i] = (uint8_t)rnd();
  memcpy(t + 32 * 5, q + 32 * 7, 32);
  int32_t* idx = (int32_t*)malloc(sizeof(int32_t) * 2 * nq);
  int32_t* dist = (int32_t*)malloc(sizeof(int32_t) * 2 * nq);
  uint8_t* good = (uint8_t*)malloc(nq);
  oracle_hamming_knn2(q, nq, t, nt, idx, dist, good);
  CHECK(idx[14] == 5 && dist[14] == 0, "knn exact match idx %d dist %d", idx[14], dist[14]);
  oracle_hamming_knn2(q, nq, t, 1, idx, dist, good);
  CHECK(idx[1] == -1, "knn nt=1 second neighbour %d", idx[1]);
  oracle_hamming_knn2(q, nq, t, 0, idx, dist, good);
  CHECK(idx[0] == -1 && idx[1] == -1, "knn nt=0");
  oracle_hamming_knn2(q, 0, t, nt, idx, dist, good);
  /* all-equal train rows: ties resolve to the lowest index */
  for (int j = 0; j < 4; ++j) memcpy(t + 32 * j, q, 32);
  oracle_hamming_knn2(q, 1, t, 4, idx, dist, good);
  CHECK(idx[0] == 0 && idx[1] == 1, "knn ties %d %d", idx[0], idx[1]);
  free(q), free(t), free(idx), free(dist), free(good);
}

static void project(const double* K, const double* R, const double* t, const double* X,
                    double* uv) {
  double c[3];
  for (int r = 0; r < 3; ++r) c[r] = R[3 * r] * X[0] + R[3 * r + 1] * X[1] + R[3 * r + 2] * X[2] + t[r];
  uv[0] = K[0] * c[0] / c[2] + K[2];
  uv[1] = K[4] * c[1] / c[2] + K[5];
}

static void case_fm(void) {
  const double K[9] = {700, 0, 600, 0, 700, 180, 0, 0, 1};
  const double I[9] = {1, 0, 0, 0, 1, 0, 0, 0, 1}, t0[3] = {0, 0, 0};
  const double a = 0.05, R[9] = {cos(a), 0, sin(a), 0, 1, 0, -sin(a), 0, cos(a)};
  const double t1[3] = {-0.4, 0.02, 0.1};
  enum { M = 200 };
  double m1[2 * M], m2[2 * M], F[9];
  uint8_t mask[M];
  float med;
  for (int i = 0; i < M; ++i) {
    double X[3] = {urand() * 8 - 4, urand() * 4 - 2, 4 + urand() * 20};
    project(K, I, t0, X, m1 + 2 * i);
    project(K, R, t1, X, m2 + 2 * i);
    if (i % 5 == 0) m2[2 * i] += 30 + 40 * urand();
  }
  int n = oracle_fm_lmeds(m1, m2, M, 7, 0, 300, mask, F, &med);
  CHECK(n >= M * 3 / 4, "fm inliers %d", n);
  n = oracle_fm_lmeds(m1, m2, 7, 7, 0, 300, mask, F, &med);
  CHECK(n == -1, "fm M=7 returned %d", n);
  n = oracle_fm_lmeds(m1, m2, 8, 7, 0, 50, mask, F, &med);
  CHECK(n >= -1 && n <= 8, "fm M=8 returned %d", n);
  for (int i = 1; i < 12; ++i) memcpy(m1 + 2 * i, m1, 16), memcpy(m2 + 2 * i, m2, 16);
  n = oracle_fm_lmeds(m1, m2, 12, 7, 0, 50, mask, F, &med);
  CHECK(n >= -1 && n <= 12, "fm duplicates returned %d", n);
}

static void case_pnp(void) {
  const double K[9] = {700, 0, 600, 0, 700, 180, 0, 0, 1};
  enum { L = 160 };
  double Q[3 * L], q[2 * L], rvec[3], tvec[3], hyp[6 * 64];
  uint8_t mask[L];
  int cnt[64];
  /* large motion: 0.6 rad about y, 1.5 m translation */
  const double a = 0.6, R[9] = {cos(a), 0, sin(a), 0, 1, 0, -sin(a), 0, cos(a)};
  const double t[3] = {1.2, -0.3, 0.8};
  for (int i = 0; i < L; ++i) {
    double* X = Q + 3 * i;
    X[0] = urand() * 6 - 3, X[1] = urand() * 3 - 1.5, X[2] = 5 + urand() * 15;
    project(K, R, t, X, q + 2 * i);
    if (i % 6 == 0) q[2 * i + 1] += 25;
  }
  int n = oracle_pnp_ransac(Q, q, L, K, 3, 0, 64, 2.0, 10, 10, rvec, tvec, mask, hyp, cnt);
  CHECK(n >= L * 3 / 4, "pnp inliers %d", n);
  CHECK(fabs(rvec[1] - a) < 1e-6 && fabs(tvec[0] - t[0]) < 1e-6, "pnp pose %g %g", rvec[1],
        tvec[0]);
  n = oracle_pnp_ransac(Q, q, 4, K, 3, 0, 8, 2.0, 10, 10, rvec, tvec, mask, NULL, NULL);
  CHECK(n == -1, "pnp L=4 returned %d", n);
  /* every point coincident: all samples degenerate */
  for (int i = 1; i < 12; ++i) memcpy(Q + 3 * i, Q, 24), memcpy(q + 2 * i, q, 16);
  n = oracle_pnp_ransac(Q, q, 12, K, 3, 0, 16, 2.0, 10, 10, rvec, tvec, mask, hyp, cnt);
  CHECK(n >= 0, "pnp coincident returned %d", n);
  /* EPnP: 4..8 exact points, then collinear */
  for (int i = 0; i < 8; ++i) {
    double* X = Q + 3 * i;
    X[0] = urand() * 6 - 3, X[1] = urand() * 3 - 1.5, X[2] = 5 + urand() * 15;
    project(K, R, t, X, q + 2 * i);
  }
  for (int m = 4; m <= 8; ++m) {
    double p[6];
    int ok = oracle_epnp(Q, q, m, K, p);
    CHECK(ok && fabs(p[1] - a) < (m == 4 ? 1e-2 : 1e-5), "epnp n=%d ok=%d ry=%g", m, ok, p[1]);
  }
  double p[6];
  CHECK(oracle_epnp(Q, q, 3, K, p) == 0, "epnp n=3 accepted");
  CHECK(oracle_epnp(Q, q, 9, K, p) == 0, "epnp n=9 accepted");
  for (int i = 0; i < 6; ++i) {
    Q[3 * i] = i, Q[3 * i + 1] = 0.5 * i, Q[3 * i + 2] = 8 + i;
    project(K, R, t, Q + 3 * i, q + 2 * i);
  }
  (void)oracle_epnp(Q, q, 6, K, p); /* collinear: any return, no fault */
}

static void case_vo(void) {
  const double P[12] = {700, 0, 600, 0, 0, 700, 180, 0, 0, 0, 1, 0};
  enum { N = 80 };
  double q1[2 * N], q2[2 * N], Q1[3 * N], Q2[3 * N], pose[6], err, errs[32];
  int ntried;
  for (int i = 0; i < N; ++i) {
    double* X = Q1 + 3 * i;
    X[0] = urand() * 6 - 3, X[1] = urand() * 3 - 1.5, X[2] = 5 + urand() * 15;
    Q2[3 * i] = X[0] + 0.1, Q2[3 * i + 1] = X[1], Q2[3 * i + 2] = X[2] - 0.8;
    q1[2 * i] = 700 * X[0] / X[2] + 600, q1[2 * i + 1] = 700 * X[1] / X[2] + 180;
    q2[2 * i] = 700 * Q2[3 * i] / Q2[3 * i + 2] + 600;
    q2[2 * i + 1] = 700 * Q2[3 * i + 1] / Q2[3 * i + 2] + 180;
  }
  int r = oracle_vo_estimate_pose(q1, q2, Q1, Q2, N, P, 1, 0, 32, 200, 5, pose, &ntried, &err, errs);
  CHECK(r >= 0 && err < 1e-3, "vo pose r=%d err=%g", r, err);
  r = oracle_vo_estimate_pose(q1, q2, Q1, Q2, 0, P, 1, 0, 32, 200, 5, pose, &ntried, &err, errs);
  CHECK(r == -1, "vo N=0 returned %d", r);
  (void)oracle_vo_estimate_pose(q1, q2, Q1, Q2, 3, P, 1, 0, 8, 50, 5, pose, &ntried, &err, errs);
}

static void case_front(void) {
  const int H = 96, W = 200;
  uint8_t* a = (uint8_t*)malloc((size_t)H * W);
  uint8_t* b = (uint8_t*)malloc((size_t)H * W);
  texture(a, H, W, W, 4);
  for (int y = 0; y < H; ++y)
    for (int x = 0; x < W; ++x) b[y * W + x] = a[y * W + (x + 2 < W ? x + 2 : W - 1)];
  float fast[3 * 64];
  int n = oracle_fast_tiles(a, H, W, W, 10, 20, 20, 10, fast, 64);
  CHECK(n == -1 || (n >= 0 && n <= 64), "fast tiles %d", n);
  n = oracle_fast_tiles(a, H, W, W, 10, 20, 20, 10, fast, 0);
  CHECK(n <= 0, "fast tiles cap 0 returned %d", n);
  /* LK on points at, near and outside the borders */
  const float pts[2 * 6] = {0, 0, (float)W - 1, (float)H - 1, 3.5f, 40, 100, 2, -5, 10, 300, 50};
  float out[12], err[6];
  uint8_t st[6];
  oracle_lk_track(a, b, H, W, pts, 6, 15, 3, 50, 0.03, 1e-4f, out, st, err);
  /* SGBM with numD + block wider than the image is the caller's job; a legal narrow case */
  int16_t* disp = (int16_t*)malloc(sizeof(int16_t) * H * W);
  oracle_sgbm(a, b, H, W, 0, 32, 11, 968, 3872, disp);
  oracle_sgbm(a, b, 24, 48, 0, 16, 5, 200, 800, disp);
  free(a), free(b), free(disp);
}

int main(int argc, char** argv) {
  int8_t pat[1024];
  const char* path = argc > 1 ? argv[1] : "bit_pattern_31.txt";
  if (!load_pattern(path, pat)) {
    fprintf(stderr, "cannot read %s\n", path);
    return 2;
  }
  case_orb(pat);
  case_knn();
  case_fm();
  case_pnp();
  case_vo();
  case_front();
  printf("san_driver: %s (%d failed checks)\n", fails ? "FAIL" : "ok", fails);
  return fails ? 1 : 0;
}
