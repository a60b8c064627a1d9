/*
 * ORACLE — test infrastructure only (see oracle/__init__.py).
 *
 * CPU restatement of the reference's alternative stereo-VO front end
 * (SURVEY.md §8f rank 4):
 *   /root/reference/visual_odometry.py:84-96   get_tiled_keypoints: cv2.FastFeatureDetector_create()
 *                                             (threshold 10, NMS, TYPE_9_16) per tile, best 10 per tile
 *   /root/reference/visual_odometry.py:98-112  track_keypoints: cv2.calcOpticalFlowPyrLK
 *                                             (winSize 15x15, maxLevel 3, COUNT 50 | EPS 0.03)
 *   /root/reference/visual_odometry.py:22-24   cv2.StereoSGBM_create(minDisparity=0, numDisparities=32,
 *                                             blockSize=11, P1=968, P2=3872).compute(left, right)
 *   /root/reference/keypoint.py:13-32          track_keypoints_left_to_right (the same LK call)
 * OpenCV is absent from this image and unpinned (requirements.txt:4), so PARITY
 * IS UNPINNED against it.  The semantics follow OpenCV 4.x as written out here:
 *
 * FAST (fast.cpp FAST_t<16>): corner at (x, y), rows/cols 3 .. size-4 of the
 *   tile, if 9 contiguous circle pixels are all > v + t or all < v - t; score =
 *   cornerScore<16> (largest threshold still a corner); strict 3x3 NMS against
 *   the score map (0 outside the detection region); keypoints in row-major order.
 *   get_kps keeps the detection order when a tile has <= 10 corners, else the
 *   first 10 of a STABLE sort by response descending (Python sorted()).
 *
 * LK (lkpyramid.cpp): buildOpticalFlowPyramid — level 0 = image, level l =
 *   pyrDown(level l-1) ((w+1)/2 x (h+1)/2, 5x5 [1 4 6 4 1]^2 / 256 rounded,
 *   BORDER_REFLECT_101), each level padded by the window size with REFLECT_101;
 *   levels stop early when the next size would be <= the window.  Derivatives:
 *   calcSharrDeriv (Scharr, reflect-101 inside the level, int16) padded with 0.
 *   LKTrackerInvoker per level from the coarsest, with 14-bit bilinear weights
 *   (cvRound, float), CV_DESCALE by 9 (image) and 14 (derivatives), minEig test
 *   (1e-4), up to 50 iterations, eps^2 = 0.0009 on delta.ddot(delta) (double),
 *   the oscillation half-step rule, status false only at level 0, and the
 *   level-0 error = sum |diff| / (32 * 15 * 15).
 *   Spec choice: OpenCV accumulates the 2x2 structure tensor and the mismatch
 *   vector in float SIMD lanes (summation order is build-specific, and the
 *   integer products exceed 2^24); here they are summed exactly in 64-bit
 *   integers and converted to float once.  Everything else is float as written.
 *
 * SGBM (stereosgbm.cpp computeDisparitySGBM, MODE_SGBM, 5 directions): preFilterCap
 *   0 -> ftzero 15; per-pixel Birchfield-Tomasi cost on the Sobel-x prefiltered
 *   image (clip to [-15, 15] + 15; columns 0 and W-1 forced to 15) plus, >> 2,
 *   on the raw intensities (columns 0 and W-1 forced to 15 as well); 11x11 box
 *   sum with replicated borders over x in [maxD, W) and all rows; path costs
 *   L = C + min(Lp[d], Lp[d+-1] + P1, minLp + P2) - (minLp + P2) for the
 *   directions left->right, up-left, up, up-right (previous row / column of the
 *   same pass, 0 outside the image) and right->left; S = sat16(sat16(L0+L1+L2+L3)
 *   + L4); best d = first minimum; uniquenessRatio 0 (never rejects);
 *   subpixel d*16 + ((S[d-1]-S[d+1])*16 + den)/(2 den) (C division), den =
 *   max(S[d-1]+S[d+1]-2S[d], 1); right-view disparities by min cost with ties
 *   to the larger x; left-right check with disp12MaxDiff <= 0 -> 1; invalid =
 *   (minD-1)*16; then medianBlur 3x3 (replicate border).  Output int16 x16.
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

int oracle_fast_score(const uint8_t* im, int stride, int x, int y, int threshold);
void oracle_fast_score_map(const uint8_t* im, int w, int h, int stride, int t, uint8_t* score);

/* ------------------------------------------------------- FAST on tiles */
/* out: [cap, 3] f32 (x, y, response); returns the count or -1 on overflow */
int oracle_fast_tiles(const uint8_t* img, int H, int W, int stride, int tile_h, int tile_w,
                      int threshold, int per_tile, float* out, int cap) {
  uint8_t* sc = (uint8_t*)malloc((size_t)tile_h * tile_w);
  int* kx = (int*)malloc(sizeof(int) * tile_h * tile_w);
  int* ky = (int*)malloc(sizeof(int) * tile_h * tile_w);
  int* ks = (int*)malloc(sizeof(int) * tile_h * tile_w);
  int n = 0;
  for (int y0 = 0; y0 < H; y0 += tile_h)
    for (int x0 = 0; x0 < W; x0 += tile_w) {
      const int h = H - y0 < tile_h ? H - y0 : tile_h;
      const int w = W - x0 < tile_w ? W - x0 : tile_w;
      const uint8_t* p = img + (size_t)y0 * stride + x0;
      int m = 0;
      if (h >= 7 && w >= 7) {
        oracle_fast_score_map(p, w, h, stride, threshold, sc);
        for (int y = 3; y <= h - 4; ++y)
          for (int x = 3; x <= w - 4; ++x) {
            const int s = sc[y * w + x];
            if (s == 0) continue;
            const uint8_t* q = sc + y * w + x;
            if (s > q[-1] && s > q[1] && s > q[-w - 1] && s > q[-w] && s > q[-w + 1] &&
                s > q[w - 1] && s > q[w] && s > q[w + 1]) {
              kx[m] = x;
              ky[m] = y;
              ks[m] = s;
              ++m;
            }
          }
      }
      int take = m;
      if (m > per_tile) {
        /* stable sort by -response, keep the first per_tile (insertion of ranks) */
        take = per_tile;
        for (int r = 0; r < take; ++r) {
          int best = -1;
          for (int i = 0; i < m; ++i)
            if (ks[i] >= 0 && (best < 0 || ks[i] > ks[best])) best = i;
          if (n >= cap) goto overflow;
          out[3 * n] = (float)(kx[best] + x0);
          out[3 * n + 1] = (float)(ky[best] + y0);
          out[3 * n + 2] = (float)ks[best];
          ks[best] = -1;
          ++n;
        }
      } else {
        for (int i = 0; i < take; ++i) {
          if (n >= cap) goto overflow;
          out[3 * n] = (float)(kx[i] + x0);
          out[3 * n + 1] = (float)(ky[i] + y0);
          out[3 * n + 2] = (float)ks[i];
          ++n;
        }
      }
    }
  free(sc); free(kx); free(ky); free(ks);
  return n;
overflow:
  free(sc); free(kx); free(ky); free(ks);
  return -1;
}

/* ------------------------------------------------------------ pyramids */
static int refl101(int i, int n) {
  if (n == 1) return 0;
  while (i < 0 || i >= n) i = i < 0 ? -i : 2 * n - 2 - i;
  return i;
}

void oracle_pyr_down(const uint8_t* src, int sw, int sh, uint8_t* dst, int dw, int dh) {
  static const int k[5] = {1, 4, 6, 4, 1};
  int* row = (int*)malloc(sizeof(int) * dw * 5);
  for (int y = 0; y < dh; ++y) {
    for (int r = 0; r < 5; ++r) {
      const uint8_t* s = src + (size_t)refl101(2 * y - 2 + r, sh) * sw;
      for (int x = 0; x < dw; ++x) {
        int acc = 0;
        for (int j = 0; j < 5; ++j) acc += k[j] * s[refl101(2 * x - 2 + j, sw)];
        row[r * dw + x] = acc;
      }
    }
    for (int x = 0; x < dw; ++x) {
      int acc = 0;
      for (int r = 0; r < 5; ++r) acc += k[r] * row[r * dw + x];
      dst[(size_t)y * dw + x] = (uint8_t)((acc + 128) >> 8);
    }
  }
  free(row);
}

/* level sizes; returns the number of levels (maxLevel actually used + 1) */
int oracle_lk_levels(int W, int H, int win, int max_level, int* lw, int* lh) {
  int w = W, h = H;
  for (int l = 0; l <= max_level; ++l) {
    lw[l] = w;
    lh[l] = h;
    w = (w + 1) / 2;
    h = (h + 1) / 2;
    if (w <= win || h <= win) return l + 1;
  }
  return max_level + 1;
}

/* calcSharrDeriv: dst [h, w, 2] int16 (Ix, Iy) */
void oracle_scharr(const uint8_t* s, int w, int h, int16_t* dst) {
  int* t0 = (int*)malloc(sizeof(int) * (w + 2));
  int* t1 = (int*)malloc(sizeof(int) * (w + 2));
  for (int y = 0; y < h; ++y) {
    const uint8_t* r0 = s + (size_t)(y > 0 ? y - 1 : h > 1 ? 1 : 0) * w;
    const uint8_t* r1 = s + (size_t)y * w;
    const uint8_t* r2 = s + (size_t)(y < h - 1 ? y + 1 : h > 1 ? h - 2 : 0) * w;
    for (int x = 0; x < w; ++x) {
      t0[x + 1] = (int16_t)((r0[x] + r2[x]) * 3 + r1[x] * 10);
      t1[x + 1] = (int16_t)(r2[x] - r0[x]);
    }
    const int x0 = w > 1 ? 1 : 0, x1 = w > 1 ? w - 2 : 0;
    t0[0] = t0[x0 + 1]; t0[w + 1] = t0[x1 + 1];
    t1[0] = t1[x0 + 1]; t1[w + 1] = t1[x1 + 1];
    for (int x = 0; x < w; ++x) {
      dst[((size_t)y * w + x) * 2] = (int16_t)(t0[x + 2] - t0[x]);
      dst[((size_t)y * w + x) * 2 + 1] = (int16_t)((t1[x + 2] + t1[x]) * 3 + t1[x + 1] * 10);
    }
  }
  free(t0);
  free(t1);
}

typedef struct {
  int w, h;
  const uint8_t* I;     /* level image, w x h */
  const int16_t* dI;    /* derivatives (prev only) */
} lklev;

static int pix(const lklev* L, int x, int y) { return L->I[(size_t)refl101(y, L->h) * L->w + refl101(x, L->w)]; }
static int der(const lklev* L, int x, int y, int c) {
  if (x < 0 || y < 0 || x >= L->w || y >= L->h) return 0;
  return L->dI[((size_t)y * L->w + x) * 2 + c];
}

#define DESCALE(x, n) (((x) + (1 << ((n)-1))) >> (n))

/* one point through all levels (LKTrackerInvoker, levels from nlev-1 down to 0) */
static void lk_point(const lklev* P, const lklev* N, int nlev, int win, int max_count, double eps2,
                     float min_eig, float px, float py, float* ox, float* oy, uint8_t* st,
                     float* err) {
  const float hw = (float)(win - 1) * 0.5f;
  const int W_BITS = 14, W_BITS1 = 14;
  const float FLT_SCALE = 1.f / (1 << 20);
  int16_t Iw[64 * 64], dIw[64 * 64 * 2];
  float npx = 0.f, npy = 0.f; /* nextPts[ptidx] */
  *st = 1;
  *err = 0.f;
  for (int level = nlev - 1; level >= 0; --level) {
    const lklev* I = P + level;
    const lklev* J = N + level;
    const float sc = (float)(1. / (1 << level));
    float prx = px * sc, pry = py * sc;
    float nx, ny;
    if (level == nlev - 1) {
      nx = prx;
      ny = pry;
    } else {
      nx = npx * 2.f;
      ny = npy * 2.f;
    }
    npx = nx;
    npy = ny;
    prx -= hw;
    pry -= hw;
    const int ipx = (int)floorf(prx), ipy = (int)floorf(pry);
    if (ipx < -win || ipx >= I->w || ipy < -win || ipy >= I->h) {
      if (level == 0) {
        *st = 0;
        *err = 0.f;
      }
      continue;
    }
    float a = prx - (float)ipx, b = pry - (float)ipy;
    int iw00 = (int)nearbyintf((1.f - a) * (1.f - b) * (float)(1 << W_BITS));
    int iw01 = (int)nearbyintf(a * (1.f - b) * (float)(1 << W_BITS));
    int iw10 = (int)nearbyintf((1.f - a) * b * (float)(1 << W_BITS));
    int iw11 = (1 << W_BITS) - iw00 - iw01 - iw10;
    int64_t iA11 = 0, iA12 = 0, iA22 = 0;
    for (int y = 0; y < win; ++y)
      for (int x = 0; x < win; ++x) {
        const int X = ipx + x, Y = ipy + y;
        const int ival = DESCALE(pix(I, X, Y) * iw00 + pix(I, X + 1, Y) * iw01 +
                                     pix(I, X, Y + 1) * iw10 + pix(I, X + 1, Y + 1) * iw11,
                                 W_BITS1 - 5);
        const int ixv = DESCALE(der(I, X, Y, 0) * iw00 + der(I, X + 1, Y, 0) * iw01 +
                                    der(I, X, Y + 1, 0) * iw10 + der(I, X + 1, Y + 1, 0) * iw11,
                                W_BITS1);
        const int iyv = DESCALE(der(I, X, Y, 1) * iw00 + der(I, X + 1, Y, 1) * iw01 +
                                    der(I, X, Y + 1, 1) * iw10 + der(I, X + 1, Y + 1, 1) * iw11,
                                W_BITS1);
        Iw[y * win + x] = (int16_t)ival;
        dIw[(y * win + x) * 2] = (int16_t)ixv;
        dIw[(y * win + x) * 2 + 1] = (int16_t)iyv;
        iA11 += (int64_t)ixv * ixv;
        iA12 += (int64_t)ixv * iyv;
        iA22 += (int64_t)iyv * iyv;
      }
    const float A11 = (float)iA11 * FLT_SCALE, A12 = (float)iA12 * FLT_SCALE,
                A22 = (float)iA22 * FLT_SCALE;
    float D = A11 * A22 - A12 * A12;
    const float dd = A11 - A22;
    const float minEig = (A22 + A11 - sqrtf(dd * dd + 4.f * A12 * A12)) / (float)(2 * win * win);
    if (minEig < min_eig || D < 1.1920928955078125e-07f) {
      if (level == 0) *st = 0;
      continue;
    }
    D = 1.f / D;
    nx -= hw;
    ny -= hw;
    float pdx = 0.f, pdy = 0.f;
    for (int j = 0; j < max_count; ++j) {
      const int inx = (int)floorf(nx), iny = (int)floorf(ny);
      if (inx < -win || inx >= J->w || iny < -win || iny >= J->h) {
        if (level == 0) *st = 0;
        break;
      }
      a = nx - (float)inx;
      b = ny - (float)iny;
      iw00 = (int)nearbyintf((1.f - a) * (1.f - b) * (float)(1 << W_BITS));
      iw01 = (int)nearbyintf(a * (1.f - b) * (float)(1 << W_BITS));
      iw10 = (int)nearbyintf((1.f - a) * b * (float)(1 << W_BITS));
      iw11 = (1 << W_BITS) - iw00 - iw01 - iw10;
      int64_t ib1 = 0, ib2 = 0;
      for (int y = 0; y < win; ++y)
        for (int x = 0; x < win; ++x) {
          const int X = inx + x, Y = iny + y;
          const int diff = DESCALE(pix(J, X, Y) * iw00 + pix(J, X + 1, Y) * iw01 +
                                       pix(J, X, Y + 1) * iw10 + pix(J, X + 1, Y + 1) * iw11,
                                   W_BITS1 - 5) -
                           Iw[y * win + x];
          ib1 += (int64_t)diff * dIw[(y * win + x) * 2];
          ib2 += (int64_t)diff * dIw[(y * win + x) * 2 + 1];
        }
      const float b1 = (float)ib1 * FLT_SCALE, b2 = (float)ib2 * FLT_SCALE;
      const float dx = (A12 * b2 - A22 * b1) * D;
      const float dy = (A12 * b1 - A11 * b2) * D;
      nx += dx;
      ny += dy;
      npx = nx + hw;
      npy = ny + hw;
      if ((double)dx * dx + (double)dy * dy <= eps2) break;
      if (j > 0 && fabs((double)(dx + pdx)) < 0.01 && fabs((double)(dy + pdy)) < 0.01) {
        npx -= dx * 0.5f;
        npy -= dy * 0.5f;
        break;
      }
      pdx = dx;
      pdy = dy;
    }
    if (*st && level == 0) {
      const float qx = npx - hw, qy = npy - hw;
      const int inx = (int)floorf(qx), iny = (int)floorf(qy);
      if (inx < -win || inx >= J->w || iny < -win || iny >= J->h) {
        *st = 0;
        continue;
      }
      const float aa = qx - (float)inx, bb = qy - (float)iny;
      iw00 = (int)nearbyintf((1.f - aa) * (1.f - bb) * (float)(1 << W_BITS));
      iw01 = (int)nearbyintf(aa * (1.f - bb) * (float)(1 << W_BITS));
      iw10 = (int)nearbyintf((1.f - aa) * bb * (float)(1 << W_BITS));
      iw11 = (1 << W_BITS) - iw00 - iw01 - iw10;
      float ev = 0.f;
      for (int y = 0; y < win; ++y)
        for (int x = 0; x < win; ++x) {
          const int X = inx + x, Y = iny + y;
          const int diff = DESCALE(pix(J, X, Y) * iw00 + pix(J, X + 1, Y) * iw01 +
                                       pix(J, X, Y + 1) * iw10 + pix(J, X + 1, Y + 1) * iw11,
                                   W_BITS1 - 5) -
                           Iw[y * win + x];
          ev += fabsf((float)diff);
        }
      *err = ev * 1.f / (float)(32 * win * win);
    }
  }
  *ox = npx;
  *oy = npy;
}

/* calcOpticalFlowPyrLK(prev, next, pts, None, winSize=(win,win), maxLevel, criteria) */
void oracle_lk_track(const uint8_t* prev, const uint8_t* next, int H, int W, const float* pts,
                     int n, int win, int max_level, int max_count, double eps, float min_eig,
                     float* out, uint8_t* status, float* err) {
  int lw[16], lh[16];
  const int nlev = oracle_lk_levels(W, H, win, max_level, lw, lh);
  lklev P[16], N[16];
  uint8_t* bufs[32];
  int16_t* ders[16];
  for (int l = 0; l < nlev; ++l) {
    bufs[2 * l] = (uint8_t*)malloc((size_t)lw[l] * lh[l]);
    bufs[2 * l + 1] = (uint8_t*)malloc((size_t)lw[l] * lh[l]);
    if (l == 0) {
      memcpy(bufs[0], prev, (size_t)W * H);
      memcpy(bufs[1], next, (size_t)W * H);
    } else {
      oracle_pyr_down(bufs[2 * l - 2], lw[l - 1], lh[l - 1], bufs[2 * l], lw[l], lh[l]);
      oracle_pyr_down(bufs[2 * l - 1], lw[l - 1], lh[l - 1], bufs[2 * l + 1], lw[l], lh[l]);
    }
    ders[l] = (int16_t*)malloc(sizeof(int16_t) * 2 * lw[l] * lh[l]);
    oracle_scharr(bufs[2 * l], lw[l], lh[l], ders[l]);
    P[l].w = N[l].w = lw[l];
    P[l].h = N[l].h = lh[l];
    P[l].I = bufs[2 * l];
    P[l].dI = ders[l];
    N[l].I = bufs[2 * l + 1];
    N[l].dI = NULL;
  }
  if (max_count < 0) max_count = 0;
  if (max_count > 100) max_count = 100;
  if (eps < 0) eps = 0;
  if (eps > 10) eps = 10;
#pragma omp parallel for schedule(dynamic, 64)
  for (int i = 0; i < n; ++i)
    lk_point(P, N, nlev, win, max_count, eps * eps, min_eig, pts[2 * i], pts[2 * i + 1],
             &out[2 * i], &out[2 * i + 1], &status[i], &err[i]);
  for (int l = 0; l < nlev; ++l) {
    free(bufs[2 * l]);
    free(bufs[2 * l + 1]);
    free(ders[l]);
  }
}

/* ----------------------------------------------------------------- SGBM */
static int16_t sat16(int v) { return (int16_t)(v > 32767 ? 32767 : v < -32768 ? -32768 : v); }

/* prefiltered channels of one row: c0 = clipped Sobel-x (+15), c1 = raw; x = 0, W-1 -> 15 */
static void sgbm_row_channels(const uint8_t* img, int H, int W, int y, int ftzero, int* c0, int* c1) {
  const uint8_t* r = img + (size_t)y * W;
  const uint8_t* rn = img + (size_t)(y > 0 ? y - 1 : y) * W;
  const uint8_t* rs = img + (size_t)(y < H - 1 ? y + 1 : y) * W;
  c0[0] = c0[W - 1] = c1[0] = c1[W - 1] = ftzero;
  for (int x = 1; x < W - 1; ++x) {
    int v = (r[x + 1] - r[x - 1]) * 2 + rn[x + 1] - rn[x - 1] + rs[x + 1] - rs[x - 1];
    v = v < -ftzero ? -ftzero : v > ftzero ? ftzero : v;
    c0[x] = v + ftzero;
    c1[x] = r[x];
  }
}

static void bt_minmax(const int* c, int W, int* lo, int* hi) {
  for (int x = 0; x < W; ++x) {
    const int v = c[x];
    const int vl = x > 0 ? (v + c[x - 1]) / 2 : v;
    const int vr = x < W - 1 ? (v + c[x + 1]) / 2 : v;
    int a = vl < vr ? vl : vr;
    a = a < v ? a : v;
    int b = vl > vr ? vl : vr;
    b = b > v ? b : v;
    lo[x] = a;
    hi[x] = b;
  }
}

/* pixel costs of row y: pc[(x - minX1) * D + d], x in [minX1, W) */
static void sgbm_pixel_cost(const uint8_t* L, const uint8_t* R, int H, int W, int y, int minD,
                            int D, int16_t* pc, int* buf) {
  const int ftzero = 15, minX1 = minD + D;
  int *l0 = buf, *l1 = l0 + W, *r0 = l1 + W, *r1 = r0 + W;
  int *l0lo = r1 + W, *l0hi = l0lo + W, *l1lo = l0hi + W, *l1hi = l1lo + W;
  int *r0lo = l1hi + W, *r0hi = r0lo + W, *r1lo = r0hi + W, *r1hi = r1lo + W;
  sgbm_row_channels(L, H, W, y, ftzero, l0, l1);
  sgbm_row_channels(R, H, W, y, ftzero, r0, r1);
  bt_minmax(l0, W, l0lo, l0hi);
  bt_minmax(l1, W, l1lo, l1hi);
  bt_minmax(r0, W, r0lo, r0hi);
  bt_minmax(r1, W, r1lo, r1hi);
  for (int x = minX1; x < W; ++x)
    for (int d = 0; d < D; ++d) {
      const int xr = x - (d + minD);
      int cost = 0;
      for (int ch = 0; ch < 2; ++ch) {
        const int u = ch ? l1[x] : l0[x], u0 = ch ? l1lo[x] : l0lo[x], u1 = ch ? l1hi[x] : l0hi[x];
        const int v = ch ? r1[xr] : r0[xr], v0 = ch ? r1lo[xr] : r0lo[xr],
                  v1 = ch ? r1hi[xr] : r0hi[xr];
        int ca = u - v1 > 0 ? u - v1 : 0;
        ca = ca > v0 - u ? ca : v0 - u;
        int cb = v - u1 > 0 ? v - u1 : 0;
        cb = cb > u0 - v ? cb : u0 - v;
        cost += (ca < cb ? ca : cb) >> (ch ? 2 : 0);
      }
      pc[(size_t)(x - minX1) * D + d] = (int16_t)cost;
    }
}

static int path_step(int C, const int16_t* Lp, int d, int D, int P1, int delta) {
  int m = Lp[d];
  const int lm = d > 0 ? Lp[d - 1] + P1 : 32767 + P1;
  const int lp = d < D - 1 ? Lp[d + 1] + P1 : 32767 + P1;
  m = m < lm ? m : lm;
  m = m < lp ? m : lp;
  m = m < delta ? m : delta;
  return C + m - delta;
}

/* disp [H, W] int16 (x16) */
void oracle_sgbm(const uint8_t* L, const uint8_t* R, int H, int W, int minD, int numD, int block,
                 int P1, int P2, int16_t* disp) {
  const int D = numD, minX1 = minD + D, W1 = W - minX1, SW2 = block / 2, SH2 = block / 2;
  const int INVALID = (minD - 1) * 16;
  const int disp12 = 1;
  if (P1 <= 0) P1 = 2;
  if (P2 <= 0) P2 = 5;
  if (P2 < P1 + 1) P2 = P1 + 1;
  int16_t* raw = (int16_t*)malloc(sizeof(int16_t) * H * W);
  for (int i = 0; i < H * W; ++i) raw[i] = (int16_t)INVALID;
  if (W1 <= 0) goto median;
  {
    int16_t* pc = (int16_t*)malloc(sizeof(int16_t) * (size_t)H * W1 * D);
#pragma omp parallel
    {
      int* buf = (int*)malloc(sizeof(int) * 16 * W);
#pragma omp for schedule(static)
      for (int y = 0; y < H; ++y)
        sgbm_pixel_cost(L, R, H, W, y, minD, D, pc + (size_t)y * W1 * D, buf);
      free(buf);
    }
    /* box sum, replicated borders */
    int16_t* C = (int16_t*)malloc(sizeof(int16_t) * (size_t)H * W1 * D);
#pragma omp parallel for schedule(static)
    for (int y = 0; y < H; ++y)
      for (int x = 0; x < W1; ++x)
        for (int d = 0; d < D; ++d) {
          int s = 0;
          for (int dy = -SH2; dy <= SH2; ++dy) {
            const int yy = y + dy < 0 ? 0 : y + dy > H - 1 ? H - 1 : y + dy;
            for (int dx = -SW2; dx <= SW2; ++dx) {
              const int xx = x + dx < 0 ? 0 : x + dx > W1 - 1 ? W1 - 1 : x + dx;
              s += pc[((size_t)yy * W1 + xx) * D + d];
            }
          }
          C[((size_t)y * W1 + x) * D + d] = (int16_t)s;
        }
    free(pc);
    /* path costs; rows top to bottom */
    int16_t* Lprev = (int16_t*)calloc((size_t)3 * (W1 + 2) * D, sizeof(int16_t)); /* dirs 1..3 */
    int* mprev = (int*)calloc((size_t)3 * (W1 + 2), sizeof(int));
    int16_t* Lcur = (int16_t*)calloc((size_t)3 * (W1 + 2) * D, sizeof(int16_t));
    int* mcur = (int*)calloc((size_t)3 * (W1 + 2), sizeof(int));
    int16_t* L0 = (int16_t*)calloc((size_t)(W1 + 2) * D, sizeof(int16_t));
    int* m0 = (int*)calloc((size_t)(W1 + 2), sizeof(int));
    int16_t* S = (int16_t*)malloc(sizeof(int16_t) * (size_t)W1 * D);
    int16_t* disp2 = (int16_t*)malloc(sizeof(int16_t) * W);
    int* cost2 = (int*)malloc(sizeof(int) * W);
    static const int16_t zeros[256] = {0};
    for (int y = 0; y < H; ++y) {
      const int16_t* Cy = C + (size_t)y * W1 * D;
      /* left -> right and the three previous-row directions (cells offset by 1) */
      for (int x = 0; x < W1; ++x) {
        const int16_t* Cp = Cy + (size_t)x * D;
        const int16_t* lp0 = x > 0 ? L0 + (size_t)x * D : zeros;
        const int dl0 = (x > 0 ? m0[x] : 0) + P2;
        int mn[4] = {32767, 32767, 32767, 32767};
        for (int d = 0; d < D; ++d) {
          int Lv[4];
          Lv[0] = path_step(Cp[d], lp0, d, D, P1, dl0);
          for (int r = 1; r <= 3; ++r) {
            const int xs = x + (r - 2) + 1; /* r=1: x-1, r=2: x, r=3: x+1 (cell index) */
            const int16_t* lp = Lprev + ((size_t)(r - 1) * (W1 + 2) + xs) * D;
            const int dl = mprev[(r - 1) * (W1 + 2) + xs] + P2;
            Lv[r] = path_step(Cp[d], lp, d, D, P1, dl);
          }
          L0[(size_t)(x + 1) * D + d] = (int16_t)Lv[0];
          for (int r = 1; r <= 3; ++r) Lcur[((size_t)(r - 1) * (W1 + 2) + x + 1) * D + d] = (int16_t)Lv[r];
          for (int r = 0; r < 4; ++r) mn[r] = mn[r] < Lv[r] ? mn[r] : Lv[r];
          S[(size_t)x * D + d] = sat16(Lv[0] + Lv[1] + Lv[2] + Lv[3]);
        }
        m0[x + 1] = mn[0];
        for (int r = 1; r <= 3; ++r) mcur[(r - 1) * (W1 + 2) + x + 1] = mn[r];
      }
      /* right -> left, selection */
      for (int x = 0; x < W; ++x) {
        raw[(size_t)y * W + x] = (int16_t)INVALID;
        disp2[x] = (int16_t)INVALID;
        cost2[x] = 32767;
      }
      int16_t* LR = L0; /* reuse: cell x+1 holds the right->left value at x */
      memset(LR + (size_t)(W1 + 1) * D, 0, sizeof(int16_t) * D);
      m0[W1 + 1] = 0;
      for (int x = W1 - 1; x >= 0; --x) {
        const int16_t* Cp = Cy + (size_t)x * D;
        const int16_t* lp = LR + (size_t)(x + 2) * D;
        const int dl = m0[x + 2] + P2;
        int mn = 32767, minS = 32767, best = -1;
        int16_t* Sp = S + (size_t)x * D;
        int16_t Lnew[256];
        for (int d = 0; d < D; ++d) {
          const int Lv = path_step(Cp[d], lp, d, D, P1, dl);
          Lnew[d] = (int16_t)Lv;
          mn = mn < Lv ? mn : Lv;
          const int sv = Sp[d] = sat16(Sp[d] + Lv);
          if (sv < minS) {
            minS = sv;
            best = d;
          }
        }
        memcpy(LR + (size_t)(x + 1) * D, Lnew, sizeof(int16_t) * D);
        m0[x + 1] = mn;
        int d = best;
        const int x2 = x + minX1 - d - minD;
        if (best >= 0 && cost2[x2] > minS) {
          cost2[x2] = minS;
          disp2[x2] = (int16_t)(d + minD);
        }
        if (0 < d && d < D - 1) {
          int den = Sp[d - 1] + Sp[d + 1] - 2 * Sp[d];
          den = den > 1 ? den : 1;
          d = d * 16 + ((Sp[d - 1] - Sp[d + 1]) * 16 + den) / (den * 2);
        } else {
          d *= 16;
        }
        raw[(size_t)y * W + x + minX1] = (int16_t)(d + minD * 16);
      }
      /* left-right consistency */
      for (int x = minX1; x < W; ++x) {
        const int d1 = raw[(size_t)y * W + x];
        if (d1 == INVALID) continue;
        const int _d = d1 >> 4, d_ = (d1 + 15) >> 4;
        const int _x = x - _d, x_ = x - d_;
        if (0 <= _x && _x < W && disp2[_x] >= minD && abs(disp2[_x] - _d) > disp12 && 0 <= x_ &&
            x_ < W && disp2[x_] >= minD && abs(disp2[x_] - d_) > disp12)
          raw[(size_t)y * W + x] = (int16_t)INVALID;
      }
      /* this row's directions 1..3 become the previous row; borders stay 0 */
      int16_t* t = Lprev; Lprev = Lcur; Lcur = t;
      int* tm = mprev; mprev = mcur; mcur = tm;
      for (int r = 0; r < 3; ++r) {
        memset(Lprev + ((size_t)r * (W1 + 2)) * D, 0, sizeof(int16_t) * D);
        memset(Lprev + ((size_t)r * (W1 + 2) + W1 + 1) * D, 0, sizeof(int16_t) * D);
        mprev[r * (W1 + 2)] = 0;
        mprev[r * (W1 + 2) + W1 + 1] = 0;
      }
    }
    free(C); free(Lprev); free(mprev); free(Lcur); free(mcur); free(L0); free(m0); free(S);
    free(disp2); free(cost2);
  }
median:
  for (int y = 0; y < H; ++y)
    for (int x = 0; x < W; ++x) {
      int v[9], k = 0;
      for (int dy = -1; dy <= 1; ++dy)
        for (int dx = -1; dx <= 1; ++dx) {
          const int yy = y + dy < 0 ? 0 : y + dy > H - 1 ? H - 1 : y + dy;
          const int xx = x + dx < 0 ? 0 : x + dx > W - 1 ? W - 1 : x + dx;
          v[k++] = raw[(size_t)yy * W + xx];
        }
      for (int i = 1; i < 9; ++i)
        for (int j = i; j > 0 && v[j - 1] > v[j]; --j) {
          const int tt = v[j]; v[j] = v[j - 1]; v[j - 1] = tt;
        }
      disp[(size_t)y * W + x] = (int16_t)v[4];
    }
  free(raw);
}
