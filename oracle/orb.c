/*
 * ORACLE — test infrastructure only (see oracle/__init__.py).
 *
 * CPU restatement of the reference's tiled ORB front end:
 *   /root/reference/orb.py:4-25   orb_detector_using_tiles (tiling, offsets, flatten)
 *   /root/reference/orb.py:28-38  orb_extraction_detect: cv2.ORB_create(nfeatures,
 *                                 scaleFactor=1.2) then .detect() and .compute()
 * OpenCV is not vendored in /root/reference and is absent from this image, so
 * the ORB internals follow OpenCV 4.x ORB_Impl semantics written out below
 * (PARITY UNPINNED against a real OpenCV build):
 *   nlevels 8, scaleFactor 1.2, edgeThreshold 31, patchSize 31, fastThreshold 20,
 *   HARRIS_SCORE (k = 0.04, block 7), WTA_K 2, firstLevel 0.
 *  1. level budget  n_l = cvRound(d), d = N(1-f)/(1-f^8) (float), d *= f; last = N - sum
 *  2. pyramid       level l size = cvRound(W / (float)1.2^l) x cvRound(H / ...);
 *                   level l = resize(level l-1) with INTER_LINEAR_EXACT
 *                   (8-bit fixed-point coefficients, (sum + 2^15) >> 16)
 *  3. FAST-9/16     threshold 20, score = OpenCV cornerScore<16>, strict 3x3 NMS,
 *                   detection rows/cols 3 .. size-4
 *  4. border        keep 31 <= x < w-31, 31 <= y < h-31 (none if w or h <= 62)
 *  5. retainBest(2 n_l) by FAST score, boundary ties kept
 *  6. Harris        7x7 block of Sobel-like integer gradients, float response
 *                   ((float)a*b - (float)c*c - k((float)a+b)((float)a+b)) * scale^4
 *  7. retainBest(n_l) by Harris response, boundary ties kept
 *  8. IC angle      moments over the radius-15 disc (umax), fastAtan2 polynomial (deg)
 *  9. blur          GaussianBlur 7x7 sigma 2 (float separable, FMA chains, RNE to u8)
 * 10. rBRIEF        bit j of byte i: I(p_{16i+2j}) < I(p_{16i+2j+1}), rotated by the angle,
 *                   offsets rounded half-to-even, bit_pattern_31
 * Canonical order within a level (OpenCV's nth_element order is
 * implementation-defined): Harris response desc, then y asc, then x asc.
 * Levels in ascending order, tiles in orb.py order (rows then columns).
 * Built with -ffp-contract=off: every float expression rounds as written.
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#define NLEV 8
#define EDGE 31
#define HALF_PATCH 15
#define FAST_T 20

typedef struct {
  float x, y, size, angle, response;
  int octave;
} okp;

static int iround_f(float v) { return (int)nearbyintf(v); }  /* cvRound(float): RNE */
static int iround_d(double v) { return (int)nearbyint(v); } /* cvRound(double): RNE */

/* ------------------------------------------------------------ pyramid sizes */
void oracle_orb_level_sizes(int w, int h, int* lw, int* lh, float* scale) {
  for (int l = 0; l < NLEV; ++l) {
    const float s = (float)pow(1.2, (double)l);
    scale[l] = s;
    lw[l] = iround_f((float)w / s);
    lh[l] = iround_f((float)h / s);
  }
}

void oracle_orb_level_budget(int nfeatures, int* n) {
  const float factor = (float)(1.0 / 1.2);
  float d = (float)nfeatures * (1 - factor) / (1 - (float)pow((double)factor, (double)NLEV));
  int sum = 0;
  for (int l = 0; l < NLEV - 1; ++l) {
    n[l] = iround_f(d);
    sum += n[l];
    d *= factor;
  }
  n[NLEV - 1] = nfeatures - sum > 0 ? nfeatures - sum : 0;
}

/* ------------------------------------------------ INTER_LINEAR_EXACT resize */
static void lin_coeffs(int dsize, int ssize, int* ofs, int* c1) {
  const double inv = (double)dsize / ssize;
  const double scale = 1.0 / inv;
  int lo = 0, hi = dsize;
  for (int d = 0; d < dsize; ++d) {
    const double fval = scale * ((double)d + 0.5) - 0.5;
    const int ival = (int)floor(fval);
    ofs[d] = 0;
    c1[d] = 0;
    if (ival >= 0 && ssize > 1) {
      if (ival < ssize - 1) {
        ofs[d] = ival;
        c1[d] = iround_d((fval - (double)ival) * 256.0);
      } else if (d < hi) {
        hi = d;
      }
    } else if (d + 1 > lo) {
      lo = d + 1;
    }
  }
  for (int d = 0; d < dsize; ++d) {
    if (d < lo) { ofs[d] = 0; c1[d] = 0; }
    if (d >= hi) { ofs[d] = ssize - 1; c1[d] = 0; }
  }
}

void oracle_resize_linear_exact(const uint8_t* src, int sw, int sh, int sstride, uint8_t* dst,
                                int dw, int dh, int dstride) {
  int* xo = (int*)malloc(sizeof(int) * dw);
  int* xc = (int*)malloc(sizeof(int) * dw);
  int* yo = (int*)malloc(sizeof(int) * dh);
  int* yc = (int*)malloc(sizeof(int) * dh);
  int* h0 = (int*)malloc(sizeof(int) * dw);
  int* h1 = (int*)malloc(sizeof(int) * dw);
  lin_coeffs(dw, sw, xo, xc);
  lin_coeffs(dh, sh, yo, yc);
  for (int y = 0; y < dh; ++y) {
    for (int k = 0; k < 2; ++k) {
      int* hb = k ? h1 : h0;
      const int sy = yo[y] + k;
      if (k == 1 && yc[y] == 0) break;
      const uint8_t* row = src + (size_t)sy * sstride;
      for (int x = 0; x < dw; ++x) {
        const int c1 = xc[x], c0 = 256 - c1;
        hb[x] = c0 * row[xo[x]] + (c1 ? c1 * row[xo[x] + 1] : 0);
      }
    }
    const int cy1 = yc[y], cy0 = 256 - cy1;
    for (int x = 0; x < dw; ++x) {
      const int v = cy0 * h0[x] + (cy1 ? cy1 * h1[x] : 0);
      int o = (v + 32768) >> 16;
      dst[(size_t)y * dstride + x] = (uint8_t)(o > 255 ? 255 : o);
    }
  }
  free(xo); free(xc); free(yo); free(yc); free(h0); free(h1);
}

/* ------------------------------------------------------------------- FAST */
static const int kCircle[16][2] = {{0, 3},  {1, 3},   {2, 2},   {3, 1},  {3, 0},  {3, -1},
                                   {2, -2}, {1, -3},  {0, -3},  {-1, -3}, {-2, -2}, {-3, -1},
                                   {-3, 0}, {-3, 1},  {-2, 2},  {-1, 3}};

static int fast_is_corner(const uint8_t* im, int stride, int x, int y, int t) {
  const int v = im[(size_t)y * stride + x];
  int cnt_d = 0, cnt_b = 0;
  for (int k = 0; k < 25; ++k) {
    const int kk = k & 15;
    const int p = im[(size_t)(y + kCircle[kk][1]) * stride + x + kCircle[kk][0]];
    if (p < v - t) { if (++cnt_d > 8) return 1; } else cnt_d = 0;
  }
  for (int k = 0; k < 25; ++k) {
    const int kk = k & 15;
    const int p = im[(size_t)(y + kCircle[kk][1]) * stride + x + kCircle[kk][0]];
    if (p > v + t) { if (++cnt_b > 8) return 1; } else cnt_b = 0;
  }
  return 0;
}

/* OpenCV cornerScore<16> */
int oracle_fast_score(const uint8_t* im, int stride, int x, int y, int threshold) {
  const int v = im[(size_t)y * stride + x];
  int d[25];
  for (int k = 0; k < 25; ++k) {
    const int kk = k & 15;
    d[k] = v - im[(size_t)(y + kCircle[kk][1]) * stride + x + kCircle[kk][0]];
  }
  int a0 = threshold;
  for (int k = 0; k < 16; k += 2) {
    int a = d[k + 1];
    for (int j = 2; j <= 8; ++j) a = a < d[k + j] ? a : d[k + j];
    int m = a < d[k] ? a : d[k];
    a0 = a0 > m ? a0 : m;
    m = a < d[k + 9] ? a : d[k + 9];
    a0 = a0 > m ? a0 : m;
  }
  int b0 = -a0;
  for (int k = 0; k < 16; k += 2) {
    int b = d[k + 1];
    for (int j = 2; j <= 8; ++j) b = b > d[k + j] ? b : d[k + j];
    int m = b > d[k] ? b : d[k];
    b0 = b0 < m ? b0 : m;
    m = b > d[k + 9] ? b : d[k + 9];
    b0 = b0 < m ? b0 : m;
  }
  return -b0 - 1;
}

/* score map (0 = not a corner) over detection rows/cols 3..size-4 */
void oracle_fast_score_map(const uint8_t* im, int w, int h, int stride, int t, uint8_t* score) {
  memset(score, 0, (size_t)w * h);
  for (int y = 3; y <= h - 4; ++y)
    for (int x = 3; x <= w - 4; ++x)
      if (fast_is_corner(im, stride, x, y, t))
        score[(size_t)y * w + x] = (uint8_t)oracle_fast_score(im, stride, x, y, t);
}

/* ----------------------------------------------------------------- Harris */
float oracle_harris(const uint8_t* im, int stride, int x0, int y0) {
  const int r = 3;
  int a = 0, b = 0, c = 0;
  for (int i = 0; i < 7; ++i)
    for (int j = 0; j < 7; ++j) {
      const uint8_t* p = im + (size_t)(y0 - r + i) * stride + (x0 - r + j);
      const int Ix = (p[1] - p[-1]) * 2 + (p[-stride + 1] - p[-stride - 1]) +
                     (p[stride + 1] - p[stride - 1]);
      const int Iy = (p[stride] - p[-stride]) * 2 + (p[stride - 1] - p[-stride - 1]) +
                     (p[stride + 1] - p[-stride + 1]);
      a += Ix * Ix;
      b += Iy * Iy;
      c += Ix * Iy;
    }
  const float scale = 1.f / ((1 << 2) * 7 * 255.f);
  const float ssss = scale * scale * scale * scale;
  const float k = 0.04f;
  return ((float)a * b - (float)c * c - k * ((float)a + b) * ((float)a + b)) * ssss;
}

/* ---------------------------------------------------------------- IC angle */
void oracle_orb_umax(int* umax) {
  const int half = HALF_PATCH;
  const int vmax = (int)floor(half * sqrt(2.f) / 2 + 1);
  const int vmin = (int)ceil(half * sqrt(2.f) / 2);
  for (int v = 0; v <= vmax; ++v) umax[v] = iround_d(sqrt((double)half * half - v * v));
  for (int v = half, v0 = 0; v >= vmin; --v) {
    while (umax[v0] == umax[v0 + 1]) ++v0;
    umax[v] = v0;
    ++v0;
  }
}

float oracle_fast_atan2(float y, float x) {
  const float r2d = (float)(180 / 3.14159265358979323846);
  const float p1 = 0.9997878412794807f * r2d, p3 = -0.3258083974640975f * r2d;
  const float p5 = 0.1555786518463281f * r2d, p7 = -0.04432655554792128f * r2d;
  const float ax = fabsf(x), ay = fabsf(y);
  float a, c, c2;
  if (ax >= ay) {
    c = ay / (ax + (float)2.2204460492503131e-16);
    c2 = c * c;
    a = (((p7 * c2 + p5) * c2 + p3) * c2 + p1) * c;
  } else {
    c = ax / (ay + (float)2.2204460492503131e-16);
    c2 = c * c;
    a = 90.f - (((p7 * c2 + p5) * c2 + p3) * c2 + p1) * c;
  }
  if (x < 0) a = 180.f - a;
  if (y < 0) a = 360.f - a;
  return a;
}

float oracle_ic_angle(const uint8_t* im, int stride, int x, int y, const int* umax) {
  const uint8_t* center = im + (size_t)y * stride + x;
  int m01 = 0, m10 = 0;
  for (int u = -HALF_PATCH; u <= HALF_PATCH; ++u) m10 += u * center[u];
  for (int v = 1; v <= HALF_PATCH; ++v) {
    int vs = 0;
    const int d = umax[v];
    for (int u = -d; u <= d; ++u) {
      const int vp = center[u + v * stride], vm = center[u - v * stride];
      vs += vp - vm;
      m10 += u * (vp + vm);
    }
    m01 += v * vs;
  }
  return oracle_fast_atan2((float)m01, (float)m10);
}

/* --------------------------------------------------------------- blur 7x7 */
void oracle_gauss_kernel7(float* k) {
  double t[7], sum = 0;
  const double sigma = 2.0, s2 = -0.5 / (sigma * sigma);
  for (int i = 0; i < 7; ++i) {
    const double x = i - 3.0;
    t[i] = exp(s2 * x * x);
    k[i] = (float)t[i];
    sum += k[i];
  }
  sum = 1.0 / sum;
  for (int i = 0; i < 7; ++i) k[i] = (float)(k[i] * sum);
}

static int refl101(int i, int n) {
  if (n == 1) return 0;
  while (i < 0 || i >= n) i = i < 0 ? -i : 2 * n - 2 - i;
  return i;
}

/* GaussianBlur(7x7, 2, 2, BORDER_REFLECT_101) of a w x h u8 image, float path:
 * row:    R = fma chain over taps 0..6 starting from 0
 * column: s = R0*k[3]; s = fma(R+k + R-k, k[3+k], s) for k = 1..3; u8(rint(s)) */
void oracle_gauss_blur7(const uint8_t* src, int w, int h, int sstride, uint8_t* dst, int dstride) {
  float k[7];
  oracle_gauss_kernel7(k);
  float* R = (float*)malloc(sizeof(float) * (size_t)w * h);
  for (int y = 0; y < h; ++y)
    for (int x = 0; x < w; ++x) {
      float s = 0.f;
      for (int t = 0; t < 7; ++t) s = fmaf((float)src[(size_t)y * sstride + refl101(x + t - 3, w)], k[t], s);
      R[(size_t)y * w + x] = s;
    }
  for (int y = 0; y < h; ++y)
    for (int x = 0; x < w; ++x) {
      float s = R[(size_t)y * w + x] * k[3];
      for (int t = 1; t <= 3; ++t)
        s = fmaf(R[(size_t)refl101(y + t, h) * w + x] + R[(size_t)refl101(y - t, h) * w + x], k[3 + t], s);
      int v = (int)nearbyintf(s);
      dst[(size_t)y * dstride + x] = (uint8_t)(v < 0 ? 0 : v > 255 ? 255 : v);
    }
  free(R);
}

/* ---------------------------------------------------------------- one patch */
typedef struct {
  int x, y, score;
  float resp;
} cand;

static int cmp_resp(const void* a, const void* b) {
  const cand* p = (const cand*)a;
  const cand* q = (const cand*)b;
  if (p->resp != q->resp) return p->resp > q->resp ? -1 : 1;
  if (p->y != q->y) return p->y < q->y ? -1 : 1;
  return p->x < q->x ? -1 : (p->x > q->x);
}

static int cmp_int_desc(const void* a, const void* b) {
  return *(const int*)b - *(const int*)a;
}

/* keypoints + descriptors of one patch (w x h, stride) -> appended at out[*n]. */
static int orb_patch(const uint8_t* patch, int w, int h, int stride, int nfeatures,
                     const int8_t* pattern, okp* out, uint8_t* desc, int cap, int* n) {
  int lw[NLEV], lh[NLEV], nl[NLEV], umax[HALF_PATCH + 2];
  float ls[NLEV];
  oracle_orb_level_sizes(w, h, lw, lh, ls);
  oracle_orb_level_budget(nfeatures, nl);
  oracle_orb_umax(umax);
  float kern[7];
  oracle_gauss_kernel7(kern);
  (void)kern;
  uint8_t* lev[NLEV];
  lev[0] = (uint8_t*)malloc((size_t)w * h);
  for (int y = 0; y < h; ++y) memcpy(lev[0] + (size_t)y * w, patch + (size_t)y * stride, w);
  for (int l = 1; l < NLEV; ++l) {
    lev[l] = (uint8_t*)malloc((size_t)lw[l] * lh[l] + 1);
    oracle_resize_linear_exact(lev[l - 1], lw[l - 1], lh[l - 1], lw[l - 1], lev[l], lw[l], lh[l], lw[l]);
  }
  int overflow = 0;
  for (int l = 0; l < NLEV; ++l) {
    const int W = lw[l], H = lh[l];
    if (W <= 2 * EDGE || H <= 2 * EDGE || nl[l] == 0) continue;
    uint8_t* sc = (uint8_t*)malloc((size_t)W * H);
    oracle_fast_score_map(lev[l], W, H, W, FAST_T, sc);
    int nc = 0, capc = 1024;
    cand* cs = (cand*)malloc(sizeof(cand) * capc);
    for (int y = 4; y <= H - 5; ++y)
      for (int x = 4; x <= W - 5; ++x) {
        const int s = sc[(size_t)y * W + x];
        if (!s) continue;
        int ok = 1;
        for (int dy = -1; dy <= 1 && ok; ++dy)
          for (int dx = -1; dx <= 1; ++dx)
            if ((dx || dy) && sc[(size_t)(y + dy) * W + x + dx] >= s) { ok = 0; break; }
        if (!ok) continue;
        if (!(x >= EDGE && y >= EDGE && x < W - EDGE && y < H - EDGE)) continue;
        if (nc == capc) { capc *= 2; cs = (cand*)realloc(cs, sizeof(cand) * capc); }
        cs[nc].x = x; cs[nc].y = y; cs[nc].score = s; cs[nc].resp = 0.f;
        ++nc;
      }
    /* retainBest(2 n_l) by FAST score (ties kept) */
    const int keep1 = 2 * nl[l];
    if (nc > keep1) {
      int* s = (int*)malloc(sizeof(int) * nc);
      for (int i = 0; i < nc; ++i) s[i] = cs[i].score;
      qsort(s, nc, sizeof(int), cmp_int_desc);
      const int thr = s[keep1 - 1];
      free(s);
      int m = 0;
      for (int i = 0; i < nc; ++i) if (cs[i].score >= thr) cs[m++] = cs[i];
      nc = m;
    }
    for (int i = 0; i < nc; ++i) cs[i].resp = oracle_harris(lev[l], W, cs[i].x, cs[i].y);
    qsort(cs, nc, sizeof(cand), cmp_resp);
    if (nc > nl[l]) {
      const float thr = cs[nl[l] - 1].resp;
      int m = nl[l];
      while (m < nc && cs[m].resp >= thr) ++m;
      nc = m;
    }
    /* blurred level for the descriptors */
    uint8_t* bl = (uint8_t*)malloc((size_t)W * H);
    oracle_gauss_blur7(lev[l], W, H, W, bl, W);
    for (int i = 0; i < nc; ++i) {
      if (*n >= cap) { overflow = 1; break; }
      okp* k = out + *n;
      k->angle = oracle_ic_angle(lev[l], W, cs[i].x, cs[i].y, umax);
      k->x = (float)cs[i].x * ls[l];
      k->y = (float)cs[i].y * ls[l];
      k->size = 31 * ls[l];
      k->response = cs[i].resp;
      k->octave = l;
      /* descriptor (compute(): level coords re-derived from the level-0 point) */
      const float sc1 = 1.f / ls[l];
      const int cx = iround_f(k->x * sc1), cy = iround_f(k->y * sc1);
      float ang = k->angle;
      ang *= (float)(3.14159265358979323846 / 180.f);
      const float a = (float)cos(ang), b = (float)sin(ang);
      uint8_t* dsc = desc + (size_t)(*n) * 32;
      for (int byte = 0; byte < 32; ++byte) {
        int val = 0;
        for (int bit = 0; bit < 8; ++bit) {
          int t[2];
          for (int e = 0; e < 2; ++e) {
            const int8_t* pp = pattern + ((byte * 8 + bit) * 4 + e * 2);
            const float px = (float)pp[0], py = (float)pp[1];
            const float xr = px * a - py * b;
            const float yr = px * b + py * a;
            const int ix = iround_f(xr), iy = iround_f(yr);
            t[e] = bl[(size_t)(cy + iy) * W + cx + ix];
          }
          val |= (t[0] < t[1]) << bit;
        }
        dsc[byte] = (uint8_t)val;
      }
      ++*n;
    }
    free(bl);
    free(cs);
    free(sc);
  }
  for (int l = 0; l < NLEV; ++l) free(lev[l]);
  return overflow;
}

/* orb_detector_using_tiles (orb.py:4-25) on one image.
 * kp: [cap][5] (x, y, size, angle, response) f32; octave [cap]; desc [cap][32].
 * Returns the keypoint count, or -(count) - 1 if cap was exceeded. */
int oracle_orb_tiles(const uint8_t* img, int H, int W, int stride, int max_kp, int overlap_div,
                     int height_div, int width_div, const int8_t* pattern, float* kp,
                     int32_t* octave, uint8_t* desc, int cap) {
  const int whole = height_div == 0 && width_div == 0;  /* orb_extraction_detect */
  const int tile_h = whole ? H : (int)((double)H / height_div);
  const int tile_w = whole ? W : (int)((double)W / width_div);
  const int ph = whole ? H : (int)(tile_h + (double)tile_h / overlap_div);
  const int pw = whole ? W : (int)(tile_w + (double)tile_w / overlap_div);
  const int ylim = whole ? 1 : H - tile_h, xlim = whole ? 1 : W - tile_w;
  okp* tmp = (okp*)malloc(sizeof(okp) * (cap > 0 ? cap : 1));
  int n = 0, overflow = 0;
  for (int y = 0; y < ylim; y += tile_h)
    for (int x = 0; x < xlim; x += tile_w) {
      const int h = ph < H - y ? ph : H - y;
      const int w = pw < W - x ? pw : W - x;
      const int n0 = n;
      overflow |= orb_patch(img + (size_t)y * stride + x, w, h, stride, max_kp, pattern, tmp, desc,
                            cap, &n);
      for (int i = n0; i < n; ++i) {
        kp[5 * i + 0] = (float)((double)tmp[i].x + x);
        kp[5 * i + 1] = (float)((double)tmp[i].y + y);
        kp[5 * i + 2] = tmp[i].size;
        kp[5 * i + 3] = tmp[i].angle;
        kp[5 * i + 4] = tmp[i].response;
        octave[i] = tmp[i].octave;
      }
    }
  free(tmp);
  return overflow ? -n - 1 : n;
}

/* Batched over images; counts[b] as oracle_orb_tiles returns. */
void oracle_orb_tiles_batch(const uint8_t* img, int B, int H, int W, int stride, int max_kp,
                            const int8_t* pattern, float* kp, int32_t* octave, uint8_t* desc,
                            int cap, int32_t* counts) {
#pragma omp parallel for schedule(dynamic, 1)
  for (int b = 0; b < B; ++b)
    counts[b] = oracle_orb_tiles(img + (size_t)b * H * stride, H, W, stride, max_kp, 2, 5, 10,
                                 pattern, kp + (size_t)b * cap * 5, octave + (size_t)b * cap,
                                 desc + (size_t)b * cap * 32, cap);
}
