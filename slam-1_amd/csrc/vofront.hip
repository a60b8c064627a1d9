// Alternative stereo-VO front end for gfx950:
//   visual_odometry.py:84-96    get_tiled_keypoints  (FAST, threshold 10, best 10 per 10x20 tile)
//   visual_odometry.py:98-112   track_keypoints      (cv2.calcOpticalFlowPyrLK, 15x15, 3 levels)
//   keypoint.py:13-32           track_keypoints_left_to_right (same LK, other filters)
//   visual_odometry.py:22-24    cv2.StereoSGBM (0..32 disparities, block 11, P1 968, P2 3872)
//   visual_odometry.py:114-134  calculate_right_qs + calc_3d
// The semantics are those restated in oracle/vofront.c (OpenCV 4.x FAST_t,
// LKTrackerInvoker, computeDisparitySGBM + medianBlur), reproduced bit for bit.
//
// Design:
//  * FAST: one wave per tile; the tile's score map and corner list stay in LDS;
//    corners are appended in detection order by ballot/mbcnt; a tile with more
//    than `per_tile` corners keeps the first ones of a stable sort by response
//    (exact rank); tiles are concatenated in row-major order by a per-image scan.
//  * LK: pyramids (pyrDown levels padded by win+1 with reflect-101, Scharr
//    derivatives padded with zeros) are built once per image and stay in HBM;
//    one wave tracks one point through every level: the 15x15 template and its
//    derivatives live in registers (4 pixels per lane), bilinear samples of the
//    next image come from L2, and the 2x2 system / mismatch vector are exact
//    64-bit wave reductions, so every lane takes the same float step.
//  * SGBM: the cost volume [y][x][d] (int16, d innermost: one 64-byte cell per
//    pixel) is built by a row kernel (prefilter + Birchfield-Tomasi + horizontal
//    box sum from LDS) and a column kernel (vertical running sum fused with the
//    top-down path); the diagonal paths run along diagonals and the left->right
//    and right->left paths along rows.  A path is walked by 16 lanes holding
//    D/16 disparities each: the d +- 1 neighbours and the min over d are DPP row
//    operations inside the 16-lane row.  The row kernel also selects the
//    disparity, interpolates, builds the right-view disparities (LDS atomicMin
//    on (cost, -x) keys) and applies the left-right check; a last kernel applies
//    the 3x3 median.
#include "common.hpp"
#include "dlt.hpp"

#include <cmath>

namespace {

constexpr int kBS = 256;

// ------------------------------------------------------------------ FAST
__device__ __forceinline__ int fast_score_t(const uint8_t* c, int st, int t) {
  const int v = c[0];
  {
    const int e0 = v - c[3 * st], e4 = v - c[3], e8 = v - c[-3 * st], e12 = v - c[-3];
    const unsigned dk = (e0 > t ? 1u : 0u) | (e4 > t ? 2u : 0u) | (e8 > t ? 4u : 0u) |
                        (e12 > t ? 8u : 0u);
    const unsigned br = (e0 < -t ? 1u : 0u) | (e4 < -t ? 2u : 0u) | (e8 < -t ? 4u : 0u) |
                        (e12 < -t ? 8u : 0u);
    const unsigned dk2 = dk & ((dk >> 1) | (dk << 3));
    const unsigned br2 = br & ((br >> 1) | (br << 3));
    if (((dk2 | br2) & 0xFu) == 0u) return 0;
  }
  int d[16];
  d[0] = v - c[3 * st];
  d[1] = v - c[3 * st + 1];
  d[2] = v - c[2 * st + 2];
  d[3] = v - c[st + 3];
  d[4] = v - c[3];
  d[5] = v - c[-st + 3];
  d[6] = v - c[-2 * st + 2];
  d[7] = v - c[-3 * st + 1];
  d[8] = v - c[-3 * st];
  d[9] = v - c[-3 * st - 1];
  d[10] = v - c[-2 * st - 2];
  d[11] = v - c[-st - 3];
  d[12] = v - c[-3];
  d[13] = v - c[st - 3];
  d[14] = v - c[2 * st - 2];
  d[15] = v - c[3 * st - 1];
  unsigned dark = 0, bright = 0;
#pragma unroll
  for (int k = 0; k < 16; ++k) {
    dark |= (d[k] > t ? 1u : 0u) << k;
    bright |= (d[k] < -t ? 1u : 0u) << k;
  }
  auto run9 = [](unsigned m) {
    unsigned mm = m | (m << 16), r = mm;
#pragma unroll
    for (int i = 1; i <= 8; ++i) r &= mm >> i;
    return (r & 0xFFFFu) != 0u;
  };
  if (!run9(dark) && !run9(bright)) return 0;
  int a0 = t;
#pragma unroll
  for (int k = 0; k < 16; k += 2) {
    int a = d[(k + 1) & 15];
#pragma unroll
    for (int j = 2; j <= 8; ++j) a = min(a, d[(k + j) & 15]);
    a0 = max(a0, min(a, d[k]));
    a0 = max(a0, min(a, d[(k + 9) & 15]));
  }
  int b0 = -a0;
#pragma unroll
  for (int k = 0; k < 16; k += 2) {
    int b = d[(k + 1) & 15];
#pragma unroll
    for (int j = 2; j <= 8; ++j) b = max(b, d[(k + j) & 15]);
    b0 = min(b0, max(b, d[k]));
    b0 = min(b0, max(b, d[(k + 9) & 15]));
  }
  return -b0 - 1;
}

struct FastGeom {
  int H, W, stride, th, tw, ntx, n_tiles, thr, per_tile;
  int map_bytes, list_cap, wave_lds;
};

// one wave per tile, 4 tiles per workgroup
__global__ __launch_bounds__(kBS) void k_fast_tiles(const uint8_t* __restrict__ img, FastGeom g,
                                                    float* __restrict__ ws_kp,
                                                    int32_t* __restrict__ ws_cnt) {
  extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
  const int wid = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int b = blockIdx.y;
  const int tile = blockIdx.x * (kBS / 64) + wid;
  const bool active = tile < g.n_tiles;
  uint8_t* sm = lds + wid * g.wave_lds;
  uint32_t* list = reinterpret_cast<uint32_t*>(sm + g.map_bytes);
  const int ty = active ? tile / g.ntx : 0, tx = active ? tile - ty * g.ntx : 0;
  const int y0 = ty * g.th, x0 = tx * g.tw;
  const int h = min(g.th, g.H - y0), w = min(g.tw, g.W - x0);
  const int rw = w - 6, rh = h - 6;  // detection region [3, w-4] x [3, h-4]
  const int npos = (active && rw > 0 && rh > 0) ? rw * rh : 0;
  const uint8_t* base = img + (size_t)b * g.H * g.stride + (size_t)y0 * g.stride + x0;
  for (int i = lane; i < g.th * g.tw; i += 64) sm[i] = 0;
  __syncthreads();
  for (int p = lane; p < npos; p += 64) {
    const int y = 3 + p / rw, x = 3 + p % rw;
    sm[y * w + x] = (uint8_t)fast_score_t(base + (size_t)y * g.stride + x, g.stride, g.thr);
  }
  __syncthreads();
  // strict 3x3 NMS in detection (row-major) order
  int m = 0;
  for (int c = 0; c < npos; c += 64) {
    const int p = c + lane;
    bool keep = false;
    uint32_t key = 0;
    if (p < npos) {
      const int y = 3 + p / rw, x = 3 + p % rw;
      const uint8_t* q = sm + y * w + x;
      const int s = q[0];
      keep = s > 0 && s > q[-1] && s > q[1] && s > q[-w - 1] && s > q[-w] && s > q[-w + 1] &&
             s > q[w - 1] && s > q[w] && s > q[w + 1];
      key = ((uint32_t)s << 24) | ((uint32_t)y << 12) | (uint32_t)x;
    }
    const unsigned long long bal = __ballot(keep);
    const int pre = __popcll(bal & ((1ull << lane) - 1ull));
    if (keep && m + pre < g.list_cap) list[m + pre] = key;
    m += __popcll(bal);
  }
  __syncthreads();
  m = min(m, g.list_cap);
  if (!active) return;
  const size_t slot = (size_t)b * g.n_tiles + tile;
  float* out = ws_kp + slot * g.per_tile * 3;
  const int take = min(m, g.per_tile);
  for (int i = lane; i < m; i += 64) {
    const uint32_t ki = list[i];
    int r = i;
    if (m > g.per_tile) {  // stable sort by response descending
      const uint32_t si = ki >> 24;
      r = 0;
      for (int j = 0; j < m; ++j) {
        const uint32_t sj = list[j] >> 24;
        r += (sj > si || (sj == si && j < i)) ? 1 : 0;
      }
    }
    if (r < take) {
      out[r * 3 + 0] = (float)((int)(ki & 4095u) + x0);
      out[r * 3 + 1] = (float)((int)((ki >> 12) & 4095u) + y0);
      out[r * 3 + 2] = (float)(ki >> 24);
    }
  }
  if (lane == 0) ws_cnt[slot] = take;
}

// concatenate the tiles of each image (row-major tile order)
__global__ __launch_bounds__(1024) void k_fast_compact(const float* __restrict__ ws_kp,
                                                       const int32_t* __restrict__ ws_cnt,
                                                       int n_tiles, int per_tile,
                                                       float* __restrict__ kp,
                                                       int32_t* __restrict__ count, int cap) {
  __shared__ int wsum[16];
  __shared__ int total;
  const int b = blockIdx.x, t = threadIdx.x, lane = t & 63, wid = t >> 6;
  const int per = (n_tiles + 1023) / 1024;
  const int t0 = min(t * per, n_tiles), t1 = min(t0 + per, n_tiles);
  const int32_t* cnt = ws_cnt + (size_t)b * n_tiles;
  int s = 0;
  for (int i = t0; i < t1; ++i) s += cnt[i];
  // block exclusive scan of s
  int inc = s;
  for (int o = 1; o < 64; o <<= 1) {
    const int v = __shfl_up(inc, o, 64);
    if (lane >= o) inc += v;
  }
  if (lane == 63) wsum[wid] = inc;
  __syncthreads();
  if (t == 0) {
    int a = 0;
    for (int i = 0; i < 16; ++i) {
      const int v = wsum[i];
      wsum[i] = a;
      a += v;
    }
    total = a;
  }
  __syncthreads();
  int off = wsum[wid] + inc - s;
  const int tot = total;
  if (t == 0) count[b] = tot > cap ? -tot - 1 : tot;
  if (tot > cap) return;
  for (int i = t0; i < t1; ++i) {
    const int c = cnt[i];
    const float* src = ws_kp + ((size_t)b * n_tiles + i) * per_tile * 3;
    float* dst = kp + ((size_t)b * cap + off) * 3;
    for (int j = 0; j < c * 3; ++j) dst[j] = src[j];
    off += c;
  }
}

// ---------------------------------------------------------------- LK pyramids
constexpr int kMaxLev = 8;

struct LkGeom {
  int nlev, B;  // levels, border (win + 1)
  int w[kMaxLev], h[kMaxLev], pitch[kMaxLev];
  long long off[kMaxLev];  // byte / element offset of level l's (0, 0) pixel in an image block
  long long img_bytes;     // one image's pyramid (bytes) == one image's derivatives (elements)
};

__host__ __device__ inline int refl101(int i, int n) {
  if (n == 1) return 0;
  while (i < 0 || i >= n) i = i < 0 ? -i : 2 * n - 2 - i;
  return i;
}

int lk_geom(int H, int W, int win, int max_level, LkGeom* g) {
  SLAM_REQUIRE(H > 0 && W > 0 && win >= 3 && win <= 16, "slam_lk: window in [3, 16]");
  SLAM_REQUIRE(max_level >= 0 && max_level < kMaxLev, "slam_lk: max_level in [0, %d]", kMaxLev - 1);
  g->B = win + 1;
  int w = W, h = H, n = 0;
  long long off = 0;
  for (int l = 0; l <= max_level; ++l) {
    g->w[l] = w;
    g->h[l] = h;
    g->pitch[l] = (w + 2 * g->B + 15) & ~15;
    g->off[l] = off + (long long)g->B * g->pitch[l] + g->B;
    off += (long long)g->pitch[l] * (h + 2 * g->B);
    n = l + 1;
    w = (w + 1) / 2;
    h = (h + 1) / 2;
    if (w <= win || h <= win) break;
  }
  g->nlev = n;
  g->img_bytes = (off + 255) & ~255ll;
  return SLAM_OK;
}

// level 0: bordered copy (reflect-101)
__global__ __launch_bounds__(kBS) void k_lk_level0(const uint8_t* __restrict__ img, int stride,
                                                   LkGeom g, uint8_t* __restrict__ pyr) {
  const int i = blockIdx.x * kBS + threadIdx.x, n = blockIdx.y;
  const int pw = g.w[0] + 2 * g.B, ph = g.h[0] + 2 * g.B;
  if (i >= pw * ph) return;
  const int y = i / pw - g.B, x = i % pw - g.B;
  const uint8_t v = img[(size_t)n * g.h[0] * stride + (size_t)refl101(y, g.h[0]) * stride +
                        refl101(x, g.w[0])];
  pyr[(size_t)n * g.img_bytes + g.off[0] + (long long)y * g.pitch[0] + x] = v;
}

// level l = pyrDown(level l-1), written with its reflect-101 border
__global__ __launch_bounds__(kBS) void k_lk_pyrdown(LkGeom g, int l, uint8_t* __restrict__ pyr) {
  const int i = blockIdx.x * kBS + threadIdx.x, n = blockIdx.y;
  const int pw = g.w[l] + 2 * g.B, ph = g.h[l] + 2 * g.B;
  if (i >= pw * ph) return;
  const int y = i / pw - g.B, x = i % pw - g.B;
  const int yi = refl101(y, g.h[l]), xi = refl101(x, g.w[l]);
  const uint8_t* s = pyr + (size_t)n * g.img_bytes + g.off[l - 1];
  const int sp = g.pitch[l - 1];
  const int k[5] = {1, 4, 6, 4, 1};
  int acc = 0;
#pragma unroll
  for (int r = 0; r < 5; ++r) {
    const uint8_t* row = s + (long long)(2 * yi - 2 + r) * sp + 2 * xi - 2;
    const int hsum = row[0] + 4 * row[1] + 6 * row[2] + 4 * row[3] + row[4];
    acc += k[r] * hsum;
  }
  pyr[(size_t)n * g.img_bytes + g.off[l] + (long long)y * g.pitch[l] + x] = (uint8_t)((acc + 128) >> 8);
}

// calcSharrDeriv of level l, zero border
__global__ __launch_bounds__(kBS) void k_lk_scharr(LkGeom g, int l, const uint8_t* __restrict__ pyr,
                                                   short2* __restrict__ der) {
  const int i = blockIdx.x * kBS + threadIdx.x, n = blockIdx.y;
  const int pw = g.w[l] + 2 * g.B, ph = g.h[l] + 2 * g.B;
  if (i >= pw * ph) return;
  const int y = i / pw - g.B, x = i % pw - g.B;
  short2 o = make_short2(0, 0);
  if (x >= 0 && y >= 0 && x < g.w[l] && y < g.h[l]) {
    const uint8_t* s = pyr + (size_t)n * g.img_bytes + g.off[l] + (long long)y * g.pitch[l] + x;
    const int p = g.pitch[l];
    auto t0 = [&](int dx) { return (int)(short)((s[-p + dx] + s[p + dx]) * 3 + s[dx] * 10); };
    auto t1 = [&](int dx) { return (int)(short)(s[p + dx] - s[-p + dx]); };
    o.x = (short)(t0(1) - t0(-1));
    o.y = (short)((t1(1) + t1(-1)) * 3 + t1(0) * 10);
  }
  der[(size_t)n * g.img_bytes + g.off[l] + (long long)y * g.pitch[l] + x] = o;
}

// Exact wave sum of per-lane int32 partials whose 16-lane row sums fit int32
// (|lane partial| <= 4 * 8160 * 4080 = 133M, so |row sum| < 2^31): DPP sums
// inside each 16-lane row, then the four row sums added in 64 bits.
__device__ __forceinline__ long long wave_sum_i32(int v) {
  v += __builtin_amdgcn_mov_dpp(v, 0xB1, 0xF, 0xF, false);   // quad_perm [1,0,3,2]
  v += __builtin_amdgcn_mov_dpp(v, 0x4E, 0xF, 0xF, false);   // quad_perm [2,3,0,1]
  v += __builtin_amdgcn_mov_dpp(v, 0x124, 0xF, 0xF, false);  // row_ror:4
  v += __builtin_amdgcn_mov_dpp(v, 0x128, 0xF, 0xF, false);  // row_ror:8
  return (long long)__builtin_amdgcn_readlane(v, 0) + (long long)__builtin_amdgcn_readlane(v, 16) +
         (long long)__builtin_amdgcn_readlane(v, 32) + (long long)__builtin_amdgcn_readlane(v, 48);
}

__device__ __forceinline__ int descale(int x, int n) { return (x + (1 << (n - 1))) >> n; }

struct LkArgs {
  const uint8_t* prev;
  const short2* der;
  const uint8_t* next;
  long long pyr_stride, der_stride;  // per pair
  int max_count;
  double eps2;
  float min_eig;
  int win;
  const float* pts;
  const int32_t* npts;
  int cap, pts_stride;  // floats per point in pts (2 or 3)
  float* out;
  uint8_t* status;
  float* err;
};

// one wave per point, all levels (LKTrackerInvoker, coarsest level first)
__global__ __launch_bounds__(kBS) void k_lk_track(LkGeom g, LkArgs a) {
  const int lane = threadIdx.x & 63;
  const int pt = blockIdx.x * (kBS / 64) + (threadIdx.x >> 6), b = blockIdx.y;
  const int n = min(max(a.npts[b], 0), a.cap);
  if (pt >= n) return;
  const int win = a.win, area = win * win;
  const float hw = (float)(win - 1) * 0.5f;
  const float FLT_SCALE = 1.f / (1 << 20);
  const size_t o = (size_t)b * a.cap + pt;
  const float px = a.pts[o * a.pts_stride], py = a.pts[o * a.pts_stride + 1];
  int st = 1;
  if (!(fabsf(px) < 1e7f) || !(fabsf(py) < 1e7f)) {  // not finite / absurd: not trackable
    if (lane == 0) {
      a.out[2 * o] = px;
      a.out[2 * o + 1] = py;
      a.status[o] = 0;
      a.err[o] = 0.f;
    }
    return;
  }
  float er = 0.f, npx = 0.f, npy = 0.f;
  const uint8_t* prevb = a.prev + b * a.pyr_stride;
  const uint8_t* nextb = a.next + b * a.pyr_stride;
  const short2* derb = a.der + b * a.der_stride;
  // this lane's window pixels: p = lane + 64 k
  int pr[4], pc[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int p = lane + 64 * k;
    pr[k] = p < area ? p / win : 0;
    pc[k] = p < area ? p % win : 0;
  }
  bool vk[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) vk[k] = lane + 64 * k < area;
  for (int level = g.nlev - 1; level >= 0; --level) {
    const int lw = g.w[level], lh = g.h[level], pitch = g.pitch[level];
    const uint8_t* I = prevb + g.off[level];
    const uint8_t* J = nextb + g.off[level];
    const short2* dI = derb + g.off[level];
    const float sc = (float)(1. / (1 << level));
    float prx = px * sc, pry = py * sc;
    float nx, ny;
    if (level == g.nlev - 1) {
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
    if (ipx < -win || ipx >= lw || ipy < -win || ipy >= lh) {
      if (level == 0) {
        st = 0;
        er = 0.f;
      }
      continue;
    }
    float fa = prx - (float)ipx, fb = pry - (float)ipy;
    int iw00 = (int)rintf((1.f - fa) * (1.f - fb) * 16384.f);
    int iw01 = (int)rintf(fa * (1.f - fb) * 16384.f);
    int iw10 = (int)rintf((1.f - fa) * fb * 16384.f);
    int iw11 = 16384 - iw00 - iw01 - iw10;
    int Iv[4], Ix[4], Iy[4];
    int s11 = 0, s12 = 0, s22 = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      Iv[k] = Ix[k] = Iy[k] = 0;
      if (vk[k]) {
        const long long q = (long long)(ipy + pr[k]) * pitch + ipx + pc[k];
        const uint8_t* s = I + q;
        Iv[k] = descale(s[0] * iw00 + s[1] * iw01 + s[pitch] * iw10 + s[pitch + 1] * iw11, 9);
        const short2* d = dI + q;
        const short2 d00 = d[0], d01 = d[1], d10 = d[pitch], d11 = d[pitch + 1];
        Ix[k] = descale(d00.x * iw00 + d01.x * iw01 + d10.x * iw10 + d11.x * iw11, 14);
        Iy[k] = descale(d00.y * iw00 + d01.y * iw01 + d10.y * iw10 + d11.y * iw11, 14);
        s11 += Ix[k] * Ix[k];
        s12 += Ix[k] * Iy[k];
        s22 += Iy[k] * Iy[k];
      }
    }
    const float A11 = (float)wave_sum_i32(s11) * FLT_SCALE;
    const float A12 = (float)wave_sum_i32(s12) * FLT_SCALE;
    const float A22 = (float)wave_sum_i32(s22) * FLT_SCALE;
    float D = A11 * A22 - A12 * A12;
    const float dd = A11 - A22;
    const float minEig = (A22 + A11 - sqrtf(dd * dd + 4.f * A12 * A12)) / (float)(2 * area);
    if (minEig < a.min_eig || D < 1.1920928955078125e-07f) {
      if (level == 0) st = 0;
      continue;
    }
    D = 1.f / D;
    nx -= hw;
    ny -= hw;
    float pdx = 0.f, pdy = 0.f;
    for (int j = 0; j < a.max_count; ++j) {
      const int inx = (int)floorf(nx), iny = (int)floorf(ny);
      if (inx < -win || inx >= lw || iny < -win || iny >= lh) {
        if (level == 0) st = 0;
        break;
      }
      fa = nx - (float)inx;
      fb = ny - (float)iny;
      iw00 = (int)rintf((1.f - fa) * (1.f - fb) * 16384.f);
      iw01 = (int)rintf(fa * (1.f - fb) * 16384.f);
      iw10 = (int)rintf((1.f - fa) * fb * 16384.f);
      iw11 = 16384 - iw00 - iw01 - iw10;
      int b1 = 0, b2 = 0;
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        if (vk[k]) {
          const uint8_t* s = J + (long long)(iny + pr[k]) * pitch + inx + pc[k];
          const int diff =
              descale(s[0] * iw00 + s[1] * iw01 + s[pitch] * iw10 + s[pitch + 1] * iw11, 9) - Iv[k];
          b1 += diff * Ix[k];
          b2 += diff * Iy[k];
        }
      }
      const float fb1 = (float)wave_sum_i32(b1) * FLT_SCALE;
      const float fb2 = (float)wave_sum_i32(b2) * FLT_SCALE;
      const float dx = (A12 * fb2 - A22 * fb1) * D;
      const float dy = (A12 * fb1 - A11 * fb2) * D;
      nx += dx;
      ny += dy;
      npx = nx + hw;
      npy = ny + hw;
      if ((double)dx * dx + (double)dy * dy <= a.eps2) break;
      if (j > 0 && fabs((double)(dx + pdx)) < 0.01 && fabs((double)(dy + pdy)) < 0.01) {
        npx -= dx * 0.5f;
        npy -= dy * 0.5f;
        break;
      }
      pdx = dx;
      pdy = dy;
    }
    if (st && level == 0) {
      const float qx = npx - hw, qy = npy - hw;
      const int inx = (int)floorf(qx), iny = (int)floorf(qy);
      if (inx < -win || inx >= lw || iny < -win || iny >= lh) {
        st = 0;
        continue;
      }
      const float aa = qx - (float)inx, bb = qy - (float)iny;
      iw00 = (int)rintf((1.f - aa) * (1.f - bb) * 16384.f);
      iw01 = (int)rintf(aa * (1.f - bb) * 16384.f);
      iw10 = (int)rintf((1.f - aa) * bb * 16384.f);
      iw11 = 16384 - iw00 - iw01 - iw10;
      int e = 0;  // sum |diff| < 2^24: exact as the reference's float sum
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        if (vk[k]) {
          const uint8_t* s = J + (long long)(iny + pr[k]) * pitch + inx + pc[k];
          const int diff =
              descale(s[0] * iw00 + s[1] * iw01 + s[pitch] * iw10 + s[pitch + 1] * iw11, 9) - Iv[k];
          e += diff < 0 ? -diff : diff;
        }
      }
      er = (float)wave_sum_i32(e) * 1.f / (float)(32 * area);
    }
  }
  if (lane == 0) {
    a.out[2 * o] = npx;
    a.out[2 * o + 1] = npy;
    a.status[o] = (uint8_t)st;
    a.err[o] = er;
  }
}

// ---------------------------------------------------------------------- SGBM
constexpr int kMaxCost = 32767;

struct SgbmGeom {
  int H, W, stride, minD, D, W1, minX1, SW2, SH2, P1, P2;
  long long vol;  // int16 elements per image volume (H * W1 * D)
};

__device__ __forceinline__ int sat16(int v) { return min(max(v, -32768), kMaxCost); }

// DPP inside 16-lane rows
__device__ __forceinline__ int dpp_shr1(int v, int old) {
  return __builtin_amdgcn_update_dpp(old, v, 0x111, 0xF, 0xF, false);
}
__device__ __forceinline__ int dpp_shl1(int v, int old) {
  return __builtin_amdgcn_update_dpp(old, v, 0x101, 0xF, 0xF, false);
}
__device__ __forceinline__ int row_min16(int v) {
  v = min(v, __builtin_amdgcn_mov_dpp(v, 0xB1, 0xF, 0xF, false));   // quad_perm [1,0,3,2]
  v = min(v, __builtin_amdgcn_mov_dpp(v, 0x4E, 0xF, 0xF, false));   // quad_perm [2,3,0,1]
  v = min(v, __builtin_amdgcn_mov_dpp(v, 0x124, 0xF, 0xF, false));  // row_ror:4
  v = min(v, __builtin_amdgcn_mov_dpp(v, 0x128, 0xF, 0xF, false));  // row_ror:8
  return v;
}

// One step of a path: Lp (this lane's DPL previous values) -> L; mp = min over d
// of the previous cell (uniform in the 16-lane row).  Returns the new min.
template <int DPL>
__device__ __forceinline__ int path_step(const int (&C)[DPL], int (&L)[DPL], int mp, int P1,
                                         int P2) {
  const int delta = mp + P2;
  const int left = dpp_shr1(L[DPL - 1], kMaxCost);
  const int right = dpp_shl1(L[0], kMaxCost);
  int Ln[DPL];
  int mn = kMaxCost;
#pragma unroll
  for (int i = 0; i < DPL; ++i) {
    const int lm = i > 0 ? L[i - 1] : left;
    const int lp = i < DPL - 1 ? L[i + 1] : right;
    const int m = min(L[i], min(lm + P1, min(lp + P1, delta)));
    Ln[i] = C[i] + m - delta;
    mn = min(mn, Ln[i]);
  }
#pragma unroll
  for (int i = 0; i < DPL; ++i) L[i] = Ln[i];
  return row_min16(mn);
}

template <int DPL>
__device__ __forceinline__ void load_cell(const int16_t* p, int (&v)[DPL]) {
  if constexpr (DPL == 2) {
    const uint32_t u = *reinterpret_cast<const uint32_t*>(p);
    v[0] = (int)(int16_t)(u & 0xFFFFu);
    v[1] = (int)(int16_t)(u >> 16);
  } else {
    const uint2 u = *reinterpret_cast<const uint2*>(p);
    v[0] = (int)(int16_t)(u.x & 0xFFFFu);
    v[1] = (int)(int16_t)(u.x >> 16);
    v[2] = (int)(int16_t)(u.y & 0xFFFFu);
    v[3] = (int)(int16_t)(u.y >> 16);
  }
}

template <int DPL>
__device__ __forceinline__ void store_cell(int16_t* p, const int (&v)[DPL]) {
  if constexpr (DPL == 2) {
    *reinterpret_cast<uint32_t*>(p) = ((uint32_t)(uint16_t)v[0]) | ((uint32_t)(uint16_t)v[1] << 16);
  } else {
    uint2 u;
    u.x = ((uint32_t)(uint16_t)v[0]) | ((uint32_t)(uint16_t)v[1] << 16);
    u.y = ((uint32_t)(uint16_t)v[2]) | ((uint32_t)(uint16_t)v[3] << 16);
    *reinterpret_cast<uint2*>(p) = u;
  }
}

// Raw cells for register prefetch rings (loads issued kPF steps ahead of use).
constexpr int kPF = 8;
template <int DPL>
struct RawCell;
template <>
struct RawCell<2> {
  uint32_t u;
  __device__ __forceinline__ void load(const int16_t* p) { u = *reinterpret_cast<const uint32_t*>(p); }
  __device__ __forceinline__ void get(int (&v)[2]) const {
    v[0] = (int)(int16_t)(u & 0xFFFFu);
    v[1] = (int)(int16_t)(u >> 16);
  }
};
template <>
struct RawCell<4> {
  uint2 u;
  __device__ __forceinline__ void load(const int16_t* p) { u = *reinterpret_cast<const uint2*>(p); }
  __device__ __forceinline__ void get(int (&v)[4]) const {
    v[0] = (int)(int16_t)(u.x & 0xFFFFu);
    v[1] = (int)(int16_t)(u.x >> 16);
    v[2] = (int)(int16_t)(u.y & 0xFFFFu);
    v[3] = (int)(int16_t)(u.y >> 16);
  }
};

// K1: per (image, row, 64-column band): prefilter + BT pixel costs + horizontal
// 11-sum (replicated at x = 0, W1-1) -> hs[y][x][d]
constexpr int kHsBand = 64;
constexpr int kHsRows = 4;

template <int D>
__global__ __launch_bounds__(kBS) void k_sgbm_hsum(const uint8_t* __restrict__ left,
                                                   const uint8_t* __restrict__ right, SgbmGeom g,
                                                   int16_t* __restrict__ hs) {
  constexpr int kMaxWin = kHsBand + 20 + 64 + D + 4;  // min_disp <= 64, block <= 21
  __shared__ uint8_t ch[4][4][kMaxWin];  // [L0,L1,R0,R1][v, lo, hi, -][col]
  __shared__ int16_t pc[(kHsBand + 20) * D];
  const int band = blockIdx.x, n = blockIdx.z, t = threadIdx.x;
  const int x0 = band * kHsBand, xe = min(x0 + kHsBand, g.W1);
  const int SW2 = g.SW2;
  // pixel-cost columns (relative to minX1), clamped: [max(x0 - SW2, 0), min(xe + SW2, W1))
  const int pc_lo = max(x0 - SW2, 0), pc_hi = min(xe + SW2, g.W1);
  // absolute image window: right columns from pc_lo + minX1 - (minD + D - 1), left up to pc_hi + minX1
  const int wlo = max(pc_lo + g.minX1 - (g.minD + D - 1) - 1, 0);
  const int whi = min(pc_hi + g.minX1 + 1, g.W);
  const int nw = whi - wlo;
  const uint8_t* img[2] = {left + (size_t)n * g.H * g.stride, right + (size_t)n * g.H * g.stride};
  __shared__ uint8_t raw[4][kMaxWin + 2];
  // kHsRows rows per workgroup (fewer, longer workgroups: the per-row work is small)
  const int y_end = min((int)(blockIdx.y + 1) * kHsRows, g.H);
  for (int y = blockIdx.y * kHsRows; y < y_end; ++y) {
    const int yn = y > 0 ? y - 1 : y, ys = y < g.H - 1 ? y + 1 : y;
    // channel values over [wlo - 1, whi + 1) are needed for the BT min/max; compute v on
    // [wlo - 1, whi + 1) into a staging pass (index c = x - wlo + 1)
    for (int i = t; i < 2 * (nw + 2); i += kBS) {
      const int im = i / (nw + 2), c = i % (nw + 2), x = wlo - 1 + c;
      uint8_t v0 = 15, v1 = 15;
      if (x >= 1 && x < g.W - 1) {
        const uint8_t* r = img[im] + (size_t)y * g.stride;
        const uint8_t* rn = img[im] + (size_t)yn * g.stride;
        const uint8_t* rs = img[im] + (size_t)ys * g.stride;
        int v = (r[x + 1] - r[x - 1]) * 2 + rn[x + 1] - rn[x - 1] + rs[x + 1] - rs[x - 1];
        v = min(max(v, -15), 15);
        v0 = (uint8_t)(v + 15);
        v1 = r[x];
      }
      raw[2 * im][c] = v0;
      raw[2 * im + 1][c] = v1;
    }
    __syncthreads();
    for (int i = t; i < 4 * nw; i += kBS) {
      const int k = i / nw, c = i % nw, x = wlo + c;
      const int v = raw[k][c + 1];
      const int vl = x > 0 ? (v + raw[k][c]) / 2 : v;
      const int vr = x < g.W - 1 ? (v + raw[k][c + 2]) / 2 : v;
      ch[k][0][c] = (uint8_t)v;
      ch[k][1][c] = (uint8_t)min(min(vl, vr), v);
      ch[k][2][c] = (uint8_t)max(max(vl, vr), v);
    }
    __syncthreads();
    const int npc = pc_hi - pc_lo;
    for (int i = t; i < npc * D; i += kBS) {
      const int xc = pc_lo + i / D, d = i % D;
      const int xa = xc + g.minX1, xr = xa - (d + g.minD);
      const int cl = xa - wlo, cr = xr - wlo;
      int cost = 0;
  #pragma unroll
      for (int c = 0; c < 2; ++c) {
        const int u = ch[c][0][cl], u0 = ch[c][1][cl], u1 = ch[c][2][cl];
        const int v = ch[2 + c][0][cr], v0 = ch[2 + c][1][cr], v1 = ch[2 + c][2][cr];
        const int c0 = max(max(0, u - v1), v0 - u);
        const int c1 = max(max(0, v - u1), u0 - v);
        cost += min(c0, c1) >> (c ? 2 : 0);
      }
      pc[(xc - pc_lo) * D + d] = (int16_t)cost;
    }
    __syncthreads();
    // sliding horizontal sums: thread = (d, run of kHsBand / (kBS / D) columns)
    int16_t* out = hs + (size_t)n * g.vol + (size_t)y * g.W1 * D;
    constexpr int kRun = kHsBand / (kBS / D);
    const int d = t % D, xr0 = x0 + (t / D) * kRun;
    if (xr0 < xe) {
      auto at = [&](int x) { return (int)pc[(min(max(x, 0), g.W1 - 1) - pc_lo) * D + d]; };
      int s = 0;
      for (int dx = -SW2; dx <= SW2; ++dx) s += at(xr0 + dx);
      out[(size_t)xr0 * D + d] = (int16_t)s;
      for (int x = xr0 + 1; x < min(xr0 + kRun, xe); ++x) {
        s += at(x + SW2) - at(x - SW2 - 1);
        out[(size_t)x * D + d] = (int16_t)s;
      }
    }

    __syncthreads();  // raw / ch / pc are reused by the next row
  }
}

// K2: per (image, 16 columns): vertical running sum -> C, fused with the
// top-down path (direction 2) -> L2.  Lane group of 16 = one column.
template <int D>
__global__ __launch_bounds__(kBS) void k_sgbm_vert(const int16_t* __restrict__ hs, SgbmGeom g,
                                                   int16_t* __restrict__ Cv,
                                                   int16_t* __restrict__ L2v) {
  constexpr int DPL = D / 16;
  const int n = blockIdx.y, t = threadIdx.x;
  const int x = blockIdx.x * 16 + (t >> 4), j = t & 15;
  const bool live = x < g.W1;  // dead groups still run the DPP (rows are independent)
  const int xs = live ? x : g.W1 - 1;
  const size_t rowst = (size_t)g.W1 * D;
  const int16_t* h = hs + (size_t)n * g.vol + (size_t)xs * D + j * DPL;
  int16_t* co = Cv + (size_t)n * g.vol + (size_t)xs * D + j * DPL;
  int16_t* lo = L2v + (size_t)n * g.vol + (size_t)xs * D + j * DPL;
  const int H = g.H, SH2 = g.SH2;
  int C[DPL], L[DPL], tmp[DPL];
#pragma unroll
  for (int i = 0; i < DPL; ++i) C[i] = L[i] = 0;
  for (int k = -SH2; k <= SH2; ++k) {
    load_cell<DPL>(h + (size_t)min(max(k, 0), H - 1) * rowst, tmp);
#pragma unroll
    for (int i = 0; i < DPL; ++i) C[i] += tmp[i];
  }
  int mp = 0;
  // rows y + SH2 (added) and y - SH2 - 1 (removed) of the running sum, kPF rows ahead
  RawCell<DPL> ra[kPF], rs[kPF];
#pragma unroll
  for (int k = 0; k < kPF; ++k) {
    ra[k].load(h + (size_t)min(k + SH2, H - 1) * rowst);
    rs[k].load(h + (size_t)max(k - SH2 - 1, 0) * rowst);
  }
  for (int y0 = 0; y0 < H; y0 += kPF) {
#pragma unroll
    for (int k = 0; k < kPF; ++k) {
      const int y = y0 + k;
      if (y < H) {
        int a[DPL], b[DPL];
        ra[k].get(a);
        rs[k].get(b);
        const int yn = y + kPF;
        if (yn < H) {
          ra[k].load(h + (size_t)min(yn + SH2, H - 1) * rowst);
          rs[k].load(h + (size_t)max(yn - SH2 - 1, 0) * rowst);
        }
        if (y > 0) {
#pragma unroll
          for (int i = 0; i < DPL; ++i) C[i] += a[i] - b[i];
        }
        mp = path_step<DPL>(C, L, mp, g.P1, g.P2);
        if (live) {
          store_cell<DPL>(co + (size_t)y * rowst, C);
          store_cell<DPL>(lo + (size_t)y * rowst, L);
        }
      }
    }
  }
}

// K3: diagonal paths.  DX = +1: from (x-1, y-1) (walk x+1, y+1);
// DX = -1: from (x+1, y-1) (walk x-1, y+1).  One 16-lane row per path.
template <int D, int DX, int DY>
__device__ __forceinline__ void sgbm_path(const int16_t* __restrict__ Cv, const SgbmGeom& g,
                                          int16_t* __restrict__ Lv);

// three path directions in one launch (blockIdx.z): 0 -> from (x-1, y-1) into
// L1, 1 -> from (x+1, y-1) into L3, 2 -> from (x+1, y) (right to left along
// the row) into L4: all independent paths in flight together
template <int D>
__global__ __launch_bounds__(kBS) void k_sgbm_paths(const int16_t* __restrict__ Cv, SgbmGeom g,
                                                    int16_t* __restrict__ L1v,
                                                    int16_t* __restrict__ L3v,
                                                    int16_t* __restrict__ L4v) {
  if (blockIdx.z == 0)
    sgbm_path<D, 1, 1>(Cv, g, L1v);
  else if (blockIdx.z == 1)
    sgbm_path<D, -1, 1>(Cv, g, L3v);
  else
    sgbm_path<D, -1, 0>(Cv, g, L4v);
}

template <int D, int DX, int DY>
__device__ __forceinline__ void sgbm_path(const int16_t* __restrict__ Cv, const SgbmGeom& g,
                                          int16_t* __restrict__ Lv) {
  constexpr int DPL = D / 16;
  const int n = blockIdx.y, t = threadIdx.x, j = t & 15;
  const int p = blockIdx.x * 16 + (t >> 4);
  const int np = DY ? g.W1 + g.H - 1 : g.H;
  if (blockIdx.x * 16 >= np) return;  // whole workgroup past the paths (uniform)
  const bool live = p < np;
  int x, y;
  if (!DY) {  // row p, walked from the right end
    x = g.W1 - 1;
    y = p;
  } else if (p < g.W1) {
    x = DX > 0 ? p : g.W1 - 1 - p;
    y = 0;
  } else {
    x = DX > 0 ? 0 : g.W1 - 1;
    y = p - g.W1 + 1;
  }
  int len = 0;
  if (live) len = DY ? min(DX > 0 ? g.W1 - x : x + 1, g.H - y) : g.W1;
  // the 16 lanes of a row share len; rows of a wave differ, so loop to the wave max
  int lmax = len;
#pragma unroll
  for (int o = 16; o < 64; o <<= 1) lmax = max(lmax, __shfl_xor(lmax, o, 64));
  const size_t rowst = (size_t)g.W1 * D;
  const int16_t* c = Cv + (size_t)n * g.vol + (size_t)y * rowst + (size_t)x * D + j * DPL;
  int16_t* lo = Lv + (size_t)n * g.vol + (size_t)y * rowst + (size_t)x * D + j * DPL;
  const long long step = (long long)DY * rowst + (long long)DX * D;
  int L[DPL];
#pragma unroll
  for (int i = 0; i < DPL; ++i) L[i] = 0;
  int mp = 0;
  RawCell<DPL> rc[kPF];
#pragma unroll
  for (int k = 0; k < kPF; ++k)
    if (k < len) rc[k].load(c + k * step);
  for (int k0 = 0; k0 < lmax; k0 += kPF) {
#pragma unroll
    for (int k = 0; k < kPF; ++k) {
      const int i = k0 + k;
      if (i < lmax) {
        int C[DPL];
        rc[k].get(C);
        if (i + kPF < len) rc[k].load(c + (i + kPF) * step);
        mp = path_step<DPL>(C, L, mp, g.P1, g.P2);
        if (i < len) store_cell<DPL>(lo + i * step, L);
      }
    }
  }
}

// K4: per 4 rows (one 16-lane row each), one left->right pass: the left->right
// path L0 and S = sat16(sat16(L0 + L1 + L2 + L3) + L4), first-minimum argmin
// by packed-key DPP min, subpixel (neighbours by DPP row shifts in the owner
// lane), right-view disparities by LDS atomicMin on (cost, -x) keys (ties to
// the larger x, as the reference's right-to-left visit), then the left-right
// check -> raw disparity row.
template <int D>
__global__ __launch_bounds__(64) void k_sgbm_row(const int16_t* __restrict__ Cv,
                                                 const int16_t* __restrict__ L1v,
                                                 const int16_t* __restrict__ L2v,
                                                 const int16_t* __restrict__ L3v,
                                                 const int16_t* __restrict__ L4v, SgbmGeom g,
                                                 int16_t* __restrict__ raw) {
  constexpr int DPL = D / 16;
  constexpr int kPFR = 16;  // cells in flight per lane and volume
  extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
  const int t = threadIdx.x, r = t >> 4, j = t & 15, n = blockIdx.y;
  const int y = blockIdx.x * 4 + r;
  const bool live = y < g.H;
  const int ys = live ? y : g.H - 1;
  const int W = g.W, W1 = g.W1, minX1 = g.minX1;
  uint32_t* cost2 = reinterpret_cast<uint32_t*>(lds) + r * W;
  // the row's left-view disparities go straight to `raw` (only live rows write)
  int16_t* out = raw + (size_t)n * g.H * W + (size_t)ys * W;
  const int INVALID = (g.minD - 1) * 16;
  for (int x = j; x < W; x += 16) {
    cost2[x] = 0xFFFFFFFFu;
    if (live) out[x] = (int16_t)INVALID;
  }
  __syncthreads();
  const size_t base = (size_t)n * g.vol + (size_t)ys * W1 * D + j * DPL;
  const int16_t* c = Cv + base;
  const int16_t* l1 = L1v + base;
  const int16_t* l2 = L2v + base;
  const int16_t* l3 = L3v + base;
  const int16_t* l4 = L4v + base;
  int L[DPL];
#pragma unroll
  for (int i = 0; i < DPL; ++i) L[i] = 0;
  int mp = 0;
  RawCell<DPL> rc[kPFR], r1[kPFR], r2[kPFR], r3[kPFR], r4[kPFR];
#pragma unroll
  for (int k = 0; k < kPFR; ++k)
    if (k < W1) {
      rc[k].load(c + (size_t)k * D);
      r1[k].load(l1 + (size_t)k * D);
      r2[k].load(l2 + (size_t)k * D);
      r3[k].load(l3 + (size_t)k * D);
      r4[k].load(l4 + (size_t)k * D);
    }
  for (int x0 = 0; x0 < W1; x0 += kPFR) {
#pragma unroll
    for (int k = 0; k < kPFR; ++k) {
      const int x = x0 + k;
      if (x < W1) {
        int C[DPL], a1[DPL], a2[DPL], a3[DPL], a4[DPL];
        rc[k].get(C);
        r1[k].get(a1);
        r2[k].get(a2);
        r3[k].get(a3);
        r4[k].get(a4);
        const int xn = x + kPFR;
        if (xn < W1) {
          rc[k].load(c + (size_t)xn * D);
          r1[k].load(l1 + (size_t)xn * D);
          r2[k].load(l2 + (size_t)xn * D);
          r3[k].load(l3 + (size_t)xn * D);
          r4[k].load(l4 + (size_t)xn * D);
        }
        mp = path_step<DPL>(C, L, mp, g.P1, g.P2);
        int S[DPL];
        int key = 0x7FFFFFFF;
#pragma unroll
        for (int q = 0; q < DPL; ++q) {
          S[q] = sat16(sat16(L[q] + a1[q] + a2[q] + a3[q]) + a4[q]);
          key = min(key, S[q] * 64 + j * DPL + q);  // first minimum over d
        }
        key = row_min16(key);
        const int minS = key >> 6;  // arithmetic shift: floor division for negative S
        int d = key - minS * 64;
        const int xa = x + minX1;
        // S[d - 1], S[d + 1] of the lane owning the best d: the neighbours across
        // lanes by DPP row shifts (as in path_step), inside the lane directly
        const int sl = dpp_shr1(S[DPL - 1], kMaxCost), sr = dpp_shl1(S[0], kMaxCost);
        int sm = 0, sp = 0;
        bool owner = false;
#pragma unroll
        for (int q = 0; q < DPL; ++q)
          if (j * DPL + q == d) {
            owner = true;
            sm = q > 0 ? S[q - 1] : sl;
            sp = q < DPL - 1 ? S[q + 1] : sr;
          }
        if (minS < kMaxCost) {  // else bestDisp = -1 in the reference: stays invalid
          if (owner) {
            const int x2 = xa - d - g.minD;
            atomicMin(&cost2[x2], ((uint32_t)(minS + 32768) << 16) | (uint32_t)(65535 - xa));
            if (0 < d && d < D - 1) {
              const int den = max(sm + sp - 2 * minS, 1);
              d = d * 16 + ((sm - sp) * 16 + den) / (den * 2);
            } else {
              d *= 16;
            }
            if (live) out[xa] = (int16_t)(d + g.minD * 16);
          }
        }
      }
    }
  }
  __threadfence_block();
  __syncthreads();
  if (!live) return;
  // left-right consistency (disp12MaxDiff 1)
  for (int x = j; x < W; x += 16) {
    int v = out[x];
    if (x >= minX1 && v != INVALID) {
      const int _d = v >> 4, d_ = (v + 15) >> 4;
      const int _x = x - _d, x_ = x - d_;
      auto disp2 = [&](int xx) {
        const uint32_t k = cost2[xx];
        return k == 0xFFFFFFFFu ? INVALID : (65535 - (int)(k & 0xFFFFu)) - xx;
      };
      if (0 <= _x && _x < W && 0 <= x_ && x_ < W) {
        const int a = disp2(_x), b = disp2(x_);
        if (a >= g.minD && abs(a - _d) > 1 && b >= g.minD && abs(b - d_) > 1)
          out[x] = (int16_t)INVALID;
      }
    }
  }
}

// K5: 3x3 median (replicate border) -> int16 disparity, optional float / 16
__device__ __forceinline__ void sort2(int& a, int& b) {
  const int lo = min(a, b), hi = max(a, b);
  a = lo;
  b = hi;
}

__global__ __launch_bounds__(kBS) void k_sgbm_median(const int16_t* __restrict__ raw, int H, int W,
                                                     int16_t* __restrict__ disp,
                                                     float* __restrict__ dispf) {
  const int i = blockIdx.x * kBS + threadIdx.x, n = blockIdx.y;
  if (i >= H * W) return;
  const int y = i / W, x = i % W;
  const int16_t* s = raw + (size_t)n * H * W;
  int v[9], k = 0;
#pragma unroll
  for (int dy = -1; dy <= 1; ++dy)
#pragma unroll
    for (int dx = -1; dx <= 1; ++dx) {
      const int yy = min(max(y + dy, 0), H - 1), xx = min(max(x + dx, 0), W - 1);
      v[k++] = s[(size_t)yy * W + xx];
    }
  // median-of-9 network
  sort2(v[1], v[2]); sort2(v[4], v[5]); sort2(v[7], v[8]);
  sort2(v[0], v[1]); sort2(v[3], v[4]); sort2(v[6], v[7]);
  sort2(v[1], v[2]); sort2(v[4], v[5]); sort2(v[7], v[8]);
  sort2(v[0], v[3]); sort2(v[5], v[8]); sort2(v[4], v[7]);
  sort2(v[3], v[6]); sort2(v[1], v[4]); sort2(v[2], v[5]);
  sort2(v[4], v[7]); sort2(v[4], v[2]); sort2(v[6], v[4]);
  sort2(v[4], v[2]);
  const size_t o = (size_t)n * H * W + i;
  disp[o] = (int16_t)v[4];
  if (dispf) dispf[o] = (float)v[4] / 16.f;
}

int sgbm_geom(int H, int W, int stride, int minD, int numD, int block, int P1, int P2,
              SgbmGeom* g) {
  SLAM_REQUIRE(H > 0 && W > 0 && stride >= W && W <= 32768, "slam_sgbm: bad image shape");
  SLAM_REQUIRE(minD >= 0 && minD <= 64, "slam_sgbm: min_disparity in [0, 64]");
  SLAM_REQUIRE(numD == 32 || numD == 64, "slam_sgbm: num_disparities 32 or 64");
  SLAM_REQUIRE(block >= 1 && (block & 1) && block <= 21, "slam_sgbm: odd block size <= 21");
  g->H = H;
  g->W = W;
  g->stride = stride;
  g->minD = minD;
  g->D = numD;
  g->minX1 = minD + numD;
  g->W1 = W - g->minX1;
  g->SW2 = g->SH2 = block / 2;
  g->P1 = P1 > 0 ? P1 : 2;
  g->P2 = max(P2 > 0 ? P2 : 5, g->P1 + 1);
  g->vol = g->W1 > 0 ? (long long)H * g->W1 * numD : 0;
  return SLAM_OK;
}

// workspace: hs/S1 (aliased), C, L1, L2, L3 volumes + raw disparity
size_t sgbm_ws(const SgbmGeom& g, int batch) {
  const size_t vol = ((size_t)g.vol * 2 + 255) & ~(size_t)255;
  const size_t rawb = ((size_t)g.H * g.W * 2 + 255) & ~(size_t)255;
  return (size_t)batch * (5 * vol + rawb);
}

template <int D>
int sgbm_launch(const uint8_t* l, const uint8_t* r, int batch, const SgbmGeom& g, uint8_t* ws,
                int16_t* disp, float* dispf, hipStream_t s) {
  const size_t vol = ((size_t)g.vol * 2 + 255) & ~(size_t)255;
  // per-kind arrays, each holds all images: offset n * g.vol elements inside
  auto arr = [&](int k) { return reinterpret_cast<int16_t*>(ws + (size_t)k * batch * vol); };
  int16_t *hs = arr(0), *C = arr(1), *L1 = arr(2), *L2 = arr(3), *L3 = arr(4);
  int16_t* raw = reinterpret_cast<int16_t*>(ws + (size_t)5 * batch * vol);
  SgbmGeom gg = g;
  gg.vol = (long long)(vol / 2);  // image stride inside an array (elements)
  if (g.W1 > 0) {
    k_sgbm_hsum<D><<<dim3((g.W1 + kHsBand - 1) / kHsBand, (g.H + kHsRows - 1) / kHsRows, batch),
                     kBS, 0, s>>>(l, r, gg, hs);
    SLAM_LAUNCHED("k_sgbm_hsum");
    k_sgbm_vert<D><<<dim3((g.W1 + 15) / 16, batch), kBS, 0, s>>>(hs, gg, C, L2);
    SLAM_LAUNCHED("k_sgbm_vert");
    const int np = g.W1 + g.H - 1;
    // L4 (right to left) reuses the horizontal-sum volume, dead after k_sgbm_vert
    k_sgbm_paths<D><<<dim3((np + 15) / 16, batch, 3), kBS, 0, s>>>(C, gg, L1, L3, hs);
    SLAM_LAUNCHED("k_sgbm_paths");

    const size_t lds = (size_t)4 * g.W * 4;
    k_sgbm_row<D><<<dim3((g.H + 3) / 4, batch), 64, lds, s>>>(C, L1, L2, L3, hs, gg, raw);
    SLAM_LAUNCHED("k_sgbm_row");
  }
  k_sgbm_median<<<dim3((g.H * g.W + kBS - 1) / kBS, batch), kBS, 0, s>>>(raw, g.H, g.W, disp,
                                                                        dispf);
  SLAM_LAUNCHED("k_sgbm_median");
  return SLAM_OK;
}

__global__ __launch_bounds__(kBS) void k_fill16(int16_t* p, size_t n, int16_t v) {
  const size_t i = (size_t)blockIdx.x * kBS + threadIdx.x;
  if (i < n) p[i] = v;
}

// ------------------------------------------------------------ VO glue
// cv2.triangulatePoints on float32 points: f64 DLT null vector, homogeneous
// result rounded to float32, divided in float32 (calc_3d).
__device__ __forceinline__ void triangulate_f32(float lx, float ly, float rx, float ry,
                                                const double* __restrict__ Pl,
                                                const double* __restrict__ Pr, float X[3]) {
  double A[4][4];
#pragma unroll
  for (int cc = 0; cc < 4; ++cc) {
    A[0][cc] = (double)lx * Pl[8 + cc] - Pl[cc];
    A[1][cc] = (double)ly * Pl[8 + cc] - Pl[4 + cc];
    A[2][cc] = (double)rx * Pr[8 + cc] - Pr[cc];
    A[3][cc] = (double)ry * Pr[8 + cc] - Pr[4 + cc];
  }
  double h[4];
  null_vector4(A, h);
  const float w = (float)h[3];
#pragma unroll
  for (int k = 0; k < 3; ++k) X[k] = (float)h[k] / w;
}

// Order-preserving compaction helper: block of 1024, returns this item's slot
// (or -1) and advances `base`.
__device__ int block_compact(bool keep, int* wsum, int& base) {
  const int t = threadIdx.x, lane = t & 63, wid = t >> 6;
  const unsigned long long bal = __ballot(keep);
  const int pre = __popcll(bal & ((1ull << lane) - 1ull));
  if (lane == 0) wsum[wid] = __popcll(bal);
  __syncthreads();
  int off = 0, tot = 0;
  for (int i = 0; i < 16; ++i) {
    const int v = wsum[i];
    off += i < wid ? v : 0;
    tot += v;
  }
  __syncthreads();
  const int slot = keep ? base + off + pre : -1;
  base += tot;
  return slot;
}

// track_keypoints filters (visual_odometry.py:102-112; keypoint.py:20-32 with lower bounds)
__global__ __launch_bounds__(1024) void k_lk_filter(const float* __restrict__ p1, int p1_stride,
                                                    const float* __restrict__ p2,
                                                    const uint8_t* __restrict__ status,
                                                    const float* __restrict__ err,
                                                    const int32_t* __restrict__ npts, int cap,
                                                    int H, int W, float max_error, int lower,
                                                    float* __restrict__ tp1,
                                                    float* __restrict__ tp2,
                                                    int32_t* __restrict__ idx,
                                                    int32_t* __restrict__ count) {
  __shared__ int wsum[16];
  const int b = blockIdx.x;
  const int n = min(max(npts[b], 0), cap);
  int base = 0;
  for (int c = 0; c < n; c += 1024) {
    const int i = c + threadIdx.x;
    bool keep = false;
    float x2 = 0.f, y2 = 0.f;
    const size_t o = (size_t)b * cap + i;
    if (i < n) {
      x2 = rintf(p2[2 * o]);  // np.around: half to even
      y2 = rintf(p2[2 * o + 1]);
      keep = status[o] && err[o] < max_error && y2 < (float)H && x2 < (float)W;
      if (lower) keep = keep && y2 > 0.f && x2 > 0.f;
    }
    const int s = block_compact(keep, wsum, base);
    if (s >= 0) {
      const size_t q = (size_t)b * cap + s;
      tp1[2 * q] = p1[o * p1_stride];
      tp1[2 * q + 1] = p1[o * p1_stride + 1];
      tp2[2 * q] = x2;
      tp2[2 * q + 1] = y2;
      if (idx) idx[q] = i;
    }
  }
  if (threadIdx.x == 0) count[b] = base;
}

// calculate_right_qs + calc_3d (visual_odometry.py:114-134)
__global__ __launch_bounds__(1024) void k_vo_right_qs_3d(
    const float* __restrict__ tp1, const float* __restrict__ tp2, const int32_t* __restrict__ cnt,
    int cap, const float* __restrict__ disp, long long disp1_stride, long long disp2_off, int H,
    int W, float min_disp, float max_disp, const double* __restrict__ Pl,
    const double* __restrict__ Pr, float* __restrict__ q1l, float* __restrict__ q1r,
    float* __restrict__ q2l, float* __restrict__ q2r, float* __restrict__ Q1,
    float* __restrict__ Q2, double* __restrict__ q1l64, double* __restrict__ q2l64,
    double* __restrict__ Q1_64, double* __restrict__ Q2_64, int32_t* __restrict__ count) {
  __shared__ int wsum[16];
  const int b = blockIdx.x;
  const int n = min(max(cnt[b], 0), cap);
  const float* d1 = disp + b * disp1_stride;
  const float* d2 = d1 + disp2_off;
  int base = 0;
  for (int c = 0; c < n; c += 1024) {
    const int i = c + threadIdx.x;
    bool keep = false;
    float ax = 0.f, ay = 0.f, bx = 0.f, by = 0.f, e1 = 0.f, e2 = 0.f;
    if (i < n) {
      const size_t o = (size_t)b * cap + i;
      ax = tp1[2 * o];
      ay = tp1[2 * o + 1];
      bx = tp2[2 * o];
      by = tp2[2 * o + 1];
      // q.astype(int): truncation toward zero; disp.T[x, y] with NumPy's negative wrap
      // (an index NumPy would reject -- below -W or not finite -- raises IndexError in
      // the reference; here the point is dropped instead of reading out of bounds)
      bool inb = true;
      auto look = [&](const float* dm, float qx, float qy) {
        if (!(fabsf(qx) < 1e9f) || !(fabsf(qy) < 1e9f)) {
          inb = false;
          return 0.f;
        }
        int x = (int)qx, y = (int)qy;
        if (x < 0) x += W;
        if (y < 0) y += H;
        if (x < 0 || x >= W || y < 0 || y >= H) {
          inb = false;
          return 0.f;
        }
        return dm[(size_t)y * W + x];
      };
      e1 = look(d1, ax, ay);
      e2 = look(d2, bx, by);
      keep = inb && min_disp < e1 && e1 < max_disp && min_disp < e2 && e2 < max_disp;
    }
    const int s = block_compact(keep, wsum, base);
    if (s >= 0) {
      const size_t q = (size_t)b * cap + s;
      const float ar = ax - e1, br = bx - e2;
      q1l[2 * q] = ax;
      q1l[2 * q + 1] = ay;
      q1r[2 * q] = ar;
      q1r[2 * q + 1] = ay;
      q2l[2 * q] = bx;
      q2l[2 * q + 1] = by;
      q2r[2 * q] = br;
      q2r[2 * q + 1] = by;
      if (q1l64) {
        q1l64[2 * q] = ax;
        q1l64[2 * q + 1] = ay;
        q2l64[2 * q] = bx;
        q2l64[2 * q + 1] = by;
      }
    }
  }
  if (threadIdx.x == 0) count[b] = base;
}

__global__ __launch_bounds__(kBS) void k_triangulate_f32(const float* __restrict__ pl,
                                                         const float* __restrict__ pr,
                                                         const int32_t* __restrict__ count,
                                                         int cap, const double* __restrict__ Pl,
                                                         const double* __restrict__ Pr,
                                                         float* __restrict__ X,
                                                         double* __restrict__ X64) {
  const int b = blockIdx.y;
  const int n = min(max(count[b], 0), cap);
  const int k = blockIdx.x * kBS + threadIdx.x;
  if (k >= n) return;
  const size_t o = (size_t)b * cap + k;
  float x[3];
  triangulate_f32(pl[2 * o], pl[2 * o + 1], pr[2 * o], pr[2 * o + 1], Pl, Pr, x);
  X[3 * o] = x[0];
  X[3 * o + 1] = x[1];
  X[3 * o + 2] = x[2];
  if (X64) {
    X64[3 * o] = (double)x[0];
    X64[3 * o + 1] = (double)x[1];
    X64[3 * o + 2] = (double)x[2];
  }
}

FastGeom fast_geom(int H, int W, int stride, int th, int tw, int thr, int per_tile) {
  FastGeom g;
  g.H = H;
  g.W = W;
  g.stride = stride;
  g.th = th;
  g.tw = tw;
  g.ntx = (W + tw - 1) / tw;
  g.n_tiles = ((H + th - 1) / th) * g.ntx;
  g.thr = min(max(thr, 0), 255);
  g.per_tile = per_tile;
  g.map_bytes = (th * tw + 15) & ~15;
  g.list_cap = max(0, th - 6) * max(0, tw - 6);
  g.list_cap = max(g.list_cap, 1);
  g.wave_lds = g.map_bytes + 4 * g.list_cap;
  g.wave_lds = (g.wave_lds + 15) & ~15;
  return g;
}

}  // namespace

// ---------------------------------------------------------------- C ABI
extern "C" int slam_fast_tiles_workspace_bytes(int batch, int H, int W, int tile_h, int tile_w,
                                               int per_tile, size_t* bytes) {
  SLAM_REQUIRE(batch >= 0 && H > 0 && W > 0 && tile_h > 0 && tile_w > 0 && per_tile > 0 && bytes,
               "slam_fast_tiles_workspace_bytes: bad args");
  const FastGeom g = fast_geom(H, W, W, tile_h, tile_w, 10, per_tile);
  *bytes = (size_t)batch * g.n_tiles * ((size_t)per_tile * 3 * sizeof(float) + sizeof(int32_t)) + 256;
  return SLAM_OK;
}

extern "C" int slam_fast_tiles(const uint8_t* d_img, int batch, int H, int W, int stride,
                               int tile_h, int tile_w, int threshold, int per_tile, void* d_ws,
                               size_t ws_bytes, float* d_kp, int32_t* d_count, int kp_cap,
                               void* stream) {
  SLAM_REQUIRE(batch >= 0 && H > 0 && W > 0 && stride >= W && kp_cap >= 0,
               "slam_fast_tiles: bad shape");
  SLAM_REQUIRE(tile_h > 0 && tile_w > 0 && tile_w < 4096 && tile_h < 4096 && per_tile > 0,
               "slam_fast_tiles: bad tile");
  const FastGeom g = fast_geom(H, W, stride, tile_h, tile_w, threshold, per_tile);
  SLAM_REQUIRE(4 * g.wave_lds <= 160 * 1024, "slam_fast_tiles: tile %dx%d too large", tile_h,
               tile_w);
  if (batch == 0) return SLAM_OK;
  SLAM_REQUIRE(d_img && d_ws && d_kp && d_count, "slam_fast_tiles: null pointer");
  size_t need = 0;
  if (int rc = slam_fast_tiles_workspace_bytes(batch, H, W, tile_h, tile_w, per_tile, &need))
    return rc;
  if (ws_bytes < need) {
    slam::set_error("slam_fast_tiles: workspace %zu < %zu bytes", ws_bytes, need);
    return SLAM_ERR_WORKSPACE;
  }
  hipStream_t s = slam::as_stream(stream);
  float* ws_kp = static_cast<float*>(d_ws);
  int32_t* ws_cnt = reinterpret_cast<int32_t*>(ws_kp + (size_t)batch * g.n_tiles * per_tile * 3);
  k_fast_tiles<<<dim3((g.n_tiles + 3) / 4, batch), kBS, 4 * g.wave_lds, s>>>(d_img, g, ws_kp,
                                                                             ws_cnt);
  SLAM_LAUNCHED("k_fast_tiles");
  k_fast_compact<<<batch, 1024, 0, s>>>(ws_kp, ws_cnt, g.n_tiles, per_tile, d_kp, d_count,
                                        kp_cap);
  SLAM_LAUNCHED("k_fast_compact");
  return SLAM_OK;
}

extern "C" int slam_lk_pyramid_layout(int H, int W, int win, int max_level, int* nlev,
                                      size_t* img_bytes) {
  LkGeom g;
  if (int rc = lk_geom(H, W, win, max_level, &g)) return rc;
  SLAM_REQUIRE(nlev && img_bytes, "slam_lk_pyramid_layout: null pointer");
  *nlev = g.nlev;
  *img_bytes = (size_t)g.img_bytes;
  return SLAM_OK;
}

extern "C" int slam_lk_build_pyramids(const uint8_t* d_img, int n_img, int H, int W, int stride,
                                      int win, int max_level, uint8_t* d_pyr, int16_t* d_deriv,
                                      void* stream) {
  LkGeom g;
  if (int rc = lk_geom(H, W, win, max_level, &g)) return rc;
  SLAM_REQUIRE(n_img >= 0 && stride >= W, "slam_lk_build_pyramids: bad shape");
  if (n_img == 0) return SLAM_OK;
  SLAM_REQUIRE(d_img && d_pyr, "slam_lk_build_pyramids: null pointer");
  hipStream_t s = slam::as_stream(stream);
  for (int l = 0; l < g.nlev; ++l) {
    const int np = (g.w[l] + 2 * g.B) * (g.h[l] + 2 * g.B);
    dim3 grid((np + kBS - 1) / kBS, n_img);
    if (l == 0)
      k_lk_level0<<<grid, kBS, 0, s>>>(d_img, stride, g, d_pyr);
    else
      k_lk_pyrdown<<<grid, kBS, 0, s>>>(g, l, d_pyr);
    SLAM_LAUNCHED("k_lk_pyr");
    if (d_deriv) {
      k_lk_scharr<<<grid, kBS, 0, s>>>(g, l, d_pyr, reinterpret_cast<short2*>(d_deriv));
      SLAM_LAUNCHED("k_lk_scharr");
    }
  }
  return SLAM_OK;
}

extern "C" int slam_lk_track(const uint8_t* d_prev_pyr, const int16_t* d_prev_deriv,
                             const uint8_t* d_next_pyr, long long pair_stride_imgs, int batch,
                             int H, int W, int win, int max_level, int max_count, double eps,
                             float min_eig, const float* d_pts, int pts_stride,
                             const int32_t* d_npts, int cap, float* d_out, uint8_t* d_status,
                             float* d_err, void* stream) {
  LkGeom g;
  if (int rc = lk_geom(H, W, win, max_level, &g)) return rc;
  SLAM_REQUIRE(batch >= 0 && cap >= 0 && (pts_stride == 2 || pts_stride == 3),
               "slam_lk_track: bad shape");
  if (batch == 0 || cap == 0) return SLAM_OK;
  SLAM_REQUIRE(d_prev_pyr && d_prev_deriv && d_next_pyr && d_pts && d_npts && d_out && d_status &&
                   d_err,
               "slam_lk_track: null pointer");
  LkArgs a;
  a.prev = d_prev_pyr;
  a.der = reinterpret_cast<const short2*>(d_prev_deriv);
  a.next = d_next_pyr;
  a.pyr_stride = pair_stride_imgs * g.img_bytes;
  a.der_stride = pair_stride_imgs * g.img_bytes;
  a.max_count = min(max(max_count, 0), 100);
  eps = fmin(fmax(eps, 0.0), 10.0);
  a.eps2 = eps * eps;
  a.min_eig = min_eig;
  a.win = win;
  a.pts = d_pts;
  a.pts_stride = pts_stride;
  a.npts = d_npts;
  a.cap = cap;
  a.out = d_out;
  a.status = d_status;
  a.err = d_err;
  k_lk_track<<<dim3((cap + 3) / 4, batch), kBS, 0, slam::as_stream(stream)>>>(g, a);
  SLAM_LAUNCHED("k_lk_track");
  return SLAM_OK;
}

extern "C" int slam_sgbm_workspace_bytes(int batch, int H, int W, int min_disp, int num_disp,
                                         int block, size_t* bytes) {
  SgbmGeom g;
  if (int rc = sgbm_geom(H, W, W, min_disp, num_disp, block, 0, 0, &g)) return rc;
  SLAM_REQUIRE(batch >= 0 && bytes, "slam_sgbm_workspace_bytes: bad args");
  *bytes = sgbm_ws(g, batch);
  return SLAM_OK;
}

extern "C" int slam_sgbm(const uint8_t* d_left, const uint8_t* d_right, int batch, int H, int W,
                         int stride, int min_disp, int num_disp, int block, int P1, int P2,
                         void* d_ws, size_t ws_bytes, int16_t* d_disp, float* d_disp_f32,
                         void* stream) {
  SgbmGeom g;
  if (int rc = sgbm_geom(H, W, stride, min_disp, num_disp, block, P1, P2, &g)) return rc;
  SLAM_REQUIRE(batch >= 0, "slam_sgbm: bad batch");
  if (batch == 0) return SLAM_OK;
  SLAM_REQUIRE(d_left && d_right && d_ws && d_disp, "slam_sgbm: null pointer");
  const size_t need = sgbm_ws(g, batch);
  if (ws_bytes < need) {
    slam::set_error("slam_sgbm: workspace %zu < %zu bytes", ws_bytes, need);
    return SLAM_ERR_WORKSPACE;
  }
  hipStream_t s = slam::as_stream(stream);
  uint8_t* ws = static_cast<uint8_t*>(d_ws);
  if (g.W1 <= 0) {
    const size_t vol = ((size_t)g.vol * 2 + 255) & ~(size_t)255;
    int16_t* raw = reinterpret_cast<int16_t*>(ws + (size_t)5 * batch * vol);
    const size_t np = (size_t)batch * H * W;
    k_fill16<<<(unsigned)((np + kBS - 1) / kBS), kBS, 0, s>>>(raw, np,
                                                              (int16_t)((min_disp - 1) * 16));
    SLAM_LAUNCHED("k_fill16");
    k_sgbm_median<<<dim3((H * W + kBS - 1) / kBS, batch), kBS, 0, s>>>(raw, H, W, d_disp,
                                                                      d_disp_f32);
    SLAM_LAUNCHED("k_sgbm_median");
    return SLAM_OK;
  }
  return num_disp == 32 ? sgbm_launch<32>(d_left, d_right, batch, g, ws, d_disp, d_disp_f32, s)
                        : sgbm_launch<64>(d_left, d_right, batch, g, ws, d_disp, d_disp_f32, s);
}

extern "C" int slam_lk_filter(const float* d_p1, int p1_stride, const float* d_p2,
                              const uint8_t* d_status, const float* d_err, const int32_t* d_npts,
                              int cap, int batch, int H, int W, float max_error, int lower_bounds,
                              float* d_tp1, float* d_tp2, int32_t* d_idx, int32_t* d_count,
                              void* stream) {
  SLAM_REQUIRE(batch >= 0 && cap >= 0 && (p1_stride == 2 || p1_stride == 3),
               "slam_lk_filter: bad shape");
  if (batch == 0) return SLAM_OK;
  SLAM_REQUIRE(d_p1 && d_p2 && d_status && d_err && d_npts && d_tp1 && d_tp2 && d_count,
               "slam_lk_filter: null pointer");
  k_lk_filter<<<batch, 1024, 0, slam::as_stream(stream)>>>(d_p1, p1_stride, d_p2, d_status, d_err,
                                                           d_npts, cap, H, W, max_error,
                                                           lower_bounds, d_tp1, d_tp2, d_idx,
                                                           d_count);
  SLAM_LAUNCHED("k_lk_filter");
  return SLAM_OK;
}

extern "C" int slam_vo_right_qs_3d(const float* d_tp1, const float* d_tp2, const int32_t* d_cnt,
                                   int cap, int batch, const float* d_disp,
                                   long long disp1_stride, long long disp2_offset, int H, int W,
                                   float min_disp, float max_disp, const double* d_Pl,
                                   const double* d_Pr, float* d_q1l, float* d_q1r, float* d_q2l,
                                   float* d_q2r, float* d_Q1, float* d_Q2, double* d_q1l64,
                                   double* d_q2l64, double* d_Q1_64, double* d_Q2_64,
                                   int32_t* d_count, void* stream) {
  SLAM_REQUIRE(batch >= 0 && cap >= 0 && H > 0 && W > 0, "slam_vo_right_qs_3d: bad shape");
  if (batch == 0) return SLAM_OK;
  SLAM_REQUIRE(d_tp1 && d_tp2 && d_cnt && d_disp && d_Pl && d_Pr && d_q1l && d_q1r && d_q2l &&
                   d_q2r && d_Q1 && d_Q2 && d_count,
               "slam_vo_right_qs_3d: null pointer");
  SLAM_REQUIRE(!!d_q1l64 == !!d_q2l64 && !!d_Q1_64 == !!d_Q2_64,
               "slam_vo_right_qs_3d: f64 outputs come in pairs");
  hipStream_t s = slam::as_stream(stream);
  k_vo_right_qs_3d<<<batch, 1024, 0, s>>>(
      d_tp1, d_tp2, d_cnt, cap, d_disp, disp1_stride, disp2_offset, H, W, min_disp, max_disp, d_Pl,
      d_Pr, d_q1l, d_q1r, d_q2l, d_q2r, d_Q1, d_Q2, d_q1l64, d_q2l64, d_Q1_64, d_Q2_64, d_count);
  SLAM_LAUNCHED("k_vo_right_qs_3d");
  if (cap == 0) return SLAM_OK;  // counts written as 0; nothing to triangulate
  // calc_3d over the kept points: one thread per point (count read on the device)
  const dim3 grid((cap + kBS - 1) / kBS, batch);
  k_triangulate_f32<<<grid, kBS, 0, s>>>(d_q1l, d_q1r, d_count, cap, d_Pl, d_Pr, d_Q1, d_Q1_64);
  SLAM_LAUNCHED("k_triangulate_f32");
  k_triangulate_f32<<<grid, kBS, 0, s>>>(d_q2l, d_q2r, d_count, cap, d_Pl, d_Pr, d_Q2, d_Q2_64);
  SLAM_LAUNCHED("k_triangulate_f32");
  return SLAM_OK;
}

extern "C" int slam_triangulate_f32(const float* d_ptl, const float* d_ptr, const int32_t* d_count,
                                    int cap, int batch, const double* d_Pl, const double* d_Pr,
                                    float* d_X, void* stream) {
  SLAM_REQUIRE(batch >= 0 && cap >= 0, "slam_triangulate_f32: bad shape");
  if (batch == 0 || cap == 0) return SLAM_OK;
  SLAM_REQUIRE(d_ptl && d_ptr && d_count && d_Pl && d_Pr && d_X,
               "slam_triangulate_f32: null pointer");
  k_triangulate_f32<<<dim3((cap + kBS - 1) / kBS, batch), kBS, 0, slam::as_stream(stream)>>>(
      d_ptl, d_ptr, d_count, cap, d_Pl, d_Pr, d_X, nullptr);
  SLAM_LAUNCHED("k_triangulate_f32");
  return SLAM_OK;
}
