// Tiled ORB (FAST-9 + Harris + IC angle + rBRIEF) for gfx950.
//
// Replaces /root/reference/orb.py:4-38: orb_detector_using_tiles cuts the image
// into overlapping patches and runs cv2.ORB_create(n, scaleFactor=1.2)
// .detect()/.compute() on each.  The semantics restated in oracle/orb.c (OpenCV
// 4.x ORB, canonical keypoint order) are reproduced bit for bit.
//
// Design: one workgroup per (image, patch).  The patch never leaves LDS: the
// pyramid is built level by level in two ping-pong LDS buffers with the
// 8-bit fixed-point INTER_LINEAR_EXACT resize, and each level runs the whole
// chain before the next is built:
//   FAST-9 score map (bit-mask arc test, cornerScore<16>) over the NMS region
//   -> strict 3x3 NMS + border filter -> LDS atomic candidate list + score
//   histogram -> retainBest(2n) threshold from a wave suffix scan -> Harris on
//   the survivors -> exact rank (response desc, y, x) -> retainBest(n) with
//   ties -> IC angle (one wave per keypoint, integer moments) -> 7x7 Gaussian
//   of the sampled region (sliding-window separable float FMA chains) ->
//   rBRIEF (32 lanes per keypoint, one descriptor byte per lane).
// HBM traffic per patch = its bytes read once + ~56 B per keypoint written.
#include "common.hpp"

#include <cmath>
#include <cstdlib>
#include <cstring>

namespace {

#include "orb_pattern.inc"

constexpr int kNLev = 8;
constexpr int kEdge = 31;
constexpr int kFastT = 20;
constexpr int kOrbWG = 512;
constexpr int kMaxTiles = 256;
constexpr int kMaxShapes = 4;
constexpr int kMaxBat = 4;  // small pyramid levels batched into one group
constexpr int kNMS0 = 29;  // score-map region starts here (needs [30, w-31])
constexpr int kBl0 = 12;   // blurred region starts here (rotated samples within +-18 of [31, w-32])
constexpr int kFqW = 320;  // queue entries per wave: < 64 carried + 256 appended per pass
constexpr int kFq = (kOrbWG / 64) * kFqW * 4;  // FAST / NMS work queues, bytes

__constant__ __attribute__((aligned(16))) int8_t c_pattern[256 * 4];

struct OrbGeom {
  int H, W, stride;
  int n_tiles, ntx, tile_h, tile_w;
  int tcap;       // keypoint slots per tile in the workspace
  int cand_cap;   // NMS candidates per level (global scratch, worst case 1/4 density)
  int list_cap;   // kept keypoints / retainBest(2n) survivors per level (LDS)
  int lds_a, lds_u, lds_l, lds_s, lds_m;  // byte offsets of the LDS regions
  int lds_fq, lds_tab;  // FAST queues and resize tables (inside U unless glob)
  int glob;       // level images in global memory (whole images too large for LDS)
  int lvl_bytes;  // global level buffer per image and ping-pong half (glob only)
  int tab_x;      // resize-coefficient slots for x (>= W); y follows
  int lds_total;
  float ls[kNLev];  // (float)pow(1.2, l)
  int nl[kNLev];    // per-level budget
  float gk[7];      // Gaussian 7-tap, sigma 2 (float)
  int nshapes;
  int sw[kMaxShapes], sh[kMaxShapes];
  int lw[kMaxShapes][kNLev], lh[kMaxShapes][kNLev];
  int nlev[kMaxShapes];  // levels to run for this shape (0..nlev-1)
  // Small levels bat0 .. nlev-1 run as ONE group (LDS variant, tiled mode):
  // their images resident together in A, every phase one pass over all of
  // them (see "batched small levels" in k_orb_tile).  bat0 == nlev: none.
  int bat0[kMaxShapes];
  int bslot[kMaxShapes][kMaxBat];     // A byte offset of group level j's image
  int bhist[kMaxShapes];              // A byte offset of hist4 [kMaxBat][256], ctr4 [kMaxBat][16]
  int bsmap[kMaxShapes][kMaxBat];     // U byte offset of level j's FAST score map
  int bbl[kMaxShapes][kMaxBat];       // U byte offset of level j's blurred image
  int bcand[kMaxShapes][kMaxBat + 1]; // level j's NMS candidates in the tile's scratch (entries)
  int bnseg[kMaxShapes][kMaxBat];     // blur row segments per column group of level j
  uint8_t tile_shape[kMaxTiles];
};

__device__ __forceinline__ int rne_f(float v) { return (int)rintf(v); }
__host__ __device__ __forceinline__ int lpitch(int w) { return (w + 3) & ~3; }

// Exact n / d for n >= 0, d >= 1 with n * d < 2^32, by a multiply-high with
// m = ceil(2^32 / d): the error n (m - 2^32/d) / 2^32 < n / 2^32 < 1/d never
// crosses an integer.  (Here n < W * H and d <= W; build_geom checks W * H * W < 2^32.)
// d == 1 gives m == 0 (2^32 does not fit): fdiv then returns n.
__device__ __forceinline__ uint32_t div_magic(uint32_t d) { return 0xFFFFFFFFu / d + 1u; }
__device__ __forceinline__ int fdiv(int n, uint32_t m) {
  return m ? (int)__umulhi((uint32_t)n, m) : n;
}

// ------------------------------------------------------------------ FAST
// Exact quick reject: any 9 consecutive circle positions contain two
// adjacent compass points (0,4,8,12), so a corner needs such a pair to be
// darker (or brighter) than v -/+ t.  Two pixels at once: the low bytes of the
// 16-bit halves of v (centre) and of the compass pixels dn (0), rt (4), up (8),
// lf (12); a half of the result is non-zero iff that pixel passes.  Every
// adjacent compass pair is one of {dn, up} with one of {rt, lf}, so "a darker
// adjacent pair" is (dn or up) and (rt or lf) darker, "p darker" being
// sat(v - t - p) != 0 and "p brighter" sat(p - (v + t)) != 0 (v_pk_sub_u16 clamp).
__device__ __forceinline__ uint32_t quick4(uint32_t v, uint32_t dn, uint32_t rt, uint32_t up,
                                           uint32_t lf) {
  typedef unsigned short u2 __attribute__((ext_vector_type(2)));
  auto h = [](uint32_t x) { return __builtin_bit_cast(u2, x & 0x00FF00FFu); };
  const u2 vv = h(v), t2 = u2{(unsigned short)kFastT, (unsigned short)kFastT};
  const u2 vlo = __builtin_elementwise_sub_sat(vv, t2), vhi = vv + t2;  // v - t (sat), v + t
  const u2 pdn = h(dn), prt = h(rt), pup = h(up), plf = h(lf);
  auto dk = [&](u2 p) { return __builtin_elementwise_sub_sat(vlo, p); };  // != 0: p < v - t
  auto br = [&](u2 p) { return __builtin_elementwise_sub_sat(p, vhi); };  // != 0: p > v + t
  const u2 d = __builtin_elementwise_min(__builtin_elementwise_max(dk(pdn), dk(pup)),
                                         __builtin_elementwise_max(dk(prt), dk(plf)));
  const u2 b = __builtin_elementwise_min(__builtin_elementwise_max(br(pdn), br(pup)),
                                         __builtin_elementwise_max(br(prt), br(plf)));
  return __builtin_bit_cast(uint32_t, __builtin_elementwise_max(d, b));
}

// -DSLAM_ORB_KO=mask (timing knock-outs, wrong keypoints; never a product
// build): 1 -- the full FAST test reads only its centre byte; 2 -- the
// resize reads one source byte per destination pixel instead of four; 4 --
// the full FAST test reads its 16 circle bytes but scores them trivially
#ifndef SLAM_ORB_KO
#define SLAM_ORB_KO 0
#endif
// Full segment test + OpenCV cornerScore<16> at c (past the quick reject).
__device__ __forceinline__ int fast_full(const uint8_t* c, int st) {
  const int v = c[0];
  if (SLAM_ORB_KO & 1) return v > 128 ? v - 100 : 0;
  if (SLAM_ORB_KO & 4) {  // the 16 reads kept, the arc minima dropped
    const int sum = c[3 * st] + c[3 * st + 1] + c[2 * st + 2] + c[st + 3] + c[3] + c[-st + 3] + c[-2 * st + 2] +
                    c[-3 * st + 1] + c[-3 * st] + c[-3 * st - 1] + c[-2 * st - 2] + c[-st - 3] + c[-3] +
                    c[st - 3] + c[2 * st - 2] + c[3 * st - 1];
    return (sum >> 4) > v + 20 ? 30 : 0;
  }
  int cc[16];  // the circle pixels, d[k] = v - cc[k]
  cc[0] = c[3 * st];
  cc[1] = c[3 * st + 1];
  cc[2] = c[2 * st + 2];
  cc[3] = c[st + 3];
  cc[4] = c[3];
  cc[5] = c[-st + 3];
  cc[6] = c[-2 * st + 2];
  cc[7] = c[-3 * st + 1];
  cc[8] = c[-3 * st];
  cc[9] = c[-3 * st - 1];
  cc[10] = c[-2 * st - 2];
  cc[11] = c[-st - 3];
  cc[12] = c[-3];
  cc[13] = c[st - 3];
  cc[14] = c[2 * st - 2];
  cc[15] = c[3 * st - 1];
  // OpenCV cornerScore<16> (d = v - cc) is max(t, A_dark, A_bright) - 1 with A_dark = the
  // largest min(d) over the 16 circular 9-arcs and A_bright the same for -d; a
  // segment test pass (9 consecutive d > t, or -d > t) is exactly A > t, so
  //   score = A > t ? A - 1 : 0,  A = max(A_dark, A_bright).
  // Both sides at once on packed int16 pairs (d, -d) (v_pk_min/max_i16), the
  // 9-arcs (k .. k+8) and (k+1 .. k+9), k even, sharing the min over k+1 .. k+8
  // built from pairwise minima (m2 -> m4 -> m8).
  typedef short s2 __attribute__((ext_vector_type(2)));
  s2 p[16];
  // (v - c, c - v) as ONE packed subtract of X = (v, c) and its swapped
  // halves (op_sel), X built by one v_lshl_or: 2 ops per circle pixel, not 3
#pragma unroll
  for (int k = 0; k < 16; ++k) {
    const uint32_t X = (uint32_t)v | ((uint32_t)cc[k] << 16);
    uint32_t r;  // lo = X.lo - X.hi, hi = X.hi - X.lo (the compiler would materialise X.yx)
    __asm__("v_pk_sub_i16 %0, %1, %1 op_sel:[0,1] op_sel_hi:[1,0]" : "=v"(r) : "v"(X));
    p[k] = __builtin_bit_cast(s2, r);
  }
  s2 m2[8], m4[8];
#pragma unroll
  for (int k = 0; k < 8; ++k)  // min over 2k+1, 2k+2
    m2[k] = __builtin_elementwise_min(p[(2 * k + 1) & 15], p[(2 * k + 2) & 15]);
#pragma unroll
  for (int k = 0; k < 8; ++k) m4[k] = __builtin_elementwise_min(m2[k], m2[(k + 1) & 7]);  // 2k+1 .. 2k+4
  s2 acc = s2{(short)kFastT, (short)kFastT};
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    const s2 m8 = __builtin_elementwise_min(m4[k], m4[(k + 2) & 7]);  // 2k+1 .. 2k+8
    acc = __builtin_elementwise_max(acc, __builtin_elementwise_min(m8, p[2 * k]));
    acc = __builtin_elementwise_max(acc, __builtin_elementwise_min(m8, p[(2 * k + 9) & 15]));
  }
  const int A = max((int)acc.x, (int)acc.y);
  return A > kFastT ? A - 1 : 0;
}

// Harris response from the window sums a = sum Ix^2, b = sum Iy^2, c = sum Ix Iy
__device__ __forceinline__ float harris_resp(int a, int b, int c) {
  const float scale = 1.f / ((1 << 2) * 7 * 255.f);
  const float ssss = scale * scale * scale * scale;
  const float k = 0.04f;
  return ((float)a * b - (float)c * c - k * ((float)a + b) * ((float)a + b)) * ssss;
}

__device__ __forceinline__ float fast_atan2_deg(float y, float x) {
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

// INTER_LINEAR_EXACT coefficient of destination index d: (ofs << 9) | c1.
__device__ __forceinline__ int lin_coeff(int d, int dsize, int ssize) {
  const double inv = (double)dsize / ssize;
  const double scale = 1.0 / inv;
  const double fval = scale * ((double)d + 0.5) - 0.5;
  const int ival = (int)floor(fval);
  if (ival >= 0 && ssize > 1) {
    if (ival < ssize - 1) return (ival << 9) | (int)rint((fval - (double)ival) * 256.0);
    return (ssize - 1) << 9;  // replicate the last source sample
  }
  return 0;  // replicate the first
}

// -DSLAM_ORB_PROFILE: per-phase shader cycles (s_memtime, thread 0 of every
// workgroup) accumulated in g_orb_prof and read by slam_orb_profile_read().
// Slots 16 + 10 l + ph split the same cycles by pyramid level l.
#ifdef SLAM_ORB_PROFILE
__device__ unsigned long long g_orb_prof[96];
#define ORB_T0() unsigned long long orb_tp = __builtin_amdgcn_s_memtime()
#define ORB_T(ph)                                                          \
  do {                                                                     \
    if (threadIdx.x == 0) {                                                \
      const unsigned long long orb_tn = __builtin_amdgcn_s_memtime();      \
      atomicAdd(&g_orb_prof[ph], orb_tn - orb_tp);                         \
      atomicAdd(&g_orb_prof[16 + 10 * orb_lv + (ph)], orb_tn - orb_tp);    \
      orb_tp = orb_tn;                                                     \
    }                                                                      \
  } while (0)
#else
#define ORB_T0() (void)0
#define ORB_T(ph) (void)0
#endif
// -DSLAM_ORB_CUT=k (profiling builds only, scripts/build_variant.sh + scripts/gpu_profile.sh): every
// level stops after phase k (1 resize, 2 FAST, 3 NMS, 6 rank, 7 IC angle,
// 8 blur), so the SQ counters of successive cuts split the LDS instructions /
// bank conflicts by phase (profiles/r3_orb_lds_phases_v1.json, git history before 1bfa753).
#ifdef SLAM_ORB_CUT
#define ORB_CUT(ph) \
  if ((ph) == SLAM_ORB_CUT) continue
#else
#define ORB_CUT(ph) (void)0
#endif

// Item i of a concatenation of up to 4 ranges (sizes n0, n1, n2, ...): its
// range j, i becomes the index inside it.
__device__ __forceinline__ int seg4(int& i, int NB, int n0, int n1, int n2) {
  int j = 0;
  if (NB > 1 && i >= n0) {
    i -= n0;
    j = 1;
    if (NB > 2 && i >= n1) {
      i -= n1;
      j = 2;
      if (NB > 3 && i >= n2) {
        i -= n2;
        j = 3;
      }
    }
  }
  return j;
}
// element j of four values (scalars, not an array in memory: a selected
// array element can be turned into a dynamically indexed private array,
// i.e. scratch, and LDS pointers into flat ones)
template <typename T>
__device__ __forceinline__ T pick4v(int j, T a0, T a1, T a2, T a3) {
  return j == 0 ? a0 : (j == 1 ? a1 : (j == 2 ? a2 : a3));
}
#define pick4(j, a) pick4v((j), (a)[0], (a)[1], (a)[2], (a)[3])

struct KP {  // one kept keypoint of the current level (LDS)
  int x, y;
  float resp, angle;
};

template <bool kGlob>
#ifndef SLAM_ORB_WPE
#define SLAM_ORB_WPE 4  // waves per SIMD the register budget is cut for (4: 128 VGPRs)
#endif
__global__ __launch_bounds__(kOrbWG) __attribute__((amdgpu_waves_per_eu(SLAM_ORB_WPE))) void k_orb_tile(const uint8_t* __restrict__ img, OrbGeom g,
                                                     float* __restrict__ ws_kp,
                                                     int32_t* __restrict__ ws_oct,
                                                     uint8_t* __restrict__ ws_desc,
                                                     int32_t* __restrict__ ws_cnt,
                                                     uint32_t* __restrict__ ws_cand,
                                                     uint8_t* __restrict__ ws_lvl) {
  // All LDS is one dynamic region with a 16-byte aligned base (Guideline 17).
  extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
  int* hist = reinterpret_cast<int*>(lds + g.lds_m);  // 256 bins of FAST score
  int* ctr = hist + 256;   // 0: candidates, 1: survivors, 2: threshold, 3: kept
  int* tabx = reinterpret_cast<int*>(lds + g.lds_tab);  // resize coefficients (x, then y)
  int* taby = tabx + g.tab_x;

  const int tile = blockIdx.x, b = blockIdx.y;
  const int t = threadIdx.x;
  const int lane = t & 63, wid = t >> 6;
  const int ty = tile / g.ntx, tx = tile - ty * g.ntx;
  const int x0 = tx * g.tile_w, y0 = ty * g.tile_h;
  const int shp = g.tile_shape[tile];
  const int pw = g.sw[shp], ph = g.sh[shp];
  // LDS: A = current level image, U = scratch (resize target, FAST score map,
  // blurred level), L = kept keypoints, S = retainBest(2n) survivors.  Only
  // one level image is resident: level l is resized from A into U and copied
  // back, so an ORB workgroup leaves room on its CU for other kernels' groups.
  // kGlob: level images in global memory (a separate instantiation, so the
  // LDS variant keeps ds_* addressing)
  uint8_t* A = kGlob ? ws_lvl + (size_t)b * 2 * g.lvl_bytes : lds + g.lds_a;
  uint8_t* U = kGlob ? A + g.lvl_bytes : lds + g.lds_u;
  KP* L = reinterpret_cast<KP*>(lds + g.lds_l);
  uint32_t* svc = reinterpret_cast<uint32_t*>(lds + g.lds_s);
  float* svr = reinterpret_cast<float*>(svc + g.list_cap);
  const size_t slot = (size_t)b * g.n_tiles + tile;
  float* okp = ws_kp + slot * g.tcap * 5;
  int32_t* ooct = ws_oct + slot * g.tcap;
  uint8_t* odesc = ws_desc + slot * g.tcap * 32;
  // NMS candidates (and, past list_cap survivors, the survivors) of this tile
  uint32_t* gcand = ws_cand + slot * 3 * (size_t)g.cand_cap;
  uint32_t* gsvc = gcand + g.cand_cap;
  float* gsvr = reinterpret_cast<float*>(gsvc + g.cand_cap);

  ORB_T0();
#ifdef SLAM_ORB_PROFILE
  int orb_lv = 0;
#endif
  // Level images are stored with a row pitch of the width rounded up to 4 bytes
  // (lpitch), so 4 adjacent pixels of a row are one aligned dword for the
  // resize stores and the blur's row windows.
  // ---- stage the patch (level 0) into LDS, 16 B per lane where aligned
  {
    const uint8_t* src = img + (size_t)b * g.H * g.stride + (size_t)y0 * g.stride + x0;
    uint8_t* dst = A;
    const int P0 = lpitch(pw);
    if ((pw & 15) == 0 && (((uintptr_t)src) & 15) == 0 && (g.stride & 15) == 0) {
      const int vpr = pw >> 4;
      for (int i = t; i < vpr * ph; i += kOrbWG) {
        const int r = i / vpr, c = i - r * vpr;
        *reinterpret_cast<uint4*>(dst + r * P0 + 16 * c) =
            *reinterpret_cast<const uint4*>(src + (size_t)r * g.stride + 16 * c);
      }
    } else {
      for (int i = t; i < pw * ph; i += kOrbWG) {
        const int r = i / pw, c = i - r * pw;
        dst[r * P0 + c] = src[(size_t)r * g.stride + c];
      }
    }
  }
  __syncthreads();
  ORB_T(0);

  // ---- resize S (SW x SH) -> D (W x H, pitch lpitch(W)), INTER_LINEAR_EXACT;
  // the tables live in U past the largest resize target (host layout)
  auto resize_level = [&](const uint8_t* S, int SW, int SH, uint8_t* D, int W, int H) {
    const int SP = lpitch(SW), P = lpitch(W);
    // x coefficients for the padded row (columns past W: any in-bounds source)
    for (int i = t; i < P; i += kOrbWG) tabx[i] = i < W ? lin_coeff(i, W, SW) : 0;
    for (int i = t; i < H; i += kOrbWG) taby[i] = lin_coeff(i, H, SH);
    __syncthreads();
    // Four adjacent destination pixels per lane: their x coefficients are one
    // 16-byte LDS read, the row coefficient one, the 16 source bytes are read
    // before the four results leave as one dword (consecutive lanes write
    // consecutive dwords).  The padding bytes of a row get junk, never read.
    const int NG = P >> 2, NT = NG * H;
    const uint32_t mNG = div_magic(NG);
    // an opaque 1 (H > 0 is checked on the host): rp[0] / rp[1] stay two
    // byte reads (merged, they become a ds_read_u16 at odd addresses, which
    // made the kernel 1.5x slower)
    const int one = g.H > 0 ? 1 : 0;
    for (int i = t; i < NT; i += kOrbWG) {
      const int y = fdiv(i, mNG), x = 4 * (i - y * NG);
      const int cy = taby[y];
      const int4 c4 = *reinterpret_cast<const int4*>(tabx + x);
      const int cx[4] = {c4.x, c4.y, c4.z, c4.w};
      const uint8_t* r0 = S + (cy >> 9) * SP;
      const int d1 = cy & 511, d0 = 256 - d1;
      int p00[4], p01[4], p10[4], p11[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const uint8_t* rp = r0 + (cx[q] >> 9);
        p00[q] = rp[0];
        if (kGlob) {
          // global level buffers: the +1 neighbours are only read with a
          // non-zero weight (the last column / row may sit on the buffer's end)
          p01[q] = (cx[q] & 511) ? rp[1] : 0;
          p10[q] = d1 ? rp[SP] : 0;
          p11[q] = ((cx[q] & 511) && d1) ? rp[SP + 1] : 0;
        } else if (SLAM_ORB_KO & 2) {
          p01[q] = p10[q] = p11[q] = p00[q];
        } else {
          // LDS: past the last source row / column lies more of the LDS
          // allocation (U follows A), and a neighbour outside the source has
          // weight 0 -- read unconditionally (no exec-mask code per byte)
          p01[q] = rp[one];
          p10[q] = rp[SP];
          p11[q] = rp[SP + one];
        }
      }
      uint32_t w = 0u;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int c1 = cx[q] & 511, c0 = 256 - c1;
        const int v = d0 * (c0 * p00[q] + c1 * p01[q]) + d1 * (c0 * p10[q] + c1 * p11[q]);
        w |= (uint32_t)min((v + 32768) >> 16, 255) << (8 * q);
      }
      *reinterpret_cast<uint32_t*>(D + y * P + x) = w;
    }
    __syncthreads();
  };

  int nout = 0;      // keypoints written for this tile (uniform)
  int overflow = 0;  // uniform
  const int nlev = g.nlev[shp];
  const int lb = kGlob ? nlev : g.bat0[shp];  // levels lb .. nlev-1: the batched group below
  for (int l = 0; l < lb; ++l) {
#ifdef SLAM_ORB_PROFILE
    orb_lv = l;
#endif
    const int W = g.lw[shp][l], H = g.lh[shp][l];
    const int P = lpitch(W);  // row pitch of the level image
    if (l > 0) {
      // ---- resize level l-1 (A) -> l (U, INTER_LINEAR_EXACT), then U -> A
      resize_level(A, g.lw[shp][l - 1], g.lh[shp][l - 1], U, W, H);
      if (kGlob) {  // global level buffers: swap roles instead of copying
        uint8_t* tmp = A;
        A = U;
        U = tmp;
      } else {
        for (int i = t; i < (P * H + 15) >> 4; i += kOrbWG)
          reinterpret_cast<uint4*>(A)[i] = reinterpret_cast<const uint4*>(U)[i];
        __syncthreads();
      }
      ORB_T(1);
    }
    ORB_CUT(1);
    uint8_t* I = A;
    const int n_l = g.nl[l];
    if (W <= 2 * kEdge || H <= 2 * kEdge || n_l == 0) continue;  // uniform

    // ---- FAST score map over [29, W-30] x [29, H-30], rows padded to a
    // multiple of 4 bytes (SW4) so the NMS below reads it a dword at a time
    const int SWd = W - 2 * kNMS0, SHd = H - 2 * kNMS0;
    const int SW4 = (SWd + 3) & ~3;
    uint8_t* Smap = U;
    const uint32_t mS4 = div_magic(SW4);
    // Four pixels per pass: the 20 quick-reject reads of the group are all
    // issued before any Smap store.  Survivors (~8% of pixels, but present
    // in ~30% of waves) are queued in a wave-private LDS list (the tail of
    // U past the score map) and take the full test packed 64 per pass
    // instead of diverging inside every wave that holds one.
    // One dword of the map (4 adjacent pixels) per lane and pass: the centre
    // row window [x-3, x+6] and the rows y -/+ 3 come from aligned dword LDS
    // reads + v_alignbyte (8 reads per 4 pixels instead of 20 byte reads), and
    // the 4 map bytes leave as one dword (survivors' scores overwrite theirs below).
    const int NG4 = SW4 >> 2, SN4 = NG4 * SHd;
    const uint32_t mG4 = div_magic(NG4);
    uint32_t* fq = reinterpret_cast<uint32_t*>(lds + g.lds_fq) + wid * kFqW;
    auto win4 = [&](int a) {  // bytes a .. a+3 of the level image (any alignment)
      const uint32_t* wp = reinterpret_cast<const uint32_t*>(I + (a & ~3));
      return __builtin_amdgcn_alignbyte(wp[1], wp[0], a & 3);
    };
    // The queue carries over passes and is drained 64 entries at a time (full
    // waves), the rest after the loop; the trip count is wave-uniform, so every
    // lane of the wave takes part in each drain.  A survivor's score byte is
    // stored after its dword of the map was zeroed (same wave, program order).
    auto fast_drain = [&](int j0) {
      const int i = (int)fq[j0 + lane];  // padded-map index: y * SW4 + x
      const int y = fdiv(i, mS4), x = i - y * SW4;
      Smap[i] = (uint8_t)fast_full(I + (y + kNMS0) * P + x + kNMS0, P);
    };
    int nq = 0;  // wave-uniform queue length
    for (int gb = wid * 64;; gb += kOrbWG) {
      const bool more = gb < SN4;  // wave-uniform
      if (more) {
      const bool gv = gb + lane < SN4;
      const int gi = min(gb + lane, SN4 - 1);
      const int y = fdiv(gi, mG4), x = 4 * (gi - y * NG4);  // map coords of the first pixel
      const int a = (y + kNMS0) * P + x + kNMS0;
      const uint32_t* wp = reinterpret_cast<const uint32_t*>(I + ((a - 3) & ~3));
      const uint32_t d0 = wp[0], d1 = wp[1], d2 = wp[2], d3 = wp[3];
      const int sh = (a - 3) & 3;
      const uint32_t up = win4(a - 3 * P), dn = win4(a + 3 * P);
      const uint32_t q0 = __builtin_amdgcn_alignbyte(d1, d0, sh);  // bytes a-3 .. a
      const uint32_t q1 = __builtin_amdgcn_alignbyte(d2, d1, sh);  // a+1 .. a+4
      const uint32_t q2 = __builtin_amdgcn_alignbyte(d3, d2, sh);  // a+5 .. a+8
      const uint64_t lo = ((uint64_t)q1 << 32) | q0;               // a-3 .. a+4
      const uint32_t cc = (uint32_t)(lo >> 24);                    // a .. a+3
      const uint32_t rt = (uint32_t)(((uint64_t)q2 << 32 | q1) >> 16);  // a+3 .. a+6
      const uint32_t okv[2] = {quick4(cc, dn, rt, up, q0), quick4(cc >> 8, dn >> 8, rt >> 8, up >> 8, q0 >> 8)};
      // most waves hold no survivor at all (flat regions): one ballot skips
      // the four queue appends
      if (__ballot(gv && (okv[0] | okv[1]) != 0u) != 0ull) {
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const bool in = gv && x + q < SWd;
          const bool ok = in && ((okv[q & 1] >> (16 * (q >> 1))) & 0xFFFFu) != 0u;
          const uint64_t m = __ballot(ok);
          if (ok)
            fq[nq + (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32),
                                                   __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u))] =
                (uint32_t)(y * SW4 + x + q);
          nq += __popcll(m);
        }
      }
      if (gv) *reinterpret_cast<uint32_t*>(Smap + y * SW4 + x) = 0u;
      }
      // full waves while the map is scanned, the remainder at the end (one
      // drain site: the cornerScore code is instantiated once)
      while (nq >= 64 || (!more && nq > 0)) {
        const int n = min(nq, 64);
        nq -= n;
        if (lane < n) fast_drain(nq);
      }
      if (!more) break;
    }
    for (int i = t; i < 256; i += kOrbWG) hist[i] = 0;
    if (t < 8) ctr[t] = 0;
    __syncthreads();
    ORB_T(2);
    ORB_CUT(2);
    // ---- strict 3x3 NMS + border [31, W-32] -> candidates: one dword of
    // the score map (4 pixels) per lane; the scored pixels (FAST corners,
    // ~8 %) are queued in the wave-private list and take the 8-neighbour test
    // 64 at a time (full waves; the queue carries over passes, the rest is
    // drained after the loop, whose trip count is wave-uniform).  The candidate
    // order is immaterial: the list is ranked by (response, y, x) below and
    // the histogram is order-free.
    {
      const int CH = H - 2 * kEdge;
      const int NG = SW4 >> 2, NT = CH * NG;
      const uint32_t mG = div_magic(NG);
      auto nms_drain = [&](int j0) {
        const uint32_t yx = fq[j0 + lane];
        const int yq = (int)(yx >> 12), xq = (int)(yx & 4095u);
        const uint8_t* sp = Smap + (yq - kNMS0) * SW4 + (xq - kNMS0);
        const int s = sp[0];
        if (s > sp[-1] && s > sp[1] && s > sp[-SW4 - 1] && s > sp[-SW4] && s > sp[-SW4 + 1] &&
            s > sp[SW4 - 1] && s > sp[SW4] && s > sp[SW4 + 1]) {
          const int k = atomicAdd(&ctr[0], 1);
          if (k < g.cand_cap) gcand[k] = ((uint32_t)s << 23) | yx;
          atomicAdd(&hist[s], 1);
        }
      };
      int nq = 0;  // wave-uniform
      for (int base = wid * 64;; base += kOrbWG) {
        const bool more = base < NT;  // wave-uniform
        const int i = more ? base + lane : NT;
        uint32_t w4 = 0u;
        int y = 0, g4 = 0;
        if (i < NT) {
          const int yy = fdiv(i, mG);
          g4 = i - yy * NG;
          y = yy + kEdge;
          w4 = *reinterpret_cast<const uint32_t*>(Smap + (y - kNMS0) * SW4 + 4 * g4);
        }
        if (__ballot(w4 != 0u) != 0ull) {  // (no scored pixel in the wave: nothing to queue)
#pragma unroll
          for (int bb = 0; bb < 4; ++bb) {
            const int x = kNMS0 + 4 * g4 + bb;
            const bool ok = ((w4 >> (8 * bb)) & 255u) != 0u && x >= kEdge && x <= W - 1 - kEdge;
            const uint64_t m = __ballot(ok);
            if (ok)
              fq[nq + (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32),
                                                     __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u))] =
                  ((uint32_t)y << 12) | (uint32_t)x;
            nq += __popcll(m);
          }
        }
        while (nq >= 64 || (!more && nq > 0)) {
          const int n = min(nq, 64);
          nq -= n;
          if (lane < n) nms_drain(nq);
        }
        if (!more) break;
      }
    }
    __syncthreads();
    ORB_T(3);
    ORB_CUT(3);
    const int ncand = ctr[0];
    if (ncand > g.cand_cap) {  // cannot happen for strict maxima (density <= 1/4); guard anyway
      overflow = 1;
      break;
    }
    // ---- retainBest(2 n_l) threshold by FAST score (ties kept)
    if (wid == 0) {
      int T = 0;
      const int K = 2 * n_l;
      if (ncand > K) {
        const int c0 = hist[4 * lane], c1 = hist[4 * lane + 1];
        const int c2 = hist[4 * lane + 2], c3 = hist[4 * lane + 3];
        const int s = c0 + c1 + c2 + c3;
        int suf = s;  // inclusive suffix sum over lanes
        for (int off = 1; off < 64; off <<= 1) {
          const int o = __shfl_down(suf, off, 64);
          if (lane + off < 64) suf += o;
        }
        int acc = suf - s;  // scores in bins >= 4*lane+4
        int tl = -1;
        acc += c3;
        if (acc >= K) tl = 4 * lane + 3;
        else {
          acc += c2;
          if (acc >= K) tl = 4 * lane + 2;
          else {
            acc += c1;
            if (acc >= K) tl = 4 * lane + 1;
            else {
              acc += c0;
              if (acc >= K) tl = 4 * lane;
            }
          }
        }
        for (int off = 32; off > 0; off >>= 1) tl = max(tl, __shfl_xor(tl, off, 64));
        T = tl;
      }
      // survivors = candidates with score >= T
      int cnt = 0;
#pragma unroll
      for (int q = 0; q < 4; ++q) cnt += 4 * lane + q >= T ? hist[4 * lane + q] : 0;
      for (int off = 32; off > 0; off >>= 1) cnt += __shfl_xor(cnt, off, 64);
      if (lane == 0) {
        ctr[2] = T;
        ctr[4] = cnt;
      }
    }
    __syncthreads();
    // ---- survivors of retainBest(2n): LDS when they fit (the normal case),
    // else this tile's global scratch (same code, slower)
    const bool sv_lds = ctr[4] <= g.list_cap;  // uniform
    uint32_t* cand = sv_lds ? svc : gsvc;
    float* cresp = sv_lds ? svr : gsvr;
    {
      const int T = ctr[2];
      for (int i = t; i < ncand; i += kOrbWG) {
        const uint32_t c = gcand[i];
        if ((int)(c >> 23) >= T) {
          const int k = atomicAdd(&ctr[1], 1);
          cand[k] = c;
        }
      }
    }
    __syncthreads();
    const int nk = ctr[1];
    ORB_T(4);
    // the IC-angle disc masks (17 rows |v| = 0..16 x 8 dwords, 0x01 per
    // in-disc column) into the histogram's slots, dead from here to the
    // next level's NMS (published by the Harris barrier)
    uint32_t* icm = reinterpret_cast<uint32_t*>(hist);
    if (t < 17 * 8) {
      const int vv = t >> 3, dd = t & 7;
      const int um = vv < 16 ? (int)((0x368'9abc'ddee'efff'fULL >> (4 * vv)) & 15u) : -1;
      uint32_t mk = 0u;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int u = 4 * dd + j - 15;
        mk |= ((u < 0 ? -u : u) <= um ? 1u : 0u) << (8 * j);
      }
      icm[t] = mk;
    }
    // Harris: 16 lanes per survivor (4 per wave): lane s of the group takes window
    // pixels s, s + 16, s + 32, s + 48 (< 49) of the 7x7 block; the integer sums
    // a, b, c are reduced over the 16 lanes (exact in any order).
    {
      const int sub = lane >> 4, sl = lane & 15;
      for (int k0 = 4 * wid; k0 < nk; k0 += 4 * (kOrbWG / 64)) {
        const int k = k0 + sub;
        const uint32_t c = cand[k < nk ? k : k0];
        const int hx = (int)(c & 4095u), hy = (int)((c >> 12) & 2047u);
        int a = 0, bq = 0, cq = 0;
#pragma unroll 2  // (fully unrolled, its 32 loads in flight spill the kernel)
        for (int u = 0; u < 4; ++u) {
          const int e = sl + 16 * u;
          if (e < 49) {
            const int i = e / 7, j = e - 7 * (e / 7);
            const uint8_t* pp = I + (hy - 3 + i) * P + (hx - 3 + j);
            const int Ix = (pp[1] - pp[-1]) * 2 + (pp[-P + 1] - pp[-P - 1]) + (pp[P + 1] - pp[P - 1]);
            const int Iy = (pp[P] - pp[-P]) * 2 + (pp[P - 1] - pp[-P - 1]) + (pp[P + 1] - pp[-P + 1]);
            a += Ix * Ix;
            bq += Iy * Iy;
            cq += Ix * Iy;
          }
        }
#pragma unroll
        for (int off = 8; off > 0; off >>= 1) {
          a += __shfl_xor(a, off, 64);
          bq += __shfl_xor(bq, off, 64);
          cq += __shfl_xor(cq, off, 64);
        }
        if (sl == 0 && k < nk) cresp[k] = harris_resp(a, bq, cq);
      }
    }
    __syncthreads();
    ORB_T(5);
    // ---- exact rank by (response desc, y asc, x asc); L[rank] holds the sorted
    // list; then retainBest(n_l): everything at least as good as the n_l-th
    // response (ties kept).  Up to 64 survivors (the usual case): wave 0 alone,
    // lane i holding survivor i, the others' keys broadcast by v_readlane.
    if (nk <= 64) {
      if (wid == 0) {
        const bool live = lane < nk;
        const uint32_t ci = live ? cand[lane] : 0u;
        const float ri = live ? cresp[lane] : 0.f;
        const uint32_t yxi = ci & 0x7FFFFFu;  // (y << 12) | x: y-major order
        int rank = 0;
        for (int j = 0; j < nk; ++j) {
          const float rj = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(ri), j));
          const uint32_t yxj = (uint32_t)__builtin_amdgcn_readlane((int)yxi, j);
          rank += (rj > ri || (rj == ri && yxj < yxi)) ? 1 : 0;
        }
        if (live) {
          L[rank].x = (int)(ci & 4095u);
          L[rank].y = (int)((ci >> 12) & 2047u);
          L[rank].resp = ri;
        }
        int mm = nk;
        if (nk > n_l) {  // the n_l-th response, then the run of its ties after it
          const uint64_t bm = __ballot(live && rank == n_l - 1);
          const float rs = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(ri),
                                                                    (int)__builtin_ctzll(bm)));
          mm = n_l + (int)__popcll(__ballot(live && rank >= n_l && ri == rs));
        }
        if (lane == 0) ctr[3] = mm;
      }
    } else {
      for (int i = t; i < nk; i += kOrbWG) {
        const float ri = cresp[i];
        const uint32_t ci = cand[i];
        const uint32_t yxi = ci & 0x7FFFFFu;
        int rank = 0;
        int j = 0;
        for (; j + 4 <= nk; j += 4) {  // 8 LDS reads in flight per step
          float rj[4];
          uint32_t yxj[4];
#pragma unroll
          for (int u = 0; u < 4; ++u) {
            rj[u] = cresp[j + u];
            yxj[u] = cand[j + u] & 0x7FFFFFu;
          }
#pragma unroll
          for (int u = 0; u < 4; ++u) rank += (rj[u] > ri || (rj[u] == ri && yxj[u] < yxi)) ? 1 : 0;
        }
        for (; j < nk; ++j) {
          const float rj = cresp[j];
          const uint32_t yxj = cand[j] & 0x7FFFFFu;
          rank += (rj > ri || (rj == ri && yxj < yxi)) ? 1 : 0;
        }
        if (rank < g.list_cap) {
          L[rank].x = (int)(ci & 4095u);
          L[rank].y = (int)((ci >> 12) & 2047u);
          L[rank].resp = ri;
        }
      }
      __syncthreads();
      if (t == 0) {
        int mm = nk;
        int ovf = 0;
        if (nk > n_l) {
          const float rs = L[n_l - 1].resp;
          mm = n_l;
          while (mm < nk && mm < g.list_cap && L[mm].resp == rs) ++mm;
          if (mm == g.list_cap && mm < nk) ovf = 1;
        } else if (nk > g.list_cap) {
          ovf = 1;
        }
        ctr[3] = ovf ? -1 : mm;
      }
    }
    __syncthreads();
    const int m = ctr[3];
    ORB_T(6);
    ORB_CUT(6);
    if (m < 0 || nout + m > g.tcap) {
      overflow = 1;
      break;
    }
    // ---- IC angle: two keypoints per wave, 32 lanes each.  Lane i of a half
    // takes dword d = i & 7 of the 32-byte row window [cx-15, cx+16] on rows
    // v = -15 + (i >> 3) + 4 it, it = 0..7 (column 16 and row 16 lie outside
    // the disc); the disc |u| <= umax[|v|] (the umax table is symmetric:
    // |u| <= umax[|v|] <=> |v| <= umax[|u|]) is a 0x01-per-column byte mask per
    // (|v|, d) from the icm table, and two v_dot4_u32_u8 per row dword give
    // sum (u + 15) val and the row sum: m10 = sum (u + 15) val - 15 sum val,
    // m01 = sum v (row sum) -- integer moments, exact in any order
    {
      const int hh = lane >> 5, i = lane & 31, d = i & 7, r = i >> 3;
      const uint32_t uoff = 0x03020100u + 0x04040404u * (uint32_t)d;  // u + 15 per byte
      for (int k0 = 2 * wid; k0 < m; k0 += 2 * (kOrbWG / 64)) {
        const int k = k0 + hh;
        const bool kv = k < m;
        const int kk = kv ? k : k0;
        const int cx = L[kk].x, cy = L[kk].y;
        uint32_t su = 0u, s1 = 0u;
        int m01 = 0;
        const int a0 = (cy - 15 + r) * P + cx - 15 + 4 * d;
#pragma unroll 2
        for (int it = 0; it < 8; ++it) {
          const int v = r + 4 * it - 15;
          const int a = a0 + 4 * it * P;
          const uint32_t* wp = reinterpret_cast<const uint32_t*>(I + (a & ~3));
          const uint32_t px = __builtin_amdgcn_alignbyte(wp[1], wp[0], a & 3);
          const uint32_t ones = icm[8 * (v < 0 ? -v : v) + d];
          const uint32_t val = px & (ones * 0xFFu);
          su = __builtin_amdgcn_udot4(uoff, val, su, false);
          const uint32_t rs = __builtin_amdgcn_udot4(0x01010101u, val, 0u, false);
          s1 += rs;
          m01 += v * (int)rs;
        }
        int m10 = (int)su - 15 * (int)s1;
        for (int off = 16; off > 0; off >>= 1) {
          m10 += __shfl_xor(m10, off, 64);
          m01 += __shfl_xor(m01, off, 64);
        }
        if (i == 0 && kv) L[k].angle = fast_atan2_deg((float)m01, (float)m10);
      }
    }
    // ---- 7x7 Gaussian (float path) over [9, W-10] x [9, H-10] into U
    const int BW = W - 2 * kBl0, BH = H - 2 * kBl0;
    const int BP = lpitch(BW);  // row pitch of the blurred level
    uint8_t* Bl = U;
    __syncthreads();  // Smap and the survivor lists are dead from here (L holds the level)
    ORB_T(7);
    ORB_CUT(7);
    // ---- keypoint records (one lane per keypoint, wave 0): the output row, and
    // L[k] becomes what rBRIEF needs -- the sample centre in blurred-level
    // coordinates and cos / sin of the angle -- computed once per keypoint
    // instead of by each of its 32 rBRIEF lanes (the f64 sin / cos sequences
    // were issued once per half wave); published by the barrier after the blur
    if (wid == 0) {
      const float ls = g.ls[l];
      for (int k = lane; k < m; k += 64) {
        const KP kp = L[k];
        const float xl = (float)kp.x * ls, yl = (float)kp.y * ls;  // pt *= layerScale
        const float inv = 1.f / ls;
        const int o = nout + k;
        okp[(size_t)o * 5 + 0] = (float)((double)xl + (double)x0);
        okp[(size_t)o * 5 + 1] = (float)((double)yl + (double)y0);
        okp[(size_t)o * 5 + 2] = 31.f * ls;
        okp[(size_t)o * 5 + 3] = kp.angle;
        okp[(size_t)o * 5 + 4] = kp.resp;
        ooct[o] = l;
        float ang = kp.angle;
        ang *= (float)(3.14159265358979323846 / 180.f);
        KP q;
        q.x = rne_f(xl * inv) - kBl0;
        q.y = rne_f(yl * inv) - kBl0;
        q.resp = (float)cos((double)ang);
        q.angle = (float)sin((double)ang);
        L[k] = q;
      }
    }
    {
      // 4 adjacent output columns per lane (x = kBl0 + 4 cg: a dword boundary of
      // the pitched level): the 10 source bytes x-3 .. x+6 of a row are the
      // three aligned dwords at x-4, x, x+4 (consecutive lanes read consecutive
      // dwords: no bank conflicts) shifted by v_alignbyte; four independent FMA
      // chains; rows slide down a per-lane segment; the four results leave as
      // one dword of the pitched blurred level.  Every output keeps the exact
      // operation order of the scalar form (row: fmaf k0..k6 from 0; column:
      // w3*k3 then fmaf(w[+d]+w[-d], k[3+d])).
      static_assert((kBl0 & 3) == 0, "blur origin must be dword aligned");
      const float k0 = g.gk[0], k1 = g.gk[1], k2 = g.gk[2], k3 = g.gk[3];
      const float k4 = g.gk[4], k5 = g.gk[5], k6 = g.gk[6];
      const int ncg = BP >> 2;
      const int nseg = max(1, kOrbWG / ncg);
      const int seg = (BH + nseg - 1) / nseg;
      for (int item = t; item < ncg * nseg; item += kOrbWG) {
        const int sg = item / ncg, cg = item - sg * ncg;
        const int r0 = sg * seg, r1 = min(BH, r0 + seg);
        if (r0 >= r1) continue;
        const int c4 = 4 * cg, x = c4 + kBl0;
        auto rowf4 = [&](int y, float4& o) {
          const uint32_t* wp = reinterpret_cast<const uint32_t*>(I + y * P + x - 4);
          const uint32_t d0 = wp[0], d1 = wp[1], d2 = wp[2];
          const uint32_t q0 = __builtin_amdgcn_alignbyte(d1, d0, 1);  // bytes x-3 .. x
          const uint32_t q1 = __builtin_amdgcn_alignbyte(d2, d1, 1);  // x+1 .. x+4
          const uint32_t q2 = d2 >> 8;                                // x+5 .. x+7
          float p[10];
          p[0] = (float)((q0 >> 0) & 0xFFu);
          p[1] = (float)((q0 >> 8) & 0xFFu);
          p[2] = (float)((q0 >> 16) & 0xFFu);
          p[3] = (float)((q0 >> 24) & 0xFFu);
          p[4] = (float)((q1 >> 0) & 0xFFu);
          p[5] = (float)((q1 >> 8) & 0xFFu);
          p[6] = (float)((q1 >> 16) & 0xFFu);
          p[7] = (float)((q1 >> 24) & 0xFFu);
          p[8] = (float)((q2 >> 0) & 0xFFu);
          p[9] = (float)((q2 >> 8) & 0xFFu);
          float r[4];
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            float acc = 0.f;
            acc = fmaf(p[j], k0, acc);
            acc = fmaf(p[j + 1], k1, acc);
            acc = fmaf(p[j + 2], k2, acc);
            acc = fmaf(p[j + 3], k3, acc);
            acc = fmaf(p[j + 4], k4, acc);
            acc = fmaf(p[j + 5], k5, acc);
            acc = fmaf(p[j + 6], k6, acc);
            r[j] = acc;
          }
          o = make_float4(r[0], r[1], r[2], r[3]);
        };
        const int yb = r0 + kBl0;  // first output row (image coords)
        // the 7 row sums of the window in a ring of registers: output row r0 + k
        // reads slots (k .. k + 6) mod 7 and its successor's new row replaces
        // slot k mod 7 -- the loop is unrolled 7 times so the ring rotates by
        // renaming (a shifted window costs 14 register moves per row).  Column
        // pass on packed pairs (columns 0-1, 2-3: v_pk_add / v_pk_mul / v_pk_fma,
        // per element the scalar form's operations); rounded results packed by
        // v_cvt_pk_u8_f32 (exact: they are integers in [0, 255])
        float4 w[7];
        static_for<0, 7>([&](auto I) { rowf4(yb - 3 + decltype(I)::value, w[decltype(I)::value]); });
        typedef float f2 __attribute__((ext_vector_type(2)));
        const f2 kk3 = {k3, k3}, kk4 = {k4, k4}, kk5 = {k5, k5}, kk6 = {k6, k6};
        for (int r = r0; r < r1; r += 7) {
          static_for<0, 7>([&](auto K) {
            constexpr int k = decltype(K)::value;
            if (r + k < r1) {
              const float4 a0 = w[k % 7], a1 = w[(k + 1) % 7], a2 = w[(k + 2) % 7];
              const float4 a3 = w[(k + 3) % 7], a4 = w[(k + 4) % 7], a5 = w[(k + 5) % 7];
              const float4 a6 = w[(k + 6) % 7];
              auto col = [&](f2 x0, f2 x1, f2 x2, f2 x3, f2 x4, f2 x5, f2 x6) {
                f2 s0 = x3 * kk3;
                s0 = __builtin_elementwise_fma(x4 + x2, kk4, s0);
                s0 = __builtin_elementwise_fma(x5 + x1, kk5, s0);
                return __builtin_elementwise_fma(x6 + x0, kk6, s0);
              };
              const f2 lo = col(f2{a0.x, a0.y}, f2{a1.x, a1.y}, f2{a2.x, a2.y}, f2{a3.x, a3.y},
                                f2{a4.x, a4.y}, f2{a5.x, a5.y}, f2{a6.x, a6.y});
              const f2 hi = col(f2{a0.z, a0.w}, f2{a1.z, a1.w}, f2{a2.z, a2.w}, f2{a3.z, a3.w},
                                f2{a4.z, a4.w}, f2{a5.z, a5.w}, f2{a6.z, a6.w});
              uint32_t packed = __builtin_amdgcn_cvt_pk_u8_f32(rintf(lo.x), 0, 0u);
              packed = __builtin_amdgcn_cvt_pk_u8_f32(rintf(lo.y), 1, packed);
              packed = __builtin_amdgcn_cvt_pk_u8_f32(rintf(hi.x), 2, packed);
              packed = __builtin_amdgcn_cvt_pk_u8_f32(rintf(hi.y), 3, packed);
              *reinterpret_cast<uint32_t*>(Bl + (r + k) * BP + c4) = packed;
              if (r + k + 1 < r1) rowf4(r + k + 1 + kBl0 + 3, w[k]);
            }
          });
        }
      }
    }
    __syncthreads();
    ORB_T(8);
    ORB_CUT(8);
    // ---- rBRIEF: 32 lanes per keypoint, one descriptor byte per lane
    {
      const int half = lane >> 5, byte = lane & 31;
      // the lane's 8 pattern pairs, one dword each (x1, y1, x2, y2 as int8),
      // kept across keypoints; converted per use (32 converted floats kept
      // live across the loop made the kernel spill)
      uint32_t pat[8];
#pragma unroll
      for (int bit = 0; bit < 8; ++bit)
        pat[bit] = reinterpret_cast<const uint32_t*>(c_pattern)[byte * 8 + bit];
      for (int k = 2 * wid + half; k < m; k += 2 * (kOrbWG / 64)) {
        const KP kp = L[k];  // (centre x, centre y, cos, sin), see above
        const int cx = kp.x, cy = kp.y;
        const float a = kp.resp, bb = kp.angle;
        int val = 0;
#pragma unroll
        for (int bit = 0; bit < 8; ++bit) {
          uint32_t pw = pat[bit];
          __asm__ volatile("" : "+v"(pw));
          const float px1 = (float)(int8_t)(pw & 0xFFu), py1 = (float)(int8_t)((pw >> 8) & 0xFFu);
          const float px2 = (float)(int8_t)((pw >> 16) & 0xFFu), py2 = (float)(int8_t)(pw >> 24);
          const int ix1 = rne_f(px1 * a - py1 * bb), iy1 = rne_f(px1 * bb + py1 * a);
          const int ix2 = rne_f(px2 * a - py2 * bb), iy2 = rne_f(px2 * bb + py2 * a);
          const int t0 = Bl[(cy + iy1) * BP + cx + ix1];
          const int t1 = Bl[(cy + iy2) * BP + cx + ix2];
          val |= (t0 < t1 ? 1 : 0) << bit;
        }
        odesc[(size_t)(nout + k) * 32 + byte] = (uint8_t)val;
      }
    }
    nout += m;
    __syncthreads();
    ORB_T(9);
  }

  // ======================= batched small levels lb .. nlev-1 =======================
  // The small levels' per-keypoint phases cost about the same fixed latency on
  // every level whatever its size (round-4 per-level profile: levels 3-6 of a
  // 216x192 patch hold 29 % of the pixels and 40 % of the cycles).  Here their
  // images are resident together in A (slots g.bslot), and each phase is ONE
  // pass over all of them: resize chain, FAST maps (U, g.bsmap), NMS (per-level
  // candidate ranges g.bcand, histograms / counters hist4 / ctr4 in A),
  // retainBest(2n) thresholds (wave j: level j), survivors, Harris, rank +
  // retainBest(n) (wave j: level j when every level has <= 64 survivors),
  // IC angle, records, blurred levels (U, g.bbl), rBRIEF.  Every keypoint's
  // arithmetic and the level-major output order are those of the per-level
  // loop above: bit-identical output.
  if (!kGlob && lb < nlev && !overflow) {
#ifdef SLAM_ORB_PROFILE
    orb_lv = lb;
#endif
    const int NB = nlev - lb;
    int* hist4 = reinterpret_cast<int*>(A + g.bhist[shp]);  // [kMaxBat][256]
    int* ctr4 = hist4 + kMaxBat * 256;  // [kMaxBat][16]: 0 candidates, 1 survivors, 2 T, 3 kept, 4 count
    int bW[kMaxBat], bH[kMaxBat], bP[kMaxBat], bSWd[kMaxBat], bSW4[kMaxBat], bNG[kMaxBat];
    int bSN4[kMaxBat], bNT[kMaxBat], bCap[kMaxBat], bC0[kMaxBat];
    uint32_t bmG[kMaxBat], bmS[kMaxBat];
    const uint8_t* bI[kMaxBat];
    uint8_t* bSm[kMaxBat];
#pragma unroll
    for (int j = 0; j < kMaxBat; ++j) {
      const int l = min(lb + j, nlev - 1);
      bW[j] = g.lw[shp][l];
      bH[j] = g.lh[shp][l];
      bP[j] = lpitch(bW[j]);
      bSWd[j] = bW[j] - 2 * kNMS0;
      bSW4[j] = (bSWd[j] + 3) & ~3;
      bNG[j] = bSW4[j] >> 2;
      bSN4[j] = j < NB ? bNG[j] * (bH[j] - 2 * kNMS0) : 0;
      bNT[j] = j < NB ? bNG[j] * (bH[j] - 2 * kEdge) : 0;
      bmG[j] = div_magic(bNG[j]);
      bmS[j] = div_magic(bSW4[j]);
      bI[j] = A + g.bslot[shp][min(j, NB - 1)];
      bSm[j] = U + g.bsmap[shp][min(j, NB - 1)];
      bC0[j] = g.bcand[shp][min(j, NB - 1)];
      bCap[j] = j < NB ? g.bcand[shp][j + 1] - g.bcand[shp][j] : 0;
    }
    // ---- (1) resize chain: level lb via U into slot 0 (level lb-1 in A is dead
    // after it), then slot j-1 -> slot j directly
    for (int j = 0; j < NB; ++j) {
      const int l = lb + j;
      uint8_t* D = j == 0 ? U : A + g.bslot[shp][j];
      const uint8_t* Sp = j == 0 ? A : A + g.bslot[shp][j - 1];
      resize_level(Sp, g.lw[shp][l - 1], g.lh[shp][l - 1], D, g.lw[shp][l], g.lh[shp][l]);
      if (j == 0) {
        for (int i = t; i < (bP[0] * bH[0] + 15) >> 4; i += kOrbWG)
          reinterpret_cast<uint4*>(A + g.bslot[shp][0])[i] = reinterpret_cast<const uint4*>(U)[i];
        __syncthreads();
      }
    }
    for (int i = t; i < NB * 256; i += kOrbWG) hist4[i] = 0;
    if (t < kMaxBat * 16) ctr4[t] = 0;
    ORB_T(1);
    // ---- (2) FAST score maps of every level, one pass (as the per-level
    // form; queue entries carry the level in bits 30-31)
    uint32_t* fq = reinterpret_cast<uint32_t*>(lds + g.lds_fq) + wid * kFqW;
    {
      const int tot = bSN4[0] + bSN4[1] + bSN4[2] + bSN4[3];
      auto fast_drain = [&](int j0) {
        const uint32_t e = fq[j0 + lane];
        const int j = (int)(e >> 30), i = (int)(e & 0x3FFFFFFFu);
        const int sw4 = pick4(j, bSW4), P = pick4(j, bP);
        const int y = fdiv(i, pick4(j, bmS)), x = i - y * sw4;
        pick4(j, bSm)[i] = (uint8_t)fast_full(pick4(j, bI) + (y + kNMS0) * P + x + kNMS0, P);
      };
      int nq = 0;
      for (int gb = wid * 64;; gb += kOrbWG) {
        const bool more = gb < tot;  // wave-uniform
        if (more) {
          const bool gv = gb + lane < tot;
          int loc = min(gb + lane, tot - 1);
          const int j = seg4(loc, NB, bSN4[0], bSN4[1], bSN4[2]);
          const uint8_t* I = pick4(j, bI);
          const int P = pick4(j, bP), NG4 = pick4(j, bNG), SW4 = pick4(j, bSW4), SWd = pick4(j, bSWd);
          uint8_t* Smap = pick4(j, bSm);
          auto win4 = [&](int a) {
            const uint32_t* wp = reinterpret_cast<const uint32_t*>(I + (a & ~3));
            return __builtin_amdgcn_alignbyte(wp[1], wp[0], a & 3);
          };
          const int y = fdiv(loc, pick4(j, bmG)), x = 4 * (loc - y * NG4);
          const int a = (y + kNMS0) * P + x + kNMS0;
          const uint32_t* wp = reinterpret_cast<const uint32_t*>(I + ((a - 3) & ~3));
          const uint32_t d0 = wp[0], d1 = wp[1], d2 = wp[2], d3 = wp[3];
          const int sh = (a - 3) & 3;
          const uint32_t up = win4(a - 3 * P), dn = win4(a + 3 * P);
          const uint32_t q0 = __builtin_amdgcn_alignbyte(d1, d0, sh);
          const uint32_t q1 = __builtin_amdgcn_alignbyte(d2, d1, sh);
          const uint32_t q2 = __builtin_amdgcn_alignbyte(d3, d2, sh);
          const uint64_t lo = ((uint64_t)q1 << 32) | q0;
          const uint32_t cc = (uint32_t)(lo >> 24);
          const uint32_t rt = (uint32_t)(((uint64_t)q2 << 32 | q1) >> 16);
          const uint32_t okv[2] = {quick4(cc, dn, rt, up, q0), quick4(cc >> 8, dn >> 8, rt >> 8, up >> 8, q0 >> 8)};
          if (__ballot(gv && (okv[0] | okv[1]) != 0u) != 0ull) {
#pragma unroll
            for (int q = 0; q < 4; ++q) {
              const bool in = gv && x + q < SWd;
              const bool ok = in && ((okv[q & 1] >> (16 * (q >> 1))) & 0xFFFFu) != 0u;
              const uint64_t m = __ballot(ok);
              if (ok)
                fq[nq + (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32),
                                                       __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u))] =
                    ((uint32_t)j << 30) | (uint32_t)(y * SW4 + x + q);
              nq += __popcll(m);
            }
          }
          if (gv) *reinterpret_cast<uint32_t*>(Smap + y * SW4 + x) = 0u;
        }
        while (nq >= 64 || (!more && nq > 0)) {
          const int n = min(nq, 64);
          nq -= n;
          if (lane < n) fast_drain(nq);
        }
        if (!more) break;
      }
    }
    __syncthreads();
    ORB_T(2);
    // ---- (3) strict 3x3 NMS + border over every level's map, one pass
    // (queue entries: level in bits 24-25, y in 12-22, x in 0-11)
    {
      const int tot = bNT[0] + bNT[1] + bNT[2] + bNT[3];
      auto nms_drain = [&](int j0) {
        const uint32_t e = fq[j0 + lane];
        const int j = (int)(e >> 24);
        const uint32_t yx = e & 0xFFFFFFu;
        const int yq = (int)(yx >> 12), xq = (int)(yx & 4095u);
        const int SW4 = pick4(j, bSW4);
        const uint8_t* sp = pick4(j, bSm) + (yq - kNMS0) * SW4 + (xq - kNMS0);
        const int s = sp[0];
        if (s > sp[-1] && s > sp[1] && s > sp[-SW4 - 1] && s > sp[-SW4] && s > sp[-SW4 + 1] &&
            s > sp[SW4 - 1] && s > sp[SW4] && s > sp[SW4 + 1]) {
          const int k = atomicAdd(&ctr4[16 * j], 1);
          if (k < pick4(j, bCap)) gcand[pick4(j, bC0) + k] = ((uint32_t)s << 23) | yx;
          atomicAdd(&hist4[256 * j + s], 1);
        }
      };
      int nq = 0;
      for (int base = wid * 64;; base += kOrbWG) {
        const bool more = base < tot;  // wave-uniform
        uint32_t w4 = 0u;
        int y = 0, g4 = 0, j = 0;
        if (more && base + lane < tot) {
          int loc = base + lane;
          j = seg4(loc, NB, bNT[0], bNT[1], bNT[2]);
          const int yy = fdiv(loc, pick4(j, bmG));
          g4 = loc - yy * pick4(j, bNG);
          y = yy + kEdge;
          w4 = *reinterpret_cast<const uint32_t*>(pick4(j, bSm) + (y - kNMS0) * pick4(j, bSW4) + 4 * g4);
        }
        if (__ballot(w4 != 0u) != 0ull) {
          const int Wj = pick4(j, bW);
#pragma unroll
          for (int bb = 0; bb < 4; ++bb) {
            const int x = kNMS0 + 4 * g4 + bb;
            const bool ok = ((w4 >> (8 * bb)) & 255u) != 0u && x >= kEdge && x <= Wj - 1 - kEdge;
            const uint64_t m = __ballot(ok);
            if (ok)
              fq[nq + (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32),
                                                     __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u))] =
                  ((uint32_t)j << 24) | ((uint32_t)y << 12) | (uint32_t)x;
            nq += __popcll(m);
          }
        }
        while (nq >= 64 || (!more && nq > 0)) {
          const int n = min(nq, 64);
          nq -= n;
          if (lane < n) nms_drain(nq);
        }
        if (!more) break;
      }
    }
    __syncthreads();
    ORB_T(3);
    // ---- (4) retainBest(2 n_l) thresholds: wave j, level j
    if (wid < NB) {
      const int j = wid;
      const int* hist = hist4 + 256 * j;
      const int ncand = ctr4[16 * j];
      int T = 0;
      const int K = 2 * g.nl[lb + j];
      if (ncand > K) {
        const int c0 = hist[4 * lane], c1 = hist[4 * lane + 1];
        const int c2 = hist[4 * lane + 2], c3 = hist[4 * lane + 3];
        const int sm = c0 + c1 + c2 + c3;
        int suf = sm;
        for (int off = 1; off < 64; off <<= 1) {
          const int o = __shfl_down(suf, off, 64);
          if (lane + off < 64) suf += o;
        }
        int acc = suf - sm;
        int tl = -1;
        acc += c3;
        if (acc >= K) tl = 4 * lane + 3;
        else {
          acc += c2;
          if (acc >= K) tl = 4 * lane + 2;
          else {
            acc += c1;
            if (acc >= K) tl = 4 * lane + 1;
            else {
              acc += c0;
              if (acc >= K) tl = 4 * lane;
            }
          }
        }
        for (int off = 32; off > 0; off >>= 1) tl = max(tl, __shfl_xor(tl, off, 64));
        T = tl;
      }
      int cnt = 0;
#pragma unroll
      for (int q = 0; q < 4; ++q) cnt += 4 * lane + q >= T ? hist[4 * lane + q] : 0;
      for (int off = 32; off > 0; off >>= 1) cnt += __shfl_xor(cnt, off, 64);
      if (lane == 0) {
        ctr4[16 * j + 2] = T;
        ctr4[16 * j + 4] = cnt;
      }
    }
    __syncthreads();
    int bN[kMaxBat], bT[kMaxBat], bCnt[kMaxBat];
    bool ovf = false;
#pragma unroll
    for (int j = 0; j < kMaxBat; ++j) {
      bN[j] = j < NB ? ctr4[16 * j] : 0;
      bT[j] = ctr4[16 * j + 2];
      bCnt[j] = j < NB ? ctr4[16 * j + 4] : 0;
      ovf = ovf || bN[j] > bCap[j];
    }
    if (ovf) {  // cannot happen for strict maxima (density <= 1/4); guard anyway
      overflow = 1;
    } else {
      // ---- (5) survivors of every level, packed level after level (LDS when
      // they all fit, the tile's global scratch otherwise)
      const int cnt_tot = bCnt[0] + bCnt[1] + bCnt[2] + bCnt[3];
      const bool sv_lds = cnt_tot <= g.list_cap;  // uniform
      uint32_t* cand = sv_lds ? svc : gsvc;
      float* cresp = sv_lds ? svr : gsvr;
      int bSo[kMaxBat];
      bSo[0] = 0;
#pragma unroll
      for (int j = 1; j < kMaxBat; ++j) bSo[j] = bSo[j - 1] + bCnt[j - 1];
      {
        const int tot = bN[0] + bN[1] + bN[2] + bN[3];
        for (int i = t; i < tot; i += kOrbWG) {
          int loc = i;
          const int j = seg4(loc, NB, bN[0], bN[1], bN[2]);
          const uint32_t c = gcand[pick4(j, bC0) + loc];
          if ((int)(c >> 23) >= pick4(j, bT)) {
            const int k = atomicAdd(&ctr4[16 * j + 1], 1);
            cand[pick4(j, bSo) + k] = c;
          }
        }
      }
      __syncthreads();
      ORB_T(4);
      // the IC-angle disc masks into the (unused) per-level histogram slots
      uint32_t* icm = reinterpret_cast<uint32_t*>(hist);
      if (t < 17 * 8) {
        const int vv = t >> 3, dd = t & 7;
        const int um = vv < 16 ? (int)((0x368'9abc'ddee'efff'fULL >> (4 * vv)) & 15u) : -1;
        uint32_t mk = 0u;
#pragma unroll
        for (int jj = 0; jj < 4; ++jj) {
          const int u = 4 * dd + jj - 15;
          mk |= ((u < 0 ? -u : u) <= um ? 1u : 0u) << (8 * jj);
        }
        icm[t] = mk;
      }
      // ---- (6) Harris on every survivor (16 lanes per survivor, as above)
      {
        const int sub = lane >> 4, sl = lane & 15;
        for (int k0 = 4 * wid; k0 < cnt_tot; k0 += 4 * (kOrbWG / 64)) {
          const int k = k0 + sub;
          int loc = k < cnt_tot ? k : k0;
          const uint32_t c = cand[loc];
          const int j = seg4(loc, NB, bCnt[0], bCnt[1], bCnt[2]);
          const uint8_t* I = pick4(j, bI);
          const int P = pick4(j, bP);
          const int hx = (int)(c & 4095u), hy = (int)((c >> 12) & 2047u);
          int a = 0, bq = 0, cq = 0;
#pragma unroll 2
          for (int u = 0; u < 4; ++u) {
            const int e = sl + 16 * u;
            if (e < 49) {
              const int i = e / 7, jx = e - 7 * (e / 7);
              const uint8_t* pp = I + (hy - 3 + i) * P + (hx - 3 + jx);
              const int Ix = (pp[1] - pp[-1]) * 2 + (pp[-P + 1] - pp[-P - 1]) + (pp[P + 1] - pp[P - 1]);
              const int Iy = (pp[P] - pp[-P]) * 2 + (pp[P - 1] - pp[-P - 1]) + (pp[P + 1] - pp[-P + 1]);
              a += Ix * Ix;
              bq += Iy * Iy;
              cq += Ix * Iy;
            }
          }
#pragma unroll
          for (int off = 8; off > 0; off >>= 1) {
            a += __shfl_xor(a, off, 64);
            bq += __shfl_xor(bq, off, 64);
            cq += __shfl_xor(cq, off, 64);
          }
          if (sl == 0 && k < cnt_tot) cresp[k] = harris_resp(a, bq, cq);
        }
      }
      __syncthreads();
      ORB_T(5);
      // ---- (7) exact rank per level + retainBest(n_l); the kept keypoints of
      // level j at L[sum of the earlier levels' kept counts ...]
      const bool small = bCnt[0] <= 64 && bCnt[1] <= 64 && bCnt[2] <= 64 && bCnt[3] <= 64;
      if (small) {
        int rank = 0, mm = 0;
        bool live = false;
        uint32_t ci = 0u;
        float ri = 0.f;
        if (wid < NB) {
          const int j = wid, nk = pick4(j, bCnt), off = pick4(j, bSo), n_l = g.nl[lb + j];
          live = lane < nk;
          ci = live ? cand[off + lane] : 0u;
          ri = live ? cresp[off + lane] : 0.f;
          const uint32_t yxi = ci & 0x7FFFFFu;
          for (int jj = 0; jj < nk; ++jj) {
            const float rj = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(ri), jj));
            const uint32_t yxj = (uint32_t)__builtin_amdgcn_readlane((int)yxi, jj);
            rank += (rj > ri || (rj == ri && yxj < yxi)) ? 1 : 0;
          }
          mm = nk;
          if (nk > n_l) {
            const uint64_t bm = __ballot(live && rank == n_l - 1);
            const float rs = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(ri),
                                                                      (int)__builtin_ctzll(bm)));
            mm = n_l + (int)__popcll(__ballot(live && rank >= n_l && ri == rs));
          }
          if (lane == 0) ctr4[16 * j + 3] = mm;
        }
        __syncthreads();
        if (wid < NB) {
          int Loff = 0;
          for (int jj = 0; jj < wid; ++jj) Loff += ctr4[16 * jj + 3];
          if (live && rank < mm) {
            L[Loff + rank].x = (int)(ci & 4095u);
            L[Loff + rank].y = (int)((ci >> 12) & 2047u);
            L[Loff + rank].resp = ri;
          }
        }
      } else {
        int Loff = 0;
        for (int j = 0; j < NB; ++j) {
          const int nk = pick4(j, bCnt), off = pick4(j, bSo), n_l = g.nl[lb + j];
          for (int i = t; i < nk; i += kOrbWG) {
            const float ri = cresp[off + i];
            const uint32_t ci = cand[off + i];
            const uint32_t yxi = ci & 0x7FFFFFu;
            int rank = 0;
            for (int jj = 0; jj < nk; ++jj) {
              const float rj = cresp[off + jj];
              const uint32_t yxj = cand[off + jj] & 0x7FFFFFu;
              rank += (rj > ri || (rj == ri && yxj < yxi)) ? 1 : 0;
            }
            if (Loff + rank < g.list_cap) {
              L[Loff + rank].x = (int)(ci & 4095u);
              L[Loff + rank].y = (int)((ci >> 12) & 2047u);
              L[Loff + rank].resp = ri;
            }
          }
          __syncthreads();
          if (t == 0) {
            int mm = nk, bad = 0;
            if (nk > n_l) {
              if (Loff + n_l > g.list_cap) {
                bad = 1;
              } else {
                const float rs = L[Loff + n_l - 1].resp;
                mm = n_l;
                while (mm < nk && Loff + mm < g.list_cap && L[Loff + mm].resp == rs) ++mm;
                if (Loff + mm == g.list_cap && mm < nk) bad = 1;
              }
            } else if (Loff + nk > g.list_cap) {
              bad = 1;
            }
            ctr4[16 * j + 3] = bad ? -1 : mm;
          }
          __syncthreads();
          const int mj = ctr4[16 * j + 3];
          if (mj < 0) break;  // (uniform) reported as overflow below
          Loff += mj;
        }
      }
      __syncthreads();
      ORB_T(6);
      int bM[kMaxBat];
      bool bad = false;
#pragma unroll
      for (int j = 0; j < kMaxBat; ++j) {
        bM[j] = j < NB ? ctr4[16 * j + 3] : 0;
        bad = bad || bM[j] < 0;
      }
      const int M = bad ? 0 : bM[0] + bM[1] + bM[2] + bM[3];
      if (bad || nout + M > g.tcap) {
        overflow = 1;
      } else {
        // ---- (8) IC angle of every kept keypoint (two per wave, as above)
        {
          const int hh = lane >> 5, i = lane & 31, d = i & 7, r = i >> 3;
          const uint32_t uoff = 0x03020100u + 0x04040404u * (uint32_t)d;
          for (int k0 = 2 * wid; k0 < M; k0 += 2 * (kOrbWG / 64)) {
            const int k = k0 + hh;
            const bool kv = k < M;
            const int kk = kv ? k : k0;
            int loc = kk;
            const int j = seg4(loc, NB, bM[0], bM[1], bM[2]);
            const uint8_t* I = pick4(j, bI);
            const int P = pick4(j, bP);
            const int cx = L[kk].x, cy = L[kk].y;
            uint32_t su = 0u, s1 = 0u;
            int m01 = 0;
            const int a0 = (cy - 15 + r) * P + cx - 15 + 4 * d;
#pragma unroll 2
            for (int it = 0; it < 8; ++it) {
              const int v = r + 4 * it - 15;
              const int a = a0 + 4 * it * P;
              const uint32_t* wp = reinterpret_cast<const uint32_t*>(I + (a & ~3));
              const uint32_t px = __builtin_amdgcn_alignbyte(wp[1], wp[0], a & 3);
              const uint32_t ones = icm[8 * (v < 0 ? -v : v) + d];
              const uint32_t val = px & (ones * 0xFFu);
              su = __builtin_amdgcn_udot4(uoff, val, su, false);
              const uint32_t rs = __builtin_amdgcn_udot4(0x01010101u, val, 0u, false);
              s1 += rs;
              m01 += v * (int)rs;
            }
            int m10 = (int)su - 15 * (int)s1;
            for (int off = 16; off > 0; off >>= 1) {
              m10 += __shfl_xor(m10, off, 64);
              m01 += __shfl_xor(m01, off, 64);
            }
            if (i == 0 && kv) L[k].angle = fast_atan2_deg((float)m01, (float)m10);
          }
        }
        __syncthreads();  // the maps and survivor lists are dead (L holds the group)
        ORB_T(7);
        // ---- (9) keypoint records (wave 0, one lane per keypoint), then the
        // blurred levels into U (threads shared in proportion to the pixels)
        if (wid == 0) {
          for (int k = lane; k < M; k += 64) {
            int loc = k;
            const int j = seg4(loc, NB, bM[0], bM[1], bM[2]);
            const int l = lb + j;
            const float ls = g.ls[l];
            const KP kp = L[k];
            const float xl = (float)kp.x * ls, yl = (float)kp.y * ls;
            const float inv = 1.f / ls;
            const int o = nout + k;
            okp[(size_t)o * 5 + 0] = (float)((double)xl + (double)x0);
            okp[(size_t)o * 5 + 1] = (float)((double)yl + (double)y0);
            okp[(size_t)o * 5 + 2] = 31.f * ls;
            okp[(size_t)o * 5 + 3] = kp.angle;
            okp[(size_t)o * 5 + 4] = kp.resp;
            ooct[o] = l;
            float ang = kp.angle;
            ang *= (float)(3.14159265358979323846 / 180.f);
            KP q;
            q.x = rne_f(xl * inv) - kBl0;
            q.y = rne_f(yl * inv) - kBl0;
            q.resp = (float)cos((double)ang);
            q.angle = (float)sin((double)ang);
            L[k] = q;
          }
        }
        int bBP[kMaxBat], bBH[kMaxBat], bSeg[kMaxBat], bItems[kMaxBat], bNcg[kMaxBat];
        uint8_t* bBl[kMaxBat];
#pragma unroll
        for (int j = 0; j < kMaxBat; ++j) {
          bBP[j] = lpitch(bW[j] - 2 * kBl0);
          bBH[j] = bH[j] - 2 * kBl0;
          bNcg[j] = bBP[j] >> 2;
          const int nseg = g.bnseg[shp][min(j, NB - 1)];
          bSeg[j] = (bBH[j] + nseg - 1) / nseg;
          bItems[j] = j < NB ? bNcg[j] * nseg : 0;
          bBl[j] = U + g.bbl[shp][min(j, NB - 1)];
        }
        {
          const float k0 = g.gk[0], k1 = g.gk[1], k2 = g.gk[2], k3 = g.gk[3];
          const float k4 = g.gk[4], k5 = g.gk[5], k6 = g.gk[6];
          const int tot = bItems[0] + bItems[1] + bItems[2] + bItems[3];
          for (int item = t; item < tot; item += kOrbWG) {
            int loc = item;
            const int j = seg4(loc, NB, bItems[0], bItems[1], bItems[2]);
            const int ncg = pick4(j, bNcg), seg = pick4(j, bSeg), BH = pick4(j, bBH), BP = pick4(j, bBP);
            const uint8_t* I = pick4(j, bI);
            const int P = pick4(j, bP);
            uint8_t* Bl = pick4(j, bBl);
            const int sg = loc / ncg, cg = loc - sg * ncg;
            const int r0 = sg * seg, r1 = min(BH, r0 + seg);
            if (r0 >= r1) continue;
            const int c4 = 4 * cg, x = c4 + kBl0;
            auto rowf4 = [&](int y, float4& o) {
              const uint32_t* wp = reinterpret_cast<const uint32_t*>(I + y * P + x - 4);
              const uint32_t d0 = wp[0], d1 = wp[1], d2 = wp[2];
              const uint32_t q0 = __builtin_amdgcn_alignbyte(d1, d0, 1);
              const uint32_t q1 = __builtin_amdgcn_alignbyte(d2, d1, 1);
              const uint32_t q2 = d2 >> 8;
              float pq[10];
              pq[0] = (float)((q0 >> 0) & 0xFFu);
              pq[1] = (float)((q0 >> 8) & 0xFFu);
              pq[2] = (float)((q0 >> 16) & 0xFFu);
              pq[3] = (float)((q0 >> 24) & 0xFFu);
              pq[4] = (float)((q1 >> 0) & 0xFFu);
              pq[5] = (float)((q1 >> 8) & 0xFFu);
              pq[6] = (float)((q1 >> 16) & 0xFFu);
              pq[7] = (float)((q1 >> 24) & 0xFFu);
              pq[8] = (float)((q2 >> 0) & 0xFFu);
              pq[9] = (float)((q2 >> 8) & 0xFFu);
              float rr[4];
#pragma unroll
              for (int jj = 0; jj < 4; ++jj) {
                float acc = 0.f;
                acc = fmaf(pq[jj], k0, acc);
                acc = fmaf(pq[jj + 1], k1, acc);
                acc = fmaf(pq[jj + 2], k2, acc);
                acc = fmaf(pq[jj + 3], k3, acc);
                acc = fmaf(pq[jj + 4], k4, acc);
                acc = fmaf(pq[jj + 5], k5, acc);
                acc = fmaf(pq[jj + 6], k6, acc);
                rr[jj] = acc;
              }
              o = make_float4(rr[0], rr[1], rr[2], rr[3]);
            };
            const int yb = r0 + kBl0;
            float4 w[7];
            static_for<0, 7>([&](auto Iq) { rowf4(yb - 3 + decltype(Iq)::value, w[decltype(Iq)::value]); });
            typedef float f2 __attribute__((ext_vector_type(2)));
            const f2 kk3 = {k3, k3}, kk4 = {k4, k4}, kk5 = {k5, k5}, kk6 = {k6, k6};
            for (int r = r0; r < r1; r += 7) {
              static_for<0, 7>([&](auto K) {
                constexpr int k = decltype(K)::value;
                if (r + k < r1) {
                  const float4 a0 = w[k % 7], a1 = w[(k + 1) % 7], a2 = w[(k + 2) % 7];
                  const float4 a3 = w[(k + 3) % 7], a4 = w[(k + 4) % 7], a5 = w[(k + 5) % 7];
                  const float4 a6 = w[(k + 6) % 7];
                  auto col = [&](f2 x0_, f2 x1_, f2 x2_, f2 x3_, f2 x4_, f2 x5_, f2 x6_) {
                    f2 s0 = x3_ * kk3;
                    s0 = __builtin_elementwise_fma(x4_ + x2_, kk4, s0);
                    s0 = __builtin_elementwise_fma(x5_ + x1_, kk5, s0);
                    return __builtin_elementwise_fma(x6_ + x0_, kk6, s0);
                  };
                  const f2 lo = col(f2{a0.x, a0.y}, f2{a1.x, a1.y}, f2{a2.x, a2.y}, f2{a3.x, a3.y},
                                    f2{a4.x, a4.y}, f2{a5.x, a5.y}, f2{a6.x, a6.y});
                  const f2 hi = col(f2{a0.z, a0.w}, f2{a1.z, a1.w}, f2{a2.z, a2.w}, f2{a3.z, a3.w},
                                    f2{a4.z, a4.w}, f2{a5.z, a5.w}, f2{a6.z, a6.w});
                  uint32_t packed = __builtin_amdgcn_cvt_pk_u8_f32(rintf(lo.x), 0, 0u);
                  packed = __builtin_amdgcn_cvt_pk_u8_f32(rintf(lo.y), 1, packed);
                  packed = __builtin_amdgcn_cvt_pk_u8_f32(rintf(hi.x), 2, packed);
                  packed = __builtin_amdgcn_cvt_pk_u8_f32(rintf(hi.y), 3, packed);
                  *reinterpret_cast<uint32_t*>(Bl + (r + k) * BP + c4) = packed;
                  if (r + k + 1 < r1) rowf4(r + k + 1 + kBl0 + 3, w[k]);
                }
              });
            }
          }
        }
        __syncthreads();
        ORB_T(8);
        // ---- (10) rBRIEF of every kept keypoint (32 lanes per keypoint)
        {
          const int half = lane >> 5, byte = lane & 31;
          uint32_t pat[8];
#pragma unroll
          for (int bit = 0; bit < 8; ++bit)
            pat[bit] = reinterpret_cast<const uint32_t*>(c_pattern)[byte * 8 + bit];
          for (int k = 2 * wid + half; k < M; k += 2 * (kOrbWG / 64)) {
            int loc = k;
            const int j = seg4(loc, NB, bM[0], bM[1], bM[2]);
            const uint8_t* Bl = pick4(j, bBl);
            const int BP = pick4(j, bBP);
            const KP kp = L[k];
            const int cx = kp.x, cy = kp.y;
            const float a = kp.resp, bb = kp.angle;
            int val = 0;
#pragma unroll
            for (int bit = 0; bit < 8; ++bit) {
              uint32_t pw = pat[bit];
              __asm__ volatile("" : "+v"(pw));
              const float px1 = (float)(int8_t)(pw & 0xFFu), py1 = (float)(int8_t)((pw >> 8) & 0xFFu);
              const float px2 = (float)(int8_t)((pw >> 16) & 0xFFu), py2 = (float)(int8_t)(pw >> 24);
              const int ix1 = rne_f(px1 * a - py1 * bb), iy1 = rne_f(px1 * bb + py1 * a);
              const int ix2 = rne_f(px2 * a - py2 * bb), iy2 = rne_f(px2 * bb + py2 * a);
              const int t0 = Bl[(cy + iy1) * BP + cx + ix1];
              const int t1 = Bl[(cy + iy2) * BP + cx + ix2];
              val |= (t0 < t1 ? 1 : 0) << bit;
            }
            odesc[(size_t)(nout + k) * 32 + byte] = (uint8_t)val;
          }
        }
        nout += M;
        __syncthreads();
        ORB_T(9);
      }
    }
  }
  if (t == 0) ws_cnt[slot] = overflow ? -1 : nout;
}

// Concatenate the tiles of each image in orb.py order.
// One wave per (image, tile): the tile's offset is the sum of the counts of the
// tiles before it (every wave reads the image's counts, <= kMaxTiles), its
// keypoints, octaves and descriptors are copied to [off, off + n).  A negative
// tile count (retained ties overflowed the tile's slots) or a total above
// kp_cap marks the image with count = -total - 1 and copies nothing.  (One
// workgroup per image walking its tiles in turn was 36 dependent load/store
// rounds: 63 us per 65 images.)
__global__ __launch_bounds__(64) void k_orb_compact(const float* __restrict__ ws_kp,
                                                    const int32_t* __restrict__ ws_oct,
                                                    const uint8_t* __restrict__ ws_desc,
                                                    const int32_t* __restrict__ ws_cnt,
                                                    int n_tiles, int tcap, float* __restrict__ kp,
                                                    int32_t* __restrict__ oct,
                                                    uint8_t* __restrict__ desc,
                                                    int32_t* __restrict__ count, int kp_cap) {
  const int b = blockIdx.x, i = blockIdx.y, lane = threadIdx.x;
  const int32_t* cnt = ws_cnt + (size_t)b * n_tiles;
  int before = 0, total = 0, ovf = 0;
  for (int t0 = 0; t0 < n_tiles; t0 += 64) {
    const int tt = t0 + lane;
    const int c = tt < n_tiles ? cnt[tt] : 0;
    ovf |= c < 0 ? 1 : 0;
    const int cc = c < 0 ? 0 : c;
    total += cc;
    before += tt < i ? cc : 0;
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    total += __shfl_xor(total, o, 64);
    before += __shfl_xor(before, o, 64);
    ovf |= __shfl_xor(ovf, o, 64);
  }
  const bool bad = ovf != 0 || total > kp_cap;
  if (i == 0 && lane == 0) count[b] = bad ? -total - 1 : total;
  if (bad) return;
  const int n = cnt[i];
  const size_t src = ((size_t)b * n_tiles + i) * tcap;
  const size_t dst = (size_t)b * kp_cap + before;
  for (int j = lane; j < n * 5; j += 64) kp[dst * 5 + j] = ws_kp[src * 5 + j];
  for (int j = lane; j < n; j += 64) oct[dst + j] = ws_oct[src + j];
  for (int j = lane; j < n * 8; j += 64)
    reinterpret_cast<uint32_t*>(desc)[dst * 8 + j] =
        reinterpret_cast<const uint32_t*>(ws_desc)[src * 8 + j];
}

// ---------------------------------------------------------------- host side
int build_geom(int H, int W, int stride, int max_kp, int overlap_div, int height_div,
               int width_div, OrbGeom* g) {
  SLAM_REQUIRE(H > 0 && W > 0 && stride >= W, "slam_orb: bad image shape");
  SLAM_REQUIRE((overlap_div > 0 && height_div > 0 && width_div > 0) ||
                   (height_div == 0 && width_div == 0),
               "slam_orb: bad tiling");
  SLAM_REQUIRE(max_kp >= 0, "slam_orb: max_kp < 0");
  memset(g, 0, sizeof(*g));
  g->H = H;
  g->W = W;
  g->stride = stride;
  // orb.py:13-20 (Python int() truncation of positive floats)
  int nty = 0, ntx = 0, ph, pw;
  if (height_div == 0 && width_div == 0) {
    // whole image as one patch: orb_extraction_detect (orb.py:28-38)
    g->tile_h = H;
    g->tile_w = W;
    ph = H;
    pw = W;
    nty = ntx = 1;
  } else {
    g->tile_h = (int)((double)H / height_div);
    g->tile_w = (int)((double)W / width_div);
    SLAM_REQUIRE(g->tile_h > 0 && g->tile_w > 0, "slam_orb: image smaller than the tile grid");
    ph = (int)(g->tile_h + (double)g->tile_h / overlap_div);
    pw = (int)(g->tile_w + (double)g->tile_w / overlap_div);
    for (int y = 0; y < H - g->tile_h; y += g->tile_h) ++nty;
    for (int x = 0; x < W - g->tile_w; x += g->tile_w) ++ntx;
  }
  g->ntx = ntx;
  g->n_tiles = nty * ntx;
  SLAM_REQUIRE(g->n_tiles <= kMaxTiles, "slam_orb: %d tiles > %d", g->n_tiles, kMaxTiles);
  // levels: budget (float arithmetic of ORB_Impl) and scales
  const float factor = (float)(1.0 / 1.2);
  float d = (float)max_kp * (1 - factor) / (1 - (float)pow((double)factor, (double)kNLev));
  int sum = 0;
  for (int l = 0; l < kNLev - 1; ++l) {
    g->nl[l] = (int)nearbyintf(d);
    sum += g->nl[l];
    d *= factor;
  }
  g->nl[kNLev - 1] = max_kp - sum > 0 ? max_kp - sum : 0;
  for (int l = 0; l < kNLev; ++l) g->ls[l] = (float)pow(1.2, (double)l);
  {
    double t[7], s = 0;
    for (int i = 0; i < 7; ++i) {
      const double x = i - 3.0;
      t[i] = exp(-0.5 / (2.0 * 2.0) * x * x);
      g->gk[i] = (float)t[i];
      s += g->gk[i];
    }
    s = 1.0 / s;
    for (int i = 0; i < 7; ++i) g->gk[i] = (float)(g->gk[i] * s);
  }
  // shapes (edge tiles may be clipped by the image bounds, numpy slicing)
  int max_a = 0, max_b = 0, max_smap = 0, max_bl = 0, max_cand = 0;
  for (int ty = 0; ty < nty; ++ty)
    for (int tx = 0; tx < ntx; ++tx) {
      const int y0 = ty * g->tile_h, x0 = tx * g->tile_w;
      const int h = min(ph, H - y0), w = min(pw, W - x0);
      int s = 0;
      for (; s < g->nshapes; ++s)
        if (g->sw[s] == w && g->sh[s] == h) break;
      if (s == g->nshapes) {
        SLAM_REQUIRE(g->nshapes < kMaxShapes, "slam_orb: too many distinct patch shapes");
        SLAM_REQUIRE(w <= 4095 && h <= 2047 && (uint64_t)w * h * w < (1ull << 32),
                     "slam_orb: patch %dx%d too large", w, h);
        g->sw[s] = w;
        g->sh[s] = h;
        int last = -1;
        for (int l = 0; l < kNLev; ++l) {
          g->lw[s][l] = (int)nearbyintf((float)w / g->ls[l]);
          g->lh[s][l] = (int)nearbyintf((float)h / g->ls[l]);
          if (g->lw[s][l] > 2 * kEdge && g->lh[s][l] > 2 * kEdge && g->nl[l] > 0) last = l;
        }
        g->nlev[s] = last + 1;
        max_a = max(max_a, lpitch(w) * h);
        if (last >= 1) max_b = max(max_b, lpitch(g->lw[s][1]) * g->lh[s][1]);
        const int W0 = w, H0 = h;
        if (W0 > 2 * kEdge && H0 > 2 * kEdge) {
          const int cand = ((W0 - 2 * kEdge + 1) / 2) * ((H0 - 2 * kEdge + 1) / 2);
          const int smap = (((((W0 - 2 * kNMS0) + 3) & ~3) * (H0 - 2 * kNMS0)) + 15) & ~15;
          const int bl = lpitch(W0 - 2 * kBl0) * (H0 - 2 * kBl0);
          max_cand = max(max_cand, cand);
          max_smap = max(max_smap, smap);
          max_bl = max(max_bl, bl);
        }
        ++g->nshapes;
      }
      g->tile_shape[ty * ntx + tx] = (uint8_t)s;
    }
  auto al = [](int v) { return (v + 15) & ~15; };
  int nmax = 0;
  for (int l = 0; l < kNLev; ++l) nmax = max(nmax, g->nl[l]);
  g->cand_cap = max(max_cand, 1);
  g->list_cap = max(2 * nmax, nmax + 256);
  int max_w = 0, max_h = 0;
  for (int s = 0; s < g->nshapes; ++s) {
    max_w = max(max_w, g->sw[s]);
    max_h = max(max_h, g->sh[s]);
  }
  g->tab_x = (max_w + 3) & ~3;
  // U holds in turn the resize target (+ the resize tables past it), the FAST
  // score map (+ the survivor queues past it) and the blurred level; sized
  // so that a 720p tile (192x216 patch) needs <= 80 KiB and two ORB
  // workgroups share a CU.
  const int tabs = (g->tab_x + max_h) * 4;
  const int max_u = max(max(al(max_smap) + kFq, max_bl), al(max_b) + tabs);
  const int lists = al(g->list_cap * (int)sizeof(KP)) + al(g->list_cap * 8) + (256 + 16) * 4;
  g->glob = al(max_a) + al(max_u) + lists > 160 * 1024;
  if (g->glob) {
    // A patch (a whole image, orb_extraction_detect on a full frame) whose
    // level images do not fit LDS keeps them in two global ping-pong buffers
    // per image (L2-resident); the lists, queues and tables stay in LDS.
    SLAM_REQUIRE(g->n_tiles == 1, "slam_orb: %d patches of %dx%d do not fit LDS", g->n_tiles, pw, ph);
    g->lvl_bytes = (max(max_a, max_u) + 64 + 255) & ~255;
    g->lds_a = g->lds_u = 0;
    g->lds_fq = 0;
    g->lds_tab = kFq;
    g->lds_l = kFq + al(tabs);
  } else {
    g->lvl_bytes = 0;
    g->lds_a = 0;
    g->lds_u = al(max_a);
    g->lds_fq = g->lds_u + al(max_smap);
    g->lds_tab = g->lds_u + al(max_b);
    g->lds_l = g->lds_u + al(max_u);
  }
  g->lds_s = g->lds_l + al(g->list_cap * (int)sizeof(KP));
  g->lds_m = g->lds_s + al(g->list_cap * 8);
  g->lds_total = g->lds_m + (256 + 16) * 4;
  // the small-level group of each shape: the smallest first level whose
  // images (+ per-level histograms / counters) fit A, FAST maps fit U below
  // the queues, blurred images fit U, candidates fit the tile scratch
  // (tiled LDS variant only; SLAM_ORB_NOBATCH=1 turns it off for A/B)
  const char* nob = getenv("SLAM_ORB_NOBATCH");
  const bool batch_ok = !g->glob && g->n_tiles > 1 && !(nob != nullptr && nob[0] == '1');
  for (int s = 0; s < g->nshapes; ++s) {
    const int nl = g->nlev[s];
    g->bat0[s] = nl;
    if (!batch_ok) continue;
    for (int lb = max(1, nl - kMaxBat); lb <= nl - 2; ++lb) {
      const int NB = nl - lb;
      bool fit = true;
      int ao = 0, uo = 0, bo = 0, co = 0;
      long px_tot = 0;
      for (int j = 0; j < NB; ++j) {
        const int l = lb + j, W = g->lw[s][l], H = g->lh[s][l];
        fit = fit && W > 2 * kEdge && H > 2 * kEdge && g->nl[l] > 0;
        g->bslot[s][j] = ao;
        ao += al(lpitch(W) * H);
        g->bsmap[s][j] = uo;
        uo += al((((W - 2 * kNMS0) + 3) & ~3) * (H - 2 * kNMS0));
        g->bbl[s][j] = bo;
        bo += al(lpitch(W - 2 * kBl0) * (H - 2 * kBl0));
        g->bcand[s][j] = co;
        co += ((W - 2 * kEdge + 1) / 2) * ((H - 2 * kEdge + 1) / 2);
        px_tot += (long)lpitch(W - 2 * kBl0) * (H - 2 * kBl0);
      }
      g->bcand[s][NB] = co;
      g->bhist[s] = ao;
      ao += kMaxBat * (256 + 16) * 4;
      fit = fit && ao <= al(max_a) && uo <= al(max_smap) && bo <= max_u && co <= g->cand_cap;
      if (!fit) continue;
      for (int j = 0; j < NB; ++j) {  // blur threads in proportion to the level's pixels
        const int l = lb + j, W = g->lw[s][l], H = g->lh[s][l];
        const int BP = lpitch(W - 2 * kBl0), ncg = BP >> 2;
        const double share = (double)kOrbWG * BP * (H - 2 * kBl0) / (double)px_tot;
        g->bnseg[s][j] = max(1, (int)(share / ncg));
      }
      g->bat0[s] = lb;
      break;
    }
  }
  // slots per tile: the budget plus 64 for retainBest's boundary ties; a single
  // patch (orb_extraction_detect) gets room for a full tie list on every level
  g->tcap = g->n_tiles == 1 ? kNLev * g->list_cap : max_kp + 64;
  SLAM_REQUIRE(g->lds_total <= 160 * 1024,
               "slam_orb: patch %dx%d needs %d B of LDS (> 160 KiB)", pw, ph, g->lds_total);
  return SLAM_OK;
}

bool g_pattern_uploaded[64] = {false};
int g_orb_lds_floor = 0;  // slam_orb_set_lds_floor

// running minimum of the per-image keypoint counts (a negative count flags a
// workspace overflow): one lane per count, integer atomicMin (order-free)
__global__ __launch_bounds__(256) void k_count_min(const int32_t* __restrict__ count, int n,
                                                   int32_t* __restrict__ dmin) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) atomicMin(dmin, count[i]);
}

}  // namespace

#ifdef SLAM_ORB_PROFILE
// phases: 0 stage, 1 resize, 2 FAST map, 3 NMS, 4 retainBest(2n), 5 Harris,
// 6 rank + retainBest(n), 7 IC angle, 8 blur, 9 rBRIEF + write (cycles summed
// over workgroups); reads and clears the counters.
extern "C" int slam_orb_profile_read(unsigned long long* out96) {
  SLAM_HIP(hipDeviceSynchronize());
  SLAM_HIP(hipMemcpyFromSymbol(out96, HIP_SYMBOL(g_orb_prof), 96 * sizeof(unsigned long long)));
  unsigned long long z[96] = {};
  SLAM_HIP(hipMemcpyToSymbol(HIP_SYMBOL(g_orb_prof), z, sizeof(z)));
  return SLAM_OK;
}
#endif

extern "C" int slam_count_min(const int32_t* d_count, int n, int32_t* d_min, void* stream) {
  SLAM_REQUIRE(n >= 0, "slam_count_min: n < 0");
  if (n == 0) return SLAM_OK;
  SLAM_REQUIRE(d_count && d_min, "slam_count_min: null pointer");
  k_count_min<<<dim3((n + 255) / 256), dim3(256), 0, slam::as_stream(stream)>>>(d_count, n, d_min);
  SLAM_LAUNCHED("k_count_min");
  return SLAM_OK;
}

extern "C" int slam_orb_set_lds_floor(int bytes) {
  SLAM_REQUIRE(bytes >= 0 && bytes <= 160 * 1024, "slam_orb_set_lds_floor: %d B", bytes);
  g_orb_lds_floor = bytes;
  return SLAM_OK;
}

extern "C" int slam_orb_workspace_bytes(int batch, int H, int W, int max_kp, int overlap_div,
                                        int height_div, int width_div, size_t* bytes) {
  OrbGeom g;
  if (int rc = build_geom(H, W, W, max_kp, overlap_div, height_div, width_div, &g)) return rc;
  SLAM_REQUIRE(bytes != nullptr && batch >= 0, "slam_orb_workspace_bytes: bad args");
  const size_t slots = (size_t)batch * g.n_tiles * g.tcap;
  *bytes = slots * (5 * sizeof(float) + sizeof(int32_t) + 32) + (size_t)batch * g.n_tiles * 4 +
           256 + (size_t)batch * g.n_tiles * 3 * g.cand_cap * sizeof(uint32_t) + 256 +
           (size_t)batch * 2 * g.lvl_bytes;
  return SLAM_OK;
}

extern "C" int slam_orb_tiles(const uint8_t* d_img, int batch, int H, int W, int stride,
                              int max_kp, int overlap_div, int height_div, int width_div,
                              void* d_ws, size_t ws_bytes, float* d_kp, int32_t* d_octave,
                              uint8_t* d_desc, int32_t* d_count, int kp_cap, void* stream) {
  OrbGeom g;
  if (int rc = build_geom(H, W, stride, max_kp, overlap_div, height_div, width_div, &g)) return rc;
  SLAM_REQUIRE(batch >= 0 && kp_cap >= 0, "slam_orb_tiles: bad batch/kp_cap");
  if (batch == 0) return SLAM_OK;
  SLAM_REQUIRE(d_img && d_ws && d_kp && d_octave && d_desc && d_count,
               "slam_orb_tiles: null pointer");
  size_t need = 0;
  if (int rc = slam_orb_workspace_bytes(batch, H, W, max_kp, overlap_div, height_div, width_div,
                                        &need))
    return rc;
  if (ws_bytes < need) {
    slam::set_error("slam_orb_tiles: workspace %zu < %zu bytes", ws_bytes, need);
    return SLAM_ERR_WORKSPACE;
  }
  hipStream_t s = slam::as_stream(stream);
  int dev = 0;
  SLAM_HIP(hipGetDevice(&dev));
  if (dev < 64 && !g_pattern_uploaded[dev]) {
    SLAM_HIP(hipMemcpyToSymbol(HIP_SYMBOL(c_pattern), kOrbPattern, sizeof(kOrbPattern)));
    g_pattern_uploaded[dev] = true;
  }
  const size_t slots = (size_t)batch * g.n_tiles * g.tcap;
  uint8_t* base = static_cast<uint8_t*>(d_ws);
  float* ws_kp = reinterpret_cast<float*>(base);
  int32_t* ws_oct = reinterpret_cast<int32_t*>(base + slots * 5 * sizeof(float));
  uint8_t* ws_desc = base + slots * (5 * sizeof(float) + sizeof(int32_t));
  int32_t* ws_cnt = reinterpret_cast<int32_t*>(ws_desc + slots * 32);
  uint32_t* ws_cand = reinterpret_cast<uint32_t*>(
      (reinterpret_cast<uintptr_t>(ws_cnt + (size_t)batch * g.n_tiles) + 255) & ~(uintptr_t)255);
  uint8_t* ws_lvl = reinterpret_cast<uint8_t*>(
      (reinterpret_cast<uintptr_t>(ws_cand + (size_t)batch * g.n_tiles * 3 * g.cand_cap) + 255) &
      ~(uintptr_t)255);
  SLAM_REQUIRE(((uintptr_t)ws_cnt & 3) == 0, "slam_orb_tiles: workspace misaligned");
  auto kern = g.glob ? k_orb_tile<true> : k_orb_tile<false>;
  kern<<<dim3(g.n_tiles, batch), kOrbWG, max(g.lds_total, g_orb_lds_floor), s>>>(d_img, g, ws_kp, ws_oct,
                                                                  ws_desc, ws_cnt, ws_cand,
                                                                  ws_lvl);
  SLAM_LAUNCHED("k_orb_tile");
  k_orb_compact<<<dim3(batch, g.n_tiles), 64, 0, s>>>(ws_kp, ws_oct, ws_desc, ws_cnt, g.n_tiles,
                                                      g.tcap, d_kp, d_octave, d_desc, d_count,
                                                      kp_cap);
  SLAM_LAUNCHED("k_orb_compact");
  return SLAM_OK;
}
