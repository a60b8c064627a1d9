// Pose-chain (loop-closure) optimisation: the live `objective` of
// /root/reference/BundleAdjustment.py:79-145 and its solver (:173-183).
//
// Parameters: m relative poses, frame i = [r0 r1 r2 t0 t1 t2] (rotation vector,
// translation; translation_and_rotation_vector_to_matrix, transformation.py:
// 23-37, cv2.Rodrigues).  Residuals (m + 2):
//   f_i = |r0|.5 + |r1|.05 + |r2| + |t0| + |t1| + (|t2| - 1).0005   (:114-127)
//   abs_0 = I, abs_{k+1} = abs_k Rel_k                                  (:128-131)
//   L_t = 1000 sum_a |abs_0[a,3] - abs_m[a,3]|                          (:132)
//   L_R = 1000 sum_ab |100 abs_0[a,b] - 100 abs_m[a,b]|                 (:133)
// objective_without_loop_closure (:79-105) is the first m rows only.
//
// Kernels:
//   k_chain_objective  one lane per parameter vector, frames in order: the
//                      reference's sequential chain product and its sums in
//                      numpy's order; batched (a finite-difference Jacobian of
//                      the reference needs 6m + 1 evaluations, one launch here)
//   k_chain_trf        one workgroup runs scipy's TRF algorithm (least_squares
//                      method='trf', x_scale='jac', the reference's solver at
//                      :182) on the device with the 'exact' trust-region
//                      subproblem: per frame its relative pose and Rodrigues
//                      derivative, prefix and suffix chain products by
//                      workgroup scans of rigid transforms, the analytic
//                      (sign-subgradient) Jacobian instead of finite
//                      differences, and every SVD-based solve of the
//                      subproblem replaced by the m + 2 dual system
//                      (J_h J_h^T + alpha I) y = f, an arrow matrix (frame
//                      rows couple only through the two loop rows) solved
//                      through its 2x2 Schur complement in O(m).
//   k_chain_trf_r      the same algorithm with every per-frame quantity in the
//                      registers / LDS column of the thread owning the frame
//                      (m <= 512; round 5: 7.8 -> 2.4 ms per 500-keyframe
//                      solve); k_chain_trf serves larger chains and the
//                      SLAM_CHAIN_TRF=lds A/B.
#include "common.hpp"

#include <cmath>

namespace {

constexpr double kW[6] = {0.5, 0.05, 1.0, 1.0, 1.0, 0.0005};  // BundleAdjustment.py:114-119

// cv2.Rodrigues (cvRodrigues2, vector -> matrix): theta < DBL_EPSILON -> I,
// else c I + (1 - c) k k^T + s [k]x with k = r * (1 / theta)
__device__ __forceinline__ void rodrigues_cv(const double r[3], double R[9]) {
  const double th = sqrt(r[0] * r[0] + r[1] * r[1] + r[2] * r[2]);
  if (th < 2.220446049250313e-16) {
    for (int a = 0; a < 9; ++a) R[a] = (a % 4 == 0) ? 1.0 : 0.0;
    return;
  }
  const double c = cos(th), s = sin(th), c1 = 1.0 - c, it = 1.0 / th;
  const double k0 = r[0] * it, k1 = r[1] * it, k2 = r[2] * it;
  const double kk[3] = {k0, k1, k2};
  const double rx[9] = {0.0, -k2, k1, k2, 0.0, -k0, -k1, k0, 0.0};
  for (int a = 0; a < 3; ++a)
    for (int b = 0; b < 3; ++b) R[3 * a + b] = (c * (a == b ? 1.0 : 0.0) + c1 * (kk[a] * kk[b])) + s * rx[3 * a + b];
}

__device__ __forceinline__ double frame_cost(const double* p) {
  double c = fabs(p[0]) * kW[0];
  c += fabs(p[1]) * kW[1];
  c += fabs(p[2]) * kW[2];
  c += fabs(p[3]) * kW[3];
  c += fabs(p[4]) * kW[4];
  c += (fabs(p[5]) - 1.0) * kW[5];
  return c;
}

// rigid transform as 12 doubles: R row-major (9), t (3)
struct Rt {
  double R[9], t[3];
};

// a * b (4x4 homogeneous product, k = 0..3 in order; the bottom row of b is
// (0, 0, 0, 1), so its terms add exact zeros / the a[.][3] column once)
__device__ __forceinline__ Rt compose(const Rt& a, const Rt& b) {
  Rt o;
  for (int r = 0; r < 3; ++r) {
    for (int c = 0; c < 3; ++c)
      o.R[3 * r + c] = (a.R[3 * r] * b.R[c] + a.R[3 * r + 1] * b.R[3 + c]) + a.R[3 * r + 2] * b.R[6 + c];
    o.t[r] = ((a.R[3 * r] * b.t[0] + a.R[3 * r + 1] * b.t[1]) + a.R[3 * r + 2] * b.t[2]) + a.t[r];
  }
  return o;
}

__device__ __forceinline__ Rt identity_rt() {
  Rt o;
  for (int a = 0; a < 9; ++a) o.R[a] = (a % 4 == 0) ? 1.0 : 0.0;
  o.t[0] = o.t[1] = o.t[2] = 0.0;
  return o;
}

__device__ __forceinline__ Rt rel_of(const double* p) {
  Rt o;
  rodrigues_cv(p, o.R);
  o.t[0] = p[3];
  o.t[1] = p[4];
  o.t[2] = p[5];
  return o;
}

// loop residuals of the final absolute pose (numpy's summation order: three
// terms in sequence; nine terms as pairwise_sum's 8-way unroll + remainder)
__device__ __forceinline__ void loop_residuals(const Rt& T, double* Lt, double* LR) {
  *Lt = ((fabs(0.0 - T.t[0]) + fabs(0.0 - T.t[1])) + fabs(0.0 - T.t[2])) * 1000.0;
  double e[9];
  for (int a = 0; a < 9; ++a) e[a] = fabs(100.0 * ((a % 4 == 0) ? 1.0 : 0.0) - 100.0 * T.R[a]);
  *LR = ((((e[0] + e[1]) + (e[2] + e[3])) + ((e[4] + e[5]) + (e[6] + e[7]))) + e[8]) * 1000.0;
}

__global__ __launch_bounds__(64) void k_chain_objective(const double* __restrict__ params, int n_vec,
                                                        int m, int loop, double* __restrict__ resid) {
  const int v = blockIdx.x * 64 + threadIdx.x;
  if (v >= n_vec) return;
  const double* x = params + (size_t)v * 6 * m;
  const int nr = m + (loop ? 2 : 0);
  double* r = resid + (size_t)v * nr;
  Rt T = identity_rt();
  for (int i = 0; i < m; ++i) {
    const double* p = x + 6 * i;
    r[i] = frame_cost(p);
    if (loop) T = compose(T, rel_of(p));
  }
  if (loop) loop_residuals(T, r + m, r + m + 1);
}

// ------------------------------------------------------------------ TRF
constexpr int kLmWG = 1024;
constexpr int kRed = kLmWG / 64;

// workspace layout (doubles), per frame unless noted
struct ChainWs {
  long long x, xt, rel, dR, pre, suf, g, h, r, sinv, fr, y, z, tot;
  __host__ __device__ explicit ChainWs(int m) {
    x = 0;                 // [6m] live parameters
    xt = x + 6ll * m;      // [6m] trial parameters
    rel = xt + 6ll * m;    // [12m] Rel_i
    dR = rel + 12ll * m;   // [27m] dR/dr_k (k = 0..2, 3x3 row-major)
    pre = dR + 27ll * m;   // [12m] P_i = Rel_0 .. Rel_{i-1}
    suf = pre + 12ll * m;  // [12m] S_i = Rel_{i+1} .. Rel_{m-1}
    g = suf + 12ll * m;    // [6m] d f_i / d x_i
    h = g + 6ll * m;       // [12m] d L_t / d x_i (6), d L_R / d x_i (6)
    r = h + 12ll * m;      // [m] frame residuals at x
    sinv = r + m;          // [6m] x_scale='jac': max over iterations of the column norms
    fr = sinv + 6ll * m;   // [4m] d0 = |gs|^2, b1 = gs.hs1, b2 = gs.hs2 (scaled rows), pad
    y = fr + 4ll * m;      // [m] dual solution (K + alpha I)^-1 f
    z = y + m;             // [m] (K + alpha I)^-1 y
    tot = z + m;
  }
};

__device__ __forceinline__ void st_rt(double* o, const Rt& a) {
  for (int k = 0; k < 9; ++k) o[k] = a.R[k];
  for (int k = 0; k < 3; ++k) o[9 + k] = a.t[k];
}
__device__ __forceinline__ Rt ld_rt(const double* o) {
  Rt a;
  for (int k = 0; k < 9; ++k) a.R[k] = o[k];
  for (int k = 0; k < 3; ++k) a.t[k] = o[9 + k];
  return a;
}

// dR/dr_k of the Rodrigues map (Gallego & Yezzi 2015):
//   theta > 0: (r_k [r]x + [r x (I - R) e_k]x) R / theta^2;  theta = 0: [e_k]x
__device__ void rodrigues_jac(const double r[3], const double R[9], double* dR) {
  const double th2 = r[0] * r[0] + r[1] * r[1] + r[2] * r[2];
  for (int k = 0; k < 3; ++k) {
    const double e0 = k == 0 ? 1.0 : 0.0, e1 = k == 1 ? 1.0 : 0.0, e2 = k == 2 ? 1.0 : 0.0;
    if (th2 < 1e-30) {
      dR[9 * k + 0] = 0.0; dR[9 * k + 1] = -e2; dR[9 * k + 2] = e1;
      dR[9 * k + 3] = e2;  dR[9 * k + 4] = 0.0; dR[9 * k + 5] = -e0;
      dR[9 * k + 6] = -e1; dR[9 * k + 7] = e0;  dR[9 * k + 8] = 0.0;
      continue;
    }
    const double u0 = e0 - R[k], u1 = e1 - R[3 + k], u2 = e2 - R[6 + k];  // (I - R) e_k
    const double v0 = r[1] * u2 - r[2] * u1, v1 = r[2] * u0 - r[0] * u2, v2 = r[0] * u1 - r[1] * u0;
    const double a0 = r[k] * r[0] + v0, a1 = r[k] * r[1] + v1, a2 = r[k] * r[2] + v2;
    // [a]x R / theta^2
    for (int j = 0; j < 3; ++j) {
      dR[9 * k + j] = (-a2 * R[3 + j] + a1 * R[6 + j]) / th2;
      dR[9 * k + 3 + j] = (a2 * R[j] - a0 * R[6 + j]) / th2;
      dR[9 * k + 6 + j] = (-a1 * R[j] + a0 * R[3 + j]) / th2;
    }
  }
}

// dR/dr_k alone (rodrigues_jac's k-th 3x3, the same operations)
__device__ __forceinline__ void rodrigues_jac_k(const double r[3], const double R[9], int k, double* D) {
  const double th2 = r[0] * r[0] + r[1] * r[1] + r[2] * r[2];
  const double e0 = k == 0 ? 1.0 : 0.0, e1 = k == 1 ? 1.0 : 0.0, e2 = k == 2 ? 1.0 : 0.0;
  if (th2 < 1e-30) {
    D[0] = 0.0; D[1] = -e2; D[2] = e1;
    D[3] = e2;  D[4] = 0.0; D[5] = -e0;
    D[6] = -e1; D[7] = e0;  D[8] = 0.0;
    return;
  }
  const double rk = k == 0 ? r[0] : (k == 1 ? r[1] : r[2]);
  const double Rk0 = k == 0 ? R[0] : (k == 1 ? R[1] : R[2]);
  const double Rk1 = k == 0 ? R[3] : (k == 1 ? R[4] : R[5]);
  const double Rk2 = k == 0 ? R[6] : (k == 1 ? R[7] : R[8]);
  const double u0 = e0 - Rk0, u1 = e1 - Rk1, u2 = e2 - Rk2;  // (I - R) e_k
  const double v0 = r[1] * u2 - r[2] * u1, v1 = r[2] * u0 - r[0] * u2, v2 = r[0] * u1 - r[1] * u0;
  const double a0 = rk * r[0] + v0, a1 = rk * r[1] + v1, a2 = rk * r[2] + v2;
  for (int j = 0; j < 3; ++j) {
    D[j] = (-a2 * R[3 + j] + a1 * R[6 + j]) / th2;
    D[3 + j] = (a2 * R[j] - a0 * R[6 + j]) / th2;
    D[6 + j] = (-a1 * R[j] + a0 * R[3 + j]) / th2;
  }
}

// deterministic workgroup sums of N values (fixed shuffle tree, then the
// waves in order); the result is on every thread
template <int N>
__device__ void wg_sum(double (&v)[N], double* red) {
  for (int q = 0; q < N; ++q)
    for (int off = 32; off > 0; off >>= 1) v[q] += __shfl_down(v[q], off, 64);
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  __syncthreads();
  if (lane == 0)
    for (int q = 0; q < N; ++q) red[q * kRed + wid] = v[q];
  __syncthreads();
  for (int q = 0; q < N; ++q) {
    double s = 0.0;
    for (int w = 0; w < kRed; ++w) s += red[q * kRed + w];
    v[q] = s;
  }
}

__device__ double wg_max(double v, double* red) {
  for (int off = 32; off > 0; off >>= 1) v = fmax(v, __shfl_down(v, off, 64));
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  __syncthreads();
  if (lane == 0) red[wid] = v;
  __syncthreads();
  double s = 0.0;
  for (int w = 0; w < kRed; ++w) s = fmax(s, red[w]);
  return s;
}

// Inclusive workgroup scan of rigid transforms in LDS (Hillis-Steele), forward
// (prefix products left to right) or backward (suffix products right to left).
__device__ void wg_scan(Rt mine, double* buf, bool forward) {
  const int t = threadIdx.x;
  __syncthreads();
  st_rt(buf + 12 * t, mine);
  __syncthreads();
  for (int d = 1; d < kLmWG; d <<= 1) {
    Rt v = ld_rt(buf + 12 * t);
    const int o = forward ? t - d : t + d;
    if (forward ? o >= 0 : o < kLmWG) v = forward ? compose(ld_rt(buf + 12 * o), v) : compose(v, ld_rt(buf + 12 * o));
    __syncthreads();
    st_rt(buf + 12 * t, v);
    __syncthreads();
  }
}

struct Seg {
  int i0, i1;
  __device__ Seg(int m) {
    const int seg = (m + kLmWG - 1) / kLmWG;
    i0 = min(m, (int)threadIdx.x * seg);
    i1 = min(m, i0 + seg);
  }
};

// Residuals at x: frame residuals (into ws.r when jac), the two loop residuals
// (fl, every thread); returns the cost 0.5 |f|^2 on every thread.  jac: also
// relative poses, Rodrigues derivatives, prefix / suffix products and the
// Jacobian rows g (frame) and h (loop).
__device__ double evaluate(const double* __restrict__ x, double* __restrict__ ws, const ChainWs& W,
                           int m, int loop, bool jac, double* red, double* buf, double fl[2]) {
  const int t = threadIdx.x;
  const Seg sg(m);
  double c2[1] = {0.0};
  Rt loc = identity_rt();
  for (int i = sg.i0; i < sg.i1; ++i) {
    const double* p = x + 6 * i;
    const double f = frame_cost(p);
    c2[0] += f * f;
    const Rt Rl = rel_of(p);
    if (jac) {
      ws[W.r + i] = f;
      st_rt(ws + W.rel + 12 * i, Rl);
      rodrigues_jac(p, Rl.R, ws + W.dR + 27 * i);
      for (int k = 0; k < 6; ++k) {
        const double s = p[k] > 0.0 ? 1.0 : (p[k] < 0.0 ? -1.0 : 0.0);
        ws[W.g + 6 * i + k] = kW[k] * s;
        ws[W.h + 12 * i + k] = 0.0;
        ws[W.h + 12 * i + 6 + k] = 0.0;
      }
    }
    if (loop) loc = compose(loc, Rl);
  }
  wg_sum<1>(c2, red);
  fl[0] = fl[1] = 0.0;
  if (!loop) return 0.5 * c2[0];
  wg_scan(loc, buf, true);
  const Rt T = ld_rt(buf + 12 * (kLmWG - 1));  // the whole chain
  loop_residuals(T, &fl[0], &fl[1]);
  const double cost = 0.5 * (c2[0] + (fl[0] * fl[0] + fl[1] * fl[1]));
  if (!jac) return cost;
  Rt P = t > 0 ? ld_rt(buf + 12 * (t - 1)) : identity_rt();  // exclusive prefix of the segment
  for (int i = sg.i0; i < sg.i1; ++i) {
    st_rt(ws + W.pre + 12 * i, P);
    P = compose(P, ld_rt(ws + W.rel + 12 * i));
  }
  wg_scan(loc, buf, false);
  Rt S = t + 1 < kLmWG ? ld_rt(buf + 12 * (t + 1)) : identity_rt();
  for (int i = sg.i1 - 1; i >= sg.i0; --i) {
    st_rt(ws + W.suf + 12 * i, S);
    S = compose(ld_rt(ws + W.rel + 12 * i), S);
  }
  // loop rows: d|t_end| = sign(t_end), d|100 I - 100 R_end| = 100 sign(R_end - I)
  double E1[3], E2[9];
  for (int a = 0; a < 3; ++a) E1[a] = T.t[a] > 0.0 ? 1.0 : (T.t[a] < 0.0 ? -1.0 : 0.0);
  for (int a = 0; a < 9; ++a) {
    const double dv = T.R[a] - ((a % 4 == 0) ? 1.0 : 0.0);
    E2[a] = dv > 0.0 ? 1.0 : (dv < 0.0 ? -1.0 : 0.0);
  }
  for (int i = sg.i0; i < sg.i1; ++i) {
    // T_end = P_i Rel_i S_i:  d/dt_k -> Rp e_k;  d/dr_k -> (Rp dR_k Rs, Rp dR_k ts)
    const Rt Pi = ld_rt(ws + W.pre + 12 * i), Si = ld_rt(ws + W.suf + 12 * i);
    const double* dR = ws + W.dR + 27 * i;
    double u[3], PE[9], G[9];  // u = Rp^T E1, G = Rp^T E2 Rs^T
    for (int a = 0; a < 3; ++a) u[a] = Pi.R[a] * E1[0] + Pi.R[3 + a] * E1[1] + Pi.R[6 + a] * E1[2];
    for (int a = 0; a < 3; ++a)
      for (int b = 0; b < 3; ++b) PE[3 * a + b] = Pi.R[a] * E2[b] + Pi.R[3 + a] * E2[3 + b] + Pi.R[6 + a] * E2[6 + b];
    for (int a = 0; a < 3; ++a)
      for (int b = 0; b < 3; ++b)
        G[3 * a + b] = PE[3 * a] * Si.R[3 * b] + PE[3 * a + 1] * Si.R[3 * b + 1] + PE[3 * a + 2] * Si.R[3 * b + 2];
    double* h = ws + W.h + 12 * i;
    for (int k = 0; k < 3; ++k) {
      const double* D = dR + 9 * k;
      double s1 = 0.0, s2 = 0.0;
      for (int a = 0; a < 3; ++a) s1 += u[a] * (D[3 * a] * Si.t[0] + D[3 * a + 1] * Si.t[1] + D[3 * a + 2] * Si.t[2]);
      for (int a = 0; a < 9; ++a) s2 += G[a] * D[a];
      h[k] = 1000.0 * s1;
      h[3 + k] = 1000.0 * u[k];
      h[6 + k] = 1e5 * s2;
      h[9 + k] = 0.0;
    }
  }
  __syncthreads();
  return cost;
}

// Arrow solve of (K + alpha I) out = rhs, K = J_h J_h^T: frame rows i couple only
// through the two loop rows.  rhs_f / out_f are per-frame arrays in ws (may
// alias), rhs_l / out_l the loop entries.  Scaled-row data: ws.fr (d0, b1, b2)
// per frame, E (|hs1|^2, hs1.hs2, |hs2|^2) global.
__device__ void arrow_solve(double* ws, const ChainWs& W, int m, int loop, double alpha, const double* E,
                            const double* rhs_f, const double rhs_l[2], double* out_f, double out_l[2],
                            double* red) {
  const Seg sg(m);
  out_l[0] = out_l[1] = 0.0;
  if (loop) {
    double s[5] = {0.0, 0.0, 0.0, 0.0, 0.0};  // S11 S12 S22 Q1 Q2
    for (int i = sg.i0; i < sg.i1; ++i) {
      const double* fr = ws + W.fr + 4 * i;
      const double da = fr[0] + alpha, b1 = fr[1], b2 = fr[2], ri = rhs_f[i];
      s[0] += b1 * b1 / da;
      s[1] += b1 * b2 / da;
      s[2] += b2 * b2 / da;
      s[3] += b1 * ri / da;
      s[4] += b2 * ri / da;
    }
    wg_sum<5>(s, red);
    const double a = E[0] + alpha - s[0], b = E[1] - s[1], c = E[2] + alpha - s[2];
    const double r1 = rhs_l[0] - s[3], r2 = rhs_l[1] - s[4];
    const double det = a * c - b * b;
    out_l[0] = (c * r1 - b * r2) / det;
    out_l[1] = (a * r2 - b * r1) / det;
  }
  __syncthreads();  // every thread has read rhs_f before out_f (may alias) is written
  for (int i = sg.i0; i < sg.i1; ++i) {
    const double* fr = ws + W.fr + 4 * i;
    out_f[i] = (rhs_f[i] - fr[1] * out_l[0] - fr[2] * out_l[1]) / (fr[0] + alpha);
  }
  __syncthreads();
}

// state[16]: 0 cost0, 1 cost, 2 nfev, 3 njev, 4 status (0 running / max_nfev,
// 1 gtol, 2 ftol, 3 xtol, 4 ftol+xtol), 5 Delta, 6 alpha, 7 iterations,
// 8.. per-call scratch.  Resumable: state[5], state[6] and ws.sinv carry over
// when first == 0 (the host loops over calls of n_iter iterations).
__global__ __launch_bounds__(kLmWG) void k_chain_trf(double* __restrict__ ws, int m, int loop,
                                                     int max_iter, int first, double ftol, double xtol,
                                                     double gtol, int max_nfev,
                                                     double* __restrict__ state) {
  const ChainWs W(m);
  __shared__ double red[5 * kRed];
  __shared__ double buf[12 * kLmWG];
  const Seg sg(m);
  double* x = ws + W.x;
  double* xt = ws + W.xt;
  double fl[2], flt[2];
  double cost = evaluate(x, ws, W, m, loop, true, red, buf, fl);
  int nfev = first ? 1 : (int)state[2], njev = first ? 1 : (int)state[3];
  // scale_inv = column norms (max over iterations; zero columns -> 1 at the start)
  auto update_scale = [&](bool init) {
    for (int i = sg.i0; i < sg.i1; ++i)
      for (int k = 0; k < 6; ++k) {
        const double gk = ws[W.g + 6 * i + k], h1 = ws[W.h + 12 * i + k], h2 = ws[W.h + 12 * i + 6 + k];
        double cn = sqrt((gk * gk + h1 * h1) + h2 * h2);
        double* si = ws + W.sinv + 6 * i + k;
        if (init) {
          *si = cn == 0.0 ? 1.0 : cn;
        } else {
          *si = fmax(*si, cn);
        }
      }
  };
  double Delta, alpha;
  if (first) {
    update_scale(true);
    double v[1] = {0.0};  // Delta = |x0 * scale_inv|
    for (int i = sg.i0; i < sg.i1; ++i)
      for (int k = 0; k < 6; ++k) {
        const double a = x[6 * i + k] * ws[W.sinv + 6 * i + k];
        v[0] += a * a;
      }
    wg_sum<1>(v, red);
    Delta = sqrt(v[0]);
    if (Delta == 0.0) Delta = 1.0;
    alpha = 0.0;
    if (threadIdx.x == 0) state[0] = cost;
  } else {
    Delta = state[5];
    alpha = state[6];
  }
  int status = 0, it = 0;
  for (; it < max_iter; ++it) {
    // g = J^T f (unscaled); gtol on its inf-norm
    double gmax = 0.0;
    for (int i = sg.i0; i < sg.i1; ++i)
      for (int k = 0; k < 6; ++k) {
        const double gk = ws[W.g + 6 * i + k] * ws[W.r + i] + ws[W.h + 12 * i + k] * fl[0] +
                          ws[W.h + 12 * i + 6 + k] * fl[1];
        gmax = fmax(gmax, fabs(gk));
      }
    gmax = wg_max(gmax, red);
    if (gmax < gtol) status = 1;
    if (status != 0 || nfev >= max_nfev) break;
    // scaled rows: gs = g / sinv, hs = h / sinv; frame data d0, b1, b2 and E
    double e[5] = {0.0, 0.0, 0.0, 0.0, 0.0};  // |hs1|^2 hs1.hs2 |hs2|^2 |g_h|^2
    for (int i = sg.i0; i < sg.i1; ++i) {
      double d0 = 0.0, b1 = 0.0, b2 = 0.0;
      for (int k = 0; k < 6; ++k) {
        const double s = 1.0 / ws[W.sinv + 6 * i + k];
        const double gs = ws[W.g + 6 * i + k] * s, h1 = ws[W.h + 12 * i + k] * s,
                     h2 = ws[W.h + 12 * i + 6 + k] * s;
        d0 += gs * gs;
        b1 += gs * h1;
        b2 += gs * h2;
        e[0] += h1 * h1;
        e[1] += h1 * h2;
        e[2] += h2 * h2;
        const double gh = gs * ws[W.r + i] + h1 * fl[0] + h2 * fl[1];
        e[3] += gh * gh;
      }
      ws[W.fr + 4 * i] = d0;
      ws[W.fr + 4 * i + 1] = b1;
      ws[W.fr + 4 * i + 2] = b2;
    }
    wg_sum<5>(e, red);
    const double E[3] = {e[0], e[1], e[2]};
    const double suf_norm = sqrt(e[3]);  // |J_h^T f|
    double actual = -1.0, cost_new = cost, step_norm = 0.0;
    bool accepted = false;
    while (actual <= 0.0 && nfev < max_nfev) {
      // ---- solve_lsq_trust_region (J rank-deficient: m + 2 < 6m): alpha with |p(alpha)| = Delta
      double aup = suf_norm / Delta, alow = 0.0;
      if (alpha == 0.0) alpha = fmax(0.001 * aup, sqrt(alow * aup));
      double yl[2], pn = 0.0;
      for (int k = 0; k < 10; ++k) {
        if (alpha < alow || alpha > aup) alpha = fmax(0.001 * aup, sqrt(alow * aup));
        // y = (K + a)^-1 f, z = (K + a)^-1 y; |p|^2 = y^T K y = f.y - a y.y;
        // sum suf^2 / (s^2 + a)^3 = (f - a y).z
        arrow_solve(ws, W, m, loop, alpha, E, ws + W.r, fl, ws + W.y, yl, red);
        double zl[2];
        arrow_solve(ws, W, m, loop, alpha, E, ws + W.y, yl, ws + W.z, zl, red);
        double q[3] = {0.0, 0.0, 0.0};  // f.y, y.y, (f - a y).z
        for (int i = sg.i0; i < sg.i1; ++i) {
          const double fi = ws[W.r + i], yi = ws[W.y + i];
          q[0] += fi * yi;
          q[1] += yi * yi;
          q[2] += (fi - alpha * yi) * ws[W.z + i];
        }
        wg_sum<3>(q, red);
        q[0] += fl[0] * yl[0] + fl[1] * yl[1];
        q[1] += yl[0] * yl[0] + yl[1] * yl[1];
        q[2] += (fl[0] - alpha * yl[0]) * zl[0] + (fl[1] - alpha * yl[1]) * zl[1];
        pn = sqrt(fmax(q[0] - alpha * q[1], 0.0));
        const double phi = pn - Delta, dphi = -q[2] / pn;
        if (phi < 0.0) aup = alpha;
        const double ratio = phi / dphi;
        alow = fmax(alow, alpha - ratio);
        alpha -= (phi + Delta) * ratio / Delta;
        if (fabs(phi) < 0.01 * Delta) break;
      }
      // the step at the final alpha, rescaled to |p| = Delta:
      // p = -(Delta / |p(alpha)|) J_h^T y, y = (K + alpha)^-1 f;  step = p / sinv
      {
        arrow_solve(ws, W, m, loop, alpha, E, ws + W.r, fl, ws + W.y, yl, red);
        double q[2] = {0.0, 0.0};
        for (int i = sg.i0; i < sg.i1; ++i) {
          const double yi = ws[W.y + i];
          q[0] += ws[W.r + i] * yi;
          q[1] += yi * yi;
        }
        wg_sum<2>(q, red);
        q[0] += fl[0] * yl[0] + fl[1] * yl[1];
        q[1] += yl[0] * yl[0] + yl[1] * yl[1];
        pn = sqrt(fmax(q[0] - alpha * q[1], 0.0));
      }
      const double c = Delta / pn;
      double pr[3] = {0.0, 0.0, 0.0};  // |x|^2, |step|^2 (unscaled), K y . f pieces
      for (int i = sg.i0; i < sg.i1; ++i) {
        const double yi = ws[W.y + i];
        for (int k = 0; k < 6; ++k) {
          const double si = ws[W.sinv + 6 * i + k];
          const double gs = ws[W.g + 6 * i + k] / si, h1 = ws[W.h + 12 * i + k] / si,
                       h2 = ws[W.h + 12 * i + 6 + k] / si;
          const double ph = -c * ((gs * yi + h1 * yl[0]) + h2 * yl[1]);
          const double st = ph / si;
          xt[6 * i + k] = x[6 * i + k] + st;
          pr[0] += x[6 * i + k] * x[6 * i + k];
          pr[1] += st * st;
        }
      }
      // J_h p per row: frame i: gs_i . p_i;  loop rows: hs_a . p  (accumulated with p)
      double jp[3] = {0.0, 0.0, 0.0};  // sum_i (gs_i.p_i)^2 + 2 f_i (gs_i.p_i), hs1.p, hs2.p
      for (int i = sg.i0; i < sg.i1; ++i) {
        const double yi = ws[W.y + i];
        double gp = 0.0;
        for (int k = 0; k < 6; ++k) {
          const double si = ws[W.sinv + 6 * i + k];
          const double gs = ws[W.g + 6 * i + k] / si, h1 = ws[W.h + 12 * i + k] / si,
                       h2 = ws[W.h + 12 * i + 6 + k] / si;
          const double ph = -c * ((gs * yi + h1 * yl[0]) + h2 * yl[1]);
          gp += gs * ph;
          jp[1] += h1 * ph;
          jp[2] += h2 * ph;
        }
        jp[0] += gp * (0.5 * gp + ws[W.r + i]);
      }
      wg_sum<3>(jp, red);
      wg_sum<3>(pr, red);
      const double quad = jp[0] + (jp[1] * (0.5 * jp[1] + fl[0]) + jp[2] * (0.5 * jp[2] + fl[1]));
      const double predicted = -quad;
      cost_new = evaluate(xt, ws, W, m, loop, false, red, buf, flt);
      ++nfev;
      const double step_h_norm = Delta;  // |p| = Delta after the rescale
      if (!isfinite(cost_new)) {
        Delta = 0.25 * step_h_norm;
        continue;
      }
      actual = cost - cost_new;
      // update_tr_radius
      double ratio;
      if (predicted > 0.0) ratio = actual / predicted;
      else if (predicted == actual) ratio = 1.0;  // both zero
      else ratio = 0.0;
      double Dn = Delta;
      if (ratio < 0.25) Dn = 0.25 * step_h_norm;
      else if (ratio > 0.75 && step_h_norm > 0.95 * Delta) Dn = 2.0 * Delta;
      step_norm = sqrt(pr[1]);
      // check_termination
      const bool ftol_ok = actual < ftol * cost && ratio > 0.25;
      const bool xtol_ok = step_norm < xtol * (xtol + sqrt(pr[0]));
      if (ftol_ok || xtol_ok) {
        status = ftol_ok && xtol_ok ? 4 : (ftol_ok ? 2 : 3);
        break;
      }
      alpha *= Delta / Dn;
      Delta = Dn;
    }
    if (actual > 0.0) {
      accepted = true;
      __syncthreads();
      for (int i = sg.i0; i < sg.i1; ++i)
        for (int k = 0; k < 6; ++k) x[6 * i + k] = xt[6 * i + k];
      cost = evaluate(x, ws, W, m, loop, true, red, buf, fl);
      ++njev;
      update_scale(false);
      __syncthreads();
    }
    (void)accepted;
    if (status != 0) {
      ++it;
      break;
    }
  }
  if (threadIdx.x == 0) {
    state[1] = cost;
    state[2] = nfev;
    state[3] = njev;
    state[4] = status;
    state[5] = Delta;
    state[6] = alpha;
    state[7] = (first ? 0.0 : state[7]) + it;
  }
}

// ------------------------------------------------------------------ TRF, register-resident
// k_chain_trf_r<F>: k_chain_trf's algorithm (the same scipy-TRF steps, tests and
// trust-radius rules) with every per-frame quantity in the registers of the
// thread that owns the frame (frames F t .. F t + F - 1 of thread t, kRW
// threads), so no pass over the frames touches global memory:
//   * reductions: a wave shuffle tree, one LDS partial per wave, ONE workgroup
//     barrier (the partial buffers alternate, so the next reduction's stores
//     cannot overtake this one's loads); every thread sums the 8 partials in
//     the same order, so every thread holds the same bits;
//   * chain products: wave shuffle scans of rigid transforms (Hillis-Steele
//     over the 64 lanes) and the 8 wave totals through LDS -- the prefix
//     P_i, the suffix S_i and the whole chain T, as k_chain_trf's LDS scans;
//   * the 'exact' subproblem's alpha iteration in TWO reductions per step:
//     the first arrow solve y = (K + a)^-1 f as before; the second one's
//     result z = (K + a)^-1 y enters only through (f - a y).z, which is
//       sum_i w_i y_i / d_i - zl_0 sum_i w_i b1_i / d_i - zl_1 sum_i w_i b2_i / d_i
//       + (fl - a yl).zl        (w = f - a y, d_i = d0_i + a)
//     so z is never formed and its sums ride on the reduction that also
//     gives f.y and y.y; the final step's c = Delta / |p| enters the step
//     and the predicted reduction linearly or quadratically, so their sums
//     are taken before c is known, in the same reduction as |p|'s.
// The sums run in another order than k_chain_trf's (rounding at 1e-16
// relative); the iterates still follow scipy's TRF to the tests' 1e-7.
constexpr int kRW = 512;
constexpr int kRWv = kRW / 64;
constexpr int kRMax = 8;

template <int N>
__device__ __forceinline__ void rsum(double (&v)[N], double* red, int& ph) {
  static_assert(N <= kRMax, "rsum: too many values");
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
#pragma unroll
  for (int q = 0; q < N; ++q)
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) v[q] += __shfl_down(v[q], off, 64);
  double* b = red + ph * (kRMax * kRWv);
  if (lane == 0) {
#pragma unroll
    for (int q = 0; q < N; ++q) b[q * kRWv + wid] = v[q];
  }
  __syncthreads();
#pragma unroll
  for (int q = 0; q < N; ++q) {
    double s = b[q * kRWv];
#pragma unroll
    for (int w = 1; w < kRWv; ++w) s += b[q * kRWv + w];
    v[q] = s;
  }
  ph ^= 1;
}

__device__ __forceinline__ double rmax(double v, double* red, int& ph) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v = fmax(v, __shfl_down(v, off, 64));
  double* b = red + ph * (kRMax * kRWv);
  if (lane == 0) b[wid] = v;
  __syncthreads();
  double s = b[0];
#pragma unroll
  for (int w = 1; w < kRWv; ++w) s = fmax(s, b[w]);
  ph ^= 1;
  return s;
}

__device__ __forceinline__ Rt shfl_up_rt(const Rt& a, int d) {
  Rt o;
#pragma unroll
  for (int k = 0; k < 9; ++k) o.R[k] = __shfl_up(a.R[k], d, 64);
#pragma unroll
  for (int k = 0; k < 3; ++k) o.t[k] = __shfl_up(a.t[k], d, 64);
  return o;
}
__device__ __forceinline__ Rt shfl_down_rt(const Rt& a, int d) {
  Rt o;
#pragma unroll
  for (int k = 0; k < 9; ++k) o.R[k] = __shfl_down(a.R[k], d, 64);
#pragma unroll
  for (int k = 0; k < 3; ++k) o.t[k] = __shfl_down(a.t[k], d, 64);
  return o;
}

// exclusive prefix product of the threads' chains (thread order) and the whole
// chain T; wb: 12 kRWv doubles of LDS (one barrier inside)
__device__ void chain_scan_fwd(const Rt& loc, double* wb, Rt& excl, Rt& tot) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  Rt v = loc;
#pragma unroll 1
  for (int d = 1; d < 64; d <<= 1) {
    const Rt o = shfl_up_rt(v, d);
    if (lane >= d) v = compose(o, v);
  }
  const Rt prev = shfl_up_rt(v, 1);
  if (lane == 63) st_rt(wb + 12 * wid, v);
  __syncthreads();
  Rt Wp = identity_rt();
  if (wid > 0) {
    Wp = ld_rt(wb);
    for (int w = 1; w < wid; ++w) Wp = compose(Wp, ld_rt(wb + 12 * w));
  }
  tot = wid > 0 ? Wp : ld_rt(wb);
  for (int w = wid > 0 ? wid : 1; w < kRWv; ++w) tot = compose(tot, ld_rt(wb + 12 * w));
  excl = lane > 0 ? (wid > 0 ? compose(Wp, prev) : prev) : Wp;
}

// exclusive suffix product of the threads' chains (one barrier inside)
__device__ void chain_scan_bwd(const Rt& loc, double* wb, Rt& excl) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  Rt v = loc;
#pragma unroll 1
  for (int d = 1; d < 64; d <<= 1) {
    const Rt o = shfl_down_rt(v, d);
    if (lane + d < 64) v = compose(v, o);
  }
  const Rt next = shfl_down_rt(v, 1);
  if (lane == 0) st_rt(wb + 12 * wid, v);
  __syncthreads();
  Rt Ws = identity_rt();
  if (wid < kRWv - 1) {
    Ws = ld_rt(wb + 12 * (kRWv - 1));
    for (int w = kRWv - 2; w > wid; --w) Ws = compose(ld_rt(wb + 12 * w), Ws);
  }
  excl = lane < 63 ? (wid < kRWv - 1 ? compose(next, Ws) : next) : Ws;
}

// per-thread frame state: x, the frame residuals and the scaled-row data in
// registers; the loop rows h, the scale and the trial x in LDS (this thread's
// column of hl: no other thread touches it, so no barrier)
template <int F>
struct Frames {
  double x[F][6], r[F], d0[F], b1[F], b2[F], y[F];
  double* hl;  // [F][24][kRW]: h (12), sinv (6), trial x (6)
  __device__ __forceinline__ double& h(int f, int k) { return hl[(f * 24 + k) * kRW + threadIdx.x]; }
  __device__ __forceinline__ double& si(int f, int k) { return hl[(f * 24 + 12 + k) * kRW + threadIdx.x]; }
  __device__ __forceinline__ double& xt(int f, int k) { return hl[(f * 24 + 18 + k) * kRW + threadIdx.x]; }
};

// cost 0.5 |f(x)|^2 (every thread) and the loop residuals fl; jac: also the
// frame residuals r, and the loop rows h (d L_t, d L_R per parameter)
template <int F, bool JAC>
__device__ double eval_r(Frames<F>& S, bool trial, int m, int loop, double* red,
                         int& ph, double* wbf, double* wbb, double fl[2]) {
  // (JAC evaluates at the live x, never at the trial x)
  const int t = threadIdx.x;
  double c2[1] = {0.0};
  Rt rel[F];
  Rt loc = identity_rt();
#pragma unroll
  for (int f = 0; f < F; ++f) {
    if (t * F + f >= m) continue;
    double xf[6];
#pragma unroll
    for (int q = 0; q < 6; ++q) xf[q] = trial ? S.xt(f, q) : S.x[f][q];
    const double fc = frame_cost(xf);
    c2[0] += fc * fc;
    if (JAC) S.r[f] = fc;
    if (loop) {
      if (F == 1) {
        loc = rel_of(xf);
      } else {
        rel[f] = rel_of(xf);
        loc = f == 0 ? rel[f] : compose(loc, rel[f]);
      }
    }
  }
  rsum<1>(c2, red, ph);
  fl[0] = fl[1] = 0.0;
  if (!loop) return 0.5 * c2[0];
  Rt ex, T;
  chain_scan_fwd(loc, wbf, ex, T);
  loop_residuals(T, &fl[0], &fl[1]);
  const double cost = 0.5 * (c2[0] + (fl[0] * fl[0] + fl[1] * fl[1]));
  if (!JAC) return cost;
  Rt exs;
  chain_scan_bwd(loc, wbb, exs);
  double E1[3], E2[9];
#pragma unroll
  for (int a = 0; a < 3; ++a) E1[a] = T.t[a] > 0.0 ? 1.0 : (T.t[a] < 0.0 ? -1.0 : 0.0);
#pragma unroll
  for (int a = 0; a < 9; ++a) {
    const double dv = T.R[a] - ((a % 4 == 0) ? 1.0 : 0.0);
    E2[a] = dv > 0.0 ? 1.0 : (dv < 0.0 ? -1.0 : 0.0);
  }
  // per frame: P_i = ex * (the thread's earlier frames), S_i = (its later frames) * exs
  Rt Sf[F];
  {
    Rt Sc = exs;
#pragma unroll
    for (int f = F - 1; f >= 0; --f) {
      Sf[f] = Sc;
      if (t * F + f < m && f > 0) Sc = compose(F == 1 ? loc : rel[f], Sc);
    }
  }
  Rt Pi = ex;
#pragma unroll
  for (int f = 0; f < F; ++f) {
    if (t * F + f >= m) continue;
    const Rt& Si = Sf[f];
    const double* Rf = F == 1 ? loc.R : rel[f].R;
    double u[3], PE[9], G[9];
    for (int a = 0; a < 3; ++a) u[a] = Pi.R[a] * E1[0] + Pi.R[3 + a] * E1[1] + Pi.R[6 + a] * E1[2];
    for (int a = 0; a < 3; ++a)
      for (int b = 0; b < 3; ++b) PE[3 * a + b] = Pi.R[a] * E2[b] + Pi.R[3 + a] * E2[3 + b] + Pi.R[6 + a] * E2[6 + b];
    for (int a = 0; a < 3; ++a)
      for (int b = 0; b < 3; ++b)
        G[3 * a + b] = PE[3 * a] * Si.R[3 * b] + PE[3 * a + 1] * Si.R[3 * b + 1] + PE[3 * a + 2] * Si.R[3 * b + 2];
#pragma unroll 1
    for (int k = 0; k < 3; ++k) {
      double D[9];
      rodrigues_jac_k(S.x[f], Rf, k, D);  // dR/dr_k only: 9 live values, not 27
      double s1 = 0.0, s2 = 0.0;
      for (int a = 0; a < 3; ++a) s1 += u[a] * (D[3 * a] * Si.t[0] + D[3 * a + 1] * Si.t[1] + D[3 * a + 2] * Si.t[2]);
      for (int a = 0; a < 9; ++a) s2 += G[a] * D[a];
      S.h(f, k) = 1000.0 * s1;
      S.h(f, 3 + k) = 1000.0 * u[k];
      S.h(f, 6 + k) = 1e5 * s2;
      S.h(f, 9 + k) = 0.0;
    }
    if (f + 1 < F) Pi = compose(Pi, F == 1 ? loc : rel[f]);
  }
  return cost;
}

__device__ __forceinline__ double sgn(double v) { return v > 0.0 ? 1.0 : (v < 0.0 ? -1.0 : 0.0); }

template <int F>
__global__ __launch_bounds__(kRW) void k_chain_trf_r(double* __restrict__ ws, int m, int loop,
                                                     int max_iter, int first, double ftol, double xtol,
                                                     double gtol, int max_nfev,
                                                     double* __restrict__ state) {
  const ChainWs W(m);
  __shared__ double red[2 * kRMax * kRWv];
  __shared__ double wbf[12 * kRWv], wbb[12 * kRWv];
  __shared__ double hl[F * 24 * kRW];
  int ph = 0;
  const int t = threadIdx.x;
  Frames<F> S;
  S.hl = hl;
#pragma unroll
  for (int f = 0; f < F; ++f) {
    const int i = t * F + f;
    const bool v = i < m;
    S.r[f] = S.d0[f] = S.b1[f] = S.b2[f] = S.y[f] = 0.0;
#pragma unroll
    for (int k = 0; k < 6; ++k) {
      S.x[f][k] = v ? ws[W.x + 6 * i + k] : 0.0;
      S.xt(f, k) = 0.0;
      S.si(f, k) = v && !first ? ws[W.sinv + 6 * i + k] : 1.0;
    }
#pragma unroll
    for (int k = 0; k < 12; ++k) S.h(f, k) = 0.0;  // (own column only: no barrier)
  }
  auto valid = [&](int f) { return t * F + f < m; };
  double fl[2], flt[2];
  double cost = eval_r<F, true>(S, false, m, loop, red, ph, wbf, wbb, fl);
  int nfev = first ? 1 : (int)state[2], njev = first ? 1 : (int)state[3];
  auto update_scale = [&](bool init) {
#pragma unroll
    for (int f = 0; f < F; ++f) {
      if (!valid(f)) continue;
#pragma unroll
      for (int k = 0; k < 6; ++k) {
        const double gk = kW[k] * sgn(S.x[f][k]), h1 = S.h(f, k), h2 = S.h(f, 6 + k);
        const double cn = sqrt((gk * gk + h1 * h1) + h2 * h2);
        S.si(f, k) = init ? (cn == 0.0 ? 1.0 : cn) : fmax(S.si(f, k), cn);
      }
    }
  };
  double Delta, alpha;
  if (first) {
    update_scale(true);
    double v[1] = {0.0};
#pragma unroll
    for (int f = 0; f < F; ++f)
#pragma unroll
      for (int k = 0; k < 6; ++k) {
        const double a = S.x[f][k] * S.si(f, k);
        v[0] += valid(f) ? a * a : 0.0;
      }
    rsum<1>(v, red, ph);
    Delta = sqrt(v[0]);
    if (Delta == 0.0) Delta = 1.0;
    alpha = 0.0;
    if (t == 0) state[0] = cost;
  } else {
    Delta = state[5];
    alpha = state[6];
  }
  double E[3] = {0.0, 0.0, 0.0};  // |hs1|^2, hs1.hs2, |hs2|^2 of the iteration
  int status = 0, it = 0;
  for (; it < max_iter; ++it) {
    double gmax = 0.0;
#pragma unroll
    for (int f = 0; f < F; ++f) {
      if (!valid(f)) continue;
#pragma unroll
      for (int k = 0; k < 6; ++k) {
        const double gk = kW[k] * sgn(S.x[f][k]) * S.r[f] + S.h(f, k) * fl[0] + S.h(f, 6 + k) * fl[1];
        gmax = fmax(gmax, fabs(gk));
      }
    }
    gmax = rmax(gmax, red, ph);
    if (gmax < gtol) status = 1;
    if (status != 0 || nfev >= max_nfev) break;
    // scaled rows: d0 = |gs|^2, b1 = gs.hs1, b2 = gs.hs2; E and |J_h^T f|^2
    double e[4] = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
    for (int f = 0; f < F; ++f) {
      double d0 = 0.0, b1 = 0.0, b2 = 0.0;
      if (valid(f)) {
#pragma unroll
        for (int k = 0; k < 6; ++k) {
          const double s = 1.0 / S.si(f, k);
          const double gs = kW[k] * sgn(S.x[f][k]) * s, h1 = S.h(f, k) * s, h2 = S.h(f, 6 + k) * s;
          d0 += gs * gs;
          b1 += gs * h1;
          b2 += gs * h2;
          e[0] += h1 * h1;
          e[1] += h1 * h2;
          e[2] += h2 * h2;
          const double gh = gs * S.r[f] + h1 * fl[0] + h2 * fl[1];
          e[3] += gh * gh;
        }
      }
      S.d0[f] = d0;
      S.b1[f] = b1;
      S.b2[f] = b2;
    }
    rsum<4>(e, red, ph);
    E[0] = e[0];
    E[1] = e[1];
    E[2] = e[2];
    const double suf_norm = sqrt(e[3]);
    double actual = -1.0, cost_new = cost;
    // y = (K + a)^-1 f into S.y, yl; returns the 2x2 matrix (mA, mB, mC, det)
    auto solve_y = [&](double a, double yl[2], double mat[4]) {
      yl[0] = yl[1] = 0.0;
      mat[0] = mat[1] = mat[2] = 0.0;
      mat[3] = 1.0;
      if (loop) {
        double s[5] = {0.0, 0.0, 0.0, 0.0, 0.0};
#pragma unroll
        for (int f = 0; f < F; ++f) {
          if (!valid(f)) continue;
          const double da = S.d0[f] + a, b1 = S.b1[f], b2 = S.b2[f], ri = S.r[f];
          s[0] += b1 * b1 / da;
          s[1] += b1 * b2 / da;
          s[2] += b2 * b2 / da;
          s[3] += b1 * ri / da;
          s[4] += b2 * ri / da;
        }
        rsum<5>(s, red, ph);
        mat[0] = E[0] + a - s[0];
        mat[1] = E[1] - s[1];
        mat[2] = E[2] + a - s[2];
        const double r1 = fl[0] - s[3], r2 = fl[1] - s[4];
        mat[3] = mat[0] * mat[2] - mat[1] * mat[1];
        yl[0] = (mat[2] * r1 - mat[1] * r2) / mat[3];
        yl[1] = (mat[0] * r2 - mat[1] * r1) / mat[3];
      }
#pragma unroll
      for (int f = 0; f < F; ++f)
        S.y[f] = valid(f) ? (S.r[f] - S.b1[f] * yl[0] - S.b2[f] * yl[1]) / (S.d0[f] + a) : 0.0;
    };
    while (actual <= 0.0 && nfev < max_nfev) {
      double aup = suf_norm / Delta, alow = 0.0;
      if (alpha == 0.0) alpha = fmax(0.001 * aup, sqrt(alow * aup));
      double yl[2], mat[4], pn = 0.0;
      for (int k = 0; k < 10; ++k) {
        if (alpha < alow || alpha > aup) alpha = fmax(0.001 * aup, sqrt(alow * aup));
        solve_y(alpha, yl, mat);
        // f.y, y.y and (f - a y).z with z = (K + a)^-1 y never formed
        double q[7] = {0.0, 0.0, 0.0, 0.0, 0.0, 0.0, 0.0};  // Z1 Z2 fy yy A B1 B2
#pragma unroll
        for (int f = 0; f < F; ++f) {
          if (!valid(f)) continue;
          const double da = S.d0[f] + alpha, yi = S.y[f], fi = S.r[f];
          const double w = fi - alpha * yi;
          q[0] += S.b1[f] * yi / da;
          q[1] += S.b2[f] * yi / da;
          q[2] += fi * yi;
          q[3] += yi * yi;
          q[4] += w * yi / da;
          q[5] += w * S.b1[f] / da;
          q[6] += w * S.b2[f] / da;
        }
        rsum<7>(q, red, ph);
        double zl0 = 0.0, zl1 = 0.0;
        if (loop) {
          const double s1 = yl[0] - q[0], s2 = yl[1] - q[1];
          zl0 = (mat[2] * s1 - mat[1] * s2) / mat[3];
          zl1 = (mat[0] * s2 - mat[1] * s1) / mat[3];
        }
        const double q0 = q[2] + (fl[0] * yl[0] + fl[1] * yl[1]);
        const double q1 = q[3] + (yl[0] * yl[0] + yl[1] * yl[1]);
        const double q2 = (q[4] - zl0 * q[5] - zl1 * q[6]) +
                          ((fl[0] - alpha * yl[0]) * zl0 + (fl[1] - alpha * yl[1]) * zl1);
        pn = sqrt(fmax(q0 - alpha * q1, 0.0));
        const double phi = pn - Delta, dphi = -q2 / pn;
        if (phi < 0.0) aup = alpha;
        const double ratio = phi / dphi;
        alow = fmax(alow, alpha - ratio);
        alpha -= (phi + Delta) * ratio / Delta;
        if (fabs(phi) < 0.01 * Delta) break;
      }
      // the step at the final alpha, rescaled to |p| = Delta:
      // p = -c J_h^T y (c = Delta / |p(alpha)|), step = p / sinv; the sums the
      // step, |step|^2 and the predicted reduction need, taken before c is known
      solve_y(alpha, yl, mat);
      double q[8] = {0.0, 0.0, 0.0, 0.0, 0.0, 0.0, 0.0, 0.0};  // fy yy |x|^2 gp'^2 gp'r h1p' h2p' st'^2
#pragma unroll
      for (int f = 0; f < F; ++f) {
        if (!valid(f)) continue;
        const double yi = S.y[f];
        q[0] += S.r[f] * yi;
        q[1] += yi * yi;
        double gp = 0.0;
#pragma unroll
        for (int k = 0; k < 6; ++k) {
          const double si = S.si(f, k);
          const double gs = kW[k] * sgn(S.x[f][k]) / si, h1 = S.h(f, k) / si, h2 = S.h(f, 6 + k) / si;
          const double php = -((gs * yi + h1 * yl[0]) + h2 * yl[1]);
          const double stp = php / si;
          q[2] += S.x[f][k] * S.x[f][k];
          q[7] += stp * stp;
          gp += gs * php;
          q[5] += h1 * php;
          q[6] += h2 * php;
        }
        q[3] += gp * gp;
        q[4] += gp * S.r[f];
      }
      rsum<8>(q, red, ph);
      pn = sqrt(fmax((q[0] + (fl[0] * yl[0] + fl[1] * yl[1])) - alpha * (q[1] + (yl[0] * yl[0] + yl[1] * yl[1])), 0.0));
      const double c = Delta / pn;
#pragma unroll
      for (int f = 0; f < F; ++f) {
        const double yi = S.y[f];
#pragma unroll
        for (int k = 0; k < 6; ++k) {
          const double si = S.si(f, k);
          const double gs = kW[k] * sgn(S.x[f][k]) / si, h1 = S.h(f, k) / si, h2 = S.h(f, 6 + k) / si;
          const double ph2 = -c * ((gs * yi + h1 * yl[0]) + h2 * yl[1]);
          S.xt(f, k) = valid(f) ? S.x[f][k] + ph2 / si : 0.0;
        }
      }
      const double jp0 = c * (0.5 * c * q[3] + q[4]), jp1 = c * q[5], jp2 = c * q[6];
      const double quad = jp0 + (jp1 * (0.5 * jp1 + fl[0]) + jp2 * (0.5 * jp2 + fl[1]));
      const double predicted = -quad;
      cost_new = eval_r<F, false>(S, true, m, loop, red, ph, wbf, wbb, flt);
      ++nfev;
      const double step_h_norm = Delta;  // |p| = Delta after the rescale
      if (!isfinite(cost_new)) {
        Delta = 0.25 * step_h_norm;
        continue;
      }
      actual = cost - cost_new;
      double ratio;
      if (predicted > 0.0) ratio = actual / predicted;
      else if (predicted == actual) ratio = 1.0;
      else ratio = 0.0;
      double Dn = Delta;
      if (ratio < 0.25) Dn = 0.25 * step_h_norm;
      else if (ratio > 0.75 && step_h_norm > 0.95 * Delta) Dn = 2.0 * Delta;
      const double step_norm = c * sqrt(q[7]);
      const bool ftol_ok = actual < ftol * cost && ratio > 0.25;
      const bool xtol_ok = step_norm < xtol * (xtol + sqrt(q[2]));
      if (ftol_ok || xtol_ok) {
        status = ftol_ok && xtol_ok ? 4 : (ftol_ok ? 2 : 3);
        break;
      }
      alpha *= Delta / Dn;
      Delta = Dn;
    }
    if (actual > 0.0) {
#pragma unroll
      for (int f = 0; f < F; ++f)
#pragma unroll
        for (int k = 0; k < 6; ++k) S.x[f][k] = S.xt(f, k);
      cost = eval_r<F, true>(S, false, m, loop, red, ph, wbf, wbb, fl);
      ++njev;
      update_scale(false);
    }
    if (status != 0) {
      ++it;
      break;
    }
  }
#pragma unroll
  for (int f = 0; f < F; ++f) {
    const int i = t * F + f;
    if (i >= m) continue;
#pragma unroll
    for (int k = 0; k < 6; ++k) {
      ws[W.x + 6 * i + k] = S.x[f][k];
      ws[W.sinv + 6 * i + k] = S.si(f, k);
    }
  }
  if (t == 0) {
    state[1] = cost;
    state[2] = nfev;
    state[3] = njev;
    state[4] = status;
    state[5] = Delta;
    state[6] = alpha;
    state[7] = (first ? 0.0 : state[7]) + it;
  }
}

}  // namespace

extern "C" int slam_pose_chain_objective(const double* d_params, int n_vec, int n_frames, int loop,
                                         double* d_resid, void* stream) {
  SLAM_REQUIRE(n_vec >= 0 && n_frames >= 0, "slam_pose_chain_objective: bad sizes");
  if (n_vec == 0) return SLAM_OK;
  SLAM_REQUIRE(d_params && d_resid, "slam_pose_chain_objective: null pointer");
  k_chain_objective<<<(n_vec + 63) / 64, 64, 0, slam::as_stream(stream)>>>(d_params, n_vec, n_frames,
                                                                         loop ? 1 : 0, d_resid);
  SLAM_LAUNCHED("k_chain_objective");
  return SLAM_OK;
}

extern "C" long long slam_pose_chain_workspace_len(int n_frames) {
  return n_frames < 0 ? -1 : ChainWs(n_frames).tot;
}

extern "C" int slam_pose_chain_trf(double* d_ws, int n_frames, int loop, int max_iter, int first,
                                   double ftol, double xtol, double gtol, int max_nfev,
                                   double* d_state, void* stream) {
  SLAM_REQUIRE(n_frames >= 1 && max_iter >= 0 && max_nfev >= 1, "slam_pose_chain_trf: bad sizes");
  SLAM_REQUIRE(d_ws && d_state, "slam_pose_chain_trf: null pointer");
  hipStream_t s = slam::as_stream(stream);
  const int lp = loop ? 1 : 0, fi = first ? 1 : 0;
  const char* form = getenv("SLAM_CHAIN_TRF");  // "lds": the round-4 kernel (A/B)
  if (form != nullptr && form[0] == 'l') {
    k_chain_trf<<<1, kLmWG, 0, s>>>(d_ws, n_frames, lp, max_iter, fi, ftol, xtol, gtol, max_nfev, d_state);
  } else if (n_frames <= kRW) {
    k_chain_trf_r<1><<<1, kRW, 0, s>>>(d_ws, n_frames, lp, max_iter, fi, ftol, xtol, gtol, max_nfev, d_state);
  } else {
    k_chain_trf<<<1, kLmWG, 0, s>>>(d_ws, n_frames, lp, max_iter, fi, ftol, xtol, gtol, max_nfev, d_state);
  }
  SLAM_LAUNCHED("k_chain_trf");
  return SLAM_OK;
}
