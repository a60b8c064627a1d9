// Bag-of-words place recognition: /root/reference/bag_of_words.py.
//
// The reference computes ORB descriptors per image (cv2.ORB_create(100) on the
// whole image; here the single-patch mode of k_orb_tile), assigns each to
// the nearest of K scikit-learn KMeans centres (hist, :24-27), histograms the
// labels, and finds the most similar earlier image by the chi-squared distance
// sum 2 (x - y)^2 / max(1, x + y) (predict_previous / predict, :30-56).  The
// vocabulary is trained by Lloyd iterations (KMeans.fit, :20).
//
// Kernels:
//   k_bow_hist    WG per image: centres and their squared norms in LDS, one
//                 descriptor per lane, label = argmin_j |c_j|^2 - 2 x.c_j (the
//                 expression scikit-learn's Lloyd / predict evaluates; first
//                 index on ties), label histogram by LDS integer atomics
//   k_bow_query   WG per query image: chi-squared distance to every allowed
//                 database histogram (one row per lane, numpy's pairwise sum
//                 order over the K bins), argmin with the first index on ties
//   k_bow_label   Lloyd E-step over the pooled descriptors, one per lane
//   k_bow_center  WG per cluster: the mean of its points in a fixed order
//                 (Lloyd's M-step; an empty cluster keeps its centre)
#include "common.hpp"

namespace {

constexpr int kBowWG = 256;
constexpr int kDim = 32;  // ORB descriptor bytes (features as float64)
constexpr int kMaxK = 128;

__device__ __forceinline__ int nearest(const uint8_t* __restrict__ d, const double* cs,
                                       const double* cn, int K) {
  double x[kDim];
  for (int k = 0; k < kDim; ++k) x[k] = (double)d[k];
  int best = 0;
  double bd = 0.0;
  for (int j = 0; j < K; ++j) {
    const double* c = cs + j * kDim;
    double dot = 0.0;
    for (int k = 0; k < kDim; ++k) dot += x[k] * c[k];
    const double dist = cn[j] + -2.0 * dot;
    if (j == 0 || dist < bd) {
      bd = dist;
      best = j;
    }
  }
  return best;
}

__device__ void stage_centers(const double* __restrict__ centers, int K, double* cs, double* cn) {
  for (int e = threadIdx.x; e < K * kDim; e += blockDim.x) cs[e] = centers[e];
  __syncthreads();
  for (int j = threadIdx.x; j < K; j += blockDim.x) {
    double s = 0.0;
    for (int k = 0; k < kDim; ++k) s += cs[j * kDim + k] * cs[j * kDim + k];
    cn[j] = s;
  }
  __syncthreads();
}

// desc [B][cap][32] u8, count [B] (or null: n_each rows each) -> labels [B][cap], hist [B][K]
__global__ __launch_bounds__(kBowWG) void k_bow_hist(const uint8_t* __restrict__ desc,
                                                     const int32_t* __restrict__ count, int n_each,
                                                     int cap, const double* __restrict__ centers,
                                                     int K, int32_t* __restrict__ labels,
                                                     int32_t* __restrict__ hist) {
  __shared__ double cs[kMaxK * kDim];
  __shared__ double cn[kMaxK];
  __shared__ int h[kMaxK];
  const int b = blockIdx.x;
  stage_centers(centers, K, cs, cn);
  for (int j = threadIdx.x; j < K; j += kBowWG) h[j] = 0;
  __syncthreads();
  const int n = count ? min(max(count[b], 0), cap) : n_each;
  for (int i = threadIdx.x; i < n; i += kBowWG) {
    const int l = nearest(desc + ((size_t)b * cap + i) * kDim, cs, cn, K);
    if (labels) labels[(size_t)b * cap + i] = l;
    atomicAdd(&h[l], 1);
  }
  __syncthreads();
  for (int j = threadIdx.x; j < K; j += kBowWG) hist[(size_t)b * K + j] = h[j];
}

// Lloyd E-step over a flat point set: one point per lane
__global__ __launch_bounds__(kBowWG) void k_bow_label(const uint8_t* __restrict__ X, int N,
                                                      const double* __restrict__ centers, int K,
                                                      int32_t* __restrict__ labels) {
  __shared__ double cs[kMaxK * kDim];
  __shared__ double cn[kMaxK];
  stage_centers(centers, K, cs, cn);
  const int i = blockIdx.x * kBowWG + threadIdx.x;
  if (i < N) labels[i] = nearest(X + (size_t)i * kDim, cs, cn, K);
}

// numpy pairwise_sum for n <= 128 (8-way unrolled partial sums, then the rest)
__device__ __forceinline__ double chi2(const int32_t* __restrict__ x, const int32_t* __restrict__ y, int K) {
  auto term = [&](int j) {
    const long long dx = (long long)x[j] - y[j];
    const long long den = max(1ll, (long long)x[j] + y[j]);
    return (double)(2 * dx * dx) / (double)den;
  };
  if (K < 8) {
    double s = 0.0;  // numpy: res = 0., then res += a[i]
    for (int j = 0; j < K; ++j) s += term(j);
    return s;
  }
  double r[8];
  for (int q = 0; q < 8; ++q) r[q] = term(q);
  int i = 8;
  for (; i < K - (K % 8); i += 8)
    for (int q = 0; q < 8; ++q) r[q] += term(i + q);
  double res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
  for (; i < K; ++i) res += term(i);
  return res;
}

// query q: db rows [0, n_db[q]) -> (argmin, min); n_db <= 0 -> (-1, -1)
__global__ __launch_bounds__(kBowWG) void k_bow_query(const int32_t* __restrict__ qh, const int32_t* __restrict__ db,
                                                      const int32_t* __restrict__ n_db, int K,
                                                      int32_t* __restrict__ out_idx,
                                                      double* __restrict__ out_val) {
  __shared__ double sv[kBowWG];
  __shared__ int si[kBowWG];
  const int q = blockIdx.x, t = threadIdx.x;
  const int n = n_db[q];
  const int32_t* x = qh + (size_t)q * K;
  double bv = 0.0;
  int bi = -1;
  for (int r = t; r < n; r += kBowWG) {
    const double v = chi2(x, db + (size_t)r * K, K);
    if (bi < 0 || v < bv) {  // rows visited in increasing order: first index kept
      bv = v;
      bi = r;
    }
  }
  sv[t] = bv;
  si[t] = bi;
  __syncthreads();
  for (int off = kBowWG / 2; off > 0; off >>= 1) {
    if (t < off) {
      const int oi = si[t + off];
      const double ov = sv[t + off];
      if (oi >= 0 && (si[t] < 0 || ov < sv[t] || (ov == sv[t] && oi < si[t]))) {
        sv[t] = ov;
        si[t] = oi;
      }
    }
    __syncthreads();
  }
  if (t == 0) {
    out_idx[q] = n > 0 ? si[0] : -1;
    out_val[q] = n > 0 ? sv[0] : -1.0;
  }
}

// Lloyd M-step: centre j = mean of its points (x as float64), fixed summation
// order (lane-strided partials, then a tree); an empty cluster keeps its centre.
__global__ __launch_bounds__(kBowWG) void k_bow_center(const uint8_t* __restrict__ X, int N,
                                                       const int32_t* __restrict__ labels,
                                                       const double* __restrict__ c_old,
                                                       double* __restrict__ c_new,
                                                       double* __restrict__ shift) {
  __shared__ double part[kBowWG][kDim + 1];
  const int j = blockIdx.x, t = threadIdx.x;
  double s[kDim];
  for (int k = 0; k < kDim; ++k) s[k] = 0.0;
  double cnt = 0.0;
  for (int i = t; i < N; i += kBowWG) {
    if (labels[i] != j) continue;
    for (int k = 0; k < kDim; ++k) s[k] += (double)X[(size_t)i * kDim + k];
    cnt += 1.0;
  }
  for (int k = 0; k < kDim; ++k) part[t][k] = s[k];
  part[t][kDim] = cnt;
  __syncthreads();
  for (int off = kBowWG / 2; off > 0; off >>= 1) {
    if (t < off)
      for (int k = 0; k <= kDim; ++k) part[t][k] += part[t + off][k];
    __syncthreads();
  }
  if (t < kDim) {
    const double n = part[0][kDim];
    const double v = n > 0.0 ? part[0][t] / n : c_old[j * kDim + t];
    c_new[j * kDim + t] = v;
    const double d = v - c_old[j * kDim + t];
    part[t][0] = d * d;  // (row 0 is read only by t < kDim above: reuse rows as scratch)
  }
  __syncthreads();
  if (t == 0 && shift) {
    double sh = 0.0;
    for (int k = 0; k < kDim; ++k) sh += part[k][0];
    shift[j] = sh;
  }
}

}  // namespace

extern "C" int slam_bow_histograms(const uint8_t* d_desc, const int32_t* d_count, int n_each,
                                   int n_img, int cap, const double* d_centers, int n_clusters,
                                   int32_t* d_labels, int32_t* d_hist, void* stream) {
  SLAM_REQUIRE(n_img >= 0 && cap >= 0 && n_clusters >= 1 && n_clusters <= kMaxK,
               "slam_bow_histograms: need 1 <= n_clusters <= %d", kMaxK);
  SLAM_REQUIRE(d_count || (n_each >= 0 && n_each <= cap), "slam_bow_histograms: bad n_each");
  if (n_img == 0) return SLAM_OK;
  SLAM_REQUIRE(d_desc && d_centers && d_hist, "slam_bow_histograms: null pointer");
  k_bow_hist<<<n_img, kBowWG, 0, slam::as_stream(stream)>>>(d_desc, d_count, n_each, cap, d_centers,
                                                           n_clusters, d_labels, d_hist);
  SLAM_LAUNCHED("k_bow_hist");
  return SLAM_OK;
}

extern "C" int slam_bow_query(const int32_t* d_qhist, int n_query, const int32_t* d_db,
                              const int32_t* d_n_db, int n_clusters, int32_t* d_idx,
                              double* d_val, void* stream) {
  SLAM_REQUIRE(n_query >= 0 && n_clusters >= 1 && n_clusters <= kMaxK,
               "slam_bow_query: need 1 <= n_clusters <= %d", kMaxK);
  if (n_query == 0) return SLAM_OK;
  SLAM_REQUIRE(d_qhist && d_db && d_n_db && d_idx && d_val, "slam_bow_query: null pointer");
  k_bow_query<<<n_query, kBowWG, 0, slam::as_stream(stream)>>>(d_qhist, d_db, d_n_db, n_clusters,
                                                              d_idx, d_val);
  SLAM_LAUNCHED("k_bow_query");
  return SLAM_OK;
}

extern "C" int slam_bow_lloyd(const uint8_t* d_X, int n_points, double* d_centers,
                              double* d_centers_tmp, int n_clusters, int n_iter,
                              int32_t* d_labels, double* d_shift, void* stream) {
  SLAM_REQUIRE(n_points >= 1 && n_iter >= 0 && n_clusters >= 1 && n_clusters <= kMaxK,
               "slam_bow_lloyd: bad sizes (1 <= n_clusters <= %d)", kMaxK);
  SLAM_REQUIRE(d_X && d_centers && d_centers_tmp && d_labels, "slam_bow_lloyd: null pointer");
  hipStream_t s = slam::as_stream(stream);
  const int grid = (n_points + kBowWG - 1) / kBowWG;
  double* cur = d_centers;
  double* nxt = d_centers_tmp;
  for (int it = 0; it < n_iter; ++it) {
    k_bow_label<<<grid, kBowWG, 0, s>>>(d_X, n_points, cur, n_clusters, d_labels);
    SLAM_LAUNCHED("k_bow_label");
    k_bow_center<<<n_clusters, kBowWG, 0, s>>>(d_X, n_points, d_labels, cur, nxt, d_shift);
    SLAM_LAUNCHED("k_bow_center");
    double* tmp = cur;
    cur = nxt;
    nxt = tmp;
  }
  if (cur != d_centers)
    SLAM_HIP(hipMemcpyAsync(d_centers, cur, sizeof(double) * n_clusters * kDim,
                            hipMemcpyDeviceToDevice, s));
  // labels of the final centres (scikit-learn's closing E-step)
  k_bow_label<<<grid, kBowWG, 0, s>>>(d_X, n_points, d_centers, n_clusters, d_labels);
  SLAM_LAUNCHED("k_bow_label");
  return SLAM_OK;
}
