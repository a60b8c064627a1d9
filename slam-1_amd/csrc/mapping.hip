// Map association: appendKeyPoints (/root/reference/keypoint.py:101-122).
//
// The reference builds a scipy KDTree over the map Qs every frame, queries the
// nearest map point of every new absolute point, and walks the points in
// order: a point whose nearest distance is below threshold * |rel_point| is
// an observation of that landmark; any other point is appended to the map
// (index len(Qs) - 1 at the time).  The tree is built before the walk, so the
// new points never match each other, and the walk is a prefix count:
//   index(d) = nn(d)                       if dist(d) < threshold |rel(d)|
//            = M + #(new points before d)  otherwise.
// Two kernels: k_map_nn (exact brute-force nearest neighbour, queries one per
// lane, the map streamed through LDS in chunks; one workgroup per (query block,
// map chunk)) and k_map_assoc (per query: fold the chunk partials in chunk
// order, the gate, a workgroup prefix scan, the appends and the output rows).
// Distances are squared sums in x, y, z order in f64 (KDTree's p = 2 sum), ties
// resolve to the lowest map index.  The map size M lives on the device, so a
// sequence of frames runs without host synchronisation.
#include "common.hpp"

#include <algorithm>

namespace {

constexpr int kNnWG = 256;      // queries per workgroup (one per lane)
constexpr int kNnChunk = 1024;  // map points per workgroup, staged in LDS (24 KiB)
constexpr int kAssocWG = 1024;

// Window strides (slam_map_windows: one launch for the same pair of every
// window, window = blockIdx.z here / blockIdx.x in k_map_assoc): map, M,
// query and count pointers and the workspace advance by these per window;
// all zero for a single map.
struct WinStride {
  size_t map, x, n, part;
};

__global__ __launch_bounds__(kNnWG) void k_map_nn(const double* __restrict__ map,
                                                  const int32_t* __restrict__ d_M,
                                                  const double* __restrict__ X,
                                                  const int32_t* __restrict__ d_n, int N,
                                                  double* __restrict__ part_d2,
                                                  int32_t* __restrict__ part_idx, WinStride ws) {
  const size_t wz = blockIdx.z;
  map += wz * ws.map;
  d_M += wz;
  X += wz * ws.x * 3;
  if (d_n) d_n += wz * ws.n;
  part_d2 += wz * ws.part;
  part_idx += wz * ws.part;
  __shared__ double sm[3 * kNnChunk];
  const int M = *d_M;
  const int n = d_n ? min(max(*d_n, 0), N) : N;
  const int base = blockIdx.y * kNnChunk;
  if (base >= M || (int)(blockIdx.x * kNnWG) >= n) return;  // uniform
  const int cnt = min(kNnChunk, M - base);
  for (int i = threadIdx.x; i < 3 * cnt; i += kNnWG) sm[i] = map[(size_t)3 * base + i];
  __syncthreads();
  const int q = blockIdx.x * kNnWG + threadIdx.x;
  if (q >= n) return;
  const double x = X[3 * q], y = X[3 * q + 1], z = X[3 * q + 2];
  double best = INFINITY;
  int bi = -1;
  for (int j = 0; j < cnt; ++j) {
    const double dx = x - sm[3 * j], dy = y - sm[3 * j + 1], dz = z - sm[3 * j + 2];
    const double d2 = (dx * dx + dy * dy) + dz * dz;
    if (d2 < best) {
      best = d2;
      bi = base + j;
    }
  }
  part_d2[(size_t)blockIdx.y * N + q] = best;
  part_idx[(size_t)blockIdx.y * N + q] = bi;
}

__global__ __launch_bounds__(kAssocWG) void k_map_assoc(
    double* __restrict__ map, int32_t* __restrict__ d_M, const double* __restrict__ X,
    const double* __restrict__ rel, const double* __restrict__ pts2d,
    const int32_t* __restrict__ d_n, int N, double threshold, int frame,
    const double* __restrict__ part_d2, const int32_t* __restrict__ part_idx,
    double* __restrict__ rows, WinStride ws) {
  const size_t wx = blockIdx.x;
  map += wx * ws.map;
  d_M += wx;
  X += wx * ws.x * 3;
  rel += wx * ws.x * 3;
  pts2d += wx * ws.x * 2;
  rows += wx * ws.x * 4;
  if (d_n) d_n += wx * ws.n;
  part_d2 += wx * ws.part;
  part_idx += wx * ws.part;
  __shared__ int wsum[kAssocWG / 64];
  const int M = *d_M;
  const int n = d_n ? min(max(*d_n, 0), N) : N;
  const int nch = (M + kNnChunk - 1) / kNnChunk;
  const int t = threadIdx.x, lane = t & 63, wid = t >> 6;
  int run = 0;  // new points appended so far (uniform)
  for (int t0 = 0; t0 < n; t0 += kAssocWG) {
    const int q = t0 + t;
    bool isnew = false;
    int idx = -1;
    if (q < n) {
      double best = INFINITY;
      for (int c = 0; c < nch; ++c) {
        const double d2 = part_d2[(size_t)c * N + q];
        if (d2 < best) {
          best = d2;
          idx = part_idx[(size_t)c * N + q];
        }
      }
      const double r0 = rel[3 * q], r1 = rel[3 * q + 1], r2 = rel[3 * q + 2];
      const double gate = threshold * sqrt((r0 * r0 + r1 * r1) + r2 * r2);
      isnew = !(sqrt(best) < gate);  // empty map: best = inf -> new
    }
    // workgroup exclusive scan of isnew (ballot per wave, then the wave totals)
    const unsigned long long bal = __ballot(isnew);
    const int pre = __popcll(bal & ((1ull << lane) - 1ull));
    if (lane == 0) wsum[wid] = __popcll(bal);
    __syncthreads();
    int wbase = 0, total = 0;
    for (int w = 0; w < kAssocWG / 64; ++w) {
      wbase += w < wid ? wsum[w] : 0;
      total += wsum[w];
    }
    if (q < n) {
      if (isnew) {
        idx = M + run + wbase + pre;
        map[3 * (size_t)idx] = X[3 * q];
        map[3 * (size_t)idx + 1] = X[3 * q + 1];
        map[3 * (size_t)idx + 2] = X[3 * q + 2];
      }
      rows[4 * (size_t)q] = (double)frame;
      rows[4 * (size_t)q + 1] = (double)idx;
      rows[4 * (size_t)q + 2] = pts2d[2 * q];
      rows[4 * (size_t)q + 3] = pts2d[2 * q + 1];
    }
    run += total;
    __syncthreads();  // wsum reuse
  }
  if (t == 0) *d_M = M + run;
}

size_t ws_bytes(int max_queries, int map_cap) {
  const size_t nch = (size_t)(map_cap + kNnChunk - 1) / kNnChunk;
  return nch * (size_t)max_queries * (sizeof(double) + sizeof(int32_t)) + 256;
}

}  // namespace

extern "C" int slam_map_workspace_bytes(int max_queries, int map_cap, size_t* bytes) {
  SLAM_REQUIRE(max_queries >= 0 && map_cap >= 0 && bytes, "slam_map_workspace_bytes: bad args");
  *bytes = ws_bytes(max_queries, map_cap);
  return SLAM_OK;
}

namespace {

// relative_to_abs3DPoints (Point3D.py:22-30) for a tracking batch: abs =
// (pose_b [X; 1])[:3] / (pose_b [X; 1])[3], one thread per point.
__global__ void k_rel_to_abs(const double* __restrict__ rel, const int32_t* __restrict__ count,
                             int cap, const double* __restrict__ poses, double* __restrict__ out) {
  const int b = blockIdx.y, i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= min(max(count[b], 0), cap)) return;
  const double* P = poses + 16 * (size_t)b;
  const double* X = rel + ((size_t)b * cap + i) * 3;
  double a[4];
  for (int r = 0; r < 4; ++r) a[r] = P[4 * r] * X[0] + P[4 * r + 1] * X[1] + P[4 * r + 2] * X[2] + P[4 * r + 3];
  double* o = out + ((size_t)b * cap + i) * 3;
  for (int r = 0; r < 3; ++r) o[r] = a[r] / a[3];
}

}  // namespace

extern "C" int slam_rel_to_abs(const double* d_rel, const int32_t* d_count, int cap, int batch,
                               const double* d_poses, double* d_abs, void* stream) {
  SLAM_REQUIRE(cap >= 0 && batch >= 0, "slam_rel_to_abs: bad shape");
  if (cap == 0 || batch == 0) return SLAM_OK;
  SLAM_REQUIRE(d_rel && d_count && d_poses && d_abs, "slam_rel_to_abs: null pointer");
  k_rel_to_abs<<<dim3((cap + 255) / 256, batch), 256, 0, slam::as_stream(stream)>>>(
      d_rel, d_count, cap, d_poses, d_abs);
  SLAM_LAUNCHED("k_rel_to_abs");
  return SLAM_OK;
}

extern "C" int slam_map_associate(double* d_map, int32_t* d_M, int map_cap, int M_bound,
                                  const double* d_abs, const double* d_rel, const double* d_pts2d,
                                  const int32_t* d_n, int N, double threshold, int frame_index,
                                  double* d_rows, void* d_ws, size_t ws_size, void* stream) {
  SLAM_REQUIRE(N >= 0 && map_cap >= 0 && M_bound >= 0, "slam_map_associate: bad shape");
  SLAM_REQUIRE(M_bound + N <= map_cap,
               "slam_map_associate: map capacity %d < M_bound %d + N %d (grow the map first)",
               map_cap, M_bound, N);
  SLAM_REQUIRE(ws_size >= ws_bytes(N, M_bound), "slam_map_associate: workspace too small");
  if (N == 0) return SLAM_OK;
  SLAM_REQUIRE(d_map && d_M && d_abs && d_rel && d_pts2d && d_rows && d_ws,
               "slam_map_associate: null pointer");
  const int nch = (M_bound + kNnChunk - 1) / kNnChunk;
  double* part_d2 = static_cast<double*>(d_ws);
  int32_t* part_idx = reinterpret_cast<int32_t*>(part_d2 + (size_t)nch * N);
  hipStream_t s = slam::as_stream(stream);
  if (nch > 0) {
    dim3 grid((N + kNnWG - 1) / kNnWG, nch);
    k_map_nn<<<grid, kNnWG, 0, s>>>(d_map, d_M, d_abs, d_n, N, part_d2, part_idx, WinStride{});
    SLAM_LAUNCHED("k_map_nn");
  }
  k_map_assoc<<<1, kAssocWG, 0, s>>>(d_map, d_M, d_abs, d_rel, d_pts2d, d_n, N, threshold,
                                     frame_index, part_d2, part_idx, d_rows, WinStride{});
  SLAM_LAUNCHED("k_map_assoc");
  return SLAM_OK;
}

extern "C" int slam_map_windows(double* d_maps, int32_t* d_M, int map_cap, int n_win, int n,
                                const double* d_abs, const double* d_rel, const double* d_pts2d,
                                const int32_t* d_count, int cap, double threshold, double* d_rows,
                                void* d_ws, size_t ws_size, void* stream) {
  SLAM_REQUIRE(n_win >= 0 && n >= 1 && cap >= 0 && map_cap >= 0, "slam_map_windows: bad shape");
  SLAM_REQUIRE((long long)n * cap <= map_cap, "slam_map_windows: map capacity %d < %d pairs x %d",
               map_cap, n, cap);
  SLAM_REQUIRE(ws_size >= (size_t)n_win * ws_bytes(cap, (n - 1) * cap),
               "slam_map_windows: workspace too small (n_win x slam_map_workspace_bytes)");
  if (n_win == 0 || cap == 0) return SLAM_OK;
  SLAM_REQUIRE(d_maps && d_M && d_abs && d_rel && d_pts2d && d_count && d_rows && d_ws,
               "slam_map_windows: null pointer");
  hipStream_t s = slam::as_stream(stream);
  SLAM_HIP(hipMemsetAsync(d_M, 0, sizeof(int32_t) * (size_t)n_win, s));
  // pair j of every window in one launch pair (the windows are independent;
  // within a window the pairs stay in order): per window its own map, size,
  // rows and a workspace slice of nch_max x cap partials -- the slice ws_bytes
  // sizes per window (none when n == 1: pair 0 meets an empty map, k_map_nn
  // never runs and k_map_assoc reads no partials)
  const int nch_max = ((n - 1) * cap + kNnChunk - 1) / kNnChunk;
  const size_t part = (size_t)nch_max * cap;
  double* part_d2 = static_cast<double*>(d_ws);
  int32_t* part_idx = reinterpret_cast<int32_t*>(part_d2 + (size_t)n_win * part);
  const WinStride wst{(size_t)map_cap * 3, (size_t)n * cap, (size_t)n, part};
  for (int j = 0; j < n; ++j) {
    const size_t b = (size_t)j;  // pair j of window 0; window w adds w * n pairs
    const int nch = (j * cap + kNnChunk - 1) / kNnChunk;
    if (nch > 0) {
      k_map_nn<<<dim3((cap + kNnWG - 1) / kNnWG, nch, n_win), kNnWG, 0, s>>>(
          d_maps, d_M, d_abs + b * cap * 3, d_count + b, cap, part_d2, part_idx, wst);
      SLAM_LAUNCHED("k_map_nn");
    }
    k_map_assoc<<<n_win, kAssocWG, 0, s>>>(d_maps, d_M, d_abs + b * cap * 3, d_rel + b * cap * 3,
                                           d_pts2d + b * cap * 2, d_count + b, cap, threshold, j,
                                           part_d2, part_idx, d_rows + b * cap * 4, wst);
    SLAM_LAUNCHED("k_map_assoc");
  }
  return SLAM_OK;
}
