/*
 * ORACLE — test infrastructure only.  Only tests/, __graft_entry__.smoke() and
 * bench.py's cpu_baseline leg may load this code, and only as the checker /
 * CPU baseline, never as the product path.
 *
 * Exact brute-force Hamming kNN-2 + Lowe ratio, a CPU restatement of what
 *   /root/reference/keypoint.py:40-51  (FlannBasedMatcher.knnMatch(k=2) + `m.distance < 0.7*n.distance`)
 *   /root/reference/Point3D.py:35-49 (same, plus the |Q| < max_Distance gate)
 * compute, with FLANN-LSH replaced by exact search.
 * Tie rule: equal distances are ordered by ascending train index
 * (cv::BFMatcher's stable order), so the best is the lowest-index minimum.
 * A train set with < 2 rows gives no good matches (ValueError truncation,
 * keypoint.py:46-51).
 */
#include <stdint.h>
#include <string.h>

static inline int hd32(const uint8_t* a, const uint8_t* b) {
  uint64_t x[4], y[4];
  memcpy(x, a, 32);
  memcpy(y, b, 32);
  return __builtin_popcountll(x[0] ^ y[0]) + __builtin_popcountll(x[1] ^ y[1]) +
         __builtin_popcountll(x[2] ^ y[2]) + __builtin_popcountll(x[3] ^ y[3]);
}

/* One (query set, train set) pair.  idx2/dist2: [nq][2], -1 = none. */
void oracle_hamming_knn2(const uint8_t* q, int nq, const uint8_t* t, int nt,
                         int32_t* idx2, int32_t* dist2, uint8_t* good) {
  for (int i = 0; i < nq; ++i) {
    int b1 = -1, b2 = -1, d1 = 1 << 30, d2 = 1 << 30;
    const uint8_t* qi = q + (size_t)i * 32;
    for (int j = 0; j < nt; ++j) {
      const int d = hd32(qi, t + (size_t)j * 32);
      if (d < d1) {
        d2 = d1; b2 = b1;
        d1 = d; b1 = j;
      } else if (d < d2) {
        d2 = d; b2 = j;
      }
    }
    idx2[2 * i] = b1;
    idx2[2 * i + 1] = b2;
    dist2[2 * i] = b1 < 0 ? -1 : d1;
    dist2[2 * i + 1] = b2 < 0 ? -1 : d2;
    good[i] = (b2 >= 0 && 10 * d1 < 7 * d2) ? 1 : 0;
  }
}

/* Batched form with the same layout as slam_hamming_knn2. */
void oracle_hamming_knn2_batch(const uint8_t* q, const int32_t* nq, int q_cap,
                               const uint8_t* t, const int32_t* nt, int t_cap,
                               int batch, int32_t* idx2, int32_t* dist2, uint8_t* good) {
#pragma omp parallel for schedule(dynamic, 1)
  for (int b = 0; b < batch; ++b) {
    int n_q = nq[b] < q_cap ? nq[b] : q_cap;
    int n_t = nt[b] < t_cap ? nt[b] : t_cap;
    if (n_q < 0) n_q = 0;
    if (n_t < 0) n_t = 0;
    oracle_hamming_knn2(q + (size_t)b * q_cap * 32, n_q, t + (size_t)b * t_cap * 32, n_t,
                        idx2 + (size_t)b * q_cap * 2, dist2 + (size_t)b * q_cap * 2,
                        good + (size_t)b * q_cap);
  }
}
