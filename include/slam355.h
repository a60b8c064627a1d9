/*
 * slam355.h — C ABI of libslam355.so, the MI355X (gfx950) hot path of the
 * DavidHan008/SLAM-1 stereo front end and local bundle adjustment.
 *
 * Conventions (every entry point):
 *   - Pointers named d_* are caller-owned DEVICE pointers (HBM).  Pointers named
 *     h_* are host pointers.  Nothing is allocated inside a hot call; scratch is
 *     a caller-provided workspace sized by the matching *_workspace_bytes query.
 *   - `stream` is a hipStream_t passed as void* (NULL = default stream).  Every
 *     compute call is asynchronous on that stream.
 *   - Return value: 0 = ok; < 0 = error.  slam_last_error() returns a
 *     thread-local message for the last failure on the calling thread.
 *   - Ragged batches: per-item element counts live in DEVICE int32 arrays so a
 *     pipeline never has to synchronise to learn them; kernels clamp every
 *     count to the stated capacity.
 *
 * The reference (Python + OpenCV + scipy) has no FFI; each function below
 * replaces the Python/OpenCV call named in its comment, and the Python host
 * package `slam355` (slam-1_amd/slam355) keeps the reference's function names
 * and signatures on top of these calls.
 */
#ifndef SLAM355_H
#define SLAM355_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SLAM355_ABI_VERSION 1

/* Error codes. */
#define SLAM_OK 0
#define SLAM_ERR_ARG (-1)      /* invalid argument / shape                  */
#define SLAM_ERR_HIP (-2)      /* HIP runtime error (launch, device)        */
#define SLAM_ERR_WORKSPACE (-3) /* workspace too small                      */
#define SLAM_ERR_COMM (-4)     /* collective error                          */

int slam_abi_version(void);
const char* slam_last_error(void);
/* Number of visible devices (0 when no GPU); never fails. */
int slam_device_count(void);

/* ------------------------------------------------------------------------
 * Brute-force Hamming kNN-2 + Lowe ratio test.
 *
 * Replaces cv2.FlannBasedMatcher(LSH).knnMatch(des_q, des_t, k=2) followed by
 * the `m.distance < 0.7 * n.distance` loop:
 *   /root/reference/keypoint.py:83-94   (track_keypoints_left_to_right_new)
 *   /root/reference/Point3D.py:199-213  (find_2D_and_3D_correspondenses)
 *   /root/reference/tracking.py:231-247 (get_matches)
 * Exact search (FLANN-LSH is approximate).  Ties are broken by
 * the lower train index, as cv::BFMatcher does.
 *
 * Batch of `batch` independent (query set, train set) pairs.
 *   d_q    [batch][q_cap][32] u8     d_nq [batch] i32 (clamped to q_cap)
 *   d_t    [batch][t_cap][32] u8     d_nt [batch] i32 (clamped to t_cap)
 * Outputs for every valid query row (rows >= nq are not written):
 *   d_idx2  [batch][q_cap][2] i32  best / second-best train index (-1 = none)
 *   d_dist2 [batch][q_cap][2] i32  their Hamming distances      (-1 = none)
 *   d_good  [batch][q_cap]    u8   1 iff both exist and 10*d1 < 7*d2
 * (`10*d1 < 7*d2` == `d1 < 0.7*d2` for every integer d1, d2 in [0, 256].)
 * A train set with fewer than 2 rows yields no good matches, mirroring the
 * reference's ValueError truncation (keypoint.py:89-94).
 * t_cap must be <= 65535.
 * ---------------------------------------------------------------------- */
int slam_hamming_knn2(const uint8_t* d_q, const int32_t* d_nq, int q_cap,
                      const uint8_t* d_t, const int32_t* d_nt, int t_cap,
                      int batch, int32_t* d_idx2, int32_t* d_dist2,
                      uint8_t* d_good, void* stream);

/* Order-preserving compaction of the good matches of slam_hamming_knn2:
 * d_pairs [batch][q_cap][2] i32 = (queryIdx, trainIdx) of the good rows in
 * query order (the `good` list of keypoint.py:90-92), d_count [batch] i32.
 * Optional extra gate (Point3D.py:209-210): if d_gate_xyz != NULL, a good
 * row q is kept only if |X[q][k]| < gate for k = 0,1,2, where
 * d_gate_xyz [batch][q_cap][3] f64. */
int slam_compact_matches(const int32_t* d_idx2, const uint8_t* d_good,
                         const int32_t* d_nq, int q_cap, int batch,
                         const double* d_gate_xyz, double gate,
                         int32_t* d_pairs, int32_t* d_count, void* stream);

#ifdef __cplusplus
}
#endif

#endif /* SLAM355_H */
