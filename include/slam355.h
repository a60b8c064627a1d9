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
 *   /root/reference/keypoint.py:40-51   (track_keypoints_left_to_right_new)
 *   /root/reference/Point3D.py:35-49  (find_2D_and_3D_correspondenses)
 *   /root/reference/tracking.py:14-30 (get_matches)
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
 * reference's ValueError truncation (keypoint.py:46-51).
 * t_cap must be <= 65535.  t_cap <= 16383 runs on the fp4 matrix cores
 * (knn2_mx_kernel: exact integer keys in f32), larger train sets on the
 * integer VALU (knn2_kernel); both give identical outputs.
 * ---------------------------------------------------------------------- */
int slam_hamming_knn2(const uint8_t* d_q, const int32_t* d_nq, int q_cap,
                      const uint8_t* d_t, const int32_t* d_nt, int t_cap,
                      int batch, int32_t* d_idx2, int32_t* d_dist2,
                      uint8_t* d_good, void* stream);

/* Kernel selection of slam_hamming_knn2 for A/B tests and benchmarks:
 * valu != 0 forces the integer-VALU kernel, 0 (default) the matrix-core one
 * where t_cap allows.  Process-wide; returns the previous setting. */
int slam_hamming_force_valu(int valu);

/* Order-preserving compaction of the good matches of slam_hamming_knn2:
 * d_pairs [batch][q_cap][2] i32 = (queryIdx, trainIdx) of the good rows in
 * query order (the `good` list of keypoint.py:47-49), d_count [batch] i32.
 * Optional extra gate (Point3D.py:45-46): if d_gate_xyz != NULL, a good
 * row q is kept only if |X[q][k]| < gate for k = 0,1,2, where
 * d_gate_xyz [batch][q_cap][3] f64. */
int slam_compact_matches(const int32_t* d_idx2, const uint8_t* d_good,
                         const int32_t* d_nq, int q_cap, int batch,
                         const double* d_gate_xyz, double gate,
                         int32_t* d_pairs, int32_t* d_count, void* stream);


/* ------------------------------------------------------------------------
 * Geometry of one tracking step (main.py:82-97), batched over frame pairs.
 * ---------------------------------------------------------------------- */

/* Gather of matched keypoints (keypoint.py:53-57, Point3D.py:50-52):
 * for k < count[b], (qi, ti) = pairs[b][k]:
 *   ptq[b][k] = (double)kpq[b][qi].xy, ptt[b][k] = (double)kpt[b][ti].xy,
 *   dq[b][k] = desq[b][qi], dt[b][k] = dest[b][ti]  (descriptors optional: NULL).
 * kp arrays are [batch][cap][5] f32 as written by slam_orb_tiles. */
int slam_gather_matches(const float* d_kpq, int kq_cap, const float* d_kpt, int kt_cap,
                        const uint8_t* d_desq, const uint8_t* d_dest, const int32_t* d_pairs,
                        const int32_t* d_count, int p_cap, int batch, double* d_ptq,
                        double* d_ptt, uint8_t* d_dq, uint8_t* d_dt, void* stream);

/* 2D-3D correspondences of find_2D_and_3D_correspondenses (Point3D.py:50-52):
 * for k < count[b], (qi, ti) = pairs[b][k]: Q1[b][k] = X[b][qi], q1[b][k] =
 * ptl[b][qi], q2[b][k] = (double)kp_next[b][ti].xy.  X [batch][xcap][3],
 * ptl [batch][xcap][2] f64; kp_next [batch][kcap][5] f32. */
int slam_gather_temporal(const double* d_X, const double* d_ptl, int xcap, const float* d_kp_next,
                         int kcap, const int32_t* d_pairs, const int32_t* d_count, int pcap,
                         int batch, double* d_Q1, double* d_q2, double* d_q1, void* stream);

/* cv2.findFundamentalMat(pts_left, pts_right, FM_LMEDS) mask (keypoint.py:59-66),
 * deterministic LMedS restated in oracle/fundamental.c: n_hyp seeded 7-point
 * hypotheses (300 = OpenCV's LMeDS count at confidence 0.99), min median of
 * the symmetric epipolar error, inliers err <= sigma^2 with OpenCV's robust
 * sigma.  d_m1/d_m2 [batch][cap][2] f64; d_mask [batch][cap] u8; d_F
 * [batch][9] (unit Frobenius norm); d_ninliers [batch] (-1: < 8 points / no model). */
int slam_fundamental_lmeds(const double* d_m1, const double* d_m2, const int32_t* d_count,
                           int cap, int batch, uint64_t seed, int item0, int n_hyp,
                           uint8_t* d_mask, double* d_F, int32_t* d_ninliers, void* stream);

/* Order-preserving compaction of pairs[b][k] (k < count[b]) where mask[b][k] != 0
 * (the `pts_left[mask]` of keypoint.py:63-66). d_out must not alias d_pairs. */
int slam_filter_pairs(const int32_t* d_pairs, const int32_t* d_count, const uint8_t* d_mask,
                      int cap, int batch, int32_t* d_out, int32_t* d_out_count, void* stream);

/* cv2.triangulatePoints + dehomogenisation (Point3D.py:14-19): per point the
 * null vector of the 4x4 DLT system (rows x*P[2]-P[0], y*P[2]-P[1] of both
 * views), one-sided Jacobi SVD in f64.  d_ptl/d_ptr [batch][cap][2] f64,
 * d_X [batch][cap][3] f64.  P matrices are 3x4 row-major f64: shared by all
 * items (proj_stride 0) or one per item (proj_stride 12). */
int slam_triangulate(const double* d_ptl, const double* d_ptr, const int32_t* d_count, int cap,
                     int batch, const double* d_Pl, const double* d_Pr, int proj_stride,
                     double* d_X, void* stream);

/* cv2.solvePnPRansac(Q, q, K, zeros(5)) (transformation.py:11-13), restated
 * deterministically (oracle/geometry.c): n_hyp hypotheses of 5 points drawn
 * from splitmix64(seed, item0 + b, h), LM from r = t = 0 (hyp_iters), score =
 * #(|reprojection error| <= reproj_thresh), best = max score / lowest h, LM
 * refinement over its inliers (refine_iters).  One workgroup per item.
 * Outputs: d_rvec/d_tvec [batch][3] (X_cam = R(rvec) X + tvec), d_ninliers
 * [batch] (-1 when count < 5, the reference's `len(Q) > 4` guard, main.py:94),
 * d_mask [batch][cap] u8 inliers of the chosen hypothesis. */
int slam_pnp_ransac(const double* d_Q, const double* d_q, const int32_t* d_count, int cap,
                    int batch, const double* d_K, uint64_t seed, int item0, int n_hyp,
                    double reproj_thresh, int hyp_iters, int refine_iters, double* d_rvec,
                    double* d_tvec, int32_t* d_ninliers, uint8_t* d_mask, double* d_ws,
                    long long ws_len, void* stream);
/* Doubles of slam_pnp_ransac's workspace d_ws (the hypothesis poses); a d_ws of
 * fewer than this many doubles (ws_len) returns SLAM_ERR_WORKSPACE.  The
 * workspace is the caller's: calls that may overlap (other streams) need their own. */
long long slam_pnp_workspace_len(int batch, int n_hyp);

/* Pose chain of main.py:94-98, 120-124 (pose_{b+1} = pose_b @ T_b with
 * T_b = [Rodrigues(-rvec_b) | -tvec_b], transformation.py:15-19; when
 * d_ninliers[b] < 0 -- PnP skipped, main.py:94 -- the previous T is reused).
 * d_state [32] f64 = (pose, T) 4x4 row-major, read and updated in place so
 * consecutive batches chain on the device; d_poses [batch][16] f64 out.
 * Replaces the host loop slam355.pipeline.chain_poses. */
int slam_pose_chain(const double* d_rvec, const double* d_tvec, const int32_t* d_ninliers,
                    int batch, double* d_state, double* d_poses, void* stream);

/* The reference's stereo visual-odometry pose estimator
 * (visual_odometry.py:135-157 estimate_pose over the residuals of :65-81),
 * restated deterministically (oracle/vo.c): dof = (rotvec, t), T = [R | t];
 * residuals f (4N) = [proj(P T, Q2) - q1 (x row, y row), proj(P T^-1, Q1) - q2
 * (x row, y row)]; max_iter hypotheses of 6 points drawn WITH replacement from
 * splitmix64(seed, item0 + b, h) (np.random.choice(range(n), 6), :139), LM from
 * dof = 0 (lm_iters; least_squares(method='lm') at :142), error = sum over k of
 * |(f[2k], f[2k+1])| (the reshape((2N, 2)) of :144-146), sequential early stop
 * after early_stop non-improving hypotheses (:147-154; 5 in the reference).
 * One workgroup per item, one lane per hypothesis (max_iter <= 128).
 * d_q1/d_q2 [batch][cap][2], d_Q1/d_Q2 [batch][cap][3] f64, d_P 3x4 row-major.
 * Outputs: d_pose [batch][6] (rotvec, t) of the selected hypothesis (zeros when
 * none improved), d_best [batch] its index (-1 if none), d_ntried [batch]
 * hypotheses the sequential loop evaluates, d_err [batch] its error. */
int slam_vo_estimate_pose(const double* d_q1, const double* d_q2, const double* d_Q1,
                          const double* d_Q2, const int32_t* d_count, int cap, int batch,
                          const double* d_P, uint64_t seed, int item0, int max_iter,
                          int lm_iters, int early_stop, double* d_pose, int32_t* d_best,
                          int32_t* d_ntried, double* d_err, void* d_ws, size_t ws_bytes,
                          void* stream);
/* Workspace of slam_vo_estimate_pose: every hypothesis' dof and error
 * (the error is np.sum's order over the pair norms: 8192-chunks of pairwise sums). */
int slam_vo_pose_workspace_bytes(int batch, int max_iter, size_t* bytes);

/* reprojection_residuals(dof, q1, q2, Q1, Q2) (visual_odometry.py:65-81) for
 * one dof per item: d_dof [batch][6]; d_res [batch][4 * cap], the first
 * 4 * count[b] entries in the reference's flattened order. */
int slam_vo_residuals(const double* d_dof, const double* d_q1, const double* d_q2,
                      const double* d_Q1, const double* d_Q2, const int32_t* d_count, int cap,
                      int batch, const double* d_P, double* d_res, void* stream);

/* relative_to_abs3DPoints (Point3D.py:22-30) for a tracking batch:
 * d_abs[b][i] = (pose_b [X;1])[:3] / (pose_b [X;1])[3] for i < d_count[b];
 * d_rel, d_abs [batch][cap][3] f64, d_poses [batch][16] f64 row-major. */
int slam_rel_to_abs(const double* d_rel, const int32_t* d_count, int cap, int batch,
                    const double* d_poses, double* d_abs, void* stream);

/* ------------------------------------------------------------------------
 * Map association: appendKeyPoints (keypoint.py:101-122).
 *
 * For each of the N new absolute points (d_abs [N][3] f64, camera-frame
 * d_rel [N][3], image coordinates d_pts2d [N][2]) the exact nearest map point
 * (the reference's KDTree(Qs).query(k=1); squared distance summed x, y, z in
 * f64, ties -> lowest index) is taken as the landmark when its distance is
 * below threshold * |rel| (:113-115); otherwise the point is appended to the
 * map with the next index (:117-118).  Queries use the map as it was before
 * the call (the tree is built first, :109).  d_map [map_cap][3] f64 and the map
 * size d_M (device int32, updated in place: sequences of frames need no host
 * synchronisation).  M_bound is any host-side upper bound of *d_M (grid
 * sizing); M_bound + N <= map_cap is required.  d_n (nullable): device count
 * of valid points (<= N).  d_rows [N][4] f64 = [frame_index, landmark index,
 * u, v] (the reference's full_index_array rows).  Workspace from
 * slam_map_workspace_bytes(N, M_bound or map_cap). */
int slam_map_workspace_bytes(int max_queries, int map_cap, size_t* bytes);
int slam_map_associate(double* d_map, int32_t* d_M, int map_cap, int M_bound,
                       const double* d_abs, const double* d_rel, const double* d_pts2d,
                       const int32_t* d_n, int N, double threshold, int frame_index,
                       double* d_rows, void* d_ws, size_t ws_size, void* stream);
/* The local maps of a tracked batch's windows (main.py:120-127 per window of n
 * consecutive frame pairs; bench.py's tracked leg): for window w < n_win, map
 * d_maps[w] ([map_cap][3], map_cap >= n * cap) restarted empty (d_M[w] = 0)
 * and fed pairs b = w n + j, j < n, in order -- slam_map_associate of
 * d_abs[b], d_rel[b] ([cap][3]), d_pts2d[b] ([cap][2]), d_count[b] valid
 * points, frame_index j, rows into d_rows[b] ([cap][4]).  One call for the
 * whole batch, the same results as n_win * n slam_map_associate calls: pair j
 * of every window runs in one launch pair (2n launches instead of 2 n n_win);
 * workspace n_win * slam_map_workspace_bytes(cap, (n - 1) * cap). */
int slam_map_windows(double* d_maps, int32_t* d_M, int map_cap, int n_win, int n,
                     const double* d_abs, const double* d_rel, const double* d_pts2d,
                     const int32_t* d_count, int cap, double threshold, double* d_rows,
                     void* d_ws, size_t ws_size, void* stream);

/* ------------------------------------------------------------------------
 * Tiled ORB detector + rBRIEF descriptor.
 *
 * Replaces orb_detector_using_tiles (/root/reference/orb.py:4-25), i.e. the
 * per-patch cv2.ORB_create(nfeatures=max_kp, scaleFactor=1.2).detect() +
 * .compute() of orb_extraction_detect (orb.py:28-38), with the OpenCV 4.x ORB
 * semantics restated in oracle/orb.c (bit-exact against it; canonical keypoint
 * order: level, Harris response desc, y, x).  Tiles follow orb.py exactly:
 * tile_h = int(H/height_div), tile_w = int(W/width_div), patches of
 * int(tile + tile/overlap_div) starting at every multiple of the tile size
 * below H - tile_h (resp. W - tile_w), clipped to the image.
 * height_div == width_div == 0 runs ORB on the whole image as one patch
 * (orb_extraction_detect itself); patches must fit the 160 KiB LDS budget.
 *
 *   d_img   [batch][H][stride] u8
 *   d_kp    [batch][kp_cap][5] f32  (x, y, size, angle [deg], response)
 *   d_octave[batch][kp_cap] i32, d_desc [batch][kp_cap][32] u8
 *   d_count [batch] i32: number of keypoints, or -(n)-1 on overflow
 *   d_ws    workspace of slam_orb_workspace_bytes(...) bytes
 * ---------------------------------------------------------------------- */
int slam_orb_workspace_bytes(int batch, int H, int W, int max_kp, int overlap_div,
                             int height_div, int width_div, size_t* bytes);
int slam_orb_tiles(const uint8_t* d_img, int batch, int H, int W, int stride, int max_kp,
                   int overlap_div, int height_div, int width_div, void* d_ws,
                   size_t ws_bytes, float* d_kp, int32_t* d_octave, uint8_t* d_desc,
                   int32_t* d_count, int kp_cap, void* stream);

/* ------------------------------------------------------------------------
 * Bundle adjustment (BAL model) — replaces the reference's BAL block
 * /root/reference/BundleAdjustment.py:287-402 (rotate / project / objective /
 * bundle_adjustment_sparsity / least_squares TRF) with Levenberg-Marquardt on
 * the normal equations: analytic 2x12 Jacobian per observation; per point
 * group (whole points, <= 128 observations) the point blocks are eliminated and
 * the group's share of the reduced camera system (camera Grams U - sum Y W^T,
 * off-diagonal sums Y W^T, Jc^T r, Jc^T u) is written as slot partials that a
 * second launch sums per block in group order (deterministic); blocked LDL^T
 * of the reduced camera system.
 *
 * Camera layout per row: [r0 r1 r2 t0 t1 t2 f k1 k2] (BundleAdjustment.py:324).
 * ---------------------------------------------------------------------- */

/* objective() residuals (BundleAdjustment.py:331-369) in the caller's
 * observation order: d_resid [n_obs][2] (= the reference's ravel order).
 * Indices must be in range (checked by the host wrapper). */
int slam_ba_residual(const double* d_cams, const double* d_pts, const int32_t* d_cam_idx,
                     const int32_t* d_pt_idx, const double* d_qs, int n_obs,
                     double* d_resid, void* stream);

/* Per-observation residual and Jacobian (clamped like objective()):
 * d_jac [n_obs][2][12] columns [w0 w1 w2 t0 t1 t2 f k1 k2 | X0 X1 X2]. */
int slam_ba_jacobian(const double* d_cams, const double* d_pts, const int32_t* d_cam_idx,
                     const int32_t* d_pt_idx, const double* d_qs, int n_obs,
                     double* d_resid, double* d_jac, void* stream);

/* LM state slots (doubles in slam_ba_problem.state). */
#define SLAM_BA_ST_LAMBDA 0
#define SLAM_BA_ST_NU 1
#define SLAM_BA_ST_COST 2      /* 0.5*|r|^2 at the live parameters           */
#define SLAM_BA_ST_COST_NEW 3  /* 0.5*|r|^2 at the last trial step            */
#define SLAM_BA_ST_PRED 4      /* predicted reduction of the last trial step   */
#define SLAM_BA_ST_RHO 5
#define SLAM_BA_ST_ACCEPTED 6  /* 1 if the last trial step was accepted        */
#define SLAM_BA_ST_CUR 7       /* which of the two parameter buffers is live   */
#define SLAM_BA_ST_ITERS 8
#define SLAM_BA_ST_NACCEPT 9
#define SLAM_BA_ST_PRED_CAM 10
#define SLAM_BA_ST_CHOL_FAIL 11 /* last solve: 0 ok, 1 not SPD, 2 dataflow solve timed out */
/* slots 12..15: phase timers of the profiling builds (SLAM_LIN_PROFILE,
 * SLAM_SOLVE_PROFILE; scripts/ba_solve_prof.py reads state[12:16]); slots 18, 19:
 * the per-panel timers of SLAM_SOLVE_PROFILE_PANEL (scripts/solve_trace.py) */
#define SLAM_BA_ST_SOLVE_FAULT 16 /* sticky: camera solves whose dataflow wait timed out
                                     * (fail code 2: a hang or a hand-off ordering bug --
                                     * the solve needs no co-residency, so a correct build
                                     * never sets it; the Python layer raises when non-zero) */
#define SLAM_BA_ST_SLOTS 20

/* Everything the LM iteration touches; all pointers are device pointers.
 * Built by the host planner (slam355/ba.py): observations sorted by
 * (point, camera); index tables are fixed for the life of a problem. */
typedef struct slam_ba_problem {
  int32_t n_cams, n_pts, n_obs;
  int32_t n_grps;        /* point groups (>= 1): <= 128 obs / points each     */
  int32_t n_blocks;      /* upper camera-pair blocks of S: all C(C+1)/2 when
                            9C <= 120, else the diagonal + every pair with a
                            common point (across all ranks), sorted          */
  int32_t n_cslots;      /* (group, camera) slots                             */
  int32_t n_bslots;      /* (group, camera-pair block) slots                  */
  int32_t lin_mode;      /* 0: slot linearisation (k_linearize; groups = point
                            groups); 1: camera-union linearisation
                            (k_lin_mfma; grp_* = chunks, slots per supergroup) */
  int32_t n_sgrps;       /* lin_mode 1: supergroups (>= 1)                    */
  int32_t tl_mode;       /* tiled solve with tl_sched: 0 dataflow (k_tl3_flow,
                            one persistent workgroup per tile column, when the
                            schedule has <= SLAM_TL_FLOW_MAX_T columns), 1 one
                            launch pair per elimination-tree level           */
  double* cams[2];              /* [C][9]  double-buffered, state[CUR] is live */
  double* pts[2];               /* [P][3]                                      */
  double* camrec[2];            /* [C][32] per-camera projection records of cams[] */
  const int32_t* obs_cam;       /* [O] (sorted by point, then camera)          */
  const int32_t* obs_pt;        /* [O]                                         */
  const double* obs_q;          /* [O][2]                                      */
  const int32_t* pt_ptr;        /* [P+1] CSR point -> obs                      */
  const int32_t* grp_ptr;       /* [n_grps+1] point range of each point group  */
  const int32_t* grp_cslot;     /* [n_grps+1] camera-slot range of each group  */
  const int32_t* cslot_cam;     /* [n_cslots] camera of each slot              */
  const int32_t* cslot_obs_ptr; /* [n_cslots+1] range in cslot_obs             */
  const int32_t* cslot_obs;     /* [O] group-local obs indices, slot by slot   */
  const int32_t* grp_bslot;     /* [n_grps+1] block-slot range of each group   */
  const int32_t* bslot_blk;     /* [n_bslots] upper block index (c1 <= c2)     */
  const int32_t* bslot_pair_ptr;/* [n_bslots+1] range in bslot_pairs           */
  const int32_t* bslot_pairs;   /* group-local o1 | o2 << 16, o1 < o2 of one point */
  const int32_t* blocks;        /* [n_blocks][2] (c1 <= c2), every upper block */
  const int32_t* cam_cslot_ptr; /* [C+1] camera -> its rows of cpart            */
  const int32_t* cslot_row;     /* [n_cslots] row of a camera slot in cpart (camera-major, group order) */
  const int32_t* blk_bslot_ptr; /* [n_blocks+1] block -> its rows of bpart (empty: no common point) */
  const int32_t* bslot_row;     /* [n_bslots] row of a block slot in bpart (block-major, group order) */
  double* cpart;                /* [n_cslots][112] U - sum Y W^T (81), Jc^T r, Jc^T u, diag U (9 each), |r|^2 */
  double* bpart;                /* [n_bslots][81] sum Y W^T                    */
  double* sys;                  /* S (dense or packed blocks) b[9C] g[9C] diagU[9C] cost[C] */
  double* chol;                 /* [slam_ba_chol_len] (9C > 120 only)           */
  double* delta_c;              /* [9C]                                        */
  double* red_part;             /* [slam_ba_red_slots(n_grps)]                 */
  double* small;                /* [4] trial |r|^2, sum pred_p (all-reduced)   */
  double* state;                /* [SLAM_BA_ST_SLOTS]                          */
  uint32_t* ticket;             /* [1] zero-initialised completion counter     */
  /* lin_mode 1 only (else may be null): points renumbered by camera span;
   * grp_ptr = chunks (<= 128 obs, <= 16 points); grp_cslot / grp_bslot are
   * indexed by supergroup. */
  const int32_t* sg_ptr;        /* [n_sgrps+1] chunk range of each supergroup    */
  const int32_t* sg_meta;       /* [n_sgrps][24] ch0 ch1 (chunk range), cslot start, m
                                   (cameras), bslot start, count, the first chunk's
                                   point and obs range, its cameras[8] (<= 7, sorted,
                                   -1 padded), pad                              */
  const int32_t* obs_meta;      /* [O] lpt | la << 8 | cobs << 16: chunk-local point,
                                   position of the obs's camera in sg_cams, and the
                                   chunk-local obs list sorted by (la, obs)      */
  const int32_t* chk_optr;      /* [n_grps+1] first observation of each group /
                                   chunk (= pt_ptr[grp_ptr]); required in both modes */
  const int32_t* chk_cptr;      /* [n_grps][8] start of each camera's run in chk_cobs */
  const int32_t* bslot_ab;      /* [n_bslots] camera pair a | b << 8 (a < b) of a block slot */
  /* Level schedule of the tiled solve (required when 9C > 120), built by
   * slam355/ba.py tl_schedule: tiles of whole cameras (64-row tiles, the rows
   * past a tile's cameras padding) in nested-dissection order, with the row
   * maps between S and the tiled system, columns grouped by elimination-tree
   * level, the dataflow solve's column table, epilogue and gather tables and
   * its product task table (12-int header; the layout is tl_schedule's and is
   * checked by the launcher).
   * tl_sched is the device copy, tl_sched_host the same array in host memory
   * (the launcher reads the level counts from it); both or neither. The
   * workspace `chol` is sized from it: slam_ba_chol_len(n_cams, tl_sched_host). */
  const int32_t* tl_sched;
  const int32_t* tl_sched_host;
  /* lin_mode 1, optional (null: the separate k_assemble launch): the assembly
   * folded into k_lin_mfma -- the supergroup that writes the LAST partial row
   * of a block sums that block's rows (deterministic order) into sys.  int32:
   * need[n_blocks] (partial rows per block), cnt[n_blocks] (zero-initialised;
   * re-armed by the assembler), cam_dblk[C] (diagonal block of each camera),
   * row_blk[n_bslots] (block of each bpart row), n_empty, empty[n_empty]
   * (blocks with no partial row here: zeroed every build). */
  int32_t* asm_tab;
  /* Optional (null: all n_blocks): the blocks this problem's assembly runs
   * over -- those with partial rows here (a landmark shard touches few of the
   * global list): asm_act[n_asm_act] ascending block indices, then a 0/1 flag
   * per block (listed or not) and a 0/1 flag per camera (its diagonal block
   * listed).  Those workgroups also write the zeros of the unlisted blocks (S
   * -0.0, and b, g -0.0 / diag U, cost +0.0 for a camera without rows: what
   * the assembly writes for them, up to the sign of a zero on the diagonal of
   * a camera this rank does not observe).  Packed systems (9C > 120) without
   * asm_tab only; n_asm_act >= 1. */
  const int32_t* asm_act;
  int32_t n_asm_act;
  int32_t asm_pad;
} slam_ba_problem;

/* Largest tile count (tl_sched[1]) the dataflow tiled solve takes: one
 * persistent workgroup per tile column (they need not all be resident). */
#define SLAM_TL_FLOW_MAX_T 256

/* Problems per batched launch (slam_ba_iterate_batch splits larger batches).
 * The descriptors travel by value in the kernel arguments: 16 x 376 B
 * (ba.hip static_asserts the size; ROCm 7.2 takes this > 4 KB argument
 * segment, exercised by tests/test_ba.py's 16-window launch). */
#ifndef SLAM_BA_MAX_BATCH
#define SLAM_BA_MAX_BATCH 16
#endif

/* ---- host planner of the camera-union linearisation (lin_mode 1) ----------
 * slam355/ba.py plan_mfma in native code (the same tables, element for
 * element; no HIP call, callable without a GPU): observations sorted by
 * (point, camera), points renumbered by camera span, chunks of <= 120
 * observations / 16 points, supergroups of <= chunks_per_wg chunks seeing
 * <= 7 cameras.  Replaces the Python planner that BundleAdjustment-style
 * callers (BundleAdjustment.py:331-402 via slam355.ba.BAProblem) pay per
 * window.  The tables go into one int32 buffer `out`, table k at info->off[k]
 * (256-byte aligned), info->len[k] entries; sizes in info.  info->ok = 0
 * (and SLAM_OK) when a point has > 120 observations or > 7 cameras: the slot
 * linearisation (lin_mode 0) applies.  chunks_per_wg <= 0: the default rule
 * of plan_mfma.  block_list (packed layout, 9C > 120; may be null): the
 * upper blocks to list, as BAProblem's block_list.  Null means "the problem's
 * own blocks"; a non-null pointer with n_block_list == 0 is an explicitly empty
 * list and fails like any list that misses a block (plan_mfma raises alike). */
enum {
  SLAM_PLAN_PERM = 0,      /* [P] device point k = caller's point perm[k]      */
  SLAM_PLAN_ORDER,         /* [O] observation order (qs[order] -> obs_q)       */
  SLAM_PLAN_OBS_CAM, SLAM_PLAN_OBS_PT, SLAM_PLAN_PT_PTR, SLAM_PLAN_GRP_PTR,
  SLAM_PLAN_GRP_CSLOT, SLAM_PLAN_CSLOT_CAM, SLAM_PLAN_GRP_BSLOT, SLAM_PLAN_BSLOT_BLK,
  SLAM_PLAN_BLOCKS, SLAM_PLAN_CAM_CSLOT_PTR, SLAM_PLAN_CSLOT_ROW, SLAM_PLAN_BLK_BSLOT_PTR,
  SLAM_PLAN_BSLOT_ROW, SLAM_PLAN_SG_PTR, SLAM_PLAN_SG_META, SLAM_PLAN_SG_CAMS,
  SLAM_PLAN_OBS_LA, SLAM_PLAN_CHK_COBS, SLAM_PLAN_OBS_META, SLAM_PLAN_CHK_OPTR,
  SLAM_PLAN_CHK_CPTR, SLAM_PLAN_BSLOT_AB,
  SLAM_PLAN_NTAB
};
typedef struct slam_ba_plan_info {
  int32_t ok, n_obs, n_grps, n_sgrps, n_cslots, n_bslots, n_blocks, chunks_per_wg;
  long long off[SLAM_PLAN_NTAB], len[SLAM_PLAN_NTAB];
  long long total;  /* int32 slots written */
} slam_ba_plan_info;
/* int32 slots `out` needs for any plan of this size (0 on bad sizes). */
long long slam_ba_plan_bound(int n_cams, int n_pts, int n_obs, int n_block_list);
int slam_ba_plan_mfma(int n_cams, int n_pts, int n_obs, const int32_t* cam_idx,
                      const int32_t* pt_idx, const int32_t* block_list, int n_block_list,
                      int chunks_per_wg, int32_t* out, long long out_cap,
                      slam_ba_plan_info* info);

/* Host staging of a batch of tracked local-BA windows (the tracked leg's
 * host side in one call; replaces a Python loop over windows, buffers and plan
 * tables -- main.py:120-127 / XXXport_files.py:44-64 build the reference's BA
 * arguments from the local map).  Window w = frames w n .. w n + n - 1 (one
 * camera each, parameters cams[w n + j][9]); observations = the first cnt[b]
 * rows (frame j, map point, u, v) of rows[b][cap][4] for its pairs b, q = (u -
 * u_off, v - v_off); points = maps[w][0 .. M[w])[3].  Each window is planned
 * (slam_ba_plan_mfma) and, when the plan exists and 9n <= 120, its float64
 * data (BAProblem's layout: cams0 pts0 cams1 pts1 init_c init_p obs_q, then
 * zeroed camrec0 camrec1 cpart bpart sys chol delta_c red_part small state,
 * each 32-double aligned) go to h64 and its plan tables (+ 8 zero int32:
 * stand-ins, ticket) to h32; probs[w] gets the device addresses of those
 * buffers at d64 / d32.  meta[w][SLAM_STAGE_META]: staged (0: the caller builds
 * that window itself), C, P, O, n_grps, n_sgrps, n_cslots, n_bslots, n_blocks,
 * int32 offset, plan length, sys length, the SLAM_STAGE_NF64 float64 offsets,
 * the SLAM_PLAN_NTAB table offsets.  need[2] = doubles / int32 used; with
 * null outputs, or when they exceed cap64 / cap32, only sizes and meta are
 * produced (grow the buffers and call again). */
#define SLAM_STAGE_NF64 17
#define SLAM_STAGE_META (12 + SLAM_STAGE_NF64 + SLAM_PLAN_NTAB)
int slam_ba_stage_windows(int n_win, int n, int cap, const double* rows, const int32_t* cnt,
                          const double* maps, int map_cap, const int32_t* M, const double* cams,
                          double u_off, double v_off, double* h64, long long cap64, int32_t* h32,
                          long long cap32, const void* d64, const void* d32,
                          slam_ba_problem* probs, long long* meta, long long* need);

/* Number of doubles red_part needs for a problem with n_grps point groups. */
int slam_ba_red_slots(int n_grps);
/* Doubles of the tiled-Cholesky workspace `chol` (needed only when 9C > 120)
 * for a tile schedule (the host copy tl_sched_host, slam355/ba.py
 * tl_schedule): its tile count tl_sched_host[1] (a schedule of whole-camera
 * tiles may have more tiles than 9C / 64) and its product slots
 * tl_sched_host[11] (the 64x64 terms L_Ik L_Jk^T that column k forms for
 * column J's first two row tiles).  NULL: ceil(9C / 64) tiles, no slots. */
long long slam_ba_chol_len(int n_cams, const int32_t* tl_sched_host);
/* Doubles in the all-reduced system buffer `sys`: dense (9C <= 120) (9C)^2,
 * packed (9C > 120) 81 * n_blocks (the listed upper camera blocks), then
 * b, g, diag U (9C each) and the per-camera cost (C). */
long long slam_ba_sys_len(int n_cams, int n_blocks);

/* Phase 1 (per rank): linearise at the live parameters and build this
 * rank's share of the reduced camera system into prob->sys. */
int slam_ba_build_system(const slam_ba_problem* prob, void* stream);
/* Phase 2 (after sys is summed over ranks): damp, Cholesky-solve for the
 * camera step, back-substitute the point step, evaluate the trial cost
 * partial sums into prob->small. */
int slam_ba_solve_step(const slam_ba_problem* prob, void* stream);
/* Phase 3 (after small is summed over ranks): LM accept/reject, lambda update. */
int slam_ba_decide(const slam_ba_problem* prob, void* stream);
/* Single-rank convenience: n_iter x (phase 1, 2, 3) with no host sync. */
int slam_ba_iterate(const slam_ba_problem* prob, int n_iter, void* stream);
/* Reset the LM state: lambda0, nu = 2, cur = 0, counters = 0. */
int slam_ba_reset(const slam_ba_problem* prob, double lambda0, void* stream);
/* Batched local BA: n_probs independent problems (e.g. the local-BA windows
 * of a tracking batch; the reference solves one BAL problem per call,
 * BundleAdjustment.py:397-402) advance n_iter LM iterations through shared
 * launches, up to SLAM_BA_MAX_BATCH problems per launch (one problem per
 * grid row).  Every problem keeps its own buffers and LM state: its iterates
 * are the ones slam_ba_iterate gives it alone.  Batched problems must use the
 * one-workgroup solver (9C <= 120); a packed problem iterates on its own. */
int slam_ba_iterate_batch(const slam_ba_problem* probs, int n_probs, int n_iter, void* stream);

/* Minimum dynamic LDS (bytes, <= 160 KiB) the one-workgroup camera solve
 * (9C <= 120) requests; 0 (default) = what it needs.  A floor above what
 * co-resident workgroups of other streams leave (e.g. > 80 KiB beside an ORB
 * workgroup) keeps its latency-bound pivot chain on CUs of its own.  Process-wide;
 * takes effect at the next launch (and is baked into graphs captured after). */
int slam_ba_set_solve_lds_floor(int bytes);

/* Minimum dynamic LDS (bytes, <= 160 KiB) k_orb_tile requests; 0 (default) =
 * what the patch needs (~79 KiB at C2: two workgroups per CU).  Between 80 and
 * ~80.6 KiB one ORB workgroup per CU leaves room for one local-BA
 * linearisation workgroup beside it.  Process-wide (A/B experiments). */
int slam_orb_set_lds_floor(int bytes);

/* *d_min = min(*d_min, d_count[0..n)) on the device (the Tracker's running
 * minimum of slam_orb_tiles' counts: a negative count flags an overflow), with
 * no host round trip. */
int slam_count_min(const int32_t* d_count, int n, int32_t* d_min, void* stream);
int slam_ba_reset_batch(const slam_ba_problem* probs, int n_probs, double lambda0, void* stream);

/* ------------------------------------------------------------------ collectives
 * The sharded local BA (replaces the one serial least_squares
 * call of BundleAdjustment.py:397-402 at C4 / C5 scale): each rank holds the
 * observations of its landmark shard and all cameras; per LM iteration the
 * packed reduced camera system and the 4-double trial buffer are summed over
 * the ranks.  RCCL (over xGMI) is loaded at the first slam_comm_* call
 * (dlopen "librccl.so.1", or SLAM_RCCL_LIB, or an RCCL already exporting the
 * nccl* symbols globally).  One rank per GPU; the communicator is used from
 * one host thread at a time. */
#define SLAM_COMM_ID_BYTES 128
typedef struct slam_comm_opaque* slam_comm_t;
/* Rank 0 creates the id (h_id: SLAM_COMM_ID_BYTES host bytes) and sends it to
 * the other ranks out of band (torch.distributed broadcast, MPI, a file). */
int slam_comm_unique_id(void* h_id);
/* Collective over the nranks processes (ncclCommInitRank); the current HIP
 * device is this rank's GPU. */
int slam_comm_init(int nranks, int rank, const void* h_id, slam_comm_t* comm);
int slam_comm_destroy(slam_comm_t comm);
/* In-place sum over the ranks of d_buf[0..n) (f64), async on stream. */
int slam_comm_allreduce_f64(slam_comm_t comm, double* d_buf, long long n, void* stream);
/* One LM iteration of a landmark-sharded problem (every rank calls it on its
 * shard; prob built with the GLOBAL problem's packed block list): phase 1,
 * all-reduce of prob->sys (slam_ba_sys_len doubles), phase 2, all-reduce of
 * prob->small (4 doubles), phase 3 -- all on `stream`, no host sync.  With
 * nranks = 1 it equals slam_ba_iterate(prob, 1, stream). */
int slam_ba_step_distributed(const slam_ba_problem* prob, slam_comm_t comm, void* stream);

/* ------------------------------------------------------------------ pose chain
 * The live pose-chain optimisation of BundleAdjustment.py:79-183 (loop
 * closure): m relative poses [r0 r1 r2 t0 t1 t2] (cv2.Rodrigues rotation
 * vector, translation), residuals f_i (weighted |.| of the six parameters,
 * :114-127) and, with loop != 0, the two loop-closure residuals of the chained
 * absolute pose (:128-134).  All pointers are device pointers. */

/* resid[v][m (+2)] = objective(params[v]) (or objective_without_loop_closure
 * when loop == 0) for n_vec parameter vectors params[v][6m]; each vector's
 * chain product runs in the reference's order.  Replaces objective /
 * objective_without_loop_closure, BundleAdjustment.py:79-145. */
int slam_pose_chain_objective(const double* params, int n_vec, int n_frames, int loop,
                              double* resid, void* stream);
/* Doubles of the LM workspace for m frames (the live parameters sit at its
 * start: ws[0 .. 6m)). */
long long slam_pose_chain_workspace_len(int n_frames);
/* scipy's TRF (least_squares method='trf', x_scale='jac', 'exact' trust-region
 * subproblem) on ws[0 .. 6m) in place, one workgroup, at most max_iter outer
 * iterations per call (first != 0 starts the run: scale, Delta; else it
 * resumes from state).  Analytic Jacobian; the subproblem's SVD solves are
 * replaced by the O(m) arrow-structured dual system.  m <= 512: every frame's
 * state in the registers of one thread (k_chain_trf_r); larger m: the LDS /
 * workspace form (environment SLAM_CHAIN_TRF=lds selects it for any m).  state[16]: cost0, cost,
 * nfev, njev, status (0 running, 1 gtol, 2 ftol, 3 xtol, 4 ftol+xtol), Delta,
 * alpha, iterations.  Replaces least_squares(objective, ..., method='trf') of
 * bundle_adjustment_with_sparsity, BundleAdjustment.py:179-183. */
int slam_pose_chain_trf(double* ws, int n_frames, int loop, int max_iter, int first, double ftol,
                        double xtol, double gtol, int max_nfev, double* state, void* stream);

/* ------------------------------------------------------------------ BoW
 * Bag-of-words place recognition (bag_of_words.py).  Descriptors are ORB rows
 * (32 bytes, used as float64 features as scikit-learn converts them); K <= 128
 * clusters, centres [K][32] f64.  All pointers are device pointers. */

/* Labels (nearest centre, argmin |c|^2 - 2 x.c, first index on ties) and label
 * histograms hist[n_img][K] of desc[n_img][cap][32] with count[n_img] rows
 * each (count null: n_each rows each); labels may be null.  Replaces
 * BoW.hist (bag_of_words.py:24-27: kmeans.predict + np.histogram). */
int slam_bow_histograms(const uint8_t* desc, const int32_t* count, int n_each, int n_img, int cap,
                        const double* centers, int n_clusters, int32_t* labels, int32_t* hist,
                        void* stream);
/* For each query histogram q: argmin / min over database rows [0, n_db[q]) of
 * sum 2 (x - y)^2 / max(1, x + y) (numpy's summation order; first index on
 * ties; n_db <= 0 -> (-1, -1)).  Replaces the chi2 loop + np.argmin/np.min of
 * BoW.predict_previous / predict (bag_of_words.py:30-56). */
int slam_bow_query(const int32_t* qhist, int n_query, const int32_t* db, const int32_t* n_db,
                   int n_clusters, int32_t* idx, double* val, void* stream);
/* n_iter Lloyd iterations (E-step, then centres = means; an empty cluster keeps
 * its centre) on X[n_points][32] in place on centers (centers_tmp: [K][32]
 * scratch), then labels of the final centres; shift[K] (optional) = squared
 * centre shift of the last iteration.  Replaces KMeans.fit's Lloyd loop
 * (bag_of_words.py:20). */
int slam_bow_lloyd(const uint8_t* X, int n_points, double* centers, double* centers_tmp,
                   int n_clusters, int n_iter, int32_t* labels, double* shift, void* stream);

/* ---------------------------------------------------------------------------
 * Alternative stereo-VO front end: FAST on tiles,
 * pyramidal Lucas-Kanade, semi-global block matching, disparity lookup and
 * float32 triangulation (csrc/vofront.hip; semantics in oracle/vofront.c).
 * ------------------------------------------------------------------------- */

/* Workspace bytes of slam_fast_tiles. */
int slam_fast_tiles_workspace_bytes(int batch, int H, int W, int tile_h, int tile_w, int per_tile,
                                    size_t* bytes);
/* FAST-9/16 (threshold, strict 3x3 NMS) on every tile_h x tile_w tile of
 * img[batch][H][stride]; per tile the detection-order corners, or the first
 * per_tile of a stable sort by response when there are more; tiles row-major.
 * kp[batch][kp_cap][3] f32 (x, y, response), count[batch] (-n-1 if > kp_cap).
 * Replaces VisualOdometry.get_tiled_keypoints (visual_odometry.py:84-96:
 * cv2.FastFeatureDetector_create().detect per tile, sorted(...)[:10]). */
int slam_fast_tiles(const uint8_t* d_img, int batch, int H, int W, int stride, int tile_h,
                    int tile_w, int threshold, int per_tile, void* d_ws, size_t ws_bytes,
                    float* d_kp, int32_t* d_count, int kp_cap, void* stream);

/* Levels actually used and bytes of one image's LK pyramid (the derivative
 * buffer of one image holds img_bytes int16x2 elements). */
int slam_lk_pyramid_layout(int H, int W, int win, int max_level, int* nlev, size_t* img_bytes);
/* Pyramids (pyrDown levels with a reflect-101 border of win+1) of n_img images
 * into d_pyr[n_img][img_bytes]; if d_deriv is not null, also their Scharr
 * derivatives (zero border) into d_deriv[n_img][img_bytes][2].  The pyramid
 * half of cv2.calcOpticalFlowPyrLK (visual_odometry.py:100, keypoint.py:19). */
int slam_lk_build_pyramids(const uint8_t* d_img, int n_img, int H, int W, int stride, int win,
                           int max_level, uint8_t* d_pyr, int16_t* d_deriv, void* stream);
/* Pyramidal LK for pair b = (prev image b * pair_stride_imgs of d_prev_pyr /
 * d_prev_deriv, next image b * pair_stride_imgs of d_next_pyr): points
 * pts[batch][cap][pts_stride] (x, y first), npts[batch] ->
 * out[batch][cap][2], status[batch][cap], err[batch][cap] (mean |diff|).
 * Replaces cv2.calcOpticalFlowPyrLK(img1, img2, pts, None, winSize=(win,win),
 * maxLevel, criteria=(EPS|COUNT, max_count, eps)) (visual_odometry.py:26-29,100). */
int slam_lk_track(const uint8_t* d_prev_pyr, const int16_t* d_prev_deriv, const uint8_t* d_next_pyr,
                  long long pair_stride_imgs, int batch, int H, int W, int win, int max_level,
                  int max_count, double eps, float min_eig, const float* d_pts, int pts_stride,
                  const int32_t* d_npts, int cap, float* d_out, uint8_t* d_status, float* d_err,
                  void* stream);
/* The filters after the LK call, order-preserving: status, err < max_error,
 * np.around(p2) inside (y < H, x < W; also > 0 when lower_bounds) ->
 * tp1/tp2[batch][cap][2] f32, idx (source index, may be null), count[batch].
 * Replaces visual_odometry.py:102-112 (lower_bounds 0) and keypoint.py:20-32
 * (lower_bounds 1). */
int slam_lk_filter(const float* d_p1, int p1_stride, const float* d_p2, const uint8_t* d_status,
                   const float* d_err, const int32_t* d_npts, int cap, int batch, int H, int W,
                   float max_error, int lower_bounds, float* d_tp1, float* d_tp2, int32_t* d_idx,
                   int32_t* d_count, void* stream);

/* Workspace bytes of slam_sgbm. */
int slam_sgbm_workspace_bytes(int batch, int H, int W, int min_disp, int num_disp, int block,
                              size_t* bytes);
/* Semi-global block matching (MODE_SGBM, 5 directions, BT cost on the
 * Sobel-prefiltered and raw images, uniqueness 0, left-right check 1, 3x3
 * median) of left/right[batch][H][stride] -> disp[batch][H][W] int16 (x16) and,
 * if not null, disp_f32 = disp / 16.  num_disp 32 or 64, min_disp in [0, 64].
 * Replaces cv2.StereoSGBM_create(...).compute(l, r) (visual_odometry.py:22-24,191). */
int slam_sgbm(const uint8_t* d_left, const uint8_t* d_right, int batch, int H, int W, int stride,
              int min_disp, int num_disp, int block, int P1, int P2, void* d_ws, size_t ws_bytes,
              int16_t* d_disp, float* d_disp_f32, void* stream);
/* calculate_right_qs + calc_3d for pair b (visual_odometry.py:114-134): disp1 =
 * d_disp + b * disp1_stride, disp2 = disp1 + disp2_offset (f32 maps [H][W]);
 * (int) truncation and NumPy's negative-index wrap; min_disp < d < max_disp;
 * q*_r = q*_l - (d, 0); Q1/Q2 = f32 homogeneous DLT points divided in f32.
 * Optional f64 copies (q1l64/q2l64, Q1_64/Q2_64, in pairs) feed
 * slam_vo_estimate_pose. */
int slam_vo_right_qs_3d(const float* d_tp1, const float* d_tp2, const int32_t* d_cnt, int cap,
                        int batch, const float* d_disp, long long disp1_stride,
                        long long disp2_offset, int H, int W, float min_disp, float max_disp,
                        const double* d_Pl, const double* d_Pr, float* d_q1l, float* d_q1r,
                        float* d_q2l, float* d_q2r, float* d_Q1, float* d_Q2, double* d_q1l64,
                        double* d_q2l64, double* d_Q1_64, double* d_Q2_64, int32_t* d_count,
                        void* stream);
/* cv2.triangulatePoints on float32 points (the homogeneous result in float32)
 * followed by Q[:3] / Q[3] in float32 (calc_3d, visual_odometry.py:129-134):
 * ptl/ptr[batch][cap][2] f32, count[batch] -> X[batch][cap][3] f32. */
int slam_triangulate_f32(const float* d_ptl, const float* d_ptr, const int32_t* d_count, int cap,
                         int batch, const double* d_Pl, const double* d_Pr, float* d_X,
                         void* stream);

#ifdef __cplusplus
}
#endif

#endif /* SLAM355_H */
