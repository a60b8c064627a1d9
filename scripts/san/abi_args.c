/* Host-side sanitizer driver for the C ABI (test infrastructure only).
 *
 * Linked against objects built with `hipcc -Xarch_host -fsanitize=address,undefined`
 * (scripts/san/build_abi_asan.sh): the host half of libslam355 (argument checks,
 * workspace arithmetic, error-string formatting, BA batch validation) runs
 * under ASan/UBSan; device code is compiled normally.  Every call below must be
 * rejected with SLAM_ERR_ARG (and a non-empty slam_last_error) BEFORE anything
 * is launched, or be a pure size query; the pointers handed in are host
 * scratch that no kernel may ever see.  Refuses to run where a GPU is visible,
 * so a validation hole can never turn into a launch on host memory. */
#include <stdint.h>
#include <stdio.h>
#include <string.h>

#include "slam355.h"

static int fails = 0, checks = 0;
static unsigned char scratch[1 << 16];
#define P ((void*)scratch)

static void expect_rc(int rc, int want, const char* what) {
  ++checks;
  const char* e = slam_last_error();
  if (rc != want || !e || !*e) {
    fprintf(stderr, "FAIL %s: rc=%d err='%s'\n", what, rc, e ? e : "(null)");
    ++fails;
  }
}
static void expect_arg(int rc, const char* what) { expect_rc(rc, SLAM_ERR_ARG, what); }
static void expect(int ok, const char* what) {
  ++checks;
  if (!ok) {
    fprintf(stderr, "FAIL %s\n", what);
    ++fails;
  }
}

int main(void) {
  if (slam_device_count() != 0) {
    fprintf(stderr, "abi_args: a GPU is visible; this driver runs on the CPU host only\n");
    return 2;
  }
  expect(slam_abi_version() == SLAM355_ABI_VERSION, "abi version");

  /* matcher / gather */
  expect_arg(slam_hamming_knn2(P, P, 10, P, P, 10, -1, P, P, P, NULL), "knn2 batch<0");
  expect_arg(slam_hamming_knn2(NULL, P, 10, P, P, 10, 2, P, P, P, NULL), "knn2 null q");
  expect_arg(slam_hamming_knn2(P, P, -3, P, P, 10, 2, P, P, P, NULL), "knn2 q_cap<0");
  expect_arg(slam_compact_matches(P, P, P, 10, 1, P, 1.0, NULL, P, NULL), "compact null out");
  expect_arg(slam_gather_matches(P, 10, P, 10, P, P, P, P, -1, 1, P, P, P, P, NULL),
             "gather p_cap<0");
  expect_arg(slam_gather_temporal(P, P, 10, P, 10, P, P, 10, 1, NULL, P, P, NULL),
             "temporal null");
  /* epipolar / pose */
  expect_arg(slam_fundamental_lmeds(P, P, P, 16, 1, 0, 0, 0, P, P, P, NULL), "fm n_hyp=0");
  expect_arg(slam_fundamental_lmeds(NULL, P, P, 16, 1, 0, 0, 10, P, P, P, NULL), "fm null");
  expect_arg(slam_filter_pairs(P, P, P, -1, 1, P, P, NULL), "filter cap<0");
  expect_arg(slam_triangulate(P, P, P, 10, 1, P, P, 0, NULL, NULL), "tri null X");
  expect_arg(slam_pnp_ransac(P, P, P, 16, 1, P, 0, 0, 0, 2.0, 10, 10, P, P, P, P, P, 0, NULL),
             "pnp n_hyp=0");
  expect_arg(slam_pnp_ransac(P, P, P, 16, 1, P, 0, 0, 64, 2.0, 10, 10, P, P, P, P, NULL, 384, NULL),
             "pnp null workspace");
  expect_rc(slam_pnp_ransac(P, P, P, 16, 2, P, 0, 0, 64, 2.0, 10, 10, P, P, P, P, P, 767, NULL),
            SLAM_ERR_WORKSPACE, "pnp workspace too short");
  expect_arg(slam_ba_iterate_batch(NULL, 3, 1, NULL), "ba iterate_batch null array");
  expect_arg(slam_ba_reset_batch(NULL, 2, 1e-4, NULL), "ba reset_batch null array");
  expect(slam_pnp_workspace_len(4, 128) == 4LL * 128 * 6, "pnp workspace len");
  expect(slam_pnp_workspace_len(1 << 30, 1 << 30) > 0, "pnp workspace len no int overflow");
  expect_arg(slam_pose_chain(P, P, P, 1, NULL, P, NULL), "pose_chain null state");
  expect_arg(slam_rel_to_abs(P, P, 10, -1, P, P, NULL), "rel_to_abs batch<0");
  {
    size_t b = 0;
    expect_arg(slam_vo_pose_workspace_bytes(-1, 10, &b), "vo ws batch<0");
    expect_rc(slam_vo_estimate_pose(P, P, P, P, P, 10, 1, P, 0, 0, 10, 10, 5, P, P, P, P, P, 0,
                                    NULL),
              SLAM_ERR_WORKSPACE, "vo workspace too small");
    expect_arg(slam_vo_residuals(P, P, P, P, P, P, -2, 1, P, P, NULL), "vo resid cap<0");
  }
  /* map */
  {
    size_t b = 0;
    expect_arg(slam_map_workspace_bytes(-1, 10, &b), "map ws <0");
    expect_arg(slam_map_associate(P, P, 10, 100, P, P, P, P, 1, 0.01, 0, P, P, 0, NULL),
               "map ws too small");
  }
  /* ORB */
  {
    size_t b = 0;
    expect_arg(slam_orb_workspace_bytes(1, 376, 1241, 64, 0, 5, 10, &b), "orb overlap_div=0");
    expect_arg(slam_orb_workspace_bytes(1, -376, 1241, 64, 2, 5, 10, &b), "orb H<0");
    expect_arg(slam_orb_workspace_bytes(1, 376, 1241, 64, 2, 5, 10, NULL), "orb null bytes");
    int rc = slam_orb_workspace_bytes(4, 376, 1241, 64, 2, 5, 10, &b);
    expect(rc == SLAM_OK && b > 0, "orb workspace bytes");
    expect_rc(slam_orb_tiles(P, 4, 376, 1241, 1241, 64, 2, 5, 10, P, b - 1, P, P, P, P, 8192,
                             NULL),
              SLAM_ERR_WORKSPACE, "orb workspace one byte short");
    expect_arg(slam_orb_tiles(P, 4, 376, 1241, 1000, 64, 2, 5, 10, P, b, P, P, P, P, 8192, NULL),
               "orb stride < W");
    expect_arg(slam_orb_workspace_bytes(1 << 20, 1 << 15, 1 << 15, 64, 2, 5, 10, &b) ==
                       SLAM_ERR_ARG
                   ? SLAM_ERR_ARG
                   : (b > (size_t)1 << 40 ? SLAM_ERR_ARG : SLAM_OK),
               "orb huge workspace rejected or exact");
  }
  /* BA */
  {
    slam_ba_problem pr;
    memset(&pr, 0, sizeof pr);
    expect_arg(slam_ba_iterate(NULL, 1, NULL), "ba null problem");
    expect_arg(slam_ba_iterate(&pr, 1, NULL), "ba zero problem");
    pr.n_cams = 5;
    expect_arg(slam_ba_build_system(&pr, NULL), "ba null buffers");
    expect(slam_ba_iterate_batch(&pr, 0, 1, NULL) == SLAM_OK, "ba batch of 0 is a no-op");
    {
      /* more problems than one launch holds: chunked, and every one is checked */
      slam_ba_problem many[SLAM_BA_MAX_BATCH + 1];
      memset(many, 0, sizeof many);
      expect_arg(slam_ba_iterate_batch(many, SLAM_BA_MAX_BATCH + 1, 1, NULL), "ba 9 bad problems");
      expect_arg(slam_ba_reset_batch(many, SLAM_BA_MAX_BATCH + 1, 1e-3, NULL), "ba reset 9 bad");
    }
    expect_arg(slam_ba_reset_batch(&pr, -1, 1e-3, NULL), "ba reset n<0");
    expect_arg(slam_ba_residual(P, P, P, P, P, -1, P, NULL), "ba residual n_obs<0");
    expect_arg(slam_ba_jacobian(P, P, P, P, P, 4, P, NULL, NULL), "ba jacobian null jac");
    int32_t sched40[12] = {1, 40, 0, 0, 0, 0, 0, 0, 0, 0, 0, 3};  /* header only: 40 tiles, 3 slots */
    expect(slam_ba_chol_len(100, NULL) > 0 && slam_ba_chol_len(100, sched40) > slam_ba_chol_len(100, NULL) && slam_ba_sys_len(100, 300) > 0, "ba sizes");
    expect(slam_ba_red_slots(7) >= 1, "ba red slots");
  }
  /* pose graph / BoW */
  expect(slam_pose_chain_workspace_len(100) > 600, "pose chain ws len");
  expect_arg(slam_pose_chain_objective(P, 1, -1, 1, P, NULL), "chain objective m<0");
  expect_arg(slam_pose_chain_trf(NULL, 10, 1, 5, 1, 1e-8, 1e-8, 1e-8, 100, P, NULL),
             "chain trf null ws");
  expect_arg(slam_bow_histograms(P, P, 10, 2, 10, P, 0, P, P, NULL), "bow K=0");
  expect_arg(slam_bow_histograms(P, P, 10, 2, 10, P, 129, P, P, NULL), "bow K>128");
  expect_arg(slam_bow_query(P, 1, P, P, 0, P, P, NULL), "bow query K=0");
  expect_arg(slam_bow_lloyd(P, 100, P, P, 8, -1, P, P, NULL), "lloyd n_iter<0");
  /* VO front end */
  {
    size_t b = 0;
    int nlev = 0;
    expect_arg(slam_fast_tiles_workspace_bytes(1, 376, 1241, 0, 20, 10, &b), "fast tile_h=0");
    expect_rc(slam_fast_tiles(P, 1, 376, 1241, 1241, 10, 20, 20, 10, P, 0, P, P, 100, NULL),
              SLAM_ERR_WORKSPACE, "fast workspace 0");
    expect_arg(slam_lk_pyramid_layout(0, 1241, 15, 3, &nlev, &b), "lk H=0");
    expect(slam_lk_pyramid_layout(376, 1241, 15, 3, &nlev, &b) == SLAM_OK && nlev >= 1 && b > 0,
           "lk layout");
    expect_arg(slam_lk_build_pyramids(NULL, 2, 376, 1241, 1241, 15, 3, P, NULL, NULL), "lk null");
    expect_arg(slam_lk_track(P, P, P, 1, 1, 376, 1241, 15, 3, 30, 0.01, 1e-4f, P, 1, P, -1, P, P,
                             P, NULL),
               "lk cap<0");
    expect_arg(slam_lk_filter(P, 2, P, P, P, P, 10, 1, 376, 1241, 4.f, 0, NULL, P, P, P, NULL),
               "lk filter null");
    expect_arg(slam_sgbm_workspace_bytes(1, 376, 1241, 0, 30, 11, &b), "sgbm num_disp%16");
    expect_arg(slam_sgbm_workspace_bytes(1, 376, 1241, 0, 32, 10, &b), "sgbm even block");
    expect_arg(slam_vo_right_qs_3d(P, P, P, 10, 1, P, 0, 0, 0, 1241, 0.f, 100.f, P, P, P, P, P, P,
                                   P, P, P, NULL, P, P, P, NULL),
               "right_qs H=0 / unpaired f64");
    expect_arg(slam_triangulate_f32(P, P, P, -1, 1, P, P, P, NULL), "tri f32 cap<0");
  }
  expect(strlen(slam_last_error()) < 4096, "error length bounded");

  printf("abi_args: %s (%d checks, %d failed)\n", fails ? "FAIL" : "ok", checks, fails);
  return fails ? 1 : 0;
}
