// Host staging of a batch of tracked local-BA windows (bench.py's tracked leg,
// slam355.ba.BAWindowSet.stage): from the host copies WindowMapper brings back
// (association rows, per-pair counts, per-window maps, the batch's camera
// parameters) to every window's BA problem -- planned by slam_ba_plan_mfma,
// its float64 data and plan tables written into the caller's pinned staging
// buffers in BAProblem's layout, and its slam_ba_problem descriptor filled
// with the device addresses those buffers are uploaded to.  One call per
// batch instead of a Python loop over windows, buffers and tables (the host
// side of the tracked leg: WindowMapper.problems + BAWindowSet.build).
// Pure host code: no HIP call, callable without a GPU.
//
// Window w (frames w n .. w n + n - 1, one BA camera each): its observations
// are the rows (frame j, map point, u, v) of its n pairs in pair order
// (mapping.hip k_map_assoc), q = (u - u_off, v - v_off); its points the first
// M[w] entries of its map.  Reference: main.py:120-127 (local map -> BA
// arguments), XXXport_files.py:44-64 (camera parameters, pixel offsets).
#include "common.hpp"

#include <algorithm>
#include <cstring>
#include <vector>

namespace {
using i64 = long long;
constexpr int kCamRec = 32;   // ba.hip kCamRec
constexpr int kCPart = 112;   // ba.hip kCPart
constexpr int kNState = SLAM_BA_ST_SLOTS;
i64 al32(i64 n) { return (std::max<i64>(n, 1) + 31) / 32 * 32; }  // BAWindowSet._al
}  // namespace

extern "C" int slam_ba_red_slots(int n_grps);
extern "C" long long slam_ba_sys_len(int n_cams, int n_blocks);

extern "C" int slam_ba_stage_windows(int n_win, int n, int cap, const double* rows,
                                     const int32_t* cnt, const double* maps, int map_cap,
                                     const int32_t* M, const double* cams, double u_off,
                                     double v_off, double* h64, long long cap64, int32_t* h32,
                                     long long cap32, const void* d64, const void* d32,
                                     slam_ba_problem* probs, long long* meta, long long* need) {
  SLAM_REQUIRE(n_win >= 0 && n >= 1 && cap >= 0 && map_cap >= 0, "slam_ba_stage_windows: bad sizes");
  SLAM_REQUIRE(rows && cnt && maps && M && cams && meta && need, "slam_ba_stage_windows: null input");
  const bool write = h64 && h32 && d64 && d32 && probs;
  i64 o64 = 0, o32 = 0;
  std::vector<int32_t> ci, pi, plan;
  std::vector<double> qs;
  for (int w = 0; w < n_win; ++w) {
    long long* mt = meta + (size_t)w * SLAM_STAGE_META;
    std::memset(mt, 0, sizeof(long long) * SLAM_STAGE_META);
    const int C = n, P = M[w];
    SLAM_REQUIRE(P >= 0 && P <= map_cap, "slam_ba_stage_windows: window %d has %d map points (cap %d)",
                 w, P, map_cap);
    // observations of the window's pairs, in pair order
    ci.clear();
    pi.clear();
    qs.clear();
    for (int b = w * n; b < (w + 1) * n; ++b) {
      const int k = std::min(std::max(cnt[b], 0), cap);
      const double* r = rows + (size_t)b * cap * 4;
      for (int q = 0; q < k; ++q) {
        const int cam = (int)r[4 * q], pt = (int)r[4 * q + 1];
        SLAM_REQUIRE(cam >= 0 && cam < C && pt >= 0 && pt < P,
                     "slam_ba_stage_windows: window %d row %d indexes camera %d / point %d", w, q,
                     cam, pt);
        ci.push_back(cam);
        pi.push_back(pt);
        qs.push_back(r[4 * q + 2] - u_off);
        qs.push_back(r[4 * q + 3] - v_off);
      }
    }
    const int O = (int)ci.size();
    mt[1] = C;
    mt[2] = P;
    mt[3] = O;
    // the camera-union plan (or none: BAWindowSet builds that window alone)
    const i64 bound = slam_ba_plan_bound(C, P, O, 0);
    SLAM_REQUIRE(bound > 0, "slam_ba_stage_windows: bad plan sizes");
    plan.resize((size_t)bound);
    slam_ba_plan_info info;
    const int rc = slam_ba_plan_mfma(C, P, O, ci.data(), pi.data(), nullptr, 0, 0, plan.data(), bound,
                                     &info);
    if (rc != SLAM_OK) return rc;
    // 9C <= 120: the one-workgroup solve (ba.py LDS_MAX_N)
    if (!info.ok || 9 * C > 120) continue;  // mt[0] = 0: not staged
    const int G = info.n_grps, n_cs = info.n_cslots, n_bs = info.n_bslots, NB = info.n_blocks;
    const i64 sys_len = slam_ba_sys_len(C, NB), red = slam_ba_red_slots(G);
    // float64 layout (BAWindowSet.build): parameters twice, initial copy,
    // observations in plan order, then the zeroed workspaces
    const i64 len64[SLAM_STAGE_NF64] = {9ll * C, 3ll * P, 9ll * C, 3ll * P, 9ll * C, 3ll * P,
                                        2ll * std::max(O, 1), (i64)kCamRec * C, (i64)kCamRec * C,
                                        (i64)kCPart * n_cs, 81ll * n_bs, sys_len, 1, 9ll * C, red, 4,
                                        kNState};
    i64 off64[SLAM_STAGE_NF64];
    for (int k = 0; k < SLAM_STAGE_NF64; ++k) {
      off64[k] = o64;
      o64 += al32(len64[k]);
    }
    const i64 nb = info.total, w32 = o32;
    o32 += al32(nb + 8);  // plan tables, 4 one-element stand-ins, ticket
    mt[0] = 1;
    mt[4] = G;
    mt[5] = info.n_sgrps;
    mt[6] = n_cs;
    mt[7] = n_bs;
    mt[8] = NB;
    mt[9] = w32;
    mt[10] = nb;
    mt[11] = sys_len;
    for (int k = 0; k < SLAM_STAGE_NF64; ++k) mt[12 + k] = off64[k];
    for (int k = 0; k < SLAM_PLAN_NTAB; ++k) mt[12 + SLAM_STAGE_NF64 + k] = info.off[k];
    if (!write || o64 > cap64 || o32 > cap32) continue;  // sizes only (the caller grows and calls again)
    // ---- float64 data
    const int32_t* perm = plan.data() + info.off[SLAM_PLAN_PERM];
    const int32_t* order = plan.data() + info.off[SLAM_PLAN_ORDER];
    const double* cw = cams + (size_t)w * n * 9;
    const double* mp = maps + (size_t)w * map_cap * 3;
    for (int rep = 0; rep < 3; ++rep) {  // cams0 / pts0, cams1 / pts1, init_c / init_p
      std::memcpy(h64 + off64[2 * rep], cw, sizeof(double) * 9 * C);
      double* pd = h64 + off64[2 * rep + 1];
      for (int k = 0; k < P; ++k)
        for (int c = 0; c < 3; ++c) pd[3 * k + c] = mp[3 * (size_t)perm[k] + c];
    }
    double* oq = h64 + off64[6];
    if (O == 0) {
      oq[0] = oq[1] = 0.0;
    } else {
      for (int k = 0; k < O; ++k) {
        oq[2 * k] = qs[2 * (size_t)order[k]];
        oq[2 * k + 1] = qs[2 * (size_t)order[k] + 1];
      }
    }
    for (int k = 7; k < SLAM_STAGE_NF64; ++k) std::memset(h64 + off64[k], 0, sizeof(double) * len64[k]);
    // ---- int32: the plan tables, then zeros (stand-ins of the lin_mode-0 tables, ticket)
    std::memcpy(h32 + w32, plan.data(), sizeof(int32_t) * nb);
    std::memset(h32 + w32 + nb, 0, sizeof(int32_t) * 8);
    // ---- the descriptor, with device addresses
    double* D = reinterpret_cast<double*>(const_cast<void*>(d64));
    int32_t* I = reinterpret_cast<int32_t*>(const_cast<void*>(d32));
    const int32_t* tab = I + w32;
    const int32_t* stand = I + w32 + nb;
    slam_ba_problem& s = probs[w];
    std::memset(&s, 0, sizeof(s));
    s.n_cams = C;
    s.n_pts = P;
    s.n_obs = O;
    s.n_grps = G;
    s.n_blocks = NB;
    s.n_cslots = n_cs;
    s.n_bslots = n_bs;
    s.lin_mode = 1;
    s.n_sgrps = info.n_sgrps;
    s.tl_mode = 0;
    s.cams[0] = D + off64[0];
    s.pts[0] = D + off64[1];
    s.cams[1] = D + off64[2];
    s.pts[1] = D + off64[3];
    s.camrec[0] = D + off64[7];
    s.camrec[1] = D + off64[8];
    s.obs_q = D + off64[6];
    s.cpart = D + off64[9];
    s.bpart = D + off64[10];
    s.sys = D + off64[11];
    s.chol = D + off64[12];
    s.delta_c = D + off64[13];
    s.red_part = D + off64[14];
    s.small = D + off64[15];
    s.state = D + off64[16];
    s.ticket = reinterpret_cast<uint32_t*>(I + w32 + nb + 4);
    s.obs_cam = tab + info.off[SLAM_PLAN_OBS_CAM];
    s.obs_pt = tab + info.off[SLAM_PLAN_OBS_PT];
    s.pt_ptr = tab + info.off[SLAM_PLAN_PT_PTR];
    s.grp_ptr = tab + info.off[SLAM_PLAN_GRP_PTR];
    s.grp_cslot = tab + info.off[SLAM_PLAN_GRP_CSLOT];
    s.cslot_cam = tab + info.off[SLAM_PLAN_CSLOT_CAM];
    s.cslot_obs_ptr = stand;
    s.cslot_obs = stand;
    s.grp_bslot = tab + info.off[SLAM_PLAN_GRP_BSLOT];
    s.bslot_blk = tab + info.off[SLAM_PLAN_BSLOT_BLK];
    s.bslot_pair_ptr = stand;
    s.bslot_pairs = stand;
    s.blocks = tab + info.off[SLAM_PLAN_BLOCKS];
    s.cam_cslot_ptr = tab + info.off[SLAM_PLAN_CAM_CSLOT_PTR];
    s.cslot_row = tab + info.off[SLAM_PLAN_CSLOT_ROW];
    s.blk_bslot_ptr = tab + info.off[SLAM_PLAN_BLK_BSLOT_PTR];
    s.bslot_row = tab + info.off[SLAM_PLAN_BSLOT_ROW];
    s.sg_ptr = tab + info.off[SLAM_PLAN_SG_PTR];
    s.sg_meta = tab + info.off[SLAM_PLAN_SG_META];
    s.obs_meta = tab + info.off[SLAM_PLAN_OBS_META];
    s.chk_optr = tab + info.off[SLAM_PLAN_CHK_OPTR];
    s.chk_cptr = tab + info.off[SLAM_PLAN_CHK_CPTR];
    s.bslot_ab = tab + info.off[SLAM_PLAN_BSLOT_AB];
  }
  need[0] = o64;
  need[1] = o32;
  return SLAM_OK;
}
