// Host planner of the camera-union linearisation (k_lin_mfma's index tables):
// slam355.ba.plan_mfma in native code, the same tables element for element,
// so the planning of a tracked local-BA window costs microseconds instead of a
// Python loop over its points.  Pure host code:
// no HIP call, callable without a GPU.
//
// Observations are sorted by (point, camera); points are renumbered by their
// camera span (first camera, last camera, index), cut greedily into chunks
// (<= kMfChunkObs observations, <= kMfChunkPts points) and the chunks into
// supergroups (<= chunks_per_wg chunks) whose points see at most kMfCams
// distinct cameras.  Every sort below is a stable counting sort, so ties keep
// the order numpy's lexsort gives them.
#include "common.hpp"

#include <algorithm>
#include <cstring>
#include <vector>

namespace {

constexpr int kMfChunkObs = 120;  // slam355.ba.MF_CHUNK_OBS
constexpr int kMfChunkPts = 16;   // MF_CHUNK_PTS
constexpr int kMfCams = 7;        // MF_CAMS
constexpr int kAlign = 64;        // int32 slots: every table starts on a 256-byte boundary

using i64 = long long;

i64 block_index(i64 c1, i64 c2, i64 C) { return c1 * C - c1 * (c1 - 1) / 2 + (c2 - c1); }

// Stable counting sort of idx by key[idx] in [0, nkeys).
void csort(std::vector<int>& idx, const std::vector<int>& key, int nkeys) {
  std::vector<int> cnt(nkeys + 1, 0);
  for (int i : idx) ++cnt[key[i] + 1];
  for (int k = 0; k < nkeys; ++k) cnt[k + 1] += cnt[k];
  std::vector<int> out(idx.size());
  for (int i : idx) out[cnt[key[i]]++] = i;
  idx.swap(out);
}

// Small sorted camera set (<= 2 kMfCams entries while merging).
struct CamSet {
  int n = 0;
  int c[2 * kMfCams + 2];
  int union_size(const CamSet& o) const {
    int i = 0, j = 0, k = 0;
    while (i < n || j < o.n) {
      if (j == o.n || (i < n && c[i] < o.c[j])) ++i;
      else if (i == n || o.c[j] < c[i]) ++j;
      else ++i, ++j;
      ++k;
    }
    return k;
  }
  void merge(const CamSet& o) {  // caller guarantees the union has <= kMfCams entries
    int tmp[2 * kMfCams + 2];
    int i = 0, j = 0, k = 0;
    while (i < n || j < o.n) {
      if (j == o.n || (i < n && c[i] < o.c[j])) tmp[k++] = c[i++];
      else if (i == n || o.c[j] < c[i]) tmp[k++] = o.c[j++];
      else tmp[k++] = c[i++], ++j;
    }
    n = k;
    std::memcpy(c, tmp, sizeof(int) * k);
  }
};

i64 al(i64 v) { return (v + kAlign - 1) / kAlign * kAlign; }

}  // namespace

extern "C" long long slam_ba_plan_bound(int n_cams, int n_pts, int n_obs, int n_block_list) {
  if (n_cams < 1 || n_pts < 0 || n_obs < 0) return 0;
  const i64 C = n_cams, P = n_pts, O = n_obs;
  const i64 G = P + 1, NS = G, ncs = kMfCams * NS, nbs = kMfCams * (kMfCams - 1) / 2 * NS;
  const i64 NB = std::max<i64>(C * (C + 1) / 2, n_block_list);
  const i64 len[SLAM_PLAN_NTAB] = {P, O, O, O, P + 1, G + 1, NS + 1, ncs, NS + 1, nbs, 2 * NB, C + 1,
                                   ncs, NB + 1, nbs, NS + 1, 24 * NS, 8 * NS, O, O, O, G + 1, 8 * G, nbs};
  i64 tot = 0;
  for (i64 l : len) tot += al(std::max<i64>(l, 1));
  return tot;
}

extern "C" int slam_ba_plan_mfma(int n_cams, int n_pts, int n_obs, const int32_t* cam_idx,
                                 const int32_t* pt_idx, const int32_t* block_list, int n_block_list,
                                 int chunks_per_wg, int32_t* out, long long out_cap,
                                 slam_ba_plan_info* info) {
  SLAM_REQUIRE(info && out, "slam_ba_plan_mfma: null output");
  SLAM_REQUIRE(n_cams >= 1 && n_pts >= 0 && n_obs >= 0, "slam_ba_plan_mfma: bad sizes");
  SLAM_REQUIRE(n_obs == 0 || (cam_idx && pt_idx), "slam_ba_plan_mfma: null indices");
  SLAM_REQUIRE(out_cap >= slam_ba_plan_bound(n_cams, n_pts, n_obs, n_block_list),
               "slam_ba_plan_mfma: out_cap %lld < slam_ba_plan_bound", out_cap);
  std::memset(info, 0, sizeof(*info));
  const int C = n_cams, P = n_pts, O = n_obs;
  for (int i = 0; i < O; ++i)
    SLAM_REQUIRE(cam_idx[i] >= 0 && cam_idx[i] < C && pt_idx[i] >= 0 && pt_idx[i] < P,
                 "slam_ba_plan_mfma: observation %d indexes camera %d / point %d out of range", i,
                 cam_idx[i], pt_idx[i]);
  std::vector<int> cam(cam_idx, cam_idx + O), pt(pt_idx, pt_idx + O);

  // ---- observations by (point, camera); per point: count, distinct cameras, span
  std::vector<int> o0(O);
  for (int i = 0; i < O; ++i) o0[i] = i;
  csort(o0, cam, C);
  csort(o0, pt, P);
  std::vector<int> cnt(P, 0), ndist(P, 0), lo(P, C), hi(P, C);
  for (int k = 0; k < O; ++k) {
    const int i = o0[k], p = pt[i], c = cam[i];
    ++cnt[p];
    if (k == 0 || pt[o0[k - 1]] != p || cam[o0[k - 1]] != c) ++ndist[p];
    lo[p] = std::min(lo[p], c);
    hi[p] = hi[p] == C ? c : std::max(hi[p], c);
  }
  for (int p = 0; p < P; ++p)
    if (cnt[p] > kMfChunkObs || ndist[p] > kMfCams) return SLAM_OK;  // info->ok = 0

  // ---- points renumbered by (first camera, last camera, index)
  std::vector<int> perm(P), inv(P);
  for (int p = 0; p < P; ++p) perm[p] = p;
  csort(perm, hi, C + 1);
  csort(perm, lo, C + 1);
  for (int k = 0; k < P; ++k) inv[perm[k]] = k;
  std::vector<int> npt(O);
  for (int i = 0; i < O; ++i) npt[i] = inv[pt[i]];
  std::vector<int> order(O);
  for (int i = 0; i < O; ++i) order[i] = i;
  csort(order, cam, C);
  csort(order, npt, std::max(P, 1));
  std::vector<int> obs_cam(O), obs_pt(O), pt_ptr(P + 1, 0);
  for (int k = 0; k < O; ++k) {
    obs_cam[k] = cam[order[k]];
    obs_pt[k] = npt[order[k]];
    ++pt_ptr[obs_pt[k] + 1];
  }
  for (int p = 0; p < P; ++p) pt_ptr[p + 1] += pt_ptr[p];

  // ---- chunks and supergroups (greedy, in point order)
  int S = chunks_per_wg;
  if (S <= 0) {
    const int est = std::max(1, (O + kMfChunkObs - 1) / kMfChunkObs);
    S = std::min(8, std::max(est >= 256 ? 3 : 1, est / 512));
  }
  S = std::max(1, S);
  std::vector<int> grp{0}, sg{0};
  std::vector<CamSet> sets;
  CamSet uni;
  int ch_obs = 0, ch_pts = 0, sg_ch = 1;
  for (int q = 0; q < P; ++q) {
    CamSet mk;
    for (int k = pt_ptr[q]; k < pt_ptr[q + 1]; ++k)
      if (k == pt_ptr[q] || obs_cam[k] != obs_cam[k - 1]) mk.c[mk.n++] = obs_cam[k];
    const int n = pt_ptr[q + 1] - pt_ptr[q];
    if (uni.union_size(mk) > kMfCams) {  // new supergroup (and chunk)
      grp.push_back(q);
      sg.push_back((int)grp.size() - 1);
      sets.push_back(uni);
      uni = CamSet();
      ch_obs = ch_pts = 0;
      sg_ch = 1;
    } else if (ch_obs + n > kMfChunkObs || ch_pts + 1 > kMfChunkPts) {  // new chunk
      grp.push_back(q);
      ch_obs = ch_pts = 0;
      if (sg_ch == S) {
        sg.push_back((int)grp.size() - 1);
        sets.push_back(uni);
        uni = CamSet();
        sg_ch = 1;
      } else {
        ++sg_ch;
      }
    }
    uni.merge(mk);
    ch_obs += n;
    ++ch_pts;
  }
  grp.push_back(P);
  sg.push_back((int)grp.size() - 1);
  sets.push_back(uni);
  const int G = (int)grp.size() - 1, NS = (int)sg.size() - 1;
  std::vector<int> sg_cams(8 * NS, -1), ms(NS);
  for (int k = 0; k < NS; ++k) {
    ms[k] = sets[k].n;
    for (int a = 0; a < sets[k].n; ++a) sg_cams[8 * k + a] = sets[k].c[a];
  }

  // ---- per observation: chunk, supergroup, camera position in the union
  std::vector<int> chunk_of_pt(P), sg_of_chunk(G);
  for (int g = 0; g < G; ++g)
    for (int q = grp[g]; q < grp[g + 1]; ++q) chunk_of_pt[q] = g;
  for (int k = 0; k < NS; ++k)
    for (int g = sg[k]; g < sg[k + 1]; ++g) sg_of_chunk[g] = k;
  std::vector<int> obs_chunk(O), obs_sg(O), obs_la(O), loc(O);
  for (int i = 0; i < O; ++i) {
    obs_chunk[i] = chunk_of_pt[obs_pt[i]];
    obs_sg[i] = sg_of_chunk[obs_chunk[i]];
    int la = 0;
    for (int a = 0; a < ms[obs_sg[i]]; ++a) la += sg_cams[8 * obs_sg[i] + a] < obs_cam[i] ? 1 : 0;
    obs_la[i] = la;
    loc[i] = i - pt_ptr[grp[obs_chunk[i]]];
  }
  // chunk-local observation lists by (la, obs); run starts per camera position
  std::vector<int> chk_cobs(O), chk_cptr(8 * G, 0);
  for (int g = 0; g < G; ++g) {
    const int b0 = pt_ptr[grp[g]], b1 = pt_ptr[grp[g + 1]];
    int c8[9] = {0};
    for (int i = b0; i < b1; ++i) ++c8[obs_la[i] + 1];
    for (int a = 0; a < 8; ++a) {
      c8[a + 1] += c8[a];
      chk_cptr[8 * g + a] = c8[a];
    }
    for (int i = b0; i < b1; ++i) chk_cobs[b0 + c8[obs_la[i]]++] = loc[i];
  }

  // ---- camera slots: (supergroup, camera), rows camera-major in supergroup order
  std::vector<int> grp_cslot(NS + 1, 0);
  for (int k = 0; k < NS; ++k) grp_cslot[k + 1] = grp_cslot[k] + ms[k];
  const int ncs = grp_cslot[NS];
  std::vector<int> cslot_cam(ncs), cslot_row(ncs), cam_cslot_ptr(C + 1, 0);
  for (int k = 0; k < NS; ++k)
    for (int a = 0; a < ms[k]; ++a) cslot_cam[grp_cslot[k] + a] = sg_cams[8 * k + a];
  {
    std::vector<int> cs(ncs);
    for (int r = 0; r < ncs; ++r) cs[r] = r;  // already in supergroup order
    csort(cs, cslot_cam, C);
    for (int r = 0; r < ncs; ++r) cslot_row[cs[r]] = r;
    for (int r = 0; r < ncs; ++r) ++cam_cslot_ptr[cslot_cam[r] + 1];
    for (int c = 0; c < C; ++c) cam_cslot_ptr[c + 1] += cam_cslot_ptr[c];
  }

  // ---- block slots: (supergroup, a < b) for cameras a, b sharing a point there
  std::vector<unsigned long long> pairs(NS, 0ull);  // bit 8 a + b
  for (int q = 0; q < P; ++q)
    for (int i = pt_ptr[q]; i < pt_ptr[q + 1]; ++i)
      for (int j = i + 1; j < pt_ptr[q + 1]; ++j)
        if (obs_cam[i] != obs_cam[j]) pairs[obs_sg[i]] |= 1ull << (8 * obs_la[i] + obs_la[j]);
  std::vector<int> grp_bslot(NS + 1, 0), bslot_a, bslot_b, bslot_sg;
  for (int k = 0; k < NS; ++k) {
    for (int bit = 0; bit < 64; ++bit)
      if ((pairs[k] >> bit) & 1ull) {
        bslot_sg.push_back(k);
        bslot_a.push_back(bit / 8);
        bslot_b.push_back(bit % 8);
      }
    grp_bslot[k + 1] = (int)bslot_sg.size();
  }
  const int nbs = (int)bslot_sg.size();
  std::vector<i64> blk(nbs);
  for (int s = 0; s < nbs; ++s)
    blk[s] = block_index(sg_cams[8 * bslot_sg[s] + bslot_a[s]], sg_cams[8 * bslot_sg[s] + bslot_b[s]], C);
  std::vector<i64> blist;
  if (9 * C > 120) {  // packed layout: the listed blocks only
    std::vector<i64> own(blk);
    for (int c = 0; c < C; ++c) own.push_back(block_index(c, c, C));
    std::sort(own.begin(), own.end());
    own.erase(std::unique(own.begin(), own.end()), own.end());
    if (block_list) {  // given (an empty list too: it misses every diagonal block)
      blist.assign(block_list, block_list + n_block_list);
      std::sort(blist.begin(), blist.end());
      blist.erase(std::unique(blist.begin(), blist.end()), blist.end());
      SLAM_REQUIRE(std::includes(blist.begin(), blist.end(), own.begin(), own.end()),
                   "slam_ba_plan_mfma: block_list misses a camera block with common points");
    } else {
      blist.swap(own);
    }
    for (auto& b : blk) b = std::lower_bound(blist.begin(), blist.end(), b) - blist.begin();
  } else {
    blist.resize((i64)C * (C + 1) / 2);
    for (size_t k = 0; k < blist.size(); ++k) blist[k] = (i64)k;
  }
  const int NB = (int)blist.size();
  SLAM_REQUIRE(NB <= std::max<i64>((i64)C * (C + 1) / 2, n_block_list),
               "slam_ba_plan_mfma: %d blocks", NB);
  std::vector<int> blk32(blk.begin(), blk.end()), bslot_row(nbs), blk_bslot_ptr(NB + 1, 0);
  {
    std::vector<int> bs(nbs);
    for (int s = 0; s < nbs; ++s) bs[s] = s;  // already in supergroup order
    csort(bs, blk32, std::max(NB, 1));
    for (int r = 0; r < nbs; ++r) bslot_row[bs[r]] = r;
    for (int s = 0; s < nbs; ++s) ++blk_bslot_ptr[blk32[s] + 1];
    for (int b = 0; b < NB; ++b) blk_bslot_ptr[b + 1] += blk_bslot_ptr[b];
  }
  // (c1, c2) of every listed block (np.triu_indices order)
  std::vector<int> blocks(2 * NB);
  {
    size_t k = 0;
    i64 idx = 0;
    for (int c1 = 0; c1 < C && k < blist.size(); ++c1)
      for (int c2 = c1; c2 < C && k < blist.size(); ++c2, ++idx)
        if (blist[k] == idx) {
          blocks[2 * k] = c1;
          blocks[2 * k + 1] = c2;
          ++k;
        }
  }

  // ---- write the tables (order: SLAM_PLAN_* in include/slam355.h)
  const int* src[SLAM_PLAN_NTAB];
  i64 len[SLAM_PLAN_NTAB];
  std::vector<int> sg_meta(24 * NS, 0), obs_meta(O), chk_optr(G + 1), bslot_ab(nbs);
  for (int k = 0; k < NS; ++k) {
    int* m = &sg_meta[24 * k];
    const int f = sg[k];
    m[0] = sg[k];
    m[1] = sg[k + 1];
    m[2] = grp_cslot[k];
    m[3] = ms[k];
    m[4] = grp_bslot[k];
    m[5] = grp_bslot[k + 1] - grp_bslot[k];
    m[6] = grp[f];
    m[7] = grp[f + 1];
    m[8] = pt_ptr[grp[f]];
    m[9] = pt_ptr[grp[f + 1]];
    for (int a = 0; a < 8; ++a) m[10 + a] = sg_cams[8 * k + a];
  }
  for (int i = 0; i < O; ++i)
    obs_meta[i] = (obs_pt[i] - grp[obs_chunk[i]]) | (obs_la[i] << 8) | (chk_cobs[i] << 16);
  for (int g = 0; g <= G; ++g) chk_optr[g] = pt_ptr[grp[g]];
  for (int s = 0; s < nbs; ++s) bslot_ab[s] = bslot_a[s] | (bslot_b[s] << 8);
  auto put = [&](int t, const std::vector<int>& v) {
    src[t] = v.data();
    len[t] = (i64)v.size();
  };
  put(SLAM_PLAN_PERM, perm);
  put(SLAM_PLAN_ORDER, order);
  put(SLAM_PLAN_OBS_CAM, obs_cam);
  put(SLAM_PLAN_OBS_PT, obs_pt);
  put(SLAM_PLAN_PT_PTR, pt_ptr);
  put(SLAM_PLAN_GRP_PTR, grp);
  put(SLAM_PLAN_GRP_CSLOT, grp_cslot);
  put(SLAM_PLAN_CSLOT_CAM, cslot_cam);
  put(SLAM_PLAN_GRP_BSLOT, grp_bslot);
  put(SLAM_PLAN_BSLOT_BLK, blk32);
  put(SLAM_PLAN_BLOCKS, blocks);
  put(SLAM_PLAN_CAM_CSLOT_PTR, cam_cslot_ptr);
  put(SLAM_PLAN_CSLOT_ROW, cslot_row);
  put(SLAM_PLAN_BLK_BSLOT_PTR, blk_bslot_ptr);
  put(SLAM_PLAN_BSLOT_ROW, bslot_row);
  put(SLAM_PLAN_SG_PTR, sg);
  put(SLAM_PLAN_SG_META, sg_meta);
  put(SLAM_PLAN_SG_CAMS, sg_cams);
  put(SLAM_PLAN_OBS_LA, obs_la);
  put(SLAM_PLAN_CHK_COBS, chk_cobs);
  put(SLAM_PLAN_OBS_META, obs_meta);
  put(SLAM_PLAN_CHK_OPTR, chk_optr);
  put(SLAM_PLAN_CHK_CPTR, chk_cptr);
  put(SLAM_PLAN_BSLOT_AB, bslot_ab);
  i64 off = 0;
  for (int t = 0; t < SLAM_PLAN_NTAB; ++t) {
    info->off[t] = off;
    info->len[t] = len[t];
    const i64 room = al(std::max<i64>(len[t], 1));
    SLAM_REQUIRE(off + room <= out_cap, "slam_ba_plan_mfma: table %d overflows out_cap", t);
    if (len[t]) std::memcpy(out + off, src[t], sizeof(int32_t) * len[t]);
    std::memset(out + off + len[t], 0, sizeof(int32_t) * (room - len[t]));
    off += room;
  }
  info->total = off;
  info->ok = 1;
  info->n_obs = O;
  info->n_grps = G;
  info->n_sgrps = NS;
  info->n_cslots = ncs;
  info->n_bslots = nbs;
  info->n_blocks = NB;
  info->chunks_per_wg = S;
  return SLAM_OK;
}
