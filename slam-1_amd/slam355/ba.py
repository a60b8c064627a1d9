"""GPU Levenberg-Marquardt bundle adjustment (BAL model) — host planner + driver.

The planner turns a reference-style BA problem (BundleAdjustment.py:331:
params = [cams (C x 9), points (P x 3)], cam_idxs, Q_idxs, qs) into the index
tables the HIP kernels in csrc/ba.hip consume, allocates the device buffers
(torch tensors as HBM containers) and runs LM iterations with all state on the
device.  Multi-GPU: each rank builds a BAProblem over ALL cameras and the
observations of its own points; `step_distributed` all-reduces the reduced
camera system (one RCCL all-reduce of ~(9C)^2 doubles) and two scalars per
iteration.
"""
from __future__ import annotations

import ctypes
import os

import numpy as np
import torch

from . import _lib
from .device import ptr, require_gpu, stream_ptr

from ._lib import BAProblemStruct as _Prob

ST = dict(LAMBDA=0, NU=1, COST=2, COST_NEW=3, PRED=4, RHO=5, ACCEPTED=6, CUR=7, ITERS=8,
          NACCEPT=9, PRED_CAM=10, CHOL_FAIL=11, SOLVE_FAULT=16)
N_STATE = 20  # SLAM_BA_ST_SLOTS
LDS_MAX_N = 120  # k_solve_blk keeps S in LDS up to 9C <= 120 (dense sys); tiled solver above


def _check_indices(n_cams, n_pts, cam_idx, pt_idx, qs):
    cam_idx = np.asarray(cam_idx).astype(np.int64).ravel()
    pt_idx = np.asarray(pt_idx).astype(np.int64).ravel()
    qs = np.asarray(qs, np.float64).reshape(-1, 2)
    if not (len(cam_idx) == len(pt_idx) == len(qs)):
        raise ValueError("cam_idxs, Q_idxs and qs must have the same length")
    if len(cam_idx) and (cam_idx.min() < 0 or cam_idx.max() >= n_cams):
        raise ValueError("camera index out of range")
    if len(pt_idx) and (pt_idx.min() < 0 or pt_idx.max() >= n_pts):
        raise ValueError("point index out of range")
    return cam_idx, pt_idx, qs


# ----------------------------------------------------------------------------- planner
GROUP_OBS = 128  # kGrp in csrc/ba.hip: observations (and points) per point group


def point_groups(pt_ptr, cap=GROUP_OBS):
    """Greedy cut of the point-sorted observation list into groups of whole
    points with <= cap observations each -> grp_ptr [G+1] (point indices).
    At least one (possibly empty) group."""
    pt_ptr = np.asarray(pt_ptr, np.int64)
    P = len(pt_ptr) - 1
    cnt = np.diff(pt_ptr)
    if P and cnt.max() > cap:
        raise ValueError(f"a point has {int(cnt.max())} observations (> {cap} per point group)")
    starts = [0]
    base = 0
    for p in range(P):
        if pt_ptr[p + 1] - pt_ptr[base] > cap or p - base >= cap:
            starts.append(p)
            base = p
    if P:
        starts.append(P)
    else:
        starts.append(0)
    return np.asarray(starts, np.int32)


def block_index(c1, c2, n_cams):
    """Index of the upper block (c1 <= c2) in np.triu_indices(n_cams) order."""
    c1 = np.asarray(c1, np.int64)
    return c1 * n_cams - c1 * (c1 - 1) // 2 + (np.asarray(c2, np.int64) - c1)


def packed(n_cams):
    """True when the reduced camera system goes to the tiled solver in the packed
    block layout (9C > 120; csrc/ba.hip sys_packed)."""
    return 9 * n_cams > LDS_MAX_N


def upper_blocks(n_cams, cam_idx, pt_idx):
    """Dense upper-block indices (np.triu_indices order) of the diagonal and of
    every camera pair with a common point: the packed block list.  Ranks of a
    sharded problem pass the list of the GLOBAL problem to BAProblem so their
    packed systems line up for the all-reduce."""
    cam_idx = np.asarray(cam_idx, np.int64).ravel()
    pt_idx = np.asarray(pt_idx, np.int64).ravel()
    o1, o2 = _pairs_by_point(cam_idx, pt_idx)
    c1, c2 = np.minimum(cam_idx[o1], cam_idx[o2]), np.maximum(cam_idx[o1], cam_idx[o2])
    diag = np.arange(n_cams)
    return np.unique(np.concatenate([block_index(diag, diag, n_cams), block_index(c1, c2, n_cams)]))


TB = 64  # tile edge of the tiled solver (csrc/ba.hip kTB)
EPI_CAMS_MAX = 16  # cameras per tile in the dataflow solve's spread epilogue (csrc/ba.hip kEpiCams)
TILE_MODE = "rows64"  # default tiling of the camera solve (tl_schedule; measured best)


def _components(adj, nodes):
    """Connected components of `nodes` in `adj` (list of sets), lowest node first."""
    nodes = set(nodes)
    out = []
    while nodes:
        root = min(nodes)
        comp, stack = {root}, [root]
        while stack:
            u = stack.pop()
            for v in adj[u]:
                if v in nodes and v not in comp:
                    comp.add(v)
                    stack.append(v)
        nodes -= comp
        out.append(comp)
    return out


def _bfs_levels(adj, comp, root):
    levels, seen = [[root]], {root}
    while True:
        nxt = sorted({v for u in levels[-1] for v in adj[u] if v in comp and v not in seen})
        if not nxt:
            return levels
        seen.update(nxt)
        levels.append(nxt)


def _bfs_order(adj, comp):
    """comp in BFS order from a pseudo-peripheral node (camera order for a
    keyframe window; the two arcs outward for a loop)."""
    levels = _bfs_levels(adj, comp, min(comp))
    for _ in range(2):  # pseudo-peripheral: restart from the far end
        far = min(levels[-1])
        lv2 = _bfs_levels(adj, comp, far)
        if len(lv2) <= len(levels):
            break
        levels = lv2
    return [v for lv in levels for v in lv]


def _chunk(adj, nodes, cap):
    """Tiles of at most `cap` nodes over the connected pieces of `nodes` (each
    piece in BFS order, so a chain of tiles follows the band): pieces that
    share no block stay in separate tiles -- independent columns."""
    out = []
    for comp in _components(adj, nodes):
        c = _bfs_order(adj, comp)
        out += [sorted(c[i:i + cap]) for i in range(0, len(c), cap)]
    return out


def _nd_tiles(adj, comp, cap, chain):
    """Nested dissection of a graph into tiles of <= cap nodes, in elimination
    order.  A component of <= cap nodes is a leaf; with `chain`, one of <=
    chain * cap nodes is a chain of tiles along its BFS order (no separator:
    fewer tiles, fewer children per column).  Otherwise its nodes are put in
    BFS order, and for every cut i of that order the separator is order[i ..
    reach(i)], reach(i) = the furthest position any node before i is coupled
    to: the nodes before and after it share no block.  The cut minimising the
    larger side plus twice the separator is taken (a band of 6-keyframe
    tracks: 5-camera separators anywhere, so the sides balance exactly; a
    loop: a BFS level's two arcs); its separator's tiles are eliminated after
    both sides."""
    if len(comp) <= cap * max(chain, 1):
        return _chunk(adj, comp, cap)
    order = _bfs_order(adj, comp)
    pos = {v: i for i, v in enumerate(order)}
    n = len(order)
    best, reach = None, -1
    for i in range(1, n):
        reach = max(reach, max((pos[w] for w in adj[order[i - 1]] if w in pos), default=i - 1))
        if reach < i or reach >= n - 1:
            continue  # order[:i] is a component of its own, or no right side
        cost = max(i, n - 1 - reach) + 2 * (reach - i + 1)
        if best is None or cost < best[0]:
            best = (cost, i, reach)
    if best is None:  # no separator: a dense chain of tiles
        return _chunk(adj, comp, cap)
    _, i, r = best
    out = []
    for side in (order[:i], order[r + 1:]):
        for sub in _components(adj, side):
            out += _nd_tiles(adj, sub, cap, chain)
    return out + _chunk(adj, order[i:r + 1], cap)


def _dist_from(adj, comp, srcs):
    """BFS distance inside comp from the nodes srcs (multi-source)."""
    dist = {v: 0 for v in srcs}
    frontier = list(srcs)
    while frontier:
        nxt = []
        for u in frontier:
            for v in adj[u]:
                if v in comp and v not in dist:
                    dist[v] = dist[u] + 1
                    nxt.append(v)
        frontier = nxt
    return dist


def _nd_order(adj, nodes, bound=frozenset()):
    """Nested-dissection order of `nodes` in the 64-row tile graph (the
    "rows64" tiling): each connected component separately; a component whose
    BFS level structure has >= 3 levels is split by its middle level, the
    separator numbered last.  `bound`: the separators already numbered after
    these nodes (their ancestors).  A component next to them is levelled from
    its node furthest from them, so that its own separator sits nearer to them:
    the part between the two separators is the smaller one (a single tile on a
    band), and the larger part -- a chain of tiles on a band, eliminated from
    its far end -- shares no row with the ancestors.  Otherwise the top of that
    chain would carry a row to an ancestor, and its parent's update with it
    would wait until after the parent's factor (a deferred row fold on the
    critical path: C4's right half, 6.5 us)."""
    out = []
    for comp in _components(adj, nodes):
        near = {u for u in comp if adj[u] & bound}
        dist = _dist_from(adj, comp, near) if near else None
        if len(comp) <= 2:
            # a chain of <= 2 tiles: its far end first (it then shares no row with
            # the ancestors), otherwise ascending
            out += sorted(comp, key=(lambda v: (-dist.get(v, 0), v)) if dist else None)
            continue
        levels = _bfs_levels(adj, comp, min(comp))
        for _ in range(2):  # pseudo-peripheral
            far = min(levels[-1])
            lv2 = _bfs_levels(adj, comp, far)
            if len(lv2) <= len(levels):
                break
            levels = lv2
        if dist:
            # from the node furthest from the ancestors, when that levels the
            # component as deeply as a pseudo-peripheral node does (a band
            # touching them at one end; not a path they bound at both ends,
            # whose middle would give levels of two tiles)
            root = min(comp, key=lambda v: (-dist.get(v, 0), v))
            lvb = _bfs_levels(adj, comp, root)
            if len(lvb) >= len(levels):
                levels = lvb
        if len(levels) < 3:
            out += sorted(comp)
            continue
        sep = set(levels[len(levels) // 2])
        out += _nd_order(adj, comp - sep, bound | sep) + sorted(sep)
    return out


def _parse_tile_mode(mode):
    mode = mode or os.environ.get("SLAM_TL_TILES") or TILE_MODE
    if mode == "rows64":
        return mode, 0, 0
    parts = mode.split(":")
    if parts[0] != "cams" or len(parts) not in (2, 3):
        raise ValueError(f"tile mode must be 'rows64' or 'cams:CAP[:CHAIN]', not {mode!r}")
    cap, chain = int(parts[1]), int(parts[2]) if len(parts) == 3 else 0
    if not 1 <= cap <= TB // 9:
        raise ValueError(f"tile mode {mode!r}: 1 <= CAP <= {TB // 9} cameras per tile")
    return "cams", cap, chain


def tile_rows(n_cams, blocks, mode=None):
    """The tiles of the camera solve as lists of rows of S (<= 64 each), in
    elimination order.  mode (default TILE_MODE, or $SLAM_TL_TILES):
      "rows64"          64 consecutive rows per tile (a camera may straddle two
                        tiles), tiles in nested-dissection order of the tile graph;
      "cams:CAP[:CH]"   whole cameras, <= CAP per tile (9 CAP rows: the rest of
                        the 64-row tile is padding, whose 16-row blocks the
                        factor skips), nested dissection of the camera graph
                        (_nd_tiles; CH: components of <= CH CAP cameras become a
                        chain of tiles instead of being split)."""
    kind, cap, chain = _parse_tile_mode(mode)
    blocks = np.asarray(blocks, np.int64).reshape(-1, 2)
    n = 9 * int(n_cams)
    if kind == "rows64":
        T = (n + TB - 1) // TB
        adj = [set() for _ in range(T)]
        for c1, c2 in blocks:
            t1 = range((9 * c1) // TB, (9 * c1 + 8) // TB + 1)
            t2 = range((9 * c2) // TB, (9 * c2 + 8) // TB + 1)
            for a_ in t1:
                for b_ in t2:
                    if a_ != b_:
                        adj[a_].add(b_)
                        adj[b_].add(a_)
        return [list(range(TB * t, min(TB * t + TB, n))) for t in _nd_order(adj, range(T))]
    adj = [set() for _ in range(int(n_cams))]
    for c1, c2 in blocks:
        if c1 != c2:
            adj[c1].add(int(c2))
            adj[c2].add(int(c1))
    out = []
    for comp in _components(adj, range(int(n_cams))):
        out += _nd_tiles(adj, comp, cap, chain)
    return [[9 * c + i for c in cams for i in range(9)] for cams in out]


# k_tl3_flow's phase costs in us (profiles/r6/prod_slots, C4 / C5 per-column
# stamps): tile hand-off, one child's diagonal update, the tile factor, a row
# tile's staging + product + publish, a product slot's wait + load, a product
# task, a later row tile's update per k
_FLOW_COST = dict(start=4.0, hand=2.6, child=1.5, factor=10.6, row=2.6, slot=2.1, task=2.0, fold=3.0)


def _flow_rs_order(T, struct, level):
    """rs(J) of the dataflow solve (every k < J with L_Jk != 0) ordered by the
    predicted time its tile (J, k) is published: columns are simulated in index
    order (children first) with _FLOW_COST, each column taking its rs tiles in
    the order chosen for it, its row tiles after its factor (rows 0 and 1 once
    their product slots are in) and its product tasks after the row tile they
    need.  Ties: elimination-tree level, then index."""
    c = _FLOW_COST
    pub, prod_t, out = {}, {}, []
    for J in range(T):
        ks = [k for k in range(J) if J in struct[k]]
        t_in = {k: pub[(k, J)] + c["hand"] for k in ks}
        order = sorted(ks, key=lambda k: (round(t_in[k], 6), level[k], k))
        out.append(order)
        t = c["start"]
        for k in order:
            t = max(t, t_in[k]) + c["child"]
        t += c["factor"]
        rows = sorted(struct[J])
        tasks = {}  # b -> [(a, b)]: J forms L_{rows[b]} J L_{rows[a]} J^T after row b
        for a, Ja in enumerate(rows):
            first2 = sorted(struct[Ja])[:2]
            for b in range(a + 1, len(rows)):
                if rows[b] in first2:
                    tasks.setdefault(b, []).append(a)
        for q, I in enumerate(rows):
            kl = [k for k in order if I in struct[k]]
            if q < 2 and kl:
                t = max(t, max(prod_t[(k, J, I)] for k in kl)) + c["slot"]
            else:
                t += c["fold"] * len(kl)
            t += c["row"]
            pub[(J, I)] = t
            for a in tasks.get(q, []):
                t += c["task"]
                prod_t[(J, rows[a], I)] = t
    return out


def tl_schedule(n_cams, blocks, mode=None):
    """Level schedule of the tiled camera solve (csrc/ba.hip tl_solve_levels).

    The 9C-row camera system is cut into tiles (tile_rows: whole cameras by
    default, at most 64 rows each, numbered in nested-dissection order), each
    held in a 64-row tile whose rows past its own are padding (identity
    diagonal, no coupling); the tile-level Cholesky structure and elimination
    tree are computed symbolically, and the columns are grouped by their height
    in the tree: the columns of one level are mutually independent, so each
    level is one panel launch (factor + L_Ik for every column of the level) and
    one update launch (A_IJ -= sum_k L_Ik L_Jk^T, b_I -= sum_k L_Ik y_k per
    target tile), and the back substitution walks the levels in reverse.  A
    banded window of T tiles needs ~log2(T) levels instead of T sequential
    panel steps.

    The same symbolic structure also drives the dataflow form of the solve
    (csrc/ba.hip k_tl3_flow: one persistent workgroup per tile column, columns
    wait for the tiles they need through device flags instead of launch
    boundaries), whose per-column table is appended.

    Returns the int32 schedule (device and host copies are the same array):
      [0] nlev, [1] T, [2] row map offset, [3] inverse row map offset,
      [4] level table offset, [5] column table offset, [6] tile size table
      offset, [7] epilogue table offset, [8] block index table offset,
      [9] gather table offset, [10] product task table offset, [11] product slots
      row map: row r of S -> row of the tiled system (tile * 64 + position)
      inverse row map: row of the tiled system -> row of S, -1 on padding rows
      tile sizes: per tile its rows of S (they come first, padding after)
      column table: per column J (rows_off, rows_cnt, rs_off, rs_cnt, upd_off)
        rows: I > J with L_IJ != 0 (ascending); rs: k < J with L_Jk != 0
        (by elimination-tree level, then index: the updates of the diagonal
        tile and the forward substitution); upd: per row I, (koff, kcnt) -- the
        k < J with L_Ik and L_Jk both nonzero (in rs order), followed by their
        product slots (rows 0 and 1; -1 for later rows)
      level table: per level (pan_off, pan_cnt, upd_off, upd_cnt, bk_off, bk_cnt)
      panel entries (k, I)         -- I == k: the diagonal tile
      update entries (I, J, koff, kcnt), I >= J, k list in `koff`
      back entries (k, soff, scnt) -- the rows I of L_Ik (ancestors)
      epilogue table: per tile (off, cnt) of the cameras it owns (list after)
      block index table: [C][C], the packed block of cameras (c1 <= c2), -1 if none
      gather table: per column its offset (T), then per column the packed-S
        offsets of its diagonal and row tiles' elements [1 + rows][64][64]
        (-1 zero, -2 unit diagonal) and its diagonal tile's rows of S [64]
      product task table: per column k (off, cnt), then its tasks (a, b, slot):
        form L_{rows[b]} k L_{rows[a]} k^T into the slot (ordered by b)"""
    blocks = np.asarray(blocks, np.int64).reshape(-1, 2)
    n = 9 * int(n_cams)
    tiles = tile_rows(int(n_cams), blocks, mode)
    T = len(tiles)
    rowmap = np.empty(n, np.int64)
    irow = np.full(T * TB, -1, np.int64)
    for I, rows in enumerate(tiles):
        rowmap[rows] = I * TB + np.arange(len(rows))
        irow[I * TB:I * TB + len(rows)] = rows
    tile_of = rowmap // TB
    # symbolic tile Cholesky (tiles already in elimination order)
    struct = [set() for _ in range(T)]
    for c1, c2 in blocks:
        for A in set(tile_of[9 * c1:9 * c1 + 9].tolist()):
            for B in set(tile_of[9 * c2:9 * c2 + 9].tolist()):
                if A != B:
                    struct[min(A, B)].add(max(A, B))
    parent = [-1] * T
    level = [0] * T
    for k in range(T):
        if struct[k]:
            pk = min(struct[k])
            parent[k] = pk
            struct[pk] |= struct[k] - {pk}
    for k in range(T):
        if parent[k] >= 0:
            level[parent[k]] = max(level[parent[k]], level[k] + 1)
    nlev = max(level) + 1 if T else 0
    cols = [[k for k in range(T) if level[k] == lv] for lv in range(nlev)]
    head = [nlev, T, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0]
    table = []
    lists = []  # (k lists / struct lists) appended after the entries

    def list_off(vals):
        lists.append(list(vals))
        return len(lists) - 1  # patched below

    pan, upd, bk = [], [], []
    for lv in range(nlev):
        p_e = []
        for k in cols[lv]:
            p_e.append((k, k))
            p_e += [(k, I) for I in sorted(struct[k])]
        tgt = {}
        for k in cols[lv]:
            sk = sorted(struct[k])
            for i, I in enumerate(sk):
                for J in sk[:i + 1]:
                    tgt.setdefault((I, J), []).append(k)
        u_e = [(I, J, list_off(ks)) for (I, J), ks in sorted(tgt.items())]
        b_e = [(k, list_off(sorted(struct[k]))) for k in cols[lv]]
        pan.append(p_e)
        upd.append(u_e)
        bk.append(b_e)
    # layout: header | row map | inverse row map | tile sizes | level table | entries | lists
    off = len(head)
    head[2] = off
    off += n
    head[3] = off
    off += T * TB
    head[6] = off
    off += T
    head[4] = off
    off += 6 * nlev
    ent_start = off
    n_ent = sum(2 * len(a) + 4 * len(b) + 3 * len(c) for a, b, c in zip(pan, upd, bk))
    list_base = ent_start + n_ent
    list_offs, o = [], list_base
    for li in lists:
        list_offs.append(o)
        o += len(li)
    ents = []
    for lv in range(nlev):
        po = ent_start + len(ents)
        for k, I in pan[lv]:
            ents += [k, I]
        uo = ent_start + len(ents)
        for I, J, li in upd[lv]:
            ents += [I, J, list_offs[li], len(lists[li])]
        bo = ent_start + len(ents)
        for k, li in bk[lv]:
            ents += [k, list_offs[li], len(lists[li])]
        table += [po, len(pan[lv]), uo, len(upd[lv]), bo, len(bk[lv])]
    flat = (head + rowmap.tolist() + irow.tolist() + [len(r) for r in tiles] + table + ents
            + [v for li in lists for v in li])
    # column table of the dataflow solve.  rs(J) in the order its tiles are
    # expected to be published (_flow_rs_order: a cost model of k_tl3_flow's
    # phases), so a column accumulates the tiles of its early children while
    # the late ones are still being factored, instead of waiting on the first
    # listed tile (the sums keep this fixed order: deterministic)
    rs = _flow_rs_order(T, struct, level)
    flow_off = len(flat)
    flat[5] = flow_off
    recs = [0] * (5 * T)
    tail = []
    base = flow_off + 5 * T

    def put(vals):
        tail.extend(vals)
        return base + len(tail) - len(vals)

    # product slots: every term L_Ik L_Jk^T of column J's rows 0 and 1 is formed
    # by column k itself once both of its tiles exist (k's task (a, b, slot):
    # its row tiles a = J and b = I), and column J sums the slots of a row's k
    # list (stored after the list) in list order
    n_slot = 0
    tasks = [[] for _ in range(T)]
    for J in range(T):
        rows = sorted(struct[J])
        r_off = put(rows)
        s_off = put(rs[J])
        pairs = []
        for qi, I in enumerate(rows):
            ks = [k for k in rs[J] if I in struct[k]]
            sl = [-1] * len(ks)
            if qi < 2:
                sl = list(range(n_slot, n_slot + len(ks)))
                n_slot += len(ks)
                for k, sk in zip(ks, sl):
                    rk = sorted(struct[k])
                    tasks[k].append((rk.index(J), rk.index(I), sk))
            pairs.append((put(ks + sl), len(ks)))
        u_off = put([v for pr in pairs for v in pr])
        recs[5 * J:5 * J + 5] = [r_off, len(rows), s_off, len(rs[J]), u_off]
    # the cameras whose share of the solve's epilogue (trial parameters,
    # projection record, predicted-reduction and cost terms) the workgroup that
    # forms x of tile k runs: those whose lowest-numbered tile is k -- a camera
    # whose rows straddle two tiles couples them, so the lower one is a
    # descendant of the other and its x is formed last
    own = [[] for _ in range(T)]
    for c in range(int(n_cams)):
        own[int(tile_of[9 * c:9 * c + 9].min())].append(c)
    if max((len(o) for o in own), default=0) > EPI_CAMS_MAX:
        raise ValueError(f"tl_schedule: a tile owns more than {EPI_CAMS_MAX} cameras' epilogue")
    epi_off = flow_off + 5 * T + len(tail)
    epi, lo = [], epi_off + 2 * T
    for o in own:
        epi += [lo, len(o)]
        lo += len(o)
    epi += [c for o in own for c in o]
    # dense camera-pair -> packed block index (-1: no block): the dataflow
    # solve gathers its tiles straight from the packed system through it
    bix = np.full((int(n_cams), int(n_cams)), -1, np.int64)
    bix[blocks[:, 0], blocks[:, 1]] = np.arange(len(blocks))
    bix_off = epi_off + len(epi)
    # per column J: for its diagonal tile and each row tile (rows order), the
    # packed-S offset of every element (i, j) of the 64 x 64 tile (-1: zero;
    # -2: a padding row's unit diagonal), then the row of S of each of the
    # diagonal tile's 64 rows (-1: padding) for the damping: the dataflow solve
    # gathers its tiles in two rounds of loads (offsets, then values)
    gt_base = bix_off + bix.size
    gofs, gtab, o = [], [], gt_base + T
    ii, jj = np.meshgrid(np.arange(TB), np.arange(TB), indexing="ij")
    for J in range(T):
        gofs.append(o)
        for I in [J] + sorted(struct[J]):
            r, c = irow[I * TB + ii], irow[J * TB + jj]
            valid = (r >= 0) & (c >= 0)
            a, b = np.maximum(r, 0) // 9, np.maximum(c, 0) // 9
            sw = a > b
            blk = np.where(sw, bix[b, a], bix[a, b])
            e = np.where(sw, 9 * (np.maximum(c, 0) % 9) + np.maximum(r, 0) % 9,
                         9 * (np.maximum(r, 0) % 9) + np.maximum(c, 0) % 9)
            g = np.where(valid & (blk >= 0), 81 * blk + e, -1)
            g = np.where(~valid & (I * TB + ii == J * TB + jj), -2, g)
            gtab.append(g.ravel())
            o += TB * TB
        gtab.append(irow[J * TB:J * TB + TB])
        o += TB
    gt = np.concatenate(gtab) if gtab else np.zeros(0, np.int64)
    if o >= 2 ** 31:
        raise ValueError("tl_schedule: the gather tables exceed int32 offsets")
    # product task table: per column (off, cnt), then its tasks (a, b, slot) by b
    pt_base = gt_base + T + len(gt)
    ptab, lo = [], pt_base + 2 * T
    for tk in tasks:
        ptab += [lo, len(tk)]
        lo += 3 * len(tk)
    ptab += [v for tk in tasks for e in sorted(tk, key=lambda e: (e[1], e[0])) for v in e]
    if lo >= 2 ** 31:
        raise ValueError("tl_schedule: the schedule exceeds int32 offsets")
    out = np.asarray(flat + recs + tail + epi + bix.ravel().tolist() + gofs + gt.tolist() + ptab, np.int32)
    out[7] = epi_off
    out[8] = bix_off
    out[9] = gt_base
    out[10] = pt_base
    out[11] = n_slot
    return out


def _pairs_by_point(cam_idx, pt_idx):
    """Observation pairs (o1 < o2 in (point, camera) order) of the same point."""
    order = np.lexsort((cam_idx, pt_idx))
    obs_pt = pt_idx[order]
    n_pts = int(obs_pt.max()) + 1 if len(obs_pt) else 0
    pt_ptr = np.zeros(n_pts + 1, np.int64)
    np.cumsum(np.bincount(obs_pt, minlength=n_pts), out=pt_ptr[1:])
    cnt = np.diff(pt_ptr)
    o1s, o2s = [], []
    for n in np.unique(cnt):
        if n < 2:
            continue
        base = pt_ptr[np.nonzero(cnt == n)[0]][:, None]
        ii, jj = np.triu_indices(n, 1)
        o1s.append((base + ii[None]).ravel())
        o2s.append((base + jj[None]).ravel())
    o1 = np.concatenate(o1s) if o1s else np.zeros(0, np.int64)
    o2 = np.concatenate(o2s) if o2s else np.zeros(0, np.int64)
    return order[o1], order[o2]


def plan(n_cams, n_pts, cam_idx, pt_idx, block_list=None):
    """Index tables for the LM kernels (host numpy, once per problem structure).

    Observations are sorted by (point, camera) and cut into point groups
    (whole points, <= GROUP_OBS observations).  Each group gets
      camera slots (g, c): its observations of camera c (group-local indices);
    block_list (packed layout only, 9C > 120): dense upper-block indices of the
      blocks to assemble (default: upper_blocks of this problem); every block
      with a common point here must be listed.
      block slots (g, c1 <= c2): its points' observation pairs o1 < o2 (cameras
        c1 <= c2; c1 == c2 only for a point observed twice by one camera);
    and each slot's partial row sits in camera- / block-major order (rows of
    one camera / block contiguous, in group order) for the assembly."""
    O = len(cam_idx)
    C = n_cams
    order = np.lexsort((cam_idx, pt_idx))  # by point, then camera
    obs_cam = cam_idx[order].astype(np.int64)
    obs_pt = pt_idx[order].astype(np.int64)
    pt_ptr = np.zeros(n_pts + 1, np.int64)
    np.cumsum(np.bincount(obs_pt, minlength=n_pts), out=pt_ptr[1:])
    grp_ptr = point_groups(pt_ptr, GROUP_OBS)
    G = len(grp_ptr) - 1
    pt_grp = np.repeat(np.arange(G), np.diff(grp_ptr))
    obs_grp = pt_grp[obs_pt] if O else np.zeros(0, np.int64)
    loc = np.arange(O) - pt_ptr[grp_ptr[:-1]][obs_grp] if O else np.zeros(0, np.int64)

    # camera slots: (group, camera), observations in group order
    ck = obs_grp * C + obs_cam
    so = np.lexsort((np.arange(O), ck))
    ukey, ustart = np.unique(ck[so], return_index=True)
    cslot_grp, cslot_cam = ukey // C, ukey % C
    cslot_obs_ptr = np.append(ustart, O)
    cslot_obs = loc[so]
    grp_cslot = np.searchsorted(cslot_grp, np.arange(G + 1))
    cam_cslots = np.lexsort((cslot_grp, cslot_cam))
    cslot_row = np.empty(len(cam_cslots), np.int64)
    cslot_row[cam_cslots] = np.arange(len(cam_cslots))
    cam_cslot_ptr = np.zeros(C + 1, np.int64)
    np.cumsum(np.bincount(cslot_cam, minlength=C), out=cam_cslot_ptr[1:])

    # block slots: per point, observation pairs (i < j) -> cameras c_i <= c_j
    cnt = np.diff(pt_ptr)
    o1s, o2s = [], []
    for n in np.unique(cnt):
        if n < 2:
            continue
        base = pt_ptr[np.nonzero(cnt == n)[0]][:, None]
        ii, jj = np.triu_indices(n, 1)
        o1s.append((base + ii[None]).ravel())
        o2s.append((base + jj[None]).ravel())
    o1 = np.concatenate(o1s) if o1s else np.zeros(0, np.int64)
    o2 = np.concatenate(o2s) if o2s else np.zeros(0, np.int64)
    NB = C * (C + 1) // 2
    blk = block_index(obs_cam[o1], obs_cam[o2], C)
    if packed(C):
        diag = np.arange(C)
        own = np.unique(np.concatenate([block_index(diag, diag, C), blk]))
        blist = own if block_list is None else np.unique(np.asarray(block_list, np.int64))
        if block_list is not None and not np.all(np.isin(own, blist)):
            raise ValueError("block_list misses a camera block with common points")
        blk = np.searchsorted(blist, blk)
        NB = len(blist)
    else:
        blist = np.arange(NB)
    bk = obs_grp[o1] * NB + blk
    sp = np.lexsort((o2, o1, bk))
    bkey, bstart = np.unique(bk[sp], return_index=True)
    bslot_grp, bslot_blk = bkey // NB, bkey % NB
    bslot_pair_ptr = np.append(bstart, len(sp))
    bslot_pairs = loc[o1[sp]] | (loc[o2[sp]] << 16)
    grp_bslot = np.searchsorted(bslot_grp, np.arange(G + 1))
    blk_bslots = np.lexsort((bslot_grp, bslot_blk))
    bslot_row = np.empty(len(blk_bslots), np.int64)
    bslot_row[blk_bslots] = np.arange(len(blk_bslots))
    blk_bslot_ptr = np.zeros(NB + 1, np.int64)
    np.cumsum(np.bincount(bslot_blk, minlength=NB), out=blk_bslot_ptr[1:])

    c1, c2 = np.triu_indices(C)
    c1, c2 = c1[blist], c2[blist]
    i32 = lambda a: np.asarray(a, np.int32)  # noqa: E731
    return dict(
        order=order, obs_cam=i32(obs_cam), obs_pt=i32(obs_pt), pt_ptr=i32(pt_ptr),
        grp_ptr=i32(grp_ptr), grp_cslot=i32(grp_cslot), cslot_cam=i32(cslot_cam),
        cslot_obs_ptr=i32(cslot_obs_ptr), cslot_obs=i32(cslot_obs), grp_bslot=i32(grp_bslot),
        bslot_blk=i32(bslot_blk), bslot_pair_ptr=i32(bslot_pair_ptr), bslot_pairs=i32(bslot_pairs),
        blocks=i32(np.stack([c1, c2], 1)), cam_cslot_ptr=i32(cam_cslot_ptr),
        cslot_row=i32(cslot_row), blk_bslot_ptr=i32(blk_bslot_ptr), bslot_row=i32(bslot_row),
        chk_optr=i32(pt_ptr[grp_ptr]), n_obs=O)


# Camera-union linearisation (csrc/ba.hip k_lin_mfma): points ordered by their
# camera span, cut into chunks and the chunks into supergroups whose points
# together see at most MF_CAMS cameras, so a supergroup's share of the
# reduced camera system is one dense (9m x 9m, m <= 7) matrix: the Schur term
# sum_p Y_p W_p^T on the f64 matrix cores, U on the vector ALUs.
MF_CHUNK_OBS = 120  # kMObs: observations per chunk (<= k_back_trial's group cap 128)
MF_CHUNK_PTS = 16   # kMPts: points per chunk
MF_CAMS = 7         # kMCams: cameras per supergroup (9m <= 63 rows: 4 MFMA tile rows)


def _popcount(x: int) -> int:
    return bin(x).count("1")


def plan_mfma(n_cams, n_pts, cam_idx, pt_idx, block_list=None, chunks_per_wg=None):
    """Index tables for the camera-union linearisation, or None when a point
    sees more than MF_CAMS cameras (then `plan` and the slot kernel are used).

    Points are renumbered: sorted by (first camera, last camera, index), so
    points with the same camera span are adjacent; `perm` [P] maps the new
    index to the caller's.  Observations are sorted by (new point, camera) and
    cut into chunks (grp_ptr: whole points, <= MF_CHUNK_OBS observations and
    <= MF_CHUNK_PTS points); consecutive chunks form supergroups (sg_ptr: a
    chunk range, <= chunks_per_wg chunks) of at most MF_CAMS distinct cameras
    (sg_cams, sorted; obs_la = position of each observation's camera in its
    supergroup's list).  Camera slots are (supergroup, camera) -- grp_cslot
    indexes supergroups here -- and block slots (supergroup, a < b) for every
    pair of its cameras that share a point (bslot_ab = a | b << 8)."""
    O, C, P = len(cam_idx), n_cams, n_pts
    cam_idx = np.asarray(cam_idx, np.int64)
    pt_idx = np.asarray(pt_idx, np.int64)
    order0 = np.lexsort((cam_idx, pt_idx))
    oc, op = cam_idx[order0], pt_idx[order0]
    cnt = np.bincount(op, minlength=P)
    if P and cnt.max() > MF_CHUNK_OBS:
        return None
    first = np.ones(O, bool)
    first[1:] = (oc[1:] != oc[:-1]) | (op[1:] != op[:-1])
    ndist = np.bincount(op[first], minlength=P)
    if P and ndist.max() > MF_CAMS:
        return None
    ptr0 = np.zeros(P + 1, np.int64)
    np.cumsum(cnt, out=ptr0[1:])
    has = cnt > 0
    lo = np.full(P, C, np.int64)
    hi = np.full(P, C, np.int64)
    if O:
        lo[has] = np.minimum.reduceat(oc, ptr0[:-1][has])
        hi[has] = np.maximum.reduceat(oc, ptr0[:-1][has])
    perm = np.lexsort((np.arange(P), hi, lo))  # new -> old
    inv = np.empty(P, np.int64)
    inv[perm] = np.arange(P)
    npt = inv[pt_idx] if O else pt_idx
    order = np.lexsort((cam_idx, npt))
    obs_cam = cam_idx[order]
    obs_pt = npt[order]
    pt_ptr = np.zeros(P + 1, np.int64)
    np.cumsum(np.bincount(obs_pt, minlength=P), out=pt_ptr[1:])
    # camera-set bitmask per (new) point
    fst = np.ones(O, bool)
    fst[1:] = (obs_cam[1:] != obs_cam[:-1]) | (obs_pt[1:] != obs_pt[:-1])
    masks = [0] * P
    for q, c in zip(obs_pt[fst].tolist(), obs_cam[fst].tolist()):
        masks[q] |= 1 << c
    cntn = np.diff(pt_ptr).tolist()
    n_chunks_est = max(1, -(-O // MF_CHUNK_OBS))
    if chunks_per_wg is None:  # enough workgroups to cover the chip, fewer partial rows
        # (a C3 window, ~310 chunks, is batched with others: 3 chunks per
        # workgroup measured best -- 1/3 of the partial-row traffic, r2 sweep)
        chunks_per_wg = int(min(8, max(3 if n_chunks_est >= 256 else 1, n_chunks_est // 512)))
    S = max(1, int(chunks_per_wg))
    grp = [0]
    sg = [0]
    sg_masks = []
    union = 0
    ch_obs = ch_pts = 0
    sg_ch = 1
    for q in range(P):
        n, mk = cntn[q], masks[q]
        if _popcount(union | mk) > MF_CAMS:  # new supergroup (and chunk)
            grp.append(q)
            sg.append(len(grp) - 1)
            sg_masks.append(union)
            union, ch_obs, ch_pts, sg_ch = 0, 0, 0, 1
        elif ch_obs + n > MF_CHUNK_OBS or ch_pts + 1 > MF_CHUNK_PTS:  # new chunk
            grp.append(q)
            ch_obs = ch_pts = 0
            if sg_ch == S:
                sg.append(len(grp) - 1)
                sg_masks.append(union)
                union, sg_ch = 0, 1
            else:
                sg_ch += 1
        union |= mk
        ch_obs += n
        ch_pts += 1
    grp.append(P)
    sg.append(len(grp) - 1)
    sg_masks.append(union)
    grp_ptr = np.asarray(grp, np.int64)
    sg_ptr = np.asarray(sg, np.int64)
    G, NS = len(grp_ptr) - 1, len(sg_ptr) - 1
    sg_cams = np.full((NS, 8), -1, np.int64)
    ms = np.zeros(NS, np.int64)
    for k, mk in enumerate(sg_masks):
        cs = [c for c in range(C) if (mk >> c) & 1] if mk else []
        ms[k] = len(cs)
        sg_cams[k, :len(cs)] = cs
    # supergroup / chunk of every observation and its camera's position in the union
    chunk_of_pt = np.repeat(np.arange(G), np.diff(grp_ptr))
    sg_of_chunk = np.repeat(np.arange(NS), np.diff(sg_ptr))
    obs_chunk = chunk_of_pt[obs_pt] if O else np.zeros(0, np.int64)
    obs_sg = sg_of_chunk[obs_chunk] if O else np.zeros(0, np.int64)
    # position of obs_cam in sg_cams[obs_sg] (sorted rows, -1 padded at the end)
    rowc = np.where(sg_cams < 0, C + 1, sg_cams)
    obs_la = (rowc[obs_sg] < obs_cam[:, None]).sum(1) if O else np.zeros(0, np.int64)
    # chunk-local observation lists sorted by (la, obs)
    loc = np.arange(O) - pt_ptr[grp_ptr[:-1]][obs_chunk] if O else np.zeros(0, np.int64)
    so = np.lexsort((loc, obs_la, obs_chunk)) if O else np.zeros(0, np.int64)
    chk_cobs = loc[so]
    chk_cptr = np.zeros((G, 8), np.int64)
    o_start = pt_ptr[grp_ptr[:-1]]
    nob = pt_ptr[grp_ptr[1:]] - o_start
    for a in range(8):
        # number of obs of the chunk with la < a
        chk_cptr[:, a] = np.bincount(obs_chunk[obs_la < a], minlength=G) if O else 0
    chk_cptr = np.minimum(chk_cptr, nob[:, None])
    # camera slots: (supergroup, a), rows camera-major in supergroup order
    grp_cslot = np.zeros(NS + 1, np.int64)
    np.cumsum(ms, out=grp_cslot[1:])
    cslot_sg = np.repeat(np.arange(NS), ms)
    cslot_cam = sg_cams[cslot_sg, np.arange(len(cslot_sg)) - grp_cslot[cslot_sg]]
    cam_cslots = np.lexsort((cslot_sg, cslot_cam))
    cslot_row = np.empty(len(cam_cslots), np.int64)
    cslot_row[cam_cslots] = np.arange(len(cam_cslots))
    cam_cslot_ptr = np.zeros(C + 1, np.int64)
    np.cumsum(np.bincount(cslot_cam, minlength=C), out=cam_cslot_ptr[1:])
    # block slots: (supergroup, a < b) co-observed within the supergroup
    o1s, o2s = [], []
    cnt_n = np.diff(pt_ptr)
    for n in np.unique(cnt_n):
        if n < 2:
            continue
        base = pt_ptr[np.nonzero(cnt_n == n)[0]][:, None]
        ii, jj = np.triu_indices(n, 1)
        o1s.append((base + ii[None]).ravel())
        o2s.append((base + jj[None]).ravel())
    o1 = np.concatenate(o1s) if o1s else np.zeros(0, np.int64)
    o2 = np.concatenate(o2s) if o2s else np.zeros(0, np.int64)
    keep = obs_cam[o1] != obs_cam[o2]
    o1, o2 = o1[keep], o2[keep]
    key = (obs_sg[o1] * 8 + obs_la[o1]) * 8 + obs_la[o2]
    ukey = np.unique(key)
    bslot_sg = ukey // 64
    bslot_a, bslot_b = (ukey // 8) % 8, ukey % 8
    grp_bslot = np.searchsorted(bslot_sg, np.arange(NS + 1))
    bc1 = sg_cams[bslot_sg, bslot_a]
    bc2 = sg_cams[bslot_sg, bslot_b]
    NB = C * (C + 1) // 2
    blk = block_index(bc1, bc2, C)
    if packed(C):
        diag = np.arange(C)
        own = np.unique(np.concatenate([block_index(diag, diag, C), blk]))
        blist = own if block_list is None else np.unique(np.asarray(block_list, np.int64))
        if block_list is not None and not np.all(np.isin(own, blist)):
            raise ValueError("block_list misses a camera block with common points")
        blk = np.searchsorted(blist, blk)
        NB = len(blist)
    else:
        blist = np.arange(NB)
    blk_bslots = np.lexsort((bslot_sg, blk))
    bslot_row = np.empty(len(blk_bslots), np.int64)
    bslot_row[blk_bslots] = np.arange(len(blk_bslots))
    blk_bslot_ptr = np.zeros(NB + 1, np.int64)
    np.cumsum(np.bincount(blk, minlength=NB), out=blk_bslot_ptr[1:])
    c1, c2 = np.triu_indices(C)
    c1, c2 = c1[blist], c2[blist]
    i32 = lambda a: np.asarray(a, np.int32)  # noqa: E731
    one = np.zeros(1, np.int32)
    # one record per supergroup (csrc/ba.hip kSgMeta): everything k_lin_mfma
    # needs before its first chunk's loads, in one hop
    sg_meta = np.zeros((NS, 24), np.int64)
    fch = sg_ptr[:-1]
    sg_meta[:, 0], sg_meta[:, 1] = sg_ptr[:-1], sg_ptr[1:]
    sg_meta[:, 2], sg_meta[:, 3] = grp_cslot[:-1], ms
    sg_meta[:, 4], sg_meta[:, 5] = grp_bslot[:-1], np.diff(grp_bslot)
    sg_meta[:, 6], sg_meta[:, 7] = grp_ptr[fch], grp_ptr[fch + 1]
    sg_meta[:, 8], sg_meta[:, 9] = pt_ptr[grp_ptr[fch]], pt_ptr[grp_ptr[fch + 1]]
    sg_meta[:, 10:18] = sg_cams
    return dict(
        mode=1, sg_meta=i32(sg_meta), perm=perm, order=order, obs_cam=i32(obs_cam), obs_pt=i32(obs_pt),
        pt_ptr=i32(pt_ptr), grp_ptr=i32(grp_ptr), grp_cslot=i32(grp_cslot),
        cslot_cam=i32(cslot_cam), cslot_obs_ptr=one, cslot_obs=one, grp_bslot=i32(grp_bslot),
        bslot_blk=i32(blk), bslot_pair_ptr=one, bslot_pairs=one,
        blocks=i32(np.stack([c1, c2], 1)), cam_cslot_ptr=i32(cam_cslot_ptr),
        cslot_row=i32(cslot_row), blk_bslot_ptr=i32(blk_bslot_ptr), bslot_row=i32(bslot_row),
        sg_ptr=i32(sg_ptr), sg_cams=i32(sg_cams), obs_la=i32(obs_la), chk_cobs=i32(chk_cobs),
        obs_meta=i32((obs_pt - grp_ptr[obs_chunk]) | (obs_la << 8) | (chk_cobs << 16))
        if O else np.zeros(0, np.int32),
        chk_optr=i32(pt_ptr[grp_ptr]), chk_cptr=i32(chk_cptr), bslot_ab=i32(bslot_a | (bslot_b << 8)),
        n_obs=O, n_grps=G, n_sgrps=NS, chunks_per_wg=S)


_PLAN_SHAPES = {"blocks": 2, "sg_meta": 24, "sg_cams": 8, "chk_cptr": 8}


def plan_mfma_native(n_cams, n_pts, cam_idx, pt_idx, block_list=None, chunks_per_wg=None):
    """plan_mfma in native code (libslam355 slam_ba_plan_mfma, host only): the
    same tables, as numpy views of ONE int32 buffer (`buf`, table k at
    `offs[k]`, 256-byte aligned) so BAProblem uploads them with a single copy.
    None when a point sees more than MF_CAMS cameras (or has more than
    MF_CHUNK_OBS observations)."""
    cam_idx = np.ascontiguousarray(cam_idx, np.int32).ravel()
    pt_idx = np.ascontiguousarray(pt_idx, np.int32).ravel()
    O = len(cam_idx)
    bl = None if block_list is None else np.ascontiguousarray(np.unique(block_list), np.int32)
    nbl = 0 if bl is None else len(bl)
    if bl is not None and nbl == 0:
        bl = np.zeros(1, np.int32)  # a non-null pointer: "given, and empty" (not "absent")
    cap = int(_lib.lib.slam_ba_plan_bound(n_cams, n_pts, O, nbl))
    if cap <= 0:
        raise ValueError("plan_mfma_native: bad sizes")
    buf = np.empty(cap, np.int32)
    info = _lib.PlanInfo()
    _lib.call("slam_ba_plan_mfma", n_cams, n_pts, O, cam_idx.ctypes.data, pt_idx.ctypes.data,
              None if bl is None else bl.ctypes.data, nbl,
              0 if chunks_per_wg is None else int(chunks_per_wg), buf.ctypes.data, cap,
              ctypes.byref(info))
    if not info.ok:
        return None
    buf = buf[:info.total]
    pl = dict(mode=1, buf=buf, offs={}, n_obs=info.n_obs, n_grps=info.n_grps,
              n_sgrps=info.n_sgrps, chunks_per_wg=info.chunks_per_wg)
    for k, name in enumerate(_lib.PLAN_TABLES):
        off, n = info.off[k], info.len[k]
        v = buf[off:off + n]
        if name in _PLAN_SHAPES:
            v = v.reshape(-1, _PLAN_SHAPES[name])
        pl[name] = v
        pl["offs"][name] = off
    one = np.zeros(1, np.int32)
    pl.update(cslot_obs_ptr=one, cslot_obs=one, bslot_pair_ptr=one, bslot_pairs=one)
    return pl


def assembly_table(n_cams, pl):
    """asm_tab of the folded assembly (include/slam355.h): need[NB] (partial rows
    per listed block: camera rows of its camera when diagonal + its block rows),
    cnt[NB] (zeros), cam_dblk[C], row_blk[n_bslots] (block of each block-major
    bpart row), n_empty, empty[] (blocks with no partial row)."""
    blocks = pl["blocks"].astype(np.int64)
    NB = len(blocks)
    bptr = pl["blk_bslot_ptr"].astype(np.int64)
    cptr = pl["cam_cslot_ptr"].astype(np.int64)
    diag = blocks[:, 0] == blocks[:, 1]
    need = np.diff(bptr)
    need[diag] += np.diff(cptr)[blocks[diag, 0]]
    cam_dblk = np.full(n_cams, -1, np.int64)
    cam_dblk[blocks[diag, 0]] = np.nonzero(diag)[0]
    if (cam_dblk < 0).any():
        raise ValueError("assembly_table: a camera's diagonal block is not listed")
    row_blk = np.repeat(np.arange(NB), np.diff(bptr))
    empty = np.nonzero(need == 0)[0]
    return np.concatenate([need, np.zeros(NB, np.int64), cam_dblk, row_blk, [len(empty)],
                           empty]).astype(np.int32)


def tiled_solve_flops(n_cams, blocks, tb=64):
    """Flops of the tiled Cholesky (csrc/ba.hip k_tl_*) for a packed block list
    [n_blocks, 2]: the 64x64 tiles it factors, solves and updates, with the
    structural fill-in tracked as the kernels track it (zero tiles skipped)."""
    n = 9 * n_cams
    T = (n + tb - 1) // tb
    nz = np.eye(T, dtype=bool)
    b = np.asarray(blocks, np.int64).reshape(-1, 2)
    i, j = np.meshgrid(np.arange(9), np.arange(9), indexing="ij")
    r = (9 * b[:, 0, None, None] + i[None]).ravel() // tb
    c = (9 * b[:, 1, None, None] + j[None]).ravel() // tb
    nz[np.maximum(r, c), np.minimum(r, c)] = True
    flops = 0.0
    g = 2.0 * tb ** 3
    for k in range(T):
        flops += tb ** 3 / 3.0 * 2  # factor + inverse of the diagonal tile
        rows = k + 1 + np.flatnonzero(nz[k + 1:, k])
        m = len(rows)
        flops += m * g + m * (m + 1) / 2 * g  # panel GEMMs + trailing updates
        if m:
            ii, jj = np.tril_indices(m)
            nz[rows[ii], rows[jj]] = True
    return flops


_MFMA_TABLES = ("sg_ptr", "sg_meta", "obs_meta", "chk_cptr", "bslot_ab")
_INDEX_TABLES = ("chk_optr", "obs_cam", "obs_pt", "pt_ptr", "grp_ptr", "grp_cslot", "cslot_cam",
                 "cslot_obs_ptr", "cslot_obs", "grp_bslot", "bslot_blk", "bslot_pair_ptr",
                 "bslot_pairs", "blocks", "cam_cslot_ptr", "cslot_row", "blk_bslot_ptr",
                 "bslot_row")


class BAProblem:
    """Device-resident BA problem + LM state.  `cams` [C,9], `pts` [P,3] float64."""

    def __init__(self, cams, pts, cam_idx, pt_idx, qs, *, lam0=1e-4, stream=None,
                 block_list=None, lin_mode="auto", chunks_per_wg=None, tl_mode="flow",
                 fold_assembly=False, tile_mode=None, active_blocks=True):
        """lin_mode: "mfma" (camera-union linearisation, k_lin_mfma: Schur
        contraction on the f64 matrix cores; points renumbered internally),
        "slot" (k_linearize, any observation structure) or "auto" (mfma when
        every point is seen by <= MF_CAMS cameras).  The tiled camera solve
        (9C > 120) follows the nested-dissection schedule of tl_schedule;
        tl_mode "flow" runs it as one dataflow launch (k_tl3_flow, on any
        stream and CU mask), "levels" one launch pair per elimination-tree level;
        tile_mode: the tiling of that solve (tile_rows; default TILE_MODE).
        active_blocks (packed systems): k_assemble only over the blocks with
        partial rows here (a landmark shard), a fill launch for the rest.
        fold_assembly (lin_mode mfma): k_lin_mfma's last supergroup per camera
        block sums the block's partial rows into the system (no k_assemble
        launch).  Off by default: measured slower (the workgroup that finishes
        last assembles every block it touched, a serial tail; 16 C3 windows
        326 vs 225 us per iteration, C4 406 vs 324 us, tracking 19.0k vs 19.9k
        frames/s, profiles/r4/fold_ab/ at f26058c; landmark shards at W = 8 too: C4
        296 vs 155 us, C5 903 vs 387 us per iteration, profiles/r6/asm_fold/)."""
        if tl_mode not in ("flow", "levels"):
            raise ValueError(f"tl_mode must be 'flow' or 'levels', not {tl_mode!r}")
        dev = require_gpu()
        cams = np.ascontiguousarray(cams, np.float64).reshape(-1, 9)
        pts = np.ascontiguousarray(pts, np.float64).reshape(-1, 3)
        C, P = len(cams), len(pts)
        cam_idx, pt_idx, qs = _check_indices(C, P, cam_idx, pt_idx, qs)
        pl = None
        if lin_mode in ("auto", "mfma"):
            pl = plan_mfma_native(C, P, cam_idx, pt_idx, block_list, chunks_per_wg)
            if pl is None and lin_mode == "mfma":
                raise ValueError(f"lin_mode 'mfma': a point is seen by more than {MF_CAMS} cameras")
        elif lin_mode != "slot":
            raise ValueError(f"lin_mode must be 'auto', 'mfma' or 'slot', not {lin_mode!r}")
        if pl is None:
            pl = plan(C, P, cam_idx, pt_idx, block_list)
            pl["mode"], pl["perm"] = 0, None
            pl["n_grps"], pl["n_sgrps"] = len(pl["grp_ptr"]) - 1, 0
        self.plan = pl
        self.lin_mode = "mfma" if pl["mode"] == 1 else "slot"
        self.perm = pl["perm"]  # device point k = caller's point perm[k] (None: identity)
        if self.perm is not None:
            pts = pts[self.perm]
        self.C, self.P, self.O = C, P, pl["n_obs"]
        self.stream = stream
        T = lambda a, dt=None: torch.from_numpy(np.ascontiguousarray(a)).to(dev)  # noqa: E731
        self.t = t = {}
        if "buf" in pl:  # native plan: every table in one buffer, one copy
            t["plan_buf"] = T(pl["buf"])
            for k in _INDEX_TABLES + _MFMA_TABLES:
                if k in pl["offs"]:
                    t[k] = t["plan_buf"][pl["offs"][k]:]  # (a zero-length table keeps its slot)
                else:
                    t[k] = T(pl[k].astype(np.int32))
        else:
            for k in _INDEX_TABLES + (_MFMA_TABLES if pl["mode"] == 1 else ()):
                arr = pl[k] if pl[k].size else np.zeros(1, np.int32)
                t[k] = T(arr.astype(np.int32))
        C9 = 9 * C
        G = pl["n_grps"]
        n_cs, n_bs = len(pl["cslot_cam"]), len(pl["bslot_blk"])
        self.sys_len = int(_lib.lib.slam_ba_sys_len(C, len(pl["blocks"])))
        self.tl_levels = C9 > LDS_MAX_N
        if self.tl_levels:  # schedule of the tiled solve (host copy; device copy below)
            self._sched_host = tl_schedule(C, pl["blocks"], tile_mode)
        # every float64 buffer in ONE device allocation (256-byte aligned
        # segments): the parameters (two LM copies + the initial copy) and the
        # permuted observations in one upload, the workspaces in one fill
        up = [("cams0", cams), ("pts0", pts), ("cams1", cams), ("pts1", pts), ("init_c", cams),
              ("init_p", pts), ("obs_q", qs[pl["order"]] if self.O else np.zeros((1, 2)))]
        zero = [("camrec0", C * 32), ("camrec1", C * 32), ("cpart", n_cs * 112), ("bpart", n_bs * 81),
                ("sys", self.sys_len), ("chol", _lib.lib.slam_ba_chol_len(C, self._sched_host.ctypes.data)
                                   if self.tl_levels else 1),
                ("delta_c", C9), ("red_part", _lib.lib.slam_ba_red_slots(G)), ("small", 4),
                ("state", N_STATE)]
        al = lambda n: (max(int(n), 1) + 31) // 32 * 32  # noqa: E731
        offs, o = {}, 0
        for k, a in up:
            offs[k] = o
            o += al(np.size(a))
        n_up = o
        for k, n in zero:
            offs[k] = o
            o += al(n)
        host = np.zeros(n_up, np.float64)
        for k, a in up:
            host[offs[k]:offs[k] + np.size(a)] = np.ravel(a)
        arena = torch.empty(o, dtype=torch.float64, device=dev)
        arena[:n_up].copy_(torch.from_numpy(host))
        arena[n_up:].zero_()
        t["f64_arena"] = arena
        for k, a in up:
            t[k] = arena[offs[k]:offs[k] + np.size(a)].view(np.shape(a))
        for k, n in zero:
            t[k] = arena[offs[k]:offs[k] + max(int(n), 1)]
        if self.tl_levels:
            t["tl_sched"] = T(self._sched_host)
        t["ticket"] = torch.zeros(1, dtype=torch.int32, device=dev)
        if stream is not None:  # the uploads and fills above ran on the current stream
            stream.wait_stream(torch.cuda.current_stream(dev))
        s = _Prob()
        s.n_cams, s.n_pts, s.n_obs, s.n_grps = C, P, self.O, G
        s.n_blocks = len(pl["blocks"])
        s.n_cslots, s.n_bslots = n_cs, n_bs
        s.lin_mode, s.n_sgrps = pl["mode"], pl["n_sgrps"]
        s.tl_mode = 0 if tl_mode == "flow" else 1
        s.cams[0], s.cams[1] = t["cams0"].data_ptr(), t["cams1"].data_ptr()
        s.pts[0], s.pts[1] = t["pts0"].data_ptr(), t["pts1"].data_ptr()
        s.camrec[0], s.camrec[1] = t["camrec0"].data_ptr(), t["camrec1"].data_ptr()
        for k in _INDEX_TABLES + ("obs_q", "cpart", "bpart", "sys", "chol", "delta_c",
                                  "red_part", "small", "state", "ticket") + \
                (_MFMA_TABLES if pl["mode"] == 1 else ()):
            setattr(s, k, t[k].data_ptr())
        if self.tl_levels:
            s.tl_sched = t["tl_sched"].data_ptr()
            s.tl_sched_host = self._sched_host.ctypes.data
        if pl["mode"] == 1 and fold_assembly:  # k_lin_mfma assembles sys itself
            t["asm_tab"] = T(assembly_table(C, pl))
            s.asm_tab = t["asm_tab"].data_ptr()
        elif self.tl_levels and active_blocks:
            # a landmark shard lists the global blocks but has partial rows for few
            # of them: k_assemble runs over the blocks with rows here (C5 rank 0
            # of 8: 3000 workgroups -> ~400), which also write the zeros of the
            # rest (table: the listed blocks, a flag per block, a flag per camera)
            blk = np.asarray(pl["blocks"]).reshape(-1, 2)
            bp = np.asarray(pl["blk_bslot_ptr"])
            cp = np.asarray(pl["cam_cslot_ptr"])
            rows = bp[1:] > bp[:-1]
            diag = blk[:, 0] == blk[:, 1]
            rows[diag] |= cp[blk[diag, 0] + 1] > cp[blk[diag, 0]]
            act = np.nonzero(rows)[0].astype(np.int32)
            if 0 < len(act) < len(blk):
                camrows = np.zeros(C, np.int32)
                camrows[blk[diag & rows, 0]] = 1
                t["asm_act"] = T(np.concatenate([act, rows.astype(np.int32), camrows]))
                s.asm_act, s.n_asm_act = t["asm_act"].data_ptr(), len(act)
        self._s = s
        self.reset(lam0)

        self._init = (t["init_c"], t["init_p"])

    def restore(self, lam0=1e-4):
        """Reload the initial parameters and reset the LM state (device copies)."""
        self.t["cams0"].copy_(self._init[0])
        self.t["pts0"].copy_(self._init[1])
        self.reset(lam0)

    # -- primitive phases -------------------------------------------------------
    def _sp(self):
        return stream_ptr(self.stream)

    def reset(self, lam0=1e-4):
        _lib.call("slam_ba_reset", ctypes.byref(self._s), float(lam0), self._sp())

    def build_system(self):
        _lib.call("slam_ba_build_system", ctypes.byref(self._s), self._sp())

    def solve_step(self):
        _lib.call("slam_ba_solve_step", ctypes.byref(self._s), self._sp())

    def decide(self):
        _lib.call("slam_ba_decide", ctypes.byref(self._s), self._sp())

    def iterate(self, n: int = 1):
        """n LM iterations, no host synchronisation (single rank)."""
        _lib.call("slam_ba_iterate", ctypes.byref(self._s), int(n), self._sp())

    def iterate_graphed(self, n: int = 1):
        """n LM iterations replayed from a captured HIP graph (one launch for
        the 13n kernels; captured on first use for each n)."""
        graphs = self.__dict__.setdefault("_graphs", {})
        if n not in graphs:
            g = torch.cuda.CUDAGraph()
            s = torch.cuda.Stream()  # capture needs a non-default stream
            s.wait_stream(torch.cuda.current_stream())
            saved = self.stream
            self.stream = s
            try:
                with torch.cuda.graph(g, stream=s):
                    self.iterate(n)
            finally:
                self.stream = saved
            torch.cuda.current_stream().wait_stream(s)
            graphs[n] = g
        with torch.cuda.stream(self.stream if self.stream is not None else
                               torch.cuda.current_stream()):
            graphs[n].replay()

    def _phase_graph(self, name, fn):
        """A captured HIP graph of one launch phase (captured on first use)."""
        graphs = self.__dict__.setdefault("_phase_graphs", {})
        if name not in graphs:
            g = torch.cuda.CUDAGraph()
            s = torch.cuda.Stream()
            s.wait_stream(torch.cuda.current_stream())
            saved = self.stream
            self.stream = s
            try:
                with torch.cuda.graph(g, stream=s):
                    fn()
            finally:
                self.stream = saved
            torch.cuda.current_stream().wait_stream(s)
            graphs[name] = g
        return graphs[name]

    def step_distributed(self, group=None, graphed=True, comm=None):
        """One LM iteration with RCCL all-reduce of the camera system (multi-rank).

        The kernels and the collectives are ordered on one stream: the body runs
        with self.stream current (torch.distributed orders its work against the
        current stream).  graphed: the linearisation (k_lin_mfma + k_assemble)
        and the solve (tiled factor + k_back_trial) are each one HIP-graph
        replay, so an iteration is 2 graph launches + k_decide + 2 collectives
        instead of ~8 kernel launches."""
        if comm is not None:  # slam355.dist.CapiComm: the whole iteration is one C call
            _lib.call("slam_ba_step_distributed", ctypes.byref(self._s), comm.handle, self._sp())
            return
        import torch.distributed as dist

        with torch.cuda.stream(self.stream if self.stream is not None
                               else torch.cuda.current_stream()):
            if graphed:
                build = self._phase_graph("build", self.build_system)
                solve = self._phase_graph("solve", self.solve_step)
                build.replay()
                dist.all_reduce(self.t["sys"], group=group)
                solve.replay()
            else:
                self.build_system()
                dist.all_reduce(self.t["sys"], group=group)
                self.solve_step()
            dist.all_reduce(self.t["small"], group=group)
            self.decide()

    # -- host views ---------------------------------------------------------------
    def state(self) -> dict:
        """The LM state; raises SlamError when a dataflow camera solve ever
        timed out in one of its flag waits (SOLVE_FAULT, fail code 2).  The
        solve makes no residency assumption (a start ticket hands out columns,
        the last retirer forms x), so a timeout means a hang or a hand-off
        ordering bug in the kernel, not a launch that was not co-resident."""
        s = self.t["state"].cpu().numpy()
        st = {k: float(s[v]) for k, v in ST.items()}
        if st["SOLVE_FAULT"] != 0.0:
            raise _lib.SlamError(f"BA camera solve: a dataflow wait timed out (fail code 2) "
                                 f"{int(st['SOLVE_FAULT'])} time(s) -- a hang or hand-off ordering "
                                 "bug in k_tl3_flow; the affected LM steps were rejected")
        return st

    def params(self):
        """(cams [C,9], pts [P,3]) at the live parameters, points in the caller's order."""
        cur = int(self.t["state"][ST["CUR"]].item() != 0)
        cams = self.t[f"cams{cur}"].cpu().numpy().copy()
        pts = self.t[f"pts{cur}"].cpu().numpy()
        if self.perm is not None:
            out = np.empty_like(pts)
            out[self.perm] = pts
            pts = out
        return cams, pts.copy()

    def cost(self) -> float:
        return self.state()["COST"]

    def solve(self, max_iters=100, ftol=1e-10, check_every=5):
        """Iterate until a batch of `check_every` iterations that accepted at
        least one step lowered the cost by less than ftol (relative), until
        lambda saturates (no step can be accepted any more), or max_iters.
        A batch whose steps were all rejected leaves the cost unchanged and
        says nothing about convergence, so it never stops the solve.
        Returns the final state dict."""
        done = 0
        st = self.state()
        while done < max_iters:
            k = min(check_every, max_iters - done)
            c0, n0 = st["COST"], st["NACCEPT"]
            self.iterate(k)
            done += k
            st = self.state()
            if st["LAMBDA"] >= 1e30:
                break
            if st["NACCEPT"] > n0 and abs(c0 - st["COST"]) <= ftol * max(st["COST"], 1e-300):
                break
        return st


class BABatch:
    """Independent BA problems (e.g. the local-BA windows of one tracking
    batch) advanced together: each LM iteration of all of them is one set of
    launches (slam_ba_iterate_batch: one problem per grid row, up to
    SLAM_BA_MAX_BATCH per launch), so B windows cost about one window's
    latency instead of B.  Every problem keeps its own device buffers and LM
    state; its iterates equal the ones BAProblem.iterate gives it alone."""

    MAX_BATCH = 16  # SLAM_BA_MAX_BATCH

    def __init__(self, problems, stream=None):
        self.problems = list(problems)
        if not self.problems:
            raise ValueError("BABatch needs at least one problem")
        if len(self.problems) > 1 and any(packed(p.C) for p in self.problems):
            raise ValueError(f"batched problems must have 9C <= {LDS_MAX_N} (one-workgroup solver)")
        self.stream = stream
        arr = (_Prob * len(self.problems))()
        for i, p in enumerate(self.problems):
            ctypes.memmove(ctypes.byref(arr[i]), ctypes.byref(p._s), ctypes.sizeof(_Prob))
        self._arr = arr
        self._graphs = {}
        # BAWindowSet problems: checked before every launch (their buffers are
        # reused two stage()/build() calls later)
        self._win = [p for p in self.problems if hasattr(p, "_live")]

    def _sp(self):
        return stream_ptr(self.stream)

    def reset(self, lam0=1e-4):
        _lib.call("slam_ba_reset_batch", self._arr, len(self.problems), float(lam0), self._sp())

    def restore(self, lam0=1e-4):
        """Reload every problem's initial parameters, reset every LM state."""
        with torch.cuda.stream(self.stream if self.stream is not None
                               else torch.cuda.current_stream()):
            # one multi-tensor copy launch for all windows: captured in a graph,
            # 2 copies per window were 2 memcpy nodes each, dispatched ~55 us
            # apart on a busy device (1 ms per launch set of 8 windows)
            torch._foreach_copy_([t for p in self.problems for t in (p.t["cams0"], p.t["pts0"])],
                                 [t for p in self.problems for t in p._init])
        self.reset(lam0)

    def iterate(self, n: int = 1):
        for p in self._win:
            p._live()
        _lib.call("slam_ba_iterate_batch", self._arr, len(self.problems), int(n), self._sp())

    def iterate_graphed(self, n: int = 1, with_restore=False):
        """n LM iterations of every problem (optionally preceded by restore())
        replayed from one captured HIP graph."""
        for p in self._win:
            p._live()
        key = (n, with_restore)
        if key not in self._graphs:
            g = torch.cuda.CUDAGraph()
            s = torch.cuda.Stream()
            s.wait_stream(torch.cuda.current_stream())
            saved = self.stream
            self.stream = s
            try:
                with torch.cuda.graph(g, stream=s):
                    if with_restore:
                        self.restore()
                    self.iterate(n)
            finally:
                self.stream = saved
            torch.cuda.current_stream().wait_stream(s)
            self._graphs[key] = g
        with torch.cuda.stream(self.stream if self.stream is not None else
                               torch.cuda.current_stream()):
            self._graphs[key].replay()

    def states(self):
        return [p.state() for p in self.problems]


# ----------------------------------------------------------------------------- kernels
def residuals(cams, pts, cam_idx, pt_idx, qs, *, jacobian=False):
    """objective()-order residuals [O,2] (and Jacobians [O,2,12]) on the GPU."""
    dev = require_gpu()
    cams = np.ascontiguousarray(cams, np.float64).reshape(-1, 9)
    pts = np.ascontiguousarray(pts, np.float64).reshape(-1, 3)
    cam_idx, pt_idx, qs = _check_indices(len(cams), len(pts), cam_idx, pt_idx, qs)
    O = len(cam_idx)
    if O == 0:
        return (np.zeros((0, 2)), np.zeros((0, 2, 12))) if jacobian else np.zeros((0, 2))
    T = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)  # noqa: E731
    tc, tp = T(cams), T(pts)
    ti, tj, tq = T(cam_idx.astype(np.int32)), T(pt_idx.astype(np.int32)), T(qs)
    r = torch.empty((O, 2), dtype=torch.float64, device=dev)
    if jacobian:
        J = torch.empty((O, 2, 12), dtype=torch.float64, device=dev)
        _lib.call("slam_ba_jacobian", ptr(tc), ptr(tp), ptr(ti), ptr(tj), ptr(tq), O, ptr(r),
                  ptr(J), stream_ptr())
        return r.cpu().numpy(), J.cpu().numpy()
    _lib.call("slam_ba_residual", ptr(tc), ptr(tp), ptr(ti), ptr(tj), ptr(tq), O, ptr(r),
              stream_ptr())
    return r.cpu().numpy()


class _WindowProblem(BAProblem):
    """A BAProblem whose buffers are views into a BAWindowSet's device memory
    (built by BAWindowSet.build / stage, not by __init__).  The kernels see raw
    pointers set at build time; the torch views (`t`, `_init`) that the
    BAProblem methods read are made on first use only.

    Lifetime: the set double-buffers its device memory, so the problems of one
    call stay valid through the next call; the call after that reuses their
    buffers, and from then on every use of them (launches, `state()`,
    `params()`, a new BABatch over them) raises RuntimeError instead of
    silently reading another batch's data."""

    def __init__(self):  # noqa: D107 (constructed by BAWindowSet only)
        pass

    def _live(self):
        if self._ws.gen[self._slot] != self._gen:
            raise RuntimeError("BAWindowSet problem used after its device buffers were reused "
                               "(problems stay valid for one further stage()/build() call)")

    @property
    def _s(self):
        self._live()
        return self._s_raw

    @property
    def t(self):
        self._live()
        if self._t is None:
            if self._views is None:  # staged by BAWindowSet.stage: offsets from its meta row
                self._views = BAWindowSet._views_of(self._d64, self._d32, self._meta)
            d64, d32, o64, o32, nb, offs = self._views
            t = {}
            for k, (o, shp) in o64.items():
                t[k] = d64[o:o + int(np.prod(shp))].view(shp)
            pb = d32[o32:o32 + nb]
            t["plan_buf"] = pb
            for k in _INDEX_TABLES + _MFMA_TABLES + ("perm",):
                t[k] = pb[offs[k]:] if k in offs else d32[o32 + nb:o32 + nb + 1]
            t["ticket"] = d32[o32 + nb + 4:o32 + nb + 5]
            self._t = t
        return self._t

    @property
    def _init(self):
        return (self.t["init_c"], self.t["init_p"])

    @property
    def perm(self):
        if self._perm is None:
            self._perm = self.t["perm"][:self.P].cpu().numpy().astype(np.int64)
        return self._perm

    @perm.setter
    def perm(self, v):
        self._perm = v


class BAWindowSet:
    """Many small BA problems built together for one launch set -- the local-BA
    windows formed from tracked frames (bench.py's tracked leg): each window
    planned by the native planner, every window's tables and float64 data
    (parameters, observations, zeroed workspaces: BAProblem's layout) staged in
    ONE pinned host buffer per type and uploaded by ONE asynchronous copy each,
    on the BA stream, into device buffers kept across calls; the returned
    problems have BAProblem's interface (state(), params(), BABatch).  Windows
    that need the slot linearisation (a point seen by more than MF_CAMS
    cameras) or the tiled solve (9C > 120) are built as ordinary BAProblems.

    Two sets of buffers alternate call by call -- pinned host staging and
    device memory alike -- so a call's problems stay valid through the next
    call (the bench's lag-2 pipeline launches step k's set while step k+1's
    is staged).  Set s is reused two calls later: its upload is ordered on
    `stream` after the launches of the problems it held (same stream), its
    host staging only after its previous upload has run (an event), and its
    generation is bumped, so the old problems then raise on any use
    (_WindowProblem._live) rather than read the new batch's data."""

    def __init__(self):
        self.dev = require_gpu()
        self.d = [[None, None], [None, None]]  # (f64, i32) device buffers per set
        self.h = [None, None]  # (f64, i32, event) host staging per set
        self.gen = [0, 0]  # calls that have filled each set
        self.k = 0

    def _claim(self):
        """The set this call fills: its generation bumped (the problems of its
        previous fill are dead from here on)."""
        slot = self.k & 1
        self.gen[slot] += 1
        return slot

    def _window(self, slot):
        bp = _WindowProblem()
        bp._ws, bp._slot, bp._gen = self, slot, self.gen[slot]
        return bp

    @staticmethod
    def _al(n):
        return (max(int(n), 1) + 31) // 32 * 32

    _F64 = ("cams0", "pts0", "cams1", "pts1", "init_c", "init_p", "obs_q", "camrec0", "camrec1",
            "cpart", "bpart", "sys", "chol", "delta_c", "red_part", "small", "state")
    META = 12 + len(_F64) + len(_lib.PLAN_TABLES)  # SLAM_STAGE_META

    @staticmethod
    def _views_of(d64, d32, m):
        """(d64, d32, {buffer: (offset, shape)}, int32 offset, plan length,
        {table: offset}) of a window staged by slam_ba_stage_windows (meta row m)."""
        C, P, O = int(m[1]), int(m[2]), int(m[3])
        n_cs, n_bs = int(m[6]), int(m[7])
        shp = {"cams0": (C, 9), "pts0": (P, 3), "cams1": (C, 9), "pts1": (P, 3), "init_c": (C, 9),
               "init_p": (P, 3), "obs_q": (max(O, 1), 2), "camrec0": (C * 32,), "camrec1": (C * 32,),
               "cpart": (max(n_cs * 112, 1),), "bpart": (max(n_bs * 81, 1),), "sys": (int(m[11]),),
               "chol": (1,), "delta_c": (9 * C,), "red_part": (max(_lib.lib.slam_ba_red_slots(int(m[4])), 1),),
               "small": (4,), "state": (N_STATE,)}
        o64 = {k: (int(m[12 + i]), shp[k]) for i, k in enumerate(BAWindowSet._F64)}
        base = 12 + len(BAWindowSet._F64)
        offs = {k: int(m[base + i]) for i, k in enumerate(_lib.PLAN_TABLES)}
        return d64, d32, o64, int(m[9]), int(m[10]), offs

    def stage(self, rows, cnt, maps, M, cams, u_off, v_off, stream, lam0=1e-4):
        """The tracked windows of one batch, staged by ONE native call
        (slam_ba_stage_windows: every window's observations from the mapper's
        rows, its plan, its float64 data and tables into the pinned staging
        buffers, its descriptor with the device addresses) and uploaded by one
        copy per type.  rows [B, cap, 4] (frame, map point, u, v), cnt [B],
        maps [W, map_cap, 3], M [W], cams [B, 9] with B = W n; window w = pairs
        w n .. w n + n - 1.  Windows the camera-union plan cannot take are
        built as ordinary BAProblems (from the same host arrays).  Returns the
        problems in window order (BAProblem interface)."""
        rows = np.ascontiguousarray(rows, np.float64)
        cnt = np.ascontiguousarray(cnt, np.int32)
        maps = np.ascontiguousarray(maps, np.float64)
        M = np.ascontiguousarray(M, np.int32)
        cams = np.ascontiguousarray(cams, np.float64).reshape(-1, 9)
        B, cap = rows.shape[0], rows.shape[1]
        W, map_cap = maps.shape[0], maps.shape[1]
        if W == 0 or B % W or len(cams) != B or len(cnt) != B or len(M) != W:
            raise ValueError("stage: rows / cnt / cams must cover W windows of B / W pairs each")
        n = B // W
        meta = np.zeros((W, self.META), np.int64)
        need = np.zeros(2, np.int64)
        probs = (_Prob * W)()
        args = (W, n, cap, rows.ctypes.data, cnt.ctypes.data, maps.ctypes.data, map_cap,
                M.ctypes.data, cams.ctypes.data, float(u_off), float(v_off))
        slot = self._claim()
        d = self.d[slot]
        hs = self.h[slot]
        if hs is not None:
            hs[2].synchronize()  # that set's previous upload has run
        for attempt in range(2):
            ok64 = hs is not None and d[0] is not None and hs[0].numel() <= d[0].numel()
            ok32 = hs is not None and d[1] is not None and hs[1].numel() <= d[1].numel()
            if ok64 and ok32:
                _lib.call("slam_ba_stage_windows", *args, hs[0].data_ptr(), hs[0].numel(),
                          hs[1].data_ptr(), hs[1].numel(), d[0].data_ptr(),
                          d[1].data_ptr(), ctypes.addressof(probs), meta.ctypes.data,
                          need.ctypes.data)
            else:
                _lib.call("slam_ba_stage_windows", *args, None, 0, None, 0, None, None, None,
                          meta.ctypes.data, need.ctypes.data)
            n64, n32 = int(need[0]), int(need[1])
            if ok64 and ok32 and n64 <= hs[0].numel() and n32 <= hs[1].numel():
                break
            # grow: pinned staging of this set and its device buffers (both sized
            # alike, so the device addresses written above stay valid)
            sz64, sz32 = max(n64, 1) * 3 // 2, max(n32, 1) * 3 // 2
            hs = [torch.zeros(sz64, dtype=torch.float64, pin_memory=True),
                  torch.zeros(sz32, dtype=torch.int32, pin_memory=True), torch.cuda.Event()]
            self.h[slot] = hs
            with torch.cuda.stream(stream):
                if d[0] is None or d[0].numel() < sz64:
                    d[0] = torch.empty(sz64, dtype=torch.float64, device=self.dev)
                if d[1] is None or d[1].numel() < sz32:
                    d[1] = torch.empty(sz32, dtype=torch.int32, device=self.dev)
        else:
            raise RuntimeError("stage: staging buffers could not be sized")
        self.k += 1
        with torch.cuda.stream(stream):
            if n64:
                d[0][:n64].copy_(hs[0][:n64], non_blocking=True)
            if n32:
                d[1][:n32].copy_(hs[1][:n32], non_blocking=True)
            hs[2].record(stream)
        out = []
        for w in range(W):
            m = meta[w]
            if not m[0]:  # not plannable here: an ordinary problem from the same rows
                om = np.concatenate([rows[b, :max(min(int(cnt[b]), cap), 0)] for b in range(w * n, w * n + n)])
                qs = np.stack([om[:, 2] - u_off, om[:, 3] - v_off], 1)
                out.append(BAProblem(cams[w * n:w * n + n].copy(), maps[w, :int(M[w])].copy(),
                                     om[:, 0].astype(np.int64), om[:, 1].astype(np.int64), qs,
                                     lam0=lam0, stream=stream))
                continue
            bp = self._window(slot)
            bp._t, bp._perm, bp._views = None, None, None
            bp._d64, bp._d32, bp._meta = d[0], d[1], m
            bp.plan, bp.lin_mode = None, "mfma"
            bp.C, bp.P, bp.O, bp.stream = int(m[1]), int(m[2]), int(m[3]), stream
            bp.sys_len, bp.tl_levels = int(m[11]), False
            bp._s_raw = probs[w]
            out.append(bp)
        built = [p for p in out if isinstance(p, _WindowProblem)]
        for i in range(0, len(built), BABatch.MAX_BATCH):
            BABatch(built[i:i + BABatch.MAX_BATCH], stream=stream).reset(lam0)
        return out

    def build(self, problems, stream, lam0=1e-4):
        specs, extra = [], []
        n64 = n32 = 0
        for w, (cams, pts, ci, pi, qs) in enumerate(problems):
            cams = np.ascontiguousarray(cams, np.float64).reshape(-1, 9)
            pts = np.ascontiguousarray(pts, np.float64).reshape(-1, 3)
            C, P = len(cams), len(pts)
            ci, pi, qs = _check_indices(C, P, ci, pi, qs)
            pl = plan_mfma_native(C, P, ci, pi) if 9 * C <= LDS_MAX_N else None
            if pl is None:
                extra.append(BAProblem(cams, pts, ci, pi, qs, lam0=lam0, stream=stream))
                continue
            if pl["perm"] is not None:
                pts = pts[pl["perm"]]
            O, G = pl["n_obs"], pl["n_grps"]
            n_cs, n_bs = len(pl["cslot_cam"]), len(pl["bslot_blk"])
            sys_len = int(_lib.lib.slam_ba_sys_len(C, len(pl["blocks"])))
            up = [("cams0", cams), ("pts0", pts), ("cams1", cams), ("pts1", pts), ("init_c", cams),
                  ("init_p", pts), ("obs_q", qs[pl["order"]] if O else np.zeros((1, 2)))]
            zero = [("camrec0", C * 32), ("camrec1", C * 32), ("cpart", n_cs * 112),
                    ("bpart", n_bs * 81), ("sys", sys_len), ("chol", 1), ("delta_c", 9 * C),
                    ("red_part", _lib.lib.slam_ba_red_slots(G)), ("small", 4), ("state", N_STATE)]
            o64 = {}
            for k, a in up:
                o64[k] = (n64, np.shape(a))
                n64 += self._al(np.size(a))
            for k, n in zero:
                o64[k] = (n64, (max(int(n), 1),))
                n64 += self._al(n)
            o32 = n32
            n32 += self._al(len(pl["buf"]) + 8)  # plan tables, 4 one-element stand-ins, ticket
            specs.append((w, C, P, pl, up, o64, o32))
        # staging (pinned, alternating sets) and device buffers (grown as needed)
        slot = self._claim()
        d = self.d[slot]
        hs = self.h[slot]
        if hs is not None:
            hs[2].synchronize()  # that set's previous upload has run
        if hs is None or hs[0].numel() < n64 or hs[1].numel() < n32:
            hs = [torch.zeros(max(n64, 1) * 3 // 2, dtype=torch.float64, pin_memory=True),
                  torch.zeros(max(n32, 1) * 3 // 2, dtype=torch.int32, pin_memory=True),
                  torch.cuda.Event()]
            self.h[slot] = hs
        self.k += 1
        h64, h32 = hs[0].numpy(), hs[1].numpy()
        h64[:n64] = 0.0
        for w, C, P, pl, up, o64, o32 in specs:
            for k, a in up:
                h64[o64[k][0]:o64[k][0] + np.size(a)] = np.ravel(a)
            nb = len(pl["buf"])
            h32[o32:o32 + nb] = pl["buf"]
            h32[o32 + nb:o32 + nb + 8] = 0
        with torch.cuda.stream(stream):
            if d[0] is None or d[0].numel() < n64:
                d[0] = torch.empty(max(n64, 1) * 3 // 2, dtype=torch.float64, device=self.dev)
            if d[1] is None or d[1].numel() < n32:
                d[1] = torch.empty(max(n32, 1) * 3 // 2, dtype=torch.int32, device=self.dev)
            d[0][:n64].copy_(hs[0][:n64], non_blocking=True)
            d[1][:n32].copy_(hs[1][:n32], non_blocking=True)
            hs[2].record(stream)
        out = [None] * len(problems)
        b64, b32 = d[0].data_ptr(), d[1].data_ptr()
        for w, C, P, pl, up, o64, o32 in specs:
            # raw pointers from the offsets (no torch view per buffer: ~30 per
            # window were most of the host build); the views are made on demand
            bp = self._window(slot)
            nb = len(pl["buf"])
            offs = pl["offs"]
            bp._t, bp._perm = None, None
            bp._views = (d[0], d[1], o64, o32, nb, offs)
            bp.plan, bp.lin_mode, bp.perm = pl, "mfma", pl["perm"]
            bp.C, bp.P, bp.O, bp.stream = C, P, pl["n_obs"], stream
            bp.sys_len, bp.tl_levels = int(o64["sys"][1][0]), False
            f64p = lambda k: b64 + 8 * o64[k][0]  # noqa: E731
            i32p = lambda k: b32 + 4 * (o32 + (offs[k] if k in offs else nb))  # noqa: E731
            s = _Prob()
            s.n_cams, s.n_pts, s.n_obs, s.n_grps = C, P, pl["n_obs"], pl["n_grps"]
            s.n_blocks = len(pl["blocks"])
            s.n_cslots, s.n_bslots = len(pl["cslot_cam"]), len(pl["bslot_blk"])
            s.lin_mode, s.n_sgrps, s.tl_mode = 1, pl["n_sgrps"], 0
            s.cams[0], s.cams[1] = f64p("cams0"), f64p("cams1")
            s.pts[0], s.pts[1] = f64p("pts0"), f64p("pts1")
            s.camrec[0], s.camrec[1] = f64p("camrec0"), f64p("camrec1")
            for k in _INDEX_TABLES + _MFMA_TABLES:
                setattr(s, k, i32p(k))
            for k in ("obs_q", "cpart", "bpart", "sys", "chol", "delta_c", "red_part", "small", "state"):
                setattr(s, k, f64p(k))
            s.ticket = b32 + 4 * (o32 + nb + 4)
            bp._s_raw = s
            out[w] = bp
        it = iter(extra)
        out = [p if p is not None else next(it) for p in out]
        # LM states of the set's problems reset together (the upload runs first: same stream)
        built = [p for p in out if isinstance(p, _WindowProblem)]
        for i in range(0, len(built), BABatch.MAX_BATCH):
            BABatch(built[i:i + BABatch.MAX_BATCH], stream=stream).reset(lam0)
        return out
