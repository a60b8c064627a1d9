"""Seeded synthetic inputs (no datasets are reachable): descriptor sets, stereo
image sequences and BA problems of the BASELINE.json config shapes.
See SURVEY.md §8d for the definitions."""
from __future__ import annotations

import numpy as np


def descriptor_set(rng, nq, nt, frac_planted=0.6, flip_p=0.08):
    """Nt uniform random 32-byte rows; Nq rows of which `frac_planted` are
    copies of random train rows with each bit flipped w.p. flip_p (d ~ 20)."""
    t = rng.integers(0, 256, (nt, 32), dtype=np.uint8)
    q = rng.integers(0, 256, (nq, 32), dtype=np.uint8)
    if nt:
        pick = rng.random(nq) < frac_planted
        src = rng.integers(0, nt, nq)
        bits = np.unpackbits(t[src], axis=1) ^ (rng.random((nq, 256)) < flip_p).astype(np.uint8)
        q[pick] = np.packbits(bits, axis=1)[pick]
    return q, t


def descriptor_batch(B, nq, nt, seed=0):
    rng = np.random.default_rng(seed)
    q = np.empty((B, nq, 32), np.uint8)
    t = np.empty((B, nt, 32), np.uint8)
    for b in range(B):
        q[b], t[b] = descriptor_set(rng, nq, nt)
    return q, np.full(B, nq, np.int32), t, np.full(B, nt, np.int32)


def _rodrigues(r):
    th = float(np.linalg.norm(r))
    if th == 0.0:
        return np.eye(3)
    k = r / th
    K = np.array([[0, -k[2], k[1]], [k[2], 0, -k[0]], [-k[1], k[0], 0]])
    return np.eye(3) + np.sin(th) * K + (1 - np.cos(th)) * K @ K


def bal_project(X, cams):
    """BAL projection (camera looks down -z, radial k1/k2) for input synthesis."""
    w = cams[:, :3]
    th = np.linalg.norm(w, axis=1)
    k = np.divide(w, th[:, None], out=np.zeros_like(w), where=th[:, None] > 0)
    K = np.zeros((len(w), 3, 3))
    K[:, 0, 1], K[:, 0, 2], K[:, 1, 2] = -k[:, 2], k[:, 1], -k[:, 0]
    K[:, 1, 0], K[:, 2, 0], K[:, 2, 1] = k[:, 2], -k[:, 1], k[:, 0]
    R = (np.eye(3)[None] + np.sin(th)[:, None, None] * K
         + (1 - np.cos(th))[:, None, None] * (K @ K))
    P = np.einsum("oij,oj->oi", R, X) + cams[:, 3:6]
    p = -P[:, :2] / P[:, 2:3]
    n = np.sum(p * p, axis=1)
    rad = 1 + cams[:, 7] * n + cams[:, 8] * n * n
    return p * (rad * cams[:, 6])[:, None]


def ba_problem(rng, n_cams, n_pts, obs_per_pt, f=716.8, noise=0.5):
    """Local-BA problem of SURVEY.md §8d: cameras 1 m apart along -z (BAL: the
    camera looks down -z), each point tracked by `obs_per_pt` consecutive
    keyframes from its anchor, sigma = `noise` px.  Returns
    (cams [C,9], pts [P,3], cam_idx [O], pt_idx [O], qs [O,2]), observations in
    shuffled order (the reference does not sort them)."""
    C = np.stack([rng.normal(0, 0.05, n_cams), rng.normal(0, 0.05, n_cams),
                  -np.arange(n_cams, dtype=float)], 1)
    rot = rng.normal(0, 0.02, (n_cams, 3))
    cams = np.zeros((n_cams, 9))
    for c in range(n_cams):
        cams[c, :3] = rot[c]
        cams[c, 3:6] = -_rodrigues(rot[c]) @ C[c]
        cams[c, 6] = f
    anchor = rng.integers(0, n_cams - obs_per_pt + 1, n_pts)
    depth = rng.uniform(8.0, 60.0, n_pts)
    X = C[anchor] + np.stack([rng.uniform(-0.4, 0.4, n_pts) * depth,
                              rng.uniform(-0.25, 0.25, n_pts) * depth, -depth], 1)
    cam_idx = (anchor[:, None] + np.arange(obs_per_pt)[None, :]).ravel()
    pt_idx = np.repeat(np.arange(n_pts), obs_per_pt)
    perm = rng.permutation(len(cam_idx))
    cam_idx, pt_idx = cam_idx[perm], pt_idx[perm]
    qs = bal_project(X[pt_idx], cams[cam_idx]) + rng.normal(0, noise, (len(cam_idx), 2))
    return cams, X, cam_idx.astype(np.int64), pt_idx.astype(np.int64), qs


def _log_so3(R):
    """Rotation vector of a rotation matrix (angle < pi)."""
    c = np.clip((np.trace(R) - 1.0) * 0.5, -1.0, 1.0)
    th = np.arccos(c)
    w = np.array([R[2, 1] - R[1, 2], R[0, 2] - R[2, 0], R[1, 0] - R[0, 1]])
    return w * 0.5 if th < 1e-12 else w * (th / (2.0 * np.sin(th)))


def ba_problem_loop(rng, n_cams, n_pts, obs_per_pt, f=716.8, noise=0.5, step=1.0):
    """Loop-closure global-BA problem (BASELINE config 5 shape): keyframes `step`
    m apart on a closed circular trajectory (the reference closes loops between
    the last and first frames, main.py:100-118), each landmark seen by
    `obs_per_pt` consecutive keyframes from its anchor, modulo n_cams, so the
    tracks of the last keyframes continue into the first ones (the loop-closure
    camera blocks of S).  BAL convention (camera looks down -z).  Returns the
    same tuple as ba_problem."""
    R0 = n_cams * step / (2.0 * np.pi)
    phi = 2.0 * np.pi * np.arange(n_cams) / n_cams
    centers = np.stack([R0 * np.cos(phi), rng.normal(0, 0.05, n_cams), R0 * np.sin(phi)], 1)
    fwd = np.stack([-np.sin(phi), np.zeros(n_cams), np.cos(phi)], 1)
    cams = np.zeros((n_cams, 9))
    Rs = np.empty((n_cams, 3, 3))
    for c in range(n_cams):
        z = -fwd[c]
        y = np.array([0.0, 1.0, 0.0])
        x = np.cross(y, z)
        R = np.stack([x, y, z]) @ _rodrigues(rng.normal(0, 0.02, 3)).T
        Rs[c] = R
        cams[c, :3] = _log_so3(R)
        cams[c, 3:6] = -R @ centers[c]
        cams[c, 6] = f
    anchor = rng.integers(0, n_cams, n_pts)
    depth = rng.uniform(8.0, 60.0, n_pts)
    side = np.cross(np.array([0.0, 1.0, 0.0]), -fwd[anchor])
    X = (centers[anchor] + fwd[anchor] * depth[:, None]
         + side * (rng.uniform(-0.4, 0.4, n_pts) * depth)[:, None]
         + np.array([0.0, 1.0, 0.0]) * (rng.uniform(-0.25, 0.25, n_pts) * depth)[:, None])
    cam_idx = ((anchor[:, None] + np.arange(obs_per_pt)[None, :]) % n_cams).ravel()
    pt_idx = np.repeat(np.arange(n_pts), obs_per_pt)
    perm = rng.permutation(len(cam_idx))
    cam_idx, pt_idx = cam_idx[perm], pt_idx[perm]
    qs = bal_project(X[pt_idx], cams[cam_idx]) + rng.normal(0, noise, (len(cam_idx), 2))
    return cams, X, cam_idx.astype(np.int64), pt_idx.astype(np.int64), qs


def pose_chain_loop(rng, m, step=1.0, rot_s=1e-3, t_s=1e-2):
    """car_params [6m] of the reference's live pose chain (BundleAdjustment.py:
    107-145: m relative poses [r0 r1 r2 t0 t1 t2], t2 the forward motion) for a
    closed planar loop of m keyframes (BASELINE config 5: 500 keyframes) --
    every relative pose turns 2 pi / m about y and moves `step` forward, so the
    exact chain closes (a planar rigid motion is a rotation about a point; its
    m-th power is the identity) -- plus the drift of tracking: Gaussian noise
    rot_s on the rotation vectors and t_s on the translations, which opens the
    loop for the loop-closure rows to pull shut."""
    p = np.zeros((m, 6))
    p[:, 1] = 2.0 * np.pi / m
    p[:, 5] = step
    p[:, :3] += rng.normal(0, rot_s, (m, 3))
    p[:, 3:] += rng.normal(0, t_s, (m, 3))
    return p.ravel()


def perturb(rng, cams, pts, rot_s=1e-3, t_s=1e-2, p_s=0.05):
    """Initialisation noise of SURVEY.md §8d (rotvec 1e-3, t 1e-2 m, points 5 cm)."""
    c = cams.copy()
    c[:, :3] += rng.normal(0, rot_s, c[:, :3].shape)
    c[:, 3:6] += rng.normal(0, t_s, c[:, 3:6].shape)
    return c, pts + rng.normal(0, p_s, pts.shape)


# ----------------------------------------------------------------------------- stereo sequences
class StereoRig:
    """Pinhole stereo pair of SURVEY.md §8d: fx = fy = 0.56 W, principal point at
    the centre, baseline 0.54 m (P_r[0,3] = -fx * b), KITTI calib.txt layout."""

    def __init__(self, W, H, baseline=0.54):
        self.W, self.H = W, H
        f = 0.56 * W
        self.K = np.array([[f, 0, W / 2.0], [0, f, H / 2.0], [0, 0, 1.0]])
        self.P_l = np.hstack([self.K, np.zeros((3, 1))])
        self.P_r = self.P_l.copy()
        self.P_r[0, 3] = -f * baseline
        self.baseline = baseline

    def calib_text(self):
        """Two lines of 12 floats, the format load_calib reads
        (/root/reference/visual_odometry_solution_methods.py:9-17)."""
        return "\n".join(" ".join(repr(float(v)) for v in P.ravel())
                         for P in (self.P_l, self.P_r)) + "\n"


def _value_noise(rng, H, W, cell=240, lo=100, hi=150):
    gh, gw = H // cell + 2, W // cell + 2
    g = rng.uniform(lo, hi, (gh, gw))
    ys = np.arange(H) / cell
    xs = np.arange(W) / cell
    y0, x0 = ys.astype(int), xs.astype(int)
    fy, fx = (ys - y0)[:, None], (xs - x0)[None, :]
    a = g[y0][:, x0]
    b = g[y0][:, x0 + 1]
    c = g[y0 + 1][:, x0]
    d = g[y0 + 1][:, x0 + 1]
    return (a * (1 - fx) + b * fx) * (1 - fy) + (c * (1 - fx) + d * fx) * fy


def make_world(rng, n_frames, n_landmarks=800):
    """Corridor of landmarks: x in [-20,20], y in [-3,3], z in [5, 80 + frames].
    Each landmark is a square patch of 16..32 px carrying its own 4x4 grid of
    random intensities, so its corners have distinctive rBRIEF descriptors
    (a sparse scene: dense clutter turns most corners into occlusion
    junctions that differ between the stereo views)."""
    z = rng.uniform(5.0, 80.0 + n_frames, n_landmarks)
    X = np.stack([rng.uniform(-20, 20, n_landmarks), rng.uniform(-3, 3, n_landmarks), z], 1)
    size = rng.integers(16, 33, n_landmarks)
    tex = rng.integers(0, 256, (n_landmarks, 4, 4)).astype(np.float64)
    return X, size, tex


def trajectory(rng, n_frames, step=1.0, yaw_sigma_deg=0.2):
    """Camera-to-world poses (4x4): forward 1 m/frame along +z, yaw jitter."""
    poses = []
    yaw = 0.0
    pos = np.zeros(3)
    for i in range(n_frames):
        c, s = np.cos(yaw), np.sin(yaw)
        R = np.array([[c, 0, s], [0, 1, 0], [-s, 0, c]])
        T = np.eye(4)
        T[:3, :3], T[:3, 3] = R, pos
        poses.append(T)
        pos = pos + R @ np.array([0, 0, step])
        yaw += np.deg2rad(rng.normal(0, yaw_sigma_deg))
    return np.stack(poses)


def render(world, T_cw_inv, rig: StereoRig, rng, x_offset=0.0, bg=None, noise=2.0):
    """Render one grayscale view: textured landmark patches (painter's order:
    far first) over value noise, plus Gaussian noise; x_offset shifts the
    camera along its x axis (right camera = +baseline)."""
    X, size, tex = world
    H, W = rig.H, rig.W
    img = (bg if bg is not None else _value_noise(rng, H, W)).copy()
    R, t = T_cw_inv[:3, :3], T_cw_inv[:3, 3]
    Xc = X @ R.T + t
    Xc[:, 0] -= x_offset
    vis = np.nonzero(Xc[:, 2] > 1.0)[0]
    Xc = Xc[vis]
    u = rig.K[0, 0] * Xc[:, 0] / Xc[:, 2] + rig.K[0, 2]
    v = rig.K[1, 1] * Xc[:, 1] / Xc[:, 2] + rig.K[1, 2]
    inb = (u > -20) & (u < W + 20) & (v > -20) & (v < H + 20)
    lid, u, v, z = vis[inb], u[inb], v[inb], Xc[inb, 2]
    order = np.argsort(-z, kind="stable")
    lid, u, v = lid[order], u[order], v[order]
    sz = size[lid]
    x0 = np.round(u - sz / 2).astype(np.int64)
    y0 = np.round(v - sz / 2).astype(np.int64)
    pix, rank, val = [], [], []
    for s in np.unique(sz):
        m = np.nonzero(sz == s)[0]
        dy, dx = np.meshgrid(np.arange(s), np.arange(s), indexing="ij")
        cell = (dy * 4 // s).ravel() * 4 + (dx * 4 // s).ravel()
        yy = y0[m, None] + dy.ravel()[None, :]
        xx = x0[m, None] + dx.ravel()[None, :]
        ok = (yy >= 0) & (yy < H) & (xx >= 0) & (xx < W)
        vals = tex[lid[m]].reshape(len(m), 16)[:, cell]
        pix.append((yy * W + xx)[ok])
        rank.append(np.broadcast_to(m[:, None], yy.shape)[ok])
        val.append(vals[ok])
    if pix:
        pix, rank, val = np.concatenate(pix), np.concatenate(rank), np.concatenate(val)
        srt = np.argsort(rank, kind="stable")
        img.reshape(-1)[pix[srt]] = val[srt]  # later (nearer) writes win
    img = img + rng.normal(0, noise, img.shape)
    return np.clip(np.rint(img), 0, 255).astype(np.uint8)


def stereo_sequence(n_frames, W=1280, H=720, seed=0, n_landmarks=800):
    """(left [F,H,W] u8, right [F,H,W] u8, poses [F,4,4] camera-to-world, rig)."""
    rng = np.random.default_rng(seed)
    rig = StereoRig(W, H)
    world = make_world(rng, n_frames, n_landmarks)
    poses = trajectory(rng, n_frames)
    bg = _value_noise(rng, H, W)
    left = np.empty((n_frames, H, W), np.uint8)
    right = np.empty((n_frames, H, W), np.uint8)
    for i in range(n_frames):
        Tinv = np.linalg.inv(poses[i])
        left[i] = render(world, Tinv, rig, rng, 0.0, bg)
        right[i] = render(world, Tinv, rig, rng, rig.baseline, bg)
    return left, right, poses, rig


# ----------------------------------------------------------------------------- textured corridor
# The landmark-sprite scene above is sparse (<= ~1200 ORB keypoints per
# 1280x720 frame); packing more sprites turns corners into occlusion junctions
# that differ between the stereo views.  The headline config (BASELINE C2:
# 2000 kp/frame) uses a textured corridor instead: every pixel lies on a
# plane (two walls, floor, ceiling, an end wall), textured with hashed random
# intensity cells fixed in world coordinates, so corners are geometrically
# consistent between views and frames.  2x2 supersampling anti-aliases far
# cells; Gaussian noise sigma 2 as in render().  Written in torch so the bench
# renders its sequence on the GPU in milliseconds per view (the CPU path is
# the same code; tests render a few views there).
CORRIDOR = dict(half_width=7.0, floor=2.0, ceiling=5.0, end=400.0, cell=0.3)


def _hash_cells(i, j, k: int):
    import torch

    h = (i * 73856093) ^ (j * 19349663) ^ (k * 83492791)
    h = (h ^ (h >> 13)) * 0x5BD1E995
    h = h ^ (h >> 15)
    return (h & 255).to(torch.float64)


def render_corridor(T_cw, rig: StereoRig, gen, x_offset=0.0, ss=2, noise=2.0, device="cpu",
                    **kw):
    """One grayscale view (uint8 torch tensor [H, W] on `device`) of the
    textured corridor from camera-to-world pose T_cw; x_offset shifts the camera
    along its x axis (right camera = +baseline).  `gen`: torch.Generator of the
    noise, on `device`."""
    import torch

    geo = dict(CORRIDOR, **kw)
    H, W, K = rig.H, rig.W, rig.K
    f64 = dict(dtype=torch.float64, device=device)
    o = (torch.arange(ss, **f64) + 0.5) / ss - 0.5
    vv = torch.arange(H, **f64)[:, None, None, None] + o[None, :, None, None]
    uu = torch.arange(W, **f64)[None, None, :, None] + o[None, None, None, :]
    x = ((uu - K[0, 2]) / K[0, 0]).expand(H, ss, W, ss)
    y = ((vv - K[1, 2]) / K[1, 1]).expand(H, ss, W, ss)
    Rn = np.asarray(T_cw, np.float64)[:3, :3]
    R = torch.as_tensor(Rn, **f64)
    c = torch.as_tensor(np.asarray(T_cw, np.float64)[:3, 3] + Rn @ np.array([x_offset, 0.0, 0.0]),
                        **f64)
    d = [R[a, 0] * x + R[a, 1] * y + R[a, 2] for a in range(3)]
    best = torch.full((H, ss, W, ss), float("inf"), **f64)
    val = torch.zeros((H, ss, W, ss), **f64)
    planes = [(0, -geo["half_width"], 0), (0, geo["half_width"], 1), (1, geo["floor"], 2),
              (1, -geo["ceiling"], 3), (2, geo["end"], 4)]
    for ax, pos, pid in planes:
        t = (pos - c[ax]) / d[ax]
        ok = (t > 0) & (t < best)
        a1, a2 = [a for a in range(3) if a != ax]
        cells = []
        for a in (a1, a2):
            q = torch.floor((c[a] + t * d[a]) / geo["cell"])
            cells.append(torch.nan_to_num(q, 0.0, 0.0, 0.0).clamp(-2.0 ** 40, 2.0 ** 40)
                         .to(torch.int64))
        v = _hash_cells(cells[0], cells[1], pid)
        best = torch.where(ok, t, best)
        val = torch.where(ok, v, val)
    img = val.mean(dim=(1, 3))
    img = img + noise * torch.randn((H, W), generator=gen, **f64)
    return torch.clamp(torch.round(img), 0, 255).to(torch.uint8)


def corridor_sequence(n_frames, W=1280, H=720, seed=0, device="cpu", as_numpy=True, frames=None,
                      **geo):
    """(left [F,H,W] u8, right [F,H,W] u8, poses [F,4,4] camera-to-world, rig) of
    the textured corridor; the trajectory is trajectory() (1 m/frame, yaw
    jitter 0.2 deg).  torch tensors on `device` unless as_numpy.  `geo`
    overrides CORRIDOR entries (e.g. a coarser `cell` at 640x480).

    frames: render only these frame indices (left/right hold them in that
    order; poses stay the whole sequence's), each view's noise drawn from a
    generator seeded by (seed, frame), so every subset of one sequence holds
    the same images -- the ranks of a sharded run render only their own
    frames.  (frames=None keeps the one sequential generator.)"""
    import torch

    rng = np.random.default_rng(seed)
    rig = StereoRig(W, H)
    poses = trajectory(rng, n_frames)
    ids = list(range(n_frames)) if frames is None else [int(f) for f in frames]
    gen = torch.Generator(device=device).manual_seed(seed)
    left = torch.empty((len(ids), H, W), dtype=torch.uint8, device=device)
    right = torch.empty((len(ids), H, W), dtype=torch.uint8, device=device)
    for k, i in enumerate(ids):
        if frames is not None:
            gen.manual_seed(seed * 1_000_003 + i)
        left[k] = render_corridor(poses[i], rig, gen, 0.0, device=device, **geo)
        right[k] = render_corridor(poses[i], rig, gen, rig.baseline, device=device, **geo)
    if as_numpy:
        return left.cpu().numpy(), right.cpu().numpy(), poses, rig
    return left, right, poses, rig
