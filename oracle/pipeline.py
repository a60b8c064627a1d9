"""ORACLE (test infrastructure only): one tracking step of /root/reference/main.py:79-97
on the CPU, chaining the oracle restatements (ORB, exact kNN-2 + ratio, seeded
F-LMedS, DLT, temporal gate, seeded PnP)."""
from __future__ import annotations

import numpy as np

from . import orb_tiles
from .geometry import fundamental_lmeds, pnp_ransac, triangulate_points_local
from .matching import stereo_matches, temporal_matches


def track_pair(left_i, right_i, left_i1, P_l, P_r, max_kp=56, seed=0, frame=0,
               max_distance=500.0, orb_cache=None):
    """-> dict with the intermediate counts and (rvec, tvec, n_inliers, inlier mask)."""
    cache = orb_cache if orb_cache is not None else {}

    def orb(img, key):
        if key not in cache:
            cache[key] = orb_tiles(img, max_kp)
        return cache[key]

    kl, _, dl = orb(left_i, ("L", frame))
    kr, _, dr = orb(right_i, ("R", frame))
    kl1, _, dl1 = orb(left_i1, ("L", frame + 1))
    pl, pr, dL, dR = stereo_matches(kl[:, :2], dl, kr[:, :2], dr)
    mask, F, nf, _ = fundamental_lmeds(pl, pr, seed=seed, item=frame)
    pl, pr, dL, dR = pl[mask], pr[mask], dL[mask], dR[mask]
    X = triangulate_points_local(pl, pr, P_l, P_r)
    q2, Q1, q1 = temporal_matches(dL, pl, kl1[:, :2], dl1, X, max_distance)
    K = np.asarray(P_l)[:3, :3]
    rv, tv, n, m = pnp_ransac(Q1, q2, K, seed=seed, item=frame)
    return dict(n_orb=(len(kl), len(kr)), n_stereo=len(mask), f_mask=mask, n_f=int(mask.sum()),
                X=X, Q1=Q1, q2=q2, q1=q1, n_temporal=len(q2), rvec=rv, tvec=tv, n_pnp=n, pnp_mask=m)
