"""Phase cycles of k_pnp on the bench's tracking batch (library built with
-DSLAM_PNP_PROFILE, which overwrites rvec with the cycle counts)."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "slam-1_amd")]

import torch  # noqa: E402

from slam355.pipeline import Tracker  # noqa: E402
from slam355.synthetic import stereo_sequence  # noqa: E402

B = 32
L, R, poses, rig = stereo_sequence(B + 1, 1280, 720, seed=1000)
trk = Tracker(B, 720, 1280, rig.P_l, rig.P_r, max_kp_per_tile=56, seed=0)
trk.imgs.copy_(torch.from_numpy(np.concatenate([L, R[:B]])))
for _ in range(3):
    trk.track(0)
torch.cuda.synchronize()
cyc = trk.rvec.cpu().numpy()
print("hypotheses / counting / refinement cycles (median over pairs):", np.median(cyc, 0))
print("temporal points per pair:", trk.t_cnt.cpu().numpy()[:8])
