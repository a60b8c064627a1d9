"""Dump the device LocalMap inputs/outputs of an 8-pair tracked batch (corridor
seed 21) to gpurun_out/localmap8.npz for CPU-side comparison with oracle.mapping."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "slam-1_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

from slam355.pipeline import LocalMap, Tracker  # noqa: E402
from slam355.synthetic import corridor_sequence  # noqa: E402

B = 8
L, R, poses, rig = corridor_sequence(B + 1, 1280, 720, seed=21)
trk = Tracker(B, 720, 1280, rig.P_l, rig.P_r, max_kp_per_tile=64, seed=6)
lm = LocalMap(trk)
trk.imgs.copy_(torch.from_numpy(np.concatenate([L[:B + 1], R[:B]])))
trk.track(0)
lm.add(0)
np.savez(os.path.join(ROOT, "gpurun_out", "localmap8.npz"), t_cnt=trk.t_cnt.cpu().numpy(),
         abs=lm.abs.cpu().numpy(), Q1=trk.Q1.cpu().numpy(), q1=trk.q1.cpu().numpy(),
         om=lm.optimization_matrix(), map=lm.store.points().cpu().numpy(),
         poses=np.stack(lm.poses))
print("saved")
