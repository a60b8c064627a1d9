"""Time slam_sgbm alone (HIP events) for the library named by SLAM355_LIB."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "slam-1_amd")]
from slam355 import vofront  # noqa: E402
from slam355.synthetic import stereo_sequence  # noqa: E402

L, R, _, _ = stereo_sequence(33, 1280, 720, seed=0)
l, r = torch.from_numpy(L).cuda(), torch.from_numpy(R).cuda()
for _ in range(2):
    vofront.sgbm(l, r, **vofront.SGBM)
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(5):
    vofront.sgbm(l, r, **vofront.SGBM)
e1.record()
torch.cuda.synchronize()
print(os.environ.get("SLAM355_LIB", "default"), f"{e0.elapsed_time(e1) / 5:.3f} ms per 33 pairs")
