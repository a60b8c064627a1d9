"""Runs the bench's C2 ORB batch (64 images of 1280x720) a few times; a
target for rocprofv3 counter passes on k_orb_tile."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "slam-1_amd")]

import torch  # noqa: E402

from slam355 import orb  # noqa: E402
from slam355.synthetic import stereo_sequence  # noqa: E402

B = 32
L, R, _, _ = stereo_sequence(B + 1, 1280, 720, seed=1000)
imgs = torch.from_numpy(np.concatenate([L, R[:B]])).cuda()
for _ in range(4):
    orb.orb_batch(imgs, 56)
torch.cuda.synchronize()
print("ok")
