"""Runs the bench's C2 ORB batch (65 textured-corridor images of 1280x720, 64 kp
per tile) a few times; a target for rocprofv3 counter passes on k_orb_tile."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "slam-1_amd")]

import torch  # noqa: E402

from slam355 import orb  # noqa: E402
from slam355.synthetic import corridor_sequence  # noqa: E402

B = 32
L, R, _, _ = corridor_sequence(B + 1, 1280, 720, seed=1000, device="cuda", as_numpy=False)
imgs = torch.cat([L, R[:B]]).contiguous()
for _ in range(4):
    orb.orb_batch(imgs, 64)
torch.cuda.synchronize()
print("ok")
