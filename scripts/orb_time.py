"""ms per ORB launch of the bench's C2 batch (65 textured-corridor images of
1280x720, 64 kp/tile) alone on the GPU, for A/B runs of library builds
(SLAM355_LIB=...): median of 30 launches timed by HIP events."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "slam-1_amd")]

import torch  # noqa: E402

from slam355 import _lib, orb  # noqa: E402
from slam355.synthetic import corridor_sequence  # noqa: E402

B = 32
L, R, _, _ = corridor_sequence(B + 1, 1280, 720, seed=1000, device="cuda", as_numpy=False)
imgs = torch.cat([L, R[:B]]).contiguous()
ws = orb.OrbWorkspace(imgs.shape[0], 720, 1280, 64)
for _ in range(3):
    ws.run(imgs)
ts = []
for _ in range(30):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    ws.run(imgs)
    e1.record()
    torch.cuda.synchronize()
    ts.append(e0.elapsed_time(e1))
cnt = ws.count.cpu().numpy()
desc = ws.desc.cpu().numpy()
chk = sum(int(desc[b, :cnt[b]].astype(np.int64).sum()) for b in range(len(cnt)))
print(f"{os.path.basename(_lib.LIB_PATH)} ms/launch median {np.median(ts):.4f} min {np.min(ts):.4f} "
      f"kp/frame {cnt.mean():.1f} desc checksum {chk}")
