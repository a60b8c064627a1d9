"""Per-phase cycle split of k_orb_tile on the bench's C2 batch (needs a library
built with -DSLAM_ORB_PROFILE)."""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "slam-1_amd")]

os.environ.setdefault("SLAM355_LIB", os.path.join(ROOT, "slam-1_amd", "prof", "libslam355_orbprof.so"))
import torch  # noqa: E402

from slam355 import _lib, orb  # noqa: E402
from slam355.synthetic import corridor_sequence  # noqa: E402

B = 32
KP = 64
L, R, _, _ = corridor_sequence(B + 1, 1280, 720, seed=1000, device="cuda", as_numpy=False)
imgs = torch.cat([L, R[:B]]).contiguous()
f = _lib.lib.slam_orb_profile_read
f.argtypes = [ctypes.c_void_p]
buf = (ctypes.c_ulonglong * 96)()
orb.orb_batch(imgs, KP)
f(buf)
ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
ev0.record()
for _ in range(5):
    orb.orb_batch(imgs, KP)
ev1.record()
torch.cuda.synchronize()
f(buf)
names = ["stage", "resize", "FAST", "NMS", "retain2n", "harris", "rank", "angle", "blur", "brief"]
tot = sum(buf[i] for i in range(10))
nwg = 5 * imgs.shape[0] * 36
print(f"ms/launch {ev0.elapsed_time(ev1) / 5:.3f}; cycles per WG {tot / nwg:.0f}")
for i, n in enumerate(names):
    print(f"  {n:9s} {buf[i] / nwg:9.0f} clk/WG  {100 * buf[i] / tot:5.1f}%")
print("per level (clk/WG):")
for lv in range(8):
    row = [buf[16 + 10 * lv + i] / nwg for i in range(10)]
    print(f"  L{lv} {sum(row):8.0f}  " + " ".join(f"{n}={v:.0f}" for n, v in zip(names, row) if v))
