"""Phase cycles of the tracking tail on the bench's batch: k_fm_hyp (one
workgroup: seven-point round, candidate evaluation, merge; candidates tested /
sent to the median select) and k_pnp (hypothesis load / counting / refinement,
median over pairs).  Library: build_prof_lib.sh tail -DSLAM_FMH_TRACE
-DSLAM_PNP_PROFILE (the latter overwrites rvec with the cycle counts)."""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "slam-1_amd")]
os.environ.setdefault("SLAM355_LIB", os.path.join(ROOT, "slam-1_amd", "prof", "libslam355_tail.so"))

import torch  # noqa: E402

from slam355 import _lib  # noqa: E402
from slam355.pipeline import Tracker  # noqa: E402
from slam355.synthetic import stereo_sequence  # noqa: E402

B = 32
L, R, poses, rig = stereo_sequence(B + 1, 1280, 720, seed=1000)
trk = Tracker(B, 720, 1280, rig.P_l, rig.P_r, max_kp_per_tile=64, seed=0)
trk.imgs.copy_(torch.from_numpy(np.concatenate([L, R[:B]])))
f = _lib.lib.slam_fmh_trace
f.argtypes = [ctypes.c_void_p]
for _ in range(3):
    trk.track(0)
    torch.cuda.synchronize()
    buf = (ctypes.c_ulonglong * 8)()
    f(buf)
    a = np.array(buf[:4], dtype=np.int64)
    print("k_fm_hyp WG(3,5) clk: seven-point", a[1] - a[0], "evaluate", a[2] - a[1], "merge", a[3] - a[2],
          "| candidates", buf[5], "median-selects", buf[6], "M", buf[7], flush=True)
cyc = trk.rvec.cpu().numpy()
print("k_pnp clk (median over pairs): hypotheses", np.median(cyc[:, 0]), "counting", np.median(cyc[:, 1]),
      "refinement", np.median(cyc[:, 2]))
print("stereo matches", trk.s_cnt.cpu().numpy()[:8] if hasattr(trk, "s_cnt") else "-",
      "temporal", trk.t_cnt.cpu().numpy()[:8])
