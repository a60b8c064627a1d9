"""Phase cycles of one k_pnp_hyp workgroup (build_prof_lib.sh pnph -DSLAM_PNPH_TRACE)."""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "slam-1_amd"), os.path.join(ROOT, "tests")]
os.environ["SLAM355_LIB"] = os.path.join(ROOT, "slam-1_amd", "prof", "libslam355_pnph.so")
import torch  # noqa: E402
from slam355 import _lib, geometry  # noqa: E402
from test_geometry import _scene  # noqa: E402

B = 8
sc = [_scene(s, n=150, large=(s % 2 == 0)) for s in range(B)]
Q = torch.from_numpy(np.stack([s[1] for s in sc])).cuda()
q = torch.from_numpy(np.stack([s[2] for s in sc])).cuda()
cnt = torch.full((B,), 150, dtype=torch.int32, device="cuda")
f = _lib.lib.slam_pnph_trace
f.argtypes = [ctypes.c_void_p]
for _ in range(3):
    geometry.pnp_ransac(Q, q, cnt, sc[0][0].K, seed=1)
    buf = (ctypes.c_ulonglong * 8)()
    f(buf)
    a = np.array(buf[:7], dtype=np.int64)
    print("sample+bary, mtm, jacobi, lrho, approx, lm:", np.diff(a).tolist(), "sweeps", buf[7])
