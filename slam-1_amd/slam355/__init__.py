"""slam355 — MI355X-native (gfx950) hot path of DavidHan008/SLAM-1.

Host code mirrors the reference's Python API (orb.py, keypoint.py, Point3D.py,
transformation.py, tracking.py, BundleAdjustment.py); every compute step runs
in hand-written HIP kernels of libslam355.so called through ctypes.
"""
from . import _lib  # noqa: F401  (fails loudly if libslam355.so is missing)

__version__ = "0.1.0"
ABI_VERSION = _lib.lib.slam_abi_version()
