"""ctypes binding of libslam355.so (the C ABI declared in include/slam355.h).

There is no CPU fallback anywhere in slam355: if the shared library is missing
or no GPU is visible, every compute entry point raises.  PyTorch-ROCm tensors
are used only as device-memory containers (``data_ptr()``) and for the HIP
stream handle.
"""
from __future__ import annotations

import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "libslam355.so")

c_int = ctypes.c_int
c_double = ctypes.c_double
c_size_t = ctypes.c_size_t
c_p = ctypes.c_void_p
c_uint64 = ctypes.c_uint64

# name -> argtypes (restype is int unless listed in _RESTYPE)
SIGNATURES = {
    "slam_abi_version": [],
    "slam_last_error": [],
    "slam_device_count": [],
    "slam_hamming_knn2": [c_p, c_p, c_int, c_p, c_p, c_int, c_int, c_p, c_p, c_p, c_p],
    "slam_compact_matches": [c_p, c_p, c_p, c_int, c_int, c_p, c_double, c_p, c_p, c_p],
}
_RESTYPE = {"slam_last_error": ctypes.c_char_p}


class SlamError(RuntimeError):
    """A libslam355 call returned a non-zero status."""


def _load():
    if not os.path.exists(LIB_PATH):
        raise ImportError(
            f"libslam355.so not found at {LIB_PATH}: build it with "
            "`make -C slam-1_amd` (or __graft_entry__.build()). slam355 has no CPU fallback."
        )
    lib = ctypes.CDLL(LIB_PATH)
    for name, argtypes in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.argtypes = argtypes
        fn.restype = _RESTYPE.get(name, c_int)
    return lib


lib = _load()


def check(rc: int, what: str = "") -> None:
    if rc != 0:
        msg = lib.slam_last_error().decode(errors="replace")
        raise SlamError(f"{what or 'libslam355'} failed ({rc}): {msg}")


def call(name: str, *args) -> None:
    check(getattr(lib, name)(*args), name)
