"""Device-memory plumbing: torch tensors as HBM containers, HIP stream handles."""
from __future__ import annotations

import ctypes

import numpy as np
import torch


def require_gpu() -> torch.device:
    """The HIP path is the only path: refuse to run without a GPU."""
    if not torch.cuda.is_available():
        raise RuntimeError(
            "slam355 runs only on an MI355X/ROCm GPU (hand-written HIP kernels); "
            "no GPU is visible and there is no CPU fallback"
        )
    return torch.device("cuda", torch.cuda.current_device())


def ptr(t: torch.Tensor | None) -> ctypes.c_void_p | None:
    if t is None:
        return None
    if not t.is_cuda:
        raise ValueError("expected a device tensor")
    if not t.is_contiguous():
        raise ValueError("expected a contiguous tensor")
    return ctypes.c_void_p(t.data_ptr())


def stream_ptr(stream: torch.cuda.Stream | None = None) -> ctypes.c_void_p:
    s = stream if stream is not None else torch.cuda.current_stream()
    return ctypes.c_void_p(s.cuda_stream)


def to_dev(a, dtype: torch.dtype | None = None) -> torch.Tensor:
    """numpy / torch -> contiguous device tensor (no copy if already there)."""
    dev = require_gpu()
    if isinstance(a, torch.Tensor):
        t = a
    else:
        t = torch.from_numpy(np.ascontiguousarray(a))
    if dtype is not None and t.dtype != dtype:
        t = t.to(dtype)
    return t.to(dev, non_blocking=True).contiguous()
