"""Drop-in for /root/reference/orb.py on the GPU (HIP kernel k_orb_tile).

orb_detector_using_tiles(image, max_number_of_kp=40, overlap_div=2, height_div=5,
width_div=10) -> (list[KeyPoint], ndarray[N, 32] uint8)   (orb.py:4-25)
orb_extraction_detect(img, max_features) -> (list[KeyPoint], ndarray | None) (orb.py:28-38)

plus the batched device API `orb_batch` used by the pipeline: a batch of
images resident in HBM -> keypoint / descriptor tensors in HBM, no host copy.
"""
from __future__ import annotations

import ctypes

import numpy as np
import torch

from . import _lib
from .device import ptr, require_gpu, stream_ptr, to_dev


class KeyPoint:
    """Stand-in for cv2.KeyPoint: the reference reads only `.pt`
    (keypoint.py:53-54, Point3D.py:52, orb.py:8-9); size/angle/response/octave
    carry the ORB values."""

    __slots__ = ("pt", "size", "angle", "response", "octave")

    def __init__(self, x, y, size=31.0, angle=-1.0, response=0.0, octave=0):
        self.pt = (float(x), float(y))
        self.size, self.angle, self.response, self.octave = float(size), float(angle), \
            float(response), int(octave)

    def __repr__(self):
        return f"KeyPoint(pt={self.pt}, octave={self.octave}, response={self.response:.3g})"


class OrbWorkspace:
    """Per-shape scratch for slam_orb_tiles (allocated once, reused per batch)."""

    def __init__(self, batch, H, W, max_kp, overlap_div=2, height_div=5, width_div=10,
                 kp_cap=None):
        dev = require_gpu()
        nb = ctypes.c_size_t(0)
        _lib.call("slam_orb_workspace_bytes", batch, H, W, max_kp, overlap_div, height_div,
                  width_div, ctypes.byref(nb))
        self.args = (batch, H, W, max_kp, overlap_div, height_div, width_div)
        self.ws = torch.empty(int(nb.value), dtype=torch.uint8, device=dev)
        if kp_cap is None:
            kp_cap = max(64, 64 * ((max_kp * 64 + 63) // 64))  # generous: tiles x cap + ties
        self.kp_cap = int(kp_cap)
        self.kp = torch.empty((batch, self.kp_cap, 5), dtype=torch.float32, device=dev)
        self.octave = torch.empty((batch, self.kp_cap), dtype=torch.int32, device=dev)
        self.desc = torch.empty((batch, self.kp_cap, 32), dtype=torch.uint8, device=dev)
        self.count = torch.empty((batch,), dtype=torch.int32, device=dev)

    def run(self, imgs: torch.Tensor, stream=None):
        B, H, W = imgs.shape
        b, h, w, max_kp, od, hd, wd = self.args
        if (B, H, W) != (b, h, w) or imgs.dtype != torch.uint8:
            raise ValueError(f"expected uint8 images of shape {(b, h, w)}, got {tuple(imgs.shape)}")
        _lib.call("slam_orb_tiles", ptr(imgs), B, H, W, imgs.stride(1), max_kp, od, hd, wd,
                  ptr(self.ws), self.ws.numel(), ptr(self.kp), ptr(self.octave), ptr(self.desc),
                  ptr(self.count), self.kp_cap, stream_ptr(stream))
        return self.kp, self.octave, self.desc, self.count


_WS_CACHE: dict = {}


def orb_batch(imgs: torch.Tensor, max_number_of_kp: int, overlap_div=2, height_div=5,
              width_div=10, kp_cap=None, stream=None):
    """Batched device ORB: imgs [B,H,W] u8 on the GPU -> (kp [B,cap,5] f32, octave, desc, count)."""
    B, H, W = imgs.shape
    key = (B, H, W, max_number_of_kp, overlap_div, height_div, width_div, kp_cap,
           imgs.device.index)
    ws = _WS_CACHE.get(key)
    if ws is None:
        ws = _WS_CACHE[key] = OrbWorkspace(B, H, W, max_number_of_kp, overlap_div, height_div,
                                           width_div, kp_cap)
    return ws.run(imgs.contiguous(), stream)


def _to_host(kp, octave, desc, count, b=0):
    n = int(count[b].item())
    if n < 0:
        raise _lib.SlamError("slam_orb_tiles: keypoint capacity exceeded")
    k = kp[b, :n].cpu().numpy()
    o = octave[b, :n].cpu().numpy()
    d = desc[b, :n].cpu().numpy()
    kps = [KeyPoint(k[i, 0], k[i, 1], k[i, 2], k[i, 3], k[i, 4], o[i]) for i in range(n)]
    return kps, d, k, o


def orb_detector_using_tiles(image, max_number_of_kp=40, overlap_div=2, height_div=5,
                             width_div=10):
    """(orb.py:4-25) -> (list[KeyPoint], (N, 32) uint8 descriptors)."""
    img = to_dev(np.ascontiguousarray(image, np.uint8)[None] if not isinstance(image, torch.Tensor)
                 else image.reshape(1, *image.shape[-2:]))
    out = orb_batch(img, max_number_of_kp, overlap_div, height_div, width_div)
    kps, d, _, _ = _to_host(*out)
    return kps, d.reshape(-1, 32)


def orb_extraction_detect(img, max_features):
    """(orb.py:28-38) ORB on the whole image as one patch -> (kps, desc or None)."""
    im = to_dev(np.ascontiguousarray(img, np.uint8)[None])
    out = orb_batch(im, max_features, 1, 0, 0)
    kps, d, _, _ = _to_host(*out)
    return kps, (d if len(kps) else None)
