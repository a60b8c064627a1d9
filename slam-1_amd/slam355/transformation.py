"""Drop-in for /root/reference/transformation.py (PnP on the GPU)."""
from __future__ import annotations

import math

import numpy as np
import torch

from . import geometry
from .device import require_gpu, to_dev


def rodrigues(rotvec):
    """cv2.Rodrigues(rotation vector) -> 3x3."""
    r = np.asarray(rotvec, float).ravel()
    th = float(np.linalg.norm(r))
    if th < np.finfo(float).eps:
        return np.eye(3)
    k = r / th
    K = np.array([[0, -k[2], k[1]], [k[2], 0, -k[0]], [-k[1], k[0], 0]])
    return math.cos(th) * np.eye(3) + (1 - math.cos(th)) * np.outer(k, k) + math.sin(th) * K


def form_transf(R, t):
    """(transformation.py:33-37)"""
    T = np.eye(4, dtype=float)
    T[:3, :3] = R
    T[:3, 3] = t
    return T


def translation_and_rotation_vector_to_matrix(rotvec, transvec):
    """(transformation.py:23-31) T = [Rodrigues(rotvec) | transvec^T]."""
    return form_transf(rodrigues(rotvec), np.transpose(np.asarray(transvec, float)))


def calculate_transformation_matrix(trackable_3D_points_time_i,
                                    trackable_left_imagecoordinates_time_i1,
                                    close_3D_points_index, far_3D_points_index, K_left,
                                    seed=0, frame=0):
    """(transformation.py:5-19) GPU RANSAC+LM PnP; keeps the reference's sign flip
    (rvec <- -rvec, tvec <- -tvec, T = [R(-rvec) | -tvec]).  `close`/`far` are
    accepted and unused, as in the reference."""
    q = np.ascontiguousarray(trackable_left_imagecoordinates_time_i1, np.float64).reshape(-1, 2)
    Q = np.ascontiguousarray(trackable_3D_points_time_i, np.float64).reshape(-1, 3)
    dev = require_gpu()
    L = len(Q)
    rv, tv, n, mask = geometry.pnp_ransac(
        to_dev((Q if L else np.zeros((1, 3)))[None]), to_dev((q if L else np.zeros((1, 2)))[None]),
        torch.tensor([L], dtype=torch.int32, device=dev), K_left, seed=seed, item0=frame)
    rotation_vector = -1 * rv[0].cpu().numpy().reshape(3, 1)
    translation_vector = -1 * tv[0].cpu().numpy().reshape(3, 1)
    T = translation_and_rotation_vector_to_matrix(rotation_vector, translation_vector)
    return T, rotation_vector, translation_vector


def eulerAnglesToRotationMatrix(theta):
    """(transformation.py:40-56)"""
    R_x = np.array([[1, 0, 0], [0, math.cos(theta[0]), -math.sin(theta[0])],
                    [0, math.sin(theta[0]), math.cos(theta[0])]])
    R_y = np.array([[math.cos(theta[1]), 0, math.sin(theta[1])], [0, 1, 0],
                    [-math.sin(theta[1]), 0, math.cos(theta[1])]])
    R_z = np.array([[math.cos(theta[2]), -math.sin(theta[2]), 0],
                    [math.sin(theta[2]), math.cos(theta[2]), 0], [0, 0, 1]])
    return np.dot(R_z, np.dot(R_y, R_x))
