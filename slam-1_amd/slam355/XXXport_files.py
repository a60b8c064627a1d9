"""Mirror of /root/reference/XXXport_files.py: the BA-problem export that turns
the tracked map into the BAL file `BundleAdjustment.read_bal_data` reads
(`ourCache/BA_file.txt`, :44-64), plus `problem_from_map`, which returns the
arrays that file round-trips to without touching the disk (Python's float repr
round-trips exactly), ready for `slam355.ba.BAProblem`.

Host-side file formatting and a per-camera rotation-matrix -> rotation-vector
conversion (scipy's Rotation, the reference's own dependency); the data-parallel
parts of map building run on the GPU (slam355.mapping).
"""
from __future__ import annotations

import os

import numpy as np
from scipy.spatial.transform import Rotation

# pixel offsets export_data subtracts from the observations (:50)
U_OFF = 1226 / 2
V_OFF = 370 / 2


def clear_textfile(file_path):
    """(:5-7)"""
    open(file_path, "w").close()


def save3DPoints(file_name, points, frame):
    """(:10-14) append 'x, y, z,frame' lines."""
    with open(file_name, "a") as f:
        f.writelines(f"{x}, {y}, {z},{frame}\n" for x, y, z in points)


def _pose(frame):
    return frame.pose if hasattr(frame, "pose") else np.asarray(frame)


def make_cam_params(camera_frames, P_left):
    """(:16-32) [rotvec(pose R), pose t, f = P_left[0][0], 0, 0] per frame, flat."""
    out = np.empty((len(camera_frames), 9))
    if len(camera_frames):
        Ts = np.stack([_pose(fr) for fr in camera_frames])
        # one stacked conversion: per matrix the same operations as one call each
        out[:, 0:3] = Rotation.from_matrix(Ts[:, :3, :3]).as_rotvec()
        out[:, 3:6] = Ts[:, :3, 3]
        out[:, 6:9] = (P_left[0][0], 0, 0)
    return out.ravel()


def make_Qs_for_BA(Qs):
    """(:34-41) flattened x, y, z."""
    return np.asarray(Qs, float).reshape(-1, 3).ravel().copy()


def _ba_text(optimization_matrix, camera_frames, Qs, P_left):
    om = np.asarray(optimization_matrix)
    lines = [f"{int(np.max(om[:, 0]) + 1)} {int(np.max(om[:, 1]) + 1)} {int(np.shape(om)[0])}\n"]
    lines += [f"{int(o[0])} {int(o[1])} {str(o[2] - U_OFF)} {str(o[3] - V_OFF)}\n" for o in om]
    for fr in camera_frames[:-1]:  # the last frame's camera is not written (:55)
        T = _pose(fr)
        r = Rotation.from_matrix(T[:3, :3]).as_rotvec()
        lines += [f"{str(r[0])}\n{str(r[1])}\n{str(r[2])}\n",
                  f"{str(T[0, 3])}\n{str(T[1, 3])}\n{str(T[2, 3])}\n",
                  f"{str(P_left[0][0])}\n0\n0\n"]
    lines += [f"{str(c[0])}\n{str(c[1])}\n{str(c[2])}\n" for c in Qs]
    return "".join(lines)


def export_data(optimization_matrix, camera_frames, Qs, P_left, cache_dir="ourCache"):
    """(:44-72) writes <cache_dir>/BA_file.txt and <cache_dir>/cam_frames.txt
    byte for byte as the reference does."""
    with open(os.path.join(cache_dir, "BA_file.txt"), "w") as f:
        f.write(_ba_text(optimization_matrix, camera_frames, Qs, P_left))
    with open(os.path.join(cache_dir, "cam_frames.txt"), "w") as f:
        for fr in camera_frames:
            T = _pose(fr)
            f.write("".join(f"{str(T[k, j])} " for k in range(3) for j in range(4)) + "\n")


def problem_from_map(optimization_matrix, camera_frames, Qs, P_left):
    """The (cam_params [C,9], Qs [P,3], cam_idxs, Q_idxs, qs [O,2]) that
    read_bal_data returns for export_data's file, without the file."""
    om = np.asarray(optimization_matrix, float)
    n_cams = int(np.max(om[:, 0]) + 1)
    n_qs = int(np.max(om[:, 1]) + 1)
    frames = list(camera_frames)
    pts = np.asarray(Qs, float).reshape(-1, 3)
    if len(frames) - 1 != n_cams or len(pts) < n_qs:
        # the file export_data would write is not readable back consistently
        raise ValueError(f"export needs {n_cams} cameras (+1 trailing frame) and {n_qs} points; "
                         f"got {len(frames)} frames and {len(pts)} points")
    cams = make_cam_params(frames[:-1], P_left).reshape(-1, 9)
    qs = np.stack([om[:, 2] - U_OFF, om[:, 3] - V_OFF], 1)
    return cams, pts[:n_qs].copy(), om[:, 0].astype(int), om[:, 1].astype(int), qs


def export_relative_transformations_matrix(rvec, tvec, index, cache_dir="ourCache"):
    """(:74-92) one 'r0 r1 r2 t0 t1 t2' line per frame (file truncated at index 0)."""
    path = os.path.join(cache_dir, "cam_frames_relative.txt")
    if index == 0:
        open(path, "w").close()
    r = np.array(rvec).ravel()
    t = np.array(tvec).ravel()
    with open(path, "a") as f:
        f.write("".join(f"{str(v)} " for v in r) + f"{str(t[0])} {str(t[1])} {str(t[2])}\n")
