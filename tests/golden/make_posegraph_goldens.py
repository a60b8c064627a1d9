"""Golden fixtures for the pose-chain optimisation and loop-closure helpers
(SURVEY.md §8f row 2), produced by the REFERENCE code in the build container
(/root/reference does not exist on the GPU box).

    python tests/golden/make_posegraph_goldens.py

What is pinned, and how:
  * BundleAdjustment.py's live pose-chain block (:79-183): `objective`,
    `objective_without_loop_closure`, `bundle_adjustment_sparsity(_without_
    loop_closure)` and `bundle_adjustment_with_sparsity` (scipy TRF, ftol 0.1,
    x_scale 'jac').  The module is imported with a stub `cv2` whose
    `Rodrigues(src, dst)` fills dst in place with OpenCV's published formula
    (cvRodrigues2: theta < DBL_EPSILON -> I, else c I + (1-c) k k^T + s [k]x);
    the module reads ourCache/equal_frames.txt at import (:12-14), so it is
    imported from a scratch directory holding that file.  The "without loop
    closure" driver (:173-177) passes `objective` (m + 2 residuals) with the
    m-row sparsity: scipy raises ValueError, recorded as such.
  * loop_closure.py:39-52: find_error, get_distribution_error and
    distribute_error on a KeyFrame chain.
Only data (inputs + outputs) is written; no reference source is copied.
"""
from __future__ import annotations

import contextlib
import io
import os
import sys
import tempfile

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import make_goldens as mg  # noqa: E402  (stub cv2, reference path)

OUT = os.path.dirname(os.path.abspath(__file__))


def _rodrigues_cv(src, dst=None):
    r = np.asarray(src, np.float64).reshape(3)
    th = float(np.sqrt(r @ r))
    if th < np.finfo(np.float64).eps:
        R = np.eye(3)
    else:
        c, s = np.cos(th), np.sin(th)
        k = r * (1.0 / th)
        rrt = np.outer(k, k)
        rx = np.array([[0, -k[2], k[1]], [k[2], 0, -k[0]], [-k[1], k[0], 0]])
        R = c * np.eye(3) + (1 - c) * rrt + s * rx
    if dst is not None:
        dst[...] = R
        return dst, None
    return R, None


def import_pose_modules():
    cv2 = mg._stub_cv2()
    cv2.Rodrigues = _rodrigues_cv
    sys.modules["cv2"] = cv2
    if not hasattr(np, "float"):
        np.float = float
    if mg.REF not in sys.path:
        sys.path.insert(0, mg.REF)
    tmp = tempfile.mkdtemp()
    os.makedirs(os.path.join(tmp, "ourCache"))
    with open(os.path.join(tmp, "ourCache", "equal_frames.txt"), "w") as f:
        f.write("0 20\n")
    cwd = os.getcwd()
    os.chdir(tmp)
    try:
        import BundleAdjustment  # noqa: E402
        import keyframe  # noqa: E402
        import loop_closure  # noqa: E402
    finally:
        os.chdir(cwd)
    return BundleAdjustment, keyframe, loop_closure


def chain_params(rng, m, rot_s=0.01, t_s=0.05):
    """m relative poses [rx ry rz tx ty tz] of a forward-moving camera."""
    p = np.zeros((m, 6))
    p[:, :3] = rng.normal(0, rot_s, (m, 3))
    p[:, 3:6] = rng.normal(0, t_s, (m, 3))
    p[:, 5] += 1.0
    return p.ravel()


def main():
    BA, keyframe, lc = import_pose_modules()
    rng = np.random.default_rng(31)
    out = {}
    # objective / sparsity on a few chains (incl. a zero rotation, a closing loop)
    for name, m in (("a", 7), ("b", 40), ("c", 250)):
        x = chain_params(rng, m)
        if name == "a":
            x[0:3] = 0.0
            x[6 * 3 + 5] = -1.0
        out[f"obj_{name}_x"] = x
        out[f"obj_{name}_r"] = BA.objective(x)
        out[f"obj_{name}_rnl"] = BA.objective_without_loop_closure(x)
    x = out["obj_a_x"]
    out["sp_loop"] = BA.bundle_adjustment_sparsity(x).toarray()
    out["sp_noloop"] = BA.bundle_adjustment_sparsity_without_loop_closure(x).toarray()
    # the reference's solver (scipy TRF, ftol 0.1, x_scale 'jac') on a 20-frame chain
    x = chain_params(rng, 20, rot_s=0.02, t_s=0.1)
    A = BA.bundle_adjustment_sparsity(x)
    with contextlib.redirect_stdout(io.StringIO()):
        r0, rf, xf = BA.bundle_adjustment_with_sparsity(x, A)
    out.update(sol_x0=x, sol_r0=r0, sol_rf=rf, sol_xf=xf)
    try:
        with contextlib.redirect_stdout(io.StringIO()):
            BA.bundle_adjustment_with_sparsity_without_loop_closure(
                x, BA.bundle_adjustment_sparsity_without_loop_closure(x))
        out["noloop_raises"] = np.array(0)
    except ValueError:
        out["noloop_raises"] = np.array(1)
    # loop_closure.py:39-52 on a KeyFrame chain
    poses = []
    T = np.eye(4)
    for i in range(12):
        R = _rodrigues_cv(rng.normal(0, 0.02, 3))[0]
        Ti = np.eye(4)
        Ti[:3, :3] = R
        Ti[:3, 3] = rng.normal(0, 0.05, 3) + [0, 0, 1]
        T = T @ Ti
        poses.append(T.copy())
    frames = [keyframe.KeyFrame(p.copy()) for p in poses]
    correct = poses[9] + rng.normal(0, 0.1, (4, 4))
    err = lc.find_error(correct, poses[9])
    derr = lc.get_distribution_error(err, 2, 10)
    frames = lc.distribute_error(frames, derr, 2, 10)
    out.update(lc_poses=np.array(poses), lc_correct=correct, lc_err=err, lc_derr=derr,
               lc_out=np.array([f.pose for f in frames]))
    np.savez_compressed(os.path.join(OUT, "posegraph_golden.npz"), **out)
    print({k: np.shape(v) for k, v in out.items()})


if __name__ == "__main__":
    main()
