"""Map association (appendKeyPoints, keypoint.py:101-122) and the BA-problem
export (XXXport_files.py:16-92): oracle + host mirror pinned to goldens made by
running the reference itself (tests/golden/make_goldens.py), GPU parity.

Association bar: bit-exact rows and map (indices, copied coordinates).  The
nearest-neighbour tie rule (lowest index) is unpinned against KDTree, which
leaves exact ties unspecified; the goldens contain none.
"""
import os
import tempfile

import numpy as np
import pytest

from oracle import mapping as om

N_FRAMES = 6


@pytest.fixture(scope="module")
def g(golden_dir):
    return np.load(os.path.join(golden_dir, "mapping_golden.npz"))


def _frame(g, i):
    return (g[f"f{i}_Qs_in"], g[f"f{i}_abs"], g[f"f{i}_pts2d"], g[f"f{i}_rel"])


# ----------------------------------------------------------------------------- CPU
def test_oracle_matches_reference_sequence(g):
    n_old = n_new = 0
    for i in range(N_FRAMES):
        Qs, absP, p2, rel = _frame(g, i)
        Qo, rows = om.append_keypoints(Qs, absP, 0.01, p2, i, rel)
        assert np.array_equal(Qo, g[f"f{i}_Qs_out"]) and np.array_equal(rows, g[f"f{i}_rows"]), i
        n_new += len(Qo) - len(Qs)
        n_old += len(rows) - (len(Qo) - len(Qs))
    assert n_old > 50 and n_new > 50  # both branches exercised


def test_export_mirror_bytes_match_reference(g):
    from slam355 import XXXport_files as xp

    class KF:
        def __init__(self, pose):
            self.pose = pose

    frames = [KF(p) for p in g["frame_poses"]]
    opt = np.vstack([g[f"f{i}_rows"] for i in range(N_FRAMES)])
    Qs = g[f"f{N_FRAMES - 1}_Qs_out"]
    P = g["P_left"]
    assert np.array_equal(xp.make_cam_params(frames, P), g["cam_params"])
    assert np.array_equal(xp.make_Qs_for_BA(Qs), g["Qs_for_BA"])
    with tempfile.TemporaryDirectory() as d:
        xp.export_data(opt, frames, Qs, P, cache_dir=d)
        ba = open(os.path.join(d, "BA_file.txt"), "rb").read()
        cf = open(os.path.join(d, "cam_frames.txt"), "rb").read()
    assert ba == g["ba_file"].tobytes()
    assert cf == g["cam_frames_file"].tobytes()


def test_problem_from_map_equals_file_round_trip(g):
    from slam355 import BundleAdjustment as BA
    from slam355 import XXXport_files as xp

    frames = list(g["frame_poses"])
    opt = np.vstack([g[f"f{i}_rows"] for i in range(N_FRAMES)])
    Qs = g[f"f{N_FRAMES - 1}_Qs_out"]
    with tempfile.TemporaryDirectory() as d:
        xp.export_data(opt, frames, Qs, g["P_left"], cache_dir=d)
        ref = BA.read_bal_data(os.path.join(d, "BA_file.txt"))
    got = xp.problem_from_map(opt, frames, Qs, g["P_left"])
    for a, b in zip(got, ref):
        assert np.array_equal(np.asarray(a), np.asarray(b))
    with pytest.raises(ValueError):
        xp.problem_from_map(opt, frames[:-1], Qs, g["P_left"])


# ----------------------------------------------------------------------------- GPU
@pytest.mark.gpu
def test_gpu_map_store_sequence_matches_reference(g):
    import torch
    from slam355.mapping import MapStore

    dev = torch.device("cuda")
    store = MapStore(capacity=64, max_queries=8)  # forces growth and workspace re-sizing
    for i in range(N_FRAMES):
        _, absP, p2, rel = _frame(g, i)
        t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)  # noqa: E731
        rows = store.append(t(absP), t(rel), t(p2), i, threshold=0.01)
        assert np.array_equal(rows.cpu().numpy(), g[f"f{i}_rows"]), i
    assert np.array_equal(store.points().cpu().numpy(), g[f"f{N_FRAMES - 1}_Qs_out"])


@pytest.mark.gpu
def test_gpu_append_keypoints_mirror(g):
    from slam355.keypoint import appendKeyPoints

    for i in range(N_FRAMES):
        Qs, absP, p2, rel = _frame(g, i)
        Qo, rows = appendKeyPoints(Qs, absP, 0.01, p2, i, rel)
        assert np.array_equal(Qo, g[f"f{i}_Qs_out"]) and np.array_equal(rows, g[f"f{i}_rows"]), i
    Qo, rows = appendKeyPoints(g["f1_Qs_in"], np.zeros((0, 3)), 0.01, np.zeros((0, 2)), 9,
                               np.zeros((0, 3)))
    assert np.array_equal(Qo, g["f1_Qs_in"]) and rows.shape == (0, 4)


@pytest.mark.gpu
def test_gpu_large_map_and_device_count_vs_oracle():
    import torch
    from slam355.mapping import MapStore

    rng = np.random.default_rng(4)
    M, N, n_valid = 70_000, 3000, 2345  # several NN chunks, several association tiles
    Qs = rng.uniform(-50, 50, (M, 3))
    rel = rng.uniform(-20, 20, (N, 3)) + [0, 0, 30]
    absP = Qs[rng.integers(0, M, N)] + rng.normal(0, 1, (N, 1)) * rng.choice([0.01, 1.0], (N, 1))
    p2 = rng.uniform(0, 1000, (N, 2))
    dev = torch.device("cuda")
    store = MapStore(capacity=M + N, max_queries=N, Qs=Qs)
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)  # noqa: E731
    cnt = torch.tensor([n_valid], dtype=torch.int32, device=dev)
    rows = store.append(t(absP), t(rel), t(p2), 17, threshold=0.01, count=cnt)
    Qo, erows = om.append_keypoints(Qs, absP[:n_valid], 0.01, p2[:n_valid], 17, rel[:n_valid])
    assert np.array_equal(rows[:n_valid].cpu().numpy(), erows)
    assert store.size() == len(Qo)
    assert np.array_equal(store.points().cpu().numpy(), Qo)
