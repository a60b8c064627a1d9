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
# SLAM355_LIB: an instrumented build of the same library (profiling scripts only)
LIB_PATH = os.environ.get("SLAM355_LIB") or os.path.join(_HERE, "libslam355.so")

c_int = ctypes.c_int
c_double = ctypes.c_double
c_size_t = ctypes.c_size_t
c_p = ctypes.c_void_p
c_uint64 = ctypes.c_uint64
c_longlong = ctypes.c_longlong

c_i32 = ctypes.c_int32


class BAProblemStruct(ctypes.Structure):
    """Mirror of `slam_ba_problem` (include/slam355.h)."""
    _fields_ = [
        ("n_cams", c_i32), ("n_pts", c_i32), ("n_obs", c_i32), ("n_grps", c_i32),
        ("n_blocks", c_i32), ("n_cslots", c_i32), ("n_bslots", c_i32), ("lin_mode", c_i32),
        ("n_sgrps", c_i32), ("tl_mode", c_i32),
        ("cams", c_p * 2), ("pts", c_p * 2), ("camrec", c_p * 2),
        ("obs_cam", c_p), ("obs_pt", c_p), ("obs_q", c_p), ("pt_ptr", c_p), ("grp_ptr", c_p),
        ("grp_cslot", c_p), ("cslot_cam", c_p), ("cslot_obs_ptr", c_p), ("cslot_obs", c_p),
        ("grp_bslot", c_p), ("bslot_blk", c_p), ("bslot_pair_ptr", c_p), ("bslot_pairs", c_p),
        ("blocks", c_p), ("cam_cslot_ptr", c_p), ("cslot_row", c_p), ("blk_bslot_ptr", c_p),
        ("bslot_row", c_p), ("cpart", c_p), ("bpart", c_p),
        ("sys", c_p), ("chol", c_p), ("delta_c", c_p), ("red_part", c_p), ("small", c_p),
        ("state", c_p), ("ticket", c_p),
        ("sg_ptr", c_p), ("sg_meta", c_p), ("obs_meta", c_p), ("chk_optr", c_p), ("chk_cptr", c_p),
        ("bslot_ab", c_p), ("tl_sched", c_p), ("tl_sched_host", c_p), ("asm_tab", c_p),
        ("asm_act", c_p), ("n_asm_act", c_int), ("asm_pad", c_int),
    ]


_PROB = ctypes.POINTER(BAProblemStruct)

PLAN_TABLES = ("perm", "order", "obs_cam", "obs_pt", "pt_ptr", "grp_ptr", "grp_cslot", "cslot_cam",
               "grp_bslot", "bslot_blk", "blocks", "cam_cslot_ptr", "cslot_row", "blk_bslot_ptr",
               "bslot_row", "sg_ptr", "sg_meta", "sg_cams", "obs_la", "chk_cobs", "obs_meta",
               "chk_optr", "chk_cptr", "bslot_ab")  # SLAM_PLAN_* order


class PlanInfo(ctypes.Structure):
    """Mirror of `slam_ba_plan_info` (include/slam355.h)."""
    _fields_ = [
        ("ok", c_i32), ("n_obs", c_i32), ("n_grps", c_i32), ("n_sgrps", c_i32),
        ("n_cslots", c_i32), ("n_bslots", c_i32), ("n_blocks", c_i32), ("chunks_per_wg", c_i32),
        ("off", ctypes.c_longlong * len(PLAN_TABLES)), ("len", ctypes.c_longlong * len(PLAN_TABLES)),
        ("total", ctypes.c_longlong),
    ]

# name -> argtypes (restype is int unless listed in _RESTYPE)
SIGNATURES = {
    "slam_abi_version": [],
    "slam_last_error": [],
    "slam_device_count": [],
    "slam_hamming_knn2": [c_p, c_p, c_int, c_p, c_p, c_int, c_int, c_p, c_p, c_p, c_p],
    "slam_compact_matches": [c_p, c_p, c_p, c_int, c_int, c_p, c_double, c_p, c_p, c_p],
    "slam_orb_workspace_bytes": [c_int, c_int, c_int, c_int, c_int, c_int, c_int,
                                 ctypes.POINTER(c_size_t)],
    "slam_orb_tiles": [c_p, c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_p,
                       c_size_t, c_p, c_p, c_p, c_p, c_int, c_p],
    "slam_gather_matches": [c_p, c_int, c_p, c_int, c_p, c_p, c_p, c_p, c_int, c_int, c_p, c_p,
                            c_p, c_p, c_p],
    "slam_gather_temporal": [c_p, c_p, c_int, c_p, c_int, c_p, c_p, c_int, c_int, c_p, c_p, c_p,
                             c_p],
    "slam_triangulate": [c_p, c_p, c_p, c_int, c_int, c_p, c_p, c_int, c_p, c_p],
    "slam_pnp_ransac": [c_p, c_p, c_p, c_int, c_int, c_p, c_uint64, c_int, c_int, c_double, c_int,
                        c_int, c_p, c_p, c_p, c_p, c_p, c_longlong, c_p],
    "slam_pnp_workspace_len": [c_int, c_int],
    "slam_pose_chain": [c_p, c_p, c_p, c_int, c_p, c_p, c_p],
    "slam_vo_estimate_pose": [c_p, c_p, c_p, c_p, c_p, c_int, c_int, c_p, c_uint64, c_int, c_int,
                              c_int, c_int, c_p, c_p, c_p, c_p, c_p, c_size_t, c_p],
    "slam_vo_pose_workspace_bytes": [c_int, c_int, ctypes.POINTER(c_size_t)],
    "slam_vo_residuals": [c_p, c_p, c_p, c_p, c_p, c_p, c_int, c_int, c_p, c_p, c_p],
    "slam_map_workspace_bytes": [c_int, c_int, ctypes.POINTER(c_size_t)],
    "slam_rel_to_abs": [c_p, c_p, c_int, c_int, c_p, c_p, c_p],
    "slam_map_windows": [c_p, c_p, c_int, c_int, c_int, c_p, c_p, c_p, c_p, c_int, c_double, c_p,
                         c_p, c_size_t, c_p],
    "slam_map_associate": [c_p, c_p, c_int, c_int, c_p, c_p, c_p, c_p, c_int, c_double, c_int,
                           c_p, c_p, c_size_t, c_p],
    "slam_fundamental_lmeds": [c_p, c_p, c_p, c_int, c_int, c_uint64, c_int, c_int, c_p, c_p, c_p,
                               c_p],
    "slam_filter_pairs": [c_p, c_p, c_p, c_int, c_int, c_p, c_p, c_p],
    "slam_ba_residual": [c_p, c_p, c_p, c_p, c_p, c_int, c_p, c_p],
    "slam_ba_jacobian": [c_p, c_p, c_p, c_p, c_p, c_int, c_p, c_p, c_p],
    "slam_ba_red_slots": [c_int],
    "slam_ba_sys_len": [c_int, c_int],
    "slam_ba_chol_len": [c_int, c_p],
    "slam_ba_build_system": [_PROB, c_p],
    "slam_ba_solve_step": [_PROB, c_p],
    "slam_ba_decide": [_PROB, c_p],
    "slam_ba_iterate": [_PROB, c_int, c_p],
    "slam_ba_reset": [_PROB, c_double, c_p],
    "slam_ba_iterate_batch": [_PROB, c_int, c_int, c_p],
    "slam_ba_set_solve_lds_floor": [c_int],
    "slam_orb_set_lds_floor": [c_int],
    "slam_count_min": [c_p, c_int, c_p, c_p],
    "slam_hamming_force_valu": [c_int],
    "slam_ba_reset_batch": [_PROB, c_int, c_double, c_p],
    "slam_pose_chain_objective": [c_p, c_int, c_int, c_int, c_p, c_p],
    "slam_bow_histograms": [c_p, c_p, c_int, c_int, c_int, c_p, c_int, c_p, c_p, c_p],
    "slam_bow_query": [c_p, c_int, c_p, c_p, c_int, c_p, c_p, c_p],
    "slam_bow_lloyd": [c_p, c_int, c_p, c_p, c_int, c_int, c_p, c_p, c_p],
    "slam_pose_chain_workspace_len": [c_int],
    "slam_fast_tiles_workspace_bytes": [c_int, c_int, c_int, c_int, c_int, c_int,
                                        ctypes.POINTER(c_size_t)],
    "slam_fast_tiles": [c_p, c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_p,
                        c_size_t, c_p, c_p, c_int, c_p],
    "slam_lk_pyramid_layout": [c_int, c_int, c_int, c_int, ctypes.POINTER(c_int),
                               ctypes.POINTER(c_size_t)],
    "slam_lk_build_pyramids": [c_p, c_int, c_int, c_int, c_int, c_int, c_int, c_p, c_p, c_p],
    "slam_lk_track": [c_p, c_p, c_p, ctypes.c_longlong, c_int, c_int, c_int, c_int, c_int, c_int,
                      c_double, ctypes.c_float, c_p, c_int, c_p, c_int, c_p, c_p, c_p, c_p],
    "slam_lk_filter": [c_p, c_int, c_p, c_p, c_p, c_p, c_int, c_int, c_int, c_int, ctypes.c_float,
                       c_int, c_p, c_p, c_p, c_p, c_p],
    "slam_sgbm_workspace_bytes": [c_int, c_int, c_int, c_int, c_int, c_int,
                                  ctypes.POINTER(c_size_t)],
    "slam_sgbm": [c_p, c_p, c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_p,
                  c_size_t, c_p, c_p, c_p],
    "slam_vo_right_qs_3d": [c_p, c_p, c_p, c_int, c_int, c_p, ctypes.c_longlong,
                            ctypes.c_longlong, c_int, c_int, ctypes.c_float, ctypes.c_float, c_p,
                            c_p, c_p, c_p, c_p, c_p, c_p, c_p, c_p, c_p, c_p, c_p, c_p, c_p],
    "slam_triangulate_f32": [c_p, c_p, c_p, c_int, c_int, c_p, c_p, c_p, c_p],
    "slam_pose_chain_trf": [c_p, c_int, c_int, c_int, c_int, c_double, c_double, c_double, c_int,
                            c_p, c_p],
    "slam_comm_unique_id": [c_p],
    "slam_comm_init": [c_int, c_int, c_p, ctypes.POINTER(c_p)],
    "slam_comm_destroy": [c_p],
    "slam_comm_allreduce_f64": [c_p, c_p, ctypes.c_longlong, c_p],
    "slam_ba_step_distributed": [_PROB, c_p, c_p],
    "slam_ba_plan_bound": [c_int, c_int, c_int, c_int],
    "slam_ba_plan_mfma": [c_int, c_int, c_int, c_p, c_p, c_p, c_int, c_int, c_p, c_longlong,
                          ctypes.POINTER(PlanInfo)],
    "slam_ba_stage_windows": [c_int, c_int, c_int, c_p, c_p, c_p, c_int, c_p, c_p, c_double,
                              c_double, c_p, c_longlong, c_p, c_longlong, c_p, c_p, c_p, c_p, c_p],
}
_RESTYPE = {"slam_last_error": ctypes.c_char_p, "slam_ba_sys_len": ctypes.c_longlong,
            "slam_ba_plan_bound": ctypes.c_longlong,
            "slam_ba_chol_len": ctypes.c_longlong, "slam_pnp_workspace_len": ctypes.c_longlong, "slam_pose_chain_workspace_len": ctypes.c_longlong}


class SlamError(RuntimeError):
    """A libslam355 call returned a non-zero status."""


def _load():
    if not os.path.exists(LIB_PATH):
        raise ImportError(
            f"libslam355.so not found at {LIB_PATH}: build it with "
            "`make -C slam-1_amd` (or __graft_entry__.build()). slam355 has no CPU fallback."
        )
    # One HIP runtime per process: torch ships its own libamdhip64.so.7 and the
    # dynamic linker binds our DT_NEEDED to whichever copy is loaded first, so
    # load torch's before ours (torch streams/allocations are passed straight in).
    import torch  # noqa: F401

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
