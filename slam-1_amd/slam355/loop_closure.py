"""Drop-in for /root/reference/loop_closure.py.

close_loop (:7-36) re-runs the GPU front end on the loop pair (ORB tiles on
three images, L->R tracking with the F-LMedS mask, triangulation, 2D-3D
correspondences, PnP) and returns the 4x4 transformation ([] when too few 3-D
points, as the reference).  find_error / get_distribution_error /
distribute_error (:39-52) are the host bookkeeping the reference runs after it
(4x4 arithmetic on the KeyFrame chain; main.py:110-118).
"""
from __future__ import annotations

from .keypoint import track_keypoints_left_to_right_new
from .orb import orb_detector_using_tiles
from .Point3D import find_2D_and_3D_correspondenses, sort_3D_points, triangulate_points_local
from .transformation import calculate_transformation_matrix


def close_loop(left_image_0, right_image_0, left_image_i, P_left, P_right, K_left):
    kpL0, desL0 = orb_detector_using_tiles(left_image_0, max_number_of_kp=200)
    kpR0, desR0 = orb_detector_using_tiles(right_image_0, max_number_of_kp=200)
    kpLi, desLi = orb_detector_using_tiles(left_image_i, max_number_of_kp=200)
    ptsL0, ptsR0, dL0, _ = track_keypoints_left_to_right_new(kpL0, desL0, kpR0, desR0,
                                                             left_image_0, right_image_0)
    Q0 = triangulate_points_local(ptsL0, ptsR0, P_left, P_right)
    q_i, Q_0, _ = find_2D_and_3D_correspondenses(dL0, ptsL0, kpLi, desLi, Q0, max_Distance=500)
    close_idx, far_idx = sort_3D_points(Q_0, close_def_in_m=70)
    transformation_matrix = []
    if len(Q_0) > 4:
        transformation_matrix, _, _ = calculate_transformation_matrix(Q_0, q_i, close_idx, far_idx,
                                                                      K_left)
    return transformation_matrix


def find_error(correct_frame, wrong_frame):
    """(:39-40)"""
    return correct_frame - wrong_frame


def get_distribution_error(error_frame, index_0, index_i):
    """(:43-44)"""
    return error_frame / (index_i - index_0)


def distribute_error(camera_frames, error_frame, index_0, index_i):
    """(:48-52) translation only, in place on objects with a `.pose` (KeyFrame)."""
    for i in range(index_0, index_i):
        camera_frames[i].pose[:3, 3] += (i - index_0) * error_frame[:3, 3]
    return camera_frames
