"""CPU ORACLE — TEST INFRASTRUCTURE ONLY.

numpy restatements of the reference's pure host helpers, pinned against the
golden vectors in tests/golden/ (generated from the reference's own
functions by tests/golden/make_golden.py).  Each cites the reference
function it follows (generate_construction_data.py).  The product package
never imports this module.
"""
from __future__ import annotations

import numpy as np
from scipy.spatial.transform import Rotation


def rot_to_quat_wxyz(R):
    """rotMtx2quaternion :475-504 (trace / largest-diagonal branches)."""
    t = R[0, 0] + R[1, 1] + R[2, 2]
    if t > 0:
        S = np.sqrt(t + 1.0) * 2
        return np.array([0.25 * S, (R[2, 1] - R[1, 2]) / S, (R[0, 2] - R[2, 0]) / S, (R[1, 0] - R[0, 1]) / S])
    if R[0, 0] > R[1, 1] and R[0, 0] > R[2, 2]:
        S = np.sqrt(1.0 + R[0, 0] - R[1, 1] - R[2, 2]) * 2
        return np.array([(R[2, 1] - R[1, 2]) / S, 0.25 * S, (R[0, 1] + R[1, 0]) / S, (R[0, 2] + R[2, 0]) / S])
    if R[1, 1] > R[2, 2]:
        S = np.sqrt(1.0 + R[1, 1] - R[0, 0] - R[2, 2]) * 2
        return np.array([(R[0, 2] - R[2, 0]) / S, (R[0, 1] + R[1, 0]) / S, 0.25 * S, (R[1, 2] + R[2, 1]) / S])
    S = np.sqrt(1.0 + R[2, 2] - R[0, 0] - R[1, 1]) * 2
    return np.array([(R[1, 0] - R[0, 1]) / S, (R[0, 2] + R[2, 0]) / S, (R[1, 2] + R[2, 1]) / S, 0.25 * S])


def cam_pos_ori(cam, aim):
    """camPosOri :507-550: columns [-fwd, -right, up] (improper), then the quaternion."""
    f = np.asarray(aim, float) - np.asarray(cam, float)
    f /= np.linalg.norm(f)
    r = np.cross(f, [0.0, 0.0, 1.0])
    n = np.linalg.norm(r)
    r = np.array([1.0, 0.0, 0.0]) if n < 1e-6 else r / n
    u = np.cross(r, f)
    u /= np.linalg.norm(u)
    return rot_to_quat_wxyz(np.stack([-f, -r, u], axis=1))


def bbox_to_pose(lo, hi, T_rowmajor16):
    """bboxDict_to_transform :553-584."""
    T = np.asarray(T_rowmajor16, float).reshape(4, 4).T
    corners = np.stack([lo, hi]).astype(float)
    center = (T @ np.r_[corners.mean(0), 1.0])[:3]
    M = T[:3, :3]
    U, _, Vt = np.linalg.svd(M)
    euler = Rotation.from_matrix(U @ Vt).as_euler("xyz", degrees=True)
    size = np.linalg.norm(M, axis=0) * np.abs(corners[1] - corners[0])
    return center, size, euler


def unproject(depth, rgb, params, pose):
    """depth_to_pointcloud_with_rgb :616-711 (valid mask, pinhole, R.from_quat)."""
    h, w = depth.shape
    fx = params["width"] * params["focal_length"] / params["horizontal_aperture"]
    fy = params["height"] * params["focal_length"] / params["vertical_aperture"]
    cx, cy = params["width"] / 2.0, params["height"] / 2.0
    vv, uu = np.mgrid[0:h, 0:w]
    with np.errstate(invalid="ignore"):
        m = np.isfinite(depth) & (depth > 0) & (depth < 250)
    z = depth[m].astype(np.float64)
    p = np.stack([(uu[m] - cx) * z / fx, (vv[m] - cy) * z / fy, z], 1)
    Rm = Rotation.from_quat(np.asarray(pose[3:], float)).as_matrix()
    xyz = p @ Rm.T + np.asarray(pose[:3], float)
    c = rgb[m][:, :3]
    c = (c * 255).astype(np.uint8) if c.max() <= 1.0 else c.astype(np.uint8)
    return np.hstack([xyz, c])


# key positions / ring constants of get_systematic_camera_positions :790-868
HEIGHTS = [1.6, 1.7, 1.8, 2.0, 2.5, 3.0]


def ring_position(j: int, z: float):
    radius = [4, 6, 8, 10, 12][j // 8]
    a = 2 * np.pi * (j % 8) / 8
    return np.array([radius * np.cos(a), radius * np.sin(a), z])
