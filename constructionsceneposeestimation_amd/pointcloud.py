"""Depth -> coloured point cloud (host side).

Restates ``depth_to_pointcloud_with_rgb`` (generate_construction_data.py:616-711),
the reference's fallback when the pointcloud annotator returns nothing
(:1729-1764): pinhole back-projection with fx = W*f/hA, fy = H*f/vA,
cx = W/2, cy = H/2 (:646-649), valid depth = finite, > 0, < 250 (:655), then
``R.from_quat(camera_pose[3:]) @ p + t`` applied directly to OpenCV-style
(X right, Y down, Z forward) camera coordinates — the reference's mirrored
convention is kept as-is so outputs match it.

The depth buffer this consumes is the renderer's ``distance_to_image_plane``
output; moving this unprojection onto the GPU (fused into the resolve) is
the first "next" row of SURVEY §8f.
"""
from __future__ import annotations

from typing import Optional

import numpy as np
from scipy.spatial.transform import Rotation


def depth_to_pointcloud_with_rgb(depth: np.ndarray, rgb: Optional[np.ndarray], camera_params: dict,
                                 camera_pose) -> Optional[np.ndarray]:
    h, w = depth.shape
    f = camera_params.get("focal_length", 18.14)
    ha = camera_params.get("horizontal_aperture", 20.955)
    va = camera_params.get("vertical_aperture", 15.2908)
    W = camera_params.get("width", w)
    H = camera_params.get("height", h)
    fx, fy = (W * f) / ha, (H * f) / va
    cx, cy = W / 2.0, H / 2.0
    u, v = np.meshgrid(np.arange(w), np.arange(h))
    with np.errstate(invalid="ignore"):
        valid = np.isfinite(depth) & (depth > 0) & (depth < 250)
    if not valid.any():
        return None
    z = depth[valid]
    x = (u[valid] - cx) * z / fx
    y = (v[valid] - cy) * z / fy
    pts = np.stack([x, y, z], axis=-1)
    Rm = Rotation.from_quat(np.asarray(camera_pose[3:], dtype=np.float64)).as_matrix()
    world = (Rm @ pts.T).T + np.asarray(camera_pose[:3], dtype=np.float64)
    if rgb is not None and rgb.size > 0 and rgb.shape[2] >= 3:
        c = rgb[valid, :3]
        c = (c * 255).astype(np.uint8) if c.max() <= 1.0 else c.astype(np.uint8)
    else:
        c = np.full((world.shape[0], 3), 255, np.uint8)
    return np.hstack([world, c])
