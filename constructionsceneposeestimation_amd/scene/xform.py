"""4x4 transform helpers (float64, column-vector convention ``p' = M @ p``).

USD stores matrices row-vector style (translation in row 3) and composes
``xformOpOrder = [A, B, C]`` so that C is applied to a point first; in
column convention that is ``M_local = A @ B @ C`` and
``M_world = M_parent @ M_local`` — the composition ``pxr`` performs for
``ComputeLocalToWorldTransform`` (generate_construction_data.py:597, 1992).
"""
from __future__ import annotations

import math
from typing import Sequence

import numpy as np


def translate(t: Sequence[float]) -> np.ndarray:
    m = np.eye(4)
    m[:3, 3] = np.asarray(t, dtype=np.float64)
    return m


def scale(s: Sequence[float]) -> np.ndarray:
    m = np.eye(4)
    m[0, 0], m[1, 1], m[2, 2] = (float(x) for x in s)
    return m


def quat_wxyz_to_mat3(w: float, x: float, y: float, z: float) -> np.ndarray:
    n = w * w + x * x + y * y + z * z
    s = 2.0 / n if n > 0 else 0.0
    return np.array([
        [1 - s * (y * y + z * z), s * (x * y - w * z), s * (x * z + w * y)],
        [s * (x * y + w * z), 1 - s * (x * x + z * z), s * (y * z - w * x)],
        [s * (x * z - w * y), s * (y * z + w * x), 1 - s * (x * x + y * y)],
    ])


def rotate_quat(q_imag_first: Sequence[float]) -> np.ndarray:
    """Crate stores GfQuat as (i, j, k, real)."""
    x, y, z, w = (float(v) for v in q_imag_first)
    m = np.eye(4)
    m[:3, :3] = quat_wxyz_to_mat3(w, x, y, z)
    return m


def rot_x(deg: float) -> np.ndarray:
    c, s = math.cos(math.radians(deg)), math.sin(math.radians(deg))
    m = np.eye(4)
    m[1, 1], m[1, 2], m[2, 1], m[2, 2] = c, -s, s, c
    return m


def rot_y(deg: float) -> np.ndarray:
    c, s = math.cos(math.radians(deg)), math.sin(math.radians(deg))
    m = np.eye(4)
    m[0, 0], m[0, 2], m[2, 0], m[2, 2] = c, s, -s, c
    return m


def rot_z(deg: float) -> np.ndarray:
    c, s = math.cos(math.radians(deg)), math.sin(math.radians(deg))
    m = np.eye(4)
    m[0, 0], m[0, 1], m[1, 0], m[1, 1] = c, -s, s, c
    return m


def rotate_xyz(deg: Sequence[float]) -> np.ndarray:
    """USD rotateXYZ: X applied first, then Y, then Z."""
    rx, ry, rz = (float(v) for v in deg)
    return rot_z(rz) @ rot_y(ry) @ rot_x(rx)


def from_usd_matrix(m_rowvec: np.ndarray) -> np.ndarray:
    return np.asarray(m_rowvec, dtype=np.float64).reshape(4, 4).T.copy()


def transform_points(m: np.ndarray, p: np.ndarray) -> np.ndarray:
    p = np.asarray(p, dtype=np.float64)
    return p @ m[:3, :3].T + m[:3, 3]
