"""Camera pose and projection math (host side, float64).

Reference anchors (generate_construction_data.py):
* ``rotMtx2quaternion`` :475-504 and ``camPosOri`` :507-550 — restated
  faithfully below, including the quirk that R = [-fwd, -right, up] is
  improper (det = -1), which for every level shot returns the non-unit
  (0.7071, 0, 0, 0) regardless of the aim point.
* ``get_obj_pose`` :587-605 — world transform -> [x, y, z, qx, qy, qz, qw].
* intrinsics :646-649 with the camera set at :1436-1443 (clip 0.5/250,
  focal 12 mm, horizontal aperture 25 mm) and vA = hA*H/W (:1736, :2038).

The schedule in this build uses :func:`look_at_world_quat`, a proper
rotation in Isaac Sim's ``camera_axes="world"`` convention (+X forward,
+Z up) — i.e. what ``camPosOri`` intends — and the renderer converts it to
the USD camera convention (-Z forward, +Y up) with :func:`world_to_usd_rot`.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Sequence, Tuple

import numpy as np

NEAR_CLIP = 0.5
FAR_CLIP = 250.0
FOCAL_LENGTH_MM = 12.0
H_APERTURE_MM = 25.0

# Isaac "world" camera axes (fwd +X, left +Y, up +Z) -> USD camera axes
# (right +X, up +Y, back +Z): columns are USD axes expressed in world-axes coords.
_WORLD_TO_USD = np.array([[0.0, 0.0, -1.0],
                          [-1.0, 0.0, 0.0],
                          [0.0, 1.0, 0.0]])


# -- faithful restatements of the reference helpers ---------------------------

def rotMtx2quaternion(R: np.ndarray) -> np.ndarray:
    """Shepperd-style matrix -> (w, x, y, z); generate_construction_data.py:475-504."""
    trace = np.trace(R)
    if trace > 0:
        S = np.sqrt(trace + 1.0) * 2
        return np.array([0.25 * S, (R[2, 1] - R[1, 2]) / S, (R[0, 2] - R[2, 0]) / S, (R[1, 0] - R[0, 1]) / S])
    if R[0, 0] > R[1, 1] and R[0, 0] > R[2, 2]:
        S = np.sqrt(1.0 + R[0, 0] - R[1, 1] - R[2, 2]) * 2
        return np.array([(R[2, 1] - R[1, 2]) / S, 0.25 * S, (R[0, 1] + R[1, 0]) / S, (R[0, 2] + R[2, 0]) / S])
    if R[1, 1] > R[2, 2]:
        S = np.sqrt(1.0 + R[1, 1] - R[0, 0] - R[2, 2]) * 2
        return np.array([(R[0, 2] - R[2, 0]) / S, (R[0, 1] + R[1, 0]) / S, 0.25 * S, (R[1, 2] + R[2, 1]) / S])
    S = np.sqrt(1.0 + R[2, 2] - R[0, 0] - R[1, 1]) * 2
    return np.array([(R[1, 0] - R[0, 1]) / S, (R[0, 2] + R[2, 0]) / S, (R[1, 2] + R[2, 1]) / S, 0.25 * S])


def camPosOri(target_point, aimed_point) -> np.ndarray:
    """Reference look-at (generate_construction_data.py:507-550), quirk included."""
    forward = np.asarray(aimed_point, np.float64) - np.asarray(target_point, np.float64)
    forward = forward / np.linalg.norm(forward)
    right = np.cross(forward, np.array([0.0, 0.0, 1.0]))
    rn = np.linalg.norm(right)
    right = np.array([1.0, 0.0, 0.0]) if rn < 1e-6 else right / rn
    up = np.cross(right, forward)
    up = up / np.linalg.norm(up)
    R = np.array([[-forward[0], -right[0], up[0]],
                  [-forward[1], -right[1], up[1]],
                  [-forward[2], -right[2], up[2]]])
    return rotMtx2quaternion(R)


# -- proper camera math used by this build ------------------------------------

def look_at_world_rot(cam, aim, world_up=(0.0, 0.0, 1.0)) -> np.ndarray:
    """Proper rotation (det +1), Isaac ``world`` axes: columns [fwd, left, up]."""
    f = np.asarray(aim, np.float64) - np.asarray(cam, np.float64)
    f = f / np.linalg.norm(f)
    r = np.cross(f, np.asarray(world_up, np.float64))
    rn = np.linalg.norm(r)
    r = np.array([0.0, -1.0, 0.0]) if rn < 1e-9 else r / rn
    u = np.cross(r, f)
    return np.stack([f, -r, u], axis=1)


def quat_wxyz_from_rot(R: np.ndarray) -> np.ndarray:
    q = rotMtx2quaternion(R)
    return q / np.linalg.norm(q)


def rot_from_quat_wxyz(q: Sequence[float]) -> np.ndarray:
    w, x, y, z = (float(v) for v in q)
    n = w * w + x * x + y * y + z * z
    s = 2.0 / n if n > 0 else 0.0
    return np.array([
        [1 - s * (y * y + z * z), s * (x * y - w * z), s * (x * z + w * y)],
        [s * (x * y + w * z), 1 - s * (x * x + z * z), s * (y * z - w * x)],
        [s * (x * z - w * y), s * (y * z + w * x), 1 - s * (x * x + y * y)],
    ])


def look_at_world_quat(cam, aim) -> np.ndarray:
    """(w, x, y, z) for ``Camera.set_world_pose`` in ``world`` axes."""
    return quat_wxyz_from_rot(look_at_world_rot(cam, aim))


def world_to_usd_rot(R_world: np.ndarray) -> np.ndarray:
    """Camera-to-world rotation in USD camera axes (-Z forward, +Y up)."""
    return R_world @ _WORLD_TO_USD


def camera_usd_transform(position, quat_wxyz_world) -> np.ndarray:
    """4x4 camera prim world transform (USD convention), column-vector form."""
    M = np.eye(4)
    M[:3, :3] = world_to_usd_rot(rot_from_quat_wxyz(quat_wxyz_world))
    M[:3, 3] = np.asarray(position, np.float64)
    return M


def view_matrix(cam_to_world: np.ndarray) -> np.ndarray:
    R = cam_to_world[:3, :3]
    t = cam_to_world[:3, 3]
    V = np.eye(4)
    V[:3, :3] = R.T
    V[:3, 3] = -R.T @ t
    return V


@dataclass(frozen=True)
class Intrinsics:
    width: int
    height: int
    focal_length: float = FOCAL_LENGTH_MM
    horizontal_aperture: float = H_APERTURE_MM
    near: float = NEAR_CLIP
    far: float = FAR_CLIP

    @property
    def vertical_aperture(self) -> float:
        return self.horizontal_aperture * (self.height / self.width)

    @property
    def fx(self) -> float:
        return (self.width * self.focal_length) / self.horizontal_aperture

    @property
    def fy(self) -> float:
        return (self.height * self.focal_length) / self.vertical_aperture

    @property
    def cx(self) -> float:
        return self.width / 2.0

    @property
    def cy(self) -> float:
        return self.height / 2.0

    def params(self) -> dict:
        """``camera_params`` block of the label record (:2039-2045)."""
        return {"horizontal_aperture": self.horizontal_aperture,
                "vertical_aperture": self.vertical_aperture,
                "focal_length": self.focal_length,
                "width": self.width, "height": self.height}

    def pixel_projection(self) -> np.ndarray:
        """4x4 whose rows 0,1,3 map camera coords to (u*w, v*w, w):
        u = cx + fx*Xc/(-Zc), v = cy - fy*Yc/(-Zc) (pixel rows go down),
        w = -Zc = distance to the image plane.  Row 2 is unused."""
        P = np.zeros((4, 4))
        P[0] = [self.fx, 0.0, -self.cx, 0.0]
        P[1] = [0.0, -self.fy, -self.cy, 0.0]
        P[2] = [0.0, 0.0, 0.0, 0.0]
        P[3] = [0.0, 0.0, -1.0, 0.0]
        return P


def get_obj_pose_from_matrix(M: np.ndarray) -> list:
    """[x, y, z, qx, qy, qz, qw] of a world transform (generate_construction_data.py:587-605)."""
    R = M[:3, :3]
    sc = np.linalg.norm(R, axis=0)
    R = R / np.where(sc > 0, sc, 1.0)
    w, x, y, z = quat_wxyz_from_rot(R)
    if w < 0:
        w, x, y, z = -w, -x, -y, -z
    return [float(M[0, 3]), float(M[1, 3]), float(M[2, 3]), float(x), float(y), float(z), float(w)]


def frame_matrices(position, quat_wxyz_world, intr: Intrinsics) -> Tuple[np.ndarray, np.ndarray, np.ndarray]:
    """(view, proj, cam_to_world) as float64; the renderer rounds view/proj to float32."""
    C = camera_usd_transform(position, quat_wxyz_world)
    return view_matrix(C), intr.pixel_projection(), C
