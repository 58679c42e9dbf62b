"""Domain-randomisation schedule: camera poses and object placement.

Restates the semantics of the reference's
``get_systematic_camera_positions`` (generate_construction_data.py:778-911)
and ``randomize_object_positions`` (:914-1231, run every 10 frames, :1542)
with one deliberate change: the reference draws from the global, unseeded
``np.random`` in sequence, so frame k depends on every draw before it.  Here
every random draw comes from a counter-based generator keyed by
``(seed, stream, index)`` — a frame's camera is a pure function of
``(seed, frame)`` and an epoch's layout of ``(seed, epoch)`` — which is what
lets the 8 GPUs of a node each own a shard of the seed space with no
communication.  The draw distributions, constants and
placement order are the reference's.
"""
from __future__ import annotations

import math
from dataclasses import dataclass
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np

from .scene import xform as X
from .scene.model import Light, Scene, Texture

HEIGHTS = [1.6, 1.7, 1.8, 2.0, 2.5, 3.0]                         # :790
DUMPER_CENTER = (-7.37, -0.59)                                  # :794
KEY_POSITIONS = [                                               # :796-838
    ([-15, -0.6], DUMPER_CENTER), ([-2, -0.6], DUMPER_CENTER), ([-7.4, 6], DUMPER_CENTER),
    ([-7.4, -7], DUMPER_CENTER), ([-12, 4], DUMPER_CENTER), ([-12, -5], DUMPER_CENTER),
    ([-4, 4], DUMPER_CENTER), ([-4, -4], DUMPER_CENTER), ([-10, 0], DUMPER_CENTER),
    ([-5, 2], DUMPER_CENTER), ([-5, -3], DUMPER_CENTER), ([-9, -4], DUMPER_CENTER),
    ([-3, -3], [0, 0]), ([-3, 3], [0, 0]), ([0, 0], [5, 0]), ([0, 0], [-5, 0]),
    ([6, 0], [0, 0]), ([0, 6], [0, 0]), ([0, -6], [0, 0]), ([-6, 0], [0, 0]),
    ([5, 5], [0, 0]), ([5, -5], [0, 0]), ([-5, 5], [0, 0]), ([-5, -5], [0, 0]),
    ([3, 0], [0, 0]), ([-3, 0], [0, 0]), ([0, 3], [0, 0]), ([0, -3], [0, 0]),
    ([-8, -3], [0, 0]), ([-8, 3], [0, 0]),
]
RADII = [4, 6, 8, 10, 12]                                       # :857
POINTS_PER_RING = 8                                             # :858
EPOCH_FRAMES = 10                                               # :1542

FENCE_X = (-9.0, 8.5)                                           # :935
FENCE_Y = (-9.0, 9.0)                                           # :936
DUMPER_AREAS = [(-7, -1), (-3, -5), (5, 0), (-5, 5), (3, -4), (6, 3), (-6, -4)]   # :1110-1118

STREAM_CAMERA_RING, STREAM_CAMERA_RANDOM, STREAM_LAYOUT, STREAM_POSE, STREAM_DR = 1, 2, 3, 4, 5
STREAM_RETRY = 6


def rng_for(seed: int, stream: int, index: int) -> np.random.Generator:
    """Counter-based stream: independent of every other (stream, index)."""
    return np.random.Generator(np.random.Philox(key=[seed & 0xFFFFFFFFFFFFFFFF,
                                                     ((stream & 0xFFFF) << 48) | (index & 0xFFFFFFFFFFFF)]))


def retry_offset(seed: int, k: int, attempt: int) -> np.ndarray:
    """Camera jitter of validation retry ``attempt`` (>= 1) of frame k: the
    reference's ``np.random.uniform(-2, 2, size=3)`` with the z offset halved
    (generate_construction_data.py:1574-1579), drawn from its own counter
    stream keyed by (seed, frame, attempt) instead of the global NumPy state."""
    off = rng_for(seed, STREAM_RETRY, (k << 4) | (attempt & 15)).uniform(-2.0, 2.0, size=3)
    off[2] *= 0.5
    return off


def camera_pose(seed: int, k: int) -> Tuple[np.ndarray, np.ndarray]:
    """(camera position, aim point) of frame k (level shots, :847-849, :876, :905)."""
    z = HEIGHTS[k % len(HEIGHTS)]
    if k < len(KEY_POSITIONS):
        cxy, txy = KEY_POSITIONS[k]
        return np.array([cxy[0], cxy[1], z], float), np.array([txy[0], txy[1], z], float)
    j = k - len(KEY_POSITIONS)
    if j < len(RADII) * POINTS_PER_RING:
        radius = RADII[j // POINTS_PER_RING]
        angle = 2 * np.pi * (j % POINTS_PER_RING) / POINTS_PER_RING
        cam = np.array([radius * np.cos(angle), radius * np.sin(angle), z])
        r = rng_for(seed, STREAM_CAMERA_RING, k)
        if r.random() < 0.4:
            tgt = np.array([DUMPER_CENTER[0] + r.uniform(-2, 2), DUMPER_CENTER[1] + r.uniform(-2, 2), z])
        else:
            tgt = np.array([0.0, 0.0, z])
        return cam, tgt
    r = rng_for(seed, STREAM_CAMERA_RANDOM, k)
    if r.random() < 0.5:
        angle = r.uniform(0, 2 * np.pi)
        dist = r.uniform(5, 12)
        cx = DUMPER_CENTER[0] + dist * np.cos(angle)
        cy = DUMPER_CENTER[1] + dist * np.sin(angle)
        tx = DUMPER_CENTER[0] + r.uniform(-1, 1)
        ty = DUMPER_CENTER[1] + r.uniform(-1, 1)
    else:
        cx, cy = r.uniform(-10, 8), r.uniform(-10, 10)
        tx, ty = r.uniform(-3, 3), r.uniform(-3, 3)
    return np.array([cx, cy, z]), np.array([tx, ty, z])


def get_systematic_camera_positions(num_frames: int = 20, seed: int = 0) -> List[Tuple[np.ndarray, np.ndarray]]:
    """Same contract as the reference function (:778): list of (cam, target)."""
    return [camera_pose(seed, k) for k in range(num_frames)]


def epoch_of(frame: int) -> int:
    return frame // EPOCH_FRAMES


# ---------------------------------------------------------------------------
# object placement (randomize_object_positions)
# ---------------------------------------------------------------------------

@dataclass
class Placement:
    x: float
    y: float
    z: float
    rotation: Optional[float]       # degrees about the object's local Z (appended rotateZ op)
    no_overlap: bool


def _is_within_fence(x, y, margin=0.0) -> bool:
    return FENCE_X[0] + margin <= x <= FENCE_X[1] - margin and FENCE_Y[0] + margin <= y <= FENCE_Y[1] - margin


def xy_radius(scene: Scene, obj: int, default: float) -> float:
    """compute_prim_xy_radius (:971-988) on the authored (epoch-0) world AABB."""
    o = scene.objects[obj]
    if o.local_bounds is None or not np.all(np.isfinite(o.local_bounds)):
        return default
    frame = object_frame(scene, obj)
    lo, hi = o.local_bounds
    corners = np.array([[x, y, z] for x in (lo[0], hi[0]) for y in (lo[1], hi[1]) for z in (lo[2], hi[2])])
    w = X.transform_points(frame, corners)
    dx = (w[:, 0].max() - w[:, 0].min()) / 2.0
    dy = (w[:, 1].max() - w[:, 1].min()) / 2.0
    return max(math.sqrt(dx * dx + dy * dy) * 0.9, 1.0)


def object_frame(scene: Scene, obj: int) -> np.ndarray:
    frames = scene.meta.get("object_frames", {})
    f = frames.get(scene.objects[obj].prim_path.split("#")[0])
    return np.asarray(f, float) if f is not None else np.eye(4)


def movable(scene: Scene) -> Dict[str, List[int]]:
    kinds: Dict[str, List[int]] = {"crane": [], "dumper": [], "human": [], "trafficcone": []}
    for j, o in enumerate(scene.objects):
        if o.kind in kinds:
            kinds[o.kind].append(j)
    for k in kinds:
        kinds[k].sort(key=lambda j: scene.objects[j].prim_path)
    return kinds


def randomize_object_positions(scene: Scene, seed: int, epoch: int) -> Dict[int, Placement]:
    """Placement of every movable object for one epoch (epoch 0 = authored layout).

    Order and constants follow :1084-1222: crane (centre +-4 m, radius >= 6 m,
    no rotation) -> dumper (7 candidate areas in random order, +-2 m, radius >=
    2.5 m, yaw U(-180,180)) -> humans (centre U(-7,7), +-4 m, r 0.8 m, yaw) ->
    cones (centre U(-6,6), +-2 m, r 0.5 m, fence margin 1 m, yaw); sum-of-radii
    non-overlap (:946-956), 80 attempts then a clamped fallback (:958-969).
    Crane parts share one placement (they are one USD prim, :1085).
    """
    if epoch == 0:
        return {}
    rng = rng_for(seed, STREAM_LAYOUT, epoch)
    placed: List[Tuple[float, float, float]] = []
    out: Dict[int, Placement] = {}

    def no_overlap(x, y, r):
        return all(math.hypot(x - px, y - py) >= r + pr for px, py, pr in placed)

    def find_valid(cx, cy, rx, ry, r, attempts=80, margin=0.5):
        for _ in range(attempts):
            x = rng.uniform(cx - rx, cx + rx)
            y = rng.uniform(cy - ry, cy + ry)
            if _is_within_fence(x, y, margin) and no_overlap(x, y, r):
                return x, y, True
        fx = float(np.clip(cx + rng.uniform(-1, 1), FENCE_X[0] + margin, FENCE_X[1] - margin))
        fy = float(np.clip(cy + rng.uniform(-1, 1), FENCE_Y[0] + margin, FENCE_Y[1] - margin))
        return fx, fy, False

    kinds = movable(scene)
    if kinds["crane"]:
        objs = kinds["crane"]
        z = object_frame(scene, objs[0])[2, 3]
        r = max(max(xy_radius(scene, j, 7.0) for j in objs), 6.0)
        x, y, ok = find_valid(0, 0, 4.0, 4.0, r)
        placed.append((x, y, r))
        for j in objs:
            out[j] = Placement(x, y, z, None, ok)
    for j in kinds["dumper"]:
        z = object_frame(scene, j)[2, 3]
        r = max(xy_radius(scene, j, 3.0), 2.5)
        best = None
        for a in rng.permutation(len(DUMPER_AREAS)):
            ax, ay = DUMPER_AREAS[int(a)]
            x, y, ok = find_valid(ax, ay, 2.0, 2.0, r)
            if ok:
                best = (x, y, ok)
                break
        if best is None:
            ax, ay = DUMPER_AREAS[0]
            best = find_valid(ax, ay, 3.0, 3.0, r)
        rot = float(rng.uniform(-180, 180))
        placed.append((best[0], best[1], r))
        out[j] = Placement(best[0], best[1], z, rot, best[2])
    for j in kinds["human"]:
        z = object_frame(scene, j)[2, 3]
        x, y, ok = find_valid(rng.uniform(-7, 7), rng.uniform(-7, 7), 4.0, 4.0, 0.8)
        rot = float(rng.uniform(-180, 180))
        placed.append((x, y, 0.8))
        out[j] = Placement(x, y, z, rot, ok)
    for j in kinds["trafficcone"]:
        z = object_frame(scene, j)[2, 3]
        cx, cy = rng.uniform(-6, 6), rng.uniform(-6, 6)
        x, y, ok = find_valid(cx, cy, 2.0, 2.0, 0.5, margin=1.0)
        rot = float(rng.uniform(-180, 180))
        placed.append((x, y, 0.5))
        out[j] = Placement(x, y, z, rot, ok)
    return out


def placed_frame(frame0: np.ndarray, p: Placement) -> np.ndarray:
    """set_prim_transform (:990-1053): translation replaced, rotateZ appended
    (applied to points first, in the object's local frame)."""
    m = frame0.copy()
    m[:3, 3] = [p.x, p.y, p.z]
    if p.rotation is not None:
        m = m @ X.rot_z(p.rotation)
    return m


def object_frames_for_epoch(scene: Scene, seed: int, epoch: int) -> List[np.ndarray]:
    frames = [object_frame(scene, j) for j in range(len(scene.objects))]
    for j, p in randomize_object_positions(scene, seed, epoch).items():
        frames[j] = placed_frame(frames[j], p)
    return frames


# ---------------------------------------------------------------------------
# Domain randomisation of lighting and textures (C4 of BASELINE.json)
# ---------------------------------------------------------------------------
# The reference fixes its lighting once (setup_scene_lighting,
# generate_construction_data.py:1289-1345: dome 500, distant light clamped to
# 1500) and never swaps textures; C4 adds per-epoch DR on top of the layout
# randomisation, drawn from its own counter-based stream so it never perturbs
# the layout or camera draws.
KEEP_TEXTURE = -2
DR_TINTS = {"autumn": (1.25, 0.85, 0.45), "dry": (1.05, 1.0, 0.7)}


@dataclass
class DRParams:
    light: Light
    textures: List[int]          # per material: texture index, -1 none, KEEP_TEXTURE


def add_dr_texture_variants(scene: Scene) -> Dict[int, List[int]]:
    """Append tinted copies of every material texture (alpha kept, so cut-out
    silhouettes stay put) and return {material: [variant texture ids]}.
    Idempotent: a second call returns the recorded variants."""
    if "dr_variants" in scene.meta:
        return {int(k): v for k, v in scene.meta["dr_variants"].items()}
    made: Dict[int, List[int]] = {}
    out: Dict[int, List[int]] = {}
    for m, mat in enumerate(scene.materials):
        if mat.texture < 0:
            continue
        if mat.texture not in made:
            base = scene.textures[mat.texture].rgba
            ids = []
            for name, tint in DR_TINTS.items():
                rgba = base.copy()
                rgba[..., :3] = np.clip(np.round(base[..., :3].astype(np.float64) * np.asarray(tint)), 0, 255)
                scene.textures.append(Texture(f"{scene.textures[mat.texture].name}:{name}", rgba.astype(np.uint8)))
                ids.append(len(scene.textures) - 1)
            made[mat.texture] = ids
        out[m] = made[mat.texture]
    scene.meta["dr_variants"] = {str(k): v for k, v in out.items()}
    return out


def domain_randomization(scene: Scene, seed: int, epoch: int, variants: Dict[int, List[int]]) -> DRParams:
    """Lighting + texture choice of one epoch (epoch 0 = authored).  Dome tint
    x U(0.8, 1.2) per channel, dome intensity 500 x U(0.6, 1.4), sun elevation
    U(20, 75) deg, azimuth U(0, 360) deg, sun intensity U(750, 1500) (the
    reference's 1500 clamp), each textured material picks its own texture or
    one of its tinted variants uniformly."""
    base = scene.light
    if epoch == 0:
        return DRParams(base, [KEEP_TEXTURE] * len(scene.materials))
    rng = rng_for(seed, STREAM_DR, epoch)
    dome = np.clip(np.asarray(base.dome_color, np.float64) * rng.uniform(0.8, 1.2, 3), 0.0, 1.0)
    dome_i = float(base.dome_intensity) * float(rng.uniform(0.6, 1.4))
    el = math.radians(float(rng.uniform(20.0, 75.0)))
    az = math.radians(float(rng.uniform(0.0, 360.0)))
    sun_dir = np.array([math.cos(el) * math.cos(az), math.cos(el) * math.sin(az), math.sin(el)])
    sun_i = float(rng.uniform(750.0, 1500.0))
    light = Light(sun_dir=sun_dir, sun_intensity=sun_i, sun_color=np.asarray(base.sun_color, np.float64),
                  dome_intensity=dome_i, dome_color=dome)
    tex = [KEEP_TEXTURE] * len(scene.materials)
    for m in sorted(variants):
        k = int(rng.integers(0, len(variants[m]) + 1))
        tex[m] = KEEP_TEXTURE if k == 0 else variants[m][k - 1]
    return DRParams(light, tex)
