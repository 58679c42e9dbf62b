"""Procedural stand-ins for the assets whose geometry is a Git-LFS pointer.

world2 references a Palfinger PK 7.501 crane, a site dumper and a digital
human (DHGen) whose meshes are missing (the prims are ``over``s,
the asset files are LFS pointers).  These proxies give config C3/C4 the same
*labelled objects* with plausible shapes and sizes:

* crane: four parts under the crane root, named after the first-level
  children of ``CRANE_PART_CHILD_MAP`` (generate_construction_data.py:110-121)
  so :func:`identity.get_object_root` resolves them to classes 6-9;
* dumper: chassis, skip, roll bar and four wheels (class 4);
* humans: a 17-joint COCO skeleton with one rigid instance per bone (class
  5); a pose is a set of instance transforms, so re-posing a human per
  randomisation epoch is a transform upload, not a mesh upload.

Tessellation follows SURVEY §8(d) ("procedural rigged humans, ~20k tris
each"): a human is 20,160 triangles (nine 1,248-triangle limb tubes, a
3,072-triangle torso, a 4,992-triangle head, two 432-triangle feet); the
crane (~36k) and the dumper (~25k) are built from the same finely
tessellated primitives, so their triangle counts are those of detailed
proxies rather than of a handful of boxes.

Everything is generated deterministically from code: no asset files.
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Tuple

import numpy as np

from .. import identity
from . import xform as X
from .model import Instance, Material, Mesh, Scene, SceneObject

COCO_JOINTS = ["nose", "left_eye", "right_eye", "left_ear", "right_ear", "left_shoulder", "right_shoulder",
               "left_elbow", "right_elbow", "left_wrist", "right_wrist", "left_hip", "right_hip", "left_knee",
               "right_knee", "left_ankle", "right_ankle"]


# ---------------------------------------------------------------------------
# unit primitives
# ---------------------------------------------------------------------------

def unit_box() -> Tuple[np.ndarray, np.ndarray]:
    """Cube [-0.5,0.5]^3, 12 triangles."""
    v = np.array([[x, y, z] for x in (-0.5, 0.5) for y in (-0.5, 0.5) for z in (-0.5, 0.5)], np.float32)
    quads = [(0, 1, 3, 2), (4, 6, 7, 5), (0, 4, 5, 1), (2, 3, 7, 6), (0, 2, 6, 4), (1, 5, 7, 3)]
    t = []
    for a, b, c, d in quads:
        t += [(a, b, c), (a, c, d)]
    return v, np.array(t, np.uint32)


def unit_cylinder(seg: int = 24) -> Tuple[np.ndarray, np.ndarray]:
    """Radius 1, z from 0 to 1, capped."""
    ang = 2 * np.pi * np.arange(seg) / seg
    ring = np.stack([np.cos(ang), np.sin(ang)], 1)
    v = np.concatenate([np.c_[ring, np.zeros(seg)], np.c_[ring, np.ones(seg)], [[0, 0, 0], [0, 0, 1]]]).astype(np.float32)
    t = []
    for i in range(seg):
        j = (i + 1) % seg
        t += [(i, j, seg + j), (i, seg + j, seg + i), (2 * seg, j, i), (2 * seg + 1, seg + i, seg + j)]
    return v, np.array(t, np.uint32)


def unit_sphere(nu: int = 20, nv: int = 14) -> Tuple[np.ndarray, np.ndarray]:
    v = [[0, 0, 1]]
    for i in range(1, nv):
        th = np.pi * i / nv
        for j in range(nu):
            ph = 2 * np.pi * j / nu
            v.append([np.sin(th) * np.cos(ph), np.sin(th) * np.sin(ph), np.cos(th)])
    v.append([0, 0, -1])
    v = np.array(v, np.float32)
    t = []
    for j in range(nu):
        t.append((0, 1 + j, 1 + (j + 1) % nu))
    for i in range(nv - 2):
        a0, b0 = 1 + i * nu, 1 + (i + 1) * nu
        for j in range(nu):
            j1 = (j + 1) % nu
            t += [(a0 + j, b0 + j, b0 + j1), (a0 + j, b0 + j1, a0 + j1)]
    last = len(v) - 1
    base = 1 + (nv - 2) * nu
    for j in range(nu):
        t.append((last, base + (j + 1) % nu, base + j))
    return v, np.array(t, np.uint32)


def grid_box(n: int) -> Tuple[np.ndarray, np.ndarray]:
    """Cube [-0.5,0.5]^3 whose faces are n x n quads (12 n^2 triangles)."""
    g = np.linspace(-0.5, 0.5, n + 1)
    verts, tris = [], []
    for axis in range(3):
        ua, va = [a for a in range(3) if a != axis]
        for sign in (-0.5, 0.5):
            base = sum(len(v) for v in verts)
            vv, uu = np.meshgrid(g, g, indexing="ij")
            p = np.zeros(((n + 1) * (n + 1), 3))
            p[:, axis] = sign
            p[:, ua] = uu.reshape(-1)
            p[:, va] = vv.reshape(-1)
            verts.append(p)
            j, i = np.meshgrid(np.arange(n), np.arange(n), indexing="ij")
            a = (base + j * (n + 1) + i).reshape(-1)
            b, c, d = a + 1, a + n + 1, a + n + 2
            t = np.stack([a, b, d, a, d, c], 1).reshape(-1, 3) if sign > 0 else \
                np.stack([a, d, b, a, c, d], 1).reshape(-1, 3)
            tris.append(t)
    return np.concatenate(verts).astype(np.float32), np.concatenate(tris).astype(np.uint32)


def unit_tube(seg: int, rings: int) -> Tuple[np.ndarray, np.ndarray]:
    """Radius 1, z from 0 to 1, `rings` bands of `seg` quads plus capped ends
    (2 seg (rings + 1) triangles)."""
    ang = 2 * np.pi * np.arange(seg) / seg
    ring = np.stack([np.cos(ang), np.sin(ang)], 1)
    z = np.repeat(np.arange(rings + 1) / rings, seg)
    v = np.concatenate([np.c_[np.tile(ring, (rings + 1, 1)), z], [[0, 0, 0], [0, 0, 1]]]).astype(np.float32)
    i = np.arange(seg)
    j = (i + 1) % seg
    t = []
    for r in range(rings):
        a0, a1 = r * seg, (r + 1) * seg
        t += [np.stack([a0 + i, a0 + j, a1 + j], 1), np.stack([a0 + i, a1 + j, a1 + i], 1)]
    c0, c1 = (rings + 1) * seg, (rings + 1) * seg + 1
    t += [np.stack([np.full(seg, c0), j, i], 1), np.stack([np.full(seg, c1), rings * seg + i, rings * seg + j], 1)]
    return v, np.concatenate(t).astype(np.uint32)


def unit_torus(seg: int, rseg: int, r: float) -> Tuple[np.ndarray, np.ndarray]:
    """Ring radius 1 about z, tube radius r (2 seg rseg triangles)."""
    a = 2 * np.pi * np.arange(seg) / seg
    b = 2 * np.pi * np.arange(rseg) / rseg
    A, B = np.meshgrid(a, b, indexing="ij")
    rr = 1.0 + r * np.cos(B)
    v = np.stack([rr * np.cos(A), rr * np.sin(A), r * np.sin(B)], -1).reshape(-1, 3).astype(np.float32)
    I, J = np.meshgrid(np.arange(seg), np.arange(rseg), indexing="ij")
    p00 = I * rseg + J
    p10 = ((I + 1) % seg) * rseg + J
    p01 = I * rseg + (J + 1) % rseg
    p11 = ((I + 1) % seg) * rseg + (J + 1) % rseg
    t = np.stack([p00, p10, p11, p00, p11, p01], -1).reshape(-1, 3)
    return v, t.astype(np.uint32)


# tessellations used by the proxies (name -> mesh); keys double as mesh names
PRIMITIVES = {
    "box": unit_box,
    "cyl": unit_cylinder,
    "sphere": unit_sphere,
    "box6": lambda: grid_box(6), "box8": lambda: grid_box(8), "box10": lambda: grid_box(10),
    "box12": lambda: grid_box(12), "box16": lambda: grid_box(16), "box20": lambda: grid_box(20),
    "tube12x8": lambda: unit_tube(12, 8), "tube16x2": lambda: unit_tube(16, 2), "tube24x8": lambda: unit_tube(24, 8),
    "tube32x4": lambda: unit_tube(32, 4), "tube32x12": lambda: unit_tube(32, 12),
    "tube48x2": lambda: unit_tube(48, 2), "tube48x12": lambda: unit_tube(48, 12),
    "tube96x6": lambda: unit_tube(96, 6), "tube128x32": lambda: unit_tube(128, 32),
    "sphere32x20": lambda: unit_sphere(32, 20), "sphere64x40": lambda: unit_sphere(64, 40),
    "torus64x24": lambda: unit_torus(64, 24, 0.42), "torus48x12": lambda: unit_torus(48, 12, 0.08),
}


def bone_matrix(a: np.ndarray, b: np.ndarray, radius: float) -> np.ndarray:
    """Unit cylinder (z 0..1) -> cylinder from a to b of the given radius.
    (Scalar float arithmetic: numpy's per-call overhead on 3-vectors was most
    of the generator's per-epoch pose time.)"""
    a0, a1, a2 = (float(v) for v in a)
    d0, d1, d2 = float(b[0]) - a0, float(b[1]) - a1, float(b[2]) - a2
    L = math.sqrt(d0 * d0 + d1 * d1 + d2 * d2)
    z0, z1, z2 = (d0 / L, d1 / L, d2 / L) if L > 0 else (0.0, 0.0, 1.0)
    h0, h1, h2 = (1.0, 0.0, 0.0) if abs(z0) < 0.9 else (0.0, 1.0, 0.0)
    x0, x1, x2 = h1 * z2 - h2 * z1, h2 * z0 - h0 * z2, h0 * z1 - h1 * z0     # helper x z
    n = math.sqrt(x0 * x0 + x1 * x1 + x2 * x2)
    x0, x1, x2 = x0 / n, x1 / n, x2 / n
    y0, y1, y2 = z1 * x2 - z2 * x1, z2 * x0 - z0 * x2, z0 * x1 - z1 * x0     # z x x
    return np.array([[x0 * radius, y0 * radius, z0 * L, a0],
                     [x1 * radius, y1 * radius, z1 * L, a1],
                     [x2 * radius, y2 * radius, z2 * L, a2],
                     [0.0, 0.0, 0.0, 1.0]])


def box_matrix(center, size, yaw_pitch: Optional[np.ndarray] = None) -> np.ndarray:
    m = X.translate(center)
    if yaw_pitch is not None:
        m = m @ yaw_pitch
    return m @ X.scale(size)


# ---------------------------------------------------------------------------
# human rig
# ---------------------------------------------------------------------------

@dataclass
class HumanRig:
    obj: int                                  # index into Scene.objects
    frame0: np.ndarray                        # authored object frame
    parts: List[Tuple[int, str]] = field(default_factory=list)   # (instance index, part name)

    REST = {
        "pelvis": (0.0, 0.0, 0.95), "neck": (0.0, 0.0, 1.45), "head": (0.0, 0.0, 1.62),
        "left_hip": (0.0, 0.10, 0.92), "right_hip": (0.0, -0.10, 0.92),
        "left_shoulder": (0.0, 0.19, 1.44), "right_shoulder": (0.0, -0.19, 1.44),
    }
    L_UPPER, L_FORE, L_THIGH, L_SHANK = 0.29, 0.26, 0.43, 0.42

    @staticmethod
    def pose_params(rng: np.random.Generator) -> Dict[str, float]:
        return {
            "l_sh_flex": rng.uniform(-50, 80), "r_sh_flex": rng.uniform(-50, 80),
            "l_sh_abd": rng.uniform(5, 45), "r_sh_abd": rng.uniform(5, 45),
            "l_elbow": rng.uniform(0, 100), "r_elbow": rng.uniform(0, 100),
            "l_hip": rng.uniform(-25, 40), "r_hip": rng.uniform(-25, 40),
            "l_knee": rng.uniform(0, 60), "r_knee": rng.uniform(0, 60),
            "head_yaw": rng.uniform(-40, 40),
        }

    @classmethod
    def joints(cls, p: Optional[Dict[str, float]] = None) -> Dict[str, np.ndarray]:
        """COCO-17 joints (+ pelvis/neck/head) in the human's local frame (X fwd, Y left, Z up)."""
        p = p or {k: 0.0 for k in ("l_sh_flex", "r_sh_flex", "l_elbow", "r_elbow", "l_hip", "r_hip", "l_knee",
                                   "r_knee", "head_yaw")} | {"l_sh_abd": 8.0, "r_sh_abd": 8.0}
        J = {k: np.array(v, float) for k, v in cls.REST.items()}

        def limb(flex_deg, abd_deg, side):
            # rest direction straight down; abduct outward about X, then flex forward about Y
            d = np.array([0.0, 0.0, -1.0])
            d = X.rot_x(side * abd_deg)[:3, :3] @ d
            return X.rot_y(-flex_deg)[:3, :3] @ d

        for side, s in (("left", 1.0), ("right", -1.0)):
            c = side[0]
            sh = J[f"{side}_shoulder"]
            du = limb(p[f"{c}_sh_flex"], p[f"{c}_sh_abd"], s)
            el = sh + cls.L_UPPER * du
            df = limb(p[f"{c}_sh_flex"] + p[f"{c}_elbow"], p[f"{c}_sh_abd"], s)
            J[f"{side}_elbow"], J[f"{side}_wrist"] = el, el + cls.L_FORE * df
            hp = J[f"{side}_hip"]
            dt = limb(p[f"{c}_hip"], 2.0, s)
            kn = hp + cls.L_THIGH * dt
            ds = limb(p[f"{c}_hip"] - p[f"{c}_knee"], 2.0, s)
            J[f"{side}_knee"], J[f"{side}_ankle"] = kn, kn + cls.L_SHANK * ds
        R = X.rot_z(p["head_yaw"])[:3, :3]
        h = J["head"]
        J["nose"] = h + R @ np.array([0.10, 0.0, 0.0])
        J["left_eye"] = h + R @ np.array([0.085, 0.032, 0.035])
        J["right_eye"] = h + R @ np.array([0.085, -0.032, 0.035])
        J["left_ear"] = h + R @ np.array([0.0, 0.078, 0.01])
        J["right_ear"] = h + R @ np.array([0.0, -0.078, 0.01])
        return J

    BONES = [  # (part, joint a, joint b, radius, material key)
        ("upperarm_l", "left_shoulder", "left_elbow", 0.050, "vest"),
        ("upperarm_r", "right_shoulder", "right_elbow", 0.050, "vest"),
        ("forearm_l", "left_elbow", "left_wrist", 0.040, "skin"),
        ("forearm_r", "right_elbow", "right_wrist", 0.040, "skin"),
        ("thigh_l", "left_hip", "left_knee", 0.075, "trousers"),
        ("thigh_r", "right_hip", "right_knee", 0.075, "trousers"),
        ("shank_l", "left_knee", "left_ankle", 0.058, "trousers"),
        ("shank_r", "right_knee", "right_ankle", 0.058, "trousers"),
        ("neck", "neck", "head", 0.045, "skin"),
    ]

    @classmethod
    def part_locals(cls, J: Dict[str, np.ndarray]) -> Dict[str, np.ndarray]:
        out = {name: bone_matrix(J[a], J[b], r) for name, a, b, r, _ in cls.BONES}
        out["torso"] = box_matrix((J["pelvis"] + J["neck"]) / 2 + np.array([0, 0, 0.02]), (0.24, 0.40, 0.56))
        out["head"] = X.translate(J["head"]) @ X.rot_z(0) @ X.scale((0.105, 0.095, 0.12))
        for side, c in (("left", "l"), ("right", "r")):
            out[f"foot_{c}"] = box_matrix(J[f"{side}_ankle"] + np.array([0.06, 0, -0.045]), (0.26, 0.10, 0.08))
        return out


# ---------------------------------------------------------------------------
# scene augmentation
# ---------------------------------------------------------------------------

PROXY_MATERIALS = {
    "crane_yellow": (0.92, 0.70, 0.08), "crane_red": (0.75, 0.10, 0.08), "crane_grey": (0.35, 0.36, 0.38),
    "dumper_orange": (0.93, 0.45, 0.06), "tyre": (0.07, 0.07, 0.07), "steel": (0.45, 0.46, 0.48),
    "vest": (0.98, 0.78, 0.05), "skin": (0.80, 0.62, 0.50), "trousers": (0.15, 0.20, 0.35),
}

# Crane parts: (first-level child name from CRANE_PART_CHILD_MAP, primitive, local matrix, material);
# several pieces may share a child (one object root each, GDP:110-121).
_BOOM = X.translate((0, 0, 2.2)) @ X.rot_y(-22)
_TELE = _BOOM @ X.translate((2.7, 0, 0)) @ X.rot_y(40)
_TIP = (_TELE @ np.array([2.8, 0.0, 0.0, 1.0]))[:3]
_HOOK = _TIP + np.array([0.0, 0.0, -1.2])
_CRANE_PARTS = [
    # cranebase: chassis block, two outrigger beams with four jacks, slewing ring (6,560 tris)
    ("S104GG03A_SW", "box16", box_matrix((0, 0, 0.30), (1.3, 1.0, 0.6)), "crane_grey"),
    ("S104GG03A_SW", "box6", box_matrix((0.45, 0, 0.18), (0.16, 3.0, 0.16)), "crane_yellow"),
    ("S104GG03A_SW", "box6", box_matrix((-0.45, 0, 0.18), (0.16, 3.0, 0.16)), "crane_yellow"),
] + [
    ("S104GG03A_SW", "tube32x4", X.translate((x, y, 0.0)) @ X.scale((0.07, 0.07, 0.35)), "steel")
    for x in (0.45, -0.45) for y in (1.45, -1.45)
] + [
    ("S104GG03A_SW", "tube96x6", X.translate((0, 0, 0.6)) @ X.scale((0.42, 0.42, 0.12)), "crane_grey"),
    # cranecolumn: column and two lift rams (10,112 tris)
    ("S104HZ01KA_SW", "tube128x32", X.translate((0, 0, 0.6)) @ X.scale((0.17, 0.17, 1.55)), "crane_red"),
    ("S104HZ01KA_SW", "tube32x12", bone_matrix((0.25, 0.1, 0.8), (0.6, 0.1, 2.0), 0.05), "steel"),
    ("S104HZ01KA_SW", "tube32x12", bone_matrix((0.25, -0.1, 0.8), (0.6, -0.1, 2.0), 0.05), "steel"),
    # craneboom: boom, two hydraulic cylinders, 20 lattice struts (8,384 tris)
    ("tn__S104EKB_AS_SW_jj7", "box20", _BOOM @ X.translate((1.35, 0, 0)) @ X.scale((2.9, 0.26, 0.32)), "crane_yellow"),
    ("tn__S104EKB_AS_SW_jj7", "tube32x12", bone_matrix((0.9, 0.17, 2.3), (2.6, 0.17, 1.9), 0.045), "steel"),
    ("tn__S104EKB_AS_SW_jj7", "tube32x12", bone_matrix((0.9, -0.17, 2.3), (2.6, -0.17, 1.9), 0.045), "steel"),
] + [
    ("tn__S104EKB_AS_SW_jj7", "tube16x2",
     _BOOM @ X.translate((0.2 + 0.25 * k, 0.14 * side, -0.16)) @ X.scale((0.015, 0.015, 0.32)), "steel")
    for k in range(10) for side in (1.0, -1.0)
] + [
    # cranetelescopic: three nested extension sections, hook block and cable (10,648 tris)
    ("S104KZ02KA_SW", "box16", _TELE @ X.translate((0.6, 0, 0)) @ X.scale((1.2, 0.19, 0.23)), "crane_yellow"),
    ("S104KZ02KA_SW", "box16", _TELE @ X.translate((1.5, 0, 0)) @ X.scale((1.1, 0.16, 0.2)), "crane_yellow"),
    ("S104KZ02KA_SW", "box16", _TELE @ X.translate((2.3, 0, 0)) @ X.scale((1.0, 0.13, 0.17)), "crane_yellow"),
    ("S104KZ02KA_SW", "sphere32x20", X.translate(_HOOK) @ X.scale((0.12, 0.12, 0.12)), "steel"),
    ("S104KZ02KA_SW", "tube12x8", bone_matrix(_TIP, _HOOK, 0.012), "steel"),
]

_WHEELS = [(1.0, 0.78), (1.0, -0.78), (-1.0, 0.78), (-1.0, -0.78)]
_DUMPER_PARTS = [  # (piece, primitive, local matrix, material): 25,728 tris
    ("chassis", "box20", box_matrix((0, 0, 0.62), (3.2, 1.5, 0.45)), "dumper_orange"),
    ("skip", "box16", X.translate((0.95, 0, 1.05)) @ X.rot_y(-12) @ X.scale((1.5, 1.65, 0.75)), "dumper_orange"),
    ("rops_l", "tube24x8", bone_matrix((-1.15, 0.55, 0.85), (-1.15, 0.55, 2.2), 0.05), "steel"),
    ("rops_r", "tube24x8", bone_matrix((-1.15, -0.55, 0.85), (-1.15, -0.55, 2.2), 0.05), "steel"),
    ("rops_top", "tube24x8", bone_matrix((-1.15, -0.55, 2.2), (-1.15, 0.55, 2.2), 0.05), "steel"),
    ("seat", "box8", box_matrix((-0.75, 0, 1.05), (0.55, 0.6, 0.45)), "steel"),
    ("hood", "box10", box_matrix((-0.2, 0, 1.0), (0.7, 1.2, 0.35)), "dumper_orange"),
    ("steering", "torus48x12", X.translate((-0.45, 0, 1.5)) @ X.rot_y(-30) @ X.scale((0.18, 0.18, 0.18)), "tyre"),
] + [
    (f"tyre_{i}", "torus64x24", X.translate((x, y, 0.46)) @ X.rot_x(90) @ X.scale((0.36, 0.36, 0.36)), "tyre")
    for i, (x, y) in enumerate(_WHEELS)
] + [
    (f"rim_{i}", "tube48x2", X.translate((x, y, 0.46)) @ X.rot_x(90) @ X.translate((0, 0, -0.15))
     @ X.scale((0.3, 0.3, 0.3)), "steel") for i, (x, y) in enumerate(_WHEELS)
]

# authored placements (world2): crane at the origin, dumper at (-7.37, 0) yawed -92.19 deg,
# DHGen at (0.81, -3.54) yawed by its SkelRoot orient; extra humans are this build's addition.
_HUMAN_FRAMES = [((0.81, -3.54), -165.76), ((-3.0, 4.0), 30.0), ((4.0, -6.0), 120.0), ((2.5, 5.5), -60.0)]


def add_proxies(scene: Scene, n_humans: int = 4, crane: bool = True, dumper: bool = True) -> Scene:
    """Append crane/dumper/human proxies to ``scene`` (in place) and return it."""
    mesh_ids: Dict[Tuple[str, str], int] = {}
    mat_ids: Dict[str, int] = {}

    def mat(name):
        if name not in mat_ids:
            scene.materials.append(Material("proxy_" + name, np.array(PROXY_MATERIALS[name]), -1, False, 0))
            mat_ids[name] = len(scene.materials) - 1
        return mat_ids[name]

    def mesh(kind, material):
        key = (kind, material)
        if key not in mesh_ids:
            v, t = PRIMITIVES[kind]()
            scene.meshes.append(Mesh(f"proxy_{kind}_{material}", v, t, np.zeros((0, 2), np.float32),
                                     np.zeros((0, 3), np.uint32), mat(material)))
            mesh_ids[key] = len(scene.meshes) - 1
        return mesh_ids[key]

    frames = scene.meta.setdefault("object_frames", {})
    next_idx = max([o.inst_idx for o in scene.objects] + [-1]) + 1

    def new_object(root, class_name, class_id, kind, frame):
        nonlocal next_idx
        scene.objects.append(SceneObject(root, class_name, class_id, next_idx, kind))
        next_idx += 1
        frames.setdefault(root.split("#")[0], frame.tolist())
        return len(scene.objects) - 1

    def add_part(obj, kind, material, local, frame):
        inst = Instance(mesh(kind, material), frame @ local, scene.objects[obj].inst_idx, obj, local)
        scene.instances.append(inst)
        return len(scene.instances) - 1

    def finish_bounds(obj):
        lo, hi = np.full(3, np.inf), np.full(3, -np.inf)
        for inst in scene.instances:
            if inst.obj == obj:
                p = X.transform_points(inst.local, scene.meshes[inst.mesh].positions)
                lo, hi = np.minimum(lo, p.min(0)), np.maximum(hi, p.max(0))
        scene.objects[obj].local_bounds = np.stack([lo, hi])

    if crane:
        frame = X.translate((0.0, 0.0015, 0.0))
        by_root: Dict[str, int] = {}
        for child, kind, local, material in _CRANE_PARTS:
            path = f"{identity.CRANE_ROOT}/{child}/proxy_mesh"
            root, cname, cid = identity.get_object_root(path)
            if root not in by_root:
                by_root[root] = new_object(root, cname, cid, "crane", frame)
            add_part(by_root[root], kind, material, local, frame)
        for o in by_root.values():
            finish_bounds(o)
    if dumper:
        frame = X.translate((-7.3687, 0.0, 0.0)) @ X.rot_z(-92.19059753)
        root, cname, cid = identity.get_object_root(f"{identity.DUMPER_ROOT}/proxy/chassis")
        o = new_object(root, cname, cid, "dumper", frame)
        for _, kind, local, material in _DUMPER_PARTS:
            add_part(o, kind, material, local, frame)
        finish_bounds(o)
    rigs = scene.meta.setdefault("human_rigs", [])
    for h in range(n_humans):
        (x, y), yaw = _HUMAN_FRAMES[h % len(_HUMAN_FRAMES)]
        if h >= len(_HUMAN_FRAMES):
            x, y = x + 1.5 * (h // len(_HUMAN_FRAMES)), y
        frame = X.translate((x, y, 0.0)) @ X.rot_z(yaw)
        seg = "DHGen" if h == 0 else f"DHGen_{h:02d}"
        root = f"/World/GroundPlane/{seg}"
        _, cname, cid = identity.get_object_root(root + "/SkelRoot/proxy")
        o = new_object(root, cname, cid, "human", frame)
        J = HumanRig.joints()
        locs = HumanRig.part_locals(J)
        mats = {name: m for name, _, _, _, m in HumanRig.BONES}
        mats.update({"torso": "vest", "head": "skin", "foot_l": "trousers", "foot_r": "trousers"})
        kinds = {name: "tube48x12" for name, *_ in HumanRig.BONES}
        kinds.update({"torso": "box16", "head": "sphere64x40", "foot_l": "box6", "foot_r": "box6"})
        parts = []
        for name, local in locs.items():
            parts.append([add_part(o, kinds[name], mats[name], local, frame), name])
        finish_bounds(o)
        rigs.append({"obj": o, "parts": parts})
    return scene


def pose_humans(scene: Scene, object_frames: List[np.ndarray], models: np.ndarray, rng_for_human) -> Dict[int, Dict]:
    """Re-pose every rigged human: writes its part instances into ``models``
    (I,4,4) and returns ``{obj: joints(local)}``."""
    out = {}
    for rig in scene.meta.get("human_rigs", []):
        o = rig["obj"]
        p = HumanRig.pose_params(rng_for_human(o))
        J = HumanRig.joints(p)
        locs = HumanRig.part_locals(J)
        for inst_i, name in rig["parts"]:
            scene.instances[inst_i]  # existence check
            models[inst_i] = object_frames[o] @ locs[name]
        out[o] = J
    return out
