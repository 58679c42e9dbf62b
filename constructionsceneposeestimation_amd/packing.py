"""Flatten a :class:`Scene` into the plain arrays the C-ABI consumes.

The layout here is the HBM layout of the scene on the GPU (DESIGN.md
"Data layout"): one global float32 position array, mesh-relative uint32
triangle arrays, one RGBA8 texel blob, and small descriptor tables.  The
same packed arrays feed the CPU oracle in the tests.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Dict, List, Optional

import numpy as np

from .scene.model import Light, Scene

MESH_DESC_FIELDS = ("vbase", "tbase", "ntris", "uvbase", "has_uv", "material")

# exposure mapping the reference's light intensities to unit-range shading:
# dome 500 x (0.75,0.85,1.0) (generate_construction_data.py:1320-1323) and the
# distant light clamped to 1500 (:1341-1342).
EXPOSURE = 1.0 / 1925.0

MATERIAL_DTYPE = np.dtype([("base", "u1", 4), ("texture", "<i4"), ("alpha_test", "<u4"),
                           ("alpha_threshold", "<u4")])
TEXTURE_DTYPE = np.dtype([("offset", "<u4"), ("width", "<u4"), ("height", "<u4"), ("pad", "<u4")])


@dataclass
class PackedScene:
    positions: np.ndarray      # [V,3] f32
    tris: np.ndarray           # [T,3] u32 (mesh relative)
    uvs: np.ndarray            # [U,2] f32
    uv_tris: np.ndarray        # [T,3] u32 (mesh relative)
    meshes: np.ndarray         # [M,6] u32
    materials: np.ndarray      # [Mat] MATERIAL_DTYPE
    texels: np.ndarray         # [N*4] u8
    textures: np.ndarray       # [Tex] TEXTURE_DTYPE
    inst_model: np.ndarray     # [I,16] f32
    inst_mesh: np.ndarray      # [I] u32
    inst_label: np.ndarray     # [I] i32
    inst_tri_base: np.ndarray  # [I+1] u32
    ambient: np.ndarray        # [3] f32
    sun: np.ndarray            # [3] f32
    sun_dir: np.ndarray        # [3] f32
    sky: np.ndarray            # [4] u8
    n_labels: int

    @property
    def n_tris(self) -> int:
        return int(self.inst_tri_base[-1])


def light_constants(light: Light):
    amb = (light.dome_color * light.dome_intensity * EXPOSURE).astype(np.float32)
    sun = (light.sun_color * light.sun_intensity * EXPOSURE).astype(np.float32)
    d = np.asarray(light.sun_dir, np.float64)
    d = (d / np.linalg.norm(d)).astype(np.float32)
    sky = np.concatenate([np.clip(np.round(light.dome_color * 255.0), 0, 255), [255]]).astype(np.uint8)
    return amb, sun, d, sky


def pack_models(models: List[np.ndarray]) -> np.ndarray:
    return np.stack([np.asarray(m, np.float64).reshape(4, 4) for m in models]).astype(np.float32).reshape(-1, 16)


def pack_scene(scene: Scene, instance_models: Optional[List[np.ndarray]] = None) -> PackedScene:
    pos, tri, uv, uvt, md = [], [], [], [], []
    vb = tb = ub = 0
    for m in scene.meshes:
        has_uv = int(m.uvs.shape[0] > 0 and m.uv_tris.shape[0] == m.n_tris)
        md.append((vb, tb, m.n_tris, ub, has_uv, m.material))
        pos.append(m.positions.astype(np.float32))
        tri.append(m.tris.astype(np.uint32))
        if has_uv:
            uv.append(m.uvs.astype(np.float32))
            uvt.append(m.uv_tris.astype(np.uint32))
        else:
            uvt.append(np.zeros((m.n_tris, 3), np.uint32))
        vb += m.positions.shape[0]
        tb += m.n_tris
        ub += m.uvs.shape[0] if has_uv else 0
    mats = np.zeros(len(scene.materials), MATERIAL_DTYPE)
    for k, mt in enumerate(scene.materials):
        mats[k]["base"][:3] = np.clip(np.round(np.asarray(mt.base_color) * 255.0), 0, 255)
        mats[k]["base"][3] = 255
        mats[k]["texture"] = mt.texture
        mats[k]["alpha_test"] = int(mt.alpha_test)
        mats[k]["alpha_threshold"] = mt.alpha_threshold
    texd = np.zeros(len(scene.textures), TEXTURE_DTYPE)
    blobs, off = [], 0
    for k, t in enumerate(scene.textures):
        h, w = t.rgba.shape[:2]
        texd[k] = (off, w, h, 0)
        blobs.append(np.ascontiguousarray(t.rgba, np.uint8).reshape(-1))
        off += w * h
    models = instance_models if instance_models is not None else [i.model for i in scene.instances]
    counts = np.array([scene.meshes[i.mesh].n_tris for i in scene.instances], np.int64)
    base = np.concatenate([[0], np.cumsum(counts)]).astype(np.uint32)
    amb, sun, d, sky = light_constants(scene.light)
    n_labels = max([o.inst_idx for o in scene.objects] + [i.inst_idx for i in scene.instances] + [-1]) + 1
    return PackedScene(
        positions=np.concatenate(pos) if pos else np.zeros((0, 3), np.float32),
        tris=np.concatenate(tri) if tri else np.zeros((0, 3), np.uint32),
        uvs=np.concatenate(uv) if uv else np.zeros((1, 2), np.float32),
        uv_tris=np.concatenate(uvt) if uvt else np.zeros((0, 3), np.uint32),
        meshes=np.array(md, np.uint32).reshape(-1, 6),
        materials=mats,
        texels=np.concatenate(blobs) if blobs else np.zeros(4, np.uint8),
        textures=texd,
        inst_model=pack_models(models),
        inst_mesh=np.array([i.mesh for i in scene.instances], np.uint32),
        inst_label=np.array([i.inst_idx for i in scene.instances], np.int32),
        inst_tri_base=base,
        ambient=amb, sun=sun, sun_dir=d, sky=sky, n_labels=n_labels,
    )
