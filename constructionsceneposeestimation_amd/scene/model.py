"""In-memory scene: unique meshes, materials, textures, instances, objects.

This is the host-side scene the GPU renderer consumes (the role the USD
stage plays for the reference: ``usd.get_context().get_stage()``,
generate_construction_data.py:1370).  Geometry is stored once per unique
mesh and referenced by instances (model matrix + identity), which is how the
crate file itself stores the 23 fences and 11 trees of world2 (values are
de-duplicated on disk).

Conventions (fixed for GPU and oracle alike):
* world space: USD stage space, Z up, metres (world2: ``upAxis = Z``,
  ``metersPerUnit = 1``);
* matrices: float64 4x4, column-vector convention ``p_world = M @ [p, 1]``;
* UVs: USD ``st`` (v = 0 at the bottom of the image).
"""
from __future__ import annotations

import io
import json
from dataclasses import dataclass, field
from typing import Dict, List, Optional

import numpy as np


@dataclass
class Mesh:
    name: str
    positions: np.ndarray            # (V,3) float32
    tris: np.ndarray                 # (T,3) uint32 -> positions
    uvs: np.ndarray                  # (U,2) float32, may be (0,2)
    uv_tris: np.ndarray              # (T,3) uint32 -> uvs, or (0,3) when no uvs
    material: int = 0

    @property
    def n_tris(self) -> int:
        return int(self.tris.shape[0])


@dataclass
class Material:
    name: str
    base_color: np.ndarray           # (3,) float in [0,1]; multiplies the texture
    texture: int = -1                # index into Scene.textures, -1 = none
    alpha_test: bool = False         # OmniPBR_Opacity with an opacity texture
    alpha_threshold: int = 0         # fragment kept iff alpha8 > threshold


@dataclass
class Texture:
    name: str
    rgba: np.ndarray                 # (H,W,4) uint8


@dataclass
class SceneObject:
    """A labelled object root (one ``inst_idx``)."""
    prim_path: str
    class_name: str
    class_id: int
    inst_idx: int
    kind: str = "static"             # crane | dumper | human | trafficcone | static
    local_bounds: Optional[np.ndarray] = None   # (2,3) float64 in the object's frame


@dataclass
class Instance:
    mesh: int
    model: np.ndarray                # (4,4) float64 world transform of the mesh
    inst_idx: int = -1               # -1: background (unlabelled)
    obj: int = -1                    # index into Scene.objects
    local: Optional[np.ndarray] = None  # (4,4) mesh transform relative to its object frame


@dataclass
class Light:
    sun_dir: np.ndarray = field(default_factory=lambda: np.array([0.3, 0.2, 0.93]))  # unit, toward the sun
    sun_intensity: float = 1500.0
    sun_color: np.ndarray = field(default_factory=lambda: np.ones(3))
    dome_intensity: float = 500.0
    dome_color: np.ndarray = field(default_factory=lambda: np.array([0.75, 0.85, 1.0]))


@dataclass
class Scene:
    meshes: List[Mesh] = field(default_factory=list)
    materials: List[Material] = field(default_factory=list)
    textures: List[Texture] = field(default_factory=list)
    instances: List[Instance] = field(default_factory=list)
    objects: List[SceneObject] = field(default_factory=list)
    light: Light = field(default_factory=Light)
    keypoints: Dict[str, np.ndarray] = field(default_factory=dict)
    meta: Dict[str, object] = field(default_factory=dict)

    # -- stats ---------------------------------------------------------------
    @property
    def n_tris_per_frame(self) -> int:
        return int(sum(self.meshes[i.mesh].n_tris for i in self.instances))

    def authored_bytes(self) -> int:
        """B_geom of SURVEY §8(d): authored arrays read once per frame when
        every instance is flattened (12 B/vertex, 12 B/tri, 8 B/uv, 12 B/uv-tri)."""
        b = 0
        for inst in self.instances:
            m = self.meshes[inst.mesh]
            b += 12 * m.positions.shape[0] + 12 * m.n_tris + 8 * m.uvs.shape[0] + 12 * m.uv_tris.shape[0]
        return b

    def texture_bytes(self) -> int:
        return int(sum(t.rgba.nbytes for t in self.textures))

    # -- (de)serialisation --------------------------------------------------
    def save_npz(self, path: str) -> None:
        arrs: Dict[str, np.ndarray] = {}
        meta = {
            "meshes": [], "materials": [], "textures": [], "instances": [], "objects": [],
            "light": {
                "sun_dir": self.light.sun_dir.tolist(), "sun_intensity": self.light.sun_intensity,
                "sun_color": self.light.sun_color.tolist(), "dome_intensity": self.light.dome_intensity,
                "dome_color": self.light.dome_color.tolist(),
            },
            "meta": self.meta,
            "keypoints": list(self.keypoints),
        }
        for i, m in enumerate(self.meshes):
            meta["meshes"].append({"name": m.name, "material": m.material})
            arrs[f"m{i}_pos"] = m.positions.astype(np.float32)
            arrs[f"m{i}_tri"] = m.tris.astype(np.uint32)
            arrs[f"m{i}_uv"] = m.uvs.astype(np.float32)
            arrs[f"m{i}_uvtri"] = m.uv_tris.astype(np.uint32)
        for mt in self.materials:
            meta["materials"].append({"name": mt.name, "base_color": list(map(float, mt.base_color)),
                                      "texture": mt.texture, "alpha_test": mt.alpha_test,
                                      "alpha_threshold": mt.alpha_threshold})
        for i, t in enumerate(self.textures):
            meta["textures"].append({"name": t.name})
            arrs[f"t{i}"] = t.rgba
        models = np.stack([inst.model for inst in self.instances]) if self.instances else np.zeros((0, 4, 4))
        arrs["inst_model"] = models
        locs = [inst.local if inst.local is not None else np.eye(4) for inst in self.instances]
        arrs["inst_local"] = np.stack(locs) if locs else np.zeros((0, 4, 4))
        for inst in self.instances:
            meta["instances"].append({"mesh": inst.mesh, "inst_idx": inst.inst_idx, "obj": inst.obj})
        for j, o in enumerate(self.objects):
            meta["objects"].append({"prim_path": o.prim_path, "class_name": o.class_name,
                                    "class_id": o.class_id, "inst_idx": o.inst_idx, "kind": o.kind})
            if o.local_bounds is not None:
                arrs[f"o{j}_bounds"] = o.local_bounds
        for k, v in self.keypoints.items():
            arrs[f"kp_{k}"] = v
        arrs["meta_json"] = np.frombuffer(json.dumps(meta).encode(), np.uint8)
        np.savez_compressed(path, **arrs)

    @staticmethod
    def load_npz(path: str) -> "Scene":
        z = np.load(path, allow_pickle=False)
        meta = json.loads(bytes(z["meta_json"]).decode())
        s = Scene()
        for i, m in enumerate(meta["meshes"]):
            s.meshes.append(Mesh(m["name"], z[f"m{i}_pos"], z[f"m{i}_tri"], z[f"m{i}_uv"].reshape(-1, 2),
                                 z[f"m{i}_uvtri"].reshape(-1, 3), m["material"]))
        for mt in meta["materials"]:
            s.materials.append(Material(mt["name"], np.array(mt["base_color"]), mt["texture"],
                                        mt["alpha_test"], mt["alpha_threshold"]))
        for i, t in enumerate(meta["textures"]):
            s.textures.append(Texture(t["name"], z[f"t{i}"]))
        for k, inst in enumerate(meta["instances"]):
            s.instances.append(Instance(inst["mesh"], z["inst_model"][k], inst["inst_idx"], inst["obj"],
                                        z["inst_local"][k]))
        for j, o in enumerate(meta["objects"]):
            b = z[f"o{j}_bounds"] if f"o{j}_bounds" in z.files else None
            s.objects.append(SceneObject(o["prim_path"], o["class_name"], o["class_id"], o["inst_idx"],
                                         o["kind"], b))
        L = meta["light"]
        s.light = Light(np.array(L["sun_dir"]), L["sun_intensity"], np.array(L["sun_color"]),
                        L["dome_intensity"], np.array(L["dome_color"]))
        s.meta = meta.get("meta", {})
        for k in meta.get("keypoints", []):
            s.keypoints[k] = z[f"kp_{k}"]
        return s
