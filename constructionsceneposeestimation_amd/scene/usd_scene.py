"""Build a :class:`Scene` from a USD crate layer.

Host-side replacement for what the reference gets from Kit's stage
(generate_construction_data.py:1370) plus its identity aggregation
(:1857-1891): traverse defined prims, compose xform ops, triangulate meshes,
resolve material bindings and group meshes into labelled object roots via
:func:`identity.get_object_root`.

Meshes that resolve to the same object root, share a material and a world
transform are merged into one mesh (the 45 sub-meshes of a fence panel);
merged meshes whose source arrays are identical on disk (the crate
de-duplicates values) are stored once and instanced.
"""
from __future__ import annotations

import os
from typing import Dict, List, Optional, Tuple

import numpy as np

from .. import identity
from . import xform as X
from .model import Instance, Light, Material, Mesh, Scene, SceneObject, Texture
from .usdc import CrateFile


def _local_matrix(c: CrateFile, prim: str) -> np.ndarray:
    order = c.attr(prim, "xformOpOrder", None)
    m = np.eye(4)
    if not order:
        return m
    for op in order:
        if op == "!resetXformStack!":
            m = np.eye(4)
            continue
        inv = op.startswith("!invert!")
        name = op[len("!invert!"):] if inv else op
        v = c.attr(prim, name, None)
        if v is None:
            continue
        kind = name.split(":")[1]
        if kind == "translate":
            o = X.translate(v)
        elif kind == "scale":
            o = X.scale(np.broadcast_to(np.asarray(v, np.float64), (3,)))
        elif kind == "orient":
            o = X.rotate_quat(v)
        elif kind == "rotateXYZ":
            o = X.rotate_xyz(v)
        elif kind in ("rotateX", "rotateY", "rotateZ"):
            o = {"rotateX": X.rot_x, "rotateY": X.rot_y, "rotateZ": X.rot_z}[kind](float(v))
        elif kind == "transform":
            o = X.from_usd_matrix(v)
        else:
            raise NotImplementedError(f"xform op {op} on {prim}")
        m = m @ (np.linalg.inv(o) if inv else o)
    return m


def _triangulate(counts: np.ndarray, fvi: np.ndarray) -> Tuple[np.ndarray, np.ndarray]:
    """Fan-triangulate; returns (position index tris, face-vertex corner tris)."""
    counts = counts.astype(np.int64)
    starts = np.concatenate([[0], np.cumsum(counts)[:-1]])
    tri_pos, tri_fv = [], []
    if counts.size and np.all(counts == 3):
        corners = np.arange(counts.size * 3).reshape(-1, 3)
        return fvi[corners].astype(np.int64), corners
    for s, n in zip(starts.tolist(), counts.tolist()):
        for k in range(1, n - 1):
            tri_fv.append((s, s + k, s + k + 1))
    tri_fv = np.array(tri_fv, np.int64).reshape(-1, 3)
    return fvi[tri_fv].astype(np.int64), tri_fv


def _mesh_arrays(c: CrateFile, prim: str):
    pts = c.attr(prim, "points")
    counts = c.attr(prim, "faceVertexCounts")
    fvi = c.attr(prim, "faceVertexIndices")
    if pts is None or counts is None or fvi is None or len(pts) == 0:
        return None
    pts = np.asarray(pts, np.float32).reshape(-1, 3)
    tri_pos, tri_fv = _triangulate(np.asarray(counts), np.asarray(fvi, np.int64))
    st = c.attr(prim, "primvars:st")
    uvs = np.zeros((0, 2), np.float32)
    uv_tris = np.zeros((0, 3), np.int64)
    if st is not None and len(st):
        uvs = np.asarray(st, np.float32).reshape(-1, 2)
        interp = c.field(prim + ".primvars:st", "interpolation", "vertex")
        base = tri_fv if interp == "faceVarying" else tri_pos
        sti = c.attr(prim, "primvars:st:indices")
        uv_tris = np.asarray(sti, np.int64)[base] if sti is not None and len(sti) else base
    key = tuple(c.rep(prim, n) for n in ("points", "faceVertexCounts", "faceVertexIndices",
                                          "primvars:st", "primvars:st:indices"))
    return pts, tri_pos, uvs, uv_tris, key


def _binding(c: CrateFile, prim: str) -> Optional[str]:
    b = c.field(prim + ".material:binding", "targetPaths")
    if isinstance(b, dict):
        items = b.get("explicitItems") or b.get("prependedItems") or b.get("appendedItems")
        if items:
            return items[0]
    return None


# Stand-ins for authored textures that live outside the repository
# (bark_0004.jpg / DB2X2_L01.png are referenced by absolute
# download paths; the cone texture is a missing LFS blob).
TEXTURE_STANDINS = {
    "bark_0004.jpg": "textures/BarkDecidious0107_M.jpg",
    "DB2X2_L01.png": "textures/Branches0018_1_S.png",
}

# Materials whose Material prims are not in this layer (they live in
# referenced/LFS assets): constant albedo from the reference's own data.
FALLBACK_COLORS = {
    "fence": (0.3057, 0.3057, 0.3057),      # cad_models/Fence/...height-2.mtl:2-4 (Kd)
    "trafficcone": (0.95, 0.35, 0.05),      # texture 'Traffic Cone UV Fixed.png' missing
    "ground": (0.5, 0.5, 0.5),              # CollisionMesh primvars:displayColor
}


def _material_for(c: CrateFile, mat_path: Optional[str], class_name: Optional[str],
                  textures: Dict[str, int], tex_loader) -> Tuple[str, Material]:
    if mat_path and c.prim_type(mat_path) == "Material":
        shaders = [k for k in c.children(mat_path) if c.prim_type(k) == "Shader"]
        sh = shaders[0] if shaders else None
        if sh:
            col = c.attr(sh, "inputs:diffuse_color_constant", (1.0, 1.0, 1.0))
            tex = c.attr(sh, "inputs:diffuse_texture", None)
            op_tex = c.attr(sh, "inputs:opacity_texture", None)
            alpha = bool(c.attr(sh, "inputs:enable_opacity", False)) and bool(
                c.attr(sh, "inputs:enable_opacity_texture", False)) and op_tex is not None
            thr = float(c.attr(sh, "inputs:opacity_threshold", 0.0) or 0.0)
            tid = -1
            if tex:
                base = os.path.basename(str(tex))
                tid = tex_loader(base)
            name = mat_path.rstrip("/").split("/")[-1]
            return name, Material(name, np.asarray(col, np.float64), tid, alpha, int(round(thr * 255)))
    key = class_name if class_name in FALLBACK_COLORS else "ground"
    return "flat_" + key, Material("flat_" + key, np.array(FALLBACK_COLORS[key]), -1, False, 0)


def _sun_from_light(c: CrateFile, path: str) -> Tuple[np.ndarray, float]:
    m = np.eye(4)
    chain = []
    p = path
    while p and p != "/":
        chain.append(p)
        p = p.rsplit("/", 1)[0] or "/"
    for q in reversed(chain):
        m = m @ _local_matrix(c, q)
    d = -m[:3, 2]                      # distant light emits along its local -Z
    to_sun = -d / np.linalg.norm(d)
    inten = float(c.attr(path, "inputs:intensity", 3000.0) or 3000.0)
    # setup_scene_lighting clamps distant lights above 2000 to 1500
    # (generate_construction_data.py:1336-1345).
    if inten > 2000:
        inten = 1500.0
    return to_sun, inten


def load_crate_scene(path: str, texture_root: Optional[str] = None, max_texture: int = 1024) -> Scene:
    c = CrateFile(path)
    scene = Scene()
    tex_index: Dict[str, int] = {}

    def tex_loader(base: str) -> int:
        if base in tex_index:
            return tex_index[base]
        rel = TEXTURE_STANDINS.get(base)
        if rel is None or texture_root is None or not os.path.exists(os.path.join(texture_root, rel)):
            tex_index[base] = -1
            return -1
        from PIL import Image
        im = Image.open(os.path.join(texture_root, rel)).convert("RGBA")
        if max(im.size) > max_texture:
            r = max_texture / max(im.size)
            im = im.resize((max(1, round(im.size[0] * r)), max(1, round(im.size[1] * r))), Image.LANCZOS)
        scene.textures.append(Texture(os.path.basename(rel), np.asarray(im, np.uint8).copy()))
        tex_index[base] = len(scene.textures) - 1
        return tex_index[base]

    # traverse defined prims depth-first in authored order
    mesh_recs = []                       # (path, world matrix)
    world: Dict[str, np.ndarray] = {"/": np.eye(4)}
    light_paths = []
    stack = [("/", np.eye(4))]
    while stack:
        p, parent = stack.pop()
        kids = c.children(p)
        for k in reversed(kids):
            if c.field(k, "specifier") != 0:          # skip 'over'/'class' (LFS-only geometry)
                continue
            if c.field(k, "active") is False:
                continue
            m = parent @ _local_matrix(c, k)
            world[k] = m
            t = c.prim_type(k)
            if t == "Mesh":
                mesh_recs.append((k, m))
            elif t == "DistantLight":
                light_paths.append(k)
            stack.append((k, m))
    # stack pops reverse-pushed children -> authored depth-first order preserved
    mesh_paths = [p for p, _ in mesh_recs]
    inst_of_mesh, objects = identity.assign_instances(mesh_paths)
    for o in objects:
        scene.objects.append(SceneObject(o["prim_path"], o["class_name"], o["class_id"], o["inst_idx"],
                                         kind=o["class_name"] if o["class_name"] in ("trafficcone",) else "static"))

    materials: Dict[str, int] = {}
    groups: Dict[tuple, dict] = {}
    for (p, m), inst_idx in zip(mesh_recs, inst_of_mesh):
        arr = _mesh_arrays(c, p)
        if arr is None:
            continue
        cls = scene.objects[inst_idx].class_name if inst_idx >= 0 else None
        mname, mat = _material_for(c, _binding(c, p), cls, tex_index, tex_loader)
        if mname not in materials:
            scene.materials.append(mat)
            materials[mname] = len(scene.materials) - 1
        root = scene.objects[inst_idx].prim_path if inst_idx >= 0 else p
        gkey = (root, materials[mname], m.round(9).tobytes())
        g = groups.setdefault(gkey, {"model": m, "inst_idx": inst_idx, "parts": [], "mat": materials[mname]})
        g["parts"].append((p, arr))

    mesh_ids: Dict[tuple, int] = {}
    for (root, mat, _), g in groups.items():
        key = (mat,) + tuple(a[4] for _, a in g["parts"])
        if key not in mesh_ids:
            pos, tri, uv, uvt = [], [], [], []
            vo = uo = 0
            any_uv = any(a[2].shape[0] for _, a in g["parts"])
            for _, (pts, tp, uvs, ut, _) in g["parts"]:
                pos.append(pts)
                tri.append(tp + vo)
                if any_uv:
                    if uvs.shape[0]:
                        uv.append(uvs)
                        uvt.append(ut + uo)
                        uo += uvs.shape[0]
                    else:
                        uv.append(np.zeros((1, 2), np.float32))
                        uvt.append(np.full_like(tp, uo))
                        uo += 1
                vo += pts.shape[0]
            name = g["parts"][0][0] if len(g["parts"]) == 1 else root + "#merged"
            scene.meshes.append(Mesh(
                name, np.concatenate(pos).astype(np.float32), np.concatenate(tri).astype(np.uint32),
                np.concatenate(uv).astype(np.float32) if uv else np.zeros((0, 2), np.float32),
                np.concatenate(uvt).astype(np.uint32) if uvt else np.zeros((0, 3), np.uint32), mat))
            mesh_ids[key] = len(scene.meshes) - 1
        obj = g["inst_idx"]
        scene.instances.append(Instance(mesh_ids[key], g["model"], obj, obj))

    # per-object local frame = world transform of the object root prim
    for o in scene.objects:
        root = o.prim_path.split("#")[0]
        frame = world.get(root, np.eye(4))
        lo, hi = np.full(3, np.inf), np.full(3, -np.inf)
        for inst in scene.instances:
            if inst.obj == o.inst_idx:
                inst.local = np.linalg.solve(frame, inst.model)
                pts = scene.meshes[inst.mesh].positions.astype(np.float64)
                lp = X.transform_points(inst.local, pts)
                lo, hi = np.minimum(lo, lp.min(0)), np.maximum(hi, lp.max(0))
        o.local_bounds = np.stack([lo, hi])
        scene.meta.setdefault("object_frames", {})[o.prim_path] = frame.tolist()

    if light_paths:
        d, inten = _sun_from_light(c, light_paths[0])
        scene.light = Light(sun_dir=d, sun_intensity=inten)
    scene.meta.update({
        "source": os.path.basename(path), "crate_version": list(c.version),
        "upAxis": c.field("/", "upAxis"), "metersPerUnit": c.field("/", "metersPerUnit"),
        "n_mesh_prims": len(mesh_recs), "n_objects": len(scene.objects),
    })
    return scene
