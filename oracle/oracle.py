"""ctypes front-end of the CPU oracle — TEST INFRASTRUCTURE ONLY.

Loaded by tests/, ``__graft_entry__.smoke()`` and bench.py's cpu_baseline
leg, as the checker.  The product path (``constructionsceneposeestimation_amd``)
never imports this module.  Render parity against the reference's RTX
renderer is unpinned (closed, absent); see csg_oracle.h.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess
from typing import Optional

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "_build", "liboracle.so")


class _Scene(C.Structure):
    _fields_ = [
        ("positions", C.c_void_p), ("tris", C.c_void_p), ("uvs", C.c_void_p), ("uv_tris", C.c_void_p),
        ("meshes", C.c_void_p), ("n_meshes", C.c_uint32),
        ("inst_model", C.c_void_p), ("inst_mesh", C.c_void_p), ("inst_label", C.c_void_p),
        ("inst_tri_base", C.c_void_p), ("n_inst", C.c_uint32),
        ("materials", C.c_void_p), ("n_materials", C.c_uint32),
        ("texels", C.c_void_p), ("textures", C.c_void_p), ("n_textures", C.c_uint32),
        ("ambient", C.c_float * 3), ("sun", C.c_float * 3), ("sun_dir", C.c_float * 3),
        ("sky", C.c_uint8 * 4),
        ("width", C.c_uint32), ("height", C.c_uint32),
        ("near_clip", C.c_float), ("far_clip", C.c_float),
    ]


class _Stats(C.Structure):
    _fields_ = [(n, C.c_uint64) for n in ("n_tris_in", "n_culled", "n_clipped", "n_raster_tris",
                                           "n_fragments", "n_alpha_killed", "n_bbox_pixels", "n_covered",
                                           "n_early_z_killed", "n_alpha_tests")]


def build() -> str:
    if not os.path.exists(_LIB_PATH) or os.path.getmtime(_LIB_PATH) < max(
            os.path.getmtime(os.path.join(_HERE, f)) for f in ("csg_oracle.c", "csg_oracle.h")):
        subprocess.run(["make", "-s", "-C", _HERE], check=True)
    return _LIB_PATH


_lib = None


def lib():
    global _lib
    if _lib is None:
        _lib = C.CDLL(build())
        vp, u32 = C.c_void_p, C.c_uint32
        _lib.oracle_render_frame.argtypes = [C.POINTER(_Scene), vp, vp, vp, vp, vp, vp, u32, C.POINTER(_Stats)]
        _lib.oracle_render_frame_ex.argtypes = [C.POINTER(_Scene), vp, vp, vp, vp, vp, vp, vp, vp, u32,
                                                C.POINTER(_Stats)]
        _lib.oracle_render_frame_cov.argtypes = [C.POINTER(_Scene), vp, vp, vp, vp, vp, vp, vp, vp, vp, u32,
                                                 C.POINTER(_Stats)]
        _lib.oracle_keypoints.argtypes = [C.POINTER(_Scene), vp, vp, vp, u32, vp, vp, vp]
        _lib.oracle_render_frames.argtypes = [C.POINTER(_Scene), vp, vp, u32, vp, vp, vp, vp, C.c_int]
        _lib.oracle_mat4_mul.argtypes = [vp, vp, vp]
    return _lib


def _ptr(a: Optional[np.ndarray]):
    return None if a is None else a.ctypes.data


class Oracle:
    """Holds a packed scene (see ``packing.PackedScene``) and renders frames."""

    def __init__(self, packed, width: int, height: int, near: float = 0.5, far: float = 250.0):
        self.p = packed
        self.width, self.height = width, height
        self._keep = []
        s = _Scene()

        def arr(a, dt):
            a = np.ascontiguousarray(a, dt)
            self._keep.append(a)
            return a.ctypes.data

        s.positions = arr(packed.positions, np.float32)
        s.tris = arr(packed.tris, np.uint32)
        s.uvs = arr(packed.uvs, np.float32)
        s.uv_tris = arr(packed.uv_tris, np.uint32)
        s.meshes = arr(packed.meshes, np.uint32)
        s.n_meshes = packed.meshes.shape[0]
        s.inst_model = arr(packed.inst_model, np.float32)
        s.inst_mesh = arr(packed.inst_mesh, np.uint32)
        s.inst_label = arr(packed.inst_label, np.int32)
        s.inst_tri_base = arr(packed.inst_tri_base, np.uint32)
        s.n_inst = packed.inst_mesh.shape[0]
        mats = np.ascontiguousarray(packed.materials)
        self._keep.append(mats)
        s.materials = mats.ctypes.data
        s.n_materials = mats.shape[0]
        s.texels = arr(packed.texels, np.uint8)
        texd = np.ascontiguousarray(packed.textures)
        self._keep.append(texd)
        s.textures = texd.ctypes.data
        s.n_textures = texd.shape[0]
        s.ambient[:] = [float(x) for x in packed.ambient]
        s.sun[:] = [float(x) for x in packed.sun]
        s.sun_dir[:] = [float(x) for x in packed.sun_dir]
        s.sky[:] = [int(x) for x in packed.sky]
        s.width, s.height = width, height
        s.near_clip, s.far_clip = near, far
        self.s = s

    def set_light(self, light) -> None:
        """Lighting for the following renders (a ``scene.model.Light``)."""
        from constructionsceneposeestimation_amd.packing import light_constants
        amb, sun, d, sky = light_constants(light)
        self.s.ambient[:] = [float(x) for x in amb]
        self.s.sun[:] = [float(x) for x in sun]
        self.s.sun_dir[:] = [float(x) for x in d]
        self.s.sky[:] = [int(x) for x in sky]

    def set_material_textures(self, texture_per_material) -> None:
        """Texture of each material for the following renders (-2 = keep)."""
        mats = np.array(self.p.materials, copy=True)
        for m, t in enumerate(texture_per_material):
            if int(t) != -2:
                mats["texture"][m] = int(t)
        self._keep.append(mats)
        self.s.materials = mats.ctypes.data

    def set_instance_models(self, models16: np.ndarray) -> None:
        a = np.ascontiguousarray(models16, np.float32).reshape(-1, 16)
        assert a.shape[0] == self.s.n_inst
        self._keep.append(a)
        self.s.inst_model = a.ctypes.data

    def render(self, view: np.ndarray, proj: np.ndarray, want_stats: bool = False, extra: bool = False,
               covered: bool = False):
        """One frame; ``extra`` adds the C5 outputs ``normals`` (H,W,3 float16)
        and ``points`` (H,W,3 float32 world xyz, NaN where nothing is hit);
        ``covered`` adds ``label_covered`` (n_labels,) uint32, the occlusion
        coverage (csg_outputs.label_covered)."""
        H, W = self.height, self.width
        rgb = np.empty((H, W, 3), np.uint8)
        inst = np.empty((H, W), np.int32)
        depth = np.empty((H, W), np.float32)
        normals = np.empty((H, W, 3), np.float16) if extra else None
        points = np.empty((H, W, 3), np.float32) if extra else None
        nl = max(int(self.p.n_labels), 1)
        stats = np.empty((nl, 5), np.uint32)
        st = _Stats()
        v = np.ascontiguousarray(view, np.float32).reshape(16)
        pr = np.ascontiguousarray(proj, np.float32).reshape(16)
        cov = np.empty(nl, np.uint32) if covered else None
        rc = lib().oracle_render_frame_cov(C.byref(self.s), _ptr(v), _ptr(pr), _ptr(rgb), _ptr(inst), _ptr(depth),
                                           _ptr(normals), _ptr(points), _ptr(stats), _ptr(cov), nl, C.byref(st))
        if rc != 0:
            raise RuntimeError(f"oracle_render_frame failed: {rc}")
        out = {"rgb": rgb, "instance": inst, "depth": depth, "inst_stats": stats}
        if covered:
            out["label_covered"] = cov
        if extra:
            out["normals"], out["points"] = normals, points
        if want_stats:
            out["stats"] = {n: int(getattr(st, n)) for n, _ in _Stats._fields_}
        return out

    def frame_state(self, models16: Optional[np.ndarray] = None, light=None, texture_per_material=None) -> "Oracle":
        """A shallow copy that renders with its own instance models, light and
        material textures (the scene arrays are shared): one per frame of a
        DR batch, so frames of different epochs can render on parallel threads."""
        o = Oracle.__new__(Oracle)
        o.p, o.width, o.height = self.p, self.width, self.height
        o._keep = list(self._keep)
        o.s = _Scene()
        C.memmove(C.addressof(o.s), C.addressof(self.s), C.sizeof(_Scene))
        if models16 is not None:
            o.set_instance_models(models16)
        if light is not None:
            o.set_light(light)
        if texture_per_material is not None:
            o.set_material_textures(texture_per_material)
        return o

    def render_parallel(self, jobs, threads: int, extra: bool = False):
        """Render ``jobs`` = [(oracle_state, view, proj)] on ``threads`` Python
        threads (each ctypes call releases the GIL; oracle_render_frame_cov is
        reentrant); returns the per-frame output dicts in order."""
        from concurrent.futures import ThreadPoolExecutor
        if threads <= 1:
            return [o.render(v, p, extra=extra) for o, v, p in jobs]
        with ThreadPoolExecutor(max_workers=threads) as ex:
            return list(ex.map(lambda j: j[0].render(j[1], j[2], extra=extra), jobs))

    def keypoints(self, view, proj, pts: np.ndarray, depth: np.ndarray):
        pts = np.ascontiguousarray(pts, np.float32).reshape(-1, 3)
        uv = np.empty((pts.shape[0], 2), np.float32)
        vis = np.empty(pts.shape[0], np.int32)
        v = np.ascontiguousarray(view, np.float32).reshape(16)
        pr = np.ascontiguousarray(proj, np.float32).reshape(16)
        d = None if depth is None else np.ascontiguousarray(depth, np.float32)   # None: no depth test
        lib().oracle_keypoints(C.byref(self.s), _ptr(v), _ptr(pr), _ptr(pts), pts.shape[0], _ptr(d),
                               _ptr(uv), _ptr(vis))
        return uv, vis

    def render_many(self, views: np.ndarray, projs: np.ndarray, threads: int = 1, outputs: bool = True,
                    models: Optional[np.ndarray] = None):
        """Render frames in parallel; ``models`` = optional per-frame [n][I][16] instance transforms."""
        n = views.shape[0]
        H, W = self.height, self.width
        rgb = np.empty((n, H, W, 3), np.uint8) if outputs else None
        inst = np.empty((n, H, W), np.int32) if outputs else None
        depth = np.empty((n, H, W), np.float32) if outputs else None
        v = np.ascontiguousarray(views, np.float32).reshape(n, 16)
        pr = np.ascontiguousarray(projs, np.float32).reshape(n, 16)
        m = None if models is None else np.ascontiguousarray(models, np.float32).reshape(n, -1)
        rc = lib().oracle_render_frames(C.byref(self.s), _ptr(v), _ptr(pr), n, _ptr(m), _ptr(rgb), _ptr(inst),
                                        _ptr(depth), threads)
        if rc != 0:
            raise RuntimeError("oracle_render_frames failed")
        return rgb, inst, depth


def mat4_mul_f32(a: np.ndarray, b: np.ndarray) -> np.ndarray:
    a = np.ascontiguousarray(a, np.float32).reshape(16)
    b = np.ascontiguousarray(b, np.float32).reshape(16)
    c = np.empty(16, np.float32)
    lib().oracle_mat4_mul(_ptr(a), _ptr(b), _ptr(c))
    return c.reshape(4, 4)


# ---------------------------------------------------------------------------
# Depth visualisation (generate_construction_data.py:1690-1709), restated in
# NumPy with the promotion rules of NumPy 1.x, the version Isaac Sim ships:
# ``depth_max - depth_min + 1e-6`` is a float64 scalar there (a float32 scalar
# plus a Python float), and dividing the float32 array by it casts it back to
# float32.  ``cv2.applyColorMap(..., COLORMAP_JET)`` is restated as the GNU
# Octave jet map OpenCV documents, sampled at k/255, stored as float32, scaled
# by 255 in float32 and rounded half to even (OpenCV is absent here: the table
# is unpinned against cv2).
# ---------------------------------------------------------------------------
def jet_lut() -> np.ndarray:
    """(256, 3) uint8 RGB."""
    x = np.arange(256, dtype=np.float64) / 255.0
    r = np.where((x >= 3 / 8) & (x < 5 / 8), 4 * x - 1.5,
                 np.where((x >= 5 / 8) & (x < 7 / 8), 1.0, np.where(x >= 7 / 8, -4 * x + 4.5, 0.0)))
    g = np.where((x >= 1 / 8) & (x < 3 / 8), 4 * x - 0.5,
                 np.where((x >= 3 / 8) & (x < 5 / 8), 1.0, np.where((x >= 5 / 8) & (x < 7 / 8), -4 * x + 3.5, 0.0)))
    b = np.where(x < 1 / 8, 4 * x + 0.5,
                 np.where((x >= 1 / 8) & (x < 3 / 8), 1.0, np.where((x >= 3 / 8) & (x < 5 / 8), -4 * x + 2.5, 0.0)))
    lut = np.stack([r, g, b], 1).astype(np.float32) * np.float32(255.0)
    return np.clip(np.rint(lut), 0, 255).astype(np.uint8)


def depth_vis(depth: np.ndarray):
    """(H, W, 3) uint8 RGB JET image and (min, max) of one depth map."""
    depth = np.asarray(depth, np.float32)
    mask = np.isfinite(depth) & (depth > 0)
    if not mask.any():
        return np.zeros(depth.shape + (3,), np.uint8), (float("nan"), float("nan"))
    dmin = np.float32(depth[mask].min())
    dmax = np.float32(depth[mask].max())
    den = np.float32(np.float64(np.float32(dmax - dmin)) + 1e-6)
    idx = np.zeros(depth.shape, np.uint8)
    q = (depth[mask] - dmin) / den
    idx[mask] = (q * np.float32(255)).astype(np.uint8)
    return jet_lut()[idx], (float(dmin), float(dmax))

