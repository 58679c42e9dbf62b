"""Python front-end of the C-ABI: one :class:`Renderer` per GPU per process.

This is the object the reference's Camera + annotator graph collapses into:
``Camera(...)`` + ``camera.initialize()`` (generate_construction_data.py:1421,
:1451) become :class:`Renderer` construction, and each
``set_world_pose`` + ``next_update_async`` + ``get_rgba()`` / ``get_data()``
round trip (:1586-1595, :1669, :1681, :1916) becomes one row of a batched
:meth:`Renderer.render` call.  Everything numeric runs in libcsg.so on the
GPU; this module only marshals arrays.
"""
from __future__ import annotations

import ctypes as C
from typing import Dict, Iterable, List, Optional, Sequence

import numpy as np

from . import _lib
from ._lib import CsgError
from .camera_math import Intrinsics
from .packing import PackedScene, light_constants, pack_scene
from .scene.model import Scene

FRAME_DTYPE = np.dtype([("view", "<f4", 16), ("proj", "<f4", 16), ("xform_set", "<u4"), ("frame_id", "<u4"),
                        ("records_hint", "<u4"), ("bins_hint", "<u4")])
assert FRAME_DTYPE.itemsize == C.sizeof(_lib.Frame)

OUTPUT_KINDS = ("rgb", "instance", "depth", "keypoints", "stats", "normals", "points", "depth_vis", "depth_range",
                "covered", "depth_stats")


def make_frames(views: np.ndarray, projs: np.ndarray, sets: Sequence[int], frame_ids: Sequence[int]) -> np.ndarray:
    n = len(frame_ids)
    fr = np.zeros(n, FRAME_DTYPE)
    fr["view"] = np.asarray(views, np.float64).reshape(n, 16).astype(np.float32)
    fr["proj"] = np.asarray(projs, np.float64).reshape(n, 16).astype(np.float32)
    fr["xform_set"] = np.asarray(sets, np.uint32)
    fr["frame_id"] = np.asarray(frame_ids, np.uint32)
    return fr


def _light_struct(light) -> "_lib.Light":
    amb, sun, d, sky = light_constants(light)
    L = _lib.Light()
    L.ambient[:] = [float(x) for x in amb]
    L.sun[:] = [float(x) for x in sun]
    L.sun_dir[:] = [float(x) for x in d]
    L.sky[:] = [int(x) for x in sky]
    return L


def scene_labels(scene: Scene) -> int:
    """Label-table length of a scene (the renderers' ``n_labels``)."""
    n = max([o.inst_idx for o in scene.objects] + [i.inst_idx for i in scene.instances] + [-1]) + 1
    return max(n, 1)


def output_spec(n: int, H: int, W: int, n_kp: int, n_labels: int, want: Iterable[str]) -> Dict[str, tuple]:
    """Host arrays a render of ``n`` frames fills for ``want``: name -> (shape, dtype)."""
    want = set(want)
    spec: Dict[str, tuple] = {}
    if "rgb" in want:
        spec["rgb"] = ((n, H, W, 3), np.uint8)
    if "instance" in want:
        spec["instance"] = ((n, H, W), np.int32)
    if "depth" in want:
        spec["depth"] = ((n, H, W), np.float32)
    if "keypoints" in want and n_kp:
        spec["keypoints_uv"] = ((n, n_kp, 2), np.float32)
        spec["keypoints_vis"] = ((n, n_kp), np.int32)
    if "stats" in want:
        spec["inst_stats"] = ((n, n_labels, 5), np.uint32)
    if "normals" in want:
        spec["normals"] = ((n, H, W, 3), np.float16)
    if "points" in want:
        spec["points"] = ((n, H, W, 3), np.float32)
    if "depth_vis" in want:   # the reference's JET depth PNG (GDP:1690-1709) and its min / max
        spec["depth_vis"] = ((n, H, W, 3), np.uint8)
    if "depth_vis" in want or "depth_range" in want:
        spec["depth_range"] = ((n, 2), np.float32)
    if "depth_stats" in want:   # the quality log's depth counts: valid, zero, inf, sum, min, max
        spec["depth_stats"] = ((n, 6), np.float64)
    if "covered" in want:     # unoccluded pixels per label (occlusionRatio)
        spec["label_covered"] = ((n, n_labels), np.uint32)
    return spec


class Renderer:
    def __init__(self, scene: Scene, width: int, height: int, max_frames: int = 8, device: int = 0,
                 intrinsics: Optional[Intrinsics] = None, records_per_frame: int = 0, bins_per_frame: int = 0,
                 frames_per_launch: int = 0):
        self.lib = _lib.load()
        self.scene = scene
        self.width, self.height = int(width), int(height)
        self.max_frames = int(max_frames)
        self.intr = intrinsics or Intrinsics(self.width, self.height)
        cfg = _lib.Config(device, self.width, self.height, self.max_frames, self.intr.near, self.intr.far,
                          records_per_frame, bins_per_frame, frames_per_launch)
        ctx = C.c_void_p()
        rc = self.lib.csg_create(C.byref(cfg), C.byref(ctx))
        if rc != 0:
            raise CsgError(f"csg_create failed ({rc})")
        self.ctx = ctx
        self.packed: PackedScene = pack_scene(scene)
        self.n_inst = len(scene.instances)
        self.n_labels = max(self.packed.n_labels, 1)
        assert self.n_labels == scene_labels(scene)
        self.n_kp = 0
        self._pinned: List[C.c_void_p] = []
        self._upload()

    # -- lifecycle ------------------------------------------------------------
    def _check(self, rc: int, what: str) -> None:
        if rc != 0:
            msg = self.lib.csg_last_error(self.ctx).decode(errors="replace")
            raise CsgError(f"{what}: status {rc}: {msg}")

    def close(self) -> None:
        if getattr(self, "ctx", None):
            for p in getattr(self, "_pinned", []):
                self.lib.csg_host_free(self.ctx, p)
            self._pinned = []
            self.lib.csg_destroy(self.ctx)
            self.ctx = None

    def __del__(self):  # pragma: no cover
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    # -- scene ---------------------------------------------------------------
    def _upload(self) -> None:
        p = self.packed
        keep = []
        meshes = (_lib.Mesh * len(self.scene.meshes))()
        for k, m in enumerate(self.scene.meshes):
            pos = np.ascontiguousarray(m.positions, np.float32)
            idx = np.ascontiguousarray(m.tris, np.uint32)
            keep += [pos, idx]
            has_uv = m.uvs.shape[0] > 0 and m.uv_tris.shape[0] == m.n_tris
            meshes[k].positions = pos.ctypes.data
            meshes[k].n_vertices = pos.shape[0]
            meshes[k].indices = idx.ctypes.data
            meshes[k].n_tris = idx.shape[0]
            if has_uv:
                uv = np.ascontiguousarray(m.uvs, np.float32)
                uvi = np.ascontiguousarray(m.uv_tris, np.uint32)
                keep += [uv, uvi]
                meshes[k].uvs, meshes[k].n_uvs, meshes[k].uv_indices = uv.ctypes.data, uv.shape[0], uvi.ctypes.data
            meshes[k].material = m.material
        mats = (_lib.Material * len(p.materials))()
        for k in range(len(p.materials)):
            mats[k].base_color[:] = [int(x) for x in p.materials[k]["base"]]
            mats[k].texture = int(p.materials[k]["texture"])
            mats[k].alpha_test = int(p.materials[k]["alpha_test"])
            mats[k].alpha_threshold = int(p.materials[k]["alpha_threshold"])
        inst = (_lib.Instance * self.n_inst)()
        for k in range(self.n_inst):
            inst[k].model[:] = [float(x) for x in p.inst_model[k]]
            inst[k].mesh = int(p.inst_mesh[k])
            inst[k].inst_idx = int(p.inst_label[k])
        self._check(self.lib.csg_upload_scene(self.ctx, meshes, len(self.scene.meshes), mats, len(p.materials), inst,
                                              self.n_inst), "upload_scene")
        for k, t in enumerate(self.scene.textures):
            a = np.ascontiguousarray(t.rgba, np.uint8)
            self._check(self.lib.csg_upload_texture(self.ctx, k, a.ctypes.data, a.shape[1], a.shape[0]),
                        "upload_texture")
        self._check(self.lib.csg_set_light(self.ctx, C.byref(_light_struct(self.scene.light))), "set_light")

    def set_dr_light(self, set_id: int, light) -> None:
        """Lighting of transform set ``set_id`` (a ``scene.model.Light``; C4 DR)."""
        self._check(self.lib.csg_set_dr_light(self.ctx, set_id, C.byref(_light_struct(light))), "set_dr_light")

    def set_dr_textures(self, set_id: int, texture_per_material) -> None:
        """Texture of each material for transform set ``set_id``: an index into
        ``scene.textures``, -1 for none, or ``_lib.KEEP_TEXTURE``."""
        t = np.ascontiguousarray(np.asarray(texture_per_material, np.int32))
        self._check(self.lib.csg_set_dr_textures(self.ctx, set_id, t.ctypes.data, t.shape[0]), "set_dr_textures")

    def set_instance_transforms(self, set_id: int, models: np.ndarray) -> None:
        m = np.ascontiguousarray(np.asarray(models, np.float64).reshape(-1, 16).astype(np.float32))
        self._check(self.lib.csg_set_instance_transforms(self.ctx, set_id, m.ctypes.data, m.shape[0]),
                    "set_instance_transforms")

    def set_keypoints(self, set_id: int, pts_world: np.ndarray) -> None:
        p = np.ascontiguousarray(np.asarray(pts_world, np.float64).reshape(-1, 3).astype(np.float32))
        self._check(self.lib.csg_set_keypoints(self.ctx, set_id, p.ctypes.data, p.shape[0]), "set_keypoints")
        self.n_kp = p.shape[0]

    # -- rendering ------------------------------------------------------------
    def output_spec(self, n: int, want: Iterable[str]) -> Dict[str, tuple]:
        """Host arrays :meth:`render` fills for ``want``: name -> (shape, dtype)."""
        return output_spec(n, self.height, self.width, self.n_kp, self.n_labels, want)

    def render(self, frames: np.ndarray, want: Iterable[str] = ("rgb", "instance", "depth"),
               out: Optional[Dict[str, np.ndarray]] = None) -> Dict[str, np.ndarray]:
        """Render a batch to host numpy arrays (synchronous; includes D2H copies).
        ``out`` supplies the arrays (e.g. views of shared memory), shaped as
        :meth:`output_spec` says; otherwise they are allocated."""
        frames = np.ascontiguousarray(frames, FRAME_DTYPE)
        n = frames.shape[0]
        spec = self.output_spec(n, want)
        if out is None:
            out = {k: np.empty(shape, dt) for k, (shape, dt) in spec.items()}
        else:
            for k, (shape, dt) in spec.items():
                a = out.get(k)
                if a is None or a.shape != shape or a.dtype != dt or not a.flags.c_contiguous:
                    raise CsgError(f"render: out[{k!r}] must be a C-contiguous {np.dtype(dt)} array of shape {shape}")
            out = {k: out[k] for k in spec}
        for s in range(0, n, self.max_frames):
            e = min(n, s + self.max_frames)
            oo = _lib.Outputs()
            for name, key in (("rgb", "rgb"), ("instance", "instance"), ("depth", "depth"),
                              ("keypoints_uv", "keypoints_uv"), ("keypoints_vis", "keypoints_vis"),
                              ("inst_stats", "inst_stats"), ("normals", "normals"), ("points", "points"),
                              ("depth_vis", "depth_vis"), ("depth_range", "depth_range"),
                              ("label_covered", "label_covered"), ("depth_stats", "depth_stats")):
                arr = out.get(key)
                if arr is not None:
                    setattr(oo, name, arr[s:e].ctypes.data)
            oo.n_labels, oo.on_device = self.n_labels, 0
            self._check(self.lib.csg_render_batch(self.ctx, frames[s:e].ctypes.data, e - s, C.byref(oo)),
                        "render_batch")
        return out

    # -- files encoded on the GPU --------------------------------------------------
    def host_buffer(self, nbytes: int) -> np.ndarray:
        """A page-locked uint8 host array of ``nbytes`` (csg_host_alloc), freed
        with the renderer; D2H copies into it run at full PCIe rate."""
        p = C.c_void_p()
        self._check(self.lib.csg_host_alloc(self.ctx, int(nbytes), C.byref(p)), "host_alloc")
        buf = (C.c_uint8 * int(nbytes)).from_address(p.value)
        arr = np.frombuffer(buf, np.uint8)
        self._pinned.append(p)
        return arr

    def free_host_buffer(self, arr: np.ndarray) -> None:
        """Release a :meth:`host_buffer` array now (instead of with the
        renderer); the caller guarantees nothing reads it any more."""
        addr = arr.ctypes.data
        for k, p in enumerate(self._pinned):
            if p.value == addr:
                self._check(self.lib.csg_host_free(self.ctx, p), "host_free")
                del self._pinned[k]
                return
        raise CsgError("free_host_buffer: not a buffer of this renderer")

    def render_files(self, frames: np.ndarray, kinds: Sequence[str], files: np.ndarray,
                     want: Iterable[str] = (), out: Optional[Dict[str, np.ndarray]] = None):
        """Render a batch (at most ``max_frames``) and encode ``kinds`` (of
        ``_lib.FILE_KINDS``: "rgb_png", "depth_csv", "depth_png", "pointcloud_txt") on the GPU
        into ``files`` (uint8 host array, pinned from :meth:`host_buffer` for
        speed), growing nothing: returns (outputs dict as :meth:`render`,
        offsets) with file j = frame * len(kinds) + k (kinds in bit order) at
        ``files[offsets[j]:offsets[j + 1]]``; ``None`` offsets' last entry
        says how many bytes were needed when ``files`` was too small (the
        files stay on the device: :meth:`copy_files`)."""
        frames = np.ascontiguousarray(frames, FRAME_DTYPE)
        n = frames.shape[0]
        if n > self.max_frames:
            raise CsgError(f"render_files: {n} frames > max_frames {self.max_frames}")
        mask = 0
        for k in kinds:
            if k not in _lib.FILE_KINDS:
                raise CsgError(f"unknown file kind {k!r}; choose from {tuple(_lib.FILE_KINDS)}")
            mask |= _lib.FILE_KINDS[k]
        spec = self.output_spec(n, want)
        if out is None:
            out = {k: np.empty(shape, dt) for k, (shape, dt) in spec.items()}
        else:
            for k, (shape, dt) in spec.items():
                a = out.get(k)
                if a is None or a.shape != shape or a.dtype != dt or not a.flags.c_contiguous:
                    raise CsgError(f"render_files: out[{k!r}] must be a C-contiguous {np.dtype(dt)} array of shape {shape}")
            out = {k: out[k] for k in spec}
        nk = bin(mask).count("1")
        offsets = np.zeros(n * nk + 1, np.uint64)
        if files.dtype != np.uint8 or not files.flags.c_contiguous:
            raise CsgError("render_files: files must be a C-contiguous uint8 array")
        oo = _lib.Outputs()
        for key in ("rgb", "instance", "depth", "keypoints_uv", "keypoints_vis", "inst_stats", "normals", "points",
                    "depth_vis", "depth_range", "label_covered", "depth_stats"):
            arr = out.get(key)
            if arr is not None:
                setattr(oo, key, arr.ctypes.data)
        oo.n_labels, oo.on_device = self.n_labels, 0
        oo.file_kinds, oo.files, oo.files_cap, oo.file_offsets = mask, files.ctypes.data, files.nbytes, offsets.ctypes.data
        rc = self.lib.csg_render_batch(self.ctx, frames.ctypes.data, n, C.byref(oo))
        if rc == _lib.ERR_CAPACITY:
            return out, None, int(offsets[-1])
        self._check(rc, "render_batch (files)")
        return out, offsets, int(offsets[-1])

    def copy_files(self, files: np.ndarray, n_files: int) -> np.ndarray:
        """The last :meth:`render_files` batch's files again (after the
        buffer was too small): returns the offsets."""
        offsets = np.zeros(n_files + 1, np.uint64)
        self._check(self.lib.csg_copy_files(self.ctx, files.ctypes.data, files.nbytes, offsets.ctypes.data),
                    "copy_files")
        return offsets

    def render_into(self, frames_ptr: int, n: int, frames_on_device: bool, rgb: int = 0, instance: int = 0,
                    depth: int = 0, kp_uv: int = 0, kp_vis: int = 0, stats: int = 0, stream: int = 0,
                    normals: int = 0, points: int = 0, depth_vis: int = 0, depth_range: int = 0,
                    covered: int = 0, depth_stats: int = 0) -> None:
        """Enqueue a batch writing device buffers (raw pointers, e.g. torch ``data_ptr()``)."""
        o = _lib.Outputs(rgb or None, instance or None, depth or None, kp_uv or None, kp_vis or None,
                         stats or None, self.n_labels, 1, normals or None, points or None, depth_vis or None,
                         depth_range or None, covered or None, 0, 0, None, 0, None, depth_stats or None)
        self._check(self.lib.csg_render_batch_async(self.ctx, frames_ptr, n, int(frames_on_device), C.byref(o),
                                                    stream or None), "render_batch_async")

    def instance_bounds(self, set_id: int = 0) -> np.ndarray:
        """(I, 2, 3) float32 world-space AABB of every instance under a transform set (GPU reduction)."""
        out = np.empty((self.n_inst, 6), np.float32)
        self._check(self.lib.csg_instance_bounds(self.ctx, set_id, out.ctypes.data), "instance_bounds")
        return out.reshape(-1, 2, 3)

    def host_id_bytes(self) -> int:
        """Bytes per instance id on the host wire of host-output batches (1, 2 or 4; csg_host_id_bytes)."""
        n = self.lib.csg_host_id_bytes(self.ctx)
        if n < 0:
            self._check(n, "host_id_bytes")
        return int(n)

    def synchronize(self) -> None:
        self._check(self.lib.csg_synchronize(self.ctx), "synchronize")

    def batch_stats(self) -> Dict[str, float]:
        st = _lib.BatchStats()
        self._check(self.lib.csg_get_batch_stats(self.ctx, C.byref(st)), "get_batch_stats")
        return {n: getattr(st, n) for n, _ in _lib.BatchStats._fields_}

    def size_work(self, frames, n: Optional[int] = None, on_device: bool = False,
                  margin: float = 0.25) -> Dict[str, float]:
        """Size the work buffers from a sizing pass over ``frames``
        (csg_size_work): a FRAME_DTYPE array, or with ``on_device`` a device
        pointer (int) to ``n`` frame records.  Writes each frame's work hints
        (``records_hint``, ``bins_hint``) into the records passed -- the array
        itself, or the device records -- so later batches of those records get
        regions of their own size.  Returns :meth:`work_info`."""
        info = _lib.WorkInfo()
        if on_device:
            self._check(self.lib.csg_size_work(self.ctx, int(frames), int(n), 1, float(margin), C.byref(info)),
                        "size_work")
        else:
            fr = np.ascontiguousarray(frames, FRAME_DTYPE)
            self._check(self.lib.csg_size_work(self.ctx, fr.ctypes.data, fr.shape[0], 0, float(margin),
                                               C.byref(info)), "size_work")
            if fr is not frames:   # a converted copy: hand the hints back
                frames["records_hint"] = fr["records_hint"]
                frames["bins_hint"] = fr["bins_hint"]
        return {k: getattr(info, k) for k, _ in _lib.WorkInfo._fields_ if k != "pad"}

    def work_info(self) -> Dict[str, float]:
        """Current work-buffer caps, the last sizing pass and the buffers' device bytes."""
        info = _lib.WorkInfo()
        self._check(self.lib.csg_get_work_info(self.ctx, C.byref(info)), "get_work_info")
        return {k: getattr(info, k) for k, _ in _lib.WorkInfo._fields_ if k != "pad"}

    def timing_reset(self) -> None:
        self._check(self.lib.csg_timing_reset(self.ctx), "timing_reset")

    def timing_read(self) -> Dict[str, float]:
        t = _lib.Timing()
        self._check(self.lib.csg_timing_read(self.ctx, C.byref(t)), "timing_read")
        return {n: getattr(t, n) for n, _ in _lib.Timing._fields_}

    def project_keypoints(self, pts_world: np.ndarray, view: np.ndarray, proj: np.ndarray):
        p = np.ascontiguousarray(np.asarray(pts_world).reshape(-1, 3), np.float32)
        v = np.ascontiguousarray(np.asarray(view).reshape(16), np.float32)
        pr = np.ascontiguousarray(np.asarray(proj).reshape(16), np.float32)
        uv = np.empty((p.shape[0], 2), np.float32)
        vis = np.empty(p.shape[0], np.int32)
        self._check(self.lib.csg_project_keypoints(self.ctx, p.ctypes.data, p.shape[0], v.ctypes.data, pr.ctypes.data,
                                                   uv.ctypes.data, vis.ctypes.data), "project_keypoints")
        return uv, vis
