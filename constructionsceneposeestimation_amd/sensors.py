"""Drop-in mirror of the reference's sensor boundary (Isaac Sim ``Camera`` +
Kit frame advance), backed by libcsg.so on the GPU.

Reference call sites (generate_construction_data.py):
``Camera(prim_path, resolution)`` :1421, ``camera.initialize()`` :1451,
clip/focal/aperture set on the USD camera :1436-1443,
``camera.set_world_pose(position, orientation)`` :1586 (orientation w-first,
Isaac "world" camera axes: +X forward, +Z up), ``await
omni.kit.app.get_app().next_update_async()`` :1592, ``camera.get_rgba()``
:1669, ``camera.get_render_product_path()`` :1461,
``camera.get_focal_length()`` / ``get_horizontal_aperture()`` :2035-2037,
``camera.add_motion_vectors_to_frame()`` :1494, ``get_obj_pose`` :587-605,
``randomize_object_positions(stage)`` :914-1231.

A frame is rendered when the frame is advanced (``next_update`` /
``next_update_async``), as in Kit; ``get_rgba`` and the annotators return
host copies of that frame, like Replicator's ``get_data()``.  This path
renders one frame per call for API compatibility; bulk generation uses
``generate.py`` (batched, device-resident).
"""
from __future__ import annotations

import asyncio
from typing import Dict, List, Optional, Sequence

import numpy as np

from . import camera_math as cm
from . import schedule
from .labels import bbox3d_records
from .renderer import Renderer, make_frames
from .workload import Workload

_CAMERAS: Dict[str, "Camera"] = {}


class Stage:
    """The mutable scene state the reference edits through ``pxr``: object
    placements (one randomisation epoch at a time) on top of a static scene."""

    def __init__(self, workload: str = "C3", seed: int = 0, n_humans: int = 4, scene=None):
        self.workload = Workload(workload, seed=seed, n_humans=n_humans, scene=scene)
        self.scene = self.workload.scene
        self.seed = seed
        self.epoch = 0
        self.version = 0

    @property
    def state(self):
        return self.workload.epoch(self.epoch)

    def randomize_object_positions(self) -> List[dict]:
        """Advance to the next randomisation epoch; returns the reference's
        per-object records ``{path, new_pos, rotation, type, no_overlap}``."""
        self.epoch += 1
        self.version += 1
        out = []
        for j, p in schedule.randomize_object_positions(self.scene, self.seed, self.epoch).items():
            o = self.scene.objects[j]
            out.append({"path": o.prim_path, "new_pos": [p.x, p.y, p.z], "rotation": p.rotation,
                        "type": o.kind, "no_overlap": p.no_overlap})
        return out

    def get_obj_pose(self, prim_path: str) -> list:
        for cam in _CAMERAS.values():
            if cam.prim_path == prim_path:
                return cam.get_obj_pose()
        for j, o in enumerate(self.scene.objects):
            if o.prim_path == prim_path:
                return cm.get_obj_pose_from_matrix(self.state.object_frames[j])
        raise ValueError(f"Prim '{prim_path}' not found.")


def randomize_object_positions(stage: Stage) -> List[dict]:
    return stage.randomize_object_positions()


class Camera:
    def __init__(self, prim_path: str = "/World/Camera_0", resolution: Sequence[int] = (1280, 720),
                 stage: Optional[Stage] = None, device: int = 0, name: Optional[str] = None):
        self.prim_path = prim_path
        self.width, self.height = int(resolution[0]), int(resolution[1])
        self.stage = stage or Stage()
        self.device = device
        self.name = name or prim_path.rstrip("/").split("/")[-1]
        self.focal_length = cm.FOCAL_LENGTH_MM
        self.horizontal_aperture = cm.H_APERTURE_MM
        self.clipping_range = (cm.NEAR_CLIP, cm.FAR_CLIP)
        self._pos = np.zeros(3)
        self._quat = np.array([1.0, 0.0, 0.0, 0.0])
        self._renderer: Optional[Renderer] = None
        self._uploaded_version = -1
        self._frame: Optional[Dict[str, np.ndarray]] = None
        self._frame_meta: Dict[str, object] = {}
        self._dirty = False
        self._frame_id = 0
        self._extra: set = set()        # extra renderer outputs requested by attached annotators
        _CAMERAS[self.get_render_product_path()] = self

    def require(self, outputs) -> None:
        """Annotators attached to this camera ask for extra renderer outputs
        (``points``, ``normals``); takes effect from the next frame."""
        new = set(outputs) - self._extra
        if new:
            self._extra |= new
            self._dirty = True

    # -- USD camera attributes (:1436-1443) -----------------------------------
    def set_clipping_range(self, near: float, far: float) -> None:
        self.clipping_range = (float(near), float(far))
        self._renderer = None

    def set_focal_length(self, f: float) -> None:
        self.focal_length = float(f)

    def set_horizontal_aperture(self, a: float) -> None:
        self.horizontal_aperture = float(a)

    def get_focal_length(self) -> float:
        return self.focal_length

    def get_horizontal_aperture(self) -> float:
        return self.horizontal_aperture

    def get_vertical_aperture(self) -> float:
        return self.horizontal_aperture * (self.height / self.width)

    def intrinsics(self) -> cm.Intrinsics:
        return cm.Intrinsics(self.width, self.height, self.focal_length, self.horizontal_aperture,
                             self.clipping_range[0], self.clipping_range[1])

    # -- lifecycle ------------------------------------------------------------
    def initialize(self) -> None:
        if self._renderer is None:
            self._renderer = Renderer(self.stage.scene, self.width, self.height, max_frames=1,
                                      device=self.device, intrinsics=self.intrinsics())
            self._uploaded_version = -1

    def add_motion_vectors_to_frame(self) -> None:
        """Accepted for API compatibility; motion vectors are not produced."""

    def get_render_product_path(self) -> str:
        return f"/Render/RenderProduct_{self.name}"

    # -- pose -----------------------------------------------------------------
    def set_world_pose(self, position=None, orientation=None, camera_axes: str = "world") -> None:
        if camera_axes != "world":
            raise NotImplementedError("only camera_axes='world' (the reference's usage) is supported")
        if position is not None:
            self._pos = np.asarray(position, np.float64).reshape(3)
        if orientation is not None:
            q = np.asarray(orientation, np.float64).reshape(4)
            n = np.linalg.norm(q)
            self._quat = q / n if n > 0 else np.array([1.0, 0, 0, 0])
        self._dirty = True

    def get_world_pose(self):
        return self._pos.copy(), self._quat.copy()

    def get_obj_pose(self) -> list:
        return cm.get_obj_pose_from_matrix(cm.camera_usd_transform(self._pos, self._quat))

    # -- rendering (called from next_update) ----------------------------------
    def _sync_stage(self) -> None:
        """Upload the stage's current epoch (transforms, keypoints, DR) if it changed."""
        self.initialize()
        r = self._renderer
        if self._uploaded_version != self.stage.version:
            st = self.stage.state
            r.set_instance_transforms(0, st.models)
            if st.keypoints.shape[0]:
                r.set_keypoints(0, st.keypoints)
            if st.dr is not None:
                r.set_dr_light(0, st.dr.light)
                r.set_dr_textures(0, st.dr.textures)
            self._uploaded_version = self.stage.version

    def _render(self) -> None:
        self._sync_stage()
        r = self._renderer
        V, P, C = cm.frame_matrices(self._pos, self._quat, self.intrinsics())
        fr = make_frames(V[None], P[None], [0], [self._frame_id])
        out = r.render(fr, want=("rgb", "instance", "depth", "keypoints", "stats") + tuple(sorted(self._extra)))
        self._frame = {k: v[0] for k, v in out.items()}
        self._frame_meta = {"view": V, "proj": P, "cam_to_world": C, "epoch": self.stage.epoch,
                            "frame_id": self._frame_id}
        self._frame_id += 1
        self._dirty = False

    def object_world_bounds(self) -> np.ndarray:
        """(n_objects, 2, 3) world AABB of each labelled object's vertices in
        the current epoch (GPU reduction over its instances; NaN if none)."""
        self._sync_stage()
        if getattr(self, "_bounds_version", None) != self.stage.version:
            ib = self._renderer.instance_bounds(0)
            ob = np.full((len(self.stage.scene.objects), 2, 3), np.nan, np.float32)
            for i, inst in enumerate(self.stage.scene.instances):
                j = inst.obj
                if j < 0 or not np.all(np.isfinite(ib[i])):
                    continue
                ob[j, 0] = np.fmin(ob[j, 0], ib[i, 0])
                ob[j, 1] = np.fmax(ob[j, 1], ib[i, 1])
            self._bounds, self._bounds_version = ob, self.stage.version
        return self._bounds

    def get_rgba(self) -> Optional[np.ndarray]:
        if self._frame is None:
            return None
        rgb = self._frame["rgb"]
        return np.concatenate([rgb, np.full(rgb.shape[:2] + (1,), 255, np.uint8)], axis=2)

    def frame_outputs(self) -> Optional[Dict[str, np.ndarray]]:
        return self._frame


def next_update() -> None:
    """Kit frame advance: render every camera whose pose or scene changed."""
    for cam in list(_CAMERAS.values()):
        if cam._dirty or cam._frame is None or cam._uploaded_version != cam.stage.version:
            cam._render()


async def next_update_async() -> None:
    next_update()
    await asyncio.sleep(0)


def get_camera(render_product_path: str) -> Camera:
    if render_product_path not in _CAMERAS:
        raise KeyError(f"no camera for render product {render_product_path!r}")
    return _CAMERAS[render_product_path]


def reset() -> None:
    """Drop every registered camera (tests)."""
    for cam in _CAMERAS.values():
        if cam._renderer is not None:
            cam._renderer.close()
    _CAMERAS.clear()
