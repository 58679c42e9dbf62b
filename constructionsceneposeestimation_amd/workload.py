"""Workloads C1-C5 of BASELINE.json as concrete scenes + schedules.

A workload bundles the scene, the resolution, the seed and the per-frame /
per-epoch state the renderer needs.  Every piece of state is a pure
function of ``(seed, frame)`` or ``(seed, epoch)``, so any shard of frames
can be produced by any process independently.

* C1  TrafficCone mesh alone, 256x256, 1 frame (CPU-runnable plumbing case)
* C2  world2 static (stands in for the missing world1.usd), 1920x1080
* C3  world2 + crane/dumper/4 rigged-human proxies, 1920x1080, RGB + instance
      segmentation + 2D keypoints (the bench workload)
* C4  C3 with per-epoch DR of lighting (dome tint/intensity, sun) and
      textures (tinted variants) on top of the layout randomisation, frames
      seed-sharded across GPUs
* C5  C3 at 3840x2160 with depth, normals (f16) and world points
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import Dict, List, Optional, Tuple

import numpy as np

from . import camera_math as cm
from . import schedule
from .scene import load_cone, load_world2
from .scene import xform as X
from .scene.model import Scene
from .scene.proxies import COCO_JOINTS, HumanRig, add_proxies, pose_humans

WORKLOADS = {
    "C1": dict(scene="cone", width=256, height=256, outputs=("rgb", "instance", "depth"),
               title="TrafficCone mesh alone"),
    "C2": dict(scene="world2", width=1920, height=1080, outputs=("rgb", "instance"),
               title="world2.usd static (stands in for the missing world1.usd), scheduled camera poses"),
    "C3": dict(scene="world2_people", width=1920, height=1080, outputs=("rgb", "instance", "keypoints"),
               title="world2.usd + crane/dumper/4 rigged-human proxies"),
    "C4": dict(scene="world2_people", width=1920, height=1080, outputs=("rgb", "instance", "keypoints"), dr=True,
               title="world2.usd + proxies, per-epoch lighting/texture/layout/pose DR"),
    "C5": dict(scene="world2_people", width=3840, height=2160,
               outputs=("rgb", "instance", "depth", "normals", "points", "keypoints"),
               title="world2.usd + crane/dumper/people proxies"),
}


def build_scene(name: str, n_humans: int = 4) -> Scene:
    if name == "cone":
        return load_cone()
    s = load_world2()
    if name == "world2":
        return s
    if name == "world2_people":
        return add_proxies(s, n_humans=n_humans)
    raise ValueError(f"unknown scene {name!r}")


def box_keypoints(bounds: np.ndarray) -> np.ndarray:
    """8 corners (x slowest, z fastest) + centre of a local AABB: (9,3)."""
    lo, hi = bounds
    c = np.array([[x, y, z] for x in (lo[0], hi[0]) for y in (lo[1], hi[1]) for z in (lo[2], hi[2])])
    return np.vstack([c, (lo + hi) / 2.0])


@dataclass
class EpochState:
    models: np.ndarray                 # (I,4,4) float64 instance transforms
    object_frames: List[np.ndarray]    # per object
    keypoints: np.ndarray              # (K,3) world
    joints: Dict[int, Dict[str, np.ndarray]] = field(default_factory=dict)
    dr: Optional["schedule.DRParams"] = None   # lighting / texture DR (C4), None = authored


class Workload:
    def __init__(self, name: str = "C3", seed: int = 0, width: Optional[int] = None,
                 height: Optional[int] = None, n_humans: int = 4, scene: Optional[Scene] = None):
        spec = WORKLOADS[name]
        self.name, self.seed = name, int(seed)
        self.width = int(width or spec["width"])
        self.height = int(height or spec["height"])
        self.outputs = spec["outputs"]
        self.scene = scene if scene is not None else build_scene(spec["scene"], n_humans)
        self.dr = bool(spec.get("dr", False))
        self.dr_variants = schedule.add_dr_texture_variants(self.scene) if self.dr else {}
        self.intr = cm.Intrinsics(self.width, self.height)
        self.base_models = np.stack([i.model for i in self.scene.instances])
        self.frames0 = [schedule.object_frame(self.scene, j) for j in range(len(self.scene.objects))]
        # keypoint table: 9 box points per labelled object, + 17 joints per rigged human
        self.kp_table: List[Tuple[int, str]] = []
        for j in range(len(self.scene.objects)):
            for k in range(9):
                self.kp_table.append((j, f"box{k}" if k < 8 else "center"))
        self.rig_objs = [r["obj"] for r in self.scene.meta.get("human_rigs", [])]
        for j in self.rig_objs:
            for n in COCO_JOINTS:
                self.kp_table.append((j, n))
        self._epoch_cache: Dict[int, EpochState] = {}
        self._cam_cache: Dict[int, tuple] = {}

    # -- per frame ------------------------------------------------------------
    def camera(self, frame: int, attempt: int = 0):
        """(V, P, C, cam, aim, q) of a frame; memoised (the generator asks for
        a frame's camera when it renders it and again for its label).
        ``attempt`` > 0: the pose of the point-cloud validation's retry
        ``attempt`` (GDP:1573-1581): the camera moved by
        schedule.retry_offset, still aimed at the frame's aim point -- a
        pitched shot whenever the jitter moved it off the aim point's height."""
        key = (frame, attempt)
        hit = self._cam_cache.get(key)
        if hit is not None:
            return hit
        cam, aim = schedule.camera_pose(self.seed, frame)
        if attempt:
            cam = cam + schedule.retry_offset(self.seed, frame, attempt)
        q = cm.look_at_world_quat(cam, aim)
        V, P, C = cm.frame_matrices(cam, q, self.intr)
        if len(self._cam_cache) >= 4096:
            self._cam_cache.clear()
        self._cam_cache[key] = out = (V, P, C, cam, aim, q)
        return out

    def install_camera(self, frame: int, cam: tuple) -> None:
        """A frame's attempt-0 camera computed elsewhere (prep_pool: the same
        Workload arguments in a worker process give the same numbers)."""
        if len(self._cam_cache) >= 4096:
            self._cam_cache.clear()
        self._cam_cache[(frame, 0)] = cam

    def frame_params(self, frame_ids, attempts=None) -> Tuple[np.ndarray, np.ndarray]:
        Vs, Ps = [], []
        for j, k in enumerate(frame_ids):
            V, P, *_ = self.camera(int(k), int(attempts[j]) if attempts is not None else 0)
            Vs.append(V)
            Ps.append(P)
        return np.stack(Vs), np.stack(Ps)

    # -- per epoch ------------------------------------------------------------
    def epoch(self, e: int) -> EpochState:
        if e in self._epoch_cache:
            return self._epoch_cache[e]
        frames = schedule.object_frames_for_epoch(self.scene, self.seed, e)
        models = self.base_models.copy()
        for i, inst in enumerate(self.scene.instances):
            if inst.obj >= 0 and self.scene.objects[inst.obj].kind != "static" and inst.local is not None:
                models[i] = frames[inst.obj] @ inst.local
        if e == 0:
            joints = {o: HumanRig.joints() for o in self.rig_objs}
        else:
            joints = pose_humans(self.scene, frames, models,
                                 lambda o: schedule.rng_for(self.seed, schedule.STREAM_POSE, e * 4096 + o))
        kps = []
        for j, o in enumerate(self.scene.objects):
            b = o.local_bounds if o.local_bounds is not None else np.zeros((2, 3))
            kps.append(X.transform_points(frames[j], box_keypoints(b)))
        for j in self.rig_objs:
            J = joints[j]
            kps.append(X.transform_points(frames[j], np.stack([J[n] for n in COCO_JOINTS])))
        st = EpochState(models, frames, np.vstack(kps) if kps else np.zeros((0, 3)), joints)
        if self.dr:
            st.dr = schedule.domain_randomization(self.scene, self.seed, e, self.dr_variants)
        if len(self._epoch_cache) >= 256:   # bounded: a long run visits each epoch once
            self._epoch_cache.pop(next(iter(self._epoch_cache)))
        self._epoch_cache[e] = st
        return st

    def install_epoch(self, e: int, st: EpochState) -> None:
        """An epoch's state computed elsewhere (prep_pool)."""
        if e in self._epoch_cache:
            return
        if len(self._epoch_cache) >= 256:
            self._epoch_cache.pop(next(iter(self._epoch_cache)))
        self._epoch_cache[e] = st

    def n_keypoints(self) -> int:
        return len(self.kp_table)
