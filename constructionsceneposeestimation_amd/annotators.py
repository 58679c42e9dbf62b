"""Mirror of ``omni.replicator.core.AnnotatorRegistry`` for the annotators the
reference attaches (generate_construction_data.py:1460-1484) plus this
build's additions.

``get_data()`` shapes follow what the reference reads:
* ``distance_to_image_plane`` -> H x W float32, inf where nothing was hit
  (:1681, quality check :318-321);
* ``instance_segmentation`` -> ``{"data": H x W uint32, "info": {"idToLabels",
  "idToSemantics"}}`` (:1818-1842); id 0 = background/unlabelled, id k+1 =
  object ``inst_idx`` k;
* ``bounding_box_3d`` -> ``{"data": structured records (semanticId, x/y/z
  min/max, 4x4 transform, occlusionRatio = 1 - visible / unoccluded pixels
  from the GPU's label coverage), "info": {"primPaths",
  "worldBounds"}}`` for the objects visible in the frame (:1780-1790,
  :1916-1922, read positionally by ``bboxDict_to_transform`` :562-564);
  ``worldBounds`` (N,2,3) is the world AABB of each object's vertices,
  reduced on the GPU;
* ``pointcloud`` -> ``{"data": (N,3) float32 world points, "pointRgb": (N,4)
  uint8, "info": {...}}`` (:1614, :1720-1724, :735);
* ``normals`` -> H x W x 3 float16 unit world-space normals facing the camera
  (0 on background; C5);
* ``rgb`` -> H x W x 4 uint8;
* ``bounding_box_2d_tight`` / ``keypoints_2d`` -> this build's per-instance
  pixel boxes and 2D keypoints (uv, visibility).
"""
from __future__ import annotations

from typing import Dict, Optional

import numpy as np

from . import sensors
from .labels import bbox3d_records

SUPPORTED = ("rgb", "distance_to_image_plane", "instance_segmentation", "bounding_box_3d",
             "bounding_box_2d_tight", "pointcloud", "keypoints_2d", "normals")
# renderer outputs an annotator needs beyond the camera's defaults
_NEEDS = {"pointcloud": ("points",), "normals": ("normals",), "bounding_box_3d": ("covered",)}


class Annotator:
    def __init__(self, name: str):
        if name not in SUPPORTED:
            raise ValueError(f"unsupported annotator {name!r}; supported: {SUPPORTED}")
        self.name = name
        self.camera: Optional[sensors.Camera] = None

    def attach(self, render_product_path) -> None:
        paths = render_product_path if isinstance(render_product_path, (list, tuple)) else [render_product_path]
        self.camera = sensors.get_camera(paths[0])
        self.camera.require(_NEEDS.get(self.name, ()))

    def detach(self) -> None:
        self.camera = None

    def get_data(self):
        if self.camera is None or self.camera.frame_outputs() is None:
            return None
        cam = self.camera
        out = cam.frame_outputs()
        meta = cam._frame_meta
        scene = cam.stage.scene
        if self.name == "rgb":
            return cam.get_rgba()
        if self.name == "distance_to_image_plane":
            return out["depth"].copy()
        if self.name == "instance_segmentation":
            ids = out["instance"]
            data = np.where(ids >= 0, ids + 1, 0).astype(np.uint32)
            present = np.unique(data[data > 0])
            by_idx = {o.inst_idx: o for o in scene.objects}
            return {"data": data, "info": {
                "idToLabels": {int(k): by_idx[int(k) - 1].prim_path for k in present},
                "idToSemantics": {int(k): {"class": by_idx[int(k) - 1].class_name} for k in present}}}
        if self.name in ("bounding_box_3d", "bounding_box_2d_tight"):
            stats = out["inst_stats"]
            vis = [j for j, o in enumerate(scene.objects) if o.inst_idx < stats.shape[0] and stats[o.inst_idx, 0] > 0]
            if self.name == "bounding_box_3d":
                recs = bbox3d_records(scene, cam.stage.state.object_frames, stats, out.get("label_covered"))
                return {"data": recs[vis], "info": {"primPaths": [scene.objects[j].prim_path for j in vis],
                                                     "idToLabels": {j: scene.objects[j].class_name for j in vis},
                                                     "worldBounds": cam.object_world_bounds()[vis]}}
            dt = np.dtype([("semanticId", "<u4"), ("x_min", "<i4"), ("y_min", "<i4"), ("x_max", "<i4"),
                           ("y_max", "<i4"), ("pixelCount", "<u4")])
            rec = np.zeros(len(vis), dt)
            for n, j in enumerate(vis):
                s = stats[scene.objects[j].inst_idx]
                rec[n] = (scene.objects[j].class_id, s[1], s[2], s[3], s[4], s[0])
            return {"data": rec, "info": {"primPaths": [scene.objects[j].prim_path for j in vis]}}
        if self.name == "pointcloud":
            # world points unprojected on the GPU inside the resolve (fused)
            m = np.isfinite(out["depth"])
            pts = out["points"][m]
            rgb = out["rgb"][m]
            rgba = np.concatenate([rgb, np.full((rgb.shape[0], 1), 255, np.uint8)], 1)
            sem = out["instance"][m]
            return {"data": pts, "pointRgb": rgba, "info": {"pointInstance": sem}}
        if self.name == "normals":
            return out["normals"].copy()
        if self.name == "keypoints_2d":
            return {"data": out.get("keypoints_uv"), "visibility": out.get("keypoints_vis"),
                    "info": {"table": cam.stage.workload.kp_table}}
        return None


class AnnotatorRegistry:
    @staticmethod
    def get_annotator(name: str, **kwargs) -> Annotator:
        return Annotator(name)
