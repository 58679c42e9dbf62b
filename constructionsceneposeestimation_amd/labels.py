"""Per-frame labels: 3D boxes, poses, visibility, keypoints, label JSON.

Reference anchors (generate_construction_data.py):
* ``bounding_box_3d`` annotator records — fields [1..6] local min/max, [7]
  4x4 row-major transform, read positionally at :562-564;
* ``bboxDict_to_transform`` :553-584 (centre = T^T mean(corners), size =
  |max-min| * column scales, euler 'xyz' degrees of the SVD-orthonormalised
  rotation) — restated here;
* label record :2056-2064 and ``save_label_json`` :608-613; the instance
  mask file ``instance_mask_%06d.npy`` :2066-2069.

This build adds ``keypoints_2d`` (per object: 8 box corners + centre, and
17 COCO joints for humans) and ``bbox_2d`` / ``pixel_count`` from the GPU's
per-instance statistics.  ``inst_idx`` is the scene-stable object index (the
reference numbers visible objects in Replicator's order, unknowable offline).
"""
from __future__ import annotations

from typing import Dict, List, Optional, Sequence

import numpy as np
from scipy.spatial.transform import Rotation

from .identity import CONSTRUCTION_CLASS

BBOX3D_DTYPE = np.dtype([("semanticId", "<u4"), ("x_min", "<f4"), ("y_min", "<f4"), ("z_min", "<f4"),
                         ("x_max", "<f4"), ("y_max", "<f4"), ("z_max", "<f4"), ("transform", "<f4", (4, 4)),
                         ("occlusionRatio", "<f4")])


COVERED_UNKNOWN = 0x80000000   # csg_outputs.label_covered flag (a tile held more than 32 labels)


def occlusion_ratios(pixels: np.ndarray, covered: np.ndarray) -> np.ndarray:
    """Per label ``1 - visible / covered`` (Replicator's bounding_box_3d
    ``occlusionRatio``, GDP:1780-1790: 0 fully visible, 1 fully occluded).
    ``pixels`` = visible pixel count (inst_stats[:, 0]), ``covered`` = the
    GPU's unoccluded coverage (label_covered); -1 where the coverage is
    unknown or the label covers nothing in the frame."""
    pixels = np.asarray(pixels, np.float64)
    covered = np.asarray(covered, np.uint32)
    known = (covered & COVERED_UNKNOWN) == 0
    cnt = (covered & ~np.uint32(COVERED_UNKNOWN)).astype(np.float64)
    ok = known & (cnt > 0)
    out = np.full(covered.shape, -1.0, np.float32)
    out[ok] = (1.0 - pixels[ok] / cnt[ok]).astype(np.float32)
    return out


def bbox3d_records(scene, object_frames: Sequence[np.ndarray], inst_stats: Optional[np.ndarray] = None,
                   covered: Optional[np.ndarray] = None) -> np.ndarray:
    """Replicator-style bounding_box_3d data for every labelled object;
    ``occlusionRatio`` from the frame's label statistics and coverage when
    given (else -1)."""
    occ = None
    if inst_stats is not None and covered is not None:
        occ = occlusion_ratios(np.asarray(inst_stats)[:, 0], covered)
    rec = np.zeros(len(scene.objects), BBOX3D_DTYPE)
    for j, o in enumerate(scene.objects):
        lo, hi = o.local_bounds if o.local_bounds is not None else (np.zeros(3), np.zeros(3))
        rec[j]["semanticId"] = o.class_id
        rec[j]["x_min"], rec[j]["y_min"], rec[j]["z_min"] = lo
        rec[j]["x_max"], rec[j]["y_max"], rec[j]["z_max"] = hi
        rec[j]["transform"] = np.asarray(object_frames[j]).T       # USD row-vector convention
        rec[j]["occlusionRatio"] = occ[o.inst_idx] if occ is not None and o.inst_idx < occ.shape[0] else -1.0
    return rec


def bboxDict_to_transform(bbox) -> tuple:
    """(center_world[3], size_world[3], euler_xyz_deg[3]) of one record (:553-584)."""
    corner = np.array([[bbox[1], bbox[2], bbox[3]], [bbox[4], bbox[5], bbox[6]]], dtype=np.float64)
    T = np.asarray(bbox[7], dtype=np.float64).reshape(4, 4).T
    center = (T @ np.append(corner.mean(axis=0), 1.0))[:3]
    rot = T[:3, :3]
    U, _, Vt = np.linalg.svd(rot)
    euler = Rotation.from_matrix(U @ Vt).as_euler("xyz", degrees=True)
    scale = np.linalg.norm(rot, axis=0)
    size = scale * np.abs(corner[1] - corner[0])
    return center.tolist(), size.tolist(), euler.tolist()


def object_poses(scene, object_frames) -> List[dict]:
    """Pose entries of every object (cache per randomisation epoch):
    bboxDict_to_transform (:553-584) of every record at once (stacked SVD and
    rotation conversion; the per-record function above is the restatement the
    golden vectors pin, this agrees with it to ~1e-15)."""
    recs = bbox3d_records(scene, object_frames)
    if len(recs) == 0:
        return []
    lo = np.stack([recs["x_min"], recs["y_min"], recs["z_min"]], 1).astype(np.float64)
    hi = np.stack([recs["x_max"], recs["y_max"], recs["z_max"]], 1).astype(np.float64)
    T = recs["transform"].astype(np.float64).transpose(0, 2, 1)
    mean = np.concatenate([(lo + hi) / 2.0, np.ones((len(recs), 1))], 1)
    center = np.einsum("nij,nj->ni", T, mean)[:, :3]
    rot = T[:, :3, :3]
    U, _, Vt = np.linalg.svd(rot)
    euler = Rotation.from_matrix(U @ Vt).as_euler("xyz", degrees=True)
    size = np.linalg.norm(rot, axis=1) * np.abs(hi - lo)
    return [{"inst_idx": o.inst_idx, "class_id": o.class_id, "class_name": o.class_name,
             "center": c, "size": sz, "rotation": e, "prim_path": o.prim_path}
            for o, c, sz, e in zip(scene.objects, center.tolist(), size.tolist(), euler.tolist())]


OBJECT_LISTS = ("visible", "frustum")


def in_frustum(scene, object_frames: Sequence[np.ndarray], view: np.ndarray, proj: np.ndarray, width: int,
               height: int, near: float, far: float) -> np.ndarray:
    """Per object of ``scene.objects``: does its 3D box (local bounds under
    its object frame, the bounding_box_3d record) meet the view frustum?  A
    box is outside when all 8 corners fail the same clip plane (W < near,
    W > far, u < 0, u > width, v < 0, v > height in the pixel projection's
    homogeneous rows 0, 1, 3); otherwise it counts as inside (conservative).
    Objects without bounds are tested as the point at their origin."""
    n = len(scene.objects)
    out = np.zeros(n, bool)
    if n == 0:
        return out
    lo = np.zeros((n, 3))
    hi = np.zeros((n, 3))
    for j, o in enumerate(scene.objects):
        if o.local_bounds is not None:
            lo[j], hi[j] = o.local_bounds
    sel = np.array([[(c >> 0) & 1, (c >> 1) & 1, (c >> 2) & 1] for c in range(8)], np.float64)
    corners = lo[:, None, :] + sel[None] * (hi - lo)[:, None, :]                  # [n][8][3]
    M = np.asarray(object_frames, np.float64).reshape(n, 4, 4)
    world = np.einsum("nij,nkj->nki", M[:, :3, :3], corners) + M[:, None, :3, 3]
    PV = np.asarray(proj, np.float64).reshape(4, 4) @ np.asarray(view, np.float64).reshape(4, 4)
    clip = np.einsum("ij,nkj->nki", PV, np.concatenate([world, np.ones((n, 8, 1))], 2))
    X, Y, Wc = clip[..., 0], clip[..., 1], clip[..., 3]
    outside = ((Wc < near).all(1) | (Wc > far).all(1) | (X < 0).all(1) | (X > width * Wc).all(1)
               | (Y < 0).all(1) | (Y > height * Wc).all(1))
    return ~outside


def label_record(frame_id: int, camera_pose: Sequence[float], camera_params: dict, poses: List[dict],
                 inst_stats: Optional[np.ndarray], kp_uv: Optional[np.ndarray], kp_vis: Optional[np.ndarray],
                 kp_table: Optional[Sequence], height: int, width: int,
                 covered: Optional[np.ndarray] = None, listed: Optional[Sequence[bool]] = None) -> dict:
    """The label JSON of one frame (:2056-2064) for the objects visible in it
    (+ ``occlusion_ratio`` per object when the coverage is given).

    Which objects are listed.  The reference lists the ``bounding_box_3d``
    annotator's primPaths (GDP:1780-1906); Replicator's inclusion rule for
    that list is closed.  By default ("visible") this build lists the objects
    with at least one visible pixel.  With ``listed`` (per object of
    ``poses``: e.g. :func:`in_frustum`, the "frustum" object list) those
    objects are listed too when no pixel of them is visible: pixel_count 0,
    bbox_2d [-1, -1, -1, -1] and occlusion_ratio 1.0 (-1.0 when the coverage
    is unknown)."""
    occ = occlusion_ratios(inst_stats[:, 0], covered) if inst_stats is not None and covered is not None else None
    cov_known = ((np.asarray(covered, np.uint32) & COVERED_UNKNOWN) == 0).tolist() if occ is not None else None
    occ = occ.tolist() if occ is not None else None
    objs = []
    kp_by_obj: Dict[int, list] = {}
    if kp_uv is not None and kp_table is not None:
        # (tolist: Python floats / ints of the same values, without a per-element numpy access)
        for (j, name), (u, v), vis in zip(kp_table, kp_uv.tolist(), kp_vis.tolist()):
            kp_by_obj.setdefault(j, []).append([name, u, v, vis])
    stats = inst_stats.tolist() if inst_stats is not None else None
    for j, p in enumerate(poses):
        i = p["inst_idx"]
        hidden = False
        if stats is not None:
            if i >= len(stats):
                continue
            hidden = stats[i][0] == 0
            if hidden and not (listed is not None and listed[j]):
                continue
        e = dict(p)
        if stats is not None:
            st = stats[i]
            e["pixel_count"] = st[0]
            e["bbox_2d"] = [-1, -1, -1, -1] if hidden else st[1:5]
            if occ is not None:
                e["occlusion_ratio"] = (1.0 if cov_known[i] else -1.0) if hidden else occ[i]
        if j in kp_by_obj:
            e["keypoints_2d"] = kp_by_obj[j]
        objs.append(e)
    return {
        "frame_id": int(frame_id),
        "camera_pose": [float(x) for x in camera_pose],
        "camera_params": camera_params,
        "objects": objs,
        "instance_mask_shape": [int(height), int(width)],
        "num_objects": len(objs),
        "class_mapping": dict(CONSTRUCTION_CLASS),
    }


_JSON = None


def json_encoder():
    """The native encoder (_csgjson.so, csrc/csg_json.cpp): the bytes of
    ``json.dumps(obj, indent=2, ensure_ascii=False)``, ~30x faster than the
    standard library's pure-Python indented encoder; built on first use."""
    global _JSON
    if _JSON is None:
        import importlib
        from .build import JSON_EXT, JSON_SOURCES, build_json, needs_build
        if needs_build(JSON_EXT, JSON_SOURCES):
            build_json()
        _JSON = importlib.import_module(__package__ + "._csgjson")
    return _JSON


def label_json_bytes(label: dict) -> bytes:
    """The label file's bytes, exactly as save_label_json (GDP:608-613) writes them."""
    return json_encoder().dumps_indent2(label)


def save_label_json(label: dict, filename: str) -> None:
    """save_label_json of the reference (GDP:608-613): ``json.dump(indent=2,
    ensure_ascii=False)`` to a UTF-8 file, through the native encoder."""
    data = label_json_bytes(label)
    with open(filename, "wb") as f:
        f.write(data)
