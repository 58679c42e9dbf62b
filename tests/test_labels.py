"""Label record schema and per-epoch poses (CPU)."""
import json

import numpy as np

from constructionsceneposeestimation_amd.labels import bbox3d_records, label_record, object_poses
from constructionsceneposeestimation_amd.workload import Workload

REF_KEYS = ["frame_id", "camera_pose", "camera_params", "objects", "instance_mask_shape", "num_objects",
            "class_mapping"]                       # generate_construction_data.py:2056-2064
REF_OBJ_KEYS = ["inst_idx", "class_id", "class_name", "center", "size", "rotation", "prim_path"]  # :1938-1946
REF_CAM_KEYS = ["horizontal_aperture", "vertical_aperture", "focal_length", "width", "height"]      # :2039-2045


def test_label_schema_matches_reference():
    wl = Workload("C3", seed=0, width=64, height=36)
    st = wl.epoch(3)
    poses = object_poses(wl.scene, st.object_frames)
    stats = np.zeros((len(wl.scene.objects), 5), np.uint32)
    stats[[0, 40], 0] = 5
    kuv = np.zeros((wl.n_keypoints(), 2), np.float32)
    kvis = np.ones(wl.n_keypoints(), np.int32)
    lab = label_record(31, [1, 2, 3, 0, 0, 0, 1], wl.intr.params(), poses, stats, kuv, kvis, wl.kp_table, 36, 64)
    assert list(lab) == REF_KEYS
    assert list(lab["camera_params"]) == REF_CAM_KEYS
    assert lab["num_objects"] == 2 and [o["inst_idx"] for o in lab["objects"]] == [0, 40]
    for o in lab["objects"]:
        assert list(o)[:7] == REF_OBJ_KEYS
    json.dumps(lab)
    # camera params: vertical aperture = hA * H / W (:2038)
    assert abs(lab["camera_params"]["vertical_aperture"] - 25.0 * 36 / 64) < 1e-12


def test_bbox_records_roundtrip_object_frames():
    wl = Workload("C3", seed=0, width=64, height=36)
    st = wl.epoch(5)
    recs = bbox3d_records(wl.scene, st.object_frames)
    poses = object_poses(wl.scene, st.object_frames)
    for j, (r, p) in enumerate(zip(recs, poses)):
        F = st.object_frames[j]
        lo, hi = wl.scene.objects[j].local_bounds
        c = F[:3, :3] @ ((lo + hi) / 2) + F[:3, 3]
        np.testing.assert_allclose(p["center"], c, rtol=1e-5, atol=1e-4)
