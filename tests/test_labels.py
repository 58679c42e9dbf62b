"""Label record schema and per-epoch poses (CPU)."""
import json

import numpy as np
import pytest

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


def test_native_label_json_matches_stdlib():
    """_csgjson.dumps_indent2 == json.dumps(indent=2, ensure_ascii=False) as
    UTF-8 (save_label_json, GDP:608-613): a full C3 label and edge values."""
    import json

    from constructionsceneposeestimation_amd import camera_math as cm
    from constructionsceneposeestimation_amd.labels import label_json_bytes, label_record, object_poses
    from constructionsceneposeestimation_amd.renderer import scene_labels
    from constructionsceneposeestimation_amd.workload import Workload
    wl = Workload("C3", seed=0)
    nl, K = scene_labels(wl.scene), wl.n_keypoints()
    st = wl.epoch(3)
    rng = np.random.default_rng(1)
    stats = rng.integers(0, 1000, (nl, 5)).astype(np.uint32)
    stats[::3, 0] = 0
    V, P, C, *_ = wl.camera(31)
    lab = label_record(31, cm.get_obj_pose_from_matrix(C), wl.intr.params(), object_poses(wl.scene, st.object_frames),
                       stats, (rng.random((K, 2)) * 2000 - 100).astype(np.float32), rng.integers(0, 3, K).astype(np.int32),
                       wl.kp_table, 1080, 1920, covered=rng.integers(0, 3000, nl).astype(np.uint32))
    assert lab["objects"] and label_json_bytes(lab) == json.dumps(lab, indent=2, ensure_ascii=False).encode()
    odd = {"s": 'q"\\\n\r\t\b\f\x01\x1f é 漢', "e": [], "d": {}, "n": None, "t": True, "f": False,
           "k": {1: 2, 2.5: 3, True: 4, None: 5, -7: [1e16, 1e15, 1e-5, 1e-4, -0.0, 0.0, 5e-324, 2 ** 70]},
           "nan": [float("nan"), float("inf"), -float("inf")], "tuple": (1, (2.5, "x"))}
    assert label_json_bytes(odd) == json.dumps(odd, indent=2, ensure_ascii=False).encode()
    with pytest.raises(TypeError):
        label_json_bytes({"x": object()})


def test_native_float_repr_random_doubles():
    from constructionsceneposeestimation_amd.labels import json_encoder
    m = json_encoder()
    rng = np.random.default_rng(5)
    xs = rng.integers(0, 2 ** 64 - 1, 50000, dtype=np.uint64).view(np.float64)
    xs = np.concatenate([xs[np.isfinite(xs)], rng.standard_normal(20000) * 10.0 ** rng.integers(-20, 20, 20000),
                         rng.random(20000).astype(np.float32).astype(np.float64)])
    bad = [x for x in xs.tolist() if m.repr_float(x) != repr(x)]
    assert not bad, bad[:5]


def test_quality_log_depth_mean_vs_reference_float32_mean():
    """The quality log's depth_mean (float64 sum / count, from the GPU's
    depth_stats) against the reference's np.mean of the float32 valid depths
    (GDP:324-328): a documented divergence in the low digits only."""
    from constructionsceneposeestimation_amd.writers import depth_stats
    rng = np.random.default_rng(3)
    d = rng.uniform(0.5, 250.0, (1080, 1920)).astype(np.float32)
    d[rng.random(d.shape) < 0.3] = np.inf
    ds = depth_stats(d)
    ours = ds["sum"] / ds["valid"]
    ref = float(np.mean(d[np.isfinite(d) & (d > 0)]))
    assert abs(ours - ref) <= 1e-6 * ref


def test_retry_offsets_follow_the_reference_jitter():
    """GDP:1574-1579: offset = uniform(-2, 2, 3), z halved; here from a counter
    stream keyed by (seed, frame, attempt): reproducible, independent per attempt."""
    from constructionsceneposeestimation_amd import schedule
    offs = np.array([schedule.retry_offset(0, f, a) for f in range(200) for a in range(1, 5)])
    assert np.abs(offs[:, :2]).max() <= 2.0 and np.abs(offs[:, 2]).max() <= 1.0
    assert np.abs(offs[:, :2]).max() > 1.9 and np.abs(offs[:, 2]).max() > 0.9
    assert np.array_equal(schedule.retry_offset(0, 7, 2), schedule.retry_offset(0, 7, 2))
    assert not np.array_equal(schedule.retry_offset(0, 7, 2), schedule.retry_offset(0, 7, 3))
    assert not np.array_equal(schedule.retry_offset(0, 7, 2), schedule.retry_offset(1, 7, 2))


def test_retried_camera_is_jittered_and_pitched():
    from constructionsceneposeestimation_amd import schedule
    from constructionsceneposeestimation_amd.workload import Workload
    wl = Workload("C3", seed=0, width=160, height=96)
    V0, P0, C0, cam0, aim0, q0 = wl.camera(12)
    V2, P2, C2, cam2, aim2, q2 = wl.camera(12, 2)
    assert np.allclose(cam2, cam0 + schedule.retry_offset(0, 12, 2)) and np.array_equal(aim2, aim0)
    assert abs(cam0[2] - aim0[2]) < 1e-12 and abs(cam2[2] - aim2[2]) > 1e-6   # level shot -> pitched
    fwd = C2[:3, :3] @ np.array([0.0, 0.0, -1.0])                             # USD camera looks down -Z
    d = (aim2 - cam2) / np.linalg.norm(aim2 - cam2)
    assert np.allclose(fwd, d, atol=1e-9)
    V, P = wl.frame_params([12, 13], attempts=[2, 0])
    assert np.array_equal(V[0], V2) and np.array_equal(V[1], wl.camera(13)[0])


def test_quality_log_counts_validation_retries(tmp_path):
    """The reference's retry bookkeeping (log_retry :278-283, log_pointcloud
    :285-300, log_frame_end :374-387): a frame that passed on its third
    attempt has retry_count 2 and two failed point-cloud checks; one that
    failed all five attempts is 'failed' with retry_count 4 (the fifth check
    ends the loop without a retry)."""
    from constructionsceneposeestimation_amd.quality_log import QualityLog
    log = QualityLog(str(tmp_path))
    ds = {"valid": 500, "total": 1000, "zero": 0, "inf": 500, "sum": 1000.0, "min": 1.0, "max": 3.0}
    rec = log.frame(n_objects=2, frame_id=3, cam_pos=[0, 0, 1], depth_stats=ds, points=500, failed_checks=[0, 40])
    assert rec["retry_count"] == 2 and rec["status"] == "success"
    bad = log.frame_failed(4, [1, 1, 1], [0, 0, 10, 0, 5])
    assert bad["retry_count"] == 4 and bad["status"] == "failed"
    st = log.statistics()
    assert st["retry_count"] == 6 and st["failed_frames"] == 1 and st["successful_frames"] == 1
    assert st["total_frames_attempted"] == 2
    assert st["pointcloud_stats"] == {"valid": 1, "empty": 4, "insufficient": 3}
    log.save()
    text = open(tmp_path / "generation_detail.log").read()
    assert text.count("! retry") == 6 and "frame 4 failed" in text
