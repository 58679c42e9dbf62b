"""GPU outputs tied to the reference's own camera math.

The reference's only in-repo pinhole code is ``depth_to_pointcloud_with_rgb``
(generate_construction_data.py:616-711): fx = W*f/hA, fy = H*f/vA, cx = W/2,
cy = H/2 (:646-649), pixels at integer (u, v), camera coordinates X right /
Y down / Z forward multiplied directly by the USD camera rotation of the
label's ``camera_pose`` (:668-685) -- which mirrors the cloud.  Its
restatement ``pointcloud.depth_to_pointcloud_with_rgb`` is golden-pinned to
the reference (tests/golden/pointcloud.npz, test_golden.py).

Here the GPU's depth, RGB and fused world points, and the GPU keypoint
projection, are fed through that pinned function with the label record's own
``camera_pose`` (get_obj_pose, :587-605) and ``camera_params`` (:2039-2045),
and compared after mapping the GPU's USD-convention points onto the
reference's mirrored convention (pixel centre vs integer pixel, Y and Z
flipped).

Stated tolerances (float32 GPU arithmetic vs the reference's float64):
* points: |delta| <= 2e-4 m + 2e-6 x distance, pixel selection and RGB exact
  (320x180 and the headline 1920x1080);
* keypoint uv: <= 2e-3 px x (width / 640) x max(1, 2 m / Z) (Z = distance to the image plane);
  visibility class exact away from the image border and pixel boundaries.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _render(wl, frame, want):
    from constructionsceneposeestimation_amd.renderer import Renderer, make_frames
    st = wl.epoch(frame // 10)
    V, P = wl.frame_params([frame])
    with Renderer(wl.scene, wl.width, wl.height, max_frames=1) as r:
        r.set_instance_transforms(0, st.models)
        r.set_keypoints(0, st.keypoints)
        out = r.render(make_frames(V, P, [0], [frame]), want=want)
    return st, {k: v[0] for k, v in out.items()}


@pytest.mark.parametrize("frame,size", [(3, (320, 180)), (47, (320, 180)), (1234, (320, 180)),
                                        (47, (1920, 1080))])   # and at the headline size (C3 1080p)
def test_gpu_points_match_reference_pointcloud_convention(frame, size):
    from constructionsceneposeestimation_amd import camera_math as cm
    from constructionsceneposeestimation_amd.pointcloud import depth_to_pointcloud_with_rgb
    from constructionsceneposeestimation_amd.workload import Workload
    wl = Workload("C3", seed=0, width=size[0], height=size[1])
    _, out = _render(wl, frame, ("rgb", "depth", "points"))
    C = wl.camera(frame)[2]
    pose = cm.get_obj_pose_from_matrix(C)        # the label's camera_pose (GDP:587-605, :2058)
    params = wl.intr.params()                    # the label's camera_params (GDP:2039-2045)
    ref = depth_to_pointcloud_with_rgb(out["depth"], out["rgb"], params, pose)
    d = out["depth"]
    valid = np.isfinite(d) & (d > 0) & (d < 250)
    assert ref is not None and ref.shape[0] == int(valid.sum()) > 2000
    # the GPU's world point -> USD camera coordinates -> the reference's mirrored pinhole coordinates
    R, t = C[:3, :3], C[:3, 3]
    pc = (out["points"][valid].astype(np.float64) - t) @ R
    dd = d[valid].astype(np.float64)
    fx = params["width"] * params["focal_length"] / params["horizontal_aperture"]     # GDP:646
    fy = params["height"] * params["focal_length"] / params["vertical_aperture"]      # GDP:647
    mirrored = np.stack([pc[:, 0] - 0.5 * dd / fx, -pc[:, 1] - 0.5 * dd / fy, -pc[:, 2]], 1)
    world = mirrored @ R.T + t
    err = np.linalg.norm(world - ref[:, :3], axis=1)
    assert err.max() <= 2e-4 + 2e-6 * dd.max(), float(err.max())
    assert np.array_equal(ref[:, 3:].astype(np.uint8), out["rgb"][valid])
    # and the GPU points themselves sit on the pinhole rays of GDP:646-649 (USD convention)
    u = np.nonzero(valid)[1] + 0.5
    v = np.nonzero(valid)[0] + 0.5
    np.testing.assert_allclose(pc[:, 0], (u - params["width"] / 2.0) * dd / fx, atol=2e-4 + 2e-6 * dd.max())
    np.testing.assert_allclose(-pc[:, 1], (v - params["height"] / 2.0) * dd / fy, atol=2e-4 + 2e-6 * dd.max())


@pytest.mark.parametrize("size", [(640, 360), (1920, 1080)])
def test_gpu_keypoints_match_reference_pinhole(size):
    from constructionsceneposeestimation_amd.workload import Workload
    wl = Workload("C3", seed=0, width=size[0], height=size[1])
    p = wl.intr.params()
    fx = p["width"] * p["focal_length"] / p["horizontal_aperture"]        # GDP:646-649
    fy = p["height"] * p["focal_length"] / p["vertical_aperture"]
    cx, cy = p["width"] / 2.0, p["height"] / 2.0
    n_in = 0
    for frame in (5, 333, 1201, 2047):
        st, out = _render(wl, frame, ("depth", "keypoints"))
        C = wl.camera(frame)[2]
        cam = (np.asarray(st.keypoints, np.float64) - C[:3, 3]) @ C[:3, :3]   # USD camera coordinates
        X, Y, Z = cam[:, 0], -cam[:, 1], -cam[:, 2]                            # pinhole: X right, Y down, Z forward
        front = Z >= 0.5 + 1e-4
        u = fx * X[front] / Z[front] + cx
        v = fy * Y[front] / Z[front] + cy
        uv = out["keypoints_uv"][front].astype(np.float64)
        # float32 view-transform rounding (~1e-7 x |p|) grows as 1/Z for keypoints close to the camera,
        # and in pixels with the focal length (the image width)
        tol = 2e-3 * (p["width"] / 640.0) * np.maximum(1.0, 2.0 / Z[front])
        err = np.abs(uv - np.stack([u, v], 1)).max(axis=1)
        assert (err <= tol).all(), f"worst error {float(err.max()):.3g} px, worst error / tolerance {float((err / tol).max()):.3g}"
        vis = out["keypoints_vis"]
        assert (vis[Z < 0.5 - 1e-4] == 0).all()
        Wd, Hd = p["width"], p["height"]
        inside = (u >= 0) & (u < Wd) & (v >= 0) & (v < Hd)
        near_edge = (np.abs(u) < 1e-2) | (np.abs(u - Wd) < 1e-2) | (np.abs(v) < 1e-2) | (np.abs(v - Hd) < 1e-2)
        away = (np.abs(u - np.round(u)) > 1e-2) & (np.abs(v - np.round(v)) > 1e-2)   # off pixel boundaries
        vf = vis[front]
        assert ((vf > 0) == inside)[~near_edge].all()
        # visible (2) iff the keypoint's distance to the image plane is within the depth under it
        k = inside & away
        depth_at = out["depth"][np.floor(v[k]).astype(int), np.floor(u[k]).astype(int)]
        zk = Z[front][k]
        clear = np.abs(zk - depth_at) > 1e-3 * np.maximum(zk, 1.0)
        assert np.array_equal((vf[k] == 2)[clear], (zk <= depth_at)[clear])
        n_in += int(k.sum())
    assert n_in > 100
