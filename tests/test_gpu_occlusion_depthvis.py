"""GPU vs oracle for the depth visualisation and the occlusion coverage.

* ``depth_vis`` / ``depth_range`` (the reference's JET depth PNG,
  generate_construction_data.py:1690-1709): bit-exact against
  ``oracle.oracle.depth_vis`` applied to the (oracle-exact) depth, on the
  float4 path (1080p) and the per-pixel path (ragged size), with and without
  a depth output requested, and for a frame that hits nothing (black, NaN).
* ``label_covered`` (bounding_box_3d occlusionRatio, :1780-1790): bit-exact
  against the oracle's untiled coverage, on the headline C3 workload and on a
  300-label scene whose tiles overflow the 32-slot table (unknown flags).
"""
import numpy as np
import pytest

from tests.conftest import WORLD2_POSES, pose_frames

pytestmark = pytest.mark.gpu

UNKNOWN = 0x80000000


def _frames(views, projs):
    from constructionsceneposeestimation_amd.renderer import make_frames
    n = views.shape[0]
    return make_frames(views, projs, [0] * n, list(range(n)))


def _oracle(scene, W, H):
    from constructionsceneposeestimation_amd.packing import pack_scene
    from oracle.oracle import Oracle
    return Oracle(pack_scene(scene), W, H)


def _check_vis(gpu, k, depth):
    from oracle.oracle import depth_vis
    img, (lo, hi) = depth_vis(depth)
    assert np.array_equal(gpu["depth_vis"][k], img), \
        f"frame {k}: depth_vis differs at {np.argwhere((gpu['depth_vis'][k] != img).any(-1))[:5].tolist()}"
    assert np.array_equal(gpu["depth_range"][k], np.array([lo, hi], np.float32), equal_nan=True)


def test_depth_vis_world2_1080p(world2):
    from constructionsceneposeestimation_amd.renderer import Renderer
    W, H = 1920, 1080
    poses = WORLD2_POSES[:4] + [([0.0, 0.0, 400.0], [0.0, 0.0, 800.0])]   # last: looks at nothing
    views, projs = pose_frames(poses, W, H)
    o = _oracle(world2, W, H)
    with Renderer(world2, W, H, max_frames=len(poses)) as r:
        gpu = r.render(_frames(views, projs), want=("rgb", "depth", "depth_vis"))
        vis_only = r.render(_frames(views, projs), want=("depth_vis",))   # depth in internal scratch
    for k in range(len(poses)):
        ref = o.render(views[k], projs[k])
        assert np.array_equal(gpu["depth"][k].view(np.uint32), ref["depth"].view(np.uint32))
        _check_vis(gpu, k, ref["depth"])
        assert np.array_equal(vis_only["depth_vis"][k], gpu["depth_vis"][k])
    assert not gpu["depth_vis"][-1].any() and np.isnan(gpu["depth_range"][-1]).all()
    assert len(np.unique(gpu["depth_vis"][0].reshape(-1, 3), axis=0)) > 100


def test_depth_vis_ragged_size(world2):
    """203 x 117: npx % 4 != 0, so both kernels take the per-pixel path."""
    from constructionsceneposeestimation_amd.renderer import Renderer
    W, H = 203, 117
    views, projs = pose_frames(WORLD2_POSES[:3], W, H)
    o = _oracle(world2, W, H)
    with Renderer(world2, W, H, max_frames=3) as r:
        gpu = r.render(_frames(views, projs), want=("depth", "depth_vis"))
    for k in range(3):
        _check_vis(gpu, k, o.render(views[k], projs[k])["depth"])


def test_depth_vis_device_outputs(world2):
    """render_into with device buffers (no depth requested) == the host path."""
    import torch
    from constructionsceneposeestimation_amd.renderer import Renderer
    W, H, n = 640, 360, 4
    views, projs = pose_frames(WORLD2_POSES[:n], W, H)
    fr = _frames(views, projs)
    with Renderer(world2, W, H, max_frames=n) as r:
        host = r.render(fr, want=("depth_vis",))
        dv = torch.empty((n, H, W, 3), dtype=torch.uint8, device="cuda")
        dr = torch.empty((n, 2), dtype=torch.float32, device="cuda")
        r.render_into(fr.ctypes.data, n, False, depth_vis=dv.data_ptr(), depth_range=dr.data_ptr())
        r.synchronize()
    assert np.array_equal(dv.cpu().numpy(), host["depth_vis"])
    assert np.array_equal(dr.cpu().numpy(), host["depth_range"], equal_nan=True)


def test_label_covered_c3_1080p():
    from constructionsceneposeestimation_amd.packing import pack_scene
    from constructionsceneposeestimation_amd.renderer import Renderer, make_frames
    from constructionsceneposeestimation_amd.workload import Workload
    from oracle.oracle import Oracle
    wl = Workload("C3", seed=0)
    frames = [1203, 2417, 3001, 4650]
    V, P = wl.frame_params(frames)
    with Renderer(wl.scene, wl.width, wl.height, max_frames=len(frames)) as r:
        for k, f in enumerate(frames):
            r.set_instance_transforms(k, wl.epoch(f // 10).models)
        gpu = r.render(make_frames(V, P, list(range(len(frames))), frames),
                       want=("rgb", "instance", "stats", "covered"))
    o = Oracle(pack_scene(wl.scene), wl.width, wl.height)
    partly = 0
    for k, f in enumerate(frames):
        o.set_instance_models(wl.epoch(f // 10).models.reshape(-1, 16))
        ref = o.render(V[k], P[k], covered=True)
        assert np.array_equal(gpu["instance"][k], ref["instance"]), f"frame {f}: instance"
        cov, vis = gpu["label_covered"][k], gpu["inst_stats"][k][:, 0]
        assert np.array_equal(cov, ref["label_covered"]), \
            f"frame {f}: covered differs for labels {np.nonzero(cov != ref['label_covered'])[0].tolist()}"
        assert not (cov & UNKNOWN).any()
        assert (cov >= vis).all() and ((vis > 0) <= (cov > 0)).all()
        partly += int(((vis > 0) & (vis < cov)).sum())
    assert partly > 0, "some object must be partly occluded"


def test_label_covered_tile_overflow(cone):
    """300 labelled cones seen from afar: tiles hold more than 32 labels, whose
    coverage is flagged unknown (and counted nowhere), exactly as the oracle's
    untiled restatement decides it."""
    from constructionsceneposeestimation_amd.renderer import Renderer
    from constructionsceneposeestimation_amd.scene.model import Instance, Scene
    sc = Scene(meshes=cone.meshes, materials=cone.materials, textures=cone.textures, light=cone.light)
    base = np.asarray(cone.instances[0].model, np.float64)
    for k in range(300):
        m = base.copy()
        m[0, 3] += 0.35 * (k % 20 - 9.5)
        m[1, 3] += 0.35 * (k // 20)
        sc.instances.append(Instance(mesh=cone.instances[0].mesh, model=m, inst_idx=k))
    W, H = 320, 180
    views, projs = pose_frames([([0.0, -14.0, 4.0], [0.0, 3.0, 0.0]), ([0.0, -3.0, 2.0], [0.0, 2.0, 0.0])], W, H)
    o = _oracle(sc, W, H)
    with Renderer(sc, W, H, max_frames=2) as r:
        gpu = r.render(_frames(views, projs), want=("instance", "stats", "covered"))
    flagged = 0
    for k in range(2):
        ref = o.render(views[k], projs[k], covered=True)
        assert np.array_equal(gpu["instance"][k], ref["instance"])
        assert np.array_equal(gpu["label_covered"][k], ref["label_covered"])
        flagged += int((ref["label_covered"] & UNKNOWN != 0).sum())
    assert flagged > 0, "the far view must overflow some tile's label table"
