"""The asynchronous, device-resident path bench.py times (render_into with
device frame records and device outputs on the caller's stream), its sticky
error reporting, and the host staging ring -- bit-exact against the
synchronous host path and the oracle."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _workload():
    from constructionsceneposeestimation_amd.workload import Workload
    return Workload("C3", seed=1, width=480, height=272)


def _upload(r, wl, epochs):
    for k, e in enumerate(epochs):
        st = wl.epoch(e)
        r.set_instance_transforms(k, st.models)
        r.set_keypoints(k, st.keypoints)


def test_render_into_device_frames_multi_chain_matches_render_and_oracle():
    import torch
    from constructionsceneposeestimation_amd.packing import pack_scene
    from constructionsceneposeestimation_amd.renderer import FRAME_DTYPE, Renderer, make_frames
    from oracle.oracle import Oracle
    wl = _workload()
    fids = [3, 7, 14, 19, 25, 26, 31, 38, 42, 44, 51, 59]
    epochs = sorted({f // 10 for f in fids})
    V, P = wl.frame_params(fids)
    fr = make_frames(V, P, [epochs.index(f // 10) for f in fids], fids)
    n, H, W = len(fids), wl.height, wl.width
    dev = torch.device("cuda", 0)
    with Renderer(wl.scene, W, H, max_frames=n, frames_per_launch=5) as r:   # chains of 5, 5, 2
        _upload(r, wl, epochs)
        host = r.render(fr, want=("rgb", "instance", "keypoints"))
        frames_dev = torch.from_numpy(fr.view(np.uint8).copy()).to(dev)
        rgb = torch.full((n, H, W, 3), 7, dtype=torch.uint8, device=dev)
        inst = torch.full((n, H, W), 7, dtype=torch.int32, device=dev)
        uv = torch.zeros((n, r.n_kp, 2), dtype=torch.float32, device=dev)
        vis = torch.zeros((n, r.n_kp), dtype=torch.int32, device=dev)
        stream = torch.cuda.current_stream(dev).cuda_stream
        r.render_into(frames_dev.data_ptr(), n, True, rgb.data_ptr(), inst.data_ptr(), kp_uv=uv.data_ptr(),
                      kp_vis=vis.data_ptr(), stream=stream)
        torch.cuda.synchronize(dev)
        r.synchronize()
        assert FRAME_DTYPE.itemsize * n == frames_dev.numel()
    assert np.array_equal(rgb.cpu().numpy(), host["rgb"])
    assert np.array_equal(inst.cpu().numpy(), host["instance"])
    assert np.array_equal(uv.cpu().numpy().view(np.uint32), host["keypoints_uv"].view(np.uint32))
    assert np.array_equal(vis.cpu().numpy(), host["keypoints_vis"])
    o = Oracle(pack_scene(wl.scene), W, H)
    for k in (0, 6, n - 1):
        st = wl.epoch(fids[k] // 10)
        o.set_instance_models(st.models.reshape(-1, 16))
        ref = o.render(V[k], P[k])
        assert np.array_equal(host["rgb"][k], ref["rgb"]) and np.array_equal(host["instance"][k], ref["instance"])


def test_back_to_back_async_host_frames_keep_their_own_cameras():
    """Async batches of host frame records enqueued back to back (more than
    the staging ring holds) each render their own cameras."""
    import ctypes as C
    from constructionsceneposeestimation_amd import _lib
    from constructionsceneposeestimation_amd.renderer import Renderer, make_frames
    wl = _workload()
    batches = [[0, 1], [10, 11], [20, 21], [30, 31], [40, 41], [50, 51]]
    epochs = sorted({f // 10 for b in batches for f in b})
    H, W = wl.height, wl.width
    with Renderer(wl.scene, W, H, max_frames=2) as r:
        _upload(r, wl, epochs)
        expect = []
        for b in batches:
            V, P = wl.frame_params(b)
            expect.append(r.render(make_frames(V, P, [epochs.index(f // 10) for f in b], b), want=("rgb",))["rgb"])
        outs = [np.empty((2, H, W, 3), np.uint8) for _ in batches]
        keep = []
        for b, o in zip(batches, outs):
            V, P = wl.frame_params(b)
            fr = make_frames(V, P, [epochs.index(f // 10) for f in b], b)
            keep.append(fr)
            oo = _lib.Outputs()
            oo.rgb, oo.n_labels, oo.on_device = o.ctypes.data, r.n_labels, 0
            r._check(r.lib.csg_render_batch_async(r.ctx, fr.ctypes.data, 2, 0, C.byref(oo), None), "async")
            fr[:] = fr[::-1]          # the caller may reuse its records at once: the library staged them
        r.synchronize()
    for e, o in zip(expect, outs):
        assert np.array_equal(e, o)


def test_device_frame_with_bad_set_is_reported_then_cleared():
    import torch
    from constructionsceneposeestimation_amd._lib import CsgError
    from constructionsceneposeestimation_amd.renderer import Renderer, make_frames
    wl = _workload()
    dev = torch.device("cuda", 0)
    H, W = wl.height, wl.width
    with Renderer(wl.scene, W, H, max_frames=1) as r:
        _upload(r, wl, [0])
        V, P = wl.frame_params([5])
        rgb = torch.empty((1, H, W, 3), dtype=torch.uint8, device=dev)
        inst = torch.empty((1, H, W), dtype=torch.int32, device=dev)
        for bad in (4000, 1 << 31):
            fr = make_frames(V, P, [bad], [5])
            fd = torch.from_numpy(fr.view(np.uint8).copy()).to(dev)
            r.render_into(fd.data_ptr(), 1, True, rgb.data_ptr(), inst.data_ptr())
            with pytest.raises(CsgError, match="transform set"):
                r.synchronize()
        r.synchronize()               # the error was read and cleared
        good = r.render(make_frames(V, P, [0], [5]), want=("rgb", "instance"))
        fd = torch.from_numpy(make_frames(V, P, [0], [5]).view(np.uint8).copy()).to(dev)
        r.render_into(fd.data_ptr(), 1, True, rgb.data_ptr(), inst.data_ptr())
        torch.cuda.synchronize(dev)
        r.synchronize()
    assert np.array_equal(rgb.cpu().numpy(), good["rgb"]) and np.array_equal(inst.cpu().numpy(), good["instance"])


def test_overflow_is_sticky_across_async_batches(world2):
    """A batch that overflows its work buffers followed by one that does not:
    synchronize() still reports the first (the flag is only cleared once it
    has been read); the synchronous path then grows the buffers and renders
    the same frame bit-exact."""
    import torch
    from constructionsceneposeestimation_amd._lib import CsgError
    from constructionsceneposeestimation_amd.packing import pack_scene
    from constructionsceneposeestimation_amd.renderer import Renderer, make_frames
    from oracle.oracle import Oracle
    from tests.conftest import WORLD2_POSES, pose_frames
    W, H = 320, 180
    views, projs = pose_frames([WORLD2_POSES[0], ([0.0, 0.0, 5.0], [1.0, 0.0, 300.0])], W, H)  # dense, then sky
    dev = torch.device("cuda", 0)
    with Renderer(world2, W, H, max_frames=1, records_per_frame=1024, bins_per_frame=1024) as r:
        rgb = torch.empty((1, H, W, 3), dtype=torch.uint8, device=dev)
        inst = torch.empty((1, H, W), dtype=torch.int32, device=dev)
        fds = [torch.from_numpy(make_frames(views[k:k + 1], projs[k:k + 1], [0], [k]).view(np.uint8).copy()).to(dev)
               for k in range(2)]
        for fd in fds:
            r.render_into(fd.data_ptr(), 1, True, rgb.data_ptr(), inst.data_ptr())
        with pytest.raises(CsgError, match="overflow"):
            r.synchronize()
        r.synchronize()
        out = r.render(make_frames(views[:1], projs[:1], [0], [0]), want=("rgb", "instance", "depth"))
    ref = Oracle(pack_scene(world2), W, H).render(views[0], projs[0])
    assert np.array_equal(out["instance"][0], ref["instance"]) and np.array_equal(out["rgb"][0], ref["rgb"])


def test_misaligned_device_outputs_are_rejected_before_any_work():
    """k_raster writes 4-pixel groups as vector stores, so device outputs must be
    aligned (instance, depth, points 16 B; normals 8 B; rgb 4 B): a misaligned
    pointer fails the call with CSG_ERR_INVALID and nothing is written."""
    import torch
    from constructionsceneposeestimation_amd._lib import CsgError
    from constructionsceneposeestimation_amd.renderer import Renderer, make_frames
    wl = _workload()
    V, P = wl.frame_params([3])
    fr = make_frames(V, P, [0], [3])
    H, W = wl.height, wl.width
    dev = torch.device("cuda", 0)
    with Renderer(wl.scene, W, H, max_frames=1) as r:
        _upload(r, wl, [0])
        buf = torch.full((H * W * 3 + 8,), 7.0, dtype=torch.float32, device=dev)
        for kw in (dict(depth=buf.data_ptr() + 4), dict(points=buf.data_ptr() + 8), dict(normals=buf.data_ptr() + 2),
                   dict(instance=buf.data_ptr() + 4), dict(rgb=buf.data_ptr() + 1)):
            with pytest.raises(CsgError, match="aligned"):
                r.render_into(fr.ctypes.data, 1, False, **kw)
        r.synchronize()
        assert bool((buf == 7.0).all())
        # aligned: renders
        r.render_into(fr.ctypes.data, 1, False, depth=buf.data_ptr())
        r.synchronize()
        assert not bool((buf[: H * W] == 7.0).all())
