"""The instance ids' host wire (round 6, csg_host_id_bytes).

The reference hands its caller an int32 instance mask
(generate_construction_data.py:1909-1910) and saves it as an int32 `.npy`
(:2066-2069).  A host-output batch sends the ids over PCIe as (id + 1) in one
byte when every label is in [-1, 254] (two bytes up to 65,534; the 300-label
scene of test_gpu_parity.test_many_labels_stats takes that path against the
oracle), and host threads widen them into the caller's int32 array before the
batch's stream completes.  Here: the widened ids equal the int32 wire's
(CSG_NARROW_IDS=0) and the device-output path's, byte for byte, for pageable
and page-locked host arrays, one launch chain and several (CSG_SPLIT_PAGEABLE),
synchronous and asynchronous batches; and the `.npy` the generator writes from them is
byte-identical to the one written from the int32 path.
"""
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _workload():
    from constructionsceneposeestimation_amd.workload import Workload
    return Workload("C3", seed=3, width=480, height=272)


def _renderer(wl, n, narrow, split_pageable=True):
    """A renderer whose context reads CSG_NARROW_IDS / CSG_SPLIT_PAGEABLE at create."""
    from constructionsceneposeestimation_amd.renderer import Renderer
    env = {"CSG_NARROW_IDS": "1" if narrow else "0", "CSG_SPLIT_PAGEABLE": "1" if split_pageable else "0"}
    old = {k: os.environ.get(k) for k in env}
    os.environ.update(env)
    try:
        r = Renderer(wl.scene, wl.width, wl.height, max_frames=n)
    finally:
        for k, v in old.items():
            if v is None:
                del os.environ[k]
            else:
                os.environ[k] = v
    return r


def _setup(r, wl, fids):
    epochs = sorted({f // 10 for f in fids})
    for k, e in enumerate(epochs):
        st = wl.epoch(e)
        r.set_instance_transforms(k, st.models)
        r.set_keypoints(k, st.keypoints)
    from constructionsceneposeestimation_amd.renderer import make_frames
    V, P = wl.frame_params(fids)
    return make_frames(V, P, [epochs.index(f // 10) for f in fids], fids)


def _pinned_out(r, n, want):
    out = {}
    for k, (shape, dt) in r.output_spec(n, want).items():
        nb = int(np.prod(shape)) * np.dtype(dt).itemsize
        out[k] = r.host_buffer(nb).view(dt).reshape(shape)
    return out


def test_narrow_wire_matches_int32_wire_and_device_outputs(tmp_path):
    import torch
    from constructionsceneposeestimation_amd import writers
    wl = _workload()
    fids = list(range(0, 400, 5))   # 80 frames: with page-locked outputs, launch chains of 32, 32, 16
    n, H, W = len(fids), wl.height, wl.width
    want = ("rgb", "instance", "keypoints")
    with _renderer(wl, n, True) as a, _renderer(wl, n, False, split_pageable=False) as b, \
            _renderer(wl, n, True, split_pageable=False) as c:
        assert a.host_id_bytes() == 1 and c.host_id_bytes() == 1, "C3's labels fit one byte"
        assert b.host_id_bytes() == 4
        fa, fb, fc = _setup(a, wl, fids), _setup(b, wl, fids), _setup(c, wl, fids)
        wide = b.render(fb, want=want)                      # int32 on the wire (pageable, one chain)
        narrow = a.render(fa, want=want)                     # narrowed (pageable: chains of 32, 32, 16)
        narrow1 = c.render(fc, want=want)                    # narrowed (pageable, one chain)
        pin = a.render(fa, want=want, out=_pinned_out(a, n, want))   # narrowed, page-locked: chains overlap
        pin = {k: v.copy() for k, v in pin.items()}   # (the page-locked buffers are freed with the renderer)
        # the device-output path (no wire at all)
        dev = torch.device("cuda", 0)
        fdev = torch.from_numpy(fa.view(np.uint8).copy()).to(dev)
        rgb = torch.empty((n, H, W, 3), dtype=torch.uint8, device=dev)
        inst = torch.empty((n, H, W), dtype=torch.int32, device=dev)
        a.render_into(fdev.data_ptr(), n, True, rgb.data_ptr(), inst.data_ptr(),
                      stream=torch.cuda.current_stream(dev).cuda_stream)
        torch.cuda.synchronize(dev)
        a.synchronize()
        dinst = inst.cpu().numpy()
        # an asynchronous host-output batch: the ids are in place once the stream is done
        a_inst = a.host_buffer(n * H * W * 4).view(np.int32).reshape(n, H, W)
        a_inst[:] = 7
        from constructionsceneposeestimation_amd import _lib
        import ctypes as C
        o = _lib.Outputs(None, a_inst.ctypes.data, None, None, None, None, a.n_labels, 0, None, None)
        a._check(a.lib.csg_render_batch_async(a.ctx, fa.ctypes.data, n, 0, C.byref(o), None), "async")
        a.synchronize()
        async_inst = a_inst.copy()
    for got in (narrow, narrow1, pin):
        assert got["instance"].dtype == np.int32
        assert np.array_equal(got["instance"], wide["instance"])
        assert np.array_equal(got["rgb"], wide["rgb"])
        assert np.array_equal(got["keypoints_vis"], wide["keypoints_vis"])
    assert np.array_equal(dinst, wide["instance"])
    assert np.array_equal(async_inst, wide["instance"])
    assert (wide["instance"] == -1).any() and (wide["instance"] >= 0).any()
    # the generator's int32 mask file (labels/instance_mask_XXXXXX.npy)
    pa, pb = str(tmp_path / "narrow.npy"), str(tmp_path / "wide.npy")
    writers.write_npy(pa, pin["instance"][3])
    writers.write_npy(pb, wide["instance"][3])
    assert open(pa, "rb").read() == open(pb, "rb").read()
    assert np.load(pa).dtype == np.int32
