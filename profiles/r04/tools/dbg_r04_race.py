"""Debug: render one C3 1080p batch repeatedly into device buffers filled with a
sentinel before each render; report pixels and keypoints no kernel wrote, and
keypoint visibility that changes between repetitions."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main(reps=12, sized=True):
    import torch
    from constructionsceneposeestimation_amd.renderer import Renderer, make_frames
    from constructionsceneposeestimation_amd.workload import Workload
    wl = Workload("C3", seed=0)
    fids = [0, 9, 131, 247, 388, 512, 777, 1023, 1500, 2047, 2222, 3001]
    epochs = sorted({f // 10 for f in fids})
    V, P = wl.frame_params(fids)
    fr = make_frames(V, P, [epochs.index(f // 10) for f in fids], fids)
    n, H, W = len(fids), wl.height, wl.width
    dev = torch.device("cuda", 0)
    with Renderer(wl.scene, W, H, max_frames=n) as r:
        for k, e in enumerate(epochs):
            st = wl.epoch(e)
            r.set_instance_transforms(k, st.models)
            r.set_keypoints(k, st.keypoints)
        fdev = torch.from_numpy(fr.view(np.uint8).copy()).to(dev)
        if sized:
            print("sized", r.size_work(fdev.data_ptr(), n, on_device=True))
        rgb = torch.empty((n, H, W, 3), dtype=torch.uint8, device=dev)
        inst = torch.empty((n, H, W), dtype=torch.int32, device=dev)
        uv = torch.empty((n, r.n_kp, 2), dtype=torch.float32, device=dev)
        vis = torch.empty((n, r.n_kp), dtype=torch.int32, device=dev)
        stream = torch.cuda.current_stream(dev).cuda_stream
        first = None
        for rep in range(reps):
            rgb.fill_(7); inst.fill_(7); uv.fill_(-7.0); vis.fill_(7)
            torch.cuda.synchronize(dev)
            r.render_into(fdev.data_ptr(), n, True, rgb.data_ptr(), inst.data_ptr(), kp_uv=uv.data_ptr(),
                          kp_vis=vis.data_ptr(), stream=stream)
            torch.cuda.synchronize(dev)
            r.synchronize()
            i = inst.cpu().numpy()
            v = vis.cpu().numpy()
            unwritten = np.argwhere(i == 7)
            tiles = sorted({(int(f), int(y) // 32, int(x) // 32) for f, y, x in unwritten})
            msg = f"rep {rep}: unwritten px {len(unwritten)} in tiles {tiles[:8]}, kp vis sentinel {int((v == 7).sum())}"
            if first is None:
                first = v.copy()
            else:
                d = np.argwhere(v != first)
                msg += f", kp vis changed {d.tolist()[:6]}"
            print(msg, flush=True)


if __name__ == "__main__":
    main()
