"""Rate of the GPU file encoders (csg_outputs.file_kinds) on C3 at 1080p:
synchronous render + encode + copy of the packed files to pinned host memory,
per batch, against the same render without files; and the encoded bytes.

    python tools/files_bench.py --batch 30 --batches 8
"""
import argparse
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from constructionsceneposeestimation_amd.renderer import Renderer, make_frames
    from constructionsceneposeestimation_amd.workload import Workload
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=30)
    ap.add_argument("--batches", type=int, default=8)
    ap.add_argument("--kinds", default="rgb_png,depth_csv,depth_png,pointcloud_txt")
    a = ap.parse_args()
    kinds = tuple(a.kinds.split(","))
    wl = Workload("C3", seed=0)
    F = a.batch
    want = ("keypoints", "stats", "covered", "depth_stats", "instance", "depth_range")
    with Renderer(wl.scene, wl.width, wl.height, max_frames=F) as r:
        batches = []
        for b in range(a.batches + 1):
            fb = list(range(1200 + b * F, 1200 + (b + 1) * F))
            epochs = sorted({f // 10 for f in fb})
            batches.append((fb, epochs, wl.frame_params(fb)))
        r.set_keypoints(0, wl.epoch(120).keypoints)   # (the keypoint count shapes the outputs)
        per_px = {"rgb_png": 3, "depth_csv": 12, "depth_png": 3, "pointcloud_txt": 72}   # upper estimates
        files = r.host_buffer(F * sum(per_px[k] for k in kinds) * wl.width * wl.height)
        spec = r.output_spec(F, want)
        host = {}
        for k, (shape, dt) in spec.items():
            buf = r.host_buffer(int(np.prod(shape)) * np.dtype(dt).itemsize)
            host[k] = np.ndarray(shape, dt, buffer=buf)
        res = {}
        for mode in ("render", "files"):
            ts, nbytes = [], 0
            for b, (fb, epochs, (V, P)) in enumerate(batches):
                for k, e in enumerate(epochs):
                    st = wl.epoch(e)
                    r.set_instance_transforms(k, st.models)
                    r.set_keypoints(k, st.keypoints)
                fr = make_frames(V, P, [epochs.index(f // 10) for f in fb], fb)
                t0 = time.perf_counter()
                if mode == "render":
                    r.render(fr, want=want, out=host)
                else:
                    out, off, need = r.render_files(fr, kinds, files, want=want, out=host)
                    assert off is not None, need
                    nbytes += need
                if b:   # first batch: warm-up
                    ts.append(time.perf_counter() - t0)
            ms = 1e3 * float(np.median(ts))
            res[mode] = {"ms_per_batch": round(ms, 2), "frames_per_s": round(F * 1e3 / ms, 1)}
            if mode == "files":
                res[mode]["file_bytes_per_frame"] = round(nbytes / (F * (len(batches))))
        res["encode_and_copy_ms_per_frame"] = round((res["files"]["ms_per_batch"] - res["render"]["ms_per_batch"]) / F, 3)
        res.update({"batch": F, "kinds": kinds, "workload": "C3 1920x1080", "host_outputs": list(want)})
        print(json.dumps(res))


if __name__ == "__main__":
    main()
