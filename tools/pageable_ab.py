"""A/B of launch-chain splitting for pageable host outputs.

Renderer.render with the default pageable numpy outputs (RGB8, int32 ids,
keypoints), C3 1080p, one batch of F frames: one launch chain
(CSG_SPLIT_PAGEABLE=0) against chains of F/8 frames (the default since this
A/B: a pageable copy blocks the host, so later chains do not render under it,
but each chain's narrowed ids are widened while the next chain copies).  And
the same batch into page-locked outputs.  Median of 5 after one warm-up; prints one JSON line.

    python tools/pageable_ab.py --frames 480
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=480)
    ap.add_argument("--reps", type=int, default=5)
    a = ap.parse_args()
    import numpy as np
    from constructionsceneposeestimation_amd.renderer import Renderer, make_frames
    from constructionsceneposeestimation_amd.workload import Workload
    wl = Workload("C3", seed=0)
    fids = list(range(a.frames))
    want = ("rgb", "instance", "keypoints")
    res = {"workload": "C3", "width": wl.width, "height": wl.height, "frames": a.frames, "want": list(want),
           "method": f"median of {a.reps} after 1 warm-up, wall clock around Renderer.render"}

    def timed(r, fr, out=None):
        r.render(fr, want=want, out=out)
        ts = []
        for _ in range(a.reps):
            t0 = time.perf_counter()
            r.render(fr, want=want, out=out)
            ts.append(time.perf_counter() - t0)
        ts.sort()
        return ts[len(ts) // 2]

    for name, env in (("pageable_one_chain", "0"), ("pageable_split", "1")):
        os.environ["CSG_SPLIT_PAGEABLE"] = env
        with Renderer(wl.scene, wl.width, wl.height, max_frames=a.frames) as r:
            epochs = sorted({f // 10 for f in fids})
            for k, e in enumerate(epochs):
                st = wl.epoch(e)
                r.set_instance_transforms(k, st.models)
                r.set_keypoints(k, st.keypoints)
            V, P = wl.frame_params(fids)
            fr = make_frames(V, P, [epochs.index(f // 10) for f in fids], fids)
            t = timed(r, fr)
            res[name] = {"seconds": round(t, 4), "frames_per_s": round(a.frames / t, 1)}
            if env == "0":   # page-locked outputs: split into copy chains
                out = {}
                for k, (shape, dt) in r.output_spec(a.frames, want).items():
                    nb = int(np.prod(shape)) * np.dtype(dt).itemsize
                    out[k] = r.host_buffer(nb).view(dt).reshape(shape)
                t = timed(r, fr, out)
                res["page_locked_split"] = {"seconds": round(t, 4), "frames_per_s": round(a.frames / t, 1)}
                del out
    os.environ.pop("CSG_SPLIT_PAGEABLE", None)
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
