"""Debug: one C3 frame at 1080p with the working-tree library vs the oracle --
which outputs differ, where, and by how much (depth bits, rgb, ids, keypoints)."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main(frames):
    from constructionsceneposeestimation_amd.packing import pack_scene
    from constructionsceneposeestimation_amd.renderer import Renderer, make_frames
    from constructionsceneposeestimation_amd.workload import Workload
    from oracle.oracle import Oracle
    wl = Workload("C3", seed=0)
    o = Oracle(pack_scene(wl.scene), wl.width, wl.height)
    for f in frames:
        st = wl.epoch(f // 10)
        V, P = wl.frame_params([f])
        with Renderer(wl.scene, wl.width, wl.height, max_frames=1) as r:
            r.set_instance_transforms(0, st.models)
            r.set_keypoints(0, st.keypoints)
            g = r.render(make_frames(V, P, [0], [f]), want=("rgb", "instance", "depth", "keypoints"))
        o.set_instance_models(st.models.reshape(-1, 16))
        ref = o.render(V[0], P[0])
        uv, vis = o.keypoints(V[0], P[0], st.keypoints, ref["depth"])
        gd, od = g["depth"][0].view(np.uint32), ref["depth"].view(np.uint32)
        bad = np.argwhere(gd != od)
        print(f"frame {f}: depth px differ {len(bad)}, rgb {int((g['rgb'][0] != ref['rgb']).any(-1).sum())}, "
              f"inst {int((g['instance'][0] != ref['instance']).sum())}, "
              f"kp vis {np.nonzero(g['keypoints_vis'][0] != vis)[0].tolist()}, "
              f"kp uv {int((g['keypoints_uv'][0].view(np.uint32) != uv.view(np.uint32)).any(-1).sum())}")
        for y, x in bad[:8]:
            a, b = g["depth"][0][y, x], ref["depth"][y, x]
            print(f"   ({x},{y}) gpu {a!r} ({gd[y, x]:#x}) oracle {b!r} ({od[y, x]:#x}) inst {g['instance'][0][y, x]} "
                  f"/ {ref['instance'][y, x]}  1/d gpu {np.float32(1) / a!r} oracle {np.float32(1) / b!r}")


if __name__ == "__main__":
    main([int(x) for x in sys.argv[1:]] or [222])
