"""Print GPU vs oracle differences of the C5 outputs for one world2 pose (debug aid)."""
import numpy as np

from constructionsceneposeestimation_amd.packing import pack_scene
from constructionsceneposeestimation_amd.renderer import Renderer, make_frames
from constructionsceneposeestimation_amd.scene import load_world2
from oracle.oracle import Oracle
from tests.conftest import WORLD2_POSES, pose_frames

W, H = 640, 360
sc = load_world2()
views, projs = pose_frames(WORLD2_POSES[:1], W, H)
with Renderer(sc, W, H, max_frames=1) as r:
    g = r.render(make_frames(views, projs, [0], [0]), want=("rgb", "instance", "depth", "normals", "points"))
o = Oracle(pack_scene(sc), W, H).render(views[0], projs[0], extra=True)
gn, on = g["normals"][0].view(np.uint16), o["normals"].view(np.uint16)
bad = np.argwhere((gn != on).any(-1))
print("normals differing px:", len(bad))
for y, x in bad[:12]:
    print((y, x), "gpu", gn[y, x], g["normals"][0][y, x], "ora", on[y, x], o["normals"][y, x], "inst", o["instance"][y, x])
gp, op = g["points"][0].view(np.uint32), o["points"].view(np.uint32)
badp = np.argwhere((gp != op).any(-1))
print("points differing px:", len(badp))
for y, x in badp[:6]:
    print((y, x), "gpu", g["points"][0][y, x], "ora", o["points"][y, x])
