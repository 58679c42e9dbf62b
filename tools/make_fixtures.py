"""Generate the committed scene fixtures from the reference's assets.

Runs only in the build container (reads /root/reference, which does not
exist on the GPU box).  Outputs under constructionsceneposeestimation_amd/assets/:

* world2_static.npz — world2.usd.backup decoded by scene/usdc.py: 5 unique
  meshes, 48 instances, 36 labelled objects (23 fence, 11 tree, 2 cone),
  715,944 triangles, full-resolution stand-in textures.
* cone.npz — the TrafficCone mesh alone (config C1).

Usage: python tools/make_fixtures.py [/root/reference]
"""
from __future__ import annotations

import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from constructionsceneposeestimation_amd.scene.model import Instance, Scene, SceneObject  # noqa: E402
from constructionsceneposeestimation_amd.scene.usd_scene import load_crate_scene  # noqa: E402

ASSETS = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                      "constructionsceneposeestimation_amd", "assets")


def main(ref: str = "/root/reference") -> None:
    os.makedirs(ASSETS, exist_ok=True)
    src = os.path.join(ref, "cad_models", "world2.usd.backup")
    # full-resolution stand-in textures (SURVEY §8(d) B_tex: leaf 766x1024 + bark 1600x1300 RGBA8 = 11.46 MB)
    scene = load_crate_scene(src, texture_root=ref, max_texture=4096)
    assert scene.meta["n_mesh_prims"] == 1060, scene.meta
    assert len(scene.objects) == 36
    assert scene.n_tris_per_frame == 715944
    scene.save_npz(os.path.join(ASSETS, "world2_static.npz"))
    print("world2_static:", len(scene.meshes), "meshes", len(scene.instances), "instances",
          scene.n_tris_per_frame, "tris", os.path.getsize(os.path.join(ASSETS, "world2_static.npz")), "bytes")

    cone_mesh_id = next(i for i, m in enumerate(scene.meshes) if m.name.endswith("Cone001"))
    cone = Scene()
    m = scene.meshes[cone_mesh_id]
    mat = scene.materials[m.material]
    cone.materials = [mat]
    m.material = 0
    cone.meshes = [m]
    model = np.diag([0.01, 0.01, 0.01, 1.0])     # authored in cm (xformOp:scale 0.01)
    cone.instances = [Instance(0, model, 0, 0, np.eye(4))]
    cone.objects = [SceneObject("/World/GroundPlane/Cone001_01", "trafficcone", 0, 0, "trafficcone",
                                np.stack([m.positions.min(0), m.positions.max(0)]).astype(np.float64) * 0.01)]
    cone.light = scene.light
    cone.meta = {"source": "world2.usd.backup:/World/GroundPlane/Cone001_01/Cone001"}
    cone.save_npz(os.path.join(ASSETS, "cone.npz"))
    print("cone:", m.n_tris, "tris")


if __name__ == "__main__":
    main(*sys.argv[1:])
