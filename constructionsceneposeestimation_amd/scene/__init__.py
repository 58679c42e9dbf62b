"""Scene IO: USD crate reader, scene model, committed fixtures, proxies."""
from __future__ import annotations

import os

from .model import Instance, Light, Material, Mesh, Scene, SceneObject, Texture

ASSETS = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "assets")


def load_world2() -> Scene:
    """world2.usd.backup decoded (715,944 triangles, 36 labelled objects)."""
    return Scene.load_npz(os.path.join(ASSETS, "world2_static.npz"))


def load_cone() -> Scene:
    """The TrafficCone mesh alone (config C1)."""
    return Scene.load_npz(os.path.join(ASSETS, "cone.npz"))


__all__ = ["Scene", "Mesh", "Material", "Texture", "Instance", "SceneObject", "Light",
           "load_world2", "load_cone", "ASSETS"]
