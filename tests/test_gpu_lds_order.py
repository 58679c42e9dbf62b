"""k_raster's cross-thread LDS hand-offs after the raster loop, exercised
where they are busiest ("LDS ordering").

A surface of ~1.5-px quads puts ~200 distinct winning triangles in every
32x16 tile, so with its 64 shade slots the resolve runs ~4 rounds per tile
(~400 per 32x32 tile over 116 slots in a 32x32 build): the shade table's keys
are re-initialised, re-filled by CAS and re-read each round, the setup
threads overwrite table entries the previous round's pixels read, the
round flag ("more") is cleared and set every round, and the label-statistic
runs, the depth-range partials (first round only), the coverage table
(k_raster<true>) and the keypoint depth test all meet in the same tiles.
64 labelled patches give each tile several labels; keypoints sit in front of
and behind the surface.  Six frames a batch, three batches each through
k_raster<false> and k_raster<true> (with the coverage output): every output
must equal the oracle's every time.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _fine_surface(n_side=8, cells=22, cell=0.05, seed=3):
    """n_side x n_side patches (one mesh, instance and label each) of
    cells x cells quads, each split into two triangles, with a small random
    relief so depths vary inside every tile."""
    from constructionsceneposeestimation_amd.scene.model import Instance, Material, Mesh, Scene, SceneObject
    rng = np.random.default_rng(seed)
    s = Scene()
    s.materials = [Material(f"m{k}", rng.uniform(0.2, 1.0, 3)) for k in range(8)]
    no_uv = (np.zeros((0, 2), np.float32), np.zeros((0, 3), np.uint32))
    g = np.arange(cells + 1)
    ii, jj = np.meshgrid(g, g, indexing="ij")
    q = (ii[:-1, :-1] * (cells + 1) + jj[:-1, :-1]).reshape(-1)
    tris = np.concatenate([np.stack([q, q + 1, q + cells + 2], 1), np.stack([q, q + cells + 2, q + cells + 1], 1)])
    span = cells * cell
    for a in range(n_side):
        for b in range(n_side):
            x0, y0 = (a - n_side / 2) * span, (b - n_side / 2) * span * 0.62
            pos = np.stack([x0 + jj * cell, y0 + ii * cell * 0.62, rng.uniform(-0.02, 0.02, ii.shape)], -1)
            k = len(s.meshes)
            s.meshes.append(Mesh(f"p{k}", pos.reshape(-1, 3).astype(np.float32), tris.astype(np.uint32), *no_uv,
                                 k % len(s.materials)))
            s.instances.append(Instance(k, np.eye(4), k, k))
            s.objects.append(SceneObject(f"/patch{k}", "fence", 2, k))
    return s


def test_multi_round_resolve_stats_range_coverage_keypoints():
    from constructionsceneposeestimation_amd import camera_math as cm
    from constructionsceneposeestimation_amd.packing import pack_scene
    from constructionsceneposeestimation_amd.renderer import Renderer, make_frames
    from oracle.oracle import Oracle, depth_vis
    W, H, F = 256, 160, 6
    sc = _fine_surface()
    intr = cm.Intrinsics(W, H)
    views, projs = [], []
    for k in range(F):
        C = np.eye(4)
        C[:3, 3] = [0.05 * k - 0.1, 0.03 * k - 0.05, 4.0 + 0.02 * k]
        views.append(cm.view_matrix(C))
        projs.append(intr.pixel_projection())
    views, projs = np.stack(views), np.stack(projs)
    assert 0.05 * intr.fx / 4.0 < 2.0            # quads of ~1.5 px: ~200 winning triangles per 32x16 tile
    rng = np.random.default_rng(9)
    u, v = rng.uniform(0, W, 300), rng.uniform(0, H, 300)
    d = np.where(np.arange(300) % 2 == 0, 3.0, 5.0)   # in front of / behind the surface (at ~4 m)
    kp = np.stack([(u - W / 2) * d / intr.fx, -(v - H / 2) * d / intr.fy, 4.0 - d], 1).astype(np.float32)
    o = Oracle(pack_scene(sc), W, H)
    refs = []
    for k in range(F):
        ref = o.render(views[k], projs[k], want_stats=True, covered=True, extra=True)
        ref["uv"], ref["vis"] = o.keypoints(views[k], projs[k], kp, ref["depth"])
        ref["dvis"], ref["drange"] = depth_vis(ref["depth"])
        refs.append(ref)
    assert len(np.unique(refs[0]["instance"])) >= 40
    assert (refs[0]["vis"] == 2).sum() > 50 and (refs[0]["vis"] == 1).sum() > 50
    # normals and points too: a 4-pixel group whose pixels finish in different
    # rounds stores them per pixel, one finished in a single round as vector stores
    want = ("rgb", "instance", "depth", "stats", "keypoints", "depth_vis", "normals", "points")
    with Renderer(sc, W, H, max_frames=F) as r:
        r.set_keypoints(0, kp)
        for cov in (False, True, False, True, False, True):
            gpu = r.render(make_frames(views, projs, [0] * F, list(range(F))), want=want + (("covered",) if cov else ()))
            for k, ref in enumerate(refs):
                for key in ("rgb", "instance"):
                    assert np.array_equal(gpu[key][k], ref[key]), f"frame {k}: {key}"
                assert np.array_equal(gpu["depth"][k].view(np.uint32), ref["depth"].view(np.uint32)), f"frame {k}"
                assert np.array_equal(gpu["normals"][k].view(np.uint16), ref["normals"].view(np.uint16)), f"frame {k}"
                assert np.array_equal(gpu["points"][k].view(np.uint32), ref["points"].view(np.uint32)), f"frame {k}"
                assert np.array_equal(gpu["inst_stats"][k], ref["inst_stats"]), f"frame {k}: label stats"
                if cov:
                    assert np.array_equal(gpu["label_covered"][k], ref["label_covered"]), f"frame {k}: coverage"
                assert np.array_equal(gpu["keypoints_vis"][k], ref["vis"]), f"frame {k}: keypoint visibility"
                assert np.array_equal(gpu["keypoints_uv"][k].view(np.uint32), ref["uv"].view(np.uint32))
                assert np.array_equal(gpu["depth_vis"][k], ref["dvis"]), f"frame {k}: depth_vis"
                assert np.array_equal(gpu["depth_range"][k], np.array(ref["drange"], np.float32), equal_nan=True)
