"""Generate golden vectors from the reference's own pure helpers.

Run ONLY in the build container (the reference is at /root/reference and
never travels to the GPU box):

    python tests/golden/make_golden.py [/root/reference]

The reference module cannot be imported (it imports omni/isaacsim/pxr/cv2 at
generate_construction_data.py:13-20 and has import-time side effects at
:1350-1373), so this script parses it with ``ast``, executes only the pure
function definitions and constant tables listed below in a namespace with
numpy + scipy, calls them on seeded synthetic inputs, and writes the inputs
and outputs as fixtures.  No reference source is copied into the repo.

Functions (reference line numbers):
  rotMtx2quaternion :475-504, camPosOri :507-550, bboxDict_to_transform :553-584,
  depth_to_pointcloud_with_rgb :616-711, get_object_root :144-233,
  get_systematic_camera_positions :778-911; tables construction_class :69-106,
  CRANE_PART_CHILD_MAP :110-121.
"""
from __future__ import annotations

import ast
import io
import json
import os
import sys
from contextlib import redirect_stdout

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

FUNCS = ["rotMtx2quaternion", "camPosOri", "bboxDict_to_transform", "depth_to_pointcloud_with_rgb",
         "get_object_root", "get_systematic_camera_positions"]
TABLES = ["construction_class", "CRANE_PART_CHILD_MAP", "_crane_part_map"]


def load_reference(ref_root: str):
    src_path = os.path.join(ref_root, "generate_construction_data.py")
    tree = ast.parse(open(src_path, encoding="utf-8").read(), filename=src_path)
    keep = []
    for node in tree.body:
        if isinstance(node, ast.FunctionDef) and node.name in FUNCS:
            keep.append(node)
        elif isinstance(node, ast.Assign) and any(isinstance(t, ast.Name) and t.id in TABLES for t in node.targets):
            keep.append(node)
    mod = ast.Module(body=keep, type_ignores=[])
    from scipy.spatial.transform import Rotation as R
    ns = {"np": np, "R": R}
    exec(compile(mod, src_path, "exec"), ns)
    missing = [f for f in FUNCS + TABLES if f not in ns]
    assert not missing, missing
    return ns


def quiet(fn, *a, **k):
    with redirect_stdout(io.StringIO()):
        return fn(*a, **k)


def main(ref_root: str = "/root/reference") -> None:
    ns = load_reference(ref_root)
    rng = np.random.default_rng(20260213)

    # 1. camPosOri: level shots (the reference's schedule), pitched shots, degenerate
    cams, aims = [], []
    for k in range(256):
        cam = np.array([rng.uniform(-15, 12), rng.uniform(-12, 12), rng.choice([1.6, 1.7, 1.8, 2.0, 2.5, 3.0])])
        if k < 128:
            aim = np.array([rng.uniform(-8, 6), rng.uniform(-6, 6), cam[2]])
        elif k < 248:
            aim = cam + rng.normal(size=3)
        else:
            aim = cam + np.array([0, 0, rng.choice([-1.0, 1.0])]) * rng.uniform(0.5, 3)
        cams.append(cam)
        aims.append(aim)
    cams, aims = np.array(cams), np.array(aims)
    q = np.array([ns["camPosOri"](c, a) for c, a in zip(cams, aims)])
    Rs = np.array([[[0.3, -0.2, 0.9], [0.1, 0.95, 0.2], [-0.9, 0.1, 0.3]]])
    np.savez(os.path.join(HERE, "campos.npz"), cam=cams, aim=aims, q=q)

    # rotMtx2quaternion on proper rotations covering all four branches
    from scipy.spatial.transform import Rotation
    mats = Rotation.random(64, random_state=7).as_matrix()
    mats = np.concatenate([mats, np.diag([1.0, -1, -1])[None], np.diag([-1.0, 1, -1])[None],
                           np.diag([-1.0, -1, 1])[None], np.eye(3)[None]])
    qs = np.array([ns["rotMtx2quaternion"](m) for m in mats])
    np.savez(os.path.join(HERE, "rotmtx2quat.npz"), R=mats, q=qs)

    # 2. camera schedule under np.random.seed(s)
    sched = {}
    for s in (0, 1, 2):
        np.random.seed(s)
        pos = quiet(ns["get_systematic_camera_positions"], 120)
        sched[f"cam_{s}"] = np.array([p[0] for p in pos])
        sched[f"aim_{s}"] = np.array([p[1] for p in pos])
    np.savez(os.path.join(HERE, "camera_schedule.npz"), **sched)

    # 3. get_object_root over world2's mesh paths + crane/dumper/human/edge cases
    from constructionsceneposeestimation_amd.scene.usdc import CrateFile
    crate = CrateFile(os.path.join(ref_root, "cad_models", "world2.usd.backup"))
    mesh_paths = [p for p, s in crate.specs.items()
                  if s.spec_type == "Prim" and crate.field(p, "typeName") == "Mesh"]
    crane = "/World/GroundPlane/tn__Pk7501SLD_PNR3879_fPM"
    extra = [crane + "/S104GG03A_SW/mesh", crane + "/s104hz01ka_sw/a/b", crane + "/tn__S104EKB_AS_SW_jj7/x",
             crane + "/S104KZ02KA_SW/y", crane + "/unknown_child/boom_part", crane + "/other/Mast_1",
             crane + "/x/chassis", crane + "/x/teleskop", crane, "/World/pk7_misc",
             "/World/GroundPlane/tn__09684481_/Body/mesh_3", "/World/GroundPlane/DHGen/SkelRoot/Outfit/c_vest",
             "/World/GroundPlane/DHGen_01/SkelRoot/m", "/World/GroundPlane/Cone001/Cone001",
             "/World/Tree/Tree", "/World/Tree/Tree_05/Tree/g1", "/World/GroundPlane/CollisionMesh",
             "/World/GroundPlane/CollisionPlane", "/World/Looks/Material__0", "/World/some_fence_mesh",
             "/World/Human_03", "/World/TrafficCone_2", "/X/Construction_Site_A/mesh", ""]
    paths = mesh_paths + extra
    roots = [list(ns["get_object_root"](p)) for p in paths]
    json.dump({"paths": paths, "roots": roots}, open(os.path.join(HERE, "object_root.json"), "w"), indent=0)

    # 4. bboxDict_to_transform on synthetic records (local box + row-major 4x4, USD convention)
    recs_lo, recs_hi, recs_T, out_c, out_s, out_e = [], [], [], [], [], []
    rots = Rotation.random(100, random_state=11)
    for k in range(100):
        lo = rng.uniform(-3, 0, 3)
        hi = lo + rng.uniform(0.05, 6, 3)
        Rm = rots[k].as_matrix() * rng.uniform(0.001, 2.0, 3)[None, :]
        M = np.eye(4)
        M[:3, :3] = Rm
        M[:3, 3] = rng.uniform(-20, 20, 3)
        T_usd = M.T.reshape(16)           # row-vector convention as the annotator reports it
        rec = (0, lo[0], lo[1], lo[2], hi[0], hi[1], hi[2], T_usd, 0.0)
        c, sz, e = ns["bboxDict_to_transform"](rec)
        recs_lo.append(lo)
        recs_hi.append(hi)
        recs_T.append(T_usd)
        out_c.append(c)
        out_s.append(sz)
        out_e.append(e)
    np.savez(os.path.join(HERE, "bbox_transform.npz"), lo=np.array(recs_lo), hi=np.array(recs_hi),
             T=np.array(recs_T), center=np.array(out_c), size=np.array(out_s), euler=np.array(out_e))

    # 5. depth_to_pointcloud_with_rgb (the reference's only in-repo pinhole math)
    pcs = {}
    for name, (h, w) in {"a": (32, 48), "b": (64, 64)}.items():
        depth = rng.uniform(0.3, 260, (h, w)).astype(np.float32)
        depth[rng.random((h, w)) < 0.1] = np.inf
        depth[0, :3] = [0.0, np.nan, 249.99]
        rgbimg = rng.integers(0, 256, (h, w, 4), dtype=np.uint8)
        params = {"horizontal_aperture": 25.0, "vertical_aperture": 25.0 * h / w, "focal_length": 12.0,
                  "width": w, "height": h}
        pose = [rng.uniform(-5, 5), rng.uniform(-5, 5), rng.uniform(1, 3)] + list(Rotation.random(
            random_state=int(h)).as_quat())
        out = quiet(ns["depth_to_pointcloud_with_rgb"], depth, rgbimg, params, pose)
        pcs[f"{name}_depth"], pcs[f"{name}_rgb"], pcs[f"{name}_pose"] = depth, rgbimg, np.array(pose)
        pcs[f"{name}_out"] = out
    np.savez(os.path.join(HERE, "pointcloud.npz"), **pcs)
    print("golden vectors written to", HERE)


if __name__ == "__main__":
    main(*sys.argv[1:])
