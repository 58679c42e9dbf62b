"""Batched dataset generator: the replacement for the reference's per-frame
``generate_data()`` loop (generate_construction_data.py:1379-2094).

Per frame the reference sets the camera, waits ~5.9 s of fixed sleeps for
Kit to render (:1592-1609), then pulls RGB / depth / point cloud / boxes and
writes them (:1668-2072).  Here a shard of frames is rendered in batches on
one GPU (camera poses and object layouts from the seeded schedule, every
frame a pure function of (seed, frame)), and host writer threads emit the
same files:

  rgb/rgb_%06d.png                 (:1672-1673)
  labels/label_%06d.json           (:2071-2072, schema :2056-2064 + keypoints_2d)
  labels/instance_mask_%06d.npy    (:2066-2069; real ids here, -1 background)
  depth/depth_%06d.npy|.csv        (:1687-1688, optional)
  pointcloud/pointcloud_%06d.txt   (:1716-1724, optional; points from the GPU resolve)
  normals/normals_%06d.npy         (C5 normals, f16, optional)
  logs/generation_summary.json     (:2090)

Sharding: ``--rank/--world`` (or RANK/WORLD_SIZE) pick the epochs this
process owns (shard.shard_of_range); no communication between shards.
Resume: frames whose label file already exists are skipped.

    python -m constructionsceneposeestimation_amd.generate --out /data/run0 --frames 1000
"""
from __future__ import annotations

import argparse
import json
import os
import sys
from concurrent.futures import ThreadPoolExecutor
from typing import List, Optional

import numpy as np

from . import camera_math as cm
from . import writers as fileio
from .labels import label_record, object_poses, save_label_json
from .quality_log import QualityLog
from .renderer import Renderer, make_frames
from .shard import shard_of_range
from .workload import Workload


def _write_png(path: str, rgb: np.ndarray) -> None:
    fileio.write_png(path, rgb, level=1)


def _write_pointcloud(path: str, points: np.ndarray, rgb: np.ndarray) -> None:
    """``x y z r g b`` per hit pixel (generate_construction_data.py:769-770);
    the world points come from the GPU resolve (NaN where nothing is hit)."""
    fileio.write_pointcloud_txt(path, points, rgb)


def _atomic(path: str, fn, *args) -> None:
    """Write through ``path + '.tmp'`` and rename: a crash never leaves a
    truncated file under the final name."""
    tmp = path + ".tmp"
    fn(tmp, *args)
    os.replace(tmp, path)


def _write_frame(files, label: dict, label_path: str) -> None:
    """Every file of one frame, then its label JSON: the label is the resume
    marker (generate_construction_data.py:1357-1367 scans labels/), so it
    appears only once the frame's other files are complete."""
    for path, fn, args in files:
        _atomic(path, fn, *args)
    _atomic(label_path, lambda path, lab: save_label_json(lab, path), label)


def default_writers() -> int:
    try:
        n = len(os.sched_getaffinity(0))
    except AttributeError:  # pragma: no cover
        n = os.cpu_count() or 1
    omp = int(os.environ.get("OMP_NUM_THREADS") or 0)   # the box's CPU share, when set
    return max(1, min(n, omp) if omp else n)


def generate(out_dir: str, frames: List[int], workload: str = "C3", seed: int = 0, batch: int = 30,
             device: int = 0, depth: bool = False, depth_csv: bool = False, pointcloud: bool = False,
             width: Optional[int] = None, height: Optional[int] = None, writers: int = 0,
             resume: bool = True, normals: bool = False) -> dict:
    wl = Workload(workload, seed=seed, width=width, height=height)
    for d in ("rgb", "labels", "depth", "pointcloud", "normals", "logs"):
        os.makedirs(os.path.join(out_dir, d), exist_ok=True)
    if resume:
        frames = [f for f in frames if not os.path.exists(os.path.join(out_dir, "labels", f"label_{f:06d}.json"))]
    depth = depth or depth_csv
    log = QualityLog(os.path.join(out_dir, "logs"))
    r = Renderer(wl.scene, wl.width, wl.height, max_frames=batch, device=device)
    intr = wl.intr
    want = (["rgb", "instance", "keypoints", "stats"] + (["depth"] if depth else [])
            + (["points"] if pointcloud else []) + (["normals"] if normals else []))
    pose_cache = {}
    n_writers = writers or default_writers()
    pool = ThreadPoolExecutor(max_workers=n_writers)
    pending = []
    for s0 in range(0, len(frames), batch):
        fb = frames[s0:s0 + batch]
        epochs = sorted({f // 10 for f in fb})
        set_of = {}
        for k, e in enumerate(epochs):
            st = wl.epoch(e)
            r.set_instance_transforms(k, st.models)
            r.set_keypoints(k, st.keypoints)
            if st.dr is not None:
                r.set_dr_light(k, st.dr.light)
                r.set_dr_textures(k, st.dr.textures)
            set_of[e] = k
            if e not in pose_cache:
                pose_cache[e] = object_poses(wl.scene, st.object_frames)
        views, projs = wl.frame_params(fb)
        out = r.render(make_frames(views, projs, [set_of[f // 10] for f in fb], fb), want=want)
        for k, f in enumerate(fb):
            V, P, C, cam, aim, q = wl.camera(f)
            lab = label_record(f, cm.get_obj_pose_from_matrix(C), intr.params(), pose_cache[f // 10],
                               out["inst_stats"][k], out["keypoints_uv"][k], out["keypoints_vis"][k],
                               wl.kp_table, wl.height, wl.width)
            log.frame(lab["num_objects"], out["depth"][k] if "depth" in out else None, out["keypoints_vis"][k])
            files = [(os.path.join(out_dir, "rgb", f"rgb_{f:06d}.png"), _write_png, (out["rgb"][k],)),
                     (os.path.join(out_dir, "labels", f"instance_mask_{f:06d}.npy"), fileio.write_npy,
                      (out["instance"][k],))]
            if depth:
                files.append((os.path.join(out_dir, "depth", f"depth_{f:06d}.npy"), fileio.write_npy,
                              (out["depth"][k],)))
                if depth_csv:
                    files.append((os.path.join(out_dir, "depth", f"depth_{f:06d}.csv"), fileio.write_depth_csv,
                                  (out["depth"][k],)))
            if pointcloud:
                files.append((os.path.join(out_dir, "pointcloud", f"pointcloud_{f:06d}.txt"), _write_pointcloud,
                              (out["points"][k], out["rgb"][k])))
            if normals:
                files.append((os.path.join(out_dir, "normals", f"normals_{f:06d}.npy"), fileio.write_npy,
                              (out["normals"][k],)))
            pending.append(pool.submit(_write_frame, files, lab,
                                       os.path.join(out_dir, "labels", f"label_{f:06d}.json")))
        # bound the queue so host memory stays flat
        while len(pending) > 4 * n_writers:
            pending.pop(0).result()
    for p in pending:
        p.result()
    pool.shutdown()
    r.close()
    log.save()
    return log.summary()


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__.split("\n\n")[0])
    ap.add_argument("--out", required=True)
    ap.add_argument("--frames", type=int, default=41, help="total frames of the run (all shards)")
    ap.add_argument("--workload", default="C3")
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--batch", type=int, default=30)
    ap.add_argument("--rank", type=int, default=int(os.environ.get("RANK", "0")))
    ap.add_argument("--world", type=int, default=int(os.environ.get("WORLD_SIZE", "1")))
    ap.add_argument("--device", type=int, default=int(os.environ.get("LOCAL_RANK", "0")))
    ap.add_argument("--width", type=int)
    ap.add_argument("--height", type=int)
    ap.add_argument("--depth", action="store_true")
    ap.add_argument("--depth-csv", action="store_true")
    ap.add_argument("--pointcloud", action="store_true")
    ap.add_argument("--normals", action="store_true")
    ap.add_argument("--no-resume", action="store_true")
    a = ap.parse_args(argv)
    frames = shard_of_range(a.rank, a.world, a.frames)
    out = os.path.join(a.out, f"shard_{a.rank:02d}") if a.world > 1 else a.out
    summary = generate(out, frames, a.workload, a.seed, a.batch, a.device, a.depth, a.depth_csv, a.pointcloud,
                       a.width, a.height, resume=not a.no_resume, normals=a.normals)
    print(json.dumps(summary))


if __name__ == "__main__":
    main()
