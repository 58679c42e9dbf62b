"""Batched dataset generator: the replacement for the reference's per-frame
``generate_data()`` loop (generate_construction_data.py:1379-2094).

Per frame the reference sets the camera, waits ~5.9 s of fixed sleeps for
Kit to render (:1592-1609), then pulls RGB / depth / point cloud / boxes and
writes them (:1668-2072).  Here a shard of frames is rendered in batches on
one GPU (camera poses and object layouts from the seeded schedule, every
frame a pure function of (seed, frame)), and host writer threads emit the
same files:

  rgb/rgb_%06d.png                 (:1672-1673)
  labels/label_%06d.json           (:2071-2072, schema :2056-2064 + keypoints_2d,
                                    bbox_2d, pixel_count; + occlusion_ratio with
                                    --occlusion)
  labels/instance_mask_%06d.npy    (:2066-2069; real ids here, -1 background)
  depth/depth_%06d.csv             (:1687-1688)
  depth/depth_%06d.png             (:1690-1709, JET colour map made on the GPU)
  depth/depth_%06d.npy             (optional)
  pointcloud/pointcloud_%06d.txt   (:1716-1757; points from the GPU resolve, text encoded on the GPU)
  normals/normals_%06d.npy         (C5 normals, f16, optional)
  logs/generation_summary.json     (:2090; statistics, frame_logs, counters)
  logs/generation_detail.log       (:254-263, per-frame entries + report)

The default outputs are the reference's (RGB PNG, depth CSV + PNG, point
cloud TXT, mask .npy, label JSON); ``--outputs`` picks others.

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
import time
import multiprocessing as mp
from concurrent.futures import ProcessPoolExecutor, ThreadPoolExecutor
from functools import partial
from typing import List, Optional

import numpy as np

from . import camera_math as cm
from . import prep_pool
from .labels import OBJECT_LISTS, in_frustum, label_record, object_poses
from .quality_log import QualityLog
from .renderer import Renderer, make_frames, output_spec, scene_labels
from .shard import shard_of_range
from .workload import Workload
from .writer_pool import WriterPool
from .writers import LabelWriter
from .writer_pool import _write_png  # noqa: F401  (the generator's PNG settings; tools/gen_bench.py)


def default_writers() -> int:
    try:
        n = len(os.sched_getaffinity(0))
    except AttributeError:  # pragma: no cover
        n = os.cpu_count() or 1
    omp = int(os.environ.get("OMP_NUM_THREADS") or 0)   # the box's CPU share, when set
    return max(1, min(n, omp) if omp else n)


def _log_done(log: QualityLog, fut, log_args: dict, points: bool) -> None:
    ds = fut.result()                       # host depth counts (writer), else the GPU's
    gpu_ds = log_args.pop("gpu_depth_stats", None)
    ds = ds if ds is not None else gpu_ds
    log.frame(depth_stats=ds, points=ds["valid"] if points and ds else None, **log_args)


OUTPUTS = ("rgb", "mask", "depth_csv", "depth_png", "depth_npy", "pointcloud", "normals")
# What the reference writes for every frame (GDP:1668-1771, 2055-2072): RGB PNG, depth CSV and
# JET depth PNG, point-cloud TXT, instance mask .npy; the label JSON is always written (it is the
# resume marker).
REFERENCE_OUTPUTS = ("rgb", "mask", "depth_csv", "depth_png", "pointcloud")


# outputs encoded on the GPU in thread mode -> their csg_outputs.file_kinds kind (_lib.FILE_KINDS)
FILE_OF_OUTPUT = (("rgb", "rgb_png"), ("depth_csv", "depth_csv"), ("depth_png", "depth_png"),
                  ("pointcloud", "pointcloud_txt"))
_PATHS = {"rgb": ("rgb", "rgb_{:06d}.png"), "depth_csv": ("depth", "depth_{:06d}.csv"),
          "depth_png": ("depth", "depth_{:06d}.png"), "pointcloud": ("pointcloud", "pointcloud_{:06d}.txt")}


def file_path(out_dir: str, output: str, frame: int) -> str:
    """The reference's file name of one output of a frame (GDP:1668-1716)."""
    d, name = _PATHS[output]
    return os.path.join(out_dir, d, name.format(frame))


def parse_outputs(spec: str) -> tuple:
    if spec in ("reference", ""):
        return REFERENCE_OUTPUTS
    if spec == "all":
        return OUTPUTS
    out = tuple(x.strip() for x in spec.split(",") if x.strip())
    bad = [x for x in out if x not in OUTPUTS]
    if bad:
        raise ValueError(f"unknown outputs {bad}; choose from {OUTPUTS}")
    return out


def render_outputs(outs: set, gpu_files: bool, host_depth: bool, occlusion: bool) -> list:
    """The renderer outputs (renderer.OUTPUT_KINDS) a run with file outputs
    ``outs`` asks for.  Label statistics and keypoints feed every label file;
    the label coverage ("covered", k_raster<true>) only ``occlusion_ratio``,
    which is not in the reference's label schema (GDP:2056-2064)."""
    if gpu_files:
        want = (["keypoints", "stats", "depth_stats"] + (["instance"] if "mask" in outs else [])
                + (["depth"] if host_depth else []) + (["depth_range"] if "depth_png" in outs else [])
                + (["normals"] if "normals" in outs else []))
    else:
        want = (["rgb", "instance", "keypoints", "stats"] + (["depth"] if host_depth else [])
                + (["depth_vis"] if "depth_png" in outs else []) + (["points"] if "pointcloud" in outs else [])
                + (["normals"] if "normals" in outs else []))
    return want + (["covered"] if occlusion else [])


def generate(out_dir: str, frames: List[int], workload: str = "C3", seed: int = 0, batch: int = 30,
             device: int = 0, depth: bool = False, depth_csv: bool = False, pointcloud: bool = False,
             width: Optional[int] = None, height: Optional[int] = None, writers: int = 0,
             resume: bool = True, normals: bool = False, outputs: Optional[tuple] = None,
             writer_mode: str = "thread", renderers: int = 0, object_list: str = "visible",
             occlusion: bool = False, sink: str = "disk", validate_pointcloud: bool = False,
             min_points: int = 100, max_retries: int = 5, prep_workers: int = -1) -> dict:
    """Render ``frames`` on one GPU and write them (``outputs``, default the
    reference's set; ``depth`` / ``depth_csv`` / ``pointcloud`` / ``normals``
    add the depth .npy, the depth .npy + CSV, the point cloud, the normals).
    ``writer_mode`` "thread" encodes in threads of this process (the native
    writers release the GIL), "process" in worker processes fed through
    shared memory (writer_pool.py; measured slower at 1080p C3: 184 vs 233
    frames/s, page faults on the shared ring and task pickling).
    ``object_list``: "visible" lists the objects with visible pixels in each
    label file; "frustum" also those whose 3D box meets the view frustum
    (labels.label_record; the reference lists Replicator's bounding_box_3d
    primPaths, whose inclusion rule is closed).
    ``occlusion`` adds each object's ``occlusion_ratio`` (Replicator's
    occlusionRatio) to the label files.  The reference never reads that field
    and its label schema (GDP:2056-2064) has none, so it is off by default: it
    needs the per-label unoccluded coverage, i.e. k_raster<true> (about +36%
    raster time).
    ``sink`` "discard" runs the whole pipeline (render, GPU encode, copy
    into the page-locked ring, writer threads) but writes every file to
    /dev/null: the generator's steady-state rate without a file system.
    ``validate_pointcloud`` (off by default, as ``enable_pointcloud_validation``
    in the reference, GDP:61): a frame whose point cloud has fewer than
    ``min_points`` points (GDP:59; the GPU's count of valid depth pixels) is
    rendered again from a jittered camera (Workload.camera's ``attempt``,
    GDP:1573-1581), up to ``max_retries`` attempts in all (GDP:60); a frame
    that fails them all is logged failed and writes no files (GDP:1662-1666).
    ``prep_workers``: processes that prepare batches ahead (epoch layouts,
    object poses, cameras; prep_pool.py), so that numpy work does not hold
    this process's GIL; -1 = two for runs of at least 20 batches, else none."""
    if object_list not in OBJECT_LISTS:
        raise ValueError(f"object_list {object_list!r}: choose from {OBJECT_LISTS}")
    outs = set(REFERENCE_OUTPUTS if outputs is None else outputs)
    if depth or depth_csv:
        outs.add("depth_npy")
    if depth_csv:
        outs.add("depth_csv")
    if pointcloud:
        outs.add("pointcloud")
    if normals:
        outs.add("normals")
    wl = Workload(workload, seed=seed, width=width, height=height)
    for d in ("rgb", "labels", "depth", "pointcloud", "normals", "logs"):
        os.makedirs(os.path.join(out_dir, d), exist_ok=True)
    if resume:
        frames = [f for f in frames if not os.path.exists(os.path.join(out_dir, "labels", f"label_{f:06d}.json"))]
    # batch preparation in worker processes, started (like the writer processes
    # below) before this process touches the GPU; each builds its own Workload
    n_prep = prep_workers if prep_workers >= 0 else (2 if len(frames) >= 20 * batch else 0)
    ppool = None
    if n_prep:
        ppool = ProcessPoolExecutor(max_workers=n_prep, mp_context=mp.get_context("spawn"),
                                    initializer=prep_pool.init, initargs=(workload, seed, width, height))
        for f in [ppool.submit(prep_pool.ping) for _ in range(2 * n_prep)]:   # every worker started now
            f.result()
    # Thread writers (the default): the PNGs, the depth CSV and the point
    # cloud are encoded on the GPU (Renderer.render_files, csg_encode.hip) and
    # the host only writes bytes; writer processes encode on the host (libcsgio).
    gpu_files = writer_mode == "thread"
    kinds = tuple(k for o, k in FILE_OF_OUTPUT if o in outs) if gpu_files else ()
    # host depth for its own files; the quality log's depth counts come from
    # the GPU (depth_stats) in thread mode, from the host depth otherwise
    host_depth = "depth_npy" in outs or (not gpu_files and bool(outs & {"depth_csv", "pointcloud"}))
    log = QualityLog(os.path.join(out_dir, "logs"))
    want = render_outputs(outs, gpu_files, host_depth, occlusion)
    if validate_pointcloud and "depth_stats" not in want:
        want.append("depth_stats")   # the per-frame valid point count the validation reads
    n_writers = writers or default_writers()
    # Renderer contexts on the device, each with its own stream and work
    # buffers, rendering alternate batches from their own threads: one batch's
    # encode and copy overlap the next ones' render (C3 1080p into RAM, 16
    # writers: 1,038 frames/s with two, 846 with one; at steady state with the
    # files to /dev/null, three: 1,823 / 515 frames/s without / with the point
    # cloud, two: 1,739 / 505; profiles/r05/generate_steady.json.  Round 6, with
    # the 1-byte id wire and two prep workers, batches of 60: three 2,028-2,150,
    # four 2,029-2,041, three with batches of 120 1,912-1,975 frames/s without
    # the point cloud; profiles/r06/ab/prep_workers/).
    n_rend = renderers or (3 if gpu_files else 1)
    # the writer processes start here, before this process touches the GPU
    pool = WriterPool(output_spec(batch, wl.height, wl.width, wl.n_keypoints(), scene_labels(wl.scene), want),
                      n_writers, n_slots=2 + n_rend, mode=writer_mode, sink=sink)
    rends = [Renderer(wl.scene, wl.width, wl.height, max_frames=batch, device=device) for _ in range(n_rend)]
    r = rends[0]
    if gpu_files:   # page-locked slots, and buffers for the encoded files (an estimate, grown on demand)
        npx = wl.width * wl.height
        est = {"rgb_png": 2 * npx, "depth_csv": 10 * npx, "depth_png": npx, "pointcloud_txt": 48 * npx}
        pool.use_pinned(r.host_buffer, batch * sum(est[k] for k in kinds) + (1 << 20) if kinds else 0,
                        free=r.free_host_buffer)
    nk = len(kinds)
    intr = wl.intr
    # thread mode: label files written natively from the frame's arrays (no GIL)
    lw = LabelWriter(wl.kp_table, wl.intr.params(), scene_labels(wl.scene), wl.height, wl.width) if gpu_files else None
    pose_cache = {}
    pending = []

    def cov_of(out, k):   # the frame's label coverage (occlusion_ratio), when rendered
        return out["label_covered"][k] if "label_covered" in out else None

    t_render = t_slot_wait = t_prep = t_main_wait = t_labels = 0.0
    d2h = []   # bytes each batch copied to the host (files + arrays), appended by the render threads
    ids_wire = r.host_id_bytes()   # instance ids cross PCIe as 1-, 2- or 4-byte values (csg_host_id_bytes)

    def wire_bytes(out):   # the host arrays' bytes as they crossed PCIe (ids narrowed, widened on the host)
        return sum(v.nbytes for v in out.values()) - (out["instance"].size * (4 - ids_wire) if "instance" in out else 0)
    t0 = time.time()
    starts = list(range(0, len(frames), batch))

    def prepare(b: int):
        """Host state of batch b (epoch layouts, object poses, cameras), made
        ahead in its own thread so the render thread only renders."""
        fb = frames[starts[b]:starts[b] + batch]
        if ppool is not None:   # computed in a worker process, installed here
            eps, cams = ppool.submit(prep_pool.prepare, list(fb), sorted({f // 10 for f in fb})).result()
            for e, (st, poses) in eps.items():
                wl.install_epoch(e, st)
                if e not in pose_cache:
                    if len(pose_cache) >= 256:
                        pose_cache.pop(next(iter(pose_cache)))
                    pose_cache[e] = poses
            for f, cam in cams.items():
                wl.install_camera(f, cam)
            return
        for e in sorted({f // 10 for f in fb}):
            st = wl.epoch(e)
            if e not in pose_cache:
                if len(pose_cache) >= 256:   # bounded over long runs (an epoch is met once)
                    pose_cache.pop(next(iter(pose_cache)))
                pose_cache[e] = object_poses(wl.scene, st.object_frames)
        wl.frame_params(fb)

    def render_batch(b: int):
        """Batch b into its slot of the writer ring (runs one batch ahead of
        the label loop, in its own thread: the C-ABI call releases the GIL)."""
        fb = frames[starts[b]:starts[b] + batch]
        if b < len(prep_f):
            prep_f[b].result()
        slot = b % pool.n_slots
        r = rends[b % n_rend]
        tw = time.time()
        if kinds:   # files buffers this renderer replaced at an earlier batch (grow_files)
            pool.release_retired(r.free_host_buffer)
        arrays = pool.arrays(slot)          # (waits until the writers are done with the slot)
        tp = time.time()
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
        views, projs = wl.frame_params(fb)
        tr = time.time()
        sets = [set_of[f // 10] for f in fb]

        def run(views, projs):
            fr = make_frames(views, projs, sets, fb)
            if kinds:
                outs_b = {k: v[:len(fb)] for k, v in arrays.items() if k not in ("files", "file_offsets")}
                out, offsets, need = r.render_files(fr, kinds, arrays["files"], want=want, out=outs_b)
                if offsets is None:   # the files did not fit: a larger buffer, no re-render
                    offsets = r.copy_files(pool.grow_files(slot, need + need // 4, alloc=r.host_buffer,
                                                           free=r.free_host_buffer), len(fb) * nk)
                arrays["file_offsets"] = offsets
                d2h.append(int(offsets[-1]) + wire_bytes(out))
            else:
                out = r.render(fr, want=want, out={k: v[:len(fb)] for k, v in arrays.items()})
                d2h.append(wire_bytes(out))
            return out

        out = run(views, projs)
        attempts, checks, failed = [0] * len(fb), [[] for _ in fb], [False] * len(fb)
        if validate_pointcloud:   # GDP:1573-1645: retry frames whose point cloud is too small
            check = range(len(fb))
            while True:
                pts = out["depth_stats"][:len(fb), 0]
                again = []
                for k in check:
                    if pts[k] >= min_points:
                        continue
                    checks[k].append(int(pts[k]))
                    if attempts[k] + 1 < max_retries:
                        attempts[k] += 1
                        again.append(k)
                    else:
                        failed[k] = True
                if not again:
                    break
                # the whole batch again, the retried frames from their jittered cameras (the
                # others render exactly as before: every frame is a pure function of its pose)
                out = run(*wl.frame_params(fb, attempts))
                check = again
        te = time.time()
        return fb, slot, out, (te - tr, tp - tw, tr - tp), attempts, checks, failed

    ahead = ThreadPoolExecutor(max_workers=n_rend)
    prep = ThreadPoolExecutor(max_workers=max(1, n_prep))
    prep_f: List = []
    kPrepAhead = 3

    def prep_until(b: int) -> None:
        while len(prep_f) < min(b, len(starts)):
            prep_f.append(prep.submit(prepare, len(prep_f)))

    try:
        prep_until(kPrepAhead + n_rend)
        queued = [ahead.submit(render_batch, b) for b in range(min(n_rend, len(starts)))]
        for b in range(len(starts)):
            tq = time.time()
            fb, slot, out, (dt, dwait, dprep), attempts, checks, failed = queued.pop(0).result()
            t_main_wait += time.time() - tq
            t_render += dt
            t_slot_wait += dwait
            t_prep += dprep
            tl = time.time()
            prep_until(b + n_rend + kPrepAhead + 1)
            if b + n_rend < len(starts):   # (renderer b % n_rend is free again)
                queued.append(ahead.submit(render_batch, b + n_rend))
            for e in sorted({f // 10 for f in fb}):
                if e not in pose_cache:
                    pose_cache[e] = object_poses(wl.scene, wl.epoch(e).object_frames)
            for k, f in enumerate(fb):
                if failed[k]:   # every validation attempt failed: logged, nothing written (GDP:1662-1666)
                    log.frame_failed(f, wl.camera(f)[3], checks[k])
                    continue
                V, P, C, cam, aim, q = wl.camera(f, attempts[k])
                listed = (in_frustum(wl.scene, wl.epoch(f // 10).object_frames, V, P, wl.width, wl.height,
                                     intr.near, intr.far) if object_list == "frustum" else None)
                if lw is not None:
                    ep = lw.epoch(f // 10, pose_cache[f // 10])
                    lab = partial(lw.write, frame_id=f, camera_pose=cm.get_obj_pose_from_matrix(C), ep=ep,
                                  inst_stats=out["inst_stats"][k], covered=cov_of(out, k),
                                  kp_uv=out["keypoints_uv"][k], kp_vis=out["keypoints_vis"][k], listed=listed)
                    n_obj = lw.n_visible(ep, out["inst_stats"][k], listed)
                else:
                    lab = label_record(f, cm.get_obj_pose_from_matrix(C), intr.params(), pose_cache[f // 10],
                                       out["inst_stats"][k], out["keypoints_uv"][k], out["keypoints_vis"][k],
                                       wl.kp_table, wl.height, wl.width, covered=cov_of(out, k),
                                       listed=listed)
                    n_obj = lab["num_objects"]
                log_args = dict(n_objects=n_obj, kp_vis=out["keypoints_vis"][k].copy(), frame_id=f,
                                cam_pos=wl.camera(f)[3] if attempts[k] else cam, failed_checks=checks[k],
                                depth_range=out["depth_range"][k].copy() if "depth_range" in out else None)
                if "depth_stats" in out:   # valid, zero, inf, sum, min, max (csg_outputs.depth_stats)
                    v = out["depth_stats"][k].tolist()
                    log_args["gpu_depth_stats"] = {"valid": int(v[0]), "zero": int(v[1]), "inf": int(v[2]),
                                                   "total": wl.width * wl.height, "sum": v[3], "min": v[4],
                                                   "max": v[5]}
                files = []
                if kinds:   # GPU-encoded: file j = frame * nk + index of its kind
                    for o, kd in FILE_OF_OUTPUT:
                        if o in outs:
                            files.append((file_path(out_dir, o, f),
                                          "encoded_pointcloud" if o == "pointcloud" else "encoded",
                                          (k * nk + kinds.index(kd),)))
                elif "rgb" in outs:
                    files.append((file_path(out_dir, "rgb", f), "png", ("rgb",)))
                if "mask" in outs:
                    files.append((os.path.join(out_dir, "labels", f"instance_mask_{f:06d}.npy"), "npy", ("instance",)))
                if "depth_npy" in outs:
                    files.append((os.path.join(out_dir, "depth", f"depth_{f:06d}.npy"), "npy", ("depth",)))
                if "depth_csv" in outs and not kinds:
                    files.append((file_path(out_dir, "depth_csv", f), "csv", ("depth",)))
                if "depth_png" in outs and not kinds:
                    files.append((file_path(out_dir, "depth_png", f), "png", ("depth_vis",)))
                if "pointcloud" in outs and not kinds:
                    files.append((file_path(out_dir, "pointcloud", f), "pointcloud", ("points", "rgb")))
                if "normals" in outs:
                    files.append((os.path.join(out_dir, "normals", f"normals_{f:06d}.npy"), "npy", ("normals",)))
                fut = pool.submit(slot, k, files, lab, os.path.join(out_dir, "labels", f"label_{f:06d}.json"))
                pending.append((fut, log_args))
            del out
            t_labels += time.time() - tl
            # log frames in order as they complete
            while pending and pending[0][0].done():
                _log_done(log, *pending.pop(0), "pointcloud" in outs)
        for p in pending:
            _log_done(log, *p, "pointcloud" in outs)
        t_done = time.time()   # every file written (teardown below: freeing page-locked buffers)
    finally:
        ahead.shutdown(wait=True)
        prep.shutdown(wait=True)
        if ppool is not None:
            ppool.shutdown(wait=True, cancel_futures=True)
        pool.close()
        t_close = time.time()
        for x in rends:
            x.close()
    wall = t_done - t0
    t_teardown = time.time() - t_close
    log.save()
    summary = log.summary()
    summary["throughput"] = {"frames": len(frames), "wall_s": round(wall, 3), "render_s": round(t_render, 3),
                             "render_thread": {"render_s": round(t_render, 3), "slot_wait_s": round(t_slot_wait, 3),
                                               "epoch_prep_s": round(t_prep, 3)},
                             "main_thread": {"wait_render_s": round(t_main_wait, 3), "labels_s": round(t_labels, 3)},
                             "frames_per_s": round(len(frames) / wall, 2) if wall > 0 else None,
                             "writers": n_writers, "writer_mode": writer_mode, "renderers": n_rend,
                             "writer_task_s": round(pool.task_s, 3), "teardown_s": round(t_teardown, 3),
                             "d2h_bytes": int(sum(d2h)), "d2h_bytes_per_frame": round(sum(d2h) / max(len(frames), 1)),
                             "d2h_gbs": round(sum(d2h) / wall / 1e9, 2) if wall > 0 else None,
                             "ids_wire_bytes": ids_wire,
                             "render_busy": round(t_render / (wall * n_rend), 3) if wall > 0 else None,
                             "sink": sink, "prep_workers": n_prep,
                             "writer_busy": round(pool.task_s / (wall * n_writers), 3) if wall > 0 else None,
                             "outputs": sorted(outs)}
    return summary


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
    ap.add_argument("--outputs", default="reference",
                    help=f"'reference' ({','.join(REFERENCE_OUTPUTS)}), 'all', or a comma list of {OUTPUTS}")
    ap.add_argument("--depth", action="store_true", help="add depth .npy")
    ap.add_argument("--depth-csv", action="store_true", help="add depth .npy and CSV")
    ap.add_argument("--pointcloud", action="store_true")
    ap.add_argument("--normals", action="store_true")
    ap.add_argument("--writers", type=int, default=0, help="writer processes (0: the CPUs this process may use)")
    ap.add_argument("--writer-mode", default="thread", choices=("thread", "process"))
    ap.add_argument("--renderers", type=int, default=0,
                    help="renderer contexts rendering alternate batches (0: 3 with writer threads, else 1)")
    ap.add_argument("--object-list", default="visible", choices=OBJECT_LISTS,
                    help="objects in each label file: with visible pixels, or also every one in the view frustum")
    ap.add_argument("--occlusion", action="store_true",
                    help="add occlusion_ratio per object to the label files (not in the reference's schema; "
                         "costs the unoccluded-coverage raster)")
    ap.add_argument("--no-resume", action="store_true")
    ap.add_argument("--sink", default="disk", choices=("disk", "discard"),
                    help="discard: the whole pipeline, every file written to /dev/null (steady-state measurement)")
    ap.add_argument("--validate-pointcloud", action="store_true",
                    help="re-render frames with fewer than --min-points points from a jittered camera "
                         "(the reference's enable_pointcloud_validation, off by default there too)")
    ap.add_argument("--min-points", type=int, default=100, help="point-cloud validation threshold (GDP:59)")
    ap.add_argument("--max-retries", type=int, default=5, help="validation attempts per frame (GDP:60)")
    ap.add_argument("--prep-workers", type=int, default=-1,
                    help="processes preparing batches ahead (-1: two for runs of >= 20 batches)")
    a = ap.parse_args(argv)
    frames = shard_of_range(a.rank, a.world, a.frames)
    out = os.path.join(a.out, f"shard_{a.rank:02d}") if a.world > 1 else a.out
    summary = generate(out, frames, a.workload, a.seed, a.batch, a.device, a.depth, a.depth_csv, a.pointcloud,
                       a.width, a.height, writers=a.writers, resume=not a.no_resume, normals=a.normals,
                       outputs=parse_outputs(a.outputs), writer_mode=a.writer_mode, renderers=a.renderers,
                       object_list=a.object_list, occlusion=a.occlusion, sink=a.sink,
                       validate_pointcloud=a.validate_pointcloud, min_points=a.min_points, max_retries=a.max_retries,
                       prep_workers=a.prep_workers)
    print(json.dumps(summary))


if __name__ == "__main__":
    main()
