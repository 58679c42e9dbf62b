"""Host-side preparation of generate()'s batches in worker processes.

Each epoch of the schedule (10 frames, generate_construction_data.py:1542)
needs its object layout, instance transforms, human poses and keypoints
(Workload.epoch; the reference's randomize_object_positions, :914-1231) and
its objects' label poses (labels.object_poses); each frame its camera
(Workload.camera; camPosOri and the look-at, :475-550).  That is numpy work
of a few ms per epoch, and in the generator's process it holds the GIL that
the writer and render threads need: at ~1.9k frames/s without the point
cloud the generator is bound by its Python threads, not by the GPU or PCIe
(profiles/r06/generate_steady.json).  Worker processes (each with its own
Workload built from the same arguments, so the same numbers) prepare whole
batches ahead and the generator installs the results in its caches.

Imports here stay light (numpy, scipy; no torch, no renderer): the workers
are started before the generator's process touches the GPU and never use it.
"""
from __future__ import annotations

import os
from typing import Dict, List, Tuple

_WL = None


def init(workload: str, seed: int, width, height) -> None:
    """Worker initialiser: the worker's own Workload (same scene, same seed)."""
    global _WL
    from .workload import Workload
    _WL = Workload(workload, seed=seed, width=width, height=height)


def ping() -> int:
    """Held briefly, so that the executor starts another worker for the next ping."""
    import time
    time.sleep(0.05)
    return os.getpid()


def prepare(frames: List[int], epochs: List[int]) -> Tuple[Dict[int, tuple], Dict[int, tuple]]:
    """The epochs' (EpochState, object poses) and the frames' attempt-0
    cameras (V, P, C, cam, aim, q), as Workload.epoch / labels.object_poses /
    Workload.camera compute them."""
    from .labels import object_poses
    wl = _WL
    eps = {}
    for e in epochs:
        st = wl.epoch(e)
        eps[e] = (st, object_poses(wl.scene, st.object_frames))
    cams = {f: wl.camera(f) for f in frames}
    return eps, cams
