"""Per-run quality counters and summary (the role of the reference's
``DataQualityLogger``, generate_construction_data.py:237-470): attempts,
successes, depth validity, label counts and an issue histogram, written as
``generation_summary.json``.  Counters are plain integers so the shards of a
multi-GPU run merge by summation (shard.merge_counters)."""
from __future__ import annotations

import json
import os
import time
from typing import Dict, Optional

import numpy as np


class QualityLog:
    def __init__(self, log_dir: Optional[str] = None):
        self.log_dir = log_dir
        self.t0 = time.time()
        self.c: Dict[str, int] = {
            "total_attempts": 0, "successful_frames": 0, "failed_frames": 0,
            "rgb_success": 0, "depth_success": 0, "labels_with_objects": 0, "labels_empty": 0,
            "total_objects": 0, "depth_valid_pixels": 0, "depth_total_pixels": 0,
            "keypoints_visible": 0, "keypoints_total": 0,
        }
        self.issues: Dict[str, int] = {}

    def frame(self, n_objects: int, depth: Optional[np.ndarray] = None, kp_vis: Optional[np.ndarray] = None):
        self.c["total_attempts"] += 1
        self.c["successful_frames"] += 1
        self.c["rgb_success"] += 1
        self.c["total_objects"] += int(n_objects)
        self.c["labels_with_objects" if n_objects else "labels_empty"] += 1
        if n_objects == 0:
            self.issue("no labelled object in view")
        if depth is not None:
            self.c["depth_success"] += 1
            fin = np.isfinite(depth)
            self.c["depth_valid_pixels"] += int(fin.sum())
            self.c["depth_total_pixels"] += int(depth.size)
        if kp_vis is not None:
            self.c["keypoints_visible"] += int((kp_vis == 2).sum())
            self.c["keypoints_total"] += int(kp_vis.size)

    def issue(self, what: str):
        self.issues[what] = self.issues.get(what, 0) + 1

    def summary(self) -> dict:
        n = max(self.c["total_attempts"], 1)
        return {"counters": dict(self.c), "issues": dict(self.issues),
                "success_rate": self.c["successful_frames"] / n,
                "avg_objects_per_frame": self.c["total_objects"] / n,
                "elapsed_s": round(time.time() - self.t0, 3)}

    def save(self) -> Optional[str]:
        if not self.log_dir:
            return None
        os.makedirs(self.log_dir, exist_ok=True)
        path = os.path.join(self.log_dir, "generation_summary.json")
        with open(path, "w") as f:
            json.dump(self.summary(), f, indent=2)
        return path
