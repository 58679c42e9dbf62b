"""Per-run quality log (the role of the reference's ``DataQualityLogger``,
generate_construction_data.py:237-470).

* ``logs/generation_detail.log``: one block per frame (camera position, RGB,
  depth validity / range / mean, point count, labels, issues) and the
  summary report at the end (:254-263, :265-387, :413-463, messages in
  English);
* ``logs/generation_summary.json``: ``statistics`` with the reference's
  fields (:243-253, :389-411), ``frame_logs`` (one entry per frame, :377-387),
  and ``counters`` -- plain integers, so the shards of a multi-GPU run merge
  by summation (shard.merge_counters).

The depth statistics take the GPU's per-frame min / max (``depth_range`` of
the depth-visualisation kernels) when given; the counts and the mean come
from one native pass over the host depth (writers.depth_stats), which the
generator runs in its writer threads.
"""
from __future__ import annotations

import json
import os
import time
from typing import Dict, List, Optional, Sequence

import numpy as np


class QualityLog:
    def __init__(self, log_dir: Optional[str] = None, detail: bool = True):
        self.log_dir = log_dir
        self.t0 = time.time()
        self.c: Dict[str, int] = {
            "total_attempts": 0, "successful_frames": 0, "failed_frames": 0,
            "rgb_success": 0, "depth_success": 0, "labels_with_objects": 0, "labels_empty": 0,
            "total_objects": 0, "depth_valid_pixels": 0, "depth_total_pixels": 0,
            "keypoints_visible": 0, "keypoints_total": 0,
        }
        self.stats = {
            "total_frames_attempted": 0, "successful_frames": 0, "failed_frames": 0, "retry_count": 0,
            "pointcloud_stats": {"valid": 0, "empty": 0, "insufficient": 0},
            "rgb_stats": {"valid": 0, "failed": 0},
            "depth_stats": {"valid": 0, "failed": 0, "all_zero": 0, "all_inf": 0},
            "label_stats": {"valid": 0, "empty": 0},
            "object_count": {"total": 0, "per_frame_avg": 0},
        }
        self.issues: Dict[str, int] = {}
        self.frame_logs: List[dict] = []
        self._lines: List[str] = []
        self.detail_path = None
        if log_dir and detail:
            os.makedirs(log_dir, exist_ok=True)
            self.detail_path = os.path.join(log_dir, "generation_detail.log")
            with open(self.detail_path, "w", encoding="utf-8") as f:
                f.write("=== generation detail log ===\n")
                f.write(f"start: {time.strftime('%Y%m%d_%H%M%S')}\n\n")

    # -- per frame -------------------------------------------------------------
    def frame(self, n_objects: int, depth: Optional[np.ndarray] = None, kp_vis: Optional[np.ndarray] = None,
              frame_id: Optional[int] = None, cam_pos: Optional[Sequence[float]] = None,
              depth_range: Optional[Sequence[float]] = None, points: Optional[int] = None,
              depth_stats: Optional[dict] = None, failed_checks: Sequence[int] = ()) -> dict:
        """Record one rendered frame (the reference's log_frame_start ...
        log_frame_end sequence for a frame that succeeded).  The depth entry
        comes from ``depth_stats`` (writers.depth_stats, computed by a writer
        thread) or from the ``depth`` array.  ``failed_checks``: the point
        counts of the point-cloud validation attempts that failed before this
        one passed (GDP:1573-1645; one retry each, log_retry :278-283)."""
        rec = {"frame_id": int(frame_id) if frame_id is not None else self.c["total_attempts"],
               "camera_position": [float(x) for x in cam_pos] if cam_pos is not None else None,
               "retry_count": 0, "status": "processing", "issues": []}
        msg = [f"\n{'=' * 60}\nframe {rec['frame_id']} start\ncamera position: {rec['camera_position']}\n"]
        self._retries(rec, msg, failed_checks)
        self.c["total_attempts"] += 1
        self.c["successful_frames"] += 1
        self.c["rgb_success"] += 1
        self.stats["rgb_stats"]["valid"] += 1
        rec["rgb"] = {"status": "valid"}
        msg.append("  + RGB ok\n")
        if depth_stats is None and depth is not None:
            from .writers import depth_stats as _stats
            depth_stats = _stats(depth)
        if depth_stats is not None:
            self._depth(rec, msg, depth_stats, depth_range)
        if points is not None:
            if points > 0:
                self.stats["pointcloud_stats"]["valid"] += 1
                rec["pointcloud"] = {"status": "valid", "points": int(points)}
                msg.append(f"  + point cloud: {int(points)} points\n")
            else:
                self.stats["pointcloud_stats"]["empty"] += 1
                rec["issues"].append("point cloud empty: no pixel hit")
                msg.append("  - point cloud empty\n")
        self.c["total_objects"] += int(n_objects)
        self.c["labels_with_objects" if n_objects else "labels_empty"] += 1
        if n_objects:
            self.stats["label_stats"]["valid"] += 1
            self.stats["object_count"]["total"] += int(n_objects)
            rec["labels"] = {"status": "valid", "object_count": int(n_objects)}
            msg.append(f"  + labels: {int(n_objects)} objects\n")
        else:
            self.stats["label_stats"]["empty"] += 1
            rec["issues"].append("no labelled object in view")
            self.issue("no labelled object in view")
            msg.append("  ! labels: 0 objects (out of view or unmatched class)\n")
        if kp_vis is not None:
            self.c["keypoints_visible"] += int((kp_vis == 2).sum())
            self.c["keypoints_total"] += int(kp_vis.size)
        self.stats["total_frames_attempted"] += 1
        self.stats["successful_frames"] += 1
        rec["status"] = "success"
        msg.append(f">>> frame {rec['frame_id']} done\n")
        self.frame_logs.append(rec)
        self._lines.append("".join(msg))
        if len(self._lines) >= 64:
            self.flush()
        return rec

    def _retries(self, rec: dict, msg: List[str], failed_checks: Sequence[int]) -> None:
        """The point-cloud validation's failed attempts (GDP:1626-1645): each
        counts as an empty or insufficient point cloud, each but a last
        failing one leads to a retry (log_retry, :278-283)."""
        for k, n in enumerate(failed_checks):
            n = int(n)
            if n == 0:
                self.stats["pointcloud_stats"]["empty"] += 1
                rec["issues"].append("point cloud empty: no pixel hit")
                msg.append("  - point cloud empty\n")
            else:
                self.stats["pointcloud_stats"]["insufficient"] += 1
                rec["issues"].append(f"point cloud insufficient: {n} points")
                msg.append(f"  - point cloud insufficient: {n} points\n")
        retries = len(failed_checks)
        rec["retry_count"] = retries
        self.stats["retry_count"] += retries
        for k in range(1, retries + 1):
            msg.append(f"  ! retry {k}\n")

    def frame_failed(self, frame_id: int, cam_pos: Optional[Sequence[float]], failed_checks: Sequence[int]) -> dict:
        """A frame whose every validation attempt failed: the reference logs it
        failed and writes nothing for it (GDP:1662-1666, log_frame_end(False)
        :374-387).  Its attempts beyond the first were retries."""
        rec = {"frame_id": int(frame_id), "camera_position": [float(x) for x in cam_pos] if cam_pos is not None else None,
               "retry_count": 0, "status": "processing", "issues": []}
        msg = [f"\n{'=' * 60}\nframe {rec['frame_id']} start\ncamera position: {rec['camera_position']}\n"]
        self._retries(rec, msg, failed_checks)
        # the last failed check ends the loop without a retry
        rec["retry_count"] = max(0, len(failed_checks) - 1)
        self.stats["retry_count"] -= 1 if failed_checks else 0
        if failed_checks:
            msg.pop()
        self.c["total_attempts"] += 1
        self.c["failed_frames"] += 1
        self.stats["total_frames_attempted"] += 1
        self.stats["failed_frames"] += 1
        rec["status"] = "failed"
        msg.append(f">>> frame {rec['frame_id']} failed\n")
        self.frame_logs.append(rec)
        self._lines.append("".join(msg))
        return rec

    def _depth(self, rec: dict, msg: List[str], ds: dict, depth_range) -> None:
        self.c["depth_success"] += 1
        n_valid, total, zero, inf = ds["valid"], ds["total"], ds["zero"], ds["inf"]
        self.c["depth_valid_pixels"] += n_valid
        self.c["depth_total_pixels"] += total
        if n_valid:
            if depth_range is not None and np.isfinite(depth_range).all():
                lo, hi = float(depth_range[0]), float(depth_range[1])   # the GPU's min / max (depth PNG)
            else:
                lo, hi = ds["min"], ds["max"]
            # float64 sum / count.  Deliberate divergence: the
            # reference's np.mean(valid_depth) (GDP:328) sums its float32 array
            # pairwise in float32 and returns a float32; the two agree to ~1e-6
            # relative (tests/test_labels.py), not in the logged low digits.
            mean = ds["sum"] / n_valid
        else:
            lo = hi = mean = 0.0
        rec["depth"] = {"status": "valid", "valid_pixels": n_valid, "total_pixels": total,
                        "valid_ratio": n_valid / total, "zero_pixels": zero, "inf_pixels": inf,
                        "depth_range": [lo, hi], "depth_mean": mean}
        if zero == total:
            self.stats["depth_stats"]["all_zero"] += 1
            rec["issues"].append("depth all zero")
            msg.append("  ! depth: all zero\n")
        elif inf == total:
            self.stats["depth_stats"]["all_inf"] += 1
            rec["issues"].append("depth all inf")
            self.issue("depth all inf")
            msg.append("  ! depth: all inf\n")
        else:
            self.stats["depth_stats"]["valid"] += 1
            msg.append(f"  + depth: valid pixels {n_valid}/{total} ({100 * n_valid / total:.1f}%)\n"
                       f"    depth range: [{lo:.2f}, {hi:.2f}] mean: {mean:.2f}\n")

    def issue(self, what: str):
        self.issues[what] = self.issues.get(what, 0) + 1

    # -- output ----------------------------------------------------------------
    def flush(self) -> None:
        if self.detail_path and self._lines:
            with open(self.detail_path, "a", encoding="utf-8") as f:
                f.write("".join(self._lines))
        self._lines = []

    def summary(self) -> dict:
        n = max(self.c["total_attempts"], 1)
        return {"counters": dict(self.c), "issues": dict(self.issues),
                "success_rate": self.c["successful_frames"] / n,
                "avg_objects_per_frame": self.c["total_objects"] / n,
                "elapsed_s": round(time.time() - self.t0, 3)}

    def statistics(self) -> dict:
        st = json.loads(json.dumps(self.stats))
        if st["successful_frames"]:
            st["object_count"]["per_frame_avg"] = st["object_count"]["total"] / st["successful_frames"]
        st["success_rate"] = st["successful_frames"] / max(1, st["total_frames_attempted"])
        return st

    def report(self) -> str:
        st = self.statistics()
        r = ["=== generation summary report ===\n\n",
             "overall:\n", f"  attempted frames: {st['total_frames_attempted']}\n",
             f"  successful frames: {st['successful_frames']}\n", f"  failed frames: {st['failed_frames']}\n",
             f"  success rate: {st['success_rate'] * 100:.1f}%\n", f"  retries: {st['retry_count']}\n\n",
             "point cloud:\n", f"  valid: {st['pointcloud_stats']['valid']}\n",
             f"  empty: {st['pointcloud_stats']['empty']}\n",
             f"  insufficient: {st['pointcloud_stats']['insufficient']}\n\n",
             "RGB:\n", f"  ok: {st['rgb_stats']['valid']}\n", f"  failed: {st['rgb_stats']['failed']}\n\n",
             "depth:\n", f"  valid: {st['depth_stats']['valid']}\n", f"  failed: {st['depth_stats']['failed']}\n",
             f"  all zero: {st['depth_stats']['all_zero']}\n", f"  all inf: {st['depth_stats']['all_inf']}\n\n",
             "labels:\n", f"  valid: {st['label_stats']['valid']}\n", f"  empty: {st['label_stats']['empty']}\n",
             f"  objects: {st['object_count']['total']}\n",
             f"  per frame: {st['object_count']['per_frame_avg']:.2f}\n\n", "issues:\n"]
        counts: Dict[str, int] = {}
        for fr in self.frame_logs:
            for issue in fr.get("issues", []):
                k = issue.split(":")[0]
                counts[k] = counts.get(k, 0) + 1
        for k, v in sorted(counts.items(), key=lambda x: x[1], reverse=True):
            r.append(f"  {k}: {v}\n")
        return "".join(r)

    def save(self) -> Optional[str]:
        if not self.log_dir:
            return None
        os.makedirs(self.log_dir, exist_ok=True)
        self.flush()
        if self.detail_path:
            with open(self.detail_path, "a", encoding="utf-8") as f:
                f.write(f"\n\n{'=' * 60}\n" + self.report())
        path = os.path.join(self.log_dir, "generation_summary.json")
        data = self.summary()
        data["statistics"] = self.statistics()
        data["frame_logs"] = self.frame_logs
        with open(path, "w", encoding="utf-8") as f:
            json.dump(data, f, indent=2, ensure_ascii=False)
        return path
