"""End-to-end generator throughput (render on the GPU + native writers to
disk), frames/s, for DESIGN.md's writer row.  Writes under $TMPDIR.

    python tools/gen_bench.py --frames 240 --writers 16
"""
import argparse
import json
import os
import shutil
import sys
import tempfile
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from constructionsceneposeestimation_amd.generate import generate  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=240)
    ap.add_argument("--batch", type=int, default=60)
    ap.add_argument("--writers", type=int, default=16)
    ap.add_argument("--workload", default="C3")
    ap.add_argument("--depth", action="store_true")
    ap.add_argument("--pointcloud", action="store_true")
    a = ap.parse_args()
    out = tempfile.mkdtemp(prefix="csg_gen_")
    try:
        generate(out, list(range(a.batch)), a.workload, seed=9, batch=a.batch, writers=a.writers)   # warm-up
        shutil.rmtree(out)
        t0 = time.perf_counter()
        s = generate(out, list(range(a.frames)), a.workload, seed=0, batch=a.batch, writers=a.writers,
                     depth=a.depth, pointcloud=a.pointcloud)
        dt = time.perf_counter() - t0
        size = sum(os.path.getsize(os.path.join(r, f)) for r, _, fs in os.walk(out) for f in fs)
        print(json.dumps({"frames": a.frames, "seconds": round(dt, 3), "frames_per_s": round(a.frames / dt, 1),
                          "writers": a.writers, "bytes_written": size, "workload": a.workload,
                          "outputs": ["rgb.png", "labels.json", "instance_mask.npy"]
                          + (["depth.npy"] if a.depth else []) + (["pointcloud.txt"] if a.pointcloud else []),
                          "successful": s["counters"]["successful_frames"]}))
    finally:
        shutil.rmtree(out, ignore_errors=True)


if __name__ == "__main__":
    main()
