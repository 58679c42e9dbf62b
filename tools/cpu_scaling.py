"""CPU-baseline thread scaling (oracle/csg_oracle.c, OpenMP over frames) on
the GPU box's host, for the footnote BASELINE.md:33 plans ("OpenMP with all
cores").  The box's rules give one GPU's jobs a 16-CPU share (OMP_NUM_THREADS
is 16 there, worker pools are sized to it), so the run stops at 16 threads and
states the all-core figure as an upper bound from the measured per-thread rate.

    python tools/cpu_scaling.py [--frames 32] [--threads 1,2,4,8,16]
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=32)
    ap.add_argument("--threads", default="1,2,4,8,16",
                    help="thread counts to measure (add the box's share if it grants more than 16)")
    a = ap.parse_args()
    from bench import Verifier, available_cpus, cpu_model, rank_frames
    from constructionsceneposeestimation_amd.workload import Workload
    wl = Workload("C3", seed=0)
    fids = rank_frames(0, 1, 1, 960)[::960 // a.frames][:a.frames]
    ver = Verifier(wl, want_kp=False)
    ver.render(fids[:2], 2)   # warm-up (page-in, epoch tables)
    rows = []
    for t in [int(x) for x in a.threads.split(",")]:
        n = a.frames if t >= 4 else max(2, a.frames * t // 8)
        t0 = time.perf_counter()
        ver.render(fids[:n], t)
        dt = time.perf_counter() - t0
        rows.append({"threads": t, "frames": n, "seconds": round(dt, 3), "frames_per_s": round(n / dt, 3)})
        print(json.dumps(rows[-1]), file=sys.stderr, flush=True)
    one = rows[0]["frames_per_s"] / rows[0]["threads"]
    best = max(rows, key=lambda r: r["frames_per_s"])
    ncpu = os.cpu_count()
    print(json.dumps({
        "what": "oracle/csg_oracle.c, C3 1920x1080 frames of the bench schedule, OpenMP over frames, wall clock",
        "cpu_model": cpu_model(), "nproc": ncpu, "available_cpus": available_cpus(),
        "omp_num_threads_env": os.environ.get("OMP_NUM_THREADS"), "cpu_share": cpu_share(),
        "measured": rows, "measured_threads": [r["threads"] for r in rows],
        "largest_measured": {"threads": best["threads"], "frames_per_s": best["frames_per_s"]},
        "parallel_efficiency_at_max": round(best["frames_per_s"] / (one * best["threads"]), 3),
        "bound": {"frames_per_s": round(one * ncpu, 1), "kind": "bound, not measured",
                  "how": f"the single-thread rate x {ncpu} CPUs (perfect scaling, no SMT or memory-bandwidth loss)"},
        "note": f"not run at {ncpu} threads: the box holds a GPU job to a {os.environ.get('OMP_NUM_THREADS') or '?'}"
                "-CPU share (OMP_NUM_THREADS, worker pools); the measured runs stop there"}))


def cpu_share() -> dict:
    """What the box grants this job: the cgroup CPU quota, if any, and the affinity set."""
    out = {"affinity": available_cpus_count()}
    for p in ("/sys/fs/cgroup/cpu.max", "/sys/fs/cgroup/cpu/cpu.cfs_quota_us"):
        try:
            out[p] = open(p).read().strip()
        except OSError:
            pass
    return out


def available_cpus_count() -> int:
    try:
        return len(os.sched_getaffinity(0))
    except AttributeError:  # pragma: no cover
        return os.cpu_count() or 1


if __name__ == "__main__":
    main()
