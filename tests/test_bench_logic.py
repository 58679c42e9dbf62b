"""bench.py's host-side arithmetic (CPU): rank sharding of the timed steps,
the verified sample, the max-over-ranks elapsed time (gloo, world size 2)
and the roofline / baseline bookkeeping."""
import os
import socket
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

import bench  # noqa: E402


@pytest.mark.parametrize("world", [1, 2, 4, 8])
def test_step_frames_are_disjoint_and_fixed_per_rank(world):
    F, W, K = 40, 2, 3
    per_rank = [bench.rank_frames(r, world, W + K, F) for r in range(world)]
    for r, fr in enumerate(per_rank):
        assert len(fr) == (W + K) * F                      # weak scaling: fixed work per rank
        assert all((f // 10) % world == r for f in fr)     # the rank's own epochs only
        assert bench.timed_frames(fr, W, K, F) == fr[W * F:]
    flat = [f for fr in per_rank for f in fr]
    assert len(set(flat)) == len(flat)                     # no frame rendered twice


def test_sample_frames_lie_in_the_last_timed_step():
    F, W, K = 240, 3, 20
    idx = bench.verify_sample_indices(F, 32)
    assert len(idx) == 32 and len(set(idx)) == 32
    assert idx[0] == 0 and idx[-1] == F - 1 and all(0 <= k < F for k in idx)
    assert bench.verify_sample_indices(F, 0) == []
    assert bench.verify_sample_indices(5, 9) == [0, 1, 2, 3, 4]
    fr = bench.rank_frames(0, 1, W + K, F)
    timed = bench.timed_frames(fr, W, K, F)
    last = timed[(K - 1) * F:]
    assert all(last[k] in timed for k in idx)


def test_value_is_aggregate_over_ranks():
    assert bench.aggregate_value(steps=20, frames_per_step=240, world=8, elapsed_max=2.0) == 20 * 240 * 8 / 2.0


def test_roofline_formula_follows_survey_8d():
    M = 10 ** 6
    r = bench.roofline(b_geom=1000 * M, b_tex=200 * M, b_out=300 * M, frames_per_launch=10, raster_ms=2.0,
                       setup_ms=1.0, records_per_frame=5 * M, fps=1000.0, traffic={"k_raster": 99})
    b_frame = 1500 * M
    # headline: BASELINE.md:44, fps x B_frame / peak
    assert r["B_frame"] == b_frame
    assert r["achieved"] == pytest.approx(1000.0 * b_frame / 1e9, rel=1e-3)
    assert r["frac"] == pytest.approx(1000.0 * b_frame / (bench.HBM_PEAK_GBS * 1e9), rel=1e-3)
    assert r["traffic"] == 99 and r["bound"] == "hbm" and r["unit"] == "GB/s" and r["avg_launch_ms"] == 2.0
    own, whole, setup = r["kernels"]
    assert own["kernel"] == whole["kernel"] == "k_raster" and setup["kernel"] == "k_setup"
    assert own["bytes_per_launch"] == 10 * (200 + 300) * M
    assert whole["bytes_per_launch"] == 10 * b_frame
    assert whole["achieved"] == pytest.approx(10 * b_frame / 2e-3 / 1e9, rel=1e-3)
    assert setup["bytes_per_launch"] == (1000 + 10 * 5 * bench.RECORD_BYTES) * M   # geometry once per launch


def test_median_timing_runs_warmup_then_five():
    calls = []
    t = bench.median_time(lambda: calls.append(1), runs=5, warmup=1)
    assert len(calls) == 6 and t >= 0.0


def test_cpu_description_is_recorded():
    assert bench.available_cpus() >= 1
    assert isinstance(bench.cpu_model(), str) and bench.cpu_model()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _rank_worker(rank, world, port, out):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    got = bench.max_over_ranks(0.5 + rank, world)
    tot = bench.sum_over_ranks([4, rank], world)
    if rank == 0:
        with open(out, "w") as fh:
            fh.write(repr((got, tot)))
    dist.barrier()
    dist.destroy_process_group()


def test_elapsed_is_max_and_counts_sum_over_ranks_gloo(tmp_path):
    import torch.multiprocessing as mp
    out = str(tmp_path / "res.txt")
    mp.spawn(_rank_worker, args=(2, _free_port(), out), nprocs=2, join=True)
    got, tot = eval(open(out).read())
    assert got == 1.5 and tot == [8, 1]


def test_default_frames_per_step_by_frame_size():
    assert bench.default_frames_per_step(1920, 1080) == bench.DEFAULT_FRAMES_PER_STEP
    assert bench.default_frames_per_step(3840, 2160) == bench.LARGE_FRAMES_PER_STEP < bench.DEFAULT_FRAMES_PER_STEP


def test_shard_report_single_rank_and_gloo_pair(tmp_path):
    import bench
    r = bench.shard_report(list(range(20, 40)), 1)
    assert r == {"ranks": 1, "timed_frames_per_rank": [20], "union": 20, "disjoint": True,
                 "epochs_mod_world": [[0]]}
    import torch.multiprocessing as mp
    mp.spawn(_shard_worker, args=(_free_port(), str(tmp_path)), nprocs=2, join=True)
    import json
    rep = json.load(open(tmp_path / "rep.json"))
    assert rep["disjoint"] and rep["union"] == 2 * 3 * 20 and rep["epochs_mod_world"] == [[0], [1]]
    # two ranks on the one device of a rehearsal box say so
    assert [d["rank"] for d in rep["devices"]] == [0, 1]
    assert rep["distinct_devices"] == 1 and rep["shared_devices"] is True
    # each rank's own timing, gathered: which rank set elapsed_max, by how much
    assert [p["rank"] for p in rep["per_rank"]] == [0, 1]
    assert rep["per_rank"][1]["stage_ms_per_step"]["ms_raster"] == 11.0
    assert rep["slowest_rank"] == 1 and rep["imbalance"] == 1.25
    # every rank's host-delivery leg: per-rank rates and the aggregate over the slowest rank's time
    dl = json.load(open(tmp_path / "delivery.json"))
    assert dl["ranks"] == 2 and [x["rank"] for x in dl["per_rank"]] == [0, 1]
    assert dl["value"] == round((480 + 480) / 2.0, 2)
    assert dl["per_rank"][0]["frames_per_s"] == 320.0 and dl["per_rank"][1]["frames_per_s"] == 240.0
    assert dl["wire_gbs"] == round((480 + 480) * 8.0e6 / 2.0 / 1e9, 2)
    assert bench.gather_delivery(None, 1) is None


def _shard_worker(rank, port, out_dir):
    import json
    import os
    import torch.distributed as dist
    import bench
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=2)
    fids = bench.rank_frames(rank, 2, 4, 20)
    dev = {"rank": rank, "local_rank": rank, "device": 0, "device_count": 1, "pci": "0000:05:00"}
    mine = {"rank": rank, "elapsed_s": 2.0 + 0.5 * rank, "frames_per_s": 30.0 / (2.0 + 0.5 * rank),
            "stage_ms_per_step": {"ms_setup": 1.0, "ms_bin": 0.5, "ms_raster": 10.0 + rank, "ms_keypoints": 0.1}}
    rep = bench.shard_report(bench.timed_frames(fids, 1, 3, 20), 2, dev, mine)
    leg = {"frames": 480, "seconds": 1.5 + 0.5 * rank, "wire_bytes": 480 * 8.0e6, "delivered_bytes": 480 * 14.5e6}
    dl = bench.gather_delivery(leg, 2)
    if rank == 0:
        json.dump(rep, open(os.path.join(out_dir, "rep.json"), "w"))
        json.dump(dl, open(os.path.join(out_dir, "delivery.json"), "w"))
    dist.barrier()
    dist.destroy_process_group()


_CHILD = r"""
import os, sys, time
r, n = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
assert os.environ["LOCAL_RANK"] == str(r) and os.environ["MASTER_ADDR"] == "127.0.0.1"
assert int(os.environ["MASTER_PORT"]) > 0
mode = sys.argv[1]
if mode == "fail" and r == n - 1:
    sys.stderr.write("rank failing on purpose\n")
    sys.exit(7)
if mode == "crash" and r == 1:
    os.kill(os.getpid(), 9)
if mode in ("fail", "crash", "hang"):
    time.sleep(120 if mode == "hang" or r == 0 else 0)   # the others wait: they must be stopped
print("noise that is not a result line")
if r == 0:
    print('{"n_gpus": %d, "rank": 0}' % n, flush=True)
"""


def _launch(mode, n, tmp_path):
    import io
    import time as _t
    script = tmp_path / "child.py"
    script.write_text(_CHILD)
    buf = io.StringIO()
    t0 = _t.time()
    rc = bench.launch_ranks(n, [sys.executable, str(script), mode], env=dict(os.environ), out=buf,
                            poll_s=0.05, grace_s=5.0)
    return rc, buf.getvalue(), _t.time() - t0


@pytest.mark.parametrize("n", [2, 4])
def test_launcher_forwards_rank0_line(tmp_path, n):
    """A plain `bench.py --gpus N` starts N ranks itself: each child sees its
    RANK / LOCAL_RANK and the shared WORLD_SIZE / MASTER_*, and only rank 0's
    JSON line is forwarded."""
    env_before = dict(os.environ)
    rc, out, _ = _launch("ok", n, tmp_path)
    assert rc == 0
    assert out.splitlines() == ['{"n_gpus": %d, "rank": 0}' % n]
    assert dict(os.environ) == env_before          # the parent's environment is untouched


@pytest.mark.parametrize("mode,code", [("fail", 7), ("crash", 1)])
def test_launcher_failing_child_gives_no_line(tmp_path, mode, code):
    """Any failing rank -- an error exit, or a rank killed by a signal --
    stops the other ranks (rank 0 sleeps 120 s here), and the launcher exits
    non-zero without printing a line."""
    rc, out, dt = _launch(mode, 3, tmp_path)
    assert rc == code and out == ""
    assert dt < 60


def test_bench_main_launches_ranks_without_torchrun(tmp_path, monkeypatch):
    """`main()` with --gpus 2 and no WORLD_SIZE hands over to launch_ranks
    before importing torch, passing its own arguments to the children."""
    seen = {}

    def fake(n, argv, **kw):
        seen["n"], seen["argv"] = n, argv
        return 5
    monkeypatch.delenv("WORLD_SIZE", raising=False)
    monkeypatch.setattr(bench, "launch_ranks", fake)
    monkeypatch.setattr(sys, "argv", ["bench.py", "--gpus", "2", "--steps", "3"])
    with pytest.raises(SystemExit) as ex:
        bench.main()
    assert ex.value.code == 5 and seen["n"] == 2
    assert seen["argv"][0] == sys.executable and seen["argv"][1].endswith("bench.py")
    assert seen["argv"][2:] == ["--gpus", "2", "--steps", "3"]


def test_shard_report_devices():
    r = bench.shard_report([1, 2], 1, {"rank": 0, "local_rank": 0, "device": 0, "device_count": 1, "pci": "0000:05:00"})
    assert r["devices"][0]["pci"] == "0000:05:00" and r["distinct_devices"] == 1 and r["shared_devices"] is False


@pytest.mark.parametrize("steps,warmup", [(20, 5), (10, 2), (200, 10)])
def test_transform_sets_fit_the_library_for_driver_runs(steps, warmup):
    """Every randomisation epoch of a rank's schedule takes one transform set:
    at the default 2,880 frames per step the driver's `--steps 20 --warmup 5`
    needs 7,200 sets (past round 4's first limit of 4,096); the library holds
    MAX_SETS and the bench fails early, with a message, beyond that."""
    F = bench.DEFAULT_FRAMES_PER_STEP
    fids = bench.rank_frames(0, 1, steps + warmup, F)
    assert len({f // 10 for f in fids}) <= bench.MAX_SETS
    src = open(os.path.join(os.path.dirname(bench.__file__), "constructionsceneposeestimation_amd", "csrc",
                            "csg_api.cpp")).read()
    assert f"constexpr uint32_t kMaxSets = {bench.MAX_SETS};" in src


def test_profiler_preload_is_detected():
    """`rocprofv3 --pmc -- python bench.py --gpus N` would start the
    ranks from a process the profiler's preload already initialised the GPU in."""
    assert bench.profiler_preload({}) is None
    assert bench.profiler_preload({"LD_PRELOAD": "/usr/lib/libfoo.so"}) is None
    assert bench.profiler_preload({"LD_PRELOAD": "/opt/rocm/lib/librocprofiler-sdk-tool.so"})
    assert bench.profiler_preload({"ROCPROF_OUTPUT_PATH": "/tmp/x"})


def test_plain_multi_gpu_bench_refuses_under_a_profiler(monkeypatch):
    monkeypatch.setattr(sys, "argv", ["bench.py", "--gpus", "2"])
    monkeypatch.delenv("WORLD_SIZE", raising=False)
    monkeypatch.setenv("ROCPROF_OUTPUT_PATH", "/tmp/x")
    called = []
    monkeypatch.setattr(bench, "launch_ranks", lambda *a, **k: called.append(a) or 0)
    with pytest.raises(SystemExit) as e:
        bench.main()
    assert e.value.code == 2 and not called
