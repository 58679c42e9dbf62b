"""The bench's N>1 path as the driver's 8-GPU run starts it: two ranks under
``torch.distributed.run`` (one process per rank, gloo for the barrier and the
max-over-ranks; no data-path collective), sharing the box's one MI355X.

The test process only starts a child (``subprocess.run``) and parses its JSON
line: each rank renders its own epochs (e = r mod N), checks 4
frames of its last timed step against the oracle, and the ranks' timed frame
sets are disjoint.
"""
import json
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.timeout(900)
def test_bench_two_ranks_under_torchrun(tmp_path):
    steps, warmup, F = 2, 1, 48
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), os.path.join(ROOT, "bench.py"),
           "--gpus", "2", "--steps", str(steps), "--warmup", str(warmup), "--frames-per-step", str(F),
           "--verify-frames-multi", "4"]
    env = dict(os.environ, MASTER_ADDR="127.0.0.1")
    log = tmp_path / "bench2.err"
    with open(log, "w") as err:
        r = subprocess.run(cmd, cwd=ROOT, env=env, stdout=subprocess.PIPE, stderr=err, text=True, timeout=840)
    tail = log.read_text()[-4000:]
    assert r.returncode == 0, f"bench at N=2 failed ({r.returncode}):\n{tail}"
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["steps"] == steps and d["warmup"] == warmup
    assert d["scaling"] == "weak" and d["value"] > 0
    assert d["verified"]["frames"] == 8 and d["verified"]["bit_exact"] is True
    sh = d["shards"]
    assert sh["ranks"] == 2 and sh["disjoint"] is True
    assert sh["timed_frames_per_rank"] == [steps * F, steps * F]
    assert sh["union"] == 2 * steps * F
    assert sh["epochs_mod_world"] == [[0], [1]]
    # value = every rank's frames over the slowest rank's time
    assert abs(d["value"] - 2 * steps * F / (d["ms_per_step"] * steps / 1e3)) <= 0.01 * d["value"]


@pytest.mark.timeout(900)
def test_bench_two_ranks_plain_command(tmp_path):
    """`python3 bench.py --gpus 2` with no torchrun and no rank environment:
    bench.py starts its two ranks itself (fresh child processes, before any
    GPU call) and forwards rank 0's line, which reports both ranks, their
    devices (here both on the box's one GPU: `shared_devices`), disjoint
    shards and the oracle check."""
    steps, warmup, F = 2, 1, 48
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", str(steps), "--warmup",
           str(warmup), "--frames-per-step", str(F), "--verify-frames-multi", "4"]
    env = {k: v for k, v in os.environ.items()
           if k not in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "LOCAL_WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT")}
    log = tmp_path / "bench2plain.err"
    with open(log, "w") as err:
        r = subprocess.run(cmd, cwd=ROOT, env=env, stdout=subprocess.PIPE, stderr=err, text=True, timeout=840)
    tail = log.read_text()[-4000:]
    assert r.returncode == 0, f"plain bench --gpus 2 failed ({r.returncode}):\n{tail}"
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["verified"]["frames"] == 8 and d["verified"]["bit_exact"] is True
    sh = d["shards"]
    assert sh["ranks"] == 2 and sh["disjoint"] is True and sh["union"] == 2 * steps * F
    assert [x["rank"] for x in sh["devices"]] == [0, 1]
    ndev = sh["devices"][0]["device_count"]
    assert all(x["device_count"] == ndev for x in sh["devices"])
    assert sh["shared_devices"] is (ndev < 2)
    assert sh["distinct_devices"] == min(2, ndev)
    # each rank's own timing (round 6): elapsed seconds, frames/s, stage times;
    # the slowest rank sets ms_per_step, and the imbalance is max/min elapsed
    prs = sh["per_rank"]
    assert [x["rank"] for x in prs] == [0, 1]
    for x in prs:
        assert x["elapsed_s"] > 0 and x["frames_per_s"] > 0
        assert set(x["stage_ms_per_step"]) == {"ms_setup", "ms_bin", "ms_raster", "ms_keypoints"}
        assert all(v >= 0 for v in x["stage_ms_per_step"].values())
    el = [x["elapsed_s"] for x in prs]
    assert sh["slowest_rank"] == el.index(max(el))
    assert abs(sh["imbalance"] - max(el) / min(el)) <= 1e-3 * sh["imbalance"]
    assert abs(d["ms_per_step"] - max(el) / steps * 1e3) <= 0.01 * d["ms_per_step"]
    # the host-delivery leg on every rank at once
    pc = d["pcie_inclusive"]
    assert pc is not None and pc["ranks"] == 2 and pc["value"] > 0
    assert [x["rank"] for x in pc["per_rank"]] == [0, 1]
    assert all(x["frames"] > 0 and x["frames_per_s"] > 0 for x in pc["per_rank"])
    assert pc["ids_wire_bytes"] == 1


@pytest.mark.timeout(600)
def test_bench_single_rank_every_leg_with_hinted_pools(tmp_path):
    """N = 1 with two launch chains per step: the sizing pass's hints and
    chain pools carry the timed steps, the PCIe-inclusive leg (host frame
    records, host outputs) and the label-statistics leg without overflow."""
    steps, warmup, F, G = 2, 1, 96, 48
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--steps", str(steps), "--warmup", str(warmup),
           "--frames-per-step", str(F), "--frames-per-launch", str(G), "--verify-frames", "4",
           "--pcie-steps", "1", "--stats-steps", "1", "--cpu-single-frames", "1"]
    log = tmp_path / "bench1.err"
    with open(log, "w") as err:
        r = subprocess.run(cmd, cwd=ROOT, stdout=subprocess.PIPE, stderr=err, text=True, timeout=540)
    tail = log.read_text()[-4000:]
    assert r.returncode == 0, f"bench at N=1 failed ({r.returncode}):\n{tail}"
    assert "failed" not in log.read_text(), tail
    d = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])
    assert d["verified"]["frames"] == 4 and d["verified"]["bit_exact"] is True
    w = d["work"]
    assert w["hinted"] is True and w["frames_per_launch"] == G
    assert w["pool_records"] < G * w["records_per_frame_cap"]
    assert d["pcie_inclusive"] is not None and d["pcie_inclusive"]["value"] > 0
    assert d["with_label_stats"] is not None
