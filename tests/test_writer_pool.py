"""The generator's writer pool (writer_pool.py) on the CPU: frames handed to
worker processes through shared memory are written byte-identically to the
thread-mode writers, label JSON last, and the shared segment is released."""
import json
import os

import numpy as np
import pytest


def _fill(arrays, n, rng):
    for k, a in arrays.items():
        if a.dtype == np.float32:
            a[...] = rng.uniform(0.5, 250.0, a.shape).astype(np.float32)
            if k == "depth":
                a[:, :2] = np.inf
        else:
            a[...] = rng.integers(0, 200, a.shape).astype(a.dtype)


def _run(tmp, mode):
    from constructionsceneposeestimation_amd.writer_pool import WriterPool
    H, W, n = 12, 20, 3
    spec = {"rgb": ((n, H, W, 3), np.uint8), "instance": ((n, H, W), np.int32), "depth": ((n, H, W), np.float32),
            "depth_vis": ((n, H, W, 3), np.uint8)}
    pool = WriterPool(spec, workers=2, n_slots=2, mode=mode)
    rng = np.random.default_rng(5)
    stats = []
    try:
        for b in range(3):                      # three batches over two slots: slot reuse waits
            slot = b % 2
            arrays = pool.arrays(slot)
            _fill(arrays, n, rng)
            for k in range(n):
                f = b * n + k
                files = [(os.path.join(tmp, f"rgb_{f}.png"), "png", ("rgb",)),
                         (os.path.join(tmp, f"mask_{f}.npy"), "npy", ("instance",)),
                         (os.path.join(tmp, f"depth_{f}.csv"), "csv", ("depth",)),
                         (os.path.join(tmp, f"depth_{f}.png"), "png", ("depth_vis",))]
                stats.append(pool.submit(slot, k, files, {"frame_id": f}, os.path.join(tmp, f"label_{f}.json")))
            del arrays
        stats = [s.result() for s in stats]
    finally:
        pool.close()
    return stats


@pytest.mark.parametrize("mode", ["thread", "process"])
def test_writer_pool_files(tmp_path, mode):
    d = tmp_path / mode
    d.mkdir()
    stats = _run(str(d), mode)
    assert len(stats) == 9 and all(s["total"] == 240 and s["inf"] == 40 for s in stats)
    for f in range(9):
        assert json.load(open(d / f"label_{f}.json")) == {"frame_id": f}
        assert np.load(d / f"mask_{f}.npy").shape == (12, 20)
    assert not list(d.glob("*.tmp"))


def test_writer_pool_process_matches_threads(tmp_path):
    for mode in ("thread", "process"):
        (tmp_path / mode).mkdir()
        _run(str(tmp_path / mode), mode)
    names = sorted(os.listdir(tmp_path / "thread"))
    assert names == sorted(os.listdir(tmp_path / "process")) and len(names) == 9 * 5
    for n in names:
        assert (tmp_path / "thread" / n).read_bytes() == (tmp_path / "process" / n).read_bytes(), n
