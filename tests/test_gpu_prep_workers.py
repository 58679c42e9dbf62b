"""generate() with its batches prepared in worker processes (prep_pool.py:
epoch layouts, object poses and cameras computed outside the generator's
process) writes the same files, byte for byte, as with the preparation in
its own thread (the reference's per-frame files, generate_construction_data.py:
1668-1711, :2055-2072)."""
import os

import pytest

pytestmark = pytest.mark.gpu


def _files(root):
    out = {}
    for d, _, fs in os.walk(root):
        if os.path.basename(d) == "logs":   # the logs carry timings
            continue
        for f in fs:
            p = os.path.join(d, f)
            out[os.path.relpath(p, root)] = open(p, "rb").read()
    return out


def test_prep_workers_write_the_same_files(tmp_path):
    from constructionsceneposeestimation_amd.generate import generate
    kw = dict(workload="C4", seed=3, batch=6, width=160, height=96)   # C4: DR lights and textures per epoch
    frames = list(range(0, 48, 2)) + [101, 355]
    a = generate(str(tmp_path / "thread"), frames, prep_workers=0, **kw)
    b = generate(str(tmp_path / "procs"), frames, prep_workers=2, **kw)
    assert a["throughput"]["prep_workers"] == 0 and b["throughput"]["prep_workers"] == 2
    assert a["counters"]["successful_frames"] == b["counters"]["successful_frames"] == len(frames)
    fa, fb = _files(tmp_path / "thread"), _files(tmp_path / "procs")
    assert fa.keys() == fb.keys() and len(fa) >= 5 * len(frames)
    for k in fa:
        assert fa[k] == fb[k], k
