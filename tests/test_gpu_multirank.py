"""The multi-GPU product path with the HIP library: ``generate --rank r
--world 2`` for r = 0 then r = 1 (in process, on the one device of the box)
writes shards whose union is byte-identical to a ``--world 1`` run --
masks, RGB PNGs, depth and label JSON (epochs e = r mod N, no
communication)."""
import json
import os

import pytest

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("workload,size", [("C3", (160, 96)), ("C4", (480, 272))])
def test_generate_two_rank_shards_union_equals_one_rank(tmp_path, workload, size):
    """C3 small, and C4 (per-epoch lights and texture swaps) at 480x272, with
    the reference's file set (RGB PNG, depth CSV + PNG, point cloud, mask,
    label) plus the depth .npy."""
    from constructionsceneposeestimation_amd.generate import main
    common = ["--frames", "40", "--workload", workload, "--seed", "4", "--batch", "7", "--width", str(size[0]),
              "--height", str(size[1]), "--depth-csv"]
    main(["--out", str(tmp_path / "one"), "--rank", "0", "--world", "1"] + common)
    for rank in (0, 1):
        main(["--out", str(tmp_path / "two"), "--rank", str(rank), "--world", "2"] + common)
    one = tmp_path / "one"
    shards = [tmp_path / "two" / f"shard_{r:02d}" for r in (0, 1)]
    counts = [0, 0]
    for f in range(40):
        owner = (f // 10) % 2
        counts[owner] += 1
        for rel in (f"rgb/rgb_{f:06d}.png", f"labels/instance_mask_{f:06d}.npy", f"labels/label_{f:06d}.json",
                    f"depth/depth_{f:06d}.npy", f"depth/depth_{f:06d}.csv", f"depth/depth_{f:06d}.png",
                    f"pointcloud/pointcloud_{f:06d}.txt"):
            a = (one / rel).read_bytes()
            assert a == (shards[owner] / rel).read_bytes(), (f, rel)
            assert not (shards[1 - owner] / rel).exists(), (f, rel)
        lab = json.loads((one / f"labels/label_{f:06d}.json").read_text())
        assert lab["frame_id"] == f
    assert counts == [20, 20]
    # no temporary files left behind; per-shard summaries add up to the single run's
    for d in [one] + shards:
        assert not [p for p in d.rglob("*.tmp")]
    tot = [json.load(open(s / "logs" / "generation_summary.json"))["counters"]["successful_frames"] for s in shards]
    assert sum(tot) == json.load(open(one / "logs" / "generation_summary.json"))["counters"]["successful_frames"] == 40
    assert os.path.isdir(tmp_path / "two")
