"""Seed-space sharding across GPUs: no collectives.

A unit of work is one randomisation epoch (10 frames, the reference
re-randomises every 10 frames, generate_construction_data.py:1542).  Rank r
of n owns epochs e with ``e % n == r``; every frame is a pure function of
``(seed, frame)`` so any partition reproduces the single-GPU output exactly.
Host-side counters (the DataQualityLogger summary) merge by summation.
"""
from __future__ import annotations

from typing import Dict, Iterable, List

EPOCH_FRAMES = 10


def shard_frames(rank: int, world: int, n_frames: int, epoch_frames: int = EPOCH_FRAMES) -> List[int]:
    """The first ``n_frames`` frame ids owned by ``rank`` (epoch-interleaved)."""
    if not 0 <= rank < world:
        raise ValueError("rank out of range")
    out: List[int] = []
    e = rank
    while len(out) < n_frames:
        out.extend(range(e * epoch_frames, (e + 1) * epoch_frames))
        e += world
    return out[:n_frames]


def shard_of_range(rank: int, world: int, total_frames: int, epoch_frames: int = EPOCH_FRAMES) -> List[int]:
    """Frames of [0, total_frames) owned by ``rank``; the union over ranks is the range."""
    return [f for f in range(total_frames) if (f // epoch_frames) % world == rank]


def merge_counters(parts: Iterable[Dict[str, int]]) -> Dict[str, int]:
    out: Dict[str, int] = {}
    for p in parts:
        for k, v in p.items():
            out[k] = out.get(k, 0) + v
    return out
