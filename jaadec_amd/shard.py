"""Stream sharding across GPUs (one process per GPU, no collectives on the data path).

AAC streams are independent: every run of consecutive frames of one stream, and
its carried DSP state, lives on exactly one rank.  Rank r owns a contiguous block of the runs,
balanced by frame count.  The only collectives anywhere are the benchmark's barrier and its
max-over-ranks timing reduction; PCM goes device -> host per rank.
"""
from __future__ import annotations

import numpy as np

from .native import Batch


def shard_runs(frame_begin: np.ndarray, world: int, rank: int) -> range:
    """Contiguous block of run indices for `rank`, balanced by frames (runs never split)."""
    n_runs = len(frame_begin) - 1
    if world <= 1:
        return range(n_runs)
    total = int(frame_begin[-1])
    # run r goes to the rank whose frame interval contains the run's first frame
    owner = np.minimum((frame_begin[:-1].astype(np.int64) * world) // max(total, 1), world - 1)
    idx = np.flatnonzero(owner == rank)
    return range(int(idx[0]), int(idx[-1]) + 1) if idx.size else range(0)


def rank_batch(batch: Batch, world: int, rank: int) -> Batch:
    """The sub-batch rank `rank` decodes (its stream slots keep their global numbers)."""
    return batch.select_runs(shard_runs(batch.frame_begin, world, rank))


def reduce_max_time(seconds: float, group=None) -> float:
    """Max over ranks of a wall time (the benchmark's only collective besides its barrier and frame
    count): a host scalar, reduced over the bench's gloo group."""
    import torch
    import torch.distributed as dist

    if not dist.is_available() or not dist.is_initialized() or dist.get_world_size() == 1:
        return seconds
    t = torch.tensor([seconds], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX, group=group)
    return float(t.item())
