"""Per-GPU frame partition for multi-GPU batches (SURVEY.md sec.8 e).

Frames are independent, so G GPUs split a batch into G contiguous frame
ranges and run the same kernel on their own range: no data-path collective.
Uniform frames split by count; mixed sizes split by payload bytes using a
prefix sum of lengths, so every rank gets about the same HBM traffic.
The only cross-rank traffic is the harness's: a barrier, the max of the
per-rank elapsed times and a sum of per-rank checksums / mismatch counts.
"""
from __future__ import annotations

from typing import List, Sequence, Tuple

import numpy as np


def uniform_range(n: int, rank: int, world: int) -> Tuple[int, int]:
    """Frames [lo, hi) of rank `rank` for n equal frames: g*n/G .. (g+1)*n/G."""
    if not 0 <= rank < world:
        raise ValueError("rank out of range")
    return (rank * n) // world, ((rank + 1) * n) // world


def sub_batches(job: int, rank: int, world: int, max_batch: int) -> Tuple[int, List[Tuple[int, int]]]:
    """Resident sub-batches of rank `rank`'s shard of a `job`-frame job.

    Every rank gets the same number of sub-batches (so the harness barriers
    pair up), each at most `max_batch` frames: returns (frames per full batch,
    [(lo, hi) global frame ranges]), covering the shard in order.  A rank with a
    shorter shard may have a short or empty last sub-batch.
    """
    if max_batch < 1:
        raise ValueError("max_batch must be >= 1")
    lo, hi = uniform_range(job, rank, world)
    max_shard = -(-job // world)
    nb = max(1, -(-max_shard // max_batch))
    n = -(-max_shard // nb)
    return n, [(min(lo + j * n, hi), min(lo + (j + 1) * n, hi)) for j in range(nb)]


def byte_balanced_ranges(lens: Sequence[int], world: int) -> List[Tuple[int, int]]:
    """Contiguous frame ranges with near-equal payload bytes per rank.

    Rank g's range starts at the first frame whose exclusive byte prefix is
    >= g * total / G.  Ranges are contiguous, disjoint and cover all frames.
    """
    lens = np.asarray(lens, dtype=np.int64)
    n = len(lens)
    excl = np.concatenate([[0], np.cumsum(lens)])  # excl[i] = bytes before frame i
    total = int(excl[-1])
    cuts = [0]
    for g in range(1, world):
        target = (g * total) // world
        cuts.append(int(np.searchsorted(excl[:n], target, side="left")))
    cuts.append(n)
    cuts = np.maximum.accumulate(np.asarray(cuts))
    return [(int(cuts[g]), int(cuts[g + 1])) for g in range(world)]


def aggregate_rate(bytes_per_rank: Sequence[int], elapsed_per_rank: Sequence[float]) -> float:
    """Whole-job bytes per second: all ranks' bytes over the slowest rank's time."""
    return float(sum(bytes_per_rank)) / max(elapsed_per_rank)
