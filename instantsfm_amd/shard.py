"""Track sharding for multi-GPU BA: points split into contiguous ranges balanced by observation count.

Because observations are track-major, each shard's observations are one contiguous slice; cameras are replicated and
the reduced camera system is summed across ranks (one all-reduce per linearization / trial).
"""
import numpy as np


def shard_ranges(pt_idx, n_points, world_size):
    """[(p_begin, p_end)] per rank, contiguous, covering [0, n_points), balanced by observations."""
    counts = np.bincount(np.asarray(pt_idx), minlength=n_points)
    cum = np.concatenate([[0], np.cumsum(counts)])
    total = cum[-1]
    bounds = [0]
    for r in range(1, world_size):
        bounds.append(int(np.searchsorted(cum, total * r / world_size, side="left")))
    bounds.append(int(n_points))
    bounds = np.maximum.accumulate(np.minimum(np.asarray(bounds), n_points))
    return [(int(bounds[r]), int(bounds[r + 1])) for r in range(world_size)]
