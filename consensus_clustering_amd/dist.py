"""Multi-GPU plan and exchange for one consensus fit (one process per GPU).

The reference has a single host and aggregates with racy in-place adds on a shared
ndarray / np.memmap (CC.py:185-195, :290).  Here every (resample, K) problem is
independent and every count is an integer sum, so a fit shards exactly:

* resamples   rank r runs k-means for h in ``shard(H, r, W)`` (no communication);
* labels      the per-rank uint8 label matrices hold 0xFF outside their resamples, so
              an element-wise MIN all-reduce assembles the full [nK, n, Hpad] matrix
              (RCCL over xGMI on the GPU; gloo in the CPU tests);
* triangle    rank r owns tiles ``shard(num_tiles, r, W)`` of the upper-triangle
              tiling (contiguous, equal-cost tiles: row-band sharding) and computes
              I, M and the histogram of its band only;
* counts      20 int64 bin counts per K, SUM all-reduce;
* matrices    (only when requested) each rank's band of M / I, SUM all-reduce.

Bit-exact for every W: integer counts, order-free reductions.

The exchanges use the default process group.  With the ``gloo`` backend (CPU tests, and
the single-GPU multi-process tests that put several ranks on one device) device tensors
are reduced through a host copy; with ``nccl`` (RCCL) they are reduced in place.
"""
from __future__ import annotations

import torch
import torch.distributed as dist


def _live() -> bool:
    return dist.is_available() and dist.is_initialized()


def world() -> tuple:
    """(rank, world_size) of the default process group, (0, 1) when not initialised."""
    if _live():
        return dist.get_rank(), dist.get_world_size()
    return 0, 1


def shard(total: int, rank: int, world_size: int) -> tuple:
    """Contiguous balanced range [begin, end) of ``total`` units for ``rank``."""
    base, rem = divmod(int(total), int(world_size))
    begin = rank * base + min(rank, rem)
    return begin, begin + base + (1 if rank < rem else 0)


def _all_reduce(t: torch.Tensor, op) -> torch.Tensor:
    if not (_live() and dist.get_world_size() > 1):
        return t
    if t.is_cuda and dist.get_backend() == "gloo":
        h = t.cpu()
        dist.all_reduce(h, op=op)
        t.copy_(h)
    else:
        dist.all_reduce(t, op=op)
    return t


def merge_labels(labels: torch.Tensor) -> torch.Tensor:
    """Assemble per-rank label matrices (0xFF where not owned) in place."""
    return _all_reduce(labels, dist.ReduceOp.MIN)


def sum_counts(t: torch.Tensor) -> torch.Tensor:
    return _all_reduce(t, dist.ReduceOp.SUM)


def barrier():
    if _live() and dist.get_world_size() > 1:
        dist.barrier()
