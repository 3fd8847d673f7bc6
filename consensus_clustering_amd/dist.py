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
"""
from __future__ import annotations

import os

import torch
import torch.distributed as dist


def _live() -> bool:
    return dist.is_available() and dist.is_initialized()


def world() -> tuple:
    """(rank, world_size) of the default process group, (0, 1) when not initialised.

    ``CCMI_SIM_RANK=r/W`` (no process group) runs rank r's shard of a W-rank fit alone, with
    the exchanges skipped: a one-GPU rehearsal of the per-rank critical path (timing only,
    the results are partial)."""
    if _live():
        return dist.get_rank(), dist.get_world_size()
    sim = os.environ.get("CCMI_SIM_RANK")
    if sim:
        r, w = (int(v) for v in sim.split("/"))
        return r, w
    return 0, 1


def shard(total: int, rank: int, world_size: int) -> tuple:
    """Contiguous balanced range [begin, end) of ``total`` units for ``rank``."""
    base, rem = divmod(int(total), int(world_size))
    begin = rank * base + min(rank, rem)
    return begin, begin + base + (1 if rank < rem else 0)


def merge_labels(labels: torch.Tensor) -> torch.Tensor:
    """Assemble per-rank label matrices (0xFF where not owned) in place."""
    if _live() and dist.get_world_size() > 1:
        dist.all_reduce(labels, op=dist.ReduceOp.MIN)
    return labels


def sum_counts(t: torch.Tensor) -> torch.Tensor:
    if _live() and dist.get_world_size() > 1:
        dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return t


def barrier():
    if _live() and dist.get_world_size() > 1:
        dist.barrier()
