"""Multi-GPU plan and exchange for one consensus fit (one process per GPU).

The reference has a single host and aggregates with racy in-place adds on a shared
ndarray / np.memmap (CC.py:185-195, :290).  Here every (resample, K) problem is
independent and every count is an integer sum, so a fit shards exactly:

* resamples   rank r runs k-means for h in ``shard(H, r, W)`` (no communication);
* labels      each rank packs its own resample columns [h0, h1) of the sample-major
              [nK, n, Hpad] label matrix into a contiguous [nK, n, hw] block
              (hw = ceil(H / W)), the blocks are ALL-GATHERED into one flat buffer
              (``all_gather_into_tensor``: RCCL over xGMI on the GPU, gloo in the CPU tests;
              the same call either way) and every block is placed back at its columns.  Per GPU
              that moves (W-1)/W of nK n H bytes; a MIN all-reduce of the whole matrix (the
              round-2 exchange) moved 2 (W-1)/W of nK n Hpad;
* triangle    rank r owns tiles ``shard(num_tiles, r, W)`` of the upper-triangle
              tiling (contiguous, equal-cost tiles: row-band sharding) and computes
              I, M and the histogram of its band only;
* counts      20 int64 bin counts per K, SUM all-reduce;
* matrices    (only when requested) each rank's band of M / I, SUM all-reduce.

Bit-exact for every W: integer counts, order-free reductions.

The exchanges use the default process group and the same collective calls on every backend.
The only backend-dependent step is ``_host_staged``: with ``gloo`` (the CPU tests, and the
single-GPU multi-process tests that put several ranks on one device) a device tensor is
exchanged through a host copy; with ``nccl`` (RCCL) in place.
"""
from __future__ import annotations

import os

import torch
import torch.distributed as dist

# Diagnostics: run the exchange collectives even in a one-rank group (CCMI_DIST_EXCHANGE_W1=1), so
# that a one-GPU box executes the RCCL calls of the N-GPU path (two ranks cannot share a device
# under RCCL); the results are those of the skipped exchange.
EXCHANGE_AT_W1 = os.environ.get("CCMI_DIST_EXCHANGE_W1") == "1"


def _live() -> bool:
    return dist.is_available() and dist.is_initialized()


def _exchange() -> bool:
    return _live() and (dist.get_world_size() > 1 or EXCHANGE_AT_W1)


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


def _host_staged(t: torch.Tensor) -> bool:
    """gloo reduces host tensors only: a device tensor goes through a host copy.  This is the one
    place the backend matters; the collectives themselves are the same calls on RCCL and gloo."""
    return t.is_cuda and dist.get_backend() == "gloo"


def _all_reduce(t: torch.Tensor, op) -> torch.Tensor:
    if not _exchange():
        return t
    buf = t.cpu() if _host_staged(t) else t
    dist.all_reduce(buf, op=op)
    if buf is not t:
        t.copy_(buf)
    return t


def all_gather_flat(t: torch.Tensor) -> torch.Tensor:
    """Every rank's contiguous ``t`` (same shape on all ranks) gathered in rank order into one
    [W, *t.shape] tensor on t's device: ``all_gather_into_tensor`` into a flat W * numel buffer
    (RCCL over xGMI on the GPU; gloo, with a host copy, in the CPU tests)."""
    W = dist.get_world_size()
    src = t.cpu() if _host_staged(t) else t
    out = torch.empty(W * src.numel(), dtype=src.dtype, device=src.device)
    dist.all_gather_into_tensor(out, src.reshape(-1))
    out = out.view((W,) + tuple(t.shape))
    return out.to(t.device) if src is not t else out


def _copy_columns(src, col_src, dst, col_dst, width):
    if src.is_cuda:
        from . import engine

        engine.copy_label_columns(src, col_src, dst, col_dst, width)
    else:  # CPU tensors occur only in the gloo CPU tests of this exchange
        dst[..., col_dst:col_dst + width].copy_(src[..., col_src:col_src + width])


def merge_labels(labels: torch.Tensor, H: int) -> torch.Tensor:
    """Assemble the full label matrix in place from every rank's own resample columns.

    labels: uint8 [nK, n, Hpad] (contiguous), this rank's columns ``shard(H, rank, W)`` filled
    (0xFF = not sampled).  After the call every rank holds every rank's columns.  Only the
    resample columns travel: a packed [nK, n, hw] block per rank, all-gathered."""
    if not _exchange():
        return labels
    rank, W = world()
    assert labels.is_contiguous() and labels.dtype == torch.uint8
    hw = -(-int(H) // W)
    lead = tuple(labels.shape[:-1])
    h0, h1 = shard(H, rank, W)
    stage = torch.full(lead + (hw,), 0xFF, dtype=torch.uint8, device=labels.device)
    _copy_columns(labels, h0, stage, 0, h1 - h0)
    blocks = all_gather_flat(stage)  # [W, nK, n, hw], rank r's block at [r]
    for r in range(W):
        if r == rank:
            continue
        a, b = shard(H, r, W)
        _copy_columns(blocks[r], 0, labels, a, b - a)
    return labels


def sum_counts(t: torch.Tensor) -> torch.Tensor:
    return _all_reduce(t, dist.ReduceOp.SUM)


def barrier():
    if _live() and dist.get_world_size() > 1:
        dist.barrier()
