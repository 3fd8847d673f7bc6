"""Multi-process (world_size 2, gloo, CPU) check of the multi-GPU plan in dist.py:
resample sharding + all-gather of each rank's label columns, row-band sharding of the triangle tiles,
SUM of histogram counts.  The per-rank compute is the CPU oracle restricted to the rank's
resamples / tiles, so what is tested is exactly the partition and the exchange."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from tests.conftest import ROOT, load_fixture

TILE = 256


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def tile_list(n):
    nb = (n + TILE - 1) // TILE
    return [(bi, bj) for bi in range(nb) for bj in range(bi, nb)]


def band_pair_counts(M, I, n, tiles):
    """numpy.histogram counts of C over the strict-upper pairs inside the given tiles."""
    from oracle import cc_oracle as O

    C = O.consensus_matrix(M.astype(np.uint16), I.astype(np.uint16))
    vals = []
    for bi, bj in tiles:
        i0, j0 = bi * TILE, bj * TILE
        blk = C[i0:min(n, i0 + TILE), j0:min(n, j0 + TILE)]
        ii, jj = np.meshgrid(np.arange(i0, i0 + blk.shape[0]), np.arange(j0, j0 + blk.shape[1]),
                             indexing="ij")
        vals.append(blk[ii < jj])
    v = np.concatenate(vals) if vals else np.zeros(0, np.float32)
    return np.histogram(v, bins=20, range=(0, 1))[0].astype(np.int64)


def _worker(rank, world, port, name, out):
    import sys

    sys.path.insert(0, ROOT)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from consensus_clustering_amd import dist as cdist
        from oracle import cc_oracle as O

        f = load_fixture(name)
        n = f["X"].shape[0]
        H = f["meta"]["H"]
        Ks = [int(k) for k in f["K_range"]]
        r, W = cdist.world()
        assert (r, W) == (rank, world)
        h0, h1 = cdist.shard(H, r, W)
        # per-rank label matrices: 0xFF outside this rank's resamples
        L = torch.full((len(Ks), n, H), 0xFF, dtype=torch.uint8)
        for k in range(len(Ks)):
            for h in range(h0, h1):
                L[k, torch.from_numpy(f["indices"][h].astype(np.int64)), h] = torch.from_numpy(
                    f["labels"][k, h].astype(np.uint8))
        cdist.merge_labels(L, H)
        full = np.full((len(Ks), n, H), 0xFF, np.uint8)
        for k in range(len(Ks)):
            for h in range(H):
                full[k, f["indices"][h], h] = f["labels"][k, h]
        np.testing.assert_array_equal(L.numpy(), full)
        # each rank: its band of tiles, from the merged labels
        tiles = tile_list(n)
        t0, t1 = cdist.shard(len(tiles), r, W)
        idx = f["indices"].astype(np.int64)
        I = O.cosample_matrix(idx, n)
        counts = torch.zeros((len(Ks), 20), dtype=torch.int64)
        for k, K in enumerate(Ks):
            lab = L[k].numpy().T.astype(np.int64)  # [H, n]
            labs = np.stack([lab[h, idx[h]] for h in range(H)])
            M = O.coassoc_matrix(idx, labs, K, n)
            counts[k] = torch.from_numpy(band_pair_counts(M, I, n, tiles[t0:t1]))
        cdist.sum_counts(counts)
        if rank == 0:
            np.save(out, counts.numpy())
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("name,world", [("blobs_n400_d8_k4", 2), ("c1_corr_raw", 2),
                                        ("c1_corr_raw", 3)])
def test_multi_rank_plan_is_exact(tmp_path, name, world):
    """World 2 and 3 (uneven resample shards: the gathered blocks are padded to ceil(H/W))."""
    out = str(tmp_path / "counts.npy")
    mp.spawn(_worker, args=(world, _free_port(), name, out), nprocs=world, join=True)
    counts = np.load(out)
    from consensus_clustering_amd import post
    from oracle import cc_oracle as O

    f = load_fixture(name)
    n = f["X"].shape[0]
    for j in range(len(f["K_range"])):
        C = O.consensus_matrix(f["mij"][j], f["iij"])
        np.testing.assert_array_equal(post.pair_counts_to_hist_counts(counts[j], n), O.bin_counts(C))


def test_shard_covers_range():
    from consensus_clustering_amd.dist import shard

    for total in (0, 1, 7, 1000, 19306):
        for W in (1, 2, 3, 8):
            parts = [shard(total, r, W) for r in range(W)]
            assert parts[0][0] == 0 and parts[-1][1] == total
            for (a, b), (c, d) in zip(parts, parts[1:]):
                assert b == c
            sizes = [b - a for a, b in parts]
            assert max(sizes) - min(sizes) <= 1
