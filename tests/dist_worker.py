"""Helper for tests/test_gpu_dist.py (not collected by pytest): runs ConsensusClustering.fit
as a W-rank torch.distributed job (gloo backend, every rank on cuda:0) and saves rank 0's
results.  It is started as a child process, so the ranks are spawned by a parent that has not
touched the GPU.

    python tests/dist_worker.py <fixture> <world> <keep 0|1> <out.npz> [backend] [H] [clusterer]

H overrides the fixture's n_iterations (fewer resamples than ranks leaves a rank without any);
clusterer 'gmm' runs the hybrid path (a host GaussianMixture per resample, tests/test_gpu_dist.py).

backend 'nccl' (RCCL) needs one device per rank, so on a one-GPU box it runs with world 1 and
CCMI_DIST_EXCHANGE_W1=1 (the exchange collectives then run on RCCL anyway).
"""
import os
import socket
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def make_clusterer(kind):
    if kind == "gmm":
        from sklearn.mixture import GaussianMixture

        return GaussianMixture(n_components=2)
    return None


def _rank(rank, world, port, name, keep, out, backend="gloo", H=0, clusterer=""):
    import torch
    import torch.distributed as dist

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    if backend == "nccl":
        dist.init_process_group("nccl", rank=rank, world_size=world, device_id=torch.device("cuda", 0))
    else:
        dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from consensus_clustering_amd import ConsensusClustering
        from tests.conftest import load_fixture

        f = load_fixture(name)
        meta = f["meta"]
        cc = ConsensusClustering(clusterer=make_clusterer(clusterer),
                                 clusterer_options={} if clusterer else {'n_init': 3},
                                 K_range=[int(k) for k in f["K_range"]], n_iterations=H or meta["H"],
                                 subsampling=meta["subsampling"], random_state=meta["random_state"],
                                 plot_cdf=False, keep_matrices=bool(keep))
        cc.fit(f["X"])
        Ks = list(cc.cdf_at_K_data)
        res = dict(
            pair_counts=np.stack([cc.pair_counts_[K] for K in Ks]),
            labels=cc.labels_.cpu().numpy(),
            pac=np.array([cc.cdf_at_K_data[K]["pac_area"] for K in Ks]),
            hist=np.stack([cc.cdf_at_K_data[K]["hist"] for K in Ks]),
        )
        if keep:
            res["mij"] = np.stack([cc.cdf_at_K_data[K]["mij"] for K in Ks])
            res["iij"] = cc.cdf_at_K_data[Ks[0]]["iij"]
        if rank == 0:
            np.savez(out, **res)
    finally:
        dist.destroy_process_group()


def main():
    import torch.multiprocessing as mp

    name, world, keep, out = sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), sys.argv[4]
    backend = sys.argv[5] if len(sys.argv) > 5 else "gloo"
    H = int(sys.argv[6]) if len(sys.argv) > 6 else 0
    clusterer = sys.argv[7] if len(sys.argv) > 7 else ""
    mp.spawn(_rank, args=(world, _free_port(), name, keep, out, backend, H, clusterer), nprocs=world, join=True)


if __name__ == "__main__":
    main()
