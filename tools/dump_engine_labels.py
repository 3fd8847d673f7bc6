"""Engine labels of the documented parity gaps, for host-side diagnosis against sklearn's
trajectory: the sparse_n4000_d128 data of tests/test_gpu_kmeans.py (K = 2..14,
H = 4, seed 3) with the sparse and the dense M-step, and the C4 shape's K = 8 resample 0 on the
wide engine.  Writes gpurun_out/diag/engine_labels.npz.

    python tools/dump_engine_labels.py
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402

from bench import SEED, make_expression_f32  # noqa: E402
from consensus_clustering_amd import engine  # noqa: E402
from consensus_clustering_amd.kmeans import BatchedKMeans, prepare_rows  # noqa: E402


def blobs(n, d, k, seed):
    from sklearn.datasets import make_blobs

    X, _ = make_blobs(n_samples=n, n_features=d, centers=k, cluster_std=1.0, center_box=(-10, 10),
                      shuffle=True, random_state=seed)
    return X.astype(np.float32)


def run(X, Ks, H, seed):
    dev = engine.require_gpu()
    n, d = X.shape
    m = int(0.8 * n)
    idx = engine.resample_indices(seed, n, m, 0, H)
    Xd, xn, _, Xhl, e = prepare_rows(X, dev)
    L = engine.new_label_matrix(len(Ks), n, engine.pad_h(H), dev)
    inert = torch.zeros((len(Ks), H), dtype=torch.float32, device=dev)
    nit = torch.zeros((len(Ks), H), dtype=torch.int32, device=dev)
    BatchedKMeans(Ks, n_init=3, random_state=seed).run(Xd, xn, d, torch.from_numpy(idx).to(dev), n, H, m, 0, H, L,
                                                       np.float32, inertia=inert, n_iter=nit, Xhl=Xhl, scale_exp=e)
    torch.cuda.synchronize()
    Lh = L.cpu().numpy()
    labs = np.stack([np.stack([Lh[k][idx[h], h] for h in range(H)]) for k in range(len(Ks))])
    return labs.astype(np.int8), inert.cpu().numpy(), nit.cpu().numpy(), e


out = {}
X = blobs(4000, 128, 8, 11)
Ks = list(range(2, 15))
os.environ.pop("CCMI_KM_DENSE", None)
out["sparse_labels"], out["sparse_inertia"], out["sparse_niter"], out["scale_exp"] = run(X, Ks, 4, 3)
os.environ["CCMI_KM_DENSE"] = "1"
out["dense_labels"], out["dense_inertia"], out["dense_niter"], _ = run(X, Ks, 4, 3)
os.environ.pop("CCMI_KM_DENSE", None)
Xc4 = make_expression_f32(5000, 20000, groups=5, seed=SEED)
out["c4_k8_labels"], out["c4_k8_inertia"], out["c4_k8_niter"], out["c4_scale_exp"] = run(Xc4, [8], 1, SEED)
os.makedirs(os.path.join(ROOT, "gpurun_out", "diag"), exist_ok=True)
np.savez_compressed(os.path.join(ROOT, "gpurun_out", "diag", "engine_labels.npz"), **out)
print("saved", {k: v.shape for k, v in out.items() if hasattr(v, "shape")})
