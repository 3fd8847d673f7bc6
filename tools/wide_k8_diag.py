"""The wide engine's (cc_kmeans_wide) one unexplained problem in tests/test_gpu_kmeans.py
(n=1200, d=300, k_true=5, K=8, resample 2, seed 7): engine vs sklearn for n_init = 1, 2, 3 (so
the best-of-init reveals each init's result), with permutation-invariant agreement.

    python tools/wide_k8_diag.py
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402
from sklearn.cluster import KMeans  # noqa: E402
from sklearn.metrics import adjusted_rand_score  # noqa: E402
from threadpoolctl import threadpool_limits  # noqa: E402

from consensus_clustering_amd import engine  # noqa: E402
from consensus_clustering_amd.kmeans import BatchedKMeans, prepare_rows  # noqa: E402
from tests.test_gpu_kmeans import blobs  # noqa: E402

n, d, k, K, h, H, seed = 1200, 300, 5, 8, 2, 4, 7
X = blobs(n, d, k, seed=n)
m = int(0.8 * n)
idx = engine.resample_indices(seed, n, m, 0, H)
dev = engine.require_gpu()
Xd, xn, _, Xhl, e = prepare_rows(X, dev)
rows = X[idx[h]]
for n_init in (1, 2, 3):
    L = engine.new_label_matrix(1, n, engine.pad_h(H), dev)
    inert = torch.zeros((1, H), dtype=torch.float32, device=dev)
    nit = torch.zeros((1, H), dtype=torch.int32, device=dev)
    BatchedKMeans([K], n_init=n_init, random_state=seed).run(Xd, xn, d, torch.from_numpy(idx).to(dev), n, H, m, 0, H,
                                                            L, np.float32, inertia=inert, n_iter=nit, Xhl=Xhl, scale_exp=e)
    torch.cuda.synchronize()
    got = L[0].cpu().numpy()[idx[h], h].astype(np.int64)
    with threadpool_limits(4):
        km = KMeans(n_clusters=K, random_state=seed, n_init=n_init).fit(rows)
    print(f"n_init={n_init}: engine inertia {float(inert[0, h]):.2f} n_iter {int(nit[0, h])} | sklearn inertia "
          f"{km.inertia_:.2f} n_iter {km.n_iter_} | identical {np.array_equal(got, km.labels_)} "
          f"ARI {adjusted_rand_score(got, km.labels_):.4f}", flush=True)
