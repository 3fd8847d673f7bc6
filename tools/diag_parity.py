"""Diagnose one fast-path problem that disagrees with sklearn float32: the engine's labels and
inertia against each of sklearn's n_init runs (same k-means++ stream, replicated with sklearn's
own _kmeans_plusplus / _kmeans_single_lloyd).

    python tools/diag_parity.py n d k_true K h H seed [bench]
(`bench`: the rows of bench.make_blobs_f32(n, d, k_true, seed), the data of the scale tests.)
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402
from sklearn.cluster._kmeans import _kmeans_plusplus, _kmeans_single_lloyd  # noqa: E402
from sklearn.datasets import make_blobs  # noqa: E402
from sklearn.utils.extmath import row_norms  # noqa: E402
from threadpoolctl import threadpool_limits  # noqa: E402

from consensus_clustering_amd import engine  # noqa: E402
from consensus_clustering_amd.kmeans import BatchedKMeans, prepare_rows  # noqa: E402

n, d, k, K, h, H, seed = (int(v) for v in sys.argv[1:8])
if len(sys.argv) > 8 and sys.argv[8] == "bench":
    from bench import make_blobs_f32

    X = make_blobs_f32(n, d, k, seed=seed)
else:
    X, _ = make_blobs(n_samples=n, n_features=d, centers=k, cluster_std=1.0, center_box=(-10, 10), shuffle=True,
                      random_state=n)
    X = X.astype(np.float32)
m = int(0.8 * n)
idx = engine.resample_indices(seed, n, m, 0, H)
dev = engine.require_gpu()
Xd, xn, _, Xhl, e = prepare_rows(X, dev)
L = engine.new_label_matrix(1, n, engine.pad_h(H), dev)
inert = torch.zeros((1, H), dtype=torch.float32, device=dev)
nit = torch.zeros((1, H), dtype=torch.int32, device=dev)
BatchedKMeans([K], n_init=3, random_state=seed).run(Xd, xn, d, torch.from_numpy(idx).to(dev), n, H, m, 0, H, L,
                                                   np.float32, inertia=inert, n_iter=nit, Xhl=Xhl, scale_exp=e)
torch.cuda.synchronize()
got = L[0].cpu().numpy()[idx[h], h].astype(np.int64)
print("engine: inertia", float(inert[0, h]), "n_iter", int(nit[0, h]))
rows = X[idx[h]]
with threadpool_limits(4):
    Xc = rows - rows.mean(axis=0)
    rs = np.random.RandomState(seed)
    xsq = row_norms(Xc, squared=True)
    sw = np.ones(len(rows), dtype=np.float32)
    tol = np.mean(np.var(Xc, axis=0)) * 1e-4
    for i in range(3):
        c0, ci = _kmeans_plusplus(Xc, K, x_squared_norms=xsq, random_state=rs, sample_weight=sw)
        lab, ine, cen, it = _kmeans_single_lloyd(Xc, sw, c0, max_iter=300, tol=tol, n_threads=4)
        print(f"sklearn init {i}: inertia {ine:.6f} n_iter {it} seeds {sorted(ci.tolist())[:10]} "
              f"label agreement with engine {np.mean(lab == got):.4f}")

from sklearn.cluster import KMeans  # noqa: E402

for th in (1, 4, 16):
    with threadpool_limits(th):
        ref = KMeans(n_clusters=K, random_state=seed, n_init=3).fit(rows)
    print(f"sklearn KMeans f32 threads={th}: inertia {ref.inertia_:.6f} agreement with engine "
          f"{np.mean(ref.labels_ == got):.5f}")
sys.path.insert(0, os.path.join(ROOT, "tests"))
from sk_parity import _fixed_point_no_worse  # noqa: E402

print("engine partition a float64 Lloyd fixed point no worse than sklearn:",
      _fixed_point_no_worse(rows, got, ref.labels_, K), "| with 1e-4 slack:",
      _fixed_point_no_worse(rows, got, ref.labels_, K, rel=1e-4))
