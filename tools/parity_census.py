"""Parity census of the f32-class k-means against sklearn's float32 KMeans on C3-shaped blobs
(d = 128, k_true = 8, K = 2..14, H resamples, several data seeds): per seed the counts of
identical / rounding-explained / unexplained label vectors (tests/sk_parity.py rules), and for
each unexplained one its label agreement and exact inertias.

    python tools/parity_census.py [n] [H] [seed ...]
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402

from tests.sk_parity import sklearn_parity  # noqa: E402
from tests.test_gpu_kmeans import blobs, run_gpu  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 4000
H = int(sys.argv[2]) if len(sys.argv) > 2 else 4
seeds = [int(s) for s in sys.argv[3:]] or [1, 2, 3, 4]
d, k_true, Ks, seed = 128, 8, list(range(2, 15)), 3
tot = np.zeros(3, dtype=int)
for ds in seeds:
    X = blobs(n, d, k_true, seed=ds)
    idx, labs, _, _, _ = run_gpu(X, Ks, H, 0.8, seed)
    print(f"data seed {ds}:", end=" ", flush=True)
    same, explained, total = sklearn_parity(X, labs, idx, Ks, seed, resamples=H, threads=16,
                                            max_unexplained=10 ** 6)
    tot += (same, explained, total - same - explained)
    # every disagreement of this data set: agreement, ARI and exact inertias (the engine's labels
    # against sklearn's float32 fit of the same rows)
    from sklearn.cluster import KMeans
    from sklearn.metrics import adjusted_rand_score
    from threadpoolctl import threadpool_limits

    def inertia(rows, lab, K):
        r = rows.astype(np.float64)
        return sum(((r[lab == c] - r[lab == c].mean(0)) ** 2).sum() for c in range(K) if np.any(lab == c))

    with threadpool_limits(16):
        for k, K in enumerate(Ks):
            for h in range(H):
                rows = X[idx[h]]
                ref = KMeans(n_clusters=K, random_state=seed, n_init=3).fit_predict(rows)
                if np.array_equal(ref, labs[k, h]):
                    continue
                print(f"   K={K} h={h}: agree {np.mean(ref == labs[k, h]):.4f} ARI {adjusted_rand_score(ref, labs[k, h]):.5f} "
                      f"inertia engine {inertia(rows, labs[k, h], K):.3f} sklearn32 {inertia(rows, ref, K):.3f}", flush=True)
print(f"census n={n} H={H} seeds {seeds}: identical {tot[0]}, explained {tot[1]}, unexplained {tot[2]} "
      f"of {tot.sum()} label vectors ({len(Ks)} K x {H} resamples x {len(seeds)} data sets)")
