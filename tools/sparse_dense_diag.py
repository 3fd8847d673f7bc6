"""Sparse vs dense M-step (CCMI_KM_DENSE) on one C3-shaped case: label agreement between the
two, each one's sklearn parity (disagreements not asserted), and for every problem where an
engine disagrees with sklearn the three fits' inertias (sklearn float32 / float64 KMeans too).

    python tools/sparse_dense_diag.py [n] [seed] [H]
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
from sklearn.cluster import KMeans  # noqa: E402
from threadpoolctl import threadpool_limits  # noqa: E402

from tests.sk_parity import sklearn_parity  # noqa: E402
from tests.test_gpu_kmeans import blobs, run_gpu  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 4000
dseed = int(sys.argv[2]) if len(sys.argv) > 2 else 11
H = int(sys.argv[3]) if len(sys.argv) > 3 else 4
d, k_true, Ks, seed = 128, 8, list(range(2, 15)), 3
X = blobs(n, d, k_true, seed=dseed)
os.environ.pop("CCMI_KM_DENSE", None)
idx, sp, _, nit_s, _ = run_gpu(X, Ks, H, 0.8, seed)
os.environ["CCMI_KM_DENSE"] = "1"
_, de, _, nit_d, _ = run_gpu(X, Ks, H, 0.8, seed)
os.environ.pop("CCMI_KM_DENSE", None)


def inertia(rows, lab, K):
    r = rows.astype(np.float64)
    return sum(((r[lab == c] - r[lab == c].mean(0)) ** 2).sum() for c in range(K) if np.any(lab == c))


diff = [(K, h) for k, K in enumerate(Ks) for h in range(H) if not np.array_equal(sp[k, h], de[k, h])]
print(f"n={n} data seed {dseed}: sparse vs dense differ in {len(diff)}/{len(Ks) * H} label vectors: {diff}")
for name, L in (("sparse", sp), ("dense", de)):
    print(name, end=": ")
    sklearn_parity(X, L, idx, Ks, seed, resamples=H, threads=8, max_unexplained=10 ** 6)
with threadpool_limits(8):
    for k, K in enumerate(Ks):
        for h in range(H):
            rows = X[idx[h]]
            ref = KMeans(n_clusters=K, random_state=seed, n_init=3).fit_predict(rows)
            if np.array_equal(ref, sp[k, h]) and np.array_equal(ref, de[k, h]):
                continue
            r64 = KMeans(n_clusters=K, random_state=seed, n_init=3).fit_predict(rows.astype(np.float64))
            print(f"K={K} h={h}: agree sparse {np.mean(ref == sp[k, h]):.5f} dense {np.mean(ref == de[k, h]):.5f}; "
                  f"exact inertia sklearn32 {inertia(rows, ref, K):.4f} sklearn64 {inertia(rows, r64, K):.4f} "
                  f"sparse {inertia(rows, sp[k, h], K):.4f} dense {inertia(rows, de[k, h], K):.4f}; "
                  f"n_iter sparse {nit_s[k, h]} dense {nit_d[k, h]}", flush=True)
