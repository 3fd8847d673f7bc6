"""Host stage of the hybrid path alone (no GPU): GaussianMixture(n_init=2) fit_predict on H
resamples (CC.py:282) through api.host_fit_predict, serial against 'multithreading' and
'multiprocessing' with n_jobs workers; labels checked identical.

    python tools/host_fit_time.py [n] [d] [H] [n_jobs]
"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
from sklearn.mixture import GaussianMixture  # noqa: E402
from threadpoolctl import threadpool_limits  # noqa: E402

from bench import make_blobs_f32  # noqa: E402
from consensus_clustering_amd.api import host_fit_predict  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 10000
d = int(sys.argv[2]) if len(sys.argv) > 2 else 16
H = int(sys.argv[3]) if len(sys.argv) > 3 else 32
nj = int(sys.argv[4]) if len(sys.argv) > 4 else 8
X = make_blobs_f32(n, d, 5, seed=0).astype(np.float64)
idx = np.stack([np.random.RandomState(h).choice(n, int(0.8 * n), replace=False) for h in range(H)])
res = {}
for n_jobs, method in ((1, "multithreading"), (nj, "multiprocessing"), (nj, "multithreading"), (nj, "multiprocessing"), (nj, "multithreading")):
    for K in (4,):
        clf = GaussianMixture(n_components=K, n_init=2, random_state=0)
        with threadpool_limits(1):
            t0 = time.perf_counter()
            lab = host_fit_predict(clf, X, idx, n_jobs=n_jobs, parallelization_method=method)
            dt = time.perf_counter() - t0
        res[(n_jobs, method, len(res))] = lab
        print(f"n={n} d={d} H={H} GaussianMixture(K=4, n_init=2): n_jobs={n_jobs} {method}: {dt:.2f} s", flush=True)
base = res[(1, "multithreading", 0)]
print("labels identical across n_jobs / methods:", all(np.array_equal(base, v) for v in res.values()))
