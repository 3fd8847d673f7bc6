"""Hybrid path timing (a foreign clusterer, CC.py:282 on the host, co-association on the GPU):
GaussianMixture(n_init=2) (NB:238-244) on blobs, n_jobs = 1 against joblib threads / processes
(CC.py:185-195), labels checked identical.

    python tools/gmm_time.py [n] [d] [H]
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
from consensus_clustering_amd import ConsensusClustering  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 10000
d = int(sys.argv[2]) if len(sys.argv) > 2 else 16
H = int(sys.argv[3]) if len(sys.argv) > 3 else 32
X = make_blobs_f32(n, d, 5, seed=0).astype(np.float64)
res = {}
for n_jobs, method in ((1, "multithreading"), (16, "multithreading"), (16, "multiprocessing"), (16, "multiprocessing")):
    cc = ConsensusClustering(clusterer=GaussianMixture(n_init=2), K_range=range(2, 7), n_iterations=H,
                             random_state=0, plot_cdf=False, n_jobs=n_jobs, parallelization_method=method,
                             keep_matrices=False)
    with threadpool_limits(1):
        t0 = time.perf_counter()
        cc.fit(X)
        dt = time.perf_counter() - t0
    res[(n_jobs, method, len(res))] = (dt, cc.labels_.cpu().numpy())
    print(f"n={n} d={d} H={H} K=2..6 GaussianMixture(n_init=2): n_jobs={n_jobs} {method}: fit {dt:.2f} s "
          f"(host fits {cc.timings_['cluster']:.2f} s)", flush=True)
base = res[(1, "multithreading", 0)][1]
print("labels identical across n_jobs / methods:",
      all(np.array_equal(base, v[1]) for v in res.values()))
