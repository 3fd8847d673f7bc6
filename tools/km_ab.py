"""Diagnostic: time the batched k-means of a C3-shaped fit with a given libccmi build.
usage: CCMI_LIB=... python tools/km_ab.py H"""
import os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np, torch
from bench import make_blobs_f32
from consensus_clustering_amd import ConsensusClustering
H = int(sys.argv[1]) if len(sys.argv) > 1 else 8
X = torch.from_numpy(make_blobs_f32(50000, 128, 8)).cuda()
cc = ConsensusClustering(K_range=list(range(2, 21)), n_iterations=H, random_state=0, plot_cdf=False, keep_matrices=False)
cc.fit(X)
torch.cuda.synchronize()
t = time.perf_counter(); cc.fit(X); torch.cuda.synchronize(); dt = time.perf_counter() - t
it = cc.kmeans_n_iter_.cpu().numpy()
print(os.environ.get("CCMI_LIB", "default"), f"fit {dt:.3f}s", {k: round(v, 3) for k, v in cc.timings_.items()})
print("counters", cc.kmeans_stats_.cpu().numpy()[:4])
print("n_iter mean per K:", dict(zip(range(2, 21), np.round(it.mean(1), 1))), "max", it.max())
