"""Diagnostic: per-phase cycle split of the k-means Lloyd sweep (stamps build)."""
import os, sys
os.environ["CCMI_LIB"] = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "consensus_clustering_amd", "libccmi_stamps.so")
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np, torch
from bench import make_blobs_f32
from consensus_clustering_amd import ConsensusClustering
H = int(sys.argv[1]) if len(sys.argv) > 1 else 8
X = make_blobs_f32(50000, 128, 8)
cc = ConsensusClustering(K_range=list(range(2, 21)), n_iterations=H, random_state=0, plot_cdf=False, keep_matrices=False)
cc.fit(torch.from_numpy(X).cuda())
st = cc.kmeans_stats_.cpu().numpy()
print("timings", cc.timings_)
print("counters", st[:4])
names = ["work1", "wait1", "work2", "wait2"]
for w in range(8):
    v = st[4 + 4 * w: 8 + 4 * w]
    tot = max(v.sum(), 1)
    print(f"wave {w} ({'MFMA' if w < 4 else 'VALU'}):", {n: f"{x/1e6:.1f}M ({100*x/tot:.0f}%)" for n, x in zip(names, v)})
it = cc.kmeans_n_iter_.cpu().numpy()
print("n_iter per K (mean over h):", dict(zip(range(2, 21), np.round(it.mean(1), 1))))
