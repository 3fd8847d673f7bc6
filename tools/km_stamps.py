"""Diagnostic: per-phase cycle split of the k-means sweep (stamps build, libccmi_stamps.so).

    python tools/km_stamps.py [H] [config]
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ["CCMI_LIB"] = os.path.join(ROOT, "consensus_clustering_amd", os.environ.get("KM_STAMPS_LIB", "libccmi_stamps.so"))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402

from bench import CONFIGS, make_blobs_f32  # noqa: E402
from consensus_clustering_amd import ConsensusClustering  # noqa: E402

H = int(sys.argv[1]) if len(sys.argv) > 1 else 8
cfg = CONFIGS[sys.argv[2] if len(sys.argv) > 2 else "c3"]
X = make_blobs_f32(cfg["n"], cfg["d"], cfg["k_true"])
cc = ConsensusClustering(K_range=cfg["Ks"], n_iterations=H, random_state=0, plot_cdf=False,
                         keep_matrices=False)
cc.fit(torch.from_numpy(X).cuda())
st = cc.kmeans_stats_.cpu().numpy()
print("timings", cc.timings_)
print("counters lloyd/seed/mrows/reloc/sweeps/ctiles", st[:6])
# phases: issue, dist, estep, mstep, commit, barrier, prologue
names = ["issue", "est4+dist", "est0-3", "mstep", "wait", "barrier", "prologue"]
for w in range(8):
    v = st[8 + 8 * w: 15 + 8 * w]
    tot = max(v.sum(), 1)
    print(f"wave {w}:", {n: f"{x / 1e6:.1f}M ({100 * x / tot:.0f}%)" for n, x in zip(names, v)})
print("post-processing cycles (wg0):", st[73] / 1e6, "M")
it = cc.kmeans_n_iter_.cpu().numpy()
print("n_iter per K (mean/max over h):", {K: (round(float(it[k].mean()), 1), int(it[k].max()))
                                          for k, K in enumerate(cfg["Ks"])})
cyc = st[80:89].astype(float)
cnt = st[96:105].astype(float)
tot = max(cyc.sum(), 1)
print("sweeps by active waves (1..8): count / share of sweep cycles / mean Mcycles:",
      {w: (int(cnt[w]), f"{100 * cyc[w] / tot:.0f}%", round(cyc[w] / max(cnt[w], 1) / 1e6, 2)) for w in range(1, 9)})
pp = st[106:110] / 1e6
print("post-processing phases (wg0, Mcycles): seeding %.1f, label compare %.1f, running sums %.1f, centre update %.1f"
      % tuple(pp))
