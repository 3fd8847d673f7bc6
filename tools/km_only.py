"""Run only the batched k-means launch of a consensus fit (profiling driver).

    python tools/km_only.py [H] [config]
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402

from bench import CONFIGS, SEED, make_blobs_f32  # noqa: E402
from consensus_clustering_amd import engine  # noqa: E402
from consensus_clustering_amd.kmeans import BatchedKMeans, prepare_rows  # noqa: E402

H = int(sys.argv[1]) if len(sys.argv) > 1 else 64
cfg = CONFIGS[sys.argv[2] if len(sys.argv) > 2 else "c3"]
dev = engine.require_gpu()
X = make_blobs_f32(cfg["n"], cfg["d"], cfg["k_true"], seed=SEED)
n, d = X.shape
m = int(cfg["frac"] * n)
idx = engine.resample_indices(SEED, n, m, 0, H)
idx_d = torch.from_numpy(idx).to(dev)
Xd, xn, _, Xhl, e = prepare_rows(X, dev)
L = engine.new_label_matrix(len(cfg["Ks"]), n, engine.pad_h(H), dev)
bk = BatchedKMeans(cfg["Ks"], n_init=3, random_state=SEED)
bk.run(Xd, xn, d, idx_d, n, H, m, 0, H, L, np.float32, Xhl=Xhl, scale_exp=e)
torch.cuda.synchronize()
print("stats", bk.stats[:6].tolist())
