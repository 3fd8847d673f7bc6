"""float64 k-means at one config shape and H under two workspace budgets (grid size effect).

    python tools/f64_budget.py CONFIG H BUDGET_GB [BUDGET_GB ...]
"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402

from bench import CONFIGS, SEED, make_blobs_f32  # noqa: E402
from consensus_clustering_amd import engine  # noqa: E402
from consensus_clustering_amd.kmeans import BatchedKMeans  # noqa: E402

cfg = CONFIGS[sys.argv[1]]
H = int(sys.argv[2])
dev = engine.require_gpu()
X = make_blobs_f32(cfg["n"], cfg["d"], cfg["k_true"], seed=SEED).astype(np.float64)
n, d = X.shape
m = int(cfg["frac"] * n)
idx_d = torch.from_numpy(engine.resample_indices(SEED, n, m, 0, H)).to(dev)
X64 = torch.from_numpy(X).to(dev)
for gb in sys.argv[3:]:
    L = engine.new_label_matrix(len(cfg["Ks"]), n, engine.pad_h(H), dev)
    bk = BatchedKMeans(cfg["Ks"], n_init=3, random_state=SEED, workspace_budget=int(float(gb) * (1 << 30)))
    ts = []
    for rep in range(2):
        torch.cuda.synchronize()
        t = time.perf_counter()
        bk.run_f64(X64, idx_d, n, H, m, 0, H, L)
        torch.cuda.synchronize()
        ts.append(time.perf_counter() - t)
    print(f"{sys.argv[1]} H={H} budget {gb} GB: {min(ts) * 1e3:.1f} ms", flush=True)
