"""Time the float64 k-means (cc_kmeans_f64) against the fast engine on a config's shape with a few
resamples (HIP events), to size precision='auto' (api.py).

    python tools/f64_time.py [config] [H]
"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402

from bench import CONFIGS, SEED, make_blobs_f32, make_expression_f32  # noqa: E402
from consensus_clustering_amd import engine  # noqa: E402
from consensus_clustering_amd.kmeans import BatchedKMeans, prepare_rows  # noqa: E402

cfg = CONFIGS[sys.argv[1] if len(sys.argv) > 1 else "c3"]
H = int(sys.argv[2]) if len(sys.argv) > 2 else 4
dev = engine.require_gpu()
if cfg.get("data") == "expression":
    X = make_expression_f32(cfg["n"], cfg["d"], groups=cfg["k_true"], seed=SEED)
else:
    X = make_blobs_f32(cfg["n"], cfg["d"], cfg["k_true"], seed=SEED)
n, d = X.shape
m = int(cfg["frac"] * n)
idx_d = torch.from_numpy(engine.resample_indices(SEED, n, m, 0, H)).to(dev)
X64 = torch.from_numpy(X.astype(np.float64)).to(dev)
res = {}
for name in ("fast", "f64"):
    L = engine.new_label_matrix(len(cfg["Ks"]), n, engine.pad_h(H), dev)
    bk = BatchedKMeans(cfg["Ks"], n_init=3, random_state=SEED)
    ts = []
    for rep in range(2):
        torch.cuda.synchronize()
        t = time.perf_counter()
        if name == "f64":
            bk.run_f64(X64, idx_d, n, H, m, 0, H, L)
        else:
            Xd, xn, _, Xhl, e = prepare_rows(X, dev)
            bk.run(Xd, xn, d, idx_d, n, H, m, 0, H, L, np.float64, Xhl=Xhl, scale_exp=e)
        torch.cuda.synchronize()
        ts.append(time.perf_counter() - t)
    res[name] = min(ts)
    print(f"{name}: {res[name] * 1e3:.1f} ms for H={H} ({res[name] / H * 1e3:.2f} ms per resample, "
          f"all {len(cfg['Ks'])} K x 3 inits)", flush=True)
print(f"f64 / fast = {res['f64'] / res['fast']:.1f}x; extrapolated full-H f64 k-means "
      f"{res['f64'] / H * cfg['H']:.1f} s vs fast {res['fast'] / H * cfg['H']:.2f} s")
