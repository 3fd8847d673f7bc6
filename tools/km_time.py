"""Time the batched k-means launch alone (HIP events), for build variants (CCMI_LIB=...).

    python tools/km_time.py [H] [config] [reps]
"""
import hashlib
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402

from bench import CONFIGS, SEED, make_blobs_f32  # noqa: E402
from consensus_clustering_amd import engine  # noqa: E402
from consensus_clustering_amd.kmeans import BatchedKMeans, prepare_rows  # noqa: E402

H = int(sys.argv[1]) if len(sys.argv) > 1 else 1000
cfg = CONFIGS[sys.argv[2] if len(sys.argv) > 2 else "c3"]
reps = int(sys.argv[3]) if len(sys.argv) > 3 else 2
dev = engine.require_gpu()
X = make_blobs_f32(cfg["n"], cfg["d"], cfg["k_true"], seed=SEED)
n, d = X.shape
m = int(cfg["frac"] * n)
idx_d = torch.from_numpy(engine.resample_indices(SEED, n, m, 0, H)).to(dev)
Xd, xn, _, Xhl, e = prepare_rows(X, dev)
L = engine.new_label_matrix(len(cfg["Ks"]), n, engine.pad_h(H), dev)
inert = torch.zeros((len(cfg["Ks"]), H), dtype=torch.float32, device=dev)
nit = torch.zeros((len(cfg["Ks"]), H), dtype=torch.int32, device=dev)
bk = BatchedKMeans(cfg["Ks"], n_init=3, random_state=SEED, max_iter=int(os.environ.get("KM_MAXITER", 300)),
                   workspace_budget=(int(os.environ["KM_BUDGET_GB"]) << 30) if "KM_BUDGET_GB" in os.environ else None)
ts = []
for r in range(reps + 1):
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    bk.run(Xd, xn, d, idx_d, n, H, m, 0, H, L, np.float32, Xhl=Xhl, scale_exp=e, inertia=inert, n_iter=nit)
    b.record()
    torch.cuda.synchronize()
    if r:
        ts.append(a.elapsed_time(b))
print(os.path.basename(os.environ.get("CCMI_LIB", "libccmi.so")), "kmeans ms", [round(t, 1) for t in ts],
      "sweeps", int(bk.stats[4]), "sparse item-sweeps", int(bk.stats[6]), "changes", int(bk.stats[7]),
      "labels sha", hashlib.sha256(L.cpu().numpy().tobytes()).hexdigest()[:16],
      "inertia sha", hashlib.sha256(inert.cpu().numpy().tobytes()).hexdigest()[:16],
      "n_iter sha", hashlib.sha256(nit.cpu().numpy().tobytes()).hexdigest()[:16],
      "ste sweeps", int(bk.stats[76]), flush=True)
st = bk.stats.cpu().numpy()
cyc, cnt = st[80:89].astype(float), st[96:105].astype(float)
tot = max(cyc.sum(), 1)
print("  sweeps by active waves: count / share of sweep cycles / mean Mcycles:",
      {w: (int(cnt[w]), f"{100 * cyc[w] / tot:.0f}%", round(cyc[w] / max(cnt[w], 1) / 1e6, 2)) for w in range(1, 9)
       if cnt[w]}, flush=True)
