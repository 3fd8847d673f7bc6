"""A/B of the float64 k-means (cc_kmeans_f64) between two builds of the library: run it on a
config's shape for H resamples, save labels / inertia / n_iter and the HIP-event time.

    CCMI_LIB=... python tools/f64_ab.py CONFIG H OUT.npz      (one build)
    python tools/f64_ab.py --compare A.npz B.npz              (bit-identical? speed-up)
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402

if sys.argv[1] == "--compare":
    a, b = np.load(sys.argv[2]), np.load(sys.argv[3])
    same = all(np.array_equal(a[k], b[k]) for k in ("labels", "inertia", "n_iter"))
    print(f"identical labels/inertia/n_iter: {same}; {float(a['ms']):.1f} ms vs {float(b['ms']):.1f} ms "
          f"({float(b['ms']) / float(a['ms']):.2f}x)")
    sys.exit(0 if same else 1)

import torch  # noqa: E402

from bench import CONFIGS, SEED, make_blobs_f32  # noqa: E402
from consensus_clustering_amd import engine  # noqa: E402
from consensus_clustering_amd.kmeans import BatchedKMeans  # noqa: E402

cfg = CONFIGS[sys.argv[1]]
H = int(sys.argv[2])
dev = engine.require_gpu()
X = make_blobs_f32(cfg["n"], cfg["d"], cfg["k_true"], seed=SEED).astype(np.float64)
X += np.random.default_rng(0).normal(scale=0.05, size=X.shape)  # float64 values off the f32 grid
n, d = X.shape
m = int(cfg["frac"] * n)
Ks = cfg["Ks"]
idx_d = torch.from_numpy(engine.resample_indices(SEED, n, m, 0, H)).to(dev)
X64 = torch.from_numpy(X).to(dev)
L = engine.new_label_matrix(len(Ks), n, engine.pad_h(H), dev)
inert = torch.zeros((len(Ks), H), dtype=torch.float64, device=dev)
nit = torch.zeros((len(Ks), H), dtype=torch.int32, device=dev)
bk = BatchedKMeans(Ks, n_init=3, random_state=SEED)
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
torch.cuda.synchronize()
e0.record()
bk.run_f64(X64, idx_d, n, H, m, 0, H, L, inertia=inert, n_iter=nit)
e1.record()
torch.cuda.synchronize()
ms = e0.elapsed_time(e1)
print(f"{sys.argv[1]} H={H}: cc_kmeans_f64 {ms:.1f} ms", flush=True)
np.savez(sys.argv[3], labels=L.cpu().numpy(), inertia=inert.cpu().numpy(), n_iter=nit.cpu().numpy(), ms=ms)
