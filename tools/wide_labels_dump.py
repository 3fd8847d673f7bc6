"""Dump the wide engine's labels / inertia / n_iter for one expression-data case (A/B of library
builds through CCMI_LIB): python tools/wide_labels_dump.py out.npz [n d H]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402

from bench import make_expression_f32  # noqa: E402
from consensus_clustering_amd import engine  # noqa: E402
from consensus_clustering_amd.kmeans import BatchedKMeans, prepare_rows  # noqa: E402

out = sys.argv[1]
n, d, H = (int(v) for v in (sys.argv[2:5] if len(sys.argv) > 4 else (5000, 20000, 64)))
Ks, seed = list(range(2, 13)), 0
dev = engine.require_gpu()
X = make_expression_f32(n, d, seed=seed)
m = int(0.8 * n)
idx_d = torch.from_numpy(engine.resample_indices(seed, n, m, 0, H)).to(dev)
Xd, xn, _, Xhl, e = prepare_rows(X, dev)
ts = []
for rep in range(2):
    L = engine.new_label_matrix(len(Ks), n, engine.pad_h(H), dev)
    inert = torch.zeros((len(Ks), H), dtype=torch.float32, device=dev)
    nit = torch.zeros((len(Ks), H), dtype=torch.int32, device=dev)
    bk = BatchedKMeans(Ks, n_init=3, random_state=seed)
    torch.cuda.synchronize()
    t = time.perf_counter()
    bk.run(Xd, xn, d, idx_d, n, H, m, 0, H, L, np.float32, inertia=inert, n_iter=nit, Xhl=Xhl, scale_exp=e)
    torch.cuda.synchronize()
    ts.append(time.perf_counter() - t)
np.savez(out, L=L.cpu().numpy(), inert=inert.cpu().numpy(), nit=nit.cpu().numpy())
print(os.path.basename(os.environ.get("CCMI_LIB", "libccmi.so")), "wide k-means s", [round(t, 3) for t in ts],
      "relocations", int(bk.stats[3]), "rounds", int(bk.stats[4]), flush=True)
