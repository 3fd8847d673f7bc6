"""Wide-engine relocation: the candidate filter (default) against every row exact
(CCMI_WIDE_RELOC_FULL=1) on the same problems: relocation count, identical labels / inertia,
and the k-means launch time of each mode.

    python tools/wide_reloc_probe.py [case ...]   (cases: c4, small)
"""
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

CASES = {
    "c4": dict(n=5000, d=20000, Ks=list(range(2, 13)), H=1000, seed=0),
    "small": dict(n=1000, d=2000, Ks=[6, 9, 12], H=64, seed=1),
    "small2": dict(n=600, d=3000, Ks=[8, 12], H=96, seed=2),
}


def run(cfg, full):
    if full:
        os.environ["CCMI_WIDE_RELOC_FULL"] = "1"
    else:
        os.environ.pop("CCMI_WIDE_RELOC_FULL", None)
    dev = engine.require_gpu()
    X = make_expression_f32(cfg["n"], cfg["d"], seed=cfg["seed"])
    n, d = X.shape
    m = int(0.8 * n)
    H, Ks = cfg["H"], cfg["Ks"]
    idx_d = torch.from_numpy(engine.resample_indices(cfg["seed"], n, m, 0, H)).to(dev)
    Xd, xn, _, Xhl, e = prepare_rows(X, dev)
    L = engine.new_label_matrix(len(Ks), n, engine.pad_h(H), dev)
    inert = torch.zeros((len(Ks), H), dtype=torch.float32, device=dev)
    bk = BatchedKMeans(Ks, n_init=3, random_state=cfg["seed"])
    torch.cuda.synchronize()
    t = time.perf_counter()
    bk.run(Xd, xn, d, idx_d, n, H, m, 0, H, L, np.float32, inertia=inert, Xhl=Xhl, scale_exp=e)
    torch.cuda.synchronize()
    return L.cpu(), inert.cpu(), int(bk.stats[3]), time.perf_counter() - t


for name in sys.argv[1:] or ["small", "small2"]:
    cfg = CASES[name]
    La, ia, ra, ta = run(cfg, False)
    Lb, ib, rb, tb = run(cfg, True)
    print(f"{name}: relocations {ra} / {rb}, labels equal {torch.equal(La, Lb)}, inertia equal "
          f"{torch.equal(ia, ib)}, filter {ta:.3f} s, all rows {tb:.3f} s", flush=True)
