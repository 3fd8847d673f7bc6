"""C1 on the float64 path: per-K equality of mij / pac_area with the reference's fixtures."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402

from tests.conftest import load_fixture  # noqa: E402
from consensus_clustering_amd import ConsensusClustering  # noqa: E402

for name in ("c1_corr_raw", "c1_corr_pt"):
    f = load_fixture(name)
    meta = f["meta"]
    cc = ConsensusClustering(K_range=[int(k) for k in f["K_range"]], n_iterations=meta["H"],
                             subsampling=meta["subsampling"], random_state=meta["random_state"],
                             plot_cdf=False).fit(f["X"])
    res = {}
    for j, K in enumerate(int(k) for k in f["K_range"]):
        d = cc.cdf_at_K_data[K]
        res[K] = (bool(np.array_equal(d["mij"], f["mij"][j])), int((d["mij"] != f["mij"][j]).sum()),
                  float(d["pac_area"] - f["pac_area"][j]))
    print(name, cc.precision_, res, flush=True)
