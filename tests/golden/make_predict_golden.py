"""Golden consensus labels for predict() (tests/test_gpu_api.py::test_predict_consensus_labels).

The reference's `_get_consensus_labels` (consensus_clustering_parallelised.py:292-314) clusters
the ROWS of the consensus matrix C with AgglomerativeClustering(n_clusters=K,
linkage=agg_clustering_linkage ('average' by default), affinity='manhattan').  Its call site is
commented out and the `affinity` keyword no longer exists in scikit-learn >= 1.4, so the
reference cannot run it as written; this script applies the same estimator with the keyword's
current name (`metric`) to the reference's own consensus matrices, rebuilt from the fixtures'
mij / iij exactly as CC.py:372-373 does, and stores the labels.

Only the K whose M the drop-in reproduces bit-for-bit are stored (blobs: K <= 4, the true number
of blobs; corr.csv: every K, float64 path).

    python tests/golden/make_predict_golden.py   (writes tests/golden/predict_golden.npz)
"""
import os
import sys

import numpy as np
from sklearn.cluster import AgglomerativeClustering

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))

from tests.conftest import load_fixture  # noqa: E402

CASES = {"blobs_n400_d8_k4": 4, "c1_corr_raw": None, "c1_corr_pt": None}


def main():
    out = {}
    for name, kmax in CASES.items():
        f = load_fixture(name)
        for j, K in enumerate(int(k) for k in f["K_range"]):
            if kmax is not None and K > kmax:
                continue
            C = np.divide(f["mij"][j], f["iij"] + 1e-6, dtype=np.float32)
            np.fill_diagonal(C, 1.0)
            agg = AgglomerativeClustering(n_clusters=K, linkage="average", metric="manhattan")
            out[f"{name}__K{K}"] = agg.fit_predict(C).astype(np.int64)
    np.savez(os.path.join(HERE, "predict_golden.npz"), **out)
    print(f"{len(out)} label vectors")


if __name__ == "__main__":
    main()
