"""Which K of the corr.csv fixtures are well posed for k-means at float precision.

For each C1 fixture and K, scikit-learn's KMeans (the reference's clusterer, CC.py:282) is run
on every resample of the fixture twice: on the float64 rows (what the reference does) and on
the same rows cast to float32.  K is recorded as well posed when both give identical labels on
EVERY resample; where they do not, the partition hinges on rounding-level near-ties, which no
independent float64 implementation (different summation order than this container's OpenBLAS)
can be expected to reproduce.  tests/test_gpu_api.py::test_corr_csv_configs requires the
float64 GPU path to reproduce the reference's mij exactly for every well-posed K.

    python tests/golden/make_wellposed.py   (writes tests/golden/c1_wellposed.json)
"""
import json
import os
import sys

import numpy as np
from sklearn.cluster import KMeans
from threadpoolctl import threadpool_limits

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))

from tests.conftest import load_fixture  # noqa: E402


def main():
    out = {}
    for name in ("c1_corr_raw", "c1_corr_pt"):
        f = load_fixture(name)
        X, idx, seed = f["X"], f["indices"], f["meta"]["random_state"]
        ok, disagree = [], {}
        with threadpool_limits(1):
            for K in (int(k) for k in f["K_range"]):
                bad = 0
                for h in range(idx.shape[0]):
                    l64 = KMeans(n_clusters=K, random_state=seed, n_init=3).fit(X[idx[h]]).labels_
                    l32 = KMeans(n_clusters=K, random_state=seed,
                                 n_init=3).fit(X[idx[h]].astype(np.float32)).labels_
                    bad += not np.array_equal(l64, l32)
                if bad == 0:
                    ok.append(K)
                else:
                    disagree[K] = bad
        out[name] = {"well_posed_K": ok, "f32_vs_f64_disagreeing_resamples": disagree}
    with open(os.path.join(HERE, "c1_wellposed.json"), "w") as fh:
        json.dump(out, fh, indent=1)
    print(out)


if __name__ == "__main__":
    main()
