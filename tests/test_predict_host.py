"""Host half of predict() (no GPU): the linkage over precomputed float64 manhattan distances
(what the GPU's cc_manhattan feeds it) gives the reference's consensus labels
(CC.py:306-312: AgglomerativeClustering on the rows of C, manhattan metric), i.e. the
golden labels of tests/golden/make_predict_golden.py."""
import numpy as np
import pytest
from scipy.spatial.distance import pdist, squareform
from sklearn.cluster import AgglomerativeClustering

from tests.conftest import GOLDEN, load_fixture


@pytest.mark.parametrize("name", ["blobs_n400_d8_k4", "c1_corr_raw", "c1_corr_pt"])
def test_precomputed_manhattan_equals_reference_semantics(name):
    g = np.load(f"{GOLDEN}/predict_golden.npz")
    f = load_fixture(name)
    n_checked = 0
    for j, K in enumerate(int(k) for k in f["K_range"]):
        key = f"{name}__K{K}"
        if key not in g.files:
            continue
        C = np.divide(f["mij"][j], f["iij"] + 1e-6, dtype=np.float32)
        np.fill_diagonal(C, 1.0)
        D = squareform(pdist(C, "cityblock"))
        lab = AgglomerativeClustering(n_clusters=K, metric="precomputed",
                                      linkage="average").fit_predict(D)
        np.testing.assert_array_equal(lab, g[key], err_msg=key)
        n_checked += 1
    assert n_checked > 0
