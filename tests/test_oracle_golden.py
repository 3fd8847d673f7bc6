"""The CPU oracle (oracle/cc_oracle.py) pinned against fixtures produced by the reference itself."""
import numpy as np
import pytest

from oracle import cc_oracle as O
from tests.conftest import load_fixture


def test_indices_replay(fixture):
    meta = fixture["meta"]
    n = fixture["X"].shape[0]
    idx = O.subsampling_indices(n, meta["H"], meta["subsampling"], meta["random_state"])
    np.testing.assert_array_equal(idx, fixture["indices"])


def test_cosample_matrix(fixture):
    n = fixture["X"].shape[0]
    I = O.cosample_matrix(fixture["indices"], n)
    dt = O.reference_dtype(fixture["meta"]["H"])
    assert fixture["iij"].dtype == dt
    np.testing.assert_array_equal(I.astype(dt), fixture["iij"])


def test_coassoc_and_cdf(fixture):
    n = fixture["X"].shape[0]
    meta = fixture["meta"]
    dt = O.reference_dtype(meta["H"])
    I = O.cosample_matrix(fixture["indices"], n)
    for j, K in enumerate(fixture["K_range"]):
        M = O.coassoc_matrix(fixture["indices"], fixture["labels"][j].astype(np.int64), int(K), n)
        np.testing.assert_array_equal(M.astype(dt), fixture["mij"][j])
        res = O.analyse(M, I, dtype=dt)
        # bit-exact: hist, cdf, edges and PAC of CC.py:316-387
        np.testing.assert_array_equal(res["hist"], fixture["hist"][j])
        np.testing.assert_array_equal(res["cdf"], fixture["cdf"][j])
        np.testing.assert_array_equal(res["bin_edges"], fixture["bin_edges"][j])
        assert res["pac_area"] == fixture["pac_area"][j]
        assert res["bin_edges"].dtype == np.float32
        assert res["hist"].dtype == np.float64


def test_known_answer_c1():
    """SURVEY §8c known answers for config 1 (corr.csv raw, seed 23, H=100)."""
    f = load_fixture("c1_corr_raw")
    pac = dict(zip(f["K_range"].tolist(), f["pac_area"].tolist()))
    expect = {2: 0.353151, 3: 0.290131, 4: 0.280618, 5: 0.214031, 6: 0.160523,
              7: 0.151011, 8: 0.134364, 9: 0.098692, 10: 0.0761}
    for K, v in expect.items():
        assert abs(pac[K] - v) < 5e-6, (K, pac[K], v)
    assert int(f["mij"][0].sum()) == 36020
    np.testing.assert_array_equal(np.diag(f["iij"])[:8], [71, 81, 80, 78, 82, 76, 79, 83])


@pytest.mark.parametrize("name", ["c1_corr_raw", "blobs_n400_d8_k4"])
def test_oracle_kmeans_labels_match_reference(name):
    """The oracle's clusterer call reproduces the labels the reference consumed (1 thread)."""
    from threadpoolctl import threadpool_limits

    f = load_fixture(name)
    meta = f["meta"]
    X = f["X"]
    with threadpool_limits(1):
        for j, K in enumerate(f["K_range"][:3]):
            for h in range(0, meta["H"], max(1, meta["H"] // 5)):
                lab = O.kmeans_labels(X[f["indices"][h]], int(K), meta["random_state"], n_init=3)
                np.testing.assert_array_equal(lab, f["labels"][j, h])
