"""Edge cases of the drop-in fit against the oracle (the reference's algorithm restated): K = 1,
the first wide-row width (d = 129), a single resample, a tiny n, and H just above a uint8
count (uint16 path)."""
import numpy as np
import pytest

from oracle import cc_oracle as O

pytestmark = pytest.mark.gpu


def _blobs(n, d, k, seed, std=0.6):
    from sklearn.datasets import make_blobs

    X, _ = make_blobs(n_samples=n, n_features=d, centers=k, cluster_std=std,
                      center_box=(-10, 10), shuffle=True, random_state=seed)
    return X.astype(np.float32)


def _check(X, Ks, H, seed=5, frac=0.8):
    from threadpoolctl import threadpool_limits

    from consensus_clustering_amd import ConsensusClustering

    cc = ConsensusClustering(K_range=Ks, n_iterations=H, subsampling=frac, random_state=seed,
                             plot_cdf=False).fit(X)
    with threadpool_limits(4):
        ref, _ = O.fit(X, Ks, H, frac, seed)
    for K in Ks:
        got = cc.cdf_at_K_data[K]
        np.testing.assert_array_equal(got["iij"], ref[K]["iij"])
        np.testing.assert_array_equal(got["mij"], ref[K]["mij"], err_msg=f"K={K}")
        np.testing.assert_array_equal(got["hist"], ref[K]["hist"])
        assert got["pac_area"] == ref[K]["pac_area"]
    return cc


def test_k_equals_one():
    cc = _check(_blobs(200, 6, 3, seed=1), [1, 2, 3], 20)
    d = cc.cdf_at_K_data[1]
    np.testing.assert_array_equal(d["mij"], d["iij"])  # one cluster: M == I


def test_first_wide_width():
    cc = _check(_blobs(300, 129, 3, seed=2), [2, 3], 10)
    assert cc.cdf_at_K_data[2]["mij"].shape == (300, 300)


def test_single_resample_and_tiny_n():
    _check(_blobs(12, 2, 2, seed=3, std=0.2), [2], 1)
    _check(_blobs(40, 3, 2, seed=4, std=0.3), [2, 3], 7, frac=0.5)


def test_uint16_counts_just_above_uint8():
    cc = _check(_blobs(120, 4, 2, seed=6), [2], 256)
    assert cc.cdf_at_K_data[2]["mij"].dtype == np.uint16
