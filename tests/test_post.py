"""Host post-processing: 20 int64 counts -> hist/cdf/bin_edges/pac bit-exact with the reference."""
import numpy as np

from consensus_clustering_amd import post
from oracle import cc_oracle as O


def test_counts_roundtrip(fixture):
    n = fixture["X"].shape[0]
    dt = O.reference_dtype(fixture["meta"]["H"])
    for j, K in enumerate(fixture["K_range"]):
        C = O.consensus_matrix(fixture["mij"][j], fixture["iij"])
        full = O.bin_counts(C)
        iu = np.triu_indices(n, 1)
        pair, _ = np.histogram(C[iu], bins=20, range=(0, 1))
        np.testing.assert_array_equal(post.pair_counts_to_hist_counts(pair, n), full)
        hist, cdf, edges, pac = post.cdf_from_counts(full)
        np.testing.assert_array_equal(hist, fixture["hist"][j])
        np.testing.assert_array_equal(cdf, fixture["cdf"][j])
        np.testing.assert_array_equal(edges, fixture["bin_edges"][j])
        assert pac == fixture["pac_area"][j]
        assert type(pac) is type(fixture["pac_area"][j])


def test_numpy2_pac_indices():
    e = post.bin_edges32()
    dbin = e[1] - e[0]
    assert dbin.dtype == np.float32
    assert (int(0.1 / dbin), int(0.9 / dbin)) == (2, 18)


def test_best_k_and_delta():
    pac = {2: 0.3, 3: 0.0, 4: 0.2, 5: 0.0}
    assert post.best_k(pac) == 3  # ties -> first K in K_range order
    areas = {2: 1.0, 3: 1.5, 4: 1.5}
    d = post.delta_k(areas)
    assert d == {2: 1.0, 3: 0.5, 4: 0.0}
    cdf = np.linspace(0.05, 1.0, 20)
    assert abs(post.cdf_area(cdf, post.bin_edges32()) - float(np.sum(np.diff(post.bin_edges32().astype(np.float64)) * cdf))) == 0
