"""Host side of the device linkage (no GPU): the oracle's restatement of scipy's nn_chain,
finished by post.linkage_finish (linkage()'s stable sort and relabelling), equals
scipy.cluster.hierarchy.linkage exactly, and post.hc_cut equals AgglomerativeClustering's labels
(CC.py:306-312) on the same precomputed distances."""
import numpy as np
import pytest
from scipy.cluster.hierarchy import linkage
from scipy.spatial.distance import pdist, squareform
from sklearn.cluster import AgglomerativeClustering

from consensus_clustering_amd import post
from oracle import cc_oracle as O


def _distances(n, seed, ties=False):
    rs = np.random.RandomState(seed)
    X = rs.rand(n, 6).astype(np.float32)
    if ties:  # duplicated rows and a coarse grid: equal distances everywhere
        X = np.round(X * 3) / 3
        X[n // 2:] = X[: n - n // 2]
    return squareform(pdist(X, "cityblock"))


@pytest.mark.parametrize("method", ["average", "complete", "weighted"])
@pytest.mark.parametrize("seed,ties", [(0, False), (1, True), (2, False)])
def test_oracle_nn_chain_matches_scipy(method, seed, ties):
    D = _distances(120, seed, ties)
    Z = post.linkage_finish(O.nn_chain(D, method), D.shape[0])
    np.testing.assert_array_equal(Z, linkage(squareform(D, checks=False), method=method))


@pytest.mark.parametrize("method", ["average", "complete"])
@pytest.mark.parametrize("K", [2, 3, 7])
def test_hc_cut_matches_agglomerative(method, K):
    D = _distances(150, 3, ties=(K == 3))
    Z = linkage(squareform(D, checks=False), method=method)
    got = post.hc_cut(K, Z[:, :2].astype(np.int64), D.shape[0])
    want = AgglomerativeClustering(n_clusters=K, metric="precomputed", linkage=method).fit_predict(D)
    np.testing.assert_array_equal(got, want)


def test_oracle_mst_prim_equals_sklearn_mst_linkage_core():
    """The oracle's Prim restatement equals sklearn's mst_linkage_core (cityblock on the rows, the
    reference's affinity='manhattan'), ties included, and the host finish (stable sort +
    _single_linkage_label) equals sklearn's single_linkage_label."""
    from scipy.spatial.distance import pdist, squareform
    from sklearn.cluster import _hierarchical_fast as hf
    from sklearn.metrics import DistanceMetric

    from consensus_clustering_amd import post
    from oracle import cc_oracle as O

    rng = np.random.default_rng(4)
    for n, ties in ((2, False), (3, True), (200, True), (500, False)):
        X = rng.random((n, 9))
        if ties:
            X = np.round(X * 3) / 3
            X[n // 2:] = X[: n - n // 2]
        want = hf.mst_linkage_core(np.ascontiguousarray(X), DistanceMetric.get_metric("cityblock"))
        got = O.mst_prim(squareform(pdist(X, "cityblock")))
        np.testing.assert_array_equal(got, want)
        np.testing.assert_array_equal(post.single_linkage_finish(got, n),
                                      hf.single_linkage_label(want[np.argsort(want.T[2], kind="mergesort")]))
