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
