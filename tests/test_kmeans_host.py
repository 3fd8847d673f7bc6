"""Host side of the batched k-means: the RandomState stream replay and the group plan."""
import numpy as np
import pytest

from consensus_clustering_amd import kmeans


@pytest.mark.parametrize("K,m,seed,dtype", [(2, 300, 0, np.float32), (7, 1000, 23, np.float32),
                                            (20, 4000, 5, np.float64)])
def test_kpp_stream_matches_sklearn(K, m, seed, dtype):
    from sklearn.cluster._kmeans import _kmeans_plusplus

    rng = np.random.default_rng(1)
    X = rng.normal(size=(m, 4)).astype(dtype)
    sw = np.ones(m, dtype=dtype)
    xsq = (X * X).sum(1)
    u, pos, stride = kmeans.kpp_tables([K], 3, seed, m, dtype)
    rs = np.random.RandomState(seed)
    for i in range(3):
        _, ind = _kmeans_plusplus(X, K, xsq, sw, rs)
        assert ind[0] == pos[0, i]
    # the uniforms of init 1 are the doubles after init 0's 1 + (K-1)*t draws
    t = kmeans.local_trials(K)
    L = 1 + (K - 1) * t
    raw = np.random.RandomState(seed).random_sample(3 * L)
    for i in range(3):
        np.testing.assert_array_equal(u[0, i, 1:L], raw[i * L + 1:(i + 1) * L])


def test_plan_covers_every_problem_once():
    Ks = list(range(2, 21))
    g = kmeans.plan(Ks, 3)
    seen = []
    for row in g:
        P = row[0]
        assert P % 3 == 0 and P <= 32
        cols = 0
        for p in range(P):
            K, kidx, init, ntr = row[1 + 4 * p: 5 + 4 * p]
            assert Ks[kidx] == K and ntr == kmeans.local_trials(K)
            assert init == p % 3
            seen.append((kidx, init))
            cols += K
        assert cols <= 128
    assert sorted(seen) == [(k, i) for k in range(len(Ks)) for i in range(3)]
    # heavy groups first
    assert g[0, 1] == 20


def test_plan_rejects_unsupported():
    from consensus_clustering_amd import _lib

    with pytest.raises(_lib.CCMIError):
        kmeans.plan([64], 3)  # 192 columns > 128
