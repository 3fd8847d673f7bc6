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


@pytest.mark.parametrize("n_sub", [1, 2, 5, 40])
def test_plan_covers_every_problem_once(n_sub):
    Ks = list(range(2, 21))
    g = kmeans.plan(Ks, 3, n_sub)
    assert len(g) == min(max(n_sub, 1), len(Ks))
    seen = []
    for row in g:
        P = row[0]
        assert P % 3 == 0 and 0 < P <= 64
        for p in range(P):
            K, kidx, init, ntr = row[1 + 4 * p: 5 + 4 * p]
            assert Ks[kidx] == K and ntr == kmeans.local_trials(K)
            assert init == p % 3
            seen.append((kidx, init))
        # largest K first inside a unit (longest critical paths admitted first)
        ks = [row[1 + 4 * p] for p in range(P)]
        assert ks == sorted(ks, reverse=True)
    assert sorted(seen) == [(k, i) for k in range(len(Ks)) for i in range(3)]


def test_plan_splits_beyond_unit_capacity():
    Ks = list(range(2, 40))  # 38 K x 3 inits = 114 problems > 64 per unit
    g = kmeans.plan(Ks, 3, 1)
    assert len(g) == 2 and g[:, 0].sum() == 114


def test_plan_rejects_unsupported():
    from consensus_clustering_amd import _lib

    with pytest.raises(_lib.CCMIError):
        kmeans.plan([128], 3)  # K > 127 (uint8 labels, 0xFF = not sampled)


def test_choose_subsets_fills_the_grid():
    assert kmeans.choose_subsets(1000, 19, 256) == 1
    s = kmeans.choose_subsets(125, 19, 256)  # 8 GPUs at C3: 125 resamples per GPU
    assert 125 * s >= 0.85 * 256
    assert kmeans.choose_subsets(4, 3, 256) == 3


def test_scale_exponent():
    assert kmeans.scale_exponent(0.0) == 0
    for amax in (1e-3, 0.7, 1.0, 3.0, 1e4, 6e4):
        e = kmeans.scale_exponent(amax)
        assert amax * 2.0 ** e <= 2 ** 14 and amax * 2.0 ** (e + 1) > 2 ** 14


@pytest.mark.parametrize("m,dtype", [(23, np.float64), (8001, np.float32), (40000, np.float32),
                                     (160000, np.float32), (99991, np.float64)])
def test_native_kpp_first_centre_matches_numpy_choice(m, dtype):
    """cc_kpp_tables' first-centre draw is numpy's legacy choice(m, p=w/w.sum()) bit for bit
    (float64 cumsum of the float32 or float64 p, searchsorted right), for every K's replay."""
    Ks = [2, 3, 11, 20, 127]
    u, pos, _ = kmeans.kpp_tables(Ks, 3, 7, m, dtype)
    sw = np.ones(m, dtype=dtype)
    for k, K in enumerate(Ks):
        rs = np.random.RandomState(7)
        t = kmeans.local_trials(K)
        for i in range(3):
            assert pos[k, i] == rs.choice(m, p=sw / sw.sum())
            np.testing.assert_array_equal(u[k, i, 1:1 + (K - 1) * t], rs.random_sample((K - 1) * t))


def test_numpy_argpartition_takes_distinct_farthest_first():
    """sklearn's relocation (_k_means_common.pyx:187) takes np.argpartition(d, -k)[:-k-1:-1]; on
    DISTINCT values this image's numpy returns the k largest in descending order for k <= 8, which
    is the order cc_kmeans_f64 relocates in (farthest first).  Ties are pinned separately
    (tests/test_gpu_kmeans.py::test_f64_relocation_with_ties_is_pinned)."""
    rng = np.random.default_rng(1)
    for _ in range(2000):
        n = int(rng.integers(2, 3000))
        k = int(rng.integers(1, min(n, 8) + 1))
        a = rng.random(n)
        got = np.argpartition(a, -k)[:-k - 1:-1]
        np.testing.assert_array_equal(got, np.argsort(-a, kind="stable")[:k])
