"""Resampling on the device (cc_resample_device, and cc_resample_device_wide for any n) against
numpy and the host replay.

Reference: consensus_clustering_parallelised.py:231-239 (`_get_subsampling_indices`): resample h
is RandomState(random_state + h).choice(n, m, replace=False) == permutation(n)[:m].  The device
kernel must reproduce it bit for bit; the host replay (cc_resample_indices) is itself pinned to
numpy in tests/test_abi.py.
"""
import numpy as np
import pytest
import torch

from consensus_clustering_amd import _lib, engine

pytestmark = pytest.mark.gpu


def _numpy(seed, n, m, h):
    return np.random.RandomState(seed + h).permutation(n)[:m].astype(np.int32)


def test_c3_shape_all_resamples_match_host_and_numpy():
    """C3: n = 50 000, m = 40 000, H = 1000 (every resample against the host replay, three
    against numpy itself)."""
    dev = engine.require_gpu()
    n, m, H, seed = 50_000, 40_000, 1000, 0
    got = engine.resample_indices_device(seed, n, m, 0, H, dev).cpu().numpy()
    ref = engine.resample_indices(seed, n, m, 0, H)
    np.testing.assert_array_equal(got, ref)
    for h in (0, 1, H - 1):
        np.testing.assert_array_equal(got[h], _numpy(seed, n, m, h))


@pytest.mark.parametrize("n,m,h0,h1,seed", [
    (1, 1, 0, 3, 5),                    # permutation(1)
    (2, 1, 0, 4, 0),
    (29, 23, 0, 100, 23),               # C1 shape
    (1000, 1000, 3, 9, 7),              # m == n, an h offset
    (65_536, 52_428, 0, 3, 11),         # largest n of the uint16 array
    (10_000, 8_000, 490, 500, 0),       # C2 shape, tail of the range
    (4_097, 17, 0, 2, 2**32 - 2),       # seed + h up to 2**32 - 1
])
@pytest.mark.parametrize("method", ["swap", "wide"])
def test_edge_shapes_match_numpy(n, m, h0, h1, seed, method):
    dev = engine.require_gpu()
    got = engine.resample_indices_device(seed, n, m, h0, h1, dev, method=method).cpu().numpy()
    assert got.shape == (h1 - h0, m)
    for k, h in enumerate(range(h0, h1)):
        np.testing.assert_array_equal(got[k], _numpy(seed, n, m, h))


def test_empty_and_rejected_arguments():
    dev = engine.require_gpu()
    assert engine.resample_indices_device(0, 100, 0, 0, 4, dev).shape == (4, 0)
    assert engine.resample_indices_device(0, 100, 80, 3, 3, dev).shape == (0, 80)
    with pytest.raises(_lib.CCMIError):
        engine.resample_indices_device(0, engine.resample_device_max_n() + 1, 10, 0, 1, dev, method="swap")
    assert engine.resample_indices_device(0, 100, 0, 0, 4, dev, method="wide").shape == (4, 0)
    with pytest.raises(ValueError):
        engine.resample_indices_device(2**32 - 1, 10, 5, 0, 2, dev)
    torch.cuda.synchronize()


def test_c5_shape_wide_matches_host_and_numpy():
    """C5: n = 200 000 > 65 536 (beyond the LDS shuffle), m = 160 000, H = 256: every resample
    of cc_resample_device_wide against the host replay, three against numpy itself; the
    workspace cap forces several resample batches."""
    dev = engine.require_gpu()
    n, m, H, seed = 200_000, 160_000, 256, 0
    cap = engine.RESAMPLE_WIDE_WS
    engine.RESAMPLE_WIDE_WS = 100 << 20  # 21 resamples per batch
    try:
        got = engine.resample_indices_device(seed, n, m, 0, H, dev).cpu().numpy()
    finally:
        engine.RESAMPLE_WIDE_WS = cap
    ref = engine.resample_indices(seed, n, m, 0, H)
    np.testing.assert_array_equal(got, ref)
    for h in (0, 1, H - 1):
        np.testing.assert_array_equal(got[h], _numpy(seed, n, m, h))


def test_fit_device_and_host_resampling_identical():
    """ConsensusClustering.fit draws the same resamples on the device and on the host: identical
    labels, pair counts and indices (C2-like blobs, small)."""
    from consensus_clustering_amd import ConsensusClustering
    rng = np.random.default_rng(4)
    centers = rng.uniform(-10, 10, size=(4, 16))
    X = np.concatenate([c + rng.normal(size=(250, 16)) for c in centers]).astype(np.float32)
    X = X[rng.permutation(len(X))]
    out = {}
    for mode in ("device", "host"):
        cc = ConsensusClustering(K_range=[2, 4, 5], n_iterations=24, random_state=9, plot_cdf=False,
                                 keep_matrices=False, resampling=mode)
        cc.fit(X)
        assert cc.resampling_ == mode
        out[mode] = cc
    a, b = out["device"], out["host"]
    np.testing.assert_array_equal(a.resampling_indices_, b.resampling_indices_)
    assert torch.equal(a.labels_, b.labels_)
    for K in (2, 4, 5):
        np.testing.assert_array_equal(a.pair_counts_[K], b.pair_counts_[K])
