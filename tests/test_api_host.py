"""Host-side API behaviour that needs no GPU: argument checks that run before any device work,
and the CDF plot (CC.py:133-134, :389-410)."""
import numpy as np
import pytest

from consensus_clustering_amd import ConsensusClustering, post


def test_seed_range_checked_for_all_resamples_before_sharding():
    """CC.py:232 seeds resample h with random_state + h; the whole H range is validated up front
    (on every rank), not per shard."""
    X = np.zeros((10, 2), dtype=np.float32)
    with pytest.raises(TypeError):
        ConsensusClustering(K_range=[2], n_iterations=5, random_state=None, plot_cdf=False).fit(X)
    with pytest.raises(ValueError, match="Seed must be between"):
        ConsensusClustering(K_range=[2], n_iterations=10, random_state=2**32 - 5,
                            plot_cdf=False).fit(X)
    with pytest.raises(ValueError, match="Seed must be between"):
        ConsensusClustering(K_range=[2], n_iterations=3, random_state=-1, plot_cdf=False).fit(X)


def test_plot_cdf_opens_and_shows_a_figure(monkeypatch):
    mpl = pytest.importorskip("matplotlib")
    mpl.use("Agg")
    import matplotlib.pyplot as plt

    shown = []
    monkeypatch.setattr(plt, "show", lambda *a, **k: shown.append(True))
    cc = ConsensusClustering(K_range=[2, 3], random_state=0, plot_cdf=True)
    counts = np.arange(20, dtype=np.int64) + 1
    cc.cdf_at_K_data = {}
    for K in (2, 3):
        hist, cdf, edges, pac = post.cdf_from_counts(counts * K)
        cc.cdf_at_K_data[K] = dict(hist=hist, cdf=cdf, bin_edges=edges, pac_area=pac)
    nfig = len(plt.get_fignums())
    ax = cc._plot_cdf()
    assert shown == [True] and len(plt.get_fignums()) == nfig + 1
    assert len(ax.get_lines()) == 2
    fig, ax2 = plt.subplots()
    assert cc._plot_cdf(ax=ax2) is ax2 and shown == [True]  # embedding: no show
    plt.close("all")


@pytest.mark.parametrize("method,n_jobs", [("multithreading", 4), ("multiprocessing", 2)])
def test_host_fit_predict_parallel_equals_serial(method, n_jobs):
    """The hybrid path's host fits (a foreign clusterer, CC.py:282) fanned out over joblib threads
    or processes as CC.py:185-195 does: the labels equal the serial loop's, in resample order."""
    from sklearn.mixture import GaussianMixture
    from threadpoolctl import threadpool_limits

    from consensus_clustering_amd.api import host_fit_predict
    from tests.conftest import load_fixture

    f = load_fixture("c1_corr_pt_gmm")
    X, idx = f["X"], f["indices"][:8]
    gmm = GaussianMixture(n_components=5, n_init=3, random_state=23)  # after set_params (CC.py:212)
    with threadpool_limits(1):
        serial = host_fit_predict(gmm, X, idx)
        par = host_fit_predict(gmm, X, idx, n_jobs=n_jobs, parallelization_method=method)
    np.testing.assert_array_equal(par, serial)
    np.testing.assert_array_equal(serial, f["labels"][0, :8])
    with pytest.raises(RuntimeError, match="unknown parallelization method"):
        host_fit_predict(gmm, X, idx, n_jobs=2, parallelization_method="mpi")
