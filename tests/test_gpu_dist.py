"""The multi-rank product path: ConsensusClustering.fit under a 2-rank process group (gloo,
both ranks on cuda:0) must give exactly the 1-rank fit — sharded resamples (k-means), the
all-gather of each rank's label columns, the row-band sharded triangle tiles (I, M, histogram),
the SUM of the bin counts and, with keep_matrices, the band SUMs of the full I and M.
Reference: the behaviour this replaces is CC.py:185-195 (joblib fan-out over resamples with
an in-place shared M), which loses updates; here every count is an integer sum."""
import os
import subprocess
import sys

import numpy as np
import pytest

from tests.conftest import ROOT, load_fixture

pytestmark = pytest.mark.gpu


def _one_rank(name, keep, H=0, clusterer=""):
    from consensus_clustering_amd import ConsensusClustering
    from tests.dist_worker import make_clusterer

    f = load_fixture(name)
    meta = f["meta"]
    cc = ConsensusClustering(clusterer=make_clusterer(clusterer),
                             clusterer_options={} if clusterer else {'n_init': 3},
                             K_range=[int(k) for k in f["K_range"]], n_iterations=H or meta["H"],
                             subsampling=meta["subsampling"], random_state=meta["random_state"],
                             plot_cdf=False, keep_matrices=keep)
    return cc.fit(f["X"])


@pytest.mark.parametrize("name,keep", [("blobs_n400_d8_k4", True), ("blobs_n400_d8_k4", False),
                                       ("blobs_n150_d5_k3_h300", True)])
def test_two_rank_fit_equals_one_rank(tmp_path, name, keep):
    out = str(tmp_path / "r0.npz")
    env = dict(os.environ, PYTHONPATH=ROOT)
    subprocess.run([sys.executable, os.path.join(ROOT, "tests", "dist_worker.py"), name, "2",
                    str(int(keep)), out], check=True, timeout=300, env=env)
    got = np.load(out)
    cc = _one_rank(name, keep)
    Ks = list(cc.cdf_at_K_data)
    np.testing.assert_array_equal(got["pair_counts"], np.stack([cc.pair_counts_[K] for K in Ks]))
    np.testing.assert_array_equal(got["labels"], cc.labels_.cpu().numpy())
    np.testing.assert_array_equal(got["pac"], np.array([cc.cdf_at_K_data[K]["pac_area"] for K in Ks]))
    np.testing.assert_array_equal(got["hist"], np.stack([cc.cdf_at_K_data[K]["hist"] for K in Ks]))
    if keep:
        np.testing.assert_array_equal(got["mij"], np.stack([cc.cdf_at_K_data[K]["mij"] for K in Ks]))
        np.testing.assert_array_equal(got["iij"], cc.cdf_at_K_data[Ks[0]]["iij"])


@pytest.mark.parametrize("name,keep", [("blobs_n400_d8_k4", True), ("blobs_n150_d5_k3_h300", False)])
def test_rccl_exchange_one_rank_equals_no_exchange(tmp_path, name, keep):
    """The exchange collectives on RCCL (backend 'nccl'): one rank per device is all a one-GPU box
    allows, so the fit runs in a one-rank RCCL group with the exchange forced on
    (CCMI_DIST_EXCHANGE_W1=1: the label all-gather, the count and matrix SUM all-reduces) and must
    equal the fit without any process group."""
    out = str(tmp_path / "r0.npz")
    env = dict(os.environ, PYTHONPATH=ROOT, CCMI_DIST_EXCHANGE_W1="1")
    subprocess.run([sys.executable, os.path.join(ROOT, "tests", "dist_worker.py"), name, "1",
                    str(int(keep)), out, "nccl"], check=True, timeout=300, env=env)
    got = np.load(out)
    cc = _one_rank(name, keep)
    Ks = list(cc.cdf_at_K_data)
    np.testing.assert_array_equal(got["pair_counts"], np.stack([cc.pair_counts_[K] for K in Ks]))
    np.testing.assert_array_equal(got["labels"], cc.labels_.cpu().numpy())
    np.testing.assert_array_equal(got["hist"], np.stack([cc.cdf_at_K_data[K]["hist"] for K in Ks]))
    if keep:
        np.testing.assert_array_equal(got["mij"], np.stack([cc.cdf_at_K_data[K]["mij"] for K in Ks]))


@pytest.mark.parametrize("clusterer", ["", "gmm"])
def test_rank_without_resamples_equals_one_rank(tmp_path, clusterer):
    """H = 1 on two ranks: rank 1 owns no resample (h0 == h1) on the GPU k-means path and on the
    hybrid path (host GaussianMixture fits, api.host_fit_predict of an empty index block), draws
    none, fits none, and still takes part in the label all-gather and the count SUMs; the result
    equals the 1-rank fit."""
    name = "blobs_n400_d8_k4"
    out = str(tmp_path / "r0.npz")
    env = dict(os.environ, PYTHONPATH=ROOT)
    subprocess.run([sys.executable, os.path.join(ROOT, "tests", "dist_worker.py"), name, "2", "0", out,
                    "gloo", "1", clusterer], check=True, timeout=300, env=env)
    got = np.load(out)
    cc = _one_rank(name, False, H=1, clusterer=clusterer)
    Ks = list(cc.cdf_at_K_data)
    np.testing.assert_array_equal(got["pair_counts"], np.stack([cc.pair_counts_[K] for K in Ks]))
    np.testing.assert_array_equal(got["labels"], cc.labels_.cpu().numpy())
    np.testing.assert_array_equal(got["hist"], np.stack([cc.cdf_at_K_data[K]["hist"] for K in Ks]))
