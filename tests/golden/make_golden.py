"""Generate the golden fixtures under tests/golden/ by running the REFERENCE itself.

Run in the development container only (the reference at /root/reference never
ships to the GPU box):

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden.py

The reference's ``ConsensusClustering`` (consensus_clustering_parallelised.py) is
imported read-only and run serially (``n_jobs=1``, the race-free path) with a
*recording clusterer*: an object that satisfies the reference's plugin protocol
(``n_clusters``/``n_components`` + ``set_params`` + ``fit_predict``, CC.py:201-214,
:282), delegates to scikit-learn, and records every label vector the reference
consumes.  The fixtures hold inputs and outputs only (data, no reference code):
X, the parameters, the resample indices the reference drew, the captured labels
per (K, h), and the reference's per-K results (mij, iij, hist, cdf, bin_edges,
pac_area).  The reference constructor deletes files in ``memmap_folder``
(CC.py:83-86), so it runs inside a fresh temporary directory.
"""
from __future__ import annotations

import json
import os
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REF = "/root/reference"


class Recorder:
    """Plugin-protocol clusterer that records labels (CC.py:205-214, :282)."""

    def __init__(self, factory, attr="n_clusters"):
        self.factory = factory
        self.attr = attr
        setattr(self, attr, 2)
        self.params = {}
        self.log = []  # (K, labels)

    def set_params(self, **params):
        self.params = dict(params)
        return self

    def fit_predict(self, X):
        K = getattr(self, self.attr)
        est = self.factory(K, **self.params)
        labels = np.asarray(est.fit_predict(X))
        self.log.append((K, labels.copy()))
        return labels


def kmeans_factory(K, **params):
    from sklearn.cluster import KMeans
    return KMeans(n_clusters=K, **params)


def gmm_factory(K, **params):
    from sklearn.mixture import GaussianMixture
    p = {"n_init": 2}
    p.update(params)  # clusterer_options override, as set_params does in CC.py:212-214
    return GaussianMixture(n_components=K, **p)


def run_reference(X, K_range, H, frac, seed, factory, attr="n_clusters", clusterer_options=None):
    from threadpoolctl import threadpool_limits

    sys.dont_write_bytecode = True
    if REF not in sys.path:
        sys.path.insert(0, REF)
    from consensus_clustering_parallelised import ConsensusClustering

    rec = Recorder(factory, attr)
    cwd = os.getcwd()
    with tempfile.TemporaryDirectory() as tmp, threadpool_limits(1):
        os.chdir(tmp)
        try:
            kw = dict(clusterer=rec, K_range=K_range, n_iterations=H, subsampling=frac,
                      random_state=seed, plot_cdf=False, n_jobs=1,
                      memmap_folder=os.path.join(tmp, "memmap"))
            if clusterer_options is not None:
                kw["clusterer_options"] = clusterer_options
            cc = ConsensusClustering(**kw)
            cc.fit(np.asarray(X))
            idx, _ = cc._subsample_X(np.asarray(X))  # deterministic redraw (CC.py:231-239)
        finally:
            os.chdir(cwd)
    return cc, idx, rec


def save_fixture(name, X, K_range, H, frac, seed, factory, attr="n_clusters", note="",
                 clusterer_options=None, keep_M=True):
    cc, idx, rec = run_reference(X, K_range, H, frac, seed, factory, attr, clusterer_options)
    Ks = list(K_range)
    m = idx.shape[1]
    labels = np.empty((len(Ks), H, m), dtype=np.int8)
    assert len(rec.log) == len(Ks) * H
    for j, K in enumerate(Ks):
        for h in range(H):
            k_rec, lab = rec.log[j * H + h]
            assert k_rec == K
            labels[j, h] = lab
    d = cc.cdf_at_K_data
    arrays = dict(
        X=np.asarray(X),
        K_range=np.array(Ks, dtype=np.int64),
        indices=idx.astype(np.int32),
        labels=labels,
        iij=d[Ks[0]]["iij"],
        hist=np.stack([d[K]["hist"] for K in Ks]),
        cdf=np.stack([d[K]["cdf"] for K in Ks]),
        bin_edges=np.stack([d[K]["bin_edges"] for K in Ks]),
        pac_area=np.array([d[K]["pac_area"] for K in Ks], dtype=np.float64),
    )
    if keep_M:
        arrays["mij"] = np.stack([d[K]["mij"] for K in Ks])
    import sklearn
    meta = dict(name=name, H=H, subsampling=frac, random_state=seed, note=note,
                clusterer_options=clusterer_options,
                numpy=np.__version__, sklearn=sklearn.__version__,
                python=sys.version.split()[0], threads=1)
    arrays["meta"] = np.array(json.dumps(meta))
    path = os.path.join(HERE, f"{name}.npz")
    np.savez_compressed(path, **arrays)
    print(name, {k: v.shape for k, v in arrays.items()},
          "pac:", dict(zip(Ks, np.round(arrays["pac_area"], 6))))


def corr_csv():
    import pandas as pd
    return pd.read_csv(os.path.join(REF, "corr.csv"), index_col=0).values


def main():
    from sklearn.datasets import make_blobs
    from sklearn.preprocessing import PowerTransformer

    Xc = corr_csv()
    # BASELINE config 1: raw corr.csv through the reference, K=2..10, H=100, 0.8, seed 23.
    save_fixture("c1_corr_raw", Xc, range(2, 11), 100, 0.8, 23, kmeans_factory,
                 note="BASELINE config 1, raw corr.csv (float64)")
    # Notebook recipe (NB cells 2-9) run serially: PowerTransformer, K=4..14, H=30, seed 23.
    Xpt = PowerTransformer().fit_transform(Xc)
    save_fixture("c1_corr_pt", Xpt, range(4, 15), 30, 0.8, 23, kmeans_factory,
                 note="notebook cells 2-9 recipe, serial")
    # Notebook cells 12-13: GaussianMixture(n_init=2) K=5..8 (foreign clusterer, hybrid path).
    save_fixture("c1_corr_pt_gmm", Xpt, range(5, 9), 30, 0.8, 23, gmm_factory,
                 attr="n_components", note="notebook cells 12-13 recipe, serial")
    # Small seeded blobs (float32), uint8 path.
    Xb, _ = make_blobs(n_samples=400, n_features=8, centers=4, cluster_std=1.0,
                       center_box=(-10, 10), shuffle=True, random_state=0)
    save_fixture("blobs_n400_d8_k4", Xb.astype(np.float32), range(2, 7), 40, 0.8, 0,
                 kmeans_factory, note="make_blobs(400, 8, 4 centers, seed 0) float32")
    # H >= 256 -> uint16 path (CC.py:107), and an odd subsampling fraction.
    Xb2, _ = make_blobs(n_samples=150, n_features=5, centers=3, cluster_std=1.5,
                        center_box=(-10, 10), shuffle=True, random_state=7)
    save_fixture("blobs_n150_d5_k3_h300", Xb2.astype(np.float32), range(2, 5), 300, 0.7, 11,
                 kmeans_factory, note="uint16 path (H=300), subsampling 0.7")


if __name__ == "__main__":
    main()
