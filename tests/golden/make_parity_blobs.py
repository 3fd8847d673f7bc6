"""End-to-end parity fixtures at a realistic size, produced by running the REFERENCE itself.

Seeded Gaussian blobs n = 3000, d = 32, k_true = 6, K = 2..12 (K well above k_true), H = 60,
subsampling 0.8, random_state 0, the default KMeans clusterer (n_init = 3), run serially
(``n_jobs=1``) through consensus_clustering_parallelised.py with the recording clusterer of
make_golden.py (CC.py:201-214, :282).  Two inputs:

* ``parity_blobs_n3000_f64``: X as float64 (the notebook's dtype, NB:63): sklearn's KMeans runs
  in float64, which precision='auto' reproduces with cc_kmeans_f64;
* ``parity_blobs_n3000_f32``: the same X cast to float32: sklearn's KMeans runs in float32, which
  the f16 hi/lo MFMA engine matches in accuracy class (22-bit operands), not in rounding.

The n x n matrices are too large to commit (11 x 9 MB per input), so each fixture holds the
inputs, the resample indices, every captured label vector, the reference's per-K hist / cdf /
bin_edges / pac_area, and SHA-256 digests of the reference's iij, of every K's mij and of every
K's cij.  The GPU test rebuilds M from the captured labels with the bit-exact co-association
and checks it against the digests first, so the reference's C is available exactly.

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_parity_blobs.py
"""
from __future__ import annotations

import hashlib
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)

from make_golden import kmeans_factory, run_reference  # noqa: E402

N, D, K_TRUE, H, FRAC, SEED = 3000, 32, 6, 60, 0.8, 0
K_RANGE = range(2, 13)


def digest(a) -> str:
    a = np.ascontiguousarray(a)
    return hashlib.sha256(a.view(np.uint8).tobytes() + str(a.dtype).encode() + str(a.shape).encode()).hexdigest()


def blobs():
    from sklearn.datasets import make_blobs

    X, _ = make_blobs(n_samples=N, n_features=D, centers=K_TRUE, cluster_std=1.0,
                      center_box=(-10, 10), shuffle=True, random_state=0)
    return X  # float64


def save(name, X):
    import sklearn

    cc, idx, rec = run_reference(X, K_RANGE, H, FRAC, SEED, kmeans_factory)
    Ks = list(K_RANGE)
    m = idx.shape[1]
    labels = np.empty((len(Ks), H, m), dtype=np.int8)
    assert len(rec.log) == len(Ks) * H
    for j, K in enumerate(Ks):
        for h in range(H):
            k_rec, lab = rec.log[j * H + h]
            assert k_rec == K
            labels[j, h] = lab
    d = cc.cdf_at_K_data
    pac = np.array([d[K]["pac_area"] for K in Ks], dtype=np.float64)
    meta = dict(name=name, H=H, subsampling=FRAC, random_state=SEED, k_true=K_TRUE,
                note=f"make_blobs({N}, {D}, {K_TRUE} centers, std 1, box (-10, 10), seed 0) "
                     f"as {X.dtype}; reference run serially, 1 BLAS thread",
                numpy=np.__version__, sklearn=sklearn.__version__,
                python=sys.version.split()[0], threads=1,
                iij_sha256=digest(d[Ks[0]]["iij"]),
                mij_sha256={str(K): digest(d[K]["mij"]) for K in Ks},
                cij_sha256={str(K): digest(d[K]["cij"]) for K in Ks},
                mij_dtype=str(d[Ks[0]]["mij"].dtype),
                best_k=int(Ks[int(np.argmin(pac))]))
    arrays = dict(
        X=np.asarray(X),
        K_range=np.array(Ks, dtype=np.int64),
        indices=idx.astype(np.int32),
        labels=labels,
        hist=np.stack([d[K]["hist"] for K in Ks]),
        cdf=np.stack([d[K]["cdf"] for K in Ks]),
        bin_edges=np.stack([d[K]["bin_edges"] for K in Ks]),
        pac_area=pac,
        meta=np.array(json.dumps(meta)),
    )
    np.savez_compressed(os.path.join(HERE, f"{name}.npz"), **arrays)
    print(name, "best_k", meta["best_k"], "pac:", dict(zip(Ks, np.round(pac, 6))))


def main():
    X = blobs()
    save("parity_blobs_n3000_f64", X)
    save("parity_blobs_n3000_f32", X.astype(np.float32))


if __name__ == "__main__":
    main()
