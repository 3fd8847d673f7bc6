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

The float32 fixture also holds the reference's own runs on 2^-22-nudged inputs
(``pac_area_nudge``, ``max_dc_nudge``; NUDGES_ONLY=1 adds them to an existing fixture).

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


NUDGES = 2  # reference runs on float32 inputs nudged by a random-sign 2^-22 relative step


def add_nudges(name="parity_blobs_n3000_f32"):
    """The reference itself on 2^-22-nudged copies of the float32 input (NUDGES draws): its PAC
    per K and its max |dC| against the un-nudged run's C, the reference's own spread under one
    input rounding, which bounds the float32-class engine (tests/test_gpu_parity_blobs.py).  The
    un-nudged C is rebuilt from the fixture's captured labels with the oracle and checked
    against the stored digests first."""
    sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
    from oracle import cc_oracle as O

    path = os.path.join(HERE, f"{name}.npz")
    with np.load(path, allow_pickle=False) as z:
        arrays = {k: z[k] for k in z.files}
    meta = json.loads(str(arrays["meta"]))
    X, idx, labels = arrays["X"], arrays["indices"].astype(np.int64), arrays["labels"]
    Ks = [int(k) for k in arrays["K_range"]]
    n = X.shape[0]
    dt = O.reference_dtype(H)
    I = O.cosample_matrix(idx, n).astype(dt)
    assert digest(I) == meta["iij_sha256"]
    C_ref = {}
    for j, K in enumerate(Ks):
        M = O.coassoc_matrix(idx, labels[j].astype(np.int64), K, n).astype(dt)
        assert digest(M) == meta["mij_sha256"][str(K)], K
        C_ref[K] = O.consensus_matrix(M, I)
        assert digest(C_ref[K]) == meta["cij_sha256"][str(K)], K
    pac = np.zeros((NUDGES, len(Ks)))
    max_dc = np.zeros((NUDGES, len(Ks)))
    for v in range(NUDGES):
        sign = np.random.default_rng([v, 3000]).choice(np.array([-1.0, 1.0]), size=X.shape)
        Xv = (X.astype(np.float64) * (1.0 + sign * 2.0 ** -22)).astype(np.float32)
        cc, idx_v, _ = run_reference(Xv, K_RANGE, H, FRAC, SEED, kmeans_factory)
        assert np.array_equal(idx_v, idx)
        for j, K in enumerate(Ks):
            d = cc.cdf_at_K_data[K]
            pac[v, j] = d["pac_area"]
            max_dc[v, j] = float(np.abs(d["cij"].astype(np.float64) - C_ref[K]).max())
        print(f"{name} nudge {v}: |dPAC|", dict(zip(Ks, np.round(np.abs(pac[v] - arrays["pac_area"]), 6))),
              "max|dC|", dict(zip(Ks, np.round(max_dc[v], 4))), flush=True)
    arrays["pac_area_nudge"] = pac
    arrays["max_dc_nudge"] = max_dc
    meta["nudge_draws"] = NUDGES
    arrays["meta"] = np.array(json.dumps(meta))
    np.savez_compressed(path, **arrays)


def main():
    if os.environ.get("NUDGES_ONLY"):
        add_nudges()
        return
    X = blobs()
    save("parity_blobs_n3000_f64", X)
    save("parity_blobs_n3000_f32", X.astype(np.float32))
    add_nudges()


if __name__ == "__main__":
    main()
