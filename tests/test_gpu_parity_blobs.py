"""End-to-end parity at a realistic size against the REFERENCE's own run.

Fixtures: tests/golden/make_parity_blobs.py ran consensus_clustering_parallelised.py itself on
seeded blobs n = 3000, d = 32, k_true = 6, K = 2..12, H = 60 (CC.py:92-136), once with float64
X and once with float32 X, recording every label vector its clusterer returned.  The reference's
M of every K is rebuilt here from those labels by the bit-exact co-association and checked
against the SHA-256 of the reference's own mij before it is used, so the reference's C is known
exactly.

* float64 input (precision='auto' -> cc_kmeans_f64, sklearn's float64 arithmetic): every label,
  every K's mij and cij, hist, cdf and PAC identical to the reference, the same best K.
* float32 input (the f16 hi/lo MFMA engine: sklearn float32's accuracy class, not its rounding):
  identical M, C, hist, cdf and PAC for K <= k_true, the same best K, and for K > k_true |dPAC|
  and max |dC| bounded by the reference's own movement under 2^-22 input nudges (two reference
  runs stored in the fixture).  sklearn's float32 fit is not reproducible there even by
  sklearn (tests/test_parity_fixtures.py, tools/sklearn_self_parity.py).
* the C2 shape (n = 10 000, d = 64, k_true = 6, K = 2..15) at H = 50 and the C3 shape
  (n = 50 000, d = 128, k_true = 8, K = 2..20) at H = 16: sklearn's float32 labels of every
  (K, h), pushed through the reference's co-association and histogram in the development
  container (tests/golden/make_sk_fixtures.py, committed as tests/golden/sk/pac_*.npz: pair counts
  per K and every label vector's digest), give the reference's PAC per K; the engine's own fit
  must have identical labels and pair counts for K <= k_true, |dPAC| above within
  max(PAC_SPREAD_FLOOR, F32_SPREAD_FACTOR x sklearn's own |dPAC| under rounding at that K: its
  float64 run and two nudged-input float32 runs), and the same best K.
"""
import numpy as np
import pytest
import torch

from tests.conftest import digest, load_fixture

pytestmark = pytest.mark.gpu

# float32 input, K > k_true, n = 3000: the engine's distance from the reference's result is
# bounded by the reference's own distance from itself under one input rounding.  The fixture holds
# two reference runs on 2^-22-nudged inputs (make_parity_blobs.py add_nudges).  Their largest
# |dPAC| over K (3.9e-4, K = 8) times F32_SPREAD_FACTOR bounds the engine's |dPAC| at every K, and
# their largest max |dC| (0.097) bounds the engine's max |dC|.  Observed, round 6: 3.9e-4 and
# 0.077.  These replace the constants 2e-3 and 0.1 of rounds 4-5.
# C2 / C3 shapes: |dPAC| per K within max(PAC_SPREAD_FLOOR, F32_SPREAD_FACTOR x the reference's
# own PAC spread under rounding at that K): the largest |dPAC| of sklearn's float64 run and of its
# float32 runs on 2^-22-nudged inputs (two draws) against its float32 run.  At the C2 shape, K = 8,
# the float64 labels move PAC by 2.48e-3 and a nudge by 3.05e-3; at the C3 shape sklearn's own
# nudges move PAC by up to 7.9e-3 at K = 4 (tests/golden/sk/pac_*.npz).  The engine's float32-class
# arithmetic is held to the same precision class, not to one rounding.  The floor (1e-4, the
# round-6 bound; 2e-3 before the nudged runs existed) covers K whose three reference runs happen
# to agree closely (C2 K = 11: 4.1e-5 against 1.1e-5).
F32_SPREAD_FACTOR = 1.5
PAC_SPREAD_FLOOR = 1e-4


def _fit(pf, **kw):
    from consensus_clustering_amd import ConsensusClustering

    meta = pf["meta"]
    cc = ConsensusClustering(K_range=[int(k) for k in pf["K_range"]], n_iterations=meta["H"],
                             subsampling=meta["subsampling"], random_state=meta["random_state"],
                             plot_cdf=False, **kw)
    return cc.fit(pf["X"])


def _reference_counts(idx_hm, labels_khm, Ks, n, H, dev):
    """int32 M per K and I (device) from labels in resample order (the reference's fixture or a
    host clusterer), through the product co-association (cc_scatter_labels, cc_cosample,
    cc_coassoc)."""
    from consensus_clustering_amd import engine

    Hpad = engine.pad_h(H)
    idx_d = torch.from_numpy(np.ascontiguousarray(idx_hm, dtype=np.int32)).to(dev)
    L = engine.new_label_matrix(len(Ks), n, Hpad, dev)
    for j in range(len(Ks)):
        lab = torch.from_numpy(np.ascontiguousarray(labels_khm[j], dtype=np.int32)).to(dev)
        engine.scatter_labels(idx_d, lab, n, L[j])
    nt = engine.num_tiles(n)
    I_tiles, I_full = engine.cosample(L[0], n, Hpad, 0, nt, want_full=True)
    edges = engine.edges_device(dev)
    Ms, counts = [], []
    for j, K in enumerate(Ks):
        c = torch.zeros(20, dtype=torch.int64, device=dev)
        M = torch.zeros((n, n), dtype=torch.int32, device=dev)
        engine.coassoc(L[j], n, Hpad, K, 0, nt, I_tiles, edges, c, M)
        Ms.append(M)
        counts.append(c.cpu().numpy())
    return Ms, I_full, counts


def _pac_of_counts(c, n):
    from consensus_clustering_amd import post

    return post.cdf_from_counts(post.pair_counts_to_hist_counts(c, n))[3]


def _label_agreement(cc, pf):
    """Problems (K, h) whose engine labels equal the recorded ones, of all."""
    L = cc.labels_
    idx = pf["indices"]
    same = 0
    for j in range(len(pf["K_range"])):
        col = L[j].cpu().numpy()
        for h in range(idx.shape[0]):
            same += np.array_equal(col[idx[h], h].astype(np.int64), pf["labels"][j, h])
    return same, len(pf["K_range"]) * idx.shape[0]


def test_float64_input_identical_to_reference():
    pf = load_fixture("parity_blobs_n3000_f64")
    meta = pf["meta"]
    cc = _fit(pf)
    assert cc.precision_ == "f64"
    Ks = [int(k) for k in pf["K_range"]]
    same, total = _label_agreement(cc, pf)
    print(f"float64 input: {same}/{total} (K, h) label vectors identical to the reference's")
    assert digest(cc.cdf_at_K_data[Ks[0]]["iij"]) == meta["iij_sha256"]
    for j, K in enumerate(Ks):
        d = cc.cdf_at_K_data[K]
        assert digest(d["mij"]) == meta["mij_sha256"][str(K)], K
        assert digest(d["cij"]) == meta["cij_sha256"][str(K)], K
        np.testing.assert_array_equal(d["hist"], pf["hist"][j])
        np.testing.assert_array_equal(d["cdf"], pf["cdf"][j])
        assert d["pac_area"] == pf["pac_area"][j], K
    assert same == total
    assert cc.best_k_ == meta["best_k"]


def test_float32_input_against_reference():
    from consensus_clustering_amd import engine

    pf = load_fixture("parity_blobs_n3000_f32")
    meta = pf["meta"]
    n, H, kt = pf["X"].shape[0], meta["H"], meta["k_true"]
    cc = _fit(pf)
    assert cc.precision_ == "fast"
    Ks = [int(k) for k in pf["K_range"]]
    dev = cc.labels_.device
    Ms, I, counts = _reference_counts(pf["indices"], pf["labels"], Ks, n, H, dev)
    assert digest(I.cpu().numpy().astype(np.uint8)) == meta["iij_sha256"]
    same, total = _label_agreement(cc, pf)
    report = []
    for j, K in enumerate(Ks):
        d = cc.cdf_at_K_data[K]
        assert digest(Ms[j].cpu().numpy().astype(np.uint8)) == meta["mij_sha256"][str(K)], K
        C_ref = engine.consensus(Ms[j], I)
        C = torch.from_numpy(d["cij"]).to(dev)
        dC = float((C - C_ref).abs().max())
        dpac = abs(float(d["pac_area"]) - float(pf["pac_area"][j]))
        report.append((K, round(dpac, 6), round(dC, 4)))
        if K <= kt:
            assert digest(d["mij"]) == meta["mij_sha256"][str(K)], K
            assert digest(d["cij"]) == meta["cij_sha256"][str(K)], K
            np.testing.assert_array_equal(d["hist"], pf["hist"][j])
            np.testing.assert_array_equal(d["cdf"], pf["cdf"][j])
            assert d["pac_area"] == pf["pac_area"][j], K
    print(f"float32 input: {same}/{total} (K, h) label vectors identical; (K, |dPAC|, max |dC|):",
          report)
    ref_dpac = float(np.abs(pf["pac_area_nudge"] - pf["pac_area"][None, :]).max())
    ref_dc = float(pf["max_dc_nudge"].max())
    print(f"reference against itself under 2^-22 input nudges: max |dPAC| {ref_dpac:.6f}, max |dC| {ref_dc:.4f}")
    assert max(r[1] for r in report) <= F32_SPREAD_FACTOR * ref_dpac, report
    assert max(r[2] for r in report) <= ref_dc, report
    assert cc.best_k_ == meta["best_k"]


def _pac_against_fixture(case):
    """The engine's fit at the fixture's shape against sklearn's labels through the reference's
    co-association (tests/golden/sk/<case>.npz)."""
    from bench import make_blobs_f32
    from consensus_clustering_amd import ConsensusClustering, post
    from tests.sk_parity import load_sk_fixture

    f = load_sk_fixture(case)
    meta = f["meta"]
    n, d, H, Ks, seed = meta["n"], meta["d"], meta["H"], meta["Ks"], meta["seed"]
    kt = {"pac_c2_h50": 6, "pac_c3_h16": 8}[case]
    X = make_blobs_f32(n, d, kt, seed=seed)
    assert digest(X) == meta["x_sha256"]
    cc = ConsensusClustering(K_range=Ks, n_iterations=H, subsampling=meta["frac"], random_state=seed,
                             plot_cdf=False, keep_matrices=False)
    cc.fit(X)
    idx = cc.resampling_indices_
    L = cc.labels_
    report, pac_ref, over = [], {}, []
    same_total = 0
    for j, K in enumerate(Ks):
        col = L[j].cpu().numpy()
        same = sum(digest(col[idx[h], h].astype(np.int8)) == f["digest32"][j, h] for h in range(H))
        same_total += same
        pac_ref[K] = float(_pac_of_counts(f["pair_counts"][j], n))
        # the reference's own precision spread at this K: sklearn's float64 labels' PAC and its
        # nudged-input float32 runs' PACs against its float32 labels' PAC
        spread = max(abs(float(_pac_of_counts(c, n)) - pac_ref[K])
                     for c in [f["pair_counts64"][j]] + [v[j] for v in f["pair_counts_nudge"]])
        dpac = abs(float(cc.pac_area_[K]) - pac_ref[K])
        report.append((K, same, round(dpac, 6), round(spread, 6)))
        if K <= kt:
            assert same == H, (K, same)
            np.testing.assert_array_equal(cc.pair_counts_[K], f["pair_counts"][j], err_msg=f"K={K}")
        if dpac > max(PAC_SPREAD_FLOOR, F32_SPREAD_FACTOR * spread):
            over.append((K, dpac, spread))
    if "digest_nudge" in f:  # sklearn against itself: its nudged-input runs' labels equal to its own
        self_same = [int((f["digest_nudge"][:, j, :] == f["digest32"][j][None, :]).sum()) for j in range(len(Ks))]
        print(f"{case}: sklearn's nudged-input float32 runs identical to its own float32 labels, per K "
              f"(of {f['digest_nudge'].shape[0] * H}):", dict(zip(Ks, self_same)))
    print(f"{case}: {same_total}/{len(Ks) * H} label vectors identical to sklearn's float32 fit; "
          f"(K, identical of {H}, |dPAC|, sklearn's own |dPAC| under rounding):", report, "best K", cc.best_k_,
          post.best_k(pac_ref))
    assert not over, over
    assert cc.best_k_ == post.best_k(pac_ref)


def test_c2_shape_h50_sklearn_labels_through_coassoc():
    """C2's shape at H = 50: identical counts for K <= k_true, bounded |dPAC| above,
    the same best K."""
    _pac_against_fixture("pac_c2_h50")


def test_c3_shape_h16_sklearn_labels_through_coassoc():
    """C3's n, d and K range at H = 16: identical labels and counts for
    K <= k_true, |dPAC| per K reported and bounded above, the same best K."""
    _pac_against_fixture("pac_c3_h16")
