"""Label-injection parity (SURVEY §4 layer 2): the reference's own labels go into the gfx950
co-sampling / co-association / histogram kernels, which must reproduce the reference's
mij, iij and histogram counts bit-for-bit (and hence hist/cdf/pac after host post-processing)."""
import numpy as np
import pytest
import torch

from consensus_clustering_amd import engine, post
from oracle import cc_oracle as O

pytestmark = pytest.mark.gpu


def _device_labels(idx, labels_list, n, H, dev):
    Hpad = engine.pad_h(H)
    idx_d = torch.from_numpy(np.ascontiguousarray(idx, dtype=np.int32)).to(dev)
    L = engine.new_label_matrix(len(labels_list), n, Hpad, dev)
    for j, lab in enumerate(labels_list):
        lab_d = torch.from_numpy(np.ascontiguousarray(lab, dtype=np.int32)).to(dev)
        engine.scatter_labels(idx_d, lab_d, n, L[j])
    return L, Hpad


def _run(L, n, Hpad, Ks, tile_ranges=None, want_full=True):
    dev = L.device
    nt = engine.num_tiles(n)
    tile_ranges = tile_ranges or [(0, nt)]
    edges = engine.edges_device(dev)
    I_full = torch.zeros((n, n), dtype=torch.int32, device=dev) if want_full else None
    counts = torch.zeros((len(Ks), 20), dtype=torch.int64, device=dev)
    Ms = [torch.zeros((n, n), dtype=torch.int32, device=dev) if want_full else None for _ in Ks]
    for (tb, te) in tile_ranges:
        I_tiles, I_part = engine.cosample(L[0], n, Hpad, tb, te, want_full=want_full)
        if want_full:
            I_full += I_part
        for j, K in enumerate(Ks):
            Mp = torch.zeros((n, n), dtype=torch.int32, device=dev) if want_full else None
            engine.coassoc(L[j], n, Hpad, int(K), tb, te, I_tiles, edges, counts[j], Mp)
            if want_full:
                Ms[j] += Mp
    torch.cuda.synchronize()
    return (I_full.cpu().numpy() if want_full else None,
            [M.cpu().numpy() if want_full else None for M in Ms], counts.cpu().numpy())


def test_fixture_label_injection(fixture):
    dev = engine.require_gpu()
    n = fixture["X"].shape[0]
    H = fixture["meta"]["H"]
    Ks = [int(k) for k in fixture["K_range"]]
    L, Hpad = _device_labels(fixture["indices"], list(fixture["labels"]), n, H, dev)
    I, Ms, counts = _run(L, n, Hpad, Ks)
    dt = O.reference_dtype(H)
    np.testing.assert_array_equal(I.astype(dt), fixture["iij"])
    for j, K in enumerate(Ks):
        np.testing.assert_array_equal(Ms[j].astype(dt), fixture["mij"][j])
        hist, cdf, edges, pac = post.cdf_from_counts(post.pair_counts_to_hist_counts(counts[j], n))
        np.testing.assert_array_equal(hist, fixture["hist"][j])
        np.testing.assert_array_equal(cdf, fixture["cdf"][j])
        np.testing.assert_array_equal(edges, fixture["bin_edges"][j])
        assert pac == fixture["pac_area"][j]


def _random_case(n, H, frac, Ks, seed):
    rng = np.random.default_rng(seed)
    m = int(frac * n)
    idx = np.stack([rng.permutation(n)[:m] for _ in range(H)]).astype(np.int32)
    truth = rng.integers(0, 7, size=n)
    labs = []
    for K in Ks:
        lab = np.empty((H, m), dtype=np.int32)
        for h in range(H):
            noisy = (truth[idx[h]] + (rng.random(m) < 0.15) * rng.integers(0, K, size=m)) % K
            lab[h] = noisy
        labs.append(lab)
    return idx, labs


@pytest.mark.parametrize("n,H,frac,Ks", [
    (700, 200, 0.8, [2, 3, 5, 9, 17]),
    (300, 131, 0.6, [33, 100, 127]),
    (513, 300, 0.9, [4, 8, 16, 32]),
])
def test_random_labels_vs_oracle(n, H, frac, Ks):
    dev = engine.require_gpu()
    idx, labs = _random_case(n, H, frac, Ks, seed=n + H)
    L, Hpad = _device_labels(idx, labs, n, H, dev)
    I, Ms, counts = _run(L, n, Hpad, Ks)
    I_ref = O.cosample_matrix(idx.astype(np.int64), n)
    np.testing.assert_array_equal(I, I_ref)
    iu = np.triu_indices(n, 1)
    for j, K in enumerate(Ks):
        M_ref = O.coassoc_matrix(idx.astype(np.int64), labs[j].astype(np.int64), K, n)
        np.testing.assert_array_equal(Ms[j], M_ref)
        C = O.consensus_matrix(M_ref.astype(np.uint16), I_ref.astype(np.uint16))
        pair, _ = np.histogram(C[iu], bins=20, range=(0, 1))
        np.testing.assert_array_equal(counts[j], pair)


def test_cosampling_count_at_H_256():
    """Co-sampling counts at the top of the range: rows 0..399 are in every one of H = 256
    resamples (i = H), rows 0..149 keep one label each (m = i = 256), rows 0 and 1 never share a
    label (m = 0 with i = 256)."""
    dev = engine.require_gpu()
    n, H, m, Ks = 600, 256, 500, [2, 3, 7]
    rng = np.random.default_rng(11)
    idx = np.stack([np.r_[np.arange(400), 400 + rng.permutation(200)[:100]] for _ in range(H)]).astype(np.int32)
    labs = []
    for K in Ks:
        lab = rng.integers(0, K, size=(H, m)).astype(np.int32)
        lab[:, :150] = rng.integers(0, 2, size=150)  # rows 0..149: one label each (m = 256)
        lab[:, 0] = np.arange(H) % K
        lab[:, 1] = (np.arange(H) + 1) % K
        labs.append(lab)
    L, Hpad = _device_labels(idx, labs, n, H, dev)
    assert Hpad == 256
    I_ref = O.cosample_matrix(idx.astype(np.int64), n)
    assert I_ref[0, 1] == 256 and I_ref[0, 399] == 256
    iu = np.triu_indices(n, 1)
    for want_full in (False, True):
        I, Ms, counts = _run(L, n, Hpad, Ks, want_full=want_full)
        for j, K in enumerate(Ks):
            M_ref = O.coassoc_matrix(idx.astype(np.int64), labs[j].astype(np.int64), K, n)
            assert M_ref[0, 1] == 0 and M_ref[2, 3] in (0, 256)
            C = O.consensus_matrix(M_ref.astype(np.uint16), I_ref.astype(np.uint16))
            pair, _ = np.histogram(C[iu], bins=20, range=(0, 1))
            np.testing.assert_array_equal(counts[j], pair, err_msg=f"K={K} want_full={want_full}")
            if want_full:
                np.testing.assert_array_equal(Ms[j], M_ref)
        if want_full:
            np.testing.assert_array_equal(I, I_ref)


def test_tile_range_sharding_is_exact():
    """Row-band sharding of the triangle (multi-GPU mode B) sums to the single-range result."""
    dev = engine.require_gpu()
    n, H, Ks = 900, 150, [3, 6]
    idx, labs = _random_case(n, H, 0.8, Ks, seed=3)
    L, Hpad = _device_labels(idx, labs, n, H, dev)
    nt = engine.num_tiles(n)
    I1, M1, c1 = _run(L, n, Hpad, Ks)
    cuts = [(0, 2), (2, 5), (5, nt)]
    I2, M2, c2 = _run(L, n, Hpad, Ks, tile_ranges=cuts)
    np.testing.assert_array_equal(I1, I2)
    np.testing.assert_array_equal(c1, c2)
    for a, b in zip(M1, M2):
        np.testing.assert_array_equal(a, b)
    _, _, c3 = _run(L, n, Hpad, Ks, want_full=False)
    np.testing.assert_array_equal(c1, c3)


@pytest.mark.parametrize("n", [333, 2052])  # the flat kernel (n % 4 != 0) and the row kernel
def test_consensus_matrix_kernel(n):
    dev = engine.require_gpu()
    rng = np.random.default_rng(0)
    I = rng.integers(0, 1001, size=(n, n)).astype(np.int32)
    I = np.maximum(I, I.T)
    M = (I * rng.random((n, n))).astype(np.int32)
    C = engine.consensus(torch.from_numpy(M).to(dev), torch.from_numpy(I).to(dev)).cpu().numpy()
    np.testing.assert_array_equal(C, O.consensus_matrix(M.astype(np.uint16), I.astype(np.uint16)))


def test_consensus_matrix_kernel_unaligned():
    # n % 4 == 0 but M 4-B aligned only (a view one element into its buffer): cc_consensus
    # must take the flat form, whose accesses are 4-B
    dev = engine.require_gpu()
    n = 2052
    rng = np.random.default_rng(1)
    I = rng.integers(0, 1001, size=(n, n)).astype(np.int32)
    I = np.maximum(I, I.T)
    M = (I * rng.random((n, n))).astype(np.int32)
    buf = torch.empty(n * n + 1, dtype=torch.int32, device=dev)
    Mv = buf[1:].view(n, n)
    Mv.copy_(torch.from_numpy(M))
    assert Mv.data_ptr() % 16 != 0
    C = engine.consensus(Mv, torch.from_numpy(I).to(dev)).cpu().numpy()
    np.testing.assert_array_equal(C, O.consensus_matrix(M.astype(np.uint16), I.astype(np.uint16)))


@pytest.mark.parametrize("H,K", [(37, 3), (256, 10), (300, 7), (1000, 20), (1500, 5)])
def test_threshold_table_binning_is_exact(H, K):
    """cc_coassoc's division-free binning (cc_bin_table thresholds) gives the same 20 counts as
    the direct numpy-exact bin on every pair (n = 700: tile (0, 1) takes the interior-tile
    path with the staged reciprocals, the others the masked path); the table itself matches the host oracle's
    per-pair bin for every (m <= i) it covers."""
    dev = engine.require_gpu()
    n = 700
    rs = np.random.RandomState(H)
    idx = np.stack([rs.permutation(n)[: int(0.8 * n)] for _ in range(H)])
    labs = [rs.randint(0, K, size=idx.shape)]
    L, Hpad = _device_labels(idx, labs, n, H, dev)
    nt = engine.num_tiles(n)
    edges = engine.edges_device(dev)
    I_tiles, _ = engine.cosample(L[0], n, Hpad, 0, nt, want_full=False)
    c_tab = torch.zeros(20, dtype=torch.int64, device=dev)
    c_div = torch.zeros(20, dtype=torch.int64, device=dev)
    engine.coassoc(L[0], n, Hpad, K, 0, nt, I_tiles, edges, c_tab, use_table=True)
    engine.coassoc(L[0], n, Hpad, K, 0, nt, I_tiles, edges, c_div, use_table=False)
    np.testing.assert_array_equal(c_tab.cpu().numpy(), c_div.cpu().numpy())
    assert int(c_tab.sum()) == n * (n - 1) // 2
    tab = engine.bin_table(dev, Hpad + 1).cpu().numpy().view(np.uint16)[: (H + 1) * 21].reshape(H + 1, 21)
    e32 = np.linspace(0, 1, 21, dtype=np.float32)
    for i in range(0, H + 1, max(1, H // 40)):
        m = np.arange(i + 1)
        x = np.float32(m) / np.float32(np.float64(i) + 1e-6)
        ref = np.clip(np.searchsorted(e32, x, side="right") - 1, 0, 19)
        got = (m[:, None] >= tab[i, 1:20][None, :]).sum(axis=1)
        np.testing.assert_array_equal(got, ref, err_msg=f"i={i}")


def test_bin_table_exhaustive():
    """Every (m <= i) pair of counts the on-chip table can hold (i < cc_bin_table_max_rows(),
    i.e. H up to ~1940): both division-free forms give the numpy-exact bin of
    f32(m) / f32(i + 1e-6) (CC.py:338-344, :372)."""
    from consensus_clustering_amd import _lib

    dev = engine.require_gpu()
    lib = _lib.load()
    assert lib.cc_bin_table_form_rows(0) == lib.cc_bin_table_max_rows()
    # the largest table of each staged form: uint16 thresholds, threshold pairs, bin triangle
    for form in (0, 1, 2):
        rows = lib.cc_bin_table_form_rows(form)
        tab = engine.bin_table(dev, rows)
        mism = torch.zeros(4, dtype=torch.int64, device=dev)
        _lib.call("cc_bin_selftest", rows, engine.edges_device(dev).data_ptr(), tab.data_ptr(),
                  mism.data_ptr(), engine.stream_ptr())
        torch.cuda.synchronize()
        assert mism.tolist() == [0, 0, 0, 0], (form, rows, mism.tolist())
    assert lib.cc_bin_table_form_rows(2) >= 257 and lib.cc_bin_table_form_rows(1) >= 1025


@pytest.mark.parametrize("pack", ["default", "exact", "pow2"])
@pytest.mark.parametrize("n,H,frac", [(300, 200, 0.7), (260, 1000, 0.8), (129, 37, 1.0)])
def test_exact_k_packing_every_k(n, H, frac, pack, monkeypatch):
    """The FP4 one-hot padded to a power of two, its exact-K packing (K = 17, 18: floor(256/K)
    resamples per super-step, unaligned label starts, a partial last step) and the i8 form of
    K <= 2, against a float one-hot product, for every K of 2..33 with labels drawn uniformly
    over all K channels (CCMI_CO_PACK forces a packing where both exist)."""
    if pack != "default":
        monkeypatch.setenv("CCMI_CO_PACK", pack)
    dev = engine.require_gpu()
    rng = np.random.default_rng(n * H)
    m = int(frac * n)
    idx = np.stack([rng.permutation(n)[:m] for _ in range(H)]).astype(np.int32)
    Ks = list(range(2, 34))
    labs = [rng.integers(0, K, size=(H, m)).astype(np.int32) for K in Ks]
    L, Hpad = _device_labels(idx, labs, n, H, dev)
    I, Ms, counts = _run(L, n, Hpad, Ks)
    I_ref = O.cosample_matrix(idx.astype(np.int64), n)
    np.testing.assert_array_equal(I, I_ref)
    iu = np.triu_indices(n, 1)
    for j, K in enumerate(Ks):
        oh = np.zeros((n, H * K), np.float32)
        for h in range(H):
            oh[idx[h], h * K + labs[j][h]] = 1.0
        M_ref = (oh @ oh.T).astype(np.int64)
        np.testing.assert_array_equal(Ms[j], M_ref, err_msg=f"K={K}")
        C = O.consensus_matrix(M_ref.astype(np.uint16), I_ref.astype(np.uint16))
        pair, _ = np.histogram(C[iu], bins=20, range=(0, 1))
        np.testing.assert_array_equal(counts[j], pair, err_msg=f"K={K}")


@pytest.mark.parametrize("streams", [1, 2, 3])
def test_coassoc_all_streams_is_exact(streams):
    """The fit's per-K launches dealt over side streams (engine.coassoc_all) give the same
    counts and M as one launch after the other, and as the oracle's histogram."""
    dev = engine.require_gpu()
    n, H, frac, Ks = 700, 90, 0.8, [2, 3, 5, 8, 13]
    idx, labels = _random_case(n, H, frac, Ks, seed=11)
    L, Hpad = _device_labels(idx, labels, n, H, dev)
    I_ref, M_ref, counts_ref = _run(L, n, Hpad, Ks)
    nt = engine.num_tiles(n)
    I_tiles, _ = engine.cosample(L[0], n, Hpad, 0, nt)
    counts = torch.zeros((len(Ks), 20), dtype=torch.int64, device=dev)
    Ms = [torch.zeros((n, n), dtype=torch.int32, device=dev) for _ in Ks]
    engine.coassoc_all(L, n, Hpad, Ks, 0, nt, I_tiles, counts, Ms, streams=streams)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(counts.cpu().numpy(), counts_ref)
    for j in range(len(Ks)):
        np.testing.assert_array_equal(Ms[j].cpu().numpy(), M_ref[j])


@pytest.mark.parametrize("seed", range(6))
def test_fit_path_counts_random_shapes(seed):
    """The fit's own calls (co-sampling tiles without the n x n matrices, then coassoc_all over the
    side streams: interior tiles take the staged-table binning) on seeded random shapes -- n off
    the tile grid, H across the three table forms, K from 2 to 40 -- against the oracle's
    histogram of C."""
    dev = engine.require_gpu()
    rng = np.random.default_rng(1000 + seed)
    n = int(rng.integers(257, 1200))
    H = [1, 129, 256, 300, 700, 1100][seed]  # table forms: triangle (H <= ~420), pairs, uint16
    frac = float(rng.uniform(0.5, 1.0))
    Ks = sorted({int(k) for k in rng.integers(2, 41, size=3)})
    Ks = [K for K in Ks if H * K <= 9000] or [2, int(rng.integers(3, 9))]
    idx, labs = _random_case(n, H, frac, Ks, seed=seed)
    L, Hpad = _device_labels(idx, labs, n, H, dev)
    nt = engine.num_tiles(n)
    I_tiles, _ = engine.cosample(L[0], n, Hpad, 0, nt, want_full=False)
    counts = torch.zeros((len(Ks), 20), dtype=torch.int64, device=dev)
    engine.coassoc_all(L, n, Hpad, Ks, 0, nt, I_tiles, counts, None, streams=3)
    counts = counts.cpu().numpy()
    I_ref = O.cosample_matrix(idx.astype(np.int64), n)
    iu = np.triu_indices(n, 1)
    for j, K in enumerate(Ks):
        M_ref = O.coassoc_matrix(idx.astype(np.int64), labs[j].astype(np.int64), K, n)
        C = O.consensus_matrix(M_ref.astype(np.uint16), I_ref.astype(np.uint16))
        pair, _ = np.histogram(C[iu], bins=20, range=(0, 1))
        np.testing.assert_array_equal(counts[j], pair, err_msg=f"n={n} H={H} K={K}")
