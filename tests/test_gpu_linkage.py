"""Device linkage of predict() (cc_linkage_nnchain): its raw merges equal the oracle's
restatement of scipy's nn_chain bit for bit (ties included), and predict() runs at the headline
n = 50 000 (CC.py:292-314), recovering a planted block structure."""
import time

import numpy as np
import pytest
import torch
from scipy.spatial.distance import pdist, squareform

from consensus_clustering_amd import engine, post
from oracle import cc_oracle as O

pytestmark = pytest.mark.gpu


def _distances(n, seed, ties=False):
    rs = np.random.RandomState(seed)
    X = rs.rand(n, 6).astype(np.float32)
    if ties:
        X = np.round(X * 3) / 3
        X[n // 2:] = X[: n - n // 2]
    return squareform(pdist(X, "cityblock"))


@pytest.mark.parametrize("method", ["average", "complete", "weighted"])
@pytest.mark.parametrize("n,seed,ties", [(2, 0, False), (3, 0, True), (257, 1, True), (1500, 2, False)])
def test_device_nn_chain_equals_oracle(method, n, seed, ties):
    D = _distances(n, seed, ties)
    want = O.nn_chain(D, method)
    got = engine.linkage_raw(torch.from_numpy(D).cuda(), method).cpu().numpy()
    np.testing.assert_array_equal(got, want)


def test_device_linkage_on_manhattan_of_consensus_rows():
    """The predict() chain on a consensus-like C: manhattan on the device, then the linkage;
    equal to scipy's linkage of pdist(C, 'cityblock')."""
    from scipy.cluster.hierarchy import linkage

    rs = np.random.RandomState(5)
    n, k = 900, 4
    g = rs.randint(0, k, n)
    C = (g[:, None] == g[None, :]).astype(np.float32) * 0.8 + rs.rand(n, n).astype(np.float32) * 0.2
    C = np.ascontiguousarray(np.minimum(C, C.T))
    np.fill_diagonal(C, 1.0)
    D = engine.manhattan(torch.from_numpy(C).cuda())
    Z = engine.linkage(D, "average")
    np.testing.assert_array_equal(Z, linkage(pdist(C, "cityblock"), method="average"))


def test_predict_headline_n():
    """n = 50 000 (BASELINE configs[2]): C with 6 planted blocks (co-clustering 0.9 inside a
    block, 0.1 across, noise) -> manhattan (float64) -> average linkage, all on the device; the
    cut at K = 6 recovers the blocks.  Prints the stage times."""
    n, k = 50_000, 6
    dev = torch.device("cuda")
    g = torch.randint(0, k, (n,), generator=torch.Generator().manual_seed(0)).to(dev)
    C = torch.where(g[:, None] == g[None, :], 0.9, 0.1).float()
    C += torch.rand((n, n), generator=torch.Generator(device=dev).manual_seed(1), device=dev) * 0.05
    C = torch.minimum(C, C.T).contiguous()
    C.fill_diagonal_(1.0)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    D = engine.manhattan(C)
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    del C
    Z = engine.linkage(D, "average")
    t2 = time.perf_counter()
    del D
    lab = post.hc_cut(k, Z[:, :2].astype(np.int64), n)
    t3 = time.perf_counter()
    print(f"predict n={n}: manhattan {t1 - t0:.2f} s, linkage {t2 - t1:.2f} s, cut {t3 - t2:.2f} s")
    gh = g.cpu().numpy()
    # the cut's clusters are the planted blocks (a bijection)
    pairs = set(zip(lab.tolist(), gh.tolist()))
    assert len(pairs) == k and len({a for a, _ in pairs}) == k and len({b for _, b in pairs}) == k


@pytest.mark.parametrize("n,seed,ties", [(2, 0, False), (3, 0, True), (257, 1, True), (1500, 2, False)])
def test_device_mst_equals_oracle(n, seed, ties):
    """cc_linkage_mst (sklearn's mst_linkage_core, the single-linkage path) equals the oracle's
    restatement bit for bit, ties included."""
    D = _distances(n, seed, ties)
    Dd = torch.from_numpy(D).cuda()
    out = torch.empty((n - 1, 3), dtype=torch.float64, device="cuda")
    from consensus_clustering_amd import _lib

    ws = torch.empty(int(_lib.load().cc_linkage_mst_workspace_bytes(n)), dtype=torch.uint8, device="cuda")
    _lib.call("cc_linkage_mst", Dd.data_ptr(), n, out.data_ptr(), ws.data_ptr(), ws.numel(), engine.stream_ptr())
    _lib.call("cc_linkage_check", ws.data_ptr(), ws.numel(), engine.stream_ptr())
    np.testing.assert_array_equal(out.cpu().numpy(), O.mst_prim(D))


@pytest.mark.parametrize("G", [0, 1, 2, 5, 16])
@pytest.mark.parametrize("n,seed,ties", [(3, 0, True), (257, 1, True), (1500, 2, False), (2000, 3, True)])
def test_grid_linkage_equals_oracle(G, n, seed, ties, monkeypatch):
    """The grid forms (G workgroups over index slices, grid barriers; CCMI_LINK_G = 0 is the
    one-workgroup kernel) give the oracle's nn_chain merges and Prim edges bit for bit, ties
    included, whatever G (slices of one entry and empty slices included)."""
    monkeypatch.setenv("CCMI_LINK_G", str(G))
    D = _distances(n, seed, ties)
    np.testing.assert_array_equal(engine.linkage_raw(torch.from_numpy(D).cuda(), "average").cpu().numpy(),
                                  O.nn_chain(D, "average"))
    from consensus_clustering_amd import _lib

    Dd = torch.from_numpy(D).cuda()
    out = torch.empty((n - 1, 3), dtype=torch.float64, device="cuda")
    ws = torch.empty(int(_lib.load().cc_linkage_mst_workspace_bytes(n)), dtype=torch.uint8, device="cuda")
    _lib.call("cc_linkage_mst", Dd.data_ptr(), n, out.data_ptr(), ws.data_ptr(), ws.numel(), engine.stream_ptr())
    _lib.call("cc_linkage_check", ws.data_ptr(), ws.numel(), engine.stream_ptr())
    np.testing.assert_array_equal(out.cpu().numpy(), O.mst_prim(D))


def test_grid_linkage_while_another_stream_is_busy(monkeypatch):
    """The grid forms started while another stream keeps the CUs busy (a chain of large GEMMs):
    the cooperative launch makes the G workgroups co-resident instead of assuming it, so the
    barriers cannot wait on a workgroup that never starts; the merges and edges still equal the
    oracle's."""
    monkeypatch.setenv("CCMI_LINK_G", "16")
    n = 2000
    D = _distances(n, 3, True)
    want_z, want_p = O.nn_chain(D, "average"), O.mst_prim(D)
    from consensus_clustering_amd import _lib

    side = torch.cuda.Stream()
    A = torch.randn(8192, 8192, device="cuda")
    torch.cuda.synchronize()
    with torch.cuda.stream(side):
        for _ in range(12):
            A = A @ A
            A /= A.abs().max()
    Z = engine.linkage_raw(torch.from_numpy(D).cuda(), "average").cpu().numpy()
    with torch.cuda.stream(side):
        for _ in range(12):
            A = A @ A
            A /= A.abs().max()
    Dd = torch.from_numpy(D).cuda()
    out = torch.empty((n - 1, 3), dtype=torch.float64, device="cuda")
    ws = torch.empty(int(_lib.load().cc_linkage_mst_workspace_bytes(n)), dtype=torch.uint8, device="cuda")
    _lib.call("cc_linkage_mst", Dd.data_ptr(), n, out.data_ptr(), ws.data_ptr(), ws.numel(), engine.stream_ptr())
    _lib.call("cc_linkage_check", ws.data_ptr(), ws.numel(), engine.stream_ptr())
    torch.cuda.synchronize()
    np.testing.assert_array_equal(Z, want_z)
    np.testing.assert_array_equal(out.cpu().numpy(), want_p)


def test_predict_single_linkage_equals_sklearn():
    """predict() with agg_clustering_linkage='single' (CC.py:306-312: AgglomerativeClustering(
    linkage='single', affinity='manhattan') on the rows of C) on the device: identical labels to
    sklearn's own fit on the same C."""
    from sklearn.cluster import AgglomerativeClustering

    from consensus_clustering_amd import ConsensusClustering
    from tests.conftest import load_fixture

    f = load_fixture("blobs_n400_d8_k4")
    meta = f["meta"]
    cc = ConsensusClustering(K_range=[int(k) for k in f["K_range"]], n_iterations=meta["H"],
                             subsampling=meta["subsampling"], random_state=meta["random_state"],
                             plot_cdf=False, agg_clustering_linkage="single").fit(f["X"])
    for K in (2, 4, 6):
        C = cc.cdf_at_K_data[K]["cij"]
        want = AgglomerativeClustering(n_clusters=K, linkage="single", metric="manhattan").fit_predict(C)
        np.testing.assert_array_equal(cc.predict(K), want, err_msg=f"K={K}")


def test_single_linkage_headline_n():
    """'single' linkage at n = 50 000 on the device (no host cap): the planted blocks of
    test_predict_headline_n are recovered; prints the MST time."""
    n, k = 50_000, 6
    dev = torch.device("cuda")
    g = torch.randint(0, k, (n,), generator=torch.Generator().manual_seed(0)).to(dev)
    C = torch.where(g[:, None] == g[None, :], 0.9, 0.1).float()
    C += torch.rand((n, n), generator=torch.Generator(device=dev).manual_seed(1), device=dev) * 0.05
    C = torch.minimum(C, C.T).contiguous()
    C.fill_diagonal_(1.0)
    D = engine.manhattan(C)
    del C
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    Z = engine.linkage_single(D)
    t1 = time.perf_counter()
    lab = post.hc_cut(k, Z[:, :2].astype(np.int64), n)
    print(f"single linkage n={n}: mst + finish {t1 - t0:.2f} s")
    pairs = set(zip(lab.tolist(), g.cpu().numpy().tolist()))
    assert len(pairs) == k and len({a for a, _ in pairs}) == k and len({b for _, b in pairs}) == k
