"""cc_kmeans_fit, the one-call C ABI for the k-means of a fit (CC.py:282): identical labels,
inertia and iteration counts to the advanced entry points driven by the Python host, for each
engine it dispatches to (batched d <= 128, wide d > 128, float64)."""
import ctypes

import numpy as np
import pytest
import torch

from consensus_clustering_amd import _lib, engine
from consensus_clustering_amd.kmeans import BatchedKMeans, prepare_rows

pytestmark = pytest.mark.gpu


def _blobs(n, d, k, seed, dtype):
    rng = np.random.default_rng(seed)
    C = rng.uniform(-6, 6, size=(k, d))
    return (C[rng.integers(0, k, n)] + rng.normal(size=(n, d))).astype(dtype)


def _fit_abi(X, Ks, H, m, h0, h1, idx_d, precision, seed=3):
    dev = idx_d.device
    n, d = X.shape
    Xd = torch.from_numpy(X).to(dev)
    L = engine.new_label_matrix(len(Ks), n, engine.pad_h(H), dev)
    idt = torch.float64 if precision == 1 else torch.float32
    inert = torch.zeros((len(Ks), H), dtype=idt, device=dev)
    nit = torch.zeros((len(Ks), H), dtype=torch.int32, device=dev)
    Ks_np = np.ascontiguousarray(np.asarray(Ks, dtype=np.int32))
    lib = _lib.load()
    wsb = lib.cc_kmeans_fit_workspace_bytes(n, d, m, h1 - h0, Ks_np.ctypes.data, len(Ks), 3, precision)
    ws = torch.empty(int(wsb) or (1 << 20), dtype=torch.uint8, device=dev)
    _lib.call("cc_kmeans_fit", Xd.data_ptr(), n, d, idx_d.data_ptr(), H, m, h0, h1, Ks_np.ctypes.data,
              len(Ks), 3, 300, 1e-4, ctypes.c_uint32(seed), precision, L.data_ptr(), L.stride(1),
              inert.data_ptr(), nit.data_ptr(), ws.data_ptr(), ws.numel(), engine.stream_ptr(dev))
    torch.cuda.synchronize()
    return L, inert, nit


def _fit_host(X, Ks, H, m, h0, h1, idx_d, precision, seed=3):
    dev = idx_d.device
    n, d = X.shape
    L = engine.new_label_matrix(len(Ks), n, engine.pad_h(H), dev)
    idt = torch.float64 if precision == 1 else torch.float32
    inert = torch.zeros((len(Ks), H), dtype=idt, device=dev)
    nit = torch.zeros((len(Ks), H), dtype=torch.int32, device=dev)
    bk = BatchedKMeans(Ks, random_state=seed)
    if precision == 1:
        bk.run_f64(torch.from_numpy(X).to(dev), idx_d, n, H, m, h0, h1, L, inertia=inert, n_iter=nit)
    else:
        Xd, xn, _, Xhl, e = prepare_rows(X, dev)
        bk.run(Xd, xn, d, idx_d, n, H, m, h0, h1, L, np.float32, inertia=inert, n_iter=nit, Xhl=Xhl,
               scale_exp=e)
    torch.cuda.synchronize()
    return L, inert, nit


@pytest.mark.parametrize("n,d,Ks,H,h0,h1,precision", [
    (3000, 50, [2, 5, 9, 17], 12, 0, 12, 0),      # cc_kmeans_batched
    (2000, 128, [3, 8], 9, 2, 7, 0),              # a shard of the resamples
    (600, 300, [2, 4, 7], 5, 0, 5, 0),            # cc_kmeans_wide
    (400, 12, [2, 3, 6], 6, 1, 6, 1),             # cc_kmeans_f64
])
def test_one_call_matches_advanced_api(n, d, Ks, H, h0, h1, precision):
    dev = engine.require_gpu()
    X = _blobs(n, d, 5, seed=n + d, dtype=np.float64 if precision == 1 else np.float32)
    m = int(0.8 * n)
    idx = engine.resample_indices(11, n, m, 0, H)
    idx_d = torch.from_numpy(idx).to(dev)
    a = _fit_abi(X, Ks, H, m, h0, h1, idx_d, precision)
    b = _fit_host(X, Ks, H, m, h0, h1, idx_d, precision)
    for x, y in zip(a, b):
        assert torch.equal(x, y)
    # resamples outside [h0, h1) untouched
    lab = a[0][:, :, :H].cpu().numpy()
    assert (lab[:, :, :h0] == 0xFF).all() and (lab[:, :, h1:H] == 0xFF).all()
    assert (lab[:, :, h0:h1] != 0xFF).sum() == len(Ks) * (h1 - h0) * m


def test_one_call_rejects_bad_k():
    dev = engine.require_gpu()
    X = _blobs(100, 4, 3, 0, np.float32)
    idx_d = torch.from_numpy(engine.resample_indices(0, 100, 80, 0, 2)).to(dev)
    with pytest.raises(_lib.CCMIError):
        _fit_abi(X, [2, 128], 2, 80, 0, 2, idx_d, 0)


@pytest.mark.parametrize("precision,dtype", [(0, np.float32), (1, np.float64)])
def test_undersized_workspace_is_rejected(precision, dtype):
    """cc_kmeans_fit checks the workspace before it carves or uploads anything: a workspace
    smaller than the tables (and, on the float32 path, the row image) is CC_ERR_ARG, and the
    guard bytes past it stay untouched."""
    dev = engine.require_gpu()
    n, d, Ks, H = 500, 16, [2, 3], 4
    m = int(0.8 * n)
    X = _blobs(n, d, 3, seed=1, dtype=dtype)
    Xd = torch.from_numpy(X).to(dev)
    idx_d = torch.from_numpy(engine.resample_indices(1, n, m, 0, H)).to(dev)
    L = engine.new_label_matrix(len(Ks), n, engine.pad_h(H), dev)
    Ks_np = np.asarray(Ks, dtype=np.int32)
    guard = torch.full((1 << 16,), 0x5A, dtype=torch.uint8, device=dev)
    for small in (0, 256, 1024):
        with pytest.raises(_lib.CCMIError, match="workspace too small"):
            _lib.call("cc_kmeans_fit", Xd.data_ptr(), n, d, idx_d.data_ptr(), H, m, 0, H,
                      Ks_np.ctypes.data, len(Ks), 3, 300, 1e-4, ctypes.c_uint32(1), precision,
                      L.data_ptr(), L.stride(1), None, None, guard.data_ptr(), small,
                      engine.stream_ptr(dev))
    torch.cuda.synchronize()
    assert bool((guard == 0x5A).all())
    assert bool((L == 0xFF).all())
