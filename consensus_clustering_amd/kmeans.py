"""Host side of the batched k-means (libccmi ``cc_kmeans_plan`` / ``cc_kmeans_batched``).

Replaces the reference's per-(K, h) ``clusterer.fit_predict(X[indices])``
(consensus_clustering_parallelised.py:282) for the default clusterer
(``KMeans()`` + ``set_params(random_state=seed, n_init=3)``, CC.py:88-90, :212-214).

What stays on the host is exactly the part that depends on numpy's RNG streams:
sklearn creates ``RandomState(seed)`` afresh for every fit (``_kmeans.py:1466``), so
every resample of a given K consumes the SAME stream: per init, one
``choice(m, p=w/w.sum())`` double for the first centre, then ``uniform(size=2+⌊ln K⌋)``
per further centre (``_kmeans.py:225, :243``).  ``kpp_tables`` replays that stream
with numpy itself (so the first-centre position is numpy's own ``choice``) and hands
the remaining doubles to the kernel.
"""
from __future__ import annotations

import numpy as np
import torch

from . import _lib, engine

GSTRIDE = 1 + 4 * 32
DPADS = (32, 64, 128)


def local_trials(K: int) -> int:
    return 2 + int(np.log(K))


def plan(Ks, n_init: int) -> np.ndarray:
    """int32 [nG, GSTRIDE] group descriptors (see include/ccmi.h)."""
    Ks = np.ascontiguousarray(np.asarray(Ks, dtype=np.int32))
    buf = np.zeros((len(Ks) + 1, GSTRIDE), dtype=np.int32)
    nG = _lib.load().cc_kmeans_plan(Ks.ctypes.data, len(Ks), int(n_init), buf.ctypes.data, buf.shape[0])
    if nG <= 0:
        _lib.check(nG, "cc_kmeans_plan")
    return buf[:nG].copy()


def kpp_tables(Ks, n_init: int, seed: int, m: int, weight_dtype=np.float32):
    """k-means++ streams of RandomState(seed) for each (K, init).

    Returns (kpp_u [nK, n_init, stride] float64, kpp_pos [nK, n_init] int32, stride).
    kpp_u[k, i, 1 + (c-1)*t + j] is the j-th uniform drawn for centre c of init i.
    """
    Ks = [int(k) for k in Ks]
    stride = max(1 + (K - 1) * local_trials(K) for K in Ks)
    u = np.zeros((len(Ks), n_init, stride), dtype=np.float64)
    pos = np.zeros((len(Ks), n_init), dtype=np.int32)
    sw = np.ones(m, dtype=weight_dtype)
    p = sw / sw.sum()
    for k, K in enumerate(Ks):
        t = local_trials(K)
        rs = np.random.RandomState(seed)
        for i in range(n_init):
            pos[k, i] = rs.choice(m, p=p)              # _kmeans.py:225
            if K > 1:
                u[k, i, 1:1 + (K - 1) * t] = rs.random_sample((K - 1) * t)  # uniform(size=t) per centre
    return u, pos, stride


def prepare_rows(X, device):
    """Mean-centred float32 rows zero-padded to dpad, and their squared norms, on device.

    X is a host array or a device tensor (already resident in HBM).  sklearn centres
    X_sub by its own mean (_kmeans.py:1479-1481); distances are translation invariant,
    so one global centring serves every resample.
    """
    n, d = X.shape
    dpad = next((p for p in DPADS if d <= p), None)
    if dpad is None:
        raise _lib.CCMIError(f"batched k-means supports d <= {DPADS[-1]} in this build (got d={d})")
    Xt = X if isinstance(X, torch.Tensor) else torch.from_numpy(np.ascontiguousarray(X))
    Xt = Xt.to(device)
    mean = Xt.to(torch.float64).mean(dim=0).to(torch.float32)
    Xd = torch.zeros((n, dpad), dtype=torch.float32, device=device)
    Xd[:, :d] = Xt.to(torch.float32) - mean
    xnorm = (Xd * Xd).sum(dim=1).contiguous()
    return Xd, xnorm, dpad


class BatchedKMeans:
    """All (h, K, init) k-means problems of a consensus fit, on one device."""

    def __init__(self, Ks, n_init=3, max_iter=300, tol=1e-4, random_state=0,
                 workspace_budget=8 << 30):
        self.Ks = [int(k) for k in Ks]
        self.n_init = int(n_init)
        self.max_iter = int(max_iter)
        self.tol = float(tol)
        self.seed = int(random_state)
        self.workspace_budget = int(workspace_budget)
        self.groups = plan(self.Ks, self.n_init)
        self.stats = None

    def run(self, Xd, xnorm, dreal, idx_d, n, H, m, h_begin, h_end, labels_nh, weight_dtype,
            inertia=None, n_iter=None):
        """Fill labels_nh[k, :, h] for h in [h_begin, h_end) (uint8 [nK, n, ldl])."""
        dev = Xd.device
        if max(self.Ks) > m:
            raise ValueError(f"n_samples={m} should be >= n_clusters={max(self.Ks)}.")
        u, pos, stride = kpp_tables(self.Ks, self.n_init, self.seed, m, weight_dtype)
        u_d = torch.from_numpy(u).to(dev)
        pos_d = torch.from_numpy(pos).to(dev)
        g_h = np.ascontiguousarray(self.groups)
        g_d = torch.from_numpy(g_h).to(dev)
        nG = g_h.shape[0]
        lib = _lib.load()
        per_h = lib.cc_kmeans_workspace_bytes(m, g_h.ctypes.data, nG, 1)
        hb = max(1, min(h_end - h_begin, self.workspace_budget // max(per_h, 1)))
        ws = torch.empty(per_h * hb, dtype=torch.uint8, device=dev)
        self.stats = torch.zeros(64, dtype=torch.int64, device=dev)  # [0:4] counters, rest: diagnostics
        ldl = labels_nh.stride(1)
        for h0 in range(h_begin, h_end, hb):
            h1 = min(h_end, h0 + hb)
            with engine.timed("cc_kmeans_batched"):
                _lib.call("cc_kmeans_batched", Xd.data_ptr(), xnorm.data_ptr(), n, int(dreal),
                          Xd.shape[1], idx_d.data_ptr(), H, m, h0, h1, g_d.data_ptr(),
                          g_h.ctypes.data, nG, self.n_init, self.max_iter, self.tol,
                          u_d.data_ptr(), stride, pos_d.data_ptr(), labels_nh.data_ptr(), ldl,
                          _lib.ptr(inertia), _lib.ptr(n_iter), self.stats.data_ptr(),
                          ws.data_ptr(), ws.numel(), engine.stream_ptr(dev))
        return labels_nh
