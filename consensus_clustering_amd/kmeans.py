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

import ctypes
import os

import numpy as np
import torch

from . import _lib, engine

USTRIDE = 1 + 4 * 64   # CC_KM_USTRIDE
DPADS = (32, 64, 128)


_WORKSPACE = {}


def workspace(device, nbytes: int) -> torch.Tensor:
    """Device scratch for the k-means launches, kept across fits: re-allocating tens of GB per
    fit costs more than the fit (the caching allocator splits freed blocks for small tensors)."""
    key = str(device)
    t = _WORKSPACE.get(key)
    if t is None or t.numel() < nbytes:
        _WORKSPACE.pop(key, None)
        del t
        t = torch.empty(int(nbytes), dtype=torch.uint8, device=device)
        _WORKSPACE[key] = t
    return t[:int(nbytes)]


def release_workspace():
    """Drop the cached k-means workspace(s)."""
    _WORKSPACE.clear()


def dpad_for(d: int) -> int:
    """Feature padding: 32/64/128 for the on-chip engine (cc_kmeans_batched), a multiple of 32
    for the wide-row path (cc_kmeans_wide, d > 128)."""
    if d <= 0:
        raise ValueError("X must have at least one feature")
    for p in DPADS:
        if d <= p:
            return p
    return (d + 31) // 32 * 32


def local_trials(K: int) -> int:
    return 2 + int(np.log(K))


def plan(Ks, n_init: int, n_sub: int = 1) -> np.ndarray:
    """int32 [nU, USTRIDE] unit descriptors (see include/ccmi.h)."""
    Ks = np.ascontiguousarray(np.asarray(Ks, dtype=np.int32))
    cap = max(int(n_sub), len(Ks)) + 1
    buf = np.zeros((cap, USTRIDE), dtype=np.int32)
    nU = _lib.load().cc_kmeans_plan(Ks.ctypes.data, len(Ks), int(n_init), int(n_sub),
                                    buf.ctypes.data, cap)
    if nU <= 0:
        _lib.check(nU, "cc_kmeans_plan")
    return buf[:nU].copy()


def choose_subsets(nh: int, n_groups: int, cus: int) -> int:
    """Units per resample: enough units to fill every CU of the persistent grid with a
    balanced last round, as few as possible (bigger units pack their sweeps better)."""
    best, best_eff = 1, -1.0
    for s in range(1, max(1, n_groups) + 1):
        units = nh * s
        rounds = -(-units // cus)
        eff = units / (cus * rounds) if units >= cus else units / cus
        if eff >= 0.85:
            return s
        if eff > best_eff + 1e-9:
            best, best_eff = s, eff
    return best


def default_seedmax(m: int) -> int:
    """Problems of a unit that may seed (k-means++) concurrently.  Each seeding problem keeps
    closest-distance columns of m rows in the workspace (7 x m f32 per slot), so the cap shrinks
    with m (<= ~110 MB of columns per workgroup).  Measured (k-means launch, round 3, with the
    workspace budget not binding): C3 m = 40k: 12 / 16 / 20 / 24 / 32 -> 1679 / 1670 / 1656 /
    1645 / 1647 ms; C5 m = 160k: 6 / 8 / 12 / 16 / 20 / 24 / 32 -> 281 / 283 / 276 / 276 / 275 /
    273 / 273 ms; C2 m = 8k: 12 / 20 / 32 -> 88.2 / 87.5 / 87.0 ms.  (Round 1 measured 6 best
    at C5: there the larger caps passed the 8 GB budget and halved the grid.)"""
    return max(2, min(24, 4_000_000 // max(int(m), 1)))


def kpp_tables(Ks, n_init: int, seed: int, m: int, weight_dtype=np.float32):
    """k-means++ streams of RandomState(seed) for each (K, init) (native cc_kpp_tables; checked
    against numpy's own RandomState in tests/test_host_kmeans.py).

    Returns (kpp_u [nK, n_init, stride] float64, kpp_pos [nK, n_init] int32, stride).
    kpp_u[k, i, 1 + (c-1)*t + j] is the j-th uniform drawn for centre c of init i.
    """
    Ks_np = np.ascontiguousarray(np.asarray([int(k) for k in Ks], dtype=np.int32))
    stride = max(1 + (int(K) - 1) * local_trials(int(K)) for K in Ks_np)
    u = np.zeros((len(Ks_np), n_init, stride), dtype=np.float64)
    pos = np.zeros((len(Ks_np), n_init), dtype=np.int32)
    _lib.call("cc_kpp_tables", Ks_np.ctypes.data, len(Ks_np), int(n_init), ctypes.c_uint32(int(seed)),
              int(m), int(np.dtype(weight_dtype) == np.float64), u.ctypes.data, stride, pos.ctypes.data)
    return u, pos, stride


def scale_exponent(amax: float) -> int:
    """e with max|X| * 2^e <= 2^14, so the f16 hi/lo operand pair stays in range."""
    if not np.isfinite(amax):
        raise ValueError("X contains non-finite values")
    if amax == 0.0:
        return 0
    return int(np.clip(14 - int(np.ceil(np.log2(amax))), -62, 62))


def prepare_rows(X, device):
    """Mean-centred float32 rows zero-padded to dpad, their squared norms, and the f16 hi/lo
    MFMA operand image of the rows, on device (native cc_prepare_rows, the same preparation
    cc_kmeans_fit does).

    X is a host array or a device tensor (already resident in HBM).  sklearn centres
    X_sub by its own mean (_kmeans.py:1479-1481); distances are translation invariant,
    so one global centring serves every resample.  Returns (Xd, xnorm, dpad, Xhl, e).
    """
    n, d = X.shape
    dpad = dpad_for(d)
    Xt = X if isinstance(X, torch.Tensor) else torch.from_numpy(np.ascontiguousarray(X))
    Xt = Xt.to(device=device, dtype=torch.float32).contiguous()
    Xd = torch.empty((n, dpad), dtype=torch.float32, device=device)
    xnorm = torch.empty((n,), dtype=torch.float32, device=device)
    Xhl = torch.empty((n, 2, dpad), dtype=torch.int16, device=device)
    lib = _lib.load()
    scratch = torch.empty(int(lib.cc_prepare_rows_scratch_bytes(n, d)), dtype=torch.uint8, device=device)
    e = ctypes.c_int(0)
    _lib.call("cc_prepare_rows", Xt.data_ptr(), n, d, dpad, Xd.data_ptr(), xnorm.data_ptr(),
              Xhl.data_ptr(), ctypes.byref(e), scratch.data_ptr(), scratch.numel(),
              engine.stream_ptr(device))
    return Xd, xnorm, dpad, Xhl, int(e.value)


DEFAULT_WORKSPACE_BUDGET = 40 << 30


class BatchedKMeans:
    """All (h, K, init) k-means problems of a consensus fit, on one device."""

    def __init__(self, Ks, n_init=3, max_iter=300, tol=1e-4, random_state=0,
                 workspace_budget=None, seedmax=None, wide_budget=96 << 30):
        self.Ks = [int(k) for k in Ks]
        self.n_init = int(n_init)
        self.max_iter = int(max_iter)
        self.tol = float(tol)
        self.seed = int(random_state)
        # None: DEFAULT_WORKSPACE_BUDGET, which the float64 path may exceed to keep its grid at the
        # kernel's occupancy; a budget the caller sets (any value) is never exceeded
        self.workspace_budget = None if workspace_budget is None else int(workspace_budget)
        self.seedmax = None if seedmax is None else int(seedmax)
        self.wide_budget = int(wide_budget)
        self.stats = None
        self.units = None

    def run(self, Xd, xnorm, dreal, idx_d, n, H, m, h_begin, h_end, labels_nh, weight_dtype,
            inertia=None, n_iter=None, Xhl=None, scale_exp=None):
        """Fill labels_nh[k, :, h] for h in [h_begin, h_end) (uint8 [nK, n, ldl])."""
        dev = Xd.device
        if max(self.Ks) > m:
            raise ValueError(f"n_samples={m} should be >= n_clusters={max(self.Ks)}.")
        if Xhl is None:
            raise _lib.CCMIError("BatchedKMeans.run needs the f16 operand image (prepare_rows)")
        nh = h_end - h_begin
        self.stats = torch.zeros(128, dtype=torch.int64, device=dev)  # [0:8] counters, rest: diagnostics
        if nh <= 0:
            return labels_nh
        if Xd.shape[1] > DPADS[-1]:
            return self._run_wide(Xd, xnorm, dreal, idx_d, n, H, m, h_begin, h_end, labels_nh,
                                  weight_dtype, inertia, n_iter, Xhl, scale_exp)
        cus = torch.cuda.get_device_properties(dev).multi_processor_count
        n_sub = int(os.environ.get("CCMI_NSUB", 0)) or choose_subsets(nh, len(self.Ks), cus)
        u_h = plan(self.Ks, self.n_init, n_sub)
        self.units = u_h
        nU = u_h.shape[0]
        seedmax = max(1, min(int(os.environ.get("CCMI_SEEDMAX", 0)) or self.seedmax or default_seedmax(m),
                             32, int(u_h[:, 0].max())))
        u, pos, stride = kpp_tables(self.Ks, self.n_init, self.seed, m, weight_dtype)
        u_d = torch.from_numpy(u).to(dev)
        pos_d = torch.from_numpy(pos).to(dev)
        u_d_units = torch.from_numpy(u_h).to(dev)
        lib = _lib.load()
        per = lambda g: lib.cc_kmeans_workspace_bytes(m, Xd.shape[1], u_h.ctypes.data, nU, seedmax, g)
        grid = min(cus, nh * nU)
        budget = min(self.workspace_budget or DEFAULT_WORKSPACE_BUDGET, int(0.5 * torch.cuda.mem_get_info(dev)[0]))
        while grid > 1 and per(grid) > budget:
            grid //= 2
        ws = workspace(dev, per(grid))
        ldl = labels_nh.stride(1)
        with engine.timed("cc_kmeans_batched"):
            _lib.call("cc_kmeans_batched", Xd.data_ptr(), Xhl.data_ptr(), xnorm.data_ptr(), n,
                      int(dreal), Xd.shape[1], int(scale_exp), idx_d.data_ptr(), H, m, h_begin,
                      h_end, u_d_units.data_ptr(), u_h.ctypes.data, nU, self.n_init,
                      self.max_iter, self.tol, u_d.data_ptr(), stride, pos_d.data_ptr(),
                      labels_nh.data_ptr(), ldl, _lib.ptr(inertia), _lib.ptr(n_iter),
                      self.stats.data_ptr(), ws.data_ptr(), ws.numel(), grid, seedmax,
                      engine.stream_ptr(dev))
        return labels_nh

    def run_f64(self, X64, idx_d, n, H, m, h_begin, h_end, labels_nh, inertia=None, n_iter=None,
                grid=None):
        """float64 path (cc_kmeans_f64): X64 is the raw [n, d] float64 input on the device."""
        dev = X64.device
        if max(self.Ks) > m:
            raise ValueError(f"n_samples={m} should be >= n_clusters={max(self.Ks)}.")
        self.stats = torch.zeros(128, dtype=torch.int64, device=dev)
        nh = h_end - h_begin
        if nh <= 0:
            return labels_nh
        lib = _lib.load()
        d = X64.shape[1]
        cus = torch.cuda.get_device_properties(dev).multi_processor_count
        for k0 in range(0, len(self.Ks), 64):  # cc_kmeans_f64 takes <= 64 K values per call
            Ks = self.Ks[k0:k0 + 64]
            Ks_np = np.ascontiguousarray(np.asarray(Ks, dtype=np.int32))
            g = int(grid or min(4 * cus, nh * len(Ks)))
            per = lambda gg: lib.cc_kmeans_f64_workspace_bytes(m, d, Ks_np.ctypes.data, len(Ks), gg, nh)
            # never more than half the free device memory.  At the DEFAULT budget the grid keeps two
            # resident workgroups per CU (the kernel's occupancy) even when their scratch exceeds
            # the budget: with one per CU the float64 fit runs ~1.25x longer
            # (profiles/r04/f64_budget_r4ak.txt).  A budget the caller set is never exceeded.
            free_half = int(0.5 * torch.cuda.mem_get_info(dev)[0])
            if self.workspace_budget is None:
                cap = min(max(DEFAULT_WORKSPACE_BUDGET, per(min(g, 2 * cus))), free_half)
            else:
                cap = min(self.workspace_budget, free_half)
            if per(g) > cap:  # the largest grid that fits (per(g) is non-decreasing in g)
                lo, hi = 1, g
                while lo < hi:
                    mid = (lo + hi + 1) // 2
                    if per(mid) <= cap:
                        lo = mid
                    else:
                        hi = mid - 1
                g = lo
            ws = workspace(dev, per(g))
            u, pos, stride = kpp_tables(Ks, self.n_init, self.seed, m, np.float64)
            u_d = torch.from_numpy(u).to(dev)
            pos_d = torch.from_numpy(pos).to(dev)
            with engine.timed("cc_kmeans_f64"):
                _lib.call("cc_kmeans_f64", X64.data_ptr(), n, d, idx_d.data_ptr(), H, m, h_begin,
                          h_end, Ks_np.ctypes.data, len(Ks), self.n_init, self.max_iter, self.tol,
                          u_d.data_ptr(), stride, pos_d.data_ptr(), labels_nh[k0].data_ptr(),
                          labels_nh.stride(1),
                          None if inertia is None else inertia[k0].data_ptr(),
                          None if n_iter is None else n_iter[k0].data_ptr(), ws.data_ptr(),
                          ws.numel(), g, engine.stream_ptr(dev))
        return labels_nh

    def _run_wide(self, Xd, xnorm, dreal, idx_d, n, H, m, h_begin, h_end, labels_nh, weight_dtype,
                  inertia, n_iter, Xhl, scale_exp):
        """d > 128: cc_kmeans_wide over batches of resamples sized to the workspace budget,
        at most 64 (K, init) problems per call."""
        dev = Xd.device
        lib = _lib.load()
        dpad = Xd.shape[1]
        nh = h_end - h_begin
        per_call = max(1, 64 // self.n_init)
        free = torch.cuda.mem_get_info(dev)[0]
        budget = min(self.wide_budget, int(0.6 * free))
        ldl = labels_nh.stride(1)
        for k0 in range(0, len(self.Ks), per_call):
            Ks = self.Ks[k0:k0 + per_call]
            Ks_np = np.ascontiguousarray(np.asarray(Ks, dtype=np.int32))
            ws1 = lib.cc_kmeans_wide_workspace_bytes(m, dpad, Ks_np.ctypes.data, len(Ks),
                                                     self.n_init, 1)
            ws2 = lib.cc_kmeans_wide_workspace_bytes(m, dpad, Ks_np.ctypes.data, len(Ks),
                                                     self.n_init, 2)
            if ws1 == 0:
                _lib.check(-1, "cc_kmeans_wide_workspace_bytes")
            per = ws2 - ws1
            cap = int(max(1, min(nh, (budget - (ws1 - per)) // per)))
            batch = -(-nh // -(-nh // cap))  # equal batches: one round-count tail per batch
            ws = workspace(dev, ws1 + per * (batch - 1))
            u, pos, stride = kpp_tables(Ks, self.n_init, self.seed, m, weight_dtype)
            u_d = torch.from_numpy(u).to(dev)
            pos_d = torch.from_numpy(pos).to(dev)
            with engine.timed("cc_kmeans_wide"):
                _lib.call("cc_kmeans_wide", Xd.data_ptr(), Xhl.data_ptr(), xnorm.data_ptr(), n,
                          int(dreal), dpad, int(scale_exp), idx_d.data_ptr(), H, m, h_begin, h_end,
                          Ks_np.ctypes.data, len(Ks), self.n_init, self.max_iter, self.tol,
                          u_d.data_ptr(), stride, pos_d.data_ptr(), labels_nh[k0].data_ptr(), ldl,
                          None if inertia is None else inertia[k0].data_ptr(),
                          None if n_iter is None else n_iter[k0].data_ptr(),
                          self.stats.data_ptr(), ws.data_ptr(), ws.numel(), batch,
                          engine.stream_ptr(dev))
        return labels_nh
