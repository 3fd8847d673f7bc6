"""Host post-processing: 20 int64 bin counts -> the reference's per-K result fields.

The device never materialises the consensus matrix on the hot path; it returns
the exact numpy.histogram bin counts of ``triu(C, 1).ravel()`` (strict upper
triangle only, see ``pair_counts_to_hist_counts``).  From those counts this
module rebuilds ``hist``, ``cdf``, ``bin_edges`` and ``pac_area`` bit-for-bit as
``_get_cdf_data`` computes them (reference ``consensus_clustering_parallelised.py``
:316-354), under numpy-2 (NEP 50) semantics:

* ``bin_edges`` are float32 (``np.linspace(0, 1, 21, dtype=float32)``, numpy
  ``_histograms_impl.py:444-452``), so ``dbin`` is ``np.float32(0.05)``;
* ``hist = counts / diff(edges).astype(float) / counts.sum()``
  (``_histograms_impl.py:900-901``);
* ``cdf = cumsum(hist) * dbin``; ``pac = cdf[int(u2/dbin) - 1] - cdf[int(u1/dbin)]``
  with float32 scalar division (u1_ind=2, u2_ind=18 for the default interval).

The north-star extensions ``cdf_area``, ``delta_k`` and ``best_k`` (no reference
implementation) are defined here.
"""
from __future__ import annotations

import numpy as np

N_BINS = 20


def bin_edges32() -> np.ndarray:
    """The exact float32 edges numpy.histogram uses for bins=20, range=(0, 1) on float32 data."""
    return np.histogram(np.zeros(1, dtype=np.float32), bins=N_BINS, range=(0, 1))[1]


def pair_counts_to_hist_counts(pair_counts, n: int) -> np.ndarray:
    """Add the n(n+1)/2 zeros that ``np.triu(C, k=1).ravel()`` contributes to bin 0.

    ``pair_counts`` are the bins of the n(n-1)/2 strict-upper-triangle pairs (CC.py:338).
    """
    c = np.asarray(pair_counts, dtype=np.int64).copy()
    if c.shape != (N_BINS,):
        raise ValueError(f"expected {N_BINS} bin counts, got shape {c.shape}")
    c[0] += n * (n + 1) // 2
    return c


def cdf_from_counts(hist_counts, PAC_interval=(0.1, 0.9)):
    """hist, cdf, bin_edges, pac_area from int64 histogram counts (CC.py:339-352)."""
    n = np.asarray(hist_counts, dtype=np.intp)
    bin_edges = bin_edges32()
    db = np.array(np.diff(bin_edges), float)
    hist = n / db / n.sum()
    dbin = bin_edges[1] - bin_edges[0]
    cdf = np.cumsum(hist) * dbin
    u1, u2 = PAC_interval
    u1_ind = int(u1 / dbin)
    u2_ind = int(u2 / dbin)
    pac_area = cdf[u2_ind - 1] - cdf[u1_ind]
    return hist, cdf, bin_edges, pac_area


def cdf_area(cdf, bin_edges) -> float:
    """Monti area under the binned CDF: Σ_b (edges[b+1] - edges[b]) · cdf[b] in float64."""
    widths = np.diff(np.asarray(bin_edges, dtype=np.float64))
    return float(np.sum(widths * np.asarray(cdf, dtype=np.float64)))


def delta_k(areas: dict) -> dict:
    """Monti Δ(K): first K -> A(K); later K -> (A(K) - A(K_prev)) / A(K_prev), in K_range order."""
    out, prev = {}, None
    for K, A in areas.items():
        out[K] = A if prev is None else (A - prev) / prev if prev != 0 else float("inf")
        prev = A
    return out


def best_k(pac: dict):
    """K with the smallest PAC area; ties -> first K in K_range order (np.argmin semantics)."""
    Ks = list(pac.keys())
    if not Ks:
        return None
    return Ks[int(np.argmin(np.array([pac[K] for K in Ks], dtype=np.float64)))]


def linkage_finish(Z, n):
    """scipy linkage()'s last steps on nn_chain's raw merges Z [n-1, 4] (x, y, distance, size in
    merge order): a stable sort by distance, then label() (scipy/cluster/_hierarchy.pyx): with a
    union-find, each merge's two clusters are renamed to their current roots (smaller first) and
    the merge creates cluster n + i."""
    Z = np.asarray(Z, dtype=np.float64)
    Z = Z[np.argsort(Z[:, 2], kind="mergesort")].copy()
    parent = list(range(2 * n - 1))
    size = [1] * (2 * n - 1)

    def find(x):
        r = x
        while parent[r] != r:
            r = parent[r]
        while parent[x] != r:
            parent[x], x = r, parent[x]
        return r

    for i in range(n - 1):
        xr, yr = find(int(Z[i, 0])), find(int(Z[i, 1]))
        Z[i, 0], Z[i, 1] = (xr, yr) if xr < yr else (yr, xr)
        parent[xr] = parent[yr] = n + i
        size[n + i] = size[xr] + size[yr]
        Z[i, 3] = size[n + i]
    return Z


def hc_cut(n_clusters, children, n_leaves):
    """Labels of the n_clusters-cluster cut of a linkage tree, as AgglomerativeClustering assigns
    them (sklearn/cluster/_agglomerative.py `_hc_cut`: a max-heap of node ids, each step
    replacing the largest by its two children; label i for the descendants of the i-th heap
    entry).  children: int [n_leaves - 1, 2] (linkage Z[:, :2])."""
    import heapq

    children = np.asarray(children, dtype=np.int64)
    nodes = [-(int(max(children[-1])) + 1)]
    for _ in range(n_clusters - 1):
        these = children[-nodes[0] - n_leaves]
        heapq.heappush(nodes, -int(these[0]))
        heapq.heappushpop(nodes, -int(these[1]))
    label = np.zeros(n_leaves, dtype=np.intp)
    for i, node in enumerate(nodes):
        stack, leaves = [-node], []
        while stack:
            v = stack.pop()
            if v < n_leaves:
                leaves.append(v)
            else:
                stack.extend(children[v - n_leaves])
        label[leaves] = i
    return label


def single_linkage_finish(mst, n):
    """sklearn's single-linkage tree from mst_linkage_core's edges [n-1, 3] (current node, new
    node, distance, in Prim order; sklearn/cluster/_agglomerative.py linkage_tree): the edges
    sorted by distance (stable mergesort), then _hierarchical_fast._single_linkage_label: with
    sklearn's UnionFind, each edge's two end points are renamed to their current clusters (left,
    right, in that order: no min/max) and the merge creates cluster n + i.  Returns Z [n-1, 4]."""
    L = np.asarray(mst, dtype=np.float64)
    L = L[np.argsort(L[:, 2], kind="mergesort")]
    parent = np.full(2 * n - 1, -1, dtype=np.int64)
    size = np.zeros(2 * n - 1, dtype=np.int64)
    size[:n] = 1
    out = np.zeros((n - 1, 4), dtype=np.float64)

    par = parent.tolist()

    def find(x):  # UnionFind.fast_find: the root, with path compression
        r = x
        while par[r] != -1:
            r = par[r]
        while x != r and par[x] != r:
            par[x], x = r, par[x]
        return r

    for i in range(n - 1):
        lc, rc = find(int(L[i, 0])), find(int(L[i, 1]))
        out[i] = (lc, rc, L[i, 2], size[lc] + size[rc])
        par[lc] = par[rc] = n + i
        size[n + i] = size[lc] + size[rc]
    return out
