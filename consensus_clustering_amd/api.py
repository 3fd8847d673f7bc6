"""Drop-in ``ConsensusClustering`` (reference: consensus_clustering_parallelised.py, "CC.py").

Same constructor keywords (CC.py:21-36), ``fit(X) -> self`` (CC.py:92-136) and the same
per-K result dict ``cdf_at_K_data[K]`` with keys consensus_labels, hist, cdf, bin_edges,
pac_area, mij, iij, cij and the reference's dtypes (CC.py:378-387): mij/iij in uint8
when n_iterations < 256 else uint16 (CC.py:107), cij float32 with a unit diagonal,
bin_edges float32, hist/cdf float64, pac_area np.float64.

What runs where (``fit``):
  resampling      numpy-RandomState replay on the device (libccmi cc_resample_device /
                  cc_resample_device_wide) or on host threads (cc_resample_indices)
  clustering      default clusterer (KMeans) -> all (h, K, init) problems in batched
                  gfx950 launches (cc_kmeans_batched); any other plugin clusterer
                  (e.g. GaussianMixture) keeps the reference's host fit_predict per
                  (K, h) and only its labels go to the GPU (hybrid path)
  I, M, histogram int8-MFMA tiles of the upper triangle (cc_cosample / cc_coassoc)
  hist/cdf/PAC    host float64 from 20 exact integer counts (post.py)
  multi-GPU       resamples and triangle tiles sharded over torch.distributed ranks
                  (dist.py); RCCL all-gather of each rank's label columns, SUM of counts

Deliberate differences, all documented in DESIGN.md: the constructor does not delete
files in ``memmap_folder`` (CC.py:83-86); the n x n matrices are materialised only when
``keep_matrices`` (default: n <= 20000) since the reference's O(n^2)-per-K retention is
infeasible at n = 50k; n_jobs / parallelization_method parallelise only the host fits of a
foreign clusterer (``host_fit_predict``: joblib threads or processes as CC.py:185-195, with
labels returned instead of added into a shared Mij, so nothing races; the default KMeans runs on
the GPU whatever n_jobs says).
Additions: ``cdf_area_``, ``delta_k_``, ``pac_area_``, ``best_k_`` and ``predict``.
"""
from __future__ import annotations

import os
import time
import warnings

import numpy as np
import torch

from . import dist, engine, post
from ._hostfit import fit_predict_chunk, fit_predict_one
from .kmeans import BatchedKMeans

KMAX = 127  # largest K: uint8 labels (0xFF = not sampled) and int8 one-hot channels


def _default_kmeans():
    from sklearn.cluster import KMeans

    return KMeans()


def _is_default_kmeans(est) -> bool:
    """KMeans configured so that the batched gfx950 k-means reproduces it."""
    try:
        from sklearn.cluster import KMeans
    except ImportError:  # pragma: no cover
        return False
    if type(est) is not KMeans:
        return False
    p = est.get_params()
    return (isinstance(p.get("init"), str) and p["init"] == "k-means++"
            and p.get("algorithm", "lloyd") in ("lloyd", "auto", "full")
            and p.get("n_init") is not None)


class ConsensusClustering:
    """Monti consensus clustering on MI355X.  Drop-in for CC.py:11."""

    def __init__(
        self,
        clusterer=None,
        clusterer_options={'n_init': 3},
        K_range=(2, 3),
        n_iterations=25,
        subsampling=0.8,
        random_state=None,
        consensus_matrix_analysis='PAC',
        PAC_interval=(0.1, 0.9),
        plot_cdf=True,
        agg_clustering_linkage='average',
        n_jobs=1,
        parallelization_method='multithreading',
        memmap_folder='./memmap',
        *,
        keep_matrices='auto',
        device=None,
        workspace_budget=None,
        precision='auto',
        resampling='auto',
    ):
        self.K_range = K_range
        self.n_iterations = n_iterations
        self.subsampling = subsampling
        self.clusterer = clusterer
        self.clusterer_options = clusterer_options

        self.consensus_matrix_analysis = consensus_matrix_analysis
        self.PAC_interval = PAC_interval
        self.plot_cdf = plot_cdf
        self.agg_clustering_linkage = agg_clustering_linkage

        self.random_state = random_state
        self.n_jobs = n_jobs
        self.parallelization_method = parallelization_method
        self.memmap_folder = memmap_folder  # kept for compatibility; never touched

        self.keep_matrices = keep_matrices
        self.device = device
        self.workspace_budget = workspace_budget
        # k-means arithmetic: 'f64' = float64 like sklearn on float64 input (cc_kmeans_f64),
        # 'fast' = the float32-class f16 hi/lo MFMA engine; 'auto' = f64 for float64 input, fast
        # for float32 (sklearn's own choice of arithmetic follows X's dtype)
        self.precision = precision
        # where the resample indices are drawn: 'device' (cc_resample_device for n <= 65536,
        # cc_resample_device_wide above), 'host' (native threads, then uploaded), 'auto' =
        # device; identical draws
        self.resampling = resampling
        self.timings_ = {}
        self._rehearsal = None  # (rank, world): bench tooling only, see fit()

        if self.clusterer is None:
            print('KMeans is set as default clusterer')
            self.clusterer = _default_kmeans()

    # ------------------------------------------------------------------ plugin
    def _set_clusterer_K(self):
        """CC.py:201-214: set n_clusters / n_components, then set_params(random_state, **opts)."""
        if hasattr(self.clusterer, 'n_clusters'):
            self.clusterer.n_clusters = self._K
        elif hasattr(self.clusterer, 'n_components'):
            self.clusterer.n_components = self._K
        else:
            raise AttributeError('clusterer has neither n_clusters nor n_components attribute')
        self.clusterer.set_params(random_state=self.random_state, **self.clusterer_options)

    def _kmeans_params(self):
        """The KMeans parameters after the reference's set_params (clusterer_options win)."""
        Ks = list(self.K_range)
        if not Ks:
            return None
        self._K = Ks[0]
        self._set_clusterer_K()
        if not _is_default_kmeans(self.clusterer):
            return None
        p = self.clusterer.get_params()
        n_init = p["n_init"]
        if n_init == "auto":
            n_init = 1  # sklearn: 'auto' -> 1 run for init='k-means++'
        return dict(n_init=int(n_init), max_iter=int(p["max_iter"]), tol=float(p["tol"]))

    # ------------------------------------------------------------------ fit
    def fit(self, X):
        """Fit on X [n_samples, n_features] and fill ``cdf_at_K_data`` (CC.py:92-136)."""
        t_start = time.perf_counter()
        if isinstance(X, torch.Tensor):  # already resident in device memory
            wdtype = np.float64 if X.dtype == torch.float64 else np.float32
        else:
            X = np.asarray(X)
            wdtype = X.dtype if X.dtype in (np.float32, np.float64) else np.float64
        self._N, _ = X.shape
        self._dtype = np.uint8 if self.n_iterations < 256 else np.uint16
        self.cdf_at_K_data = dict()
        n, H = self._N, int(self.n_iterations)
        m = int(self.subsampling * n)
        Ks = [int(K) for K in self.K_range]
        self._check_k_range(Ks)
        # the reference seeds resample h with random_state + h (CC.py:232): validate the whole
        # H range once, on every rank, before sharding (a rank-local check would let the other
        # ranks go on into the exchanges and hang)
        if self.random_state is None:
            raise TypeError("unsupported operand type(s) for +: 'NoneType' and 'int'")
        if H > 0 and (int(self.random_state) < 0 or int(self.random_state) + H - 1 > 2**32 - 1):
            raise ValueError("Seed must be between 0 and 2**32 - 1")
        rank, W = dist.world()
        # a refit replaces the previous results: their device buffers are dropped first, so the
        # new label matrix and indices reuse that memory instead of growing the pool by a set
        self.labels_ = self._idx_dev = self._idx_host = None
        self.kmeans_inertia_ = self.kmeans_n_iter_ = self.kmeans_stats_ = None
        self.partial_ = False
        if self._rehearsal is not None:
            # one-GPU rehearsal of rank r's share of a W-rank fit (bench tooling only): the
            # exchanges are skipped, so every count below covers rank r's share alone
            if W > 1:
                raise RuntimeError("rehearsal runs without a process group")
            rank, W = self._rehearsal
            self.partial_ = True
            warnings.warn(f"rehearsing rank {rank} of {W}: results are PARTIAL (timing only)")
        dev = engine.require_gpu(self.device)
        keep = self.keep_matrices
        if keep == 'auto':
            keep = n <= 20000

        # resampling (CC.py:216-241): each rank replays only its own resamples [h0, h1); rows
        # outside the shard stay zero and are never read (the co-sampling counts come from the
        # merged label matrix, not from the indices)
        h0, h1 = dist.shard(H, rank, W)
        if self.resampling not in ('auto', 'device', 'host'):
            raise ValueError("resampling must be 'auto', 'device' or 'host'")
        on_dev = self.resampling != 'host'
        self.resampling_ = 'device' if on_dev else 'host'
        idx = None  # host copy, made only when a host consumer needs it (resampling_indices_)
        if on_dev:
            idx_d = (torch.empty if (h0, h1) == (0, H) else torch.zeros)((H, m), dtype=torch.int32, device=dev)
            if h1 > h0:
                engine.resample_indices_device(self.random_state, n, m, h0, h1, dev, out=idx_d[h0:h1])
        else:
            own = engine.resample_indices(self.random_state, n, m, h0, h1) if h1 > h0 else None
            if (h0, h1) == (0, H):
                idx = own
                idx_d = torch.from_numpy(idx).to(dev)
            else:
                idx = np.zeros((H, m), dtype=np.int32)
                idx_d = torch.zeros((H, m), dtype=torch.int32, device=dev)
                if own is not None:
                    idx[h0:h1] = own
                    idx_d[h0:h1] = torch.from_numpy(own).to(dev)
        Hpad = engine.pad_h(H)
        labels = engine.new_label_matrix(max(len(Ks), 1), n, Hpad, dev)
        if on_dev:
            torch.cuda.synchronize(dev)  # stage timing only: the k-means waits for the indices anyway
        t_rs = time.perf_counter()

        km = self._kmeans_params()
        self.backend_ = 'gpu-kmeans' if km is not None else 'host-clusterer'
        precision = self.precision
        if precision == 'auto':
            # the reference's clusterer computes in X's dtype (CC.py:282): float64 input keeps
            # sklearn's float64 arithmetic (cc_kmeans_f64) whatever the size; the float32-class
            # engine is opt-in for it (precision='fast')
            precision = 'f64' if (wdtype == np.float64 and km is not None) else 'fast'
        if precision not in ('f64', 'fast'):
            raise ValueError("precision must be 'auto', 'f64' or 'fast'")
        self.precision_ = precision if km is not None else None
        if Ks and km is not None:
            bk = BatchedKMeans(Ks, n_init=km["n_init"], max_iter=km["max_iter"], tol=km["tol"],
                               random_state=self.random_state,
                               workspace_budget=self.workspace_budget)
            self.kmeans_n_iter_ = torch.zeros((len(Ks), H), dtype=torch.int32, device=dev)
            if precision == 'f64':
                # float64 input: the reference's clusterer runs in float64 (CC.py:282)
                X64 = (X.to(dev, torch.float64) if isinstance(X, torch.Tensor)
                       else torch.from_numpy(np.ascontiguousarray(X, dtype=np.float64)).to(dev))
                self.kmeans_inertia_ = torch.zeros((len(Ks), H), dtype=torch.float64, device=dev)
                bk.run_f64(X64.contiguous(), idx_d, n, H, m, h0, h1, labels,
                           inertia=self.kmeans_inertia_, n_iter=self.kmeans_n_iter_)
            else:
                Xd, xnorm, _, Xhl, sexp = _prepare(X, dev)
                self.kmeans_inertia_ = torch.zeros((len(Ks), H), dtype=torch.float32, device=dev)
                bk.run(Xd, xnorm, X.shape[1], idx_d, n, H, m, h0, h1, labels, weight_dtype=wdtype,
                       inertia=self.kmeans_inertia_, n_iter=self.kmeans_n_iter_, Xhl=Xhl,
                       scale_exp=sexp)
            self.kmeans_stats_ = bk.stats
        elif Ks:
            if isinstance(X, torch.Tensor):
                X = X.cpu().numpy()
            if idx is None:
                idx = idx_d.cpu().numpy()
            for k, K in enumerate(Ks):
                self._K = K
                self._set_clusterer_K()
                lab = host_fit_predict(self.clusterer, X, idx[h0:h1], self.n_jobs,
                                       self.parallelization_method)
                if lab.size and (lab.min() < 0 or lab.max() >= K):
                    raise ValueError(f"clusterer labels must lie in [0, {K})")
                engine.scatter_labels(idx_d[h0:h1].contiguous(), torch.from_numpy(lab).to(dev), n,
                                      labels[k], h_offset=h0)
        dist.merge_labels(labels, H)
        torch.cuda.synchronize(dev)
        t_cl = time.perf_counter()

        # co-sampling, co-association and histogram over this rank's band of tiles
        nt = engine.num_tiles(n)
        t0, t1 = dist.shard(nt, rank, W)
        I_tiles, I_full = engine.cosample(labels[0], n, Hpad, t0, t1, want_full=keep)
        counts = torch.zeros((len(Ks), post.N_BINS), dtype=torch.int64, device=dev)
        M_full = [None] * len(Ks)
        if keep:
            M_full = [torch.zeros((n, n), dtype=torch.int32, device=dev) for _ in Ks]
        engine.coassoc_all(labels, n, Hpad, Ks, t0, t1, I_tiles, counts, M_full if keep else None,
                           streams=int(os.environ.get("CCMI_CO_STREAMS", 3)))
        dist.sum_counts(counts)
        if keep:
            dist.sum_counts(I_full)
            for M in M_full:
                dist.sum_counts(M)
        counts_h = counts.cpu().numpy()
        t_co = time.perf_counter()

        # host post-processing (CC.py:316-387)
        iij = I_full.cpu().numpy().astype(self._dtype) if keep else None
        for k, K in enumerate(Ks):
            hist, cdf, bin_edges, pac_area = post.cdf_from_counts(
                post.pair_counts_to_hist_counts(counts_h[k], n), self.PAC_interval)
            res = dict(consensus_labels=[], hist=hist, cdf=cdf, bin_edges=bin_edges,
                       pac_area=pac_area)
            if keep:
                res['mij'] = M_full[k].cpu().numpy().astype(self._dtype)
                res['iij'] = iij
                res['cij'] = engine.consensus(M_full[k], I_full).cpu().numpy()
            else:
                res['mij'] = res['iij'] = res['cij'] = None
            self.cdf_at_K_data[K] = res
        self.pair_counts_ = {K: counts_h[k] for k, K in enumerate(Ks)}
        self._idx_host, self._idx_dev = idx, idx_d  # rows [h0, h1) of this rank (all at W = 1)
        self.resample_range_ = (h0, h1)
        self.labels_ = labels  # device uint8 [nK, n, Hpad]; 0xFF = not sampled
        self._finish_selection()
        self.timings_ = dict(resample=t_rs - t_start, cluster=t_cl - t_rs,
                             coassoc=t_co - t_cl, post=time.perf_counter() - t_co,
                             total=time.perf_counter() - t_start)
        if self.plot_cdf and rank == 0:
            self._plot_cdf()
        return self

    def _check_k_range(self, Ks):
        """Every K of K_range must be an integer in [1, 127] (the uint8 label format and the
        int8 co-association), checked before any clustering runs."""
        for K in Ks:
            if K < 1 or K > KMAX:
                raise ValueError(f"K_range values must lie in [1, {KMAX}], got {K}")

    def _finish_selection(self):
        d = self.cdf_at_K_data
        self.pac_area_ = {K: float(v['pac_area']) for K, v in d.items()}
        self.cdf_area_ = {K: post.cdf_area(v['cdf'], v['bin_edges']) for K, v in d.items()}
        self.delta_k_ = post.delta_k(self.cdf_area_)
        self.best_k_ = post.best_k(self.pac_area_)

    # ------------------------------------------------------------------ extras
    def _device_counts(self, K):
        """int32 M and I (n x n, on the GPU) of one K, recomputed from the fitted label
        matrix (CC.py:264 and :287-290) when the fit did not keep them."""
        if getattr(self, 'labels_', None) is None:
            raise ValueError("fit() first")
        Ks = list(self.cdf_at_K_data)
        k = Ks.index(K)
        n = self._N
        labels = self.labels_
        Hpad = labels.shape[2]
        nt = engine.num_tiles(n)
        I_tiles, I_full = engine.cosample(labels[0], n, Hpad, 0, nt, want_full=True)
        counts = torch.zeros(post.N_BINS, dtype=torch.int64, device=labels.device)
        M = torch.zeros((n, n), dtype=torch.int32, device=labels.device)
        engine.coassoc(labels[k], n, Hpad, K, 0, nt, I_tiles, engine.edges_device(labels.device),
                       counts, M)
        return M, I_full

    def _consensus_device(self, K):
        """float32 C for one K on the device (the kept cij when the fit kept its matrices)."""
        v = self.cdf_at_K_data[K]
        if v.get('cij') is not None:
            return torch.from_numpy(np.ascontiguousarray(v['cij'])).to(self.labels_.device)
        M, I = self._device_counts(K)
        C = engine.consensus(M, I)
        del M, I
        return C

    def consensus_matrix(self, K):
        """float32 C for one K (CC.py:372-373), recomputed on the GPU when not kept."""
        v = self.cdf_at_K_data[K]
        if v.get('cij') is not None:
            return v['cij']
        M, I = self._device_counts(K)
        return engine.consensus(M, I).cpu().numpy()

    def export_memmap(self, folder=None, Ks=None):
        """Write each K's co-association counts as the reference's process-mode file
        (CC.py:147-159): ``<folder>/_temp_{K}``, a raw C-order n x n array of the count dtype
        (uint8 if n_iterations < 256 else uint16), readable with
        ``np.memmap(path, dtype, mode='r', shape=(n, n))``.  Returns {K: path}."""
        import os

        folder = self.memmap_folder if folder is None else folder
        os.makedirs(folder, exist_ok=True)
        out = {}
        for K in (self.cdf_at_K_data if Ks is None else Ks):
            mij = self.cdf_at_K_data[K].get('mij')
            if mij is None:
                mij = self._device_counts(K)[0].cpu().numpy().astype(self._dtype)
            path = os.path.join(folder, f'_temp_{K}')
            mm = np.memmap(path, dtype=self._dtype, shape=(self._N, self._N), mode='w+')
            mm[:] = mij
            mm.flush()
            del mm
            out[K] = path
        return out

    def predict(self, K=None, distance='manhattan'):
        """Consensus labels for K (default ``best_k_``).

        distance='manhattan' (default) is the reference's intended semantics
        (`_get_consensus_labels`, CC.py:292-314): agglomerative clustering with
        ``agg_clustering_linkage`` of the ROWS of C under the manhattan metric
        (``AgglomerativeClustering(n_clusters=K, linkage=..., affinity='manhattan')``, CC.py:306-312;
        sklearn >= 1.4 spells the keyword ``metric``).  Everything runs on the GPU: C from the
        label matrix (cc_coassoc, cc_consensus), the n x n manhattan distances in float64 with
        scipy's summation order (cc_manhattan, bit-identical to
        ``scipy.spatial.distance.pdist(C, 'cityblock')``), and for 'average', 'complete' and
        'weighted' linkage scipy's nn_chain (cc_linkage_nnchain), whose merges the host sorts,
        relabels and cuts as scipy's linkage() and sklearn's ``_hc_cut`` do; for 'single' linkage
        sklearn's own mst_linkage_core (Prim, cc_linkage_mst), sorted and labelled as sklearn's
        linkage_tree does.  n is bounded by HBM (C, then 8 n^2 bytes of distances: 20 GB at
        n = 50 000).

        distance='1-C' is an opt-in variant: the same linkage over 1 - C as a precomputed
        consensus distance.
        """
        K = self.best_k_ if K is None else K
        n = self._N
        link = self.agg_clustering_linkage
        # sklearn's checks (AgglomerativeClustering's parameter validation, check_array's minimum
        # of 2 samples, _hc_cut), raised before any device work
        if isinstance(K, bool) or not isinstance(K, (int, np.integer)) or K < 1:
            raise ValueError("The 'n_clusters' parameter of AgglomerativeClustering must be an int "
                             f"in the range [1, inf) or None. Got {K!r} instead.")
        if n < 2:
            raise ValueError(f"Found array with {n} sample(s) (shape=({n}, {n})) while a minimum of "
                             "2 is required by AgglomerativeClustering.")
        if K > n:
            raise ValueError("Cannot extract more clusters than samples: "
                             f"{K} clusters were given for a tree with {n} leaves.")
        if K not in self.cdf_at_K_data:
            raise KeyError(f"K = {K} is not in K_range of the fit")
        if link == 'ward':
            raise ValueError("ward linkage needs the euclidean metric; the reference's manhattan "
                             "consensus linkage supports 'average', 'complete' and 'single'")
        if distance not in ('manhattan', '1-C'):
            raise ValueError("distance must be 'manhattan' or '1-C'")
        if link in engine.LINKAGE_METHODS or link == 'single':
            C = self._consensus_device(K)
            if distance == 'manhattan':
                D = engine.manhattan(C)
            else:
                D = 1.0 - C.double()
            del C
            Z = engine.linkage_single(D) if link == 'single' else engine.linkage(D, link)
            del D
            return post.hc_cut(K, Z[:, :2].astype(np.int64), n)
        raise ValueError(f"unknown linkage {link!r}: 'average', 'complete', 'weighted' or 'single'")

    @property
    def resampling_indices_(self):
        """int32 [H, m] host copy of the resample indices (rows [h0, h1) of this rank; copied
        from the device on first access when they were drawn there)."""
        if getattr(self, '_idx_host', None) is None and getattr(self, '_idx_dev', None) is not None:
            self._idx_host = self._idx_dev.cpu().numpy()
        return getattr(self, '_idx_host', None)

    def _plot_cdf(self, ax=None):
        """Consensus CDF per K as a step curve over the bin upper edges, with the PAC interval
        shaded (the ``plot_cdf`` option of CC.py:133-134; presentation only, host matplotlib).
        With no ``ax`` it opens a new figure and shows it, as the reference does; pass ``ax`` to
        draw into an existing figure.  Returns the axes, or None when matplotlib is not
        installed."""
        try:
            import matplotlib.pyplot as plt
        except ImportError:  # pragma: no cover
            return None
        show = ax is None
        if show:
            ax = plt.figure().gca()
        lo, hi = self.PAC_interval
        ax.axvspan(lo, hi, color='0.9', zorder=0)
        for K, res in self.cdf_at_K_data.items():
            upper = np.asarray(res['bin_edges'][1:], dtype=np.float64)
            ax.step(upper, res['cdf'], where='post', label=f'K={K} (PAC {float(res["pac_area"]):.3f})')
        ax.set_xlim(0.0, 1.0)
        ax.set_ylim(0.0, 1.02)
        ax.set_xlabel('consensus value')
        ax.set_ylabel('fraction of pairs <= value')
        ax.legend(fontsize='small')
        if show:
            plt.show()
        return ax


def _clone(clusterer):
    """An independent copy of a plugin clusterer with the same parameters: sklearn's ``clone``
    for estimators (get_params), else a deep copy."""
    if hasattr(clusterer, 'get_params'):
        try:
            from sklearn.base import clone

            return clone(clusterer)
        except Exception:  # not a clonable sklearn estimator
            pass
    import copy

    return copy.deepcopy(clusterer)


def _fit_predict_one(clusterer, Xs):
    return fit_predict_one(clusterer, Xs)


def host_fit_predict(clusterer, X, idx, n_jobs=1, parallelization_method='multithreading'):
    """int32 labels [len(idx), m] of ``clusterer.fit_predict(X[idx[h]])`` for every resample h
    (CC.py:282), the hybrid path's host stage for a clusterer the GPU k-means does not replace.

    n_jobs == 1: one call after the other on the clusterer itself (CC.py:180-183).  Otherwise the
    resamples fan out over joblib workers as CC.py:185-195 does: threads for
    'multithreading', processes for 'multiprocessing' (n_jobs=-1: all cores).  Labels are
    RETURNED, not accumulated into a shared matrix, so the workers cannot race (the reference adds
    into one shared Mij from every worker); under threads each task fits its own copy of the
    clusterer (the reference shares one, whose fit_predict can return another thread's labels).
    A process task carries a contiguous chunk of resamples (about four chunks per worker), and
    its function lives in a module that does not import torch (_hostfit), so a worker starts
    with sklearn alone.

    'multithreading' runs a picklable clusterer on the same process pool: a host fit is GIL-bound
    numpy glue for most foreign clusterers (GaussianMixture's EM measured 1.8x SLOWER on 16
    joblib threads than serially, profiles/r04/rec_r4ai/gmm_time.txt), and the labels do not
    depend on where a fit runs.  A clusterer that cannot be pickled stays on threads, each task
    fitting its own clone.  The labels do not depend on n_jobs or the method as long as the
    clusterer's randomness comes from its random_state, which _set_clusterer_K sets to the int
    seed (CC.py:212) before every K."""
    H = len(idx)
    if H == 0:
        m = idx.shape[1] if getattr(idx, 'ndim', 1) == 2 else 0
        return np.empty((0, m), dtype=np.int32)
    if n_jobs == 1:
        return np.stack([_fit_predict_one(clusterer, X[i]) for i in idx]).astype(np.int32)
    from joblib import Parallel, delayed, effective_n_jobs, parallel_config

    if parallelization_method not in ('multithreading', 'multiprocessing'):
        raise RuntimeError(f'unknown parallelization method: {parallelization_method}')
    if parallelization_method == 'multithreading' and not _picklable(clusterer):
        out = Parallel(n_jobs=n_jobs, prefer='threads')(
            delayed(fit_predict_one)(_clone(clusterer), X[i]) for i in idx)
    else:
        chunks = max(1, min(H, 4 * effective_n_jobs(n_jobs)))
        bounds = np.linspace(0, H, chunks + 1).astype(int)
        # one BLAS thread per worker: loky would give each worker cpu_count // n_jobs threads,
        # and cpu_count is the whole machine's on a shared node (16 workers x 16 threads on a
        # 16-CPU share measured 7x slower than the serial loop)
        with parallel_config(backend='loky', inner_max_num_threads=1):
            parts = Parallel(n_jobs=n_jobs)(
                delayed(fit_predict_chunk)(clusterer, [X[i] for i in idx[a:b]])
                for a, b in zip(bounds[:-1], bounds[1:]) if b > a)
        out = [lab for part in parts for lab in part]
    return np.stack(out).astype(np.int32)


def _picklable(obj):
    import pickle

    try:
        pickle.dumps(obj)
        return True
    except Exception:
        return False


def _prepare(X, dev):
    from .kmeans import prepare_rows

    if not isinstance(X, torch.Tensor) and X.dtype.kind != 'f':
        X = np.asarray(X, dtype=np.float64)
    return prepare_rows(X, dev)
