"""sklearn-side parity fixtures for the float32-class and float64 k-means tests, generated ONCE in
the development container so that the GPU tests classify the engine's labels against committed
data instead of re-running sklearn on whatever CPU the GPU box has.

The reference's clusterer call is ``KMeans(n_clusters=K).set_params(random_state=seed,
n_init=3).fit_predict(X[idx[h]])`` (CC.py:88-90, :201-214, :282) with
``idx[h] = RandomState(seed + h).choice(n, int(0.8 n), replace=False)`` (CC.py:216-241).  Every
fit here is that call, on one BLAS/OpenMP thread (deterministic; sklearn's Lloyd reduces the
per-thread centre sums in scheduling order when threaded).  For the small cases (n <= 5000,
d <= 3000) the reference itself is also run with the recording clusterer of make_golden.py and
its recorded labels must equal these fits (the call is the same; checked, not assumed).

Three kinds of fixture under tests/golden/sk/:

* ``<case>.npz`` (kind "classify"): for the problems a test checks with tests/sk_parity.py,
  sklearn's float32 labels (``ref32``), and for each problem the rounding-sensitivity evidence
  sklearn itself gives: its float64 fit, eight 2^-22 nudges of the inputs, the same fit on 8
  threads and on copies at four buffer alignments, sklearn's algorithm at the engine's operand
  precision (sk_parity.kmeans_at_engine_precision, scale exponents 4 and 7; for 64 < d <= 128
  also with the d = 128 engine's sparse M-step), and sklearn's fit opened up
  (sk_parity.sklearn_inits: the same Cython Lloyd step by step): its other inits whose
  partition inertia is within NEIGHBOUR_MAX_DSS of the chosen one's, and the near-tie
  assignments along every init's float32 trajectory.  Each perturbation whose labels differ
  from ref32 sets a reason bit and its labels are kept as a "variant" (digest, labels, ARI and
  relative partition inertia to ref32); a near tie sets its own bit.  Problems checked for
  identity only store a label digest.
* ``f64_c3shape.npz`` (kind "f64"): sklearn float64 label digests, n_iter and inertia at the C3
  shape (n = 50 000, m = 40 000, d = 128, K = 2..20, 2 resamples) for cc_kmeans_f64.
* ``pac_<case>.npz`` (kind "pac"): sklearn float32 (and float64) labels of every (K, h) at H resamples, pushed
  through the reference's co-association and histogram (CC.py:284-290, :338-344, numpy on row
  blocks, the same per-element C = float32(M) / float32(I + 1e-6) and numpy.histogram binning,
  counts summed over blocks) -> the 20 strict-upper pair counts per K, plus every label
  vector's digest.  The float64 fits' counts, and those of PAC_NUDGES float32 runs on
  2^-22-nudged inputs (``pair_counts_nudge``), give the reference's own PAC spread under
  rounding, against which the engine's |dPAC| is bounded (``digest_nudge``: their label
  digests).  PAC_NUDGES_ONLY=1 adds the nudged runs to existing PAC fixtures.

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_sk_fixtures.py [case ...]
"""
from __future__ import annotations

import hashlib
import json
import os
import sys
import time
from concurrent.futures import ProcessPoolExecutor

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
OUT = os.path.join(HERE, "sk")
sys.path.insert(0, ROOT)
sys.path.insert(0, HERE)

# reason bits (tests/sk_parity.py reads the same values)
F32_F64, NUDGE, THREADS, ALIGN, ENGINE, ENGINE_SPARSE, NEAR_TIE, OTHER_INIT = 1, 2, 4, 8, 16, 32, 64, 128
NUDGE_DRAWS = 8  # random-sign 2^-22 relative nudges of the inputs per problem


def digest(a) -> str:
    a = np.ascontiguousarray(a)
    return hashlib.sha256(a.view(np.uint8).tobytes() + str(a.dtype).encode() + str(a.shape).encode()).hexdigest()


def _blobs(n, d, k, seed, std=1.0, dtype=np.float32):
    from sklearn.datasets import make_blobs

    X, _ = make_blobs(n_samples=n, n_features=d, centers=k, cluster_std=std,
                      center_box=(-10, 10), shuffle=True, random_state=seed)
    return X.astype(dtype)


def _expr(n, d, seed, groups=5):
    from bench import make_expression_f32

    return make_expression_f32(n, d, groups=groups, seed=seed)


# Each case mirrors one GPU test's data exactly (the test asserts the X digest):
#   X(), Ks, seed, frac, classify = resamples checked with sk_parity, ref = identity-only resamples
CASES = {
    # tests/test_gpu_kmeans.py::test_labels_match_sklearn (blobs(n, d, k_true, seed=n), seed 7, H)
    "lab_n1500_d16": dict(X=lambda: _blobs(1500, 16, 5, 1500), Ks=[2, 3, 4, 5, 6, 8], seed=7, classify=range(6)),
    "lab_n2000_d64": dict(X=lambda: _blobs(2000, 64, 4, 2000), Ks=[2, 3, 4, 7], seed=7, classify=range(5)),
    "lab_n1200_d128": dict(X=lambda: _blobs(1200, 128, 6, 1200), Ks=[3, 6, 10], seed=7, classify=range(4)),
    "lab_n29_d29": dict(X=lambda: _blobs(29, 29, 3, 29), Ks=[2, 3, 5], seed=7, classify=range(5)),
    "lab_n1200_d300": dict(X=lambda: _blobs(1200, 300, 5, 1200), Ks=[2, 3, 5, 8], seed=7, classify=range(4)),
    "lab_n700_d2000": dict(X=lambda: _blobs(700, 2000, 4, 700), Ks=[2, 4, 6], seed=7, classify=range(3)),
    # tests/test_gpu_kmeans.py::test_wide_expression_like
    "expr_n1000_d3000": dict(X=lambda: _expr(1000, 3000, 3), Ks=[2, 3, 5, 7], seed=0, classify=range(3)),
    # tests/test_gpu_kmeans.py::test_sparse_mstep_against_dense (C3-shaped rows, 8 blobs)
    "sparse_n4000_d128": dict(X=lambda: _blobs(4000, 128, 8, 11), Ks=list(range(2, 15)), seed=3,
                              classify=range(4)),
    # tests/test_gpu_scale.py full-size configs (bench.make_blobs_f32 / make_expression_f32, SEED 0)
    "c3_full": dict(X=lambda: _blobs(50_000, 128, 8, 0), Ks=list(range(2, 21)), seed=0, classify=[2],
                    ref=[0, 1]),
    "c2_full": dict(X=lambda: _blobs(10_000, 64, 6, 0), Ks=list(range(2, 16)), seed=0, classify=[3, 4],
                    ref=[0, 1, 2]),
    "c4_full": dict(X=lambda: _expr(5_000, 20_000, 0), Ks=list(range(2, 13)), seed=0, classify=[0]),
    # C5 (n = 200 000, m = 160 000, d = 32, K = 2..10): the d = 32 pair-mode engine at its real m
    "c5_full": dict(X=lambda: _blobs(200_000, 32, 6, 0), Ks=list(range(2, 11)), seed=0, classify=[0, 1]),
}
def _f64_noisy(n, d, k):
    """tests/test_gpu_kmeans.py::test_f64_labels_match_sklearn_float64's rows: blobs at seed n + d
    (float32, then float64) plus N(0, 0.5^2) noise from default_rng(0)."""
    X = _blobs(n, d, k, n + d).astype(np.float64)
    X += np.random.default_rng(0).normal(scale=0.5, size=X.shape)
    return X


# tests/test_gpu_kmeans.py::test_f64_labels_match_sklearn_float64 (seed 3): sklearn float64 label
# digests, n_iter and inertia of every (K, h)
F64_SMALL = {
    "f64_n29_d29": dict(X=lambda: _f64_noisy(29, 29, 3), Ks=[2, 3, 4, 5, 6, 7, 8, 9, 10], seed=3, H=6),
    "f64_n600_d12": dict(X=lambda: _f64_noisy(600, 12, 4), Ks=[2, 3, 4, 6, 9], seed=3, H=4),
    "f64_n300_d150": dict(X=lambda: _f64_noisy(300, 150, 3), Ks=[2, 3, 5], seed=3, H=3),
}
F64_CASE = dict(X=lambda: _blobs(50_000, 128, 8, 5, dtype=np.float64), Ks=list(range(2, 21)), seed=0, H=2)
PAC_CASES = {
    # tests/test_gpu_parity_blobs.py: C2 shape at H = 50, C3 shape at H = 16
    "pac_c2_h50": dict(X=lambda: _blobs(10_000, 64, 6, 0), Ks=list(range(2, 16)), seed=0, H=50),
    "pac_c3_h16": dict(X=lambda: _blobs(50_000, 128, 8, 0), Ks=list(range(2, 21)), seed=0, H=16),
}

_X = {}


def indices(n, seed, h, frac=0.8):
    return np.random.RandomState(seed + h).choice(n, size=int(frac * n), replace=False)


def _fit(rows, K, seed, threads=1):
    from sklearn.cluster import KMeans
    from threadpoolctl import threadpool_limits

    with threadpool_limits(threads):
        km = KMeans(n_clusters=K, random_state=seed, n_init=3).fit(rows)
    return km.labels_.astype(np.int8), int(km.n_iter_), float(km.inertia_)


def _classify_task(args):
    """ref32 of one (K, h) and every perturbation sklearn offers (sk_parity's reasons)."""
    from tests.sk_parity import aligned_copy, kmeans_at_engine_precision
    from threadpoolctl import threadpool_limits

    case, K, h = args
    X, seed = _X[case], CASES[case]["seed"]
    rows = X[indices(X.shape[0], seed, h)]
    t0 = time.time()
    ref32 = _fit(rows, K, seed)[0]
    variants = []  # (reason bit, labels)

    def note(bit, lab):
        if not np.array_equal(lab, ref32):
            variants.append((bit, np.asarray(lab, dtype=np.int8)))

    note(F32_F64, _fit(rows.astype(np.float64), K, seed)[0])
    for draw in range(NUDGE_DRAWS):
        rng = np.random.default_rng(1000 * K + h + 7919 * draw)
        sign = np.where(rng.random(rows.shape) < 0.5, 1.0, -1.0)
        note(NUDGE, _fit((rows.astype(np.float64) * (1.0 + sign * 2.0 ** -22)).astype(np.float32), K, seed)[0])
    note(THREADS, _fit(rows, K, seed, threads=8)[0])
    for off in (4, 8, 16, 32):
        note(ALIGN, _fit(aligned_copy(rows, off), K, seed)[0])
    with threadpool_limits(1):
        for sx in (4, 7):
            note(ENGINE, kmeans_at_engine_precision(rows, K, seed, 3, s=sx).astype(np.int8))
        if 64 < rows.shape[1] <= 128:  # the d = 128 engine's sparse M-step (kmeans.hip kSparse)
            for sx in (4, 7):
                note(ENGINE_SPARSE, kmeans_at_engine_precision(rows, K, seed, 3, s=sx, sparse=True).astype(np.int8))
    # sklearn's fit opened up (tests/sk_parity.py sklearn_inits): its per-init results and the
    # near-tie assignments along each init's float32 trajectory.  A near tie (a row whose two
    # nearest centres are closer than float32's distance error) is a rounding-decided label
    # of sklearn's own run; another init whose fixed point is within NEIGHBOUR_MAX_DSS of the
    # chosen one's partition inertia is the labelling best-of-n_init picks when that rounding
    # moves the chosen init's fixed point.
    from tests.sk_parity import NEIGHBOUR_MAX_DSS, partition_ss, sklearn_inits

    init_labels, _, ties, best = sklearn_inits(rows, K, seed)
    assert np.array_equal(best, ref32), (case, K, h, "opened-up sklearn != KMeans.fit")
    near_tie = int(ties.sum())
    ss0 = partition_ss(rows, ref32.astype(np.int64), K)
    from sklearn.cluster._k_means_common import _is_same_clustering

    for lab in init_labels:
        if _is_same_clustering(lab.astype(np.int32), ref32.astype(np.int32), K):
            continue  # the chosen partition itself (labels permuted): no new evidence
        if abs(partition_ss(rows, lab.astype(np.int64), K) - ss0) <= NEIGHBOUR_MAX_DSS * ss0:
            note(OTHER_INIT, lab)
    # unique variants, reason bits OR-ed
    uniq = []
    for bit, lab in variants:
        for u in uniq:
            if np.array_equal(u[1], lab):
                u[0] |= bit
                break
        else:
            uniq.append([bit, lab])
    reasons = NEAR_TIE if near_tie else 0
    for bit, _ in uniq:
        reasons |= bit
    # sklearn's own spread: each variant's adjusted Rand index to ref32 and its relative partition
    # inertia difference (tests/sk_parity.py bounds a neighbour by these)
    from sklearn.metrics import adjusted_rand_score
    from tests.sk_parity import partition_ss

    ss_ref = partition_ss(rows, ref32.astype(np.int64), K)
    for u in uniq:
        lab = u[1].astype(np.int64)
        u.append(float(adjusted_rand_score(ref32.astype(np.int64), lab)))
        u.append(float((partition_ss(rows, lab, K) - ss_ref) / ss_ref))
    print(f"  {case} K={K} h={h}: reasons={reasons} variants={len(uniq)} near_ties={near_tie} "
          f"ari_min={min([u[2] for u in uniq], default=1.0):.4f} ({time.time() - t0:.1f} s)", flush=True)
    return case, K, h, ref32, reasons, uniq


def _ref_task(args):
    case, K, h, dt = args
    X = _X[case]
    spec = CASES.get(case) or PAC_CASES.get(case) or F64_SMALL.get(case) or F64_CASE
    rows = X[indices(X.shape[0], spec["seed"], h)]
    lab, nit, inert = _fit(rows.astype(dt), K, spec["seed"])
    return case, K, h, lab, nit, inert


def _pair_counts_task(args):
    """Strict-upper pair counts of one K from labels [H, m] (CC.py:284-290, :338-344)."""
    case, K, labs = args
    X = _X[case]
    spec = PAC_CASES[case]
    n, H = X.shape[0], spec["H"]
    idx = np.stack([indices(n, spec["seed"], h) for h in range(H)])
    dt = np.uint8 if H < 256 else np.uint16  # CC.py:107
    O = np.zeros((n, H * K), dtype=np.float32)
    S = np.zeros((n, H), dtype=np.float32)
    for h in range(H):
        O[idx[h], h * K + labs[h].astype(np.int64)] = 1.0
        S[idx[h], h] = 1.0
    counts = np.zeros(20, dtype=np.int64)
    B = 1024
    for r0 in range(0, n, B):
        r1 = min(n, r0 + B)
        M = np.rint(O[r0:r1] @ O[r0:].T).astype(dt)
        I = np.rint(S[r0:r1] @ S[r0:].T).astype(dt)
        C = np.divide(M, I + 1e-6, dtype=np.float32)  # CC.py:372
        # strict upper pairs: column j (absolute r0 + c) > row i (absolute r0 + r)
        keep = np.arange(r0, n)[None, :] > np.arange(r0, r1)[:, None]
        counts += np.histogram(C[keep], bins=20, range=(0, 1))[0]
    return K, counts


def _reference_check(case, ref):
    """The reference run with make_golden's recording clusterer records the same labels."""
    from make_golden import kmeans_factory, run_reference

    spec = CASES[case]
    X = _X[case]
    hmax = max(list(spec["classify"]) + list(spec.get("ref", []))) + 1
    _, idx, rec = run_reference(X, spec["Ks"], hmax, 0.8, spec["seed"], kmeans_factory)
    for j, K in enumerate(spec["Ks"]):
        for h in range(hmax):
            k_rec, lab = rec.log[j * hmax + h]
            assert k_rec == K
            assert np.array_equal(idx[h], indices(X.shape[0], spec["seed"], h))
            if (K, h) in ref:
                assert np.array_equal(lab.astype(np.int8), ref[(K, h)]), (case, K, h)
    print(f"  {case}: the reference's recorded labels equal the direct fits", flush=True)


def make_classify(case, ex):
    spec = CASES[case]
    X = _X[case]
    Ks, hs, rhs = spec["Ks"], list(spec["classify"]), list(spec.get("ref", []))
    t0 = time.time()
    res = list(ex.map(_classify_task, [(case, K, h) for K in Ks for h in hs]))
    refs = list(ex.map(_ref_task, [(case, K, h, np.float32) for K in Ks for h in rhs]))
    m = int(0.8 * X.shape[0])
    ref32 = np.zeros((len(Ks), len(hs), m), dtype=np.int8)
    reasons = np.zeros((len(Ks), len(hs)), dtype=np.int32)
    var_dig, var_owner, var_bits, var_ari, var_dss, var_lab = [], [], [], [], [], []
    by = {}
    for (_, K, h, r32, rs, uniq) in res:
        k, c = Ks.index(K), hs.index(h)
        ref32[k, c] = r32
        reasons[k, c] = rs
        by[(K, h)] = r32
        for bit, lab, ari, dss in uniq:
            var_dig.append(digest(lab))
            var_owner.append((k, c))
            var_bits.append(bit)
            var_ari.append(ari)
            var_dss.append(dss)
            var_lab.append(np.asarray(lab, dtype=np.int8))
    ref_digest = np.full((len(Ks), max(1, len(rhs))), "", dtype="U64")
    for (_, K, h, lab, _, _) in refs:
        ref_digest[Ks.index(K), rhs.index(h)] = digest(lab)
        by[(K, h)] = lab
    if X.shape[0] <= 5000 and X.shape[1] <= 3000:
        _reference_check(case, by)
    import sklearn

    meta = dict(kind="classify", case=case, n=X.shape[0], d=X.shape[1], Ks=Ks, seed=spec["seed"], frac=0.8,
                classify=hs, ref=rhs, x_sha256=digest(X), sklearn=sklearn.__version__, numpy=np.__version__,
                threads=1, nudge_draws=NUDGE_DRAWS, reason_bits=dict(f32_f64=F32_F64, nudge=NUDGE, threads=THREADS, align=ALIGN,
                                            engine=ENGINE, engine_sparse=ENGINE_SPARSE, near_tie=NEAR_TIE,
                                            other_init=OTHER_INIT))
    np.savez_compressed(os.path.join(OUT, f"{case}.npz"), ref32=ref32, reasons=reasons,
                        var_digest=np.array(var_dig, dtype="U64"),
                        var_owner=np.array(var_owner, dtype=np.int32).reshape(-1, 2),
                        var_bits=np.array(var_bits, dtype=np.int32), ref_digest=ref_digest,
                        var_ari=np.array(var_ari, dtype=np.float64), var_dss=np.array(var_dss, dtype=np.float64),
                        var_labels=(np.stack(var_lab) if var_lab else np.zeros((0, m), dtype=np.int8)),
                        meta=np.array(json.dumps(meta)))
    print(f"{case}: {len(res)} classified, {len(refs)} identity-only, {len(var_dig)} variants, "
          f"sensitive {int((reasons > 0).sum())} ({time.time() - t0:.0f} s)", flush=True)


def make_f64(ex, case="f64_c3shape"):
    spec = F64_SMALL.get(case, F64_CASE)
    X = _X[case]
    Ks, H = spec["Ks"], spec["H"]
    t0 = time.time()
    res = list(ex.map(_ref_task, [(case, K, h, np.float64) for K in Ks for h in range(H)]))
    dig = np.full((len(Ks), H), "", dtype="U64")
    nit = np.zeros((len(Ks), H), dtype=np.int32)
    inert = np.zeros((len(Ks), H), dtype=np.float64)
    for (_, K, h, lab, it, ine) in res:
        k = Ks.index(K)
        dig[k, h], nit[k, h], inert[k, h] = digest(lab), it, ine
    note = ("make_blobs(50000, 128, 8 centers, std 1, box (-10, 10), seed 5) float64"
            if case == "f64_c3shape" else "tests/test_gpu_kmeans.py blobs + N(0, 0.5^2) noise")
    meta = dict(kind="f64", case=case, n=X.shape[0], d=X.shape[1], Ks=Ks, seed=spec["seed"], frac=0.8,
                H=H, x_sha256=digest(X), note=note + "; sklearn KMeans(n_init=3) float64, 1 thread")
    np.savez_compressed(os.path.join(OUT, f"{case}.npz"), digest64=dig, n_iter=nit, inertia=inert,
                        meta=np.array(json.dumps(meta)))
    print(f"{case}: {len(res)} fits ({time.time() - t0:.0f} s); n_iter {nit.min()}..{nit.max()}", flush=True)


PAC_NUDGES = 2  # extra reference runs per PAC case: the float32 fit on 2^-22-nudged inputs


def _nudge_task(args):
    """sklearn's float32 fit of one (K, h) on rows nudged by a random-sign 2^-22 relative step
    (draw v), the rounding perturbation sk_parity's per-problem cloud uses."""
    case, K, h, v = args
    X = _X[case]
    spec = PAC_CASES[case]
    rows = X[indices(X.shape[0], spec["seed"], h)]
    sign = np.random.default_rng([v, K, h]).choice(np.array([-1.0, 1.0]), size=rows.shape)
    lab = _fit((rows.astype(np.float64) * (1.0 + sign * 2.0 ** -22)).astype(np.float32), K, spec["seed"])[0]
    return K, h, lab


def add_pac_nudges(case, ex):
    """Add pair_counts_nudge [PAC_NUDGES, nK, 20] to an existing PAC fixture: the reference's
    PAC under input rounding, next to its float64 run, for the engine's |dPAC| bound."""
    path = os.path.join(OUT, f"{case}.npz")
    with np.load(path, allow_pickle=False) as z:
        old = {k: z[k] for k in z.files}
    spec = PAC_CASES[case]
    Ks, H = spec["Ks"], spec["H"]
    n, m = _X[case].shape[0], int(0.8 * _X[case].shape[0])
    t0 = time.time()
    out = np.zeros((PAC_NUDGES, len(Ks), 20), dtype=np.int64)
    dig = np.full((PAC_NUDGES, len(Ks), H), "", dtype="U64")
    for v in range(PAC_NUDGES):
        labs = {K: np.zeros((H, m), dtype=np.int8) for K in Ks}
        for K, h, lab in ex.map(_nudge_task, [(case, K, h, v) for K in Ks for h in range(H)]):
            labs[K][h] = lab
            dig[v, Ks.index(K), h] = digest(lab)
        for K, c in ex.map(_pair_counts_task, [(case, K, labs[K]) for K in Ks]):
            out[v, Ks.index(K)] = c
        assert np.all(out[v].sum(axis=1) == n * (n - 1) // 2)
        print(f"  {case}: nudge draw {v} ({time.time() - t0:.0f} s)", flush=True)
    meta = json.loads(str(old["meta"]))
    meta["nudge_draws"] = PAC_NUDGES
    old["meta"] = np.array(json.dumps(meta))
    old["pair_counts_nudge"] = out
    old["digest_nudge"] = dig
    np.savez_compressed(path, **old)


def make_pac(case, ex):
    spec = PAC_CASES[case]
    X = _X[case]
    Ks, H = spec["Ks"], spec["H"]
    t0 = time.time()
    m = int(0.8 * X.shape[0])
    n = X.shape[0]
    out = {}
    for dt, tag in ((np.float32, "32"), (np.float64, "64")):
        res = list(ex.map(_ref_task, [(case, K, h, dt) for K in Ks for h in range(H)]))
        labs = {K: np.zeros((H, m), dtype=np.int8) for K in Ks}
        dig = np.full((len(Ks), H), "", dtype="U64")
        for (_, K, h, lab, _, _) in res:
            labs[K][h] = lab
            dig[Ks.index(K), h] = digest(lab)
        print(f"  {case}: {len(res)} sklearn float{tag} fits ({time.time() - t0:.0f} s)", flush=True)
        counts = np.zeros((len(Ks), 20), dtype=np.int64)
        for K, c in ex.map(_pair_counts_task, [(case, K, labs[K]) for K in Ks]):
            counts[Ks.index(K)] = c
        assert np.all(counts.sum(axis=1) == n * (n - 1) // 2)
        out[tag] = (counts, dig)
    counts, dig = out["32"]
    meta = dict(kind="pac", case=case, n=n, d=X.shape[1], Ks=Ks, seed=spec["seed"], frac=0.8, H=H,
                x_sha256=digest(X), threads=1)
    np.savez_compressed(os.path.join(OUT, f"{case}.npz"), pair_counts=counts, digest32=dig,
                        pair_counts64=out["64"][0], digest64=out["64"][1], meta=np.array(json.dumps(meta)))
    print(f"{case}: pair counts of {len(Ks)} K ({time.time() - t0:.0f} s)", flush=True)


def main(argv):
    os.makedirs(OUT, exist_ok=True)
    want = argv or list(CASES) + ["f64_c3shape"] + list(F64_SMALL) + list(PAC_CASES)
    for c in want:
        spec = (CASES.get(c) or PAC_CASES.get(c) or F64_SMALL.get(c)
                or (F64_CASE if c == "f64_c3shape" else None))
        assert spec is not None, c
        _X[c] = spec["X"]()
    workers = int(os.environ.get("SK_WORKERS", "8"))
    with ProcessPoolExecutor(workers) as ex:  # fork: the workers see _X
        for c in want:
            if c in CASES:
                make_classify(c, ex)
            elif c in PAC_CASES:
                if os.environ.get("PAC_NUDGES_ONLY"):
                    add_pac_nudges(c, ex)
                else:
                    make_pac(c, ex)
                    add_pac_nudges(c, ex)
            else:
                make_f64(ex, c)


if __name__ == "__main__":
    sys.dont_write_bytecode = True
    main(sys.argv[1:])
