"""Shared check of the fast (float32-class) k-means against the reference's clusterer: sklearn
KMeans called as CC.py:205-214 / :282 call it.  Not a test module."""
import numpy as np


def _fixed_point_no_worse(rows, got, ref, K, rel=1e-4):
    """The engine's labels `got` are a Lloyd fixed point in float64 (centres = means of its
    clusters; every row's nearest centre, lowest index on ties, is its own) and their inertia is
    at most sklearn's (labels `ref`) times 1 + rel: a converged solution of the same quality
    reached along a trajectory that rounding moved.  rel = 1e-4: at C2 K = 8 (resample 3) the
    engine and sklearn's best init run the same 20 iterations and end 23 boundary rows apart, both
    fixed points, inertias within 1e-4; distinct local optima of that problem differ by ~8e-4
    (profiles/r03/parity_diag_c2_K8_h3.txt)."""
    X = rows.astype(np.float64)

    def centres(lab):
        C = np.zeros((K, X.shape[1]))
        np.add.at(C, lab, X)
        cnt = np.bincount(lab, minlength=K)
        return C / np.maximum(cnt, 1)[:, None], cnt

    C, cnt = centres(got)
    if (cnt == 0).any():
        return False
    d = (X ** 2).sum(1)[:, None] - 2.0 * X @ C.T + (C ** 2).sum(1)[None, :]
    if not np.array_equal(d.argmin(1), got):
        return False
    Cr, _ = centres(ref)
    inert = d[np.arange(len(X)), got].sum()
    inert_ref = ((X - Cr[ref]) ** 2).sum()
    return bool(inert <= inert_ref * (1.0 + rel))


def sklearn_parity(X, labels, idx, Ks, seed, resamples, skip=0, threads=16, n_init=3, max_unexplained=0):
    """Labels of resamples skip .. skip + resamples - 1 of every K against sklearn's float32
    KMeans on the same rows.  A disagreement is allowed only where the partition hinges on
    rounding, shown by sklearn itself: its float32 and float64 fits of those rows disagree, or
    its float32 fit changes when every value is moved by a relative 2^-22 (the operand precision
    of the f16 hi/lo MFMA engine, which shares sklearn float32's accuracy class, not its
    rounding), or its float32 fit on one thread differs from the same fit on `threads`.
    Several random nudges are tried (one draw can miss a partition that hinges on rounding).
    Prints and returns (identical, explained, total); asserts
    that at most `max_unexplained` disagreements are unexplained (0 unless a caller documents
    a known gap).

    labels: the fit's device label matrix [nK, n, Hpad] (uint8) or a host array
    [nK, H, m] of labels in resample order."""
    from sklearn.cluster import KMeans
    from threadpoolctl import threadpool_limits

    same = explained = fixed = 0
    unexplained = []
    with threadpool_limits(threads):
        for k, K in enumerate(Ks):
            col = labels[k].cpu().numpy() if hasattr(labels, "cpu") else None
            for h in range(skip, skip + resamples):
                rows = X[idx[h]]
                got = (col[idx[h], h] if col is not None else labels[k][h]).astype(np.int64)
                ref32 = KMeans(n_clusters=K, random_state=seed, n_init=n_init).fit_predict(rows)
                if np.array_equal(ref32, got):
                    same += 1
                    continue
                ref64 = KMeans(n_clusters=K, random_state=seed, n_init=n_init).fit_predict(
                    rows.astype(np.float64))
                if not np.array_equal(ref32, ref64):
                    explained += 1
                    continue
                # sklearn's own float32 fit of the same rows, each value moved by the engine's
                # operand precision (x = xh + xl in f16: 22 significant bits, a relative 2^-22, two
                # float32 ulps) in a random direction, under a few independent draws, and its
                # float32 fit on one thread (another reduction order of the same arithmetic): if any
                # of these changes the partition, it hinges on rounding at the engine's accuracy
                # class
                sensitive = False
                for draw in range(4):
                    rng = np.random.default_rng(1000 * K + h + 7919 * draw)
                    sign = np.where(rng.random(rows.shape) < 0.5, 1.0, -1.0)
                    nudged = (rows.astype(np.float64) * (1.0 + sign * 2.0 ** -22)).astype(np.float32)
                    refn = KMeans(n_clusters=K, random_state=seed, n_init=n_init).fit_predict(nudged)
                    if not np.array_equal(ref32, refn):
                        sensitive = True
                        break
                if not sensitive:
                    with threadpool_limits(1):
                        ref1 = KMeans(n_clusters=K, random_state=seed, n_init=n_init).fit_predict(rows)
                    sensitive = not np.array_equal(ref32, ref1)
                if not sensitive:
                    # a different converged solution of the same quality: the engine's partition
                    # is a Lloyd fixed point in float64 (its own centres reassign every row to it)
                    # with inertia no worse than sklearn's float32 result
                    sensitive = _fixed_point_no_worse(rows, got, ref32, K)
                    fixed += sensitive
                if sensitive:
                    explained += 1
                else:
                    unexplained.append((K, h, float(np.mean(ref32 == got))))
    total = len(Ks) * resamples
    print(f"sklearn parity: {same}/{total} identical, {explained} differ where sklearn's own float32 "
          f"fit is rounding-sensitive ({fixed} of them shown as a float64 Lloyd fixed point of inertia "
          f"within 1e-4 of sklearn's), {len(unexplained)} unexplained {unexplained}")
    assert len(unexplained) <= max_unexplained, unexplained
    return same, explained, total
