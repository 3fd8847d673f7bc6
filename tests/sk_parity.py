"""Shared check of the fast (float32-class) k-means against the reference's clusterer: sklearn
KMeans called as CC.py:205-214 / :282 call it.  Not a test module."""
import numpy as np


def aligned_copy(a, offset):
    """A copy of `a` whose buffer starts `offset` bytes past a 64-B boundary."""
    raw = np.empty(a.nbytes + 128, dtype=np.uint8)
    base = (-raw.ctypes.data) % 64 + offset
    out = raw[base:base + a.nbytes].view(a.dtype).reshape(a.shape)
    out[...] = a
    return out


def _dot22(X, C, s):
    """x . c at the fast engine's operand precision: x = xh + xl, c = ch + cl, f16 halves of the
    values scaled by 2^s, products xh ch + xh cl + xl ch (exact), summed per 16 features in
    float64 and accumulated across the blocks in float32 (the v_mfma_f32_32x32x16_f16 chain)."""
    def split(a):
        a = (a.astype(np.float32) * np.float32(2.0 ** s)).astype(np.float32)
        hi = a.astype(np.float16).astype(np.float64)
        return hi, (a - hi.astype(np.float32)).astype(np.float16).astype(np.float64)
    xh, xl = split(X)
    ch, cl = split(C)
    n, d = X.shape
    nb = (d + 15) // 16
    pad = nb * 16 - d

    def blocks(a):
        return np.pad(a, ((0, 0), (0, pad))).reshape(a.shape[0], nb, 16)
    xh, xl, ch, cl = blocks(xh), blocks(xl), blocks(ch), blocks(cl)
    acc = np.zeros((n, C.shape[0]), np.float32)
    if nb <= 64:  # few blocks: one matmul per block
        for k in range(nb):
            q = xh[:, k] @ ch[:, k].T + xh[:, k] @ cl[:, k].T + xl[:, k] @ ch[:, k].T
            acc = (acc + q.astype(np.float32)).astype(np.float32)
    else:  # wide rows: per-block products in float64 in batches, then the float32 chain
        for b0 in range(0, nb, 64):
            b = slice(b0, b0 + 64)
            p = (np.einsum("nbk,cbk->bnc", xh[:, b], ch[:, b]) + np.einsum("nbk,cbk->bnc", xh[:, b], cl[:, b])
                 + np.einsum("nbk,cbk->bnc", xl[:, b], ch[:, b])).astype(np.float32)
            for q in p:
                acc = (acc + q).astype(np.float32)
    return acc * np.float32(2.0 ** (-2 * s))


def kmeans_at_engine_precision(rows, K, seed, n_init=3, s=4, max_iter=300, tol=1e-4):
    """sklearn KMeans (1.7: KMeans.fit with k-means++ from sklearn's own _kmeans_plusplus and the
    same RandomState stream, _kmeans_single_lloyd, relocation, _average_centers, tol, strict
    convergence, the final E-step, best of n_init with _is_same_clustering) whose Lloyd E-step
    distances |c|^2 - 2 x.c (_dot22) and M-step sums (one-hot x the f16 halves, float32
    accumulation) are computed at the fast engine's operand precision; every other step is
    sklearn's float32 path.  Labels of the best init."""
    from sklearn.cluster._k_means_common import _is_same_clustering
    from sklearn.cluster._kmeans import _kmeans_plusplus, _tolerance
    from sklearn.utils.extmath import row_norms

    X = np.array(rows, dtype=np.float32, copy=True)
    tol_abs = _tolerance(X, tol)
    X -= X.mean(axis=0)
    xsq = row_norms(X, squared=True)
    rs = np.random.RandomState(seed)
    w = np.ones(X.shape[0], dtype=np.float32)
    Xs = X * np.float32(2.0 ** s)
    Xh = Xs.astype(np.float16).astype(np.float64)
    Xl = (Xs - Xh.astype(np.float32)).astype(np.float16).astype(np.float64)
    best = None
    for _ in range(n_init):
        centers, _ = _kmeans_plusplus(X, K, xsq, w, rs)
        centers = centers.astype(np.float32)
        labels_old = np.full(X.shape[0], -1)
        strict = False

        def msum(labels):
            # M-step sums at the engine's precision: one-hot x (xl, then xh) per 16-row block
            # (exact block sums of the 2^s-scaled halves), accumulated in float32 in row order
            acc = np.zeros((K, X.shape[1]), np.float32)
            oh = np.zeros((X.shape[0], K))
            oh[np.arange(X.shape[0]), labels] = 1.0
            for r in range(0, X.shape[0], 16):
                b = slice(r, r + 16)
                acc = (acc + (oh[b].T @ Xl[b]).astype(np.float32)).astype(np.float32)
                acc = (acc + (oh[b].T @ Xh[b]).astype(np.float32)).astype(np.float32)
            return acc * np.float32(2.0 ** -s)

        def estep(cen):
            d = (row_norms(cen, squared=True)[None, :] - np.float32(2) * _dot22(X, cen, s)).astype(np.float32)
            return d.argmin(axis=1)

        for it in range(max_iter):
            labels = estep(centers)
            cnt = np.bincount(labels, minlength=K).astype(np.float32)
            sums = msum(labels)
            empty = np.flatnonzero(cnt == 0)
            if len(empty):
                dist = ((X - centers[labels]) ** 2).sum(axis=1)
                if dist.max() > 0:
                    far = np.argpartition(dist, -len(empty))[:-len(empty) - 1:-1]
                    for e, r in zip(empty, far):
                        sums[labels[r]] -= X[r]
                        sums[e] = X[r]
                        cnt[e] = 1
                        cnt[labels[r]] -= 1
            am = int(np.argmax(cnt))
            new = np.empty_like(sums)
            for j in range(K):
                new[j] = sums[j] * np.float32(1.0 / cnt[j]) if cnt[j] > 0 else sums[am]
            shift = np.sqrt(((new - centers) ** 2).sum(axis=1, dtype=np.float32)) ** 2
            centers = new
            if np.array_equal(labels, labels_old):
                strict = True
                break
            if shift.sum() <= tol_abs:
                break
            labels_old = labels
        if not strict:
            labels = estep(centers)
        inertia = float(((X - centers[labels]) ** 2).sum(dtype=np.float64))
        if best is None or (inertia < best[0] and not _is_same_clustering(
                labels.astype(np.int32), best[1].astype(np.int32), K)):
            best = (inertia, labels)
    return best[1].astype(np.int64)


def sklearn_parity(X, labels, idx, Ks, seed, resamples, skip=0, threads=16, n_init=3, max_unexplained=0):
    """Labels of resamples skip .. skip + resamples - 1 of every K against sklearn's float32
    KMeans on the same rows.  A disagreement is allowed only where sklearn itself shows that the
    partition hinges on rounding:
      * its float32 and float64 fits of those rows disagree; or
      * its float32 fit changes when every value moves by a relative 2^-22 in a random direction
        (the operand precision of the f16 hi/lo MFMA engine, which shares sklearn float32's
        accuracy class, not its rounding), under any of four draws; or
      * its float32 fit is not reproducible: the same call on one thread, or on a copy of the
        same rows at another buffer alignment (4, 8, 16 or 32 B past 64), gives other labels
        (tests/test_parity_fixtures.py: 1-61 of 2400 labels move that way at n = 3000, K = 12);
      * sklearn's own algorithm with its Lloyd distances at the engine's operand precision
        (kmeans_at_engine_precision, two scale exponents) gives other labels than its float32
        fit: the partition hinges on rounding at the engine's accuracy class.  The emulation is
        checked to reproduce sklearn on well-posed problems (tests/test_sk_parity_host.py).
    A different local optimum that sklearn reaches from no such perturbation is unexplained.
    Prints and returns (identical, explained, total); asserts that at most `max_unexplained`
    disagreements are unexplained (0 unless a caller documents a known gap).

    labels: the fit's device label matrix [nK, n, Hpad] (uint8) or a host array
    [nK, H, m] of labels in resample order."""
    from sklearn.cluster import KMeans
    from threadpoolctl import threadpool_limits

    def fit(rows):
        return KMeans(n_clusters=K, random_state=seed, n_init=n_init).fit_predict(rows)

    same = explained = 0
    why = {"f32!=f64": 0, "nudge": 0, "irreproducible": 0, "engine-precision": 0}
    unexplained = []
    with threadpool_limits(threads):
        for k, K in enumerate(Ks):
            col = labels[k].cpu().numpy() if hasattr(labels, "cpu") else None
            for h in range(skip, skip + resamples):
                rows = X[idx[h]]
                got = (col[idx[h], h] if col is not None else labels[k][h]).astype(np.int64)
                ref32 = fit(rows)
                if np.array_equal(ref32, got):
                    same += 1
                    continue
                reason = None
                if not np.array_equal(ref32, fit(rows.astype(np.float64))):
                    reason = "f32!=f64"
                if reason is None:
                    for draw in range(4):
                        rng = np.random.default_rng(1000 * K + h + 7919 * draw)
                        sign = np.where(rng.random(rows.shape) < 0.5, 1.0, -1.0)
                        nudged = (rows.astype(np.float64) * (1.0 + sign * 2.0 ** -22)).astype(np.float32)
                        if not np.array_equal(ref32, fit(nudged)):
                            reason = "nudge"
                            break
                if reason is None:
                    with threadpool_limits(1):
                        if not np.array_equal(ref32, fit(rows)):
                            reason = "irreproducible"
                if reason is None:
                    for off in (4, 8, 16, 32):
                        if not np.array_equal(ref32, fit(aligned_copy(rows, off))):
                            reason = "irreproducible"
                            break
                if reason is None:
                    for sx in (4, 7):
                        if not np.array_equal(ref32, kmeans_at_engine_precision(rows, K, seed, n_init, s=sx)):
                            reason = "engine-precision"
                            break
                if reason is not None:
                    explained += 1
                    why[reason] += 1
                else:
                    unexplained.append((K, h, float(np.mean(ref32 == got))))
    total = len(Ks) * resamples
    print(f"sklearn parity: {same}/{total} identical, {explained} differ where sklearn's own float32 "
          f"fit is rounding-sensitive {why}, {len(unexplained)} unexplained {unexplained}")
    assert len(unexplained) <= max_unexplained, unexplained
    return same, explained, total
