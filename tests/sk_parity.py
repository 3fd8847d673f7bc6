"""Shared check of the fast (float32-class) k-means against the reference's clusterer: sklearn
KMeans called as CC.py:205-214 / :282 call it.  Not a test module."""
import numpy as np


def sklearn_parity(X, labels, idx, Ks, seed, resamples, skip=0, threads=16, n_init=3):
    """Labels of resamples skip .. skip + resamples - 1 of every K against sklearn's float32
    KMeans on the same rows.  A disagreement is allowed only where sklearn's own float32 and
    float64 fits of those rows disagree (the partition hinges on rounding, the accuracy class
    the f16 hi/lo MFMA engine shares with sklearn's float32 sgemm).  Prints and returns
    (identical, explained, total); asserts that no disagreement is unexplained.

    labels: the fit's device label matrix [nK, n, Hpad] (uint8) or a host array
    [nK, H, m] of labels in resample order."""
    from sklearn.cluster import KMeans
    from threadpoolctl import threadpool_limits

    same = explained = 0
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
                else:
                    unexplained.append((K, h, float(np.mean(ref32 == got))))
    total = len(Ks) * resamples
    print(f"sklearn parity: {same}/{total} identical, {explained} differ where sklearn f32 != f64, "
          f"{len(unexplained)} unexplained {unexplained}")
    assert not unexplained, unexplained
    return same, explained, total
