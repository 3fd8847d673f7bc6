"""sklearn KMeans with its k-means++ distances evaluated at the wide engine's operand precision
(f16 hi/lo products, f32 accumulation per 16 features): does the n=1200, d=300, K=8 problem of
tests/test_gpu_kmeans.py hinge on seeding rounding?  (It does not: same labels, same inertia;
nor on tol.)  CPU only:  python tools/emu_seed.py"""
import numpy as np, sys
sys.path.insert(0, __import__('os').path.dirname(__import__('os').path.dirname(__import__('os').path.abspath(__file__))))
from tests.test_gpu_kmeans import blobs
from consensus_clustering_amd import engine
import sklearn.cluster._kmeans as KM
from sklearn.cluster import KMeans
from threadpoolctl import threadpool_limits

orig = KM._euclidean_distances
def split(a, s):
    xs = (a.astype(np.float32) * np.float32(2.0**s)).astype(np.float32)
    hi = xs.astype(np.float16).astype(np.float32)
    lo = (xs - hi).astype(np.float16).astype(np.float32)
    return hi, lo
def emu(X, Y, X_norm_squared=None, Y_norm_squared=None, squared=False):
    # engine-like: x.c from f16 hi/lo (xh ch + xh cl + xl ch), f32 accumulation per 16-feature block
    s = 4
    Xh, Xl = split(X, s); Yh, Yl = split(Y, s)
    d = X.shape[1]
    acc = np.zeros((X.shape[0], Y.shape[0]), np.float32)
    for k in range(0, d, 16):
        sl = slice(k, k+16)
        blk = (Xh[:, sl].astype(np.float64) @ Yh[:, sl].T.astype(np.float64)
               + Xh[:, sl].astype(np.float64) @ Yl[:, sl].T + Xl[:, sl].astype(np.float64) @ Yh[:, sl].T)
        acc = (acc + blk.astype(np.float32)).astype(np.float32)
    dot = acc * np.float32(2.0**(-2*s))
    xn = (X.astype(np.float32)**2).sum(1, dtype=np.float32)
    yn = (Y.astype(np.float32)**2).sum(1, dtype=np.float32)
    D = (xn[:, None] + yn[None, :] - np.float32(2) * dot).astype(X.dtype)
    np.maximum(D, 0, out=D)
    return D
X = blobs(1200, 300, 5, seed=1200)
idx = engine.resample_indices(7, 1200, 960, 0, 4)
rows = X[idx[2]]
with threadpool_limits(1):
    ref = KMeans(n_clusters=8, random_state=7, n_init=3).fit(rows)
    print('sklearn', ref.inertia_)
    KM._euclidean_distances = emu
    e = KMeans(n_clusters=8, random_state=7, n_init=3).fit(rows)
    print('emulated seeding', e.inertia_, (e.labels_ == ref.labels_).mean())
    for s in range(3):
        km = KMeans(n_clusters=8, random_state=7, n_init=1)
        # per-init comparison
    KM._euclidean_distances = orig
with threadpool_limits(1):
    for init in range(3):
        pass
    for tol in (1e-4, 0.999e-4, 0.99e-4, 0.9e-4, 0.5e-4, 1e-5, 0):
        k = KMeans(n_clusters=8, random_state=7, n_init=3, tol=tol).fit(rows)
        print('tol', tol, k.inertia_, (k.labels_==ref.labels_).mean(), k.n_iter_)
    # each init separately
    from sklearn.utils import check_random_state
    for tol in (1e-4, 0):
        rs = check_random_state(7)
        km = KMeans(n_clusters=8, random_state=7, n_init=3, tol=tol, verbose=0)
        km.fit(rows)
