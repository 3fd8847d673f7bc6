"""Search seeded duplicate-heavy datasets for sklearn float64 fits that relocate >= 2 empty clusters
at once (np.argpartition intercepted), split by tied / distinct farthest distances; the tied seeds
feed tests/test_gpu_kmeans.py::test_f64_relocation_with_ties_is_pinned.  CPU only."""
import numpy as np, warnings
warnings.filterwarnings('ignore')
import sklearn.cluster._k_means_common as C
from sklearn.cluster import KMeans
from threadpoolctl import threadpool_limits
def make(seed):
    rng=np.random.default_rng(seed)
    n=int(rng.integers(20,60)); d=int(rng.integers(1,4))
    nd=int(rng.integers(5,12))
    base=rng.normal(size=(nd,d))*rng.uniform(0.5,5)
    X=base[rng.integers(0,nd,n)]+rng.normal(size=(n,d))*rng.choice([0,0.01,0.3])
    K=int(rng.integers(3,nd+3))
    return X,K
calls=[]
class NP:
    def __getattr__(self, k): return getattr(np, k)
    def argpartition(self, a, kth, *args, **kw):
        a=np.asarray(a); r=np.argpartition(a, kth, *args, **kw); calls.append((a.copy(), kth, r.copy())); return r
res={'distinct':[], 'ties':[]}
with threadpool_limits(1):
    C.np=NP()
    for seed in range(3000):
        X,K=make(seed)
        calls.clear()
        KMeans(n_clusters=K, random_state=seed, n_init=3).fit(X)
        kinds=set()
        for a,kth,r in calls:
            ne=-kth
            if a.max()==0: continue
            top=np.sort(a)[::-1][:ne+1]
            if ne>=2:
                tie = len(np.unique(a[r[-ne:]]))<ne or (a==a[r[-ne]]).sum()>1
                kinds.add('ties' if tie else 'distinct')
        for k in kinds: res[k].append(seed)
    C.np=np
print({k:(len(v),v[:12]) for k,v in res.items()})
