"""Would exact bound-based skipping (Hamerly / Elkan) shorten K1's Lloyd sweeps at C3?  (VERDICT r5,
next 1.)  Float64 Lloyd on one C3 resample (make_blobs n = 50 000, d = 128, 8 centres, seed 0;
m = 40 000) for every K and 3 k-means++ inits, with Elkan's per-centre lower bounds (the tightest
triangle-inequality bounds; Hamerly's single lower bound is looser): a row is ACTIVE in an
iteration when its upper bound reaches any lower bound, i.e. when an exact engine could not prove
its label unchanged.  Prints per problem the active fraction per iteration, and at the end the
share of the E-step work (rows x K) that is active and the share of 32-row tiles (resample order,
as K1 streams them) holding at least one active row for that ONE problem (a sweep serves ~12
problems at once, so the union is larger still).

    python tools/bound_skip_sim.py 2 3 ... 20   (profiles/r06/bound_skip_sim_c3.txt)
"""
import numpy as np, sys
from sklearn.datasets import make_blobs
from sklearn.cluster import kmeans_plusplus
n,d,kt=50000,128,8
X,_=make_blobs(n_samples=n,n_features=d,centers=kt,cluster_std=1.0,center_box=(-10,10),shuffle=True,random_state=0)
X=X.astype(np.float64); X-=X.mean(0)
rs=np.random.RandomState(0); idx=rs.permutation(n)[:40000]; Xs=X[idx]
tol=1e-4*np.mean(np.var(Xs,axis=0))
xn=(Xs**2).sum(1)
tot_full=0; tot_act=0; tot_tile=0
for K in [int(a) for a in sys.argv[1:]]:
  for init in range(3):
    C,_=kmeans_plusplus(Xs,K,random_state=np.random.RandomState(init))
    D=np.sqrt(np.maximum(xn[:,None]-2*Xs@C.T+(C**2).sum(1)[None],0))
    lab=D.argmin(1); u=D[np.arange(len(D)),lab].copy(); L=D.copy()
    acts=[];tiles=[]
    for it in range(300):
      Cn=np.array([Xs[lab==c].mean(0) if (lab==c).any() else C[c] for c in range(K)])
      sh=np.sqrt(((Cn-C)**2).sum(1)); C=Cn
      u+=sh[lab]; L-=sh[None,:]
      L[np.arange(len(L)),lab]=np.inf
      act=(u[:,None]>=L).any(1)
      acts.append(act.mean()); tiles.append(act.reshape(-1,32).any(1).mean())
      D=np.sqrt(np.maximum(xn[:,None]-2*Xs@C.T+(C**2).sum(1)[None],0))
      nl=D.argmin(1)
      assert (nl[~act]==lab[~act]).all()
      u[act]=D[act,nl[act]]; L[act]=D[act]
      ch=(nl!=lab).sum(); lab=nl
      if ch==0 or (sh**2).sum()<=tol: break
    tot_full+=len(acts)*K; tot_act+=sum(a*K for a in acts); tot_tile+=sum(a*K for a in tiles)
    print(K,init,len(acts),'mean act %.3f tile %.3f'%(np.mean(acts),np.mean(tiles)),' '.join('%.3f'%a for a in acts[:40]),flush=True)
print('work frac rows %.3f tiles %.3f'%(tot_act/tot_full,tot_tile/tot_full))
