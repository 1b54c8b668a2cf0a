"""Simulation (CPU, numpy): tile skipping with per-block bounds.

ub over blocks of B labels (16384 = the kernel's tile, down to 256):
sum_v C[x,v] * maxc[v, block] against mneed(tau_final, gx + gmin_block); a
16384-target tile is scanned when any of its blocks may hold a target that
reaches the final tau.  Reports tiles per row by B, and "perfect" (tiles that
hold a target scoring >= tau).  python tools/sim_blockbound.py
"""
import os
import sys
import numpy as np
import scipy.sparse as sp
sys.path[:0] = [os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", d) for d in ("distributed-pathsim_amd", "oracle")]
from dpathsim.synth import synth_config; import pathsim_oracle as po
W=16384; k=10
t=synth_config('config3').typed(); co=po.COracle.from_typed(t); cp,cc,cv,s,gg=co.export()
NA,NV=t.n_authors,t.n_mids; cp=cp[:NA+1]; cc=cc[:cp[-1]]; cv=cv[:cp[-1]].astype(np.int64); gg=gg[:NA].astype(np.int64)
C=sp.csr_matrix((cv,cc,cp),shape=(NA,NV))
order=np.argsort(gg,kind='stable'); rank=np.empty(NA,np.int64); rank[order]=np.arange(NA)
T=(NA+W-1)//W; g_lab=gg[order]
row_of=np.repeat(np.arange(NA),np.diff(cp)); lab_of_row=rank
res={}
for B in (16384,4096,2048,1024,256):
    nb=(NA+B-1)//B
    mx=np.zeros((NV,nb),np.int64); np.maximum.at(mx,(cc,lab_of_row[row_of]//B),cv)
    gmin=g_lab[np.arange(nb)*B]
    res[B]=(mx,gmin,nb)
n_v=np.bincount(cc,minlength=NV); deg=np.diff(cp)
terms=np.add.reduceat(n_v[cc],cp[:-1])*(deg>0)
rng=np.random.default_rng(7); qs=np.quantile(terms,[0,0.33,0.66,1.0])
for band in range(3):
    pool=np.flatnonzero((terms>=qs[band])&(terms<=qs[band+1])&(deg>0))
    rows=rng.choice(pool,40,replace=False)
    acc={B:0 for B in res}; perf=0; n=0
    for x in rows:
        a0,a1=cp[x],cp[x+1]; v,a=cc[a0:a1],cv[a0:a1]
        mrow=np.asarray(C@sp.csr_matrix((a,v,[0,len(v)]),shape=(1,NV)).T.todense()).ravel(); mrow[x]=0
        sc=2.0*mrow/(gg[x]+gg); tau=np.sort(sc)[-k]
        if tau<=0: continue
        n+=1
        perf+=len(np.unique(lab_of_row[np.flatnonzero(sc>=tau)]//W))
        for B,(mx,gmin,nb) in res.items():
            ub=(a[:,None]*mx[v]).sum(0); mneed=np.ceil(tau*(gg[x]+gmin)/2.0-1e-9)
            live=ub>=mneed   # blocks that may hold a winner
            per=W//B
            tl=live.reshape(-1) if per==1 else np.pad(live,(0,T*per-nb)).reshape(T,per).any(1)
            acc[B]+=tl.sum()
    print(f"band {band}: rows {n}: tiles/row by block-bound granularity "+"  ".join(f"{B}:{acc[B]/n:.1f}" for B in res)+f"  perfect {perf/n:.1f}",flush=True)
