"""Certified-bound pass rates of b-bit per-row row codes on isotropic 768-dim unit rows (numpy restatement
of sq8_bounds' interval): per query, the rows whose upper bound reaches the k-th best lower
bound, and the 610-row wave lists that would hold more than 16 of them.  One C3 shard: 1.25M rows, k = 10.
CPU only (≈ 8 GB of host memory)."""
import numpy as np
rng=np.random.default_rng(2)
N,D=1_250_000,768
X=np.empty((N,D),np.float32)
for i in range(0,N,250000):
    b=rng.standard_normal((min(250000,N-i),D),dtype=np.float32); b/=np.linalg.norm(b,axis=1,keepdims=True); X[i:i+len(b)]=b
k=10; LIST=610
def quant(bits):
    m=2**(bits-1)-1
    s=np.abs(X).max(1)/m
    q=np.clip(np.rint(X/s[:,None]),-m,m).astype(np.float32)
    dx=np.linalg.norm(X-q*s[:,None],axis=1); sq=np.linalg.norm(q*s[:,None],axis=1)
    return q,s,dx,sq
for bits in (8,6):
    q,s,dx,sq=quant(bits)
    for j in range(3):
        b=rng.standard_normal(D).astype(np.float32); b/=np.linalg.norm(b)
        qm=127 if bits==8 else 119
        sb=np.abs(b).max()/qm; qb=np.clip(np.rint(b/sb),-qm,qm); db=np.linalg.norm(b-qb*sb); nqb=np.linalg.norm(qb*sb)
        approx=(q@(qb*sb).astype(np.float32))*s
        err=sq*db+dx*(nqb+db)
        lb=approx-err; ub=approx+err
        L=np.sort(lb)[-k]
        surv=ub>=L
        per=surv[:N//LIST*LIST].reshape(-1,LIST).sum(1)
        print(bits, j, "survivors", int(surv.sum()), f"{surv.mean()*100:.3f}%", "lists>16:", int((per>16).sum()), "of", len(per), "max per list", int(per.max()))
    del q
