#!/usr/bin/env python3
"""Host-side estimate of the hub cut (BuArgs::cut_edges) on one first
bottom-up level: builds the RMAT graph on the host (bit-identical to the
device generator; scale 26 takes ~12 min and ~30 GB), runs the CPU oracle,
and for level L of each root counts the frontier's top-down edges outside the
top-K vertices by degree and the row entries a bottom-up scan reads with and
without the cut (rows in neighbour-degree order, as hub_col).
    python3 tools/hub_cut_analysis.py 26 17872028:2 8766153:2
Output of that run: profiles/r3_hub_cut_cpu_analysis_rmat26.txt."""
import sys, time, numpy as np
sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__))))
import distributed_cuda_bfs_amd as dbfs
from distributed_cuda_bfs_amd.ops import graph as G
t=time.time()
scale=int(sys.argv[1]); roots=[(int(a.split(':')[0]), int(a.split(':')[1])) for a in sys.argv[2:]]
p=G.rmat_params(scale)
u,v=G.generate_edges(p)
csr=G.build_csr(p.n,u,v); del u,v
ro=np.asarray(csr.row_off); col=np.asarray(csr.col)
print("csr %.0f s, nnz %d" % (time.time()-t, len(col)), flush=True)
deg=np.diff(ro).astype(np.int64)
order=np.argsort(-deg, kind="stable"); rank=np.empty(p.n, np.int32); rank[order]=np.arange(p.n, dtype=np.int32); del order
nz=np.nonzero(deg)[0]
BIG=np.int32(2**31-1)
Ks=[1<<10,1<<12,1<<14,1<<16,(1<<19)-4096]
for r,L in roots:
    lev=np.asarray(G.cpu_bfs(csr,r)[0])
    F=(lev==L); U=(lev>L)
    fr=np.nonzero(F)[0]
    print(f"root {r} level {L}: |F| {len(fr)} F edges {deg[fr].sum()} F ranks<2^12 {np.sum(rank[fr]<4096)} <2^16 {np.sum(rank[fr]<65536)} <2^19 {np.sum(rank[fr]<(1<<19)-4096)}", flush=True)
    for K in Ks: print(f"   K {K}: TD prepass edges {deg[fr][rank[fr]>=K].sum()}  vertices {np.sum(rank[fr]>=K)}")
    rows=nz[U[nz]]
    base_scan=0; found=0; cut_scan={K:0 for K in Ks}; pre={K:0 for K in Ks}
    FK={K:(F & (rank>=K)) for K in Ks}
    CH=1<<22
    for i in range(0,len(rows),CH):
        rr=rows[i:i+CH]
        lens=deg[rr]; starts=ro[rr]
        idx=np.repeat(starts - np.concatenate([[0],np.cumsum(lens)[:-1]]), lens) + np.arange(lens.sum())
        c=col[idx]; rk=rank[c]; isF=F[c]
        seg=np.concatenate([[0],np.cumsum(lens)[:-1]])
        rowid=np.repeat(np.arange(len(rr)), lens)
        mfr=np.minimum.reduceat(np.where(isF,rk,BIG),seg)
        f=mfr<BIG; found+=f.sum()
        lt=np.add.reduceat((rk<mfr[rowid]).astype(np.int64),seg)
        base_scan+=np.where(f,lt+1,lens).sum()
        for K in Ks:
            # rows pre-claimed by the TD pass (a frontier neighbour of rank >= K) are skipped
            prec=np.logical_or.reduceat(FK[K][c],seg)
            isFK=isF&(rk<K)
            m=np.minimum.reduceat(np.where(isFK,rk,BIG),seg)
            fk=m<BIG
            ltk=np.add.reduceat((rk<m[rowid]).astype(np.int64),seg)
            nk=np.add.reduceat((rk<K).astype(np.int64),seg)
            sc=np.where(fk,ltk+1,np.maximum(nk,1))
            cut_scan[K]+=np.where(prec,0,sc).sum(); pre[K]+=prec.sum()
    print(f"   unvisited rows {len(rows)} found {found}; entries scanned now {base_scan}", flush=True)
    for K in Ks: print(f"   K {K}: BU scanned {cut_scan[K]} ({cut_scan[K]/base_scan:.2f}x), rows pre-claimed {pre[K]}", flush=True)
    print("  %.0f s" % (time.time()-t), flush=True)
