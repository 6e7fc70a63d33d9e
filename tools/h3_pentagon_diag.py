#!/usr/bin/env python3
"""Neighbour-walk consistency check around H3 pentagon base cells.

A Python restatement of H3 v3.7 h3NeighborRotations over the derived tables
(tools/gen_h3_neighbors.py), asserted equal to the oracle's C version, is compared
with cell geometry: the centres of res-2 cells are estimated by sampling 3e6 random
points through the oracle's geoToH3, and every walked neighbour must be among the 6
(5 for a pentagon) nearest centres.  Prints the failing (source base cell, target
base cell) pairs.  Test infrastructure (imports oracle/)."""
import sys, io, contextlib
sys.path.insert(0,'tools'); sys.path.insert(0,'oracle')
import gen_h3_neighbors as G, gen_h3_tables as T, oracle as O, numpy as np
with contextlib.redirect_stdout(io.StringIO()):
    nb, nr, (D2, A2, D3, A3) = G.build()
P=set(T.PENTAGONS)
CCW={0:0,1:5,5:4,4:6,6:2,2:3,3:1}; CW={v:k for k,v in CCW.items()}
def dg(h,r): return (h>>((15-r)*3))&7
def sd(h,r,d): s=(15-r)*3; return (h&~(7<<s))|(d<<s)
def res(h): return (h>>52)&15
def base(h): return (h>>45)&127
def lead(h):
    for r in range(1,res(h)+1):
        if dg(h,r): return dg(h,r)
    return 0
def rot(h, m):
    for r in range(1,res(h)+1): h=sd(h,r,m[dg(h,r)])
    return h
def rotpent(h):
    found=False
    for r in range(1,res(h)+1):
        h=sd(h,r,CCW[dg(h,r)])
        if not found and dg(h,r)!=0:
            found=True
            if lead(h)==1: h=rot(h,CCW)
    return h
def neighbor(h, d, rots, NB=nb, NR=nr, variant=None):
    for _ in range(rots[0]): d=CCW[d]
    ob=base(h); old_lead=lead(h); newrot=0
    r=res(h)-1
    while True:
        if r==-1:
            b=NB[ob][d]; newrot=NR[ob][d]
            if b==127:
                b=NB[ob][5]; newrot=NR[ob][5]; h=(h&~(127<<45))|(b<<45); h=rot(h,CCW); rots[0]+=1
            else: h=(h&~(127<<45))|(b<<45)
            break
        od=dg(h,r+1)
        if (r+1)%2: h=sd(h,r+1,D2[od][d]); nx=A2[od][d]
        else: h=sd(h,r+1,D3[od][d]); nx=A3[od][d]
        if nx: d=nx; r-=1
        else: break
    b=base(h)
    if b in P:
        adj=False
        if lead(h)==1:
            if ob!=b:
                cw = T.PENT_CW_OFFSET[b]
                f = HOME[ob][0]
                h = rot(h, CW) if f in cw else rot(h, CCW)
                adj=True
            else:
                if old_lead==0: return 0
                elif old_lead==3: h=rot(h,CCW); rots[0]+=1
                elif old_lead==5: h=rot(h,CW); rots[0]+=5
                else: return 0
        for _ in range(newrot): h=rotpent(h)
        if ob!=b:
            if b in (4,117):
                if ob not in (118,8) and lead(h)!=3: rots[0]+=1
            elif lead(h)==5 and not adj: rots[0]+=1
    else:
        for _ in range(newrot): h=rot(h,CCW)
    rots[0]=(rots[0]+newrot)%6
    return h
with contextlib.redirect_stdout(io.StringIO()):
    HOME, bc_of, rt, cen = T.build()
# check python neighbor == C oracle
import ctypes
L=O._h3_kring_lib()
rng=np.random.default_rng(3); N=3000000
lon=rng.uniform(-180,180,N); lat=np.degrees(np.arcsin(rng.uniform(-1,1,N)))
R=2
cells=O.h3_points_to_cells(lon,lat,R).astype(np.int64)
x=np.cos(np.radians(lat))*np.cos(np.radians(lon)); y=np.cos(np.radians(lat))*np.sin(np.radians(lon)); z=np.sin(np.radians(lat))
uc, inv = np.unique(cells, return_inverse=True)
cnt=np.bincount(inv); C=np.stack([np.bincount(inv,x)/cnt,np.bincount(inv,y)/cnt,np.bincount(inv,z)/cnt],1)
C/=np.linalg.norm(C,axis=1)[:,None]
idx={int(c):i for i,c in enumerate(uc)}
fails={}
for c in uc:
    c=int(c)
    if base(c) not in P and not any(nb[base(c)][d] in P for d in range(7) if nb[base(c)][d]!=127): continue
    v=C[idx[c]]; d=np.linalg.norm(C-v,axis=1); o=np.argsort(d)
    k = 5 if (base(c) in P and lead(c)==0) else 6
    geo=set(int(uc[j]) for j in o[1:1+k])
    for dd in range(1,7):
        r=[0]; n=neighbor(c,dd,r)
        rc=ctypes.c_int(0); nc=L.orc_h3_neighbor_rotations(c,dd,ctypes.byref(rc))
        assert n==nc or (n==0 and nc==0), (hex(c),dd,hex(n),hex(nc))
        if n and n not in geo:
            key=(base(c), base(n))
            fails.setdefault(key,[]).append((hex(c),dd))
for k,v in sorted(fails.items()): print(k, len(v), v[:2])
