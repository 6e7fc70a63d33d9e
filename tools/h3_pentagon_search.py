#!/usr/bin/env python3
"""Search of a pentagon base cell's unpublished face rotations (faceIjkBaseCells) for the
assignment under which res-2 neighbour walks inside the pentagon agree with the cells'
sampled geometry.  Needs tools/h3_pentagon_search_lib.c built as a
shared library (gcc -O2 -fPIC -shared -Ioracle -o /tmp/ex/libexplore.so ... -lm -lpthread).
Usage: h3_pentagon_search.py <base cell> [res].  Test infrastructure."""
import os, sys, ctypes, io, contextlib, itertools
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import numpy as np, gen_h3_tables as T
with contextlib.redirect_stdout(io.StringIO()):
    home, bc_of, rot, cen = T.build()
L = ctypes.CDLL(os.environ.get('H3_SEARCH_LIB', '/tmp/ex/libexplore.so'))
dp=ctypes.POINTER(ctypes.c_double); u64p=ctypes.POINTER(ctypes.c_uint64)
L.orc_h3_points_to_cells.argtypes=[dp,dp,ctypes.c_int64,ctypes.c_int,ctypes.c_int,u64p,ctypes.c_int]
L.orc_h3_neighbor_rotations.restype=ctypes.c_uint64
L.orc_h3_neighbor_rotations.argtypes=[ctypes.c_uint64,ctypes.c_int,ctypes.POINTER(ctypes.c_int)]
L.ex_get.restype=ctypes.c_int
RES=int(sys.argv[2]) if len(sys.argv)>2 else 2
def cells_of(lon,lat):
    out=np.zeros(len(lon),dtype=np.uint64)
    L.orc_h3_points_to_cells(lon.ctypes.data_as(dp),lat.ctypes.data_as(dp),len(lon),RES,8,out.ctypes.data_as(u64p),8)
    return out.astype(np.int64)
def score(b, lon, lat, x):
    cells=cells_of(lon,lat)
    uc,inv=np.unique(cells,return_inverse=True)
    cnt=np.bincount(inv); C=np.stack([np.bincount(inv,x[:,q])/cnt for q in range(3)],1); C/=np.linalg.norm(C,axis=1)[:,None]
    idx={int(c):i for i,c in enumerate(uc)}
    v0=cen[b][0]
    bad=0; tot=0
    for c in uc:
        c=int(c)
        if (c>>45)&127!=b: continue
        v=C[idx[c]]
        if np.dot(v,v0) < np.cos(0.12): continue  # interior cells only (well sampled all round)
        d=np.linalg.norm(C-v,axis=1); o=np.argsort(d)
        lead=0
        for r in range(1,RES+1):
            dg=(c>>((15-r)*3))&7
            if dg: lead=dg; break
        k=5 if lead==0 else 6
        geo=set(int(uc[j]) for j in o[1:1+k])
        for dd in range(1,7):
            rr=ctypes.c_int(0); n=L.orc_h3_neighbor_rotations(c,dd,ctypes.byref(rr))
            if n==0 or (n>>45)&127!=b: continue
            tot+=1
            if int(n) not in geo: bad+=1
    return bad,tot
b=int(sys.argv[1])
v0=cen[b][0]
rng=np.random.default_rng(0); N=600000
# points within 0.3 rad of the vertex
z=rng.uniform(np.cos(0.3),1,N); ph=rng.uniform(0,2*np.pi,N); s=np.sqrt(1-z*z)
e1=np.cross([0,0,1.0],v0); e1/=np.linalg.norm(e1); e2=np.cross(v0,e1)
x=(z[:,None]*v0+ (s*np.cos(ph))[:,None]*e1 + (s*np.sin(ph))[:,None]*e2)
lat=np.degrees(np.arcsin(x[:,2])); lon=np.degrees(np.arctan2(x[:,1],x[:,0]))
lat=np.ascontiguousarray(lat); lon=np.ascontiguousarray(lon)
keys={}
for key,bc in bc_of.items():
    if bc==b: keys.setdefault(key[0],[]).append(key)
faces=[f for f in keys if f!=home[b][0]]
cur={f: rot[keys[f][0]] for f in keys}
def apply(assign):
    for f,ks in keys.items():
        for (ff,i,j,k) in ks: L.ex_set(ff,i,j,k, b | (assign[f]<<8))
print("pentagon",b,"home",home[b][0],"faces",faces,"current",cur, "cw", T.PENT_CW_OFFSET[b])
apply(cur); print("current score", score(b,lon,lat,x))
import time
t=time.time()
a=dict(cur)
for sweep in range(2):
    for f in faces:
        res=[]
        for v in range(6):
            a2=dict(a); a2[f]=v; apply(a2); res.append((score(b,lon,lat,x)[0],v))
        a[f]=min(res)[1]
        print("face",f,"scores",res, "%.0fs"%(time.time()-t), flush=True)
apply(a); print("final",a,score(b,lon,lat,x), "was", cur)
