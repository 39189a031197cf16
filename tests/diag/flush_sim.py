"""Diagnostic (CPU): how many global flushes the table scatter's units make per distinct table entry
under different sample processing orders, on one marched 8192-ray bench batch (oracle marcher)."""
import sys, numpy as np, torch
import os
ROOT=os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0]=[ROOT,os.path.join(ROOT,'normal-clustering-nerf_amd')]
from oracle import vren_ref, field_ref
from ncnerf_amd.synthetic import SyntheticScene, morton3d_np
scene=SyntheticScene(); b=scene.batch(8192, seed=1)
o,d=b['rays_o'],b['rays_d']
_,ht,_=vren_ref.ray_aabb_intersect(o,d,np.zeros((1,3),np.float32),np.full((1,3),0.5,np.float32),1)
ht=ht[:,0].copy(); m=(ht[:,0]>=0)&(ht[:,0]<0.01); ht[m,0]=0.01
rays_a,xyzs,dirs,deltas,ts,cnt=vren_ref.raymarching_train(o,d,ht,scene.bitfield,1,0.5,0.0,np.random.default_rng(0).random(8192).astype(np.float32),128,1024)
S=int(cnt[0]); x=xyzs[:S]+0.5
print("samples",S)
levels,_=field_ref.grid_levels(0.5)
def entries(x, lv):
    pos=(x.astype(np.float64)*lv['scale']+0.5).astype(np.float32); fl=np.floor(pos); pg=fl.astype(np.int64)
    out=[]
    for c in range(8):
        p=pg+np.array([(c>>k)&1 for k in range(3)])
        if lv['res']**3<=lv['params']:
            e=p[:,0]+lv['res']*p[:,1]+lv['res']**2*p[:,2]
        else:
            e=(p[:,0]^(p[:,1]*2654435761)^(p[:,2]*805459861))&0xFFFFFFFF
        out.append(e%lv['params'])
    return np.stack(out,1)
def flushes(E, unit):
    tot=0
    for s in range(0,len(E),unit):
        tot+=len(np.unique(E[s:s+unit]))
    return tot
mort=morton3d_np(*(np.clip((x*1023).astype(np.int64),0,1023).T))
orders={"ray": np.arange(S), "morton_global": np.argsort(mort,kind='stable')}
w=np.arange(S)//65536; orders["morton_64k_windows"]=np.lexsort((mort,w))
w=np.arange(S)//4096; orders["morton_4k_windows"]=np.lexsort((mort,w))
for l in range(6,16):
    lv=levels[l]; E=entries(x,lv)
    unit = 2048 if l==15 else 4096
    distinct=len(np.unique(E))
    res={k: flushes(E[v],unit) for k,v in orders.items()}
    print(l, lv['res'], "distinct", distinct, "contribs", E.size, {k: round(vv/distinct,2) for k,vv in res.items()}, "lds-adds/unit-distinct", round(E.size/res['ray'],2))
print("coarse cell-keyed units")
tot_c=0
for l in range(0,10):
    lv=levels[l]
    pos=(x.astype(np.float64)*lv['scale']+0.5).astype(np.float32); pg=np.floor(pos).astype(np.int64)
    key=pg[:,0]+2048*pg[:,1]+2048*2048*pg[:,2]
    span=1024*4*(4 if l<6 else 2)
    nc=sum(len(np.unique(key[s:s+span])) for s in range(0,S,span))
    tot_c+=nc*16
    print(l, "cells flushed", nc, "floats", nc*16)
print("coarse float atomics", tot_c)
tot_f=0
for l in range(10,16):
    E=entries(x,levels[l]); unit=2048 if l==15 else 4096
    tot_f+=flushes(E,unit)*2
print("fine float atomics", tot_f, "total MB", (tot_c+tot_f)*4/1e6)
