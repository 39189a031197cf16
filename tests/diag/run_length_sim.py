"""Diagnostic (CPU): records per sample of the table scatter (a lane's consecutive samples in one cell
summed before the table) for chunk lengths 1-32, per level, on one marched bench batch (DESIGN §7
round-5 findings)."""
import os, sys, numpy as np
ROOT=os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))); sys.path[:0]=[ROOT, ROOT+'/normal-clustering-nerf_amd']
from oracle import field_ref, vren_ref
from ncnerf_amd.synthetic import SyntheticScene
scene=SyntheticScene(); b=scene.batch(8192, seed=1)
o,d=b['rays_o'],b['rays_d']
_,ht,_=vren_ref.ray_aabb_intersect(o,d,np.zeros((1,3),np.float32),np.full((1,3),0.5,np.float32),1)
ht=ht[:,0].copy(); m=(ht[:,0]>=0)&(ht[:,0]<0.01); ht[m,0]=0.01
_,xyzs,_,_,_,cnt=vren_ref.raymarching_train(o,d,ht,scene.bitfield,1,0.5,0.0,np.random.default_rng(0).random(8192).astype(np.float32),128,1024)
S=int(cnt[0]); x=xyzs[:S]+0.5
levels,_=field_ref.grid_levels(0.5)
for l in range(0,16):
    lv=levels[l]
    pg=np.floor((x.astype(np.float64)*lv['scale']+0.5).astype(np.float32)).astype(np.int64)
    key=pg[:,0]+4096*pg[:,1]+4096*4096*pg[:,2]
    ch=key[1:]!=key[:-1]
    out=[]
    for L in (1,2,4,8,16,32):
        # runs when a lane holds L consecutive samples: a run breaks at cell change or chunk boundary
        brk=ch.copy(); idx=np.arange(1,S); brk|=(idx%L==0)
        out.append(round((1+brk.sum())/S,3))
    print(l, lv['res'], 'records/sample for chunk 1,2,4,8,16,32:', out)
