"""Pending-entry count of the BSP walk's trail at each push (DESIGN.md section 4,
"HBM traffic": the compact-trail estimate).  Test-side helper, not a test: it
uses the CPU oracle for each ray's hit and replays bsp.wgsl's walk
(bsp.wgsl:10-81) with an explicit stack, ending at the first leaf whose interval
holds the hit.  usage: python tests/trail_sim.py [config] [ntris] [rays]"""
import sys, types, numpy as np, collections, time
import os
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT); sys.path.insert(0, os.path.join(ROOT, 'tests'))
from importlib import import_module
import oracle_ffi as O
cfgn=int(sys.argv[1]) if len(sys.argv)>1 else 3
cfg=import_module('02562_raytracer_amd.configs').WORKLOADS[cfgn]
nt = int(sys.argv[2]) if len(sys.argv)>2 else None
NR = int(sys.argv[3]) if len(sys.argv)>3 else 3000
mesh=cfg.mesh(nt)
tree,planes,ids,aabb,D=mesh.bsp_tree(20,4).arrays()
pos,nrm,idx,mats,lights=mesh.arrays()
m=types.SimpleNamespace(pos=pos,nrm=nrm,idx=idx,ntris=idx.shape[0],mats=np.ascontiguousarray(mats),lights=lights)
b=types.SimpleNamespace(aabb=aabb,tree=tree,planes=planes,ids=ids,max_depth=D)
sc=O.SceneRef(m,b)
eye,tgt,up,cc=cfg.camera
u=O.make_uniform(eye,tgt,up,cc,cfg.width,cfg.height)
rng=np.random.default_rng(1)
hist=collections.Counter(); maxp=collections.Counter()
def walk(o,d,tmin,tmax,thit,tri):
    node=0; stack=[]; mp=0
    for _ in range(100000):
        a=tree[node,0]&3
        if a==3:
            cnt=tree[node,0]>>2; f=tree[node,1]
            if tri is not None and tmin<=thit<=tmax and tri in ids[f:f+cnt]: return mp
            if not stack: return mp
            node,tmin,tmax=stack.pop(); continue
        ad=d[a]; ao=o[a]
        near,far=(tree[node,2],tree[node,3]) if ad>=0 else (tree[node,3],tree[node,2])
        den=np.float32(1e-8) if abs(ad)<1e-8 else ad
        t=np.float32((planes[node]-ao)/den)
        if t>tmax: node=near
        elif t<tmin: node=far
        else:
            hist[len(stack)]+=1
            stack.append((far,t,tmax)); mp=max(mp,len(stack)); tmax=t; node=near
    return mp
t0=time.time()
for k in range(NR):
    x=int(rng.integers(cfg.width)); y=int(rng.integers(cfg.height))
    o,d=O.camera_ray(u,x,y,float(rng.random())/cfg.height,float(rng.random())/cfg.height)
    hit,tri,dist=O.trace_one(sc,'BSP',o,d,1e-4,5000.0)
    maxp[walk(o,d,np.float32(1e-4),np.float32(5000.0),dist,tri if hit else None)]+=1
    if hit:
        p=(o+d*np.float32(dist)).astype(np.float32); dd=np.array([0,1,0],np.float32)
        h2,t2,d2=O.trace_one(sc,'BSP',p,dd,1e-4,999999.0-1e-4)
        maxp[walk(p,dd,np.float32(1e-4),np.float32(999999.0-1e-4),d2,t2 if h2 else None)]+=1
tot=sum(hist.values())
print('cfg',cfgn,'rays',sum(maxp.values()),'pushes',tot,'time',round(time.time()-t0,1))
print('push at pending p:', {k:round(v/tot,5) for k,v in sorted(hist.items())})
mt=sum(maxp.values())
print('max pending per ray:', {k:round(v/mt,5) for k,v in sorted(maxp.items())})
