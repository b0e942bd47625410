#!/usr/bin/env python3
"""CPU simulation of the top-k threshold search (maxk_topk.hip): average count steps per row
for several first gallop steps and row distributions.  Development tool."""
import numpy as np
rng=np.random.default_rng(0)
def key(x):
    u=x.astype(np.float32).view(np.uint32).astype(np.int64)
    return np.where(u & 0x80000000, (~u)&0xffffffff, u|0x80000000)
def run(rows,k,step0):
    prevT=0xbf800000; steps=0
    for x in rows:
        kk=key(x)
        cnt=lambda t: int((kk>=t).sum()) if t<=0xffffffff else 0
        c0=cnt(prevT); steps+=1
        if c0==k: T=prevT; prevT=T; continue
        exact=False
        if c0>k:
            lo=prevT; step=step0
            while True:
                t=lo+step; c=cnt(t); steps+=1
                if c==k: T=t; exact=True; break
                if c<k: hi=t; break
                lo=t; step<<=2
        else:
            hi=prevT; step=step0
            while True:
                t=hi-step if hi>step else 0; c=cnt(t); steps+=1
                if c==k: T=t; exact=True; break
                if c>k: lo=t; break
                hi=t; step<<=2
        while not exact and hi-lo>1:
            mid=lo+((hi-lo)>>1); c=cnt(mid); steps+=1
            if c==k: T=mid; exact=True; break
            if c>k: lo=mid
            else: hi=mid
        if not exact: T=lo
        prevT=T
    return steps/len(rows)
rows=rng.random((3000,256),dtype=np.float32)
for s0 in (1<<10,1<<12,1<<14,1<<16,1<<18):
    print(s0, run(rows,32,s0))
rows=rng.standard_normal((3000,256)).astype(np.float32)
print('normal', [ (s0, run(rows,32,s0)) for s0 in (1<<12,1<<16,1<<18)])
rows=rng.random((3000,256),dtype=np.float32)
print('unif', [(s0, run(rows,32,s0)) for s0 in (1<<19,1<<20,1<<21,1<<22)])
print('unif k=8', [(s0, run(rows,8,s0)) for s0 in (1<<12,1<<18,1<<20)])
print('unif k=64', [(s0, run(rows,64,s0)) for s0 in (1<<12,1<<18,1<<20)])
rows=(rng.standard_normal((3000,256))*0.01).astype(np.float32)
print('normal*0.01', [(s0, run(rows,32,s0)) for s0 in (1<<12,1<<18,1<<20)])
rows=np.maximum(rng.standard_normal((3000,256)),0).astype(np.float32)
print('relu', [(s0, run(rows,32,s0)) for s0 in (1<<12,1<<18,1<<20)])
