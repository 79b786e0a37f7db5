"""Host model of the seeded cell scan's per-lane candidate counts at config 3 (diagnostics): uniform envs of
N = 256 in a 253 box, the 42 x 6 grid, disk radius = 4th-neighbour distance; prints the wave-max pair iterations for
lanes in agent order, in cell order and sorted by count, and the lane mean."""
import numpy as np
rng=np.random.default_rng(0)
N=256; box=253.0; gx,gy=42,6; cwx,cwy=box/gx,box/gy
res={'rand':[], 'sorted':[], 'mean':[]}
for env in range(200):
    p=rng.uniform(0,box,(N,2))
    d=np.abs(p[:,None]-p[None]); d=np.minimum(d,box-d); D=np.sqrt((d**2).sum(-1))
    r=np.sort(D,1)[:,4]*(1+2**-12)+box*1e-5
    cx=np.minimum((p[:,0]/cwx).astype(int),gx-1); cy=np.minimum((p[:,1]/cwy).astype(int),gy-1)
    cnt=np.zeros((gy,gx),int); np.add.at(cnt,(cy,cx),1)
    tot=np.zeros(N,int)
    for i in range(N):
        x,y=p[i]; q0=int(np.floor((y-r[i])/cwy)); q1=int(np.floor((y+r[i])/cwy))
        for q in range(q0,q1+1):
            ylo=q*cwy; dy=max(ylo-y, y-(ylo+cwy),0)
            if dy>r[i]: continue
            hw=np.sqrt(max(r[i]**2-dy*dy,0))
            xa=int(np.floor((x-hw)/cwx)); xb=int(np.floor((x+hw)/cwx))
            for c in range(xa,xb+1): tot[i]+=cnt[q%gy, c%gx]
    order=np.lexsort((cx,cy))
    for name,o in (('rand',np.arange(N)),('sorted',order)):
        t=tot[o].reshape(4,64); res[name].append(np.ceil(t.max(1)/2).mean())
    res['mean'].append(tot.mean()/2)
print({k:np.mean(v) for k,v in res.items()})
# balance: sort lanes by tot
r2=[]; r3=[]
rng=np.random.default_rng(1)
for env in range(100):
    p=rng.uniform(0,box,(N,2))
    d=np.abs(p[:,None]-p[None]); d=np.minimum(d,box-d); D=np.sqrt((d**2).sum(-1))
    r=np.sort(D,1)[:,4]*(1+2**-12)+box*1e-5
    cx=np.minimum((p[:,0]/cwx).astype(int),gx-1); cy=np.minimum((p[:,1]/cwy).astype(int),gy-1)
    cnt=np.zeros((gy,gx),int); np.add.at(cnt,(cy,cx),1)
    tot=np.zeros(N,int)
    for i in range(N):
        x,y=p[i]; q0=int(np.floor((y-r[i])/cwy)); q1=int(np.floor((y+r[i])/cwy))
        for q in range(q0,q1+1):
            ylo=q*cwy; dy=max(ylo-y, y-(ylo+cwy),0)
            if dy>r[i]: continue
            hw=np.sqrt(max(r[i]**2-dy*dy,0))
            xa=int(np.floor((x-hw)/cwx)); xb=int(np.floor((x+hw)/cwx))
            for c in range(xa,xb+1): tot[i]+=cnt[q%gy, c%gx]
    t=np.sort(tot).reshape(4,64); r2.append(np.ceil(t.max(1)/2).mean())
    # exact disk count (candidates strictly inside r) -- lower bound if cells were tiny
    r3.append(((D<=r[:,None]).sum(1)).mean()/2)
print('sorted-by-tot', np.mean(r2), 'disk-only mean', np.mean(r3))
