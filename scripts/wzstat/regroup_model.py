"""Model of the rounds kernel's lane utilisation under pixel regroupings
(round 6): per-pixel rounds / per-round clamp iterations from
wzrounds.cpp on the bench recipe (synth.frames_numpy), then the trips a wave
of 64 pixels pays as one loop nest, as round-wise launches over compacted
lists, with block-level compaction between rounds, and sorted by
(noisy) predictors.  Tooling only.  Build libwz2.so first (see wzrounds.cpp)."""
import ctypes as C, numpy as np, os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from siril_amd import synth
L=C.CDLL(os.environ.get('WZ_LIB', '/tmp/wz/libwz2.so'))
n=100; h=8; w=16384
fr=synth.frames_numpy(n,h,w,seed=3).reshape(n,-1)
ncol=fr.shape[1]
out=np.zeros((ncol,20),np.int32)
L.wz_stats2(fr.ctypes.data_as(C.c_void_p), n, C.c_longlong(ncol), C.c_float(3), C.c_float(3), out.ctypes.data_as(C.c_void_p))
route=out[:,0]; rounds=out[:,1]; iters=out[:,2]; it=out[:,4:20]
ok=route==0
print('pixels',ncol,'route0 frac',ok.mean(),'rounds avg',rounds[ok].mean(),'iters avg',iters[ok].mean())
print('iters per round avg (pixels in round):',[round(float(it[rounds>r][:,r].mean()),2) for r in range(5)], 'frac in round', [round(float((rounds>r).mean()),3) for r in range(6)])
CR=4.0  # cost of a round's overhead in units of one clamp iteration
def nest_cost(idx):  # one wave = pixels idx (64)
    c=0.0
    R=rounds[idx].max()
    for r in range(R):
        act=rounds[idx]>r
        if act.any(): c+=CR+it[idx][act][:,r].max()
    return c
def useful(idx):
    return (rounds[idx]*CR+iters[idx]).sum()/64.0
W=ncol//64
tot=sum(nest_cost(np.arange(k*64,(k+1)*64)) for k in range(W)); use=sum(useful(np.arange(k*64,(k+1)*64)) for k in range(W))
print('nest: lane util %.3f, cost per pixel %.2f'%(use/tot, tot*64/ncol/64))
# round-wise: pass r runs round r for compacted pixels still going
tot2=0.0
for r in range(int(rounds.max())):
    act=np.nonzero(rounds>r)[0]
    for k in range(0,len(act),64):
        idx=act[k:k+64]; tot2+=CR+it[idx][:,r].max()
print('round-wise: lane util %.3f (cost ratio to nest %.3f)'%(use/tot2, tot2/tot))
# oracle sort by total work within windows
for win in (256,1024,4096):
    tot3=0.0
    work=rounds*CR+iters
    for s0 in range(0,ncol,win):
        idx=np.arange(s0,min(ncol,s0+win)); idx=idx[np.argsort(work[idx])]
        for k in range(0,len(idx),64): tot3+=nest_cost(idx[k:k+64])
    print('sorted by true work, window %d: cost ratio %.3f'%(win, tot3/tot))
work=rounds*CR+iters
r1=it[:,0]
for key,name in ((r1,'round-1 iters'),):
    for win in (1024, 4096):
        tot3=0.0
        for s0 in range(0,ncol,win):
            idx=np.arange(s0,min(ncol,s0+win)); idx=idx[np.argsort(key[idx],kind='stable')]
            for k in range(0,len(idx),64): tot3+=nest_cost(idx[k:k+64])
        print('sorted by %s, window %d: cost ratio %.3f'%(name,win, tot3/tot))
# noisy proxy: r1 + noise
rng=np.random.default_rng(0)
for sd in (1.0,2.0,3.0):
    key=r1+rng.normal(0,sd,ncol)
    tot3=0.0
    for s0 in range(0,ncol,1024):
        idx=np.arange(s0,min(ncol,s0+1024)); idx=idx[np.argsort(key[idx],kind='stable')]
        for k in range(0,len(idx),64): tot3+=nest_cost(idx[k:k+64])
    print('sorted by r1 + N(0,%g), window 1024: cost ratio %.3f'%(sd, tot3/tot))
print('corr(r1, total work)', np.corrcoef(r1, work)[0,1])
print('r1 distribution', np.bincount(r1)[:25])
def block_compact(B):
    tot4=0.0
    for s0 in range(0,ncol,B):
        idx=np.arange(s0,min(ncol,s0+B))
        R=int(rounds[idx].max())
        for r in range(R):
            act=idx[rounds[idx]>r]   # compacted each round within the block
            for k in range(0,len(act),64):
                w=act[k:k+64]; tot4+=CR+it[w][:,r].max()
    return tot4
for B in (256,512,1024):
    print('block-level compaction every round, block %d: cost ratio %.3f'%(B, block_compact(B)/tot))
for B in (128,192):
    print('block-level compaction every round, block %d: cost ratio %.3f'%(B, block_compact(B)/tot))
