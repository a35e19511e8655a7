"""Multi-phase variant of tools/r06_sched_sim.py (profiles/r06/park/sched_multiphase.txt)."""
import numpy as np, heapq
exec(open('tools/r06_sched_sim.py').read().split("print('--- cut at 50')")[0].split("# predictor at iteration 25")[0])
def g(key,default): return np.array([x.get(key,default) for x in f],float)
F=lambda key: np.log10(np.maximum(g(key,1),1e-30))
base=15e3+54e3
def phases(cuts, restore=15e3, gap=44e3):
    # robot progress: duration until iteration c ~ base + 54k*min(ru, rho updates before c) + 3.7k*min(it,c)
    # (rho updates spread uniformly over the robot's checks: approximate refactor count before c)
    total=0.0
    prev=0
    remaining=np.ones(len(it),bool)
    frac_ru=lambda c: np.minimum(ru, np.floor(ru*np.minimum(c,it)/np.maximum(it,1)+0.5))
    for j,c in enumerate(list(cuts)+[10**9]):
        cc=min(c,10**9)
        start = (base if prev==0 else restore) + 3.7e3*(np.minimum(it,cc)-np.minimum(it,prev)) + 54e3*(frac_ru(cc)-frac_ru(prev))
        d=np.where(remaining, start, 0.0)
        if prev==0: order=range(len(it))
        else: order=np.argsort(-F('du%d'%prev))
        total+=ls(d,[i for i in order if remaining[i]])+ (gap if j>0 else 0)
        remaining = remaining & (it>cc)
        prev=cc
        if not remaining.any(): break
    return total
print('one launch', ls(dur,range(len(dur))))
for cuts in ([50],[75],[50,100],[50,125],[75,150],[50,100,150],[25,75,125]):
    print(cuts, phases(cuts), 'gain %.3f'%(ls(dur,range(len(dur)))/phases(cuts)))
