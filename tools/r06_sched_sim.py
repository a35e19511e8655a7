"""List-scheduling simulation of the C2 dispatch tail: one launch in input order, LPT, and the
two-phase (park / resume) solve with several orderings (profiles/r06/park/sched_sim.txt)."""
import numpy as np, heapq
import json
rows=json.load(open('profiles/r06/park/iters_checks.json'))
it=np.array([r[0] for r in rows],float); ru=np.array([r[1] for r in rows],float)
f=[r[2] for r in rows]
print('iters mean %.1f median %.0f p90 %.0f max %.0f'%(it.mean(),np.median(it),np.percentile(it,90),it.max()))
print('frac done by 25/50/75/100:', [(it<=k).mean() for k in (25,50,75,100)])
dur=15e3+54e3*(1+ru)+3.7e3*it  # cycles
def ls(d, order, slots=1024):
    h=[0.0]*slots; heapq.heapify(h)
    for i in order:
        t=heapq.heappop(h); heapq.heappush(h,t+d[i])
    return max(h)
ideal=dur.sum()/1024
M0=ls(dur,range(len(dur)))
Ml=ls(dur,np.argsort(-dur))
print('ideal %.0f inorder %.0f (eff %.3f) LPT %.0f (eff %.3f)'%(ideal,M0,ideal/M0,Ml,ideal/Ml))
# predictor at iteration 25
def g(k,key,default): return np.array([x.get(key,default) for x in f],float)
alive=it>25
X=np.column_stack([np.log10(g(0,'pr25',1)), np.log10(g(0,'du25',1)), np.log10(g(0,'rho25',0.1)), g(0,'ru25',0)])
y=it
m=alive
A=np.column_stack([X[m],np.ones(m.sum())])
coef,*_=np.linalg.lstsq(A,y[m],rcond=None)
pred=np.full(len(it),0.0); pred[m]=A@coef
r2=1-np.sum((y[m]-pred[m])**2)/np.sum((y[m]-y[m].mean())**2)
print('R2 linear at iter 25 (alive robots):',r2)
# two-phase: phase A = setup + first factorization + min(it,25) iterations + first check
dA=15e3+54e3+3.7e3*np.minimum(it,25)+ 54e3*np.minimum(ru, g(0,'ru25',0))
dB=np.maximum(dur-dA,0)
MA=ls(dA,range(len(dA)))
restore=5e3
dBr=np.where(alive,dB+restore,0)
for name,order in [('pred',np.argsort(-pred)),('inorder',range(len(dB))),('oracle',np.argsort(-dBr))]:
    MB=ls(dBr,[i for i in order if alive[i]])
    print('two-phase %s: A %.0f + B %.0f = %.0f (vs inorder %.0f): gain %.3f'%(name,MA,MB,MA+MB,M0,M0/(MA+MB)))
print('--- cut at 50')
alive=it>50
F=lambda key,d: np.log10(np.maximum(g(0,key,d),1e-30))
X=np.column_stack([F('pr25',1),F('du25',1),F('pr50',1),F('du50',1),F('rho50',0.1),F('rho25',0.1),g(0,'ru25',0)])
m=alive
A=np.column_stack([X[m],np.ones(m.sum())])
coef,*_=np.linalg.lstsq(A,y[m],rcond=None)
pred=np.full(len(it),0.0); pred[m]=A@coef
r2=1-np.sum((y[m]-pred[m])**2)/np.sum((y[m]-y[m].mean())**2)
print('R2 linear at iter 50:',r2)
# rate-based predictor: remaining ~ max over (log(pr50)/rate_p, log(du50)/rate_d)
rp=(F('pr25',1)-F('pr50',1))/25; rd=(F('du25',1)-F('du50',1))/25
rem=np.maximum(np.where(rp>1e-3,F('pr50',1)/np.maximum(rp,1e-3),400), np.where(rd>1e-3,F('du50',1)/np.maximum(rd,1e-3),400))
c2=np.corrcoef(np.minimum(rem[m],500),y[m])[0,1]
print('corr rate-predictor', c2)
ru50 = np.array([0]*len(it))
dA=15e3+54e3+3.7e3*np.minimum(it,50)+54e3*np.minimum(ru,1)
dB=np.maximum(dur-dA,0)
MA=ls(dA,range(len(dA)))
dBr=np.where(alive,dB+5e3,0)
for name,order in [('pred',np.argsort(-pred)),('rate',np.argsort(-rem)),('oracle',np.argsort(-dBr))]:
    MB=ls(dBr,[i for i in order if alive[i]])
    print('two-phase50 %s: A %.0f + B %.0f = %.0f: gain %.3f'%(name,MA,MB,MA+MB,M0/(MA+MB)))
rng=np.random.default_rng(0)
for name,order in [('inorder',range(len(dB))),('random',rng.permutation(len(dB))),('rev-inorder',range(len(dB)-1,-1,-1))]:
    MB=ls(dBr,[i for i in order if alive[i]])
    print('two-phase50 %s: A %.0f + B %.0f = %.0f: gain %.3f'%(name,MA,MB,MA+MB,M0/(MA+MB)))
for cut in (75,100):
    alive=it>cut
    dA=15e3+54e3+3.7e3*np.minimum(it,cut)+54e3*np.minimum(ru,1)
    dB=np.maximum(dur-dA,0); dBr=np.where(alive,dB+5e3,0)
    MA=ls(dA,range(len(dA)))
    for name,order in [('inorder',range(len(dB))),('oracle',np.argsort(-dBr))]:
        MB=ls(dBr,[i for i in order if alive[i]])
        print('two-phase%d %s: A %.0f + B %.0f = %.0f: gain %.3f'%(cut,name,MA,MB,MA+MB,M0/(MA+MB)))
print('--- single features at 50')
alive=it>50; m=alive
for key in ['pr25','du25','pr50','du50','rho25','rho50']:
    x=F(key,1)
    print(key, 'corr %.3f'%np.corrcoef(x[m],y[m])[0,1])
x=np.maximum(F('pr50',1),F('du50',1)); print('max(pr50,du50) corr %.3f'%np.corrcoef(x[m],y[m])[0,1])
x=F('pr50',1)+F('du50',1); print('sum corr %.3f'%np.corrcoef(x[m],y[m])[0,1])
print('coef', coef)
print('--- pessimistic: restore 15k, gap 44k cycles, cut 50, linear pred')
alive=it>50; m=alive
X=np.column_stack([F('pr25',1),F('du25',1),F('pr50',1),F('du50',1),F('rho50',0.1),F('rho25',0.1),g(0,'ru25',0)])
A=np.column_stack([X[m],np.ones(m.sum())]); coef,*_=np.linalg.lstsq(A,y[m],rcond=None)
pred=np.full(len(it),0.0); pred[m]=A@coef
dA=15e3+54e3+3.7e3*np.minimum(it,50)+54e3*np.minimum(ru,1)
dB=np.maximum(dur-dA,0)
for rest in (5e3,15e3,30e3):
    dBr=np.where(alive,dB+rest,0)
    MA=ls(dA,range(len(dA))); MB=ls(dBr,[i for i in np.argsort(-pred) if alive[i]])
    print('restore %.0fk: gain %.3f'%(rest/1e3, M0/(MA+MB+44e3)))
# simple predictor: du50 alone
dBr=np.where(alive,dB+15e3,0)
for name,key in [('du50',F('du50',1)),('sum50',F('pr50',1)+F('du50',1))]:
    MB=ls(dBr,[i for i in np.argsort(-key) if alive[i]])
    print('pred %s restore 15k: gain %.3f'%(name, M0/(MA+MB+44e3)))
print('--- predictor potential at cut 50 (restore 15k)')
alive=it>50; m=alive
dA=15e3+54e3+3.7e3*np.minimum(it,50)+54e3*np.minimum(ru,1)
dB=np.maximum(dur-dA,0); dBr=np.where(alive,dB+15e3,0)
MA=ls(dA,range(len(dA)))
def mb(order): return ls(dBr,[i for i in order if alive[i]])
print('oracle LPT MB', mb(np.argsort(-dBr)))
print('du50 MB', mb(np.argsort(-F('du50',1))))
from sklearn.ensemble import GradientBoostingRegressor
from sklearn.model_selection import cross_val_predict
feats=np.column_stack([F('pr25',1),F('du25',1),F('pr50',1),F('du50',1),F('rho50',0.1),F('rho25',0.1),g(0,'ru25',0)])
gb=GradientBoostingRegressor(n_estimators=200,max_depth=3)
pred=np.zeros(len(it)); pred[m]=cross_val_predict(gb,feats[m],dBr[m],cv=5)
r2=1-np.sum((dBr[m]-pred[m])**2)/np.sum((dBr[m]-dBr[m].mean())**2)
print('GBR R2 %.3f MB'%r2, mb(np.argsort(-pred)))
