"""Per-robot iteration counts, rho updates and check residuals of the C2 bench batch (oracle trace),
for the dispatch-tail scheduling simulations (tools/r06_sched_sim.py, profiles/r06/park)."""
import json
import sys, numpy as np, heapq
sys.path[:0]=['go1-qp-mpc-controller_amd','oracle']
import mpcqp, pyoracle
N=10
st=mpcqp.synthetic_go1(4096,seed=1000,gait='trot'); recs=mpcqp.assemble_compute_grf(st,N)
p=pyoracle.default_params(N)
rows=[]
for b in range(4096):
    out,_,tr=pyoracle.solve(p,recs[b],trace=True)
    f={}
    for e in tr:
        if e[0]==25: f['pr25']=e[2]/e[4]; f['du25']=e[3]/e[5]; f['rho25']=e[6]; f['ru25']=e[1]
        if e[0]%25==0: f["pr%d"%e[0]]=e[2]/e[4]; f["du%d"%e[0]]=e[3]/e[5]; f["rho%d"%e[0]]=e[6]
    rows.append((out['iters'],out['rho_updates'],f))
json.dump([[int(a), int(b), c] for a, b, c in rows], open('profiles/r06/park/iters_checks.json', 'w'))
