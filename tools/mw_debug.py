"""Compares wave_kernel (path 3) and mw_kernel (path 4) intermediates after max_iter iterations.
Run with MPCQP_LIB pointing at a -DMPCQP_DBG=<d> variant (1 G, 2 h, 3 x, 4 s, 5 w)."""
import os, sys, numpy as np
sys.path[:0] = ['go1-qp-mpc-controller_amd', 'oracle', 'tests']
import mpcqp
from gpu_helpers import solve_gpu
N = int(sys.argv[1]) if len(sys.argv) > 1 else 2
st = mpcqp.synthetic_go1(4, seed=7, gait='trot')
recs = mpcqp.assemble_compute_grf(st, N)
np.set_printoptions(precision=4, linewidth=220)
print('lib', os.environ.get('MPCQP_LIB'))
for mi in (1,):
    p = mpcqp.default_params(N, max_iter=mi)
    out = {}
    for path in (3, 4):
        with mpcqp.MpcQpSolver(p) as s:
            s.set_solver(path)
            r, sol, _ = solve_gpu(s, recs)
        out[path] = sol.reshape(4, N, 12)
    for k in range(N):
        print('step', k, 'wave', out[3][0][k])
        print('step', k, 'mw  ', out[4][0][k])
