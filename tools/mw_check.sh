set -uo pipefail
O=gpurun_out/r2q; mkdir -p $O
timeout -k 10 200 python -u - > $O/mw_parity.txt 2>&1 << 'PY'
import sys, numpy as np, torch
sys.path[:0] = ['go1-qp-mpc-controller_amd', 'oracle', 'tests']
import mpcqp, pyoracle as o
from gpu_helpers import solve_gpu, rel_err_u0
for N in (10, 4, 1, 2, 7, 20):
    for gait in ('trot', 'mixed'):
        st = mpcqp.synthetic_go1(256, seed=5 + N, gait=gait, mixed_mu=(gait == 'mixed'))
        recs = mpcqp.assemble_compute_grf(st, N)
        p = mpcqp.default_params(N)
        with mpcqp.MpcQpSolver(p) as s:
            s.set_solver(4)
            got, _, _ = solve_gpu(s, recs)
        ref = o.solve_batch(o.default_params(N), recs, nthreads=8)
        err = rel_err_u0(got['u0'], ref['u0'])
        print(N, gait, 'maxerr', float(err.max()), 'status_eq', bool((got['status'] == ref['status']).all()),
              'iters_eq', float((got['iters'] == ref['iters']).mean()), flush=True)
PY
timeout -k 10 200 python bench.py --solver mw > $O/bench_mw.json 2> $O/bench_mw.err
python -c "import json; d=json.load(open('$O/bench_mw.json')); print(d['value'], d['ms_per_step'], d['parity'])"
