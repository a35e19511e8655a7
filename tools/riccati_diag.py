#!/usr/bin/env python3
"""Riccati path vs oracle statistics (u0 error, iteration drift) and kernel time per horizon."""
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in ("go1-qp-mpc-controller_amd", "oracle", "tests"):
    sys.path.insert(0, os.path.join(REPO, p))
import numpy as np
import torch

import mpcqp
import pyoracle
from gpu_helpers import rel_err_u0, solve_gpu


def stats(N, path, gait, B=64, seed=5):
    st = mpcqp.synthetic_go1(B, seed=seed, gait=gait, mixed_mu=(gait == "mixed"))
    recs = mpcqp.assemble_compute_grf(st, N)
    with mpcqp.MpcQpSolver(mpcqp.default_params(N), debug=True) as s:
        s.set_solver(path)
        got, _, _ = solve_gpu(s, recs)
    op = pyoracle.default_params(N)
    ref = pyoracle.solve_batch(op, recs, nthreads=8)
    err = rel_err_u0(got["u0"], ref["u0"])
    di = got["iters"].astype(int) - ref["iters"].astype(int)
    print(f"N={N} path={path} {gait}: u0 err max {np.nanmax(err):.3e} med {np.median(err):.3e}; "
          f"status eq {np.mean(got['status'] == ref['status']):.3f}; iters eq {np.mean(di == 0):.3f} "
          f"drift [{di.min()},{di.max()}]; gpu iters mean {got['iters'].mean():.1f}", flush=True)


def timing(N, path, B=4096, reps=5):
    st = mpcqp.synthetic_go1(B, seed=9, gait="trot")
    recs = mpcqp.assemble_compute_grf(st, N)
    with mpcqp.MpcQpSolver(mpcqp.default_params(N), debug=True) as s:
        s.set_solver(path)
        s.reserve(B)
        d_rec = torch.from_numpy(recs).cuda()
        d_res = torch.zeros((B, mpcqp._lib.RESULT_DOUBLES), dtype=torch.float64, device="cuda")
        d_sol = torch.zeros((B, s.n), dtype=torch.float64, device="cuda")
        st_ = torch.cuda.current_stream().cuda_stream
        s.solve_device(d_rec.data_ptr(), B, d_res.data_ptr(), d_sol.data_ptr(), st_)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            s.solve_device(d_rec.data_ptr(), B, d_res.data_ptr(), d_sol.data_ptr(), st_)
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / reps
        print(f"timing N={N} path={path} B={B}: {ms:.3f} ms  {B / ms * 1e3:.0f} QP/s  slots {s.slots}", flush=True)


if __name__ == "__main__":
    pyoracle.build()
    for N, path in ((10, 2), (20, 2), (15, 2), (1, 2)):
        for gait in ("trot", "stance", "mixed"):
            stats(N, path, gait)
    for N, path in ((10, 1), (10, 2), (20, 2)):
        timing(N, path)
