#!/usr/bin/env python3
"""Fixed-work solve for per-iteration cost measurements: every robot runs exactly --iters ADMM
iterations (eps 0, adaptive rho off, so no early exit and one factorization).  Run it under
rocprofv3 --pmc for two iteration counts; the counter difference / iteration difference is the
cost of one ADMM iteration (plus 1/25 of a termination check), unperturbed by instrumentation.

  rocprofv3 --pmc SQ_INSTS_VALU ... -- python3 tools/iter_cost.py --iters 100
"""
import argparse
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "go1-qp-mpc-controller_amd"))
import mpcqp  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=100)
    ap.add_argument("--batch", type=int, default=4096)
    ap.add_argument("--horizon", type=int, default=10)
    ap.add_argument("--reps", type=int, default=3)
    a = ap.parse_args()
    p = mpcqp.default_params(a.horizon, max_iter=a.iters, eps_abs=0.0, eps_rel=0.0, adaptive_rho=0,
                             eps_prim_inf=0.0, eps_dual_inf=0.0)
    st = mpcqp.synthetic_go1(a.batch, seed=1000, gait="trot")
    recs = mpcqp.assemble_compute_grf(st, a.horizon)
    d_rec = torch.from_numpy(recs).cuda()
    d_res = torch.zeros((a.batch, mpcqp._lib.RESULT_DOUBLES), dtype=torch.float64, device="cuda")
    with mpcqp.MpcQpSolver(p) as s:
        stream = torch.cuda.current_stream().cuda_stream
        for _ in range(a.reps):
            s.solve_device(d_rec.data_ptr(), a.batch, d_res.data_ptr(), 0, stream)
        torch.cuda.synchronize()
    res = np.frombuffer(d_res.cpu().numpy().tobytes(), dtype=mpcqp.RESULT_DTYPE)
    print("iters", np.unique(res["iters"]), "rho_updates", np.unique(res["rho_updates"]))


if __name__ == "__main__":
    main()
