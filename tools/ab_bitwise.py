#!/usr/bin/env python3
"""Bitwise A/B of two libmpcqp builds: `python tools/ab_bitwise.py dump OUT.npz` (library chosen with
MPCQP_LIB) solves C2 (4096 trot robots, N = 10), a C5 sample (2048 mixed-gait robots, random mu),
a C4 sample (1024 robots, N = 20) and 6 warm-started ticks of 512 robots, and stores the raw result
records and solutions; `python tools/ab_bitwise.py cmp A.npz B.npz` reports which arrays differ."""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "go1-qp-mpc-controller_amd"))


def dump(out):
    import torch
    import mpcqp
    res = {}
    cases = [("c2", 10, mpcqp.synthetic_go1(4096, seed=1000, gait="trot")),
             ("c5", 10, mpcqp.synthetic_go1(2048, seed=5, gait="mixed", mixed_mu=True)),
             ("c4", 20, mpcqp.synthetic_go1(1024, seed=1000, gait="trot"))]
    stream = torch.cuda.current_stream().cuda_stream
    for name, N, st in cases:
        recs = mpcqp.assemble_compute_grf(st, N)
        B = recs.shape[0]
        with mpcqp.MpcQpSolver(mpcqp.default_params(N)) as s:
            d_rec = torch.from_numpy(recs).cuda()
            d_res = torch.zeros((B, mpcqp._lib.RESULT_DOUBLES), dtype=torch.float64, device="cuda")
            d_sol = torch.zeros((B, 12 * N), dtype=torch.float64, device="cuda")
            s.solve_device(d_rec.data_ptr(), B, d_res.data_ptr(), d_sol.data_ptr(), stream)
            torch.cuda.synchronize()
            res[name + "_res"] = d_res.cpu().numpy()
            res[name + "_sol"] = d_sol.cpu().numpy()
    T, B, N = 6, 512, 10
    ticks = mpcqp.records.synthetic_go1_ticks(B, T, seed=61, gait="trot", swing_ticks=3)
    with mpcqp.MpcQpSolver(mpcqp.default_params(N)) as s:
        d_state = torch.zeros((B, s.warm_state_size), dtype=torch.float64, device="cuda")
        d_res = torch.zeros((B, mpcqp._lib.RESULT_DOUBLES), dtype=torch.float64, device="cuda")
        for t in range(T):
            d_rec = torch.from_numpy(mpcqp.assemble_compute_grf(ticks[t], N)).cuda()
            s.solve_warm_device(d_rec.data_ptr(), B, d_state.data_ptr(), d_res.data_ptr(), 0, stream)
            torch.cuda.synchronize()
            res[f"warm{t}_res"] = d_res.cpu().numpy()
        res["warm_state"] = d_state.cpu().numpy()
    np.savez(out, **res)
    print("dumped", out, sorted(res))


def cmp(a, b):
    A, B = np.load(a), np.load(b)
    bad = 0
    for k in sorted(A.files):
        same = A[k].tobytes() == B[k].tobytes()
        bad += not same
        print(f"{k:12s} {'bitwise equal' if same else 'DIFFERS'}")
    print("ALL EQUAL" if bad == 0 else f"{bad} arrays differ")
    return bad


if __name__ == "__main__":
    if sys.argv[1] == "dump":
        dump(sys.argv[2])
    else:
        sys.exit(1 if cmp(sys.argv[2], sys.argv[3]) else 0)
