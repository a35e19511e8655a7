#!/usr/bin/env python3
"""Phase cost breakdown of solve_kernel by timing settings that isolate each phase.

  A: max_iter=1, adaptive_rho=0                 condensation + Ruiz + 1 inverse + 1 iteration
  B: A with scaling=0                           condensation + 1 inverse + 1 iteration
  C: max_iter=101, eps=0, adaptive_rho=0        A + 100 ADMM iterations (no refactor)
  D: default settings                           production
  Q: build_qp kernel alone                      condensation (256-thread variant) + H/g/l/u writes
Prints per-instance-per-CU microseconds (kernel time * CUs / batch) and per-iteration cost.
"""
import argparse
import json
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "go1-qp-mpc-controller_amd"))
import mpcqp  # noqa: E402


def time_solve(params, recs, reps=5):
    B = recs.shape[0]
    with mpcqp.MpcQpSolver(params) as s:
        d_rec = torch.from_numpy(recs).cuda()
        d_res = torch.zeros((B, mpcqp._lib.RESULT_DOUBLES), dtype=torch.float64, device="cuda")
        st = torch.cuda.current_stream().cuda_stream
        s.solve_device(d_rec.data_ptr(), B, d_res.data_ptr(), 0, st)
        torch.cuda.synchronize()
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(reps)]
        for a, b in ev:
            a.record()
            s.solve_device(d_rec.data_ptr(), B, d_res.data_ptr(), 0, st)
            b.record()
        torch.cuda.synchronize()
        ms = float(np.median([a.elapsed_time(b) for a, b in ev]))
        res = np.frombuffer(d_res.cpu().numpy().tobytes(), dtype=mpcqp.RESULT_DTYPE)
        return ms, res


def time_build(params, recs, reps=5):
    B = recs.shape[0]
    n, m = 12 * params.horizon, 20 * params.horizon
    with mpcqp.MpcQpSolver(params) as s:
        d_rec = torch.from_numpy(recs).cuda()
        P = torch.empty((B, n, n), dtype=torch.float64, device="cuda")
        q = torch.empty((B, n), dtype=torch.float64, device="cuda")
        l = torch.empty((B, m), dtype=torch.float64, device="cuda")
        u = torch.empty((B, m), dtype=torch.float64, device="cuda")
        st = torch.cuda.current_stream().cuda_stream
        args = (d_rec.data_ptr(), B, P.data_ptr(), q.data_ptr(), l.data_ptr(), u.data_ptr(), st)
        s.build_qp_device(*args)
        torch.cuda.synchronize()
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(reps)]
        for a, b in ev:
            a.record()
            s.build_qp_device(*args)
            b.record()
        torch.cuda.synchronize()
        return float(np.median([a.elapsed_time(b) for a, b in ev]))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=4096)
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    cus = torch.cuda.get_device_properties(0).multi_processor_count
    st = mpcqp.synthetic_go1(a.batch, seed=1000, gait="trot")
    recs = mpcqp.assemble_compute_grf(st, 10)
    B = a.batch
    with mpcqp.MpcQpSolver(mpcqp.default_params(10)) as s:
        slots = s.slots
    per = lambda ms: ms * 1e3 * min(slots, B) / B  # µs of a resident slot per instance  # noqa: E731
    out = {"batch": B, "cus": cus, "slots": slots, "threads": mpcqp.load().mpcqp_solve_threads(10)}
    A, _ = time_solve(mpcqp.default_params(10, max_iter=1, adaptive_rho=0), recs)
    Bt, _ = time_solve(mpcqp.default_params(10, max_iter=1, adaptive_rho=0, scaling=0), recs)
    C, _ = time_solve(mpcqp.default_params(10, max_iter=101, adaptive_rho=0, eps_abs=0.0, eps_rel=0.0), recs)
    D, res = time_solve(mpcqp.default_params(10), recs)
    Q = time_build(mpcqp.default_params(10), recs)
    out.update({
        "ms": {"A_setup_1iter": A, "B_noscale": Bt, "C_101iter": C, "D_default": D, "Q_build": Q},
        "us_per_instance_slot": {"setup(cond+ruiz+inv+1it)": per(A), "ruiz": per(A - Bt),
                                 "iteration": per(C - A) / 100, "default_total": per(D),
                                 "condense_buildkernel": Q * 1e3 * cus / B},
        "mean_iters": float(res["iters"].mean()), "mean_rho_updates": float(res["rho_updates"].mean()),
    })
    it = out["us_per_instance_slot"]
    est_inv = per(Bt) - it["iteration"]  # condense + inverse
    out["us_per_instance_slot"]["condense+inverse"] = est_inv
    print(json.dumps(out, indent=1))
    if a.out:
        with open(a.out, "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
