"""Balance-controller measurement: balance QPs/s on one MI355X for a batch
of seeded Go1 robots (HIP events around mpcqp_balance_solve_device, inputs resident in HBM),
parity vs the CPU oracle on a sample, and the oracle's rate on host threads.
usage: python tools/balance_bench.py [--batch B] [--steps K] [--gait mixed]"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "go1-qp-mpc-controller_amd"), os.path.join(REPO, "oracle")]
import mpcqp  # noqa: E402
from mpcqp import balance as bal  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=65536)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--gait", default="trot")
    ap.add_argument("--cpu-sample", type=int, default=4096)
    a = ap.parse_args()
    B = a.batch
    recs = bal.assemble_balance(mpcqp.synthetic_go1(B, seed=2024, gait=a.gait))
    s = mpcqp.MpcQpSolver(mpcqp.default_params(1))
    bp = mpcqp._lib.default_balance_params()
    d_rec = torch.from_numpy(recs).cuda()
    d_res = torch.zeros((B, mpcqp._lib.RESULT_DOUBLES), dtype=torch.float64, device="cuda")
    st = torch.cuda.current_stream()
    for _ in range(a.warmup):
        s.balance_solve_device(bp, d_rec.data_ptr(), B, d_res.data_ptr(), st.cuda_stream)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(st)
    for _ in range(a.steps):
        s.balance_solve_device(bp, d_rec.data_ptr(), B, d_res.data_ptr(), st.cuda_stream)
    e1.record(st)
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / a.steps
    got = np.frombuffer(d_res.cpu().numpy().tobytes(), dtype=mpcqp.RESULT_DTYPE)
    import pyoracle as po  # checker / CPU baseline only
    n = min(a.cpu_sample, B)
    th = min(16, os.cpu_count() or 1)
    t0 = time.perf_counter()
    ref = po.balance_solve_batch(po.default_params(1), po.default_balance_params(), recs[:n], th)
    cpu_s = time.perf_counter() - t0
    err = np.abs(got["u0"][:n] - ref["u0"]).max(1) / np.maximum(np.abs(ref["u0"]).max(1), 1.0)
    print(json.dumps({
        "metric": "balance QP solves/sec (12 vars, 20 rows, fresh OSQP per tick)", "value": B / (ms * 1e-3),
        "unit": "QP/s", "batch": B, "gait": a.gait, "ms_per_launch": ms, "dtype": "f64",
        "cpu_baseline": {"value": n / cpu_s, "unit": "QP/s", "cores": th, "kind": "port",
                         "sample": f"first {n} robots on oracle/mpc_oracle.c orc_balance_solve"},
        "parity": {"max_rel_err_u0": float(err.max()), "status_equal": bool((got["status"][:n] == ref["status"]).all()),
                   "iters_equal": bool((got["iters"][:n] == ref["iters"]).all())},
        "stats": {"mean_iters": float(got["iters"].mean()), "max_iters": int(got["iters"].max()),
                  "solved_frac": float((got["status"] == 1).mean())}}))
    s.close()


if __name__ == "__main__":
    main()
