#!/usr/bin/env python3
"""Batch split of the wave-path solve (mpcqp_debug_set_split): one batch solved as K parts on the
handle's internal streams, forked from and joined to the caller's stream.  Prints ms per step and
QP/s for each K (HIP events on the caller's stream, steps do not overlap) and whether the results
are bitwise those of K = 1.

  python tools/split_exp.py [--batch 4096] [--horizon 10] [--gait trot] [--mixed-mu] [--ks 1 2 4 8]
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
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--batch", type=int, default=4096)
    ap.add_argument("--horizon", type=int, default=10)
    ap.add_argument("--gait", default="trot")
    ap.add_argument("--mixed-mu", action="store_true")
    ap.add_argument("--seed", type=int, default=1000)
    ap.add_argument("--ks", type=int, nargs="*", default=[1, 2, 3, 4, 6, 8, 0])
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    st = mpcqp.synthetic_go1(a.batch, seed=a.seed, gait=a.gait, mixed_mu=a.mixed_mu)
    recs = torch.from_numpy(mpcqp.assemble_compute_grf(st, a.horizon)).to(dev)
    RD = mpcqp._lib.RESULT_DOUBLES
    stream = torch.cuda.current_stream(dev)
    ref = None
    with mpcqp.MpcQpSolver(mpcqp.default_params(a.horizon), device=0) as s:
        s.reserve(a.batch)
        res = torch.zeros((a.batch, RD), dtype=torch.float64, device=dev)
        for K in a.ks:
            s.set_split(K)

            def step():
                s.solve_device(recs.data_ptr(), a.batch, res.data_ptr(), 0, stream.cuda_stream)

            for _ in range(3):
                step()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            times = []
            for _ in range(a.steps):
                e0.record(stream)
                step()
                e1.record(stream)
                torch.cuda.synchronize()
                times.append(e0.elapsed_time(e1))
            out = res.cpu().numpy().copy()
            if ref is None:
                ref = out
            same = bool(np.array_equal(out.view(np.uint64), ref.view(np.uint64)))
            ms = float(np.median(times))
            print(f"batch {a.batch} N={a.horizon} {a.gait}{' mixed-mu' if a.mixed_mu else ''} K={K}: "
                  f"{ms:.4f} ms per step (median of {a.steps}), {a.batch / ms * 1e3:.0f} QP/s, "
                  f"bitwise equal to K={a.ks[0]}: {same}, hand-off {s.handoff_counts()}", flush=True)


if __name__ == "__main__":
    main()
