#!/usr/bin/env python3
"""Experiment: one C2 batch (4096 trot robots, N = 10) solved as K sub-batches on K handles and
streams, launched together every step and joined before the next step (steps do not overlap), so
that one part's scale_kernel can run beside another part's wave_kernel and the parts' dispatch
tails interleave.  Prints ms per step for each K (HIP events on the joining stream).

  python tools/split_exp.py [--steps 20] [--ks 1 2 4]
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
    ap.add_argument("--ks", type=int, nargs="*", default=[1, 2, 4])
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    st = mpcqp.synthetic_go1(a.batch, seed=1000, gait="trot")
    recs = torch.from_numpy(mpcqp.assemble_compute_grf(st, 10)).to(dev)
    RD = mpcqp._lib.RESULT_DOUBLES
    main_stream = torch.cuda.current_stream(dev)
    ref = None
    for K in a.ks:
        per = a.batch // K
        solvers = [mpcqp.MpcQpSolver(mpcqp.default_params(10), device=0) for _ in range(K)]
        streams = [torch.cuda.Stream(dev) for _ in range(K)]
        res = torch.zeros((a.batch, RD), dtype=torch.float64, device=dev)
        for s in solvers:
            s.reserve(per)

        def step():
            for i, (s, sm) in enumerate(zip(solvers, streams)):
                sm.wait_stream(main_stream)
                s.solve_device(recs[i * per:].data_ptr(), per, res[i * per:].data_ptr(), 0, sm.cuda_stream)
            for sm in streams:
                main_stream.wait_stream(sm)

        for _ in range(3):
            step()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        times = []
        for _ in range(a.steps):
            e0.record(main_stream)
            step()
            e1.record(main_stream)
            torch.cuda.synchronize()
            times.append(e0.elapsed_time(e1))
        out = res.cpu().numpy()
        if ref is None:
            ref = out
        same = bool(np.array_equal(out.view(np.uint64), ref.view(np.uint64)))
        ms = float(np.median(times))
        print(f"K={K}: {ms:.4f} ms per step (median of {a.steps}), {a.batch / ms * 1e3:.0f} QP/s, "
              f"bitwise equal to K={a.ks[0]}: {same}", flush=True)
        for s in solvers:
            s.close()


if __name__ == "__main__":
    main()
