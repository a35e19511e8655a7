#!/usr/bin/env python3
"""Kernel time vs batch size (reveals how many robots actually run concurrently per CU)."""
import json
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "go1-qp-mpc-controller_amd"))
import mpcqp  # noqa: E402


def main():
    import argparse
    ap = argparse.ArgumentParser()
    ap.add_argument("--horizon", type=int, default=10)
    h = ap.parse_args().horizon
    out = {"horizon": h}
    st = mpcqp.synthetic_go1(4096, seed=1000, gait="trot")
    recs_all = mpcqp.assemble_compute_grf(st, h)
    with mpcqp.MpcQpSolver(mpcqp.default_params(h)) as s:
        out["slots"] = s.slots
        for B in [128, 256, 384, 512, 768, 1024, 1536, 2048, 4096]:
            d_rec = torch.from_numpy(np.ascontiguousarray(recs_all[:B])).cuda()
            d_res = torch.zeros((B, mpcqp._lib.RESULT_DOUBLES), dtype=torch.float64, device="cuda")
            stream = torch.cuda.current_stream().cuda_stream
            s.solve_device(d_rec.data_ptr(), B, d_res.data_ptr(), 0, stream)
            torch.cuda.synchronize()
            ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(5)]
            for a, b in ev:
                a.record()
                s.solve_device(d_rec.data_ptr(), B, d_res.data_ptr(), 0, stream)
                b.record()
            torch.cuda.synchronize()
            out[B] = round(float(np.median([a.elapsed_time(b) for a, b in ev])), 4)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
