#!/usr/bin/env python3
"""Median shader cycles between consecutive phase marks of the first factorization (marks 14 .. 15,
including the MFMA Gauss-Jordan's internal marks 60-64) on a -DMPCQP_PHASE_TIMING library
(MPCQP_LIB).  usage: python tools/gj_marks.py [--horizon 10]"""
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
    ap.add_argument("--horizon", type=int, default=10)
    ap.add_argument("--batch", type=int, default=4096)
    ap.add_argument("--traced", type=int, default=256)
    a = ap.parse_args()
    st = mpcqp.synthetic_go1(a.batch, seed=1000, gait="trot")
    recs = mpcqp.assemble_compute_grf(st, a.horizon)
    with mpcqp.MpcQpSolver(mpcqp.default_params(a.horizon)) as s:
        d_rec = torch.from_numpy(recs).cuda()
        d_res = torch.zeros((a.batch, mpcqp._lib.RESULT_DOUBLES), dtype=torch.float64, device="cuda")
        tr = torch.full((a.traced, 64, 4), float("nan"), dtype=torch.float64, device="cuda")
        stream = torch.cuda.current_stream().cuda_stream
        s.solve_device_trace(d_rec.data_ptr(), a.batch, d_res.data_ptr(), 0, tr.data_ptr(), a.traced, stream)
        torch.cuda.synchronize()
        marks = tr.cpu().numpy()
    seqs = {}
    for b in range(a.traced):
        mk = marks[b]
        mk = mk[~np.isnan(mk[:, 0])]
        ids, cyc = mk[:, 0].astype(int), mk[:, 1]
        if 14 not in ids:
            continue
        i0 = list(ids).index(14)
        i1 = i0 + list(ids[i0:]).index(15)
        for n, i in enumerate(range(i0, i1)):
            seqs.setdefault((n, ids[i], ids[i + 1]), []).append(cyc[i + 1] - cyc[i])
    tot = 0.0
    for (n, x, y), v in sorted(seqs.items()):
        m = float(np.median(v))
        tot += m
        print(f"{n:3d}  {x:3d} -> {y:3d}  {m:9.0f} cycles  ({len(v)} robots)")
    print(f"total 14 -> 15: {tot:.0f} cycles")


if __name__ == "__main__":
    main()
