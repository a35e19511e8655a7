#!/usr/bin/env python3
"""Per-robot start / end timeline of wave_kernel on the GPU: run a library built with
-DMPCQP_PHASE_TIMING -DMPCQP_PHASE_TIMING_ENDS (marks 0 and 20 only, plus the wave's HW_ID /
XCC_ID; `make -C go1-qp-mpc-controller_amd variant OUT=../variants/ends.so DEFS="..."`) selected
with MPCQP_LIB, trace every robot, and report how well the SIMD slots are kept busy: the kernel's
span, the sum of robot durations over the slots used, the busy fraction, the tail (time during which
fewer than half the slots still run) and the duration spread against the iteration count."""
import argparse
import json
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "go1-qp-mpc-controller_amd"))
import mpcqp  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=4096)
    ap.add_argument("--horizon", type=int, default=10)
    ap.add_argument("--order", default="none", choices=["none", "iters_desc", "iters_asc"])
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    st = mpcqp.synthetic_go1(a.batch, seed=1000, gait="trot")
    recs = mpcqp.assemble_compute_grf(st, a.horizon)
    with mpcqp.MpcQpSolver(mpcqp.default_params(a.horizon)) as s:
        d_rec = torch.from_numpy(recs).cuda()
        d_res = torch.zeros((a.batch, mpcqp._lib.RESULT_DOUBLES), dtype=torch.float64, device="cuda")
        tr = torch.full((a.batch, 64, 4), float("nan"), dtype=torch.float64, device="cuda")
        stream = torch.cuda.current_stream().cuda_stream
        if a.order != "none":  # reorder the batch by a first solve's iteration counts
            s.solve_device(d_rec.data_ptr(), a.batch, d_res.data_ptr(), 0, stream)
            torch.cuda.synchronize()
            it = np.frombuffer(d_res.cpu().numpy().tobytes(), dtype=mpcqp.RESULT_DTYPE)["iters"]
            perm = np.argsort(-it if a.order == "iters_desc" else it, kind="stable")
            d_rec = torch.from_numpy(np.ascontiguousarray(recs[perm])).cuda()
        for _ in range(3):
            tr.fill_(float("nan"))
            s.solve_device_trace(d_rec.data_ptr(), a.batch, d_res.data_ptr(), 0, tr.data_ptr(), a.batch, stream)
        torch.cuda.synchronize()
        mk = tr.cpu().numpy()
        res = np.frombuffer(d_res.cpu().numpy().tobytes(), dtype=mpcqp.RESULT_DTYPE)
    t0 = mk[:, 0, 2]  # mark 0, memrealtime (100 MHz)
    t1 = mk[:, 1, 2]  # mark 20
    c0, c1 = mk[:, 0, 1], mk[:, 1, 1]
    hw = mk[:, 0, 3].astype(np.uint64)
    hwid = hw & np.uint64(0xFFFFFFFF)
    xcc = hw >> np.uint64(32)
    simd = (hwid >> np.uint64(4)) & np.uint64(3)
    cu = (hwid >> np.uint64(8)) & np.uint64(15)
    sh = (hwid >> np.uint64(12)) & np.uint64(1)
    se = (hwid >> np.uint64(13)) & np.uint64(7)
    slot = (((xcc * np.uint64(8) + se) * np.uint64(2) + sh) * np.uint64(16) + cu) * np.uint64(4) + simd
    cus = (((xcc * np.uint64(8) + se) * np.uint64(2) + sh) * np.uint64(16) + cu)
    dur = (t1 - t0) * 10.0  # ns
    span = (t1.max() - t0.min()) * 10.0
    nslots = len(np.unique(slot))
    busy = dur.sum() / (nslots * span)
    # tail: time from the moment half the slots have gone idle for good to the end
    last_end = {}
    for sl, e in zip(slot, t1):
        last_end[sl] = max(last_end.get(sl, 0), e)
    ends = np.sort(np.array(list(last_end.values())))
    half = ends[len(ends) // 2]
    tail = (t1.max() - half) * 10.0
    per_slot = np.array([dur[slot == sl].sum() for sl in np.unique(slot)])
    it = res["iters"].astype(float)
    out = {
        "span_us": span / 1e3,
        "slots": int(nslots),
        "cus": int(len(np.unique(cus))),
        "xccs": int(len(np.unique(xcc))),
        "robots_per_slot_max": int(np.bincount(np.unique(slot, return_inverse=True)[1]).max()),
        "busy_fraction": float(busy),
        "ideal_span_us": float(dur.sum() / nslots / 1e3),
        "tail_half_idle_us": tail / 1e3,
        "slot_work_us": {"min": per_slot.min() / 1e3, "median": float(np.median(per_slot)) / 1e3,
                         "max": per_slot.max() / 1e3},
        "robot_us": {"min": dur.min() / 1e3, "median": float(np.median(dur)) / 1e3, "max": dur.max() / 1e3},
        "cycles_per_iter_fit": float(np.polyfit(it, c1 - c0, 1)[0]),
        "cycles_fixed_fit": float(np.polyfit(it, c1 - c0, 1)[1]),
        "order": a.order,
    }
    print(json.dumps(out, indent=1))
    if a.out:
        with open(a.out, "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
