#!/usr/bin/env python3
"""Randomized parity sweep of the product solve against the CPU oracle (test infrastructure, run on
a GPU box): many seeds x gaits x horizons x weight scalings, cold solves; per case the fraction of
robots whose status and iteration count equal the oracle's and the worst u0 relative error.
  python tools/fuzz_parity.py [--seeds 8] [--batch 512] [--out file.json]"""
import argparse
import json
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "go1-qp-mpc-controller_amd"))
sys.path.insert(0, os.path.join(REPO, "oracle"))
import mpcqp  # noqa: E402
import pyoracle  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seeds", type=int, default=8)
    ap.add_argument("--batch", type=int, default=512)
    ap.add_argument("--out", default="")
    ap.add_argument("--horizons", default="10,20")
    ap.add_argument("--gaits", default="trot,stance,mixed")
    ap.add_argument("--scales", default="1,100,0.01")
    a = ap.parse_args()
    pyoracle.build()
    nthr = min(16, os.cpu_count() or 1)
    rows = []
    worst = {"iters_equal_frac": 1.0, "max_rel_err_u0": 0.0}
    for N in [int(x) for x in a.horizons.split(",")]:
        for gait in a.gaits.split(","):
            mixed = gait == "mixed"
            for wscale in [float(x) for x in a.scales.split(",")]:
                for seed in range(a.seeds):
                    st = mpcqp.synthetic_go1(a.batch, seed=7000 + 97 * seed + N, gait=gait, mixed_mu=mixed)
                    recs = mpcqp.assemble_compute_grf(st, N)
                    p0 = mpcqp.default_params(N)
                    kw = {"q_weights": [w * wscale for w in p0.q_weights]}
                    p = mpcqp.default_params(N, **kw)
                    with mpcqp.MpcQpSolver(p) as s:
                        d_rec = torch.from_numpy(recs).cuda()
                        d_res = torch.zeros((a.batch, mpcqp._lib.RESULT_DOUBLES), dtype=torch.float64, device="cuda")
                        s.solve_device(d_rec.data_ptr(), a.batch, d_res.data_ptr(), 0,
                                       torch.cuda.current_stream().cuda_stream)
                        torch.cuda.synchronize()
                        got = np.frombuffer(d_res.cpu().numpy().tobytes(), dtype=mpcqp.RESULT_DTYPE)
                    op = pyoracle.default_params(N, q=list(p.q_weights), r=list(p.r_weights))
                    ref = pyoracle.solve_batch(op, recs, nthreads=nthr)
                    err = np.max(np.abs(got["u0"] - ref["u0"]), axis=1) / np.maximum(np.max(np.abs(ref["u0"]), axis=1), 1.0)
                    row = {"N": N, "gait": gait, "q_scale": wscale, "seed": seed,
                           "status_equal_frac": float(np.mean(got["status"] == ref["status"])),
                           "iters_equal_frac": float(np.mean(got["iters"] == ref["iters"])),
                           "max_rel_err_u0": float(np.max(err)), "mean_iters": float(got["iters"].mean())}
                    rows.append(row)
                    worst["iters_equal_frac"] = min(worst["iters_equal_frac"], row["iters_equal_frac"])
                    worst["max_rel_err_u0"] = max(worst["max_rel_err_u0"], row["max_rel_err_u0"])
                    print(json.dumps(row), flush=True)
    out = {"cases": len(rows), "robots": len(rows) * a.batch, "worst": worst, "rows": rows}
    print(json.dumps({"cases": out["cases"], "robots": out["robots"], "worst": worst}))
    if a.out:
        json.dump(out, open(a.out, "w"), indent=1)


if __name__ == "__main__":
    main()
