#!/usr/bin/env python3
"""In-kernel phase timing of the default solve (wave_kernel): run a library built with
-DMPCQP_PHASE_TIMING (`make -C go1-qp-mpc-controller_amd variant OUT=../abtest/timing.so
DEFS=-DMPCQP_PHASE_TIMING`, selected with MPCQP_LIB) and report median shader-clock cycles per
robot: setup (marks 0 -> 4), each factorization (10 -> 12), the mean ADMM iteration (loop time
minus factorizations over the iteration count) and, inside iteration 60, the KKT solve (40 -> 45),
the ADMM update (45 -> 46) and the rest of the iteration (46 -> 47); the termination check of
iteration 75 (48 -> 49: P~x 48 -> 50, norms and reductions 50 -> 51, termination / infeasibility
tests and adapt_rho 51 -> 52, the rest 52 -> 49)."""
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
    ap.add_argument("--traced", type=int, default=512)
    ap.add_argument("--horizon", type=int, default=10)
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    st = mpcqp.synthetic_go1(a.batch, seed=1000, gait="trot")
    recs = mpcqp.assemble_compute_grf(st, a.horizon)
    with mpcqp.MpcQpSolver(mpcqp.default_params(a.horizon)) as s:
        d_rec = torch.from_numpy(recs).cuda()
        d_res = torch.zeros((a.batch, mpcqp._lib.RESULT_DOUBLES), dtype=torch.float64, device="cuda")
        tr = torch.full((a.traced, 64, 4), float("nan"), dtype=torch.float64, device="cuda")
        stream = torch.cuda.current_stream().cuda_stream
        for _ in range(2):
            tr.fill_(float("nan"))
            s.solve_device_trace(d_rec.data_ptr(), a.batch, d_res.data_ptr(), 0, tr.data_ptr(), a.traced, stream)
        torch.cuda.synchronize()
        marks = tr.cpu().numpy().reshape(a.traced, 64, 4)
        res = np.frombuffer(d_res.cpu().numpy().tobytes(), dtype=mpcqp.RESULT_DTYPE)
    ph = {k: [] for k in ("setup", "factor", "f_pre", "fp_rprime", "fp_rinv", "fp_b6r_g", "fp_chol", "fp_bvw",
                          "fp_write", "f_buildS", "f_gj", "f_post", "iter_cycles", "check75", "ck_px", "ck_norms", "ck_tests", "ck_tail", "it_kkt",
                          "it_update", "it_rest", "kkt_a", "kkt_back", "kkt_g", "kkt_fwd", "kkt_u", "total", "shader_ghz")}
    for b in range(a.traced):
        mk = marks[b]
        mk = mk[~np.isnan(mk[:, 0])]
        ids, cyc = mk[:, 0].astype(int), mk[:, 1]
        at = {}
        for i, c in zip(ids, cyc):
            at.setdefault(i, []).append(c)
        ph["shader_ghz"].append((cyc[-1] - cyc[0]) / max(mk[-1, 2] - mk[0, 2], 1) * 0.1)
        if 4 not in at:  # (MPCQP_PHASE_TIMING_ENDS builds: marks 0 and 20 only)
            if 20 in at:
                ph["total"].append(at[20][0] - at[0][0])
            continue
        ph["setup"].append(at[4][0] - at[0][0])
        fac = [at[12][k] - at[10][k] for k in range(min(len(at[10]), len(at.get(12, []))))]
        ph["factor"] += fac
        if 13 in at and 14 in at and 15 in at:  # Schur-form sub-phases (first factorization)
            ph["f_pre"].append(at[13][0] - at[10][0])
            ph["f_buildS"].append(at[14][0] - at[13][0])
            ph["f_gj"].append(at[15][0] - at[14][0])
            ph["f_post"].append(at[12][0] - at[15][0])
        if all(k in at for k in (21, 22, 23, 24, 25)):  # finer marks of the Schur prologue
            ph["fp_rprime"].append(at[25][0] - at[10][0])
            ph["fp_rinv"].append(at[21][0] - at[25][0])
            ph["fp_b6r_g"].append(at[22][0] - at[21][0])
            ph["fp_chol"].append(at[23][0] - at[22][0])
            ph["fp_bvw"].append(at[24][0] - at[23][0])
            ph["fp_write"].append(at[13][0] - at[24][0])
        if 20 not in at:  # (trace full: a robot with many factorizations; skipped)
            continue
        ph["total"].append(at[20][0] - at[0][0])
        ph["iter_cycles"].append((at[20][0] - at[4][0] - sum(fac)) / max(int(res["iters"][b]), 1))
        if 40 in at and 45 in at:
            ph["it_kkt"].append(at[45][0] - at[40][0])
            ph["it_update"].append(at[46][0] - at[45][0])
            ph["it_rest"].append(at[47][0] - at[46][0])
            if all(k in at for k in (41, 42, 43, 44)):  # Riccati-form KKT sub-phases
                ph["kkt_a"].append(at[41][0] - at[40][0])
                ph["kkt_back"].append(at[42][0] - at[41][0])
                ph["kkt_g"].append(at[43][0] - at[42][0])
                ph["kkt_fwd"].append(at[44][0] - at[43][0])
                ph["kkt_u"].append(at[45][0] - at[44][0])
        if 48 in at and 49 in at:
            ph["check75"].append(at[49][0] - at[48][0])
        if all(k in at for k in (48, 50, 51, 52, 49)):
            ph["ck_px"].append(at[50][0] - at[48][0])
            ph["ck_norms"].append(at[51][0] - at[50][0])
            ph["ck_tests"].append(at[52][0] - at[51][0])
            ph["ck_tail"].append(at[49][0] - at[52][0])
    out = {k: float(np.median(v)) for k, v in ph.items() if v}
    out["mean_iters"] = float(res["iters"][: a.traced].mean())
    out["factorizations_per_robot"] = len(ph["factor"]) / a.traced
    print(json.dumps(out, indent=1))
    if a.out:
        with open(a.out, "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
