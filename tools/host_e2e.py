"""End-to-end rate through the host-pointer wrapper (mpcqp_solve_batch_host): H2D of the records,
the solve, D2H of the results, synchronised — the PCIe-inclusive number DESIGN §6 quotes beside
the device-resident bench value.  usage: python tools/host_e2e.py [--batch 4096] [--reps 10]"""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "go1-qp-mpc-controller_amd"))
import mpcqp  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=4096)
    ap.add_argument("--reps", type=int, default=10)
    a = ap.parse_args()
    recs = mpcqp.assemble_compute_grf(mpcqp.synthetic_go1(a.batch, seed=1, gait="trot"), 10)
    with mpcqp.MpcQpSolver(mpcqp.default_params(10)) as s:
        s.solve_host(recs)  # warm-up (allocates staging)
        t0 = time.perf_counter()
        for _ in range(a.reps):
            s.solve_host(recs)
        ms = (time.perf_counter() - t0) / a.reps * 1e3
    print(json.dumps({"batch": a.batch, "ms_per_call_host_e2e": ms, "qp_per_s_host_e2e": a.batch / (ms * 1e-3),
                      "bytes_h2d": int(recs.nbytes), "bytes_d2h": a.batch * mpcqp.RESULT_DTYPE.itemsize}))


if __name__ == "__main__":
    main()
