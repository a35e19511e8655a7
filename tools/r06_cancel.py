"""Round-6 calibration of the Schur form's hand-off indicators (VERDICT r05 "do this" 6), on the GPU.

Needs a conditioning-study build (MPCQP_LIB): -DMPCQP_TRACE_COND (the check trace holds, per check,
the cancellation amp = max|R'^-1 w| / max|u| of that KKT solve and the latest factorization's max
S_ii) with both hand-offs disabled (-DMPCQP_SCHUR_SMAX=1e300 -DMPCQP_SCHUR_AMP=1e300), so that every
robot is solved by the Schur form to the end.  Per robot: the largest amp and max S_ii over its checks
and its u0 error against the oracle.  For candidate bounds, the worst u0 error among the robots a bound
keeps in the Schur form and how many it hands over.

usage: python tools/r06_cancel.py OUT.json
"""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(REPO, "go1-qp-mpc-controller_amd"), os.path.join(REPO, "oracle"), os.path.join(REPO, "tests")):
    sys.path.insert(0, p)

import numpy as np  # noqa: E402

import mpcqp  # noqa: E402
import pyoracle  # noqa: E402
from gpu_helpers import rel_err_u0, solve_gpu  # noqa: E402


def cases():
    out = []
    for gait in ("stance", "mixed"):
        for scale in (1.0, 5.0, 100.0):
            st = mpcqp.synthetic_go1(512, seed=7000 + 97 * 5 + 10, gait=gait, mixed_mu=(gait == "mixed"))
            p0 = mpcqp.default_params(10)
            out.append((f"{gait}_x{scale:g}", mpcqp.default_params(10, q_weights=[w * scale for w in p0.q_weights]),
                        mpcqp.assemble_compute_grf(st, 10)))
    for name in ("go1_mixed", "go1_trot", "gazebo_weights", "edge"):
        d = np.load(os.path.join(REPO, "tests", "golden", name + ".npz"))
        N = d["records"].shape[1]
        N = next(n for n in range(1, 21) if mpcqp.rec_size(n) == N)
        out.append((name, mpcqp.default_params(N, q_weights=list(d["q_weights"]), r_weights=list(d["r_weights"])),
                    d["records"]))
    st = mpcqp.synthetic_go1(2048, seed=5, gait="mixed", mixed_mu=True)
    out.append(("c5_sample", mpcqp.default_params(10), mpcqp.assemble_compute_grf(st, 10)))
    st = mpcqp.synthetic_go1(2048, seed=1000, gait="trot")
    out.append(("c2_sample", mpcqp.default_params(10), mpcqp.assemble_compute_grf(st, 10)))
    return out


def main():
    pyoracle.build()
    rows = []
    for name, p, recs in cases():
        if p.horizon > 10:
            continue
        with mpcqp.MpcQpSolver(p) as s:
            got, _, tr = solve_gpu(s, recs, trace=True)
        ref = pyoracle.solve_batch(pyoracle.default_params(p.horizon, q=list(p.q_weights), r=list(p.r_weights)),
                                   recs, nthreads=16)
        err = rel_err_u0(got["u0"], ref["u0"])
        it_eq = got["iters"] == ref["iters"]
        for b in range(recs.shape[0]):
            t = tr[b]
            ok = np.isfinite(t[:, 0]) & (t[:, 0] > 0)
            amp = float(np.max(t[ok, 1])) if ok.any() else 0.0
            smax = float(np.max(t[ok, 2])) if ok.any() else 0.0
            rows.append({"case": name, "robot": b, "amp": amp, "smax": smax, "err": float(err[b]),
                         "iters_equal": bool(it_eq[b])})
        e = np.array([r["err"] for r in rows if r["case"] == name])
        a = np.array([r["amp"] for r in rows if r["case"] == name])
        print(f"{name:16s} robots {len(e):5d} max err {e.max():.2e} max amp {a.max():.2e} iters_equal "
              f"{int(np.sum(it_eq))}/{len(e)}", flush=True)
    amp = np.array([r["amp"] for r in rows])
    smax = np.array([r["smax"] for r in rows])
    err = np.array([r["err"] for r in rows])
    table = []
    for ta in (1e2, 3e2, 1e3, 3e3, 1e4, 3e4, 1e5, 1e300):
        for ts in (1e3, 3e3, 1e4, 1e300):
            keep = (amp <= ta) & (smax <= ts)
            table.append({"amp_bound": ta, "smax_bound": ts, "handed": int(np.sum(~keep)),
                          "worst_kept_err": float(np.max(err[keep])) if keep.any() else 0.0})
    for row in table:
        print(f"amp <= {row['amp_bound']:.0e} smax <= {row['smax_bound']:.0e}: hands over {row['handed']:5d} "
              f"of {len(err)}, worst kept u0 err {row['worst_kept_err']:.2e}")
    # correlation of error with the indicators over robots with a visible error
    m = err > 1e-12
    if m.sum() > 3:
        print("corr log err vs log amp %.3f, vs log smax %.3f, vs log amp*smax %.3f" % (
            np.corrcoef(np.log10(err[m]), np.log10(amp[m]))[0, 1],
            np.corrcoef(np.log10(err[m]), np.log10(smax[m]))[0, 1],
            np.corrcoef(np.log10(err[m]), np.log10(amp[m] * smax[m]))[0, 1]))
    with open(sys.argv[1], "w") as f:
        json.dump({"lib": os.environ.get("MPCQP_LIB"), "table": table, "robots": rows}, f)


if __name__ == "__main__":
    main()
