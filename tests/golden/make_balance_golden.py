"""Generate tests/golden/balance.npz — golden vectors for the single-step QP balance controller
(A1RobotControl.cpp:321-332, :377-444).

Produced by the CPU oracle (orc_balance_solve) in THIS container; every instance is validated
before it is written:
  * the formulation (H, g, C, l, u) against tests/numpy_reference.balance_qp (an independent
    numpy restatement) to 1e-13 relative;
  * the converged oracle solution (eps 1e-9) against an independent dense primal-dual interior-
    point solve (objective within 1e-7 relative).
Run:  python tests/golden/make_balance_golden.py
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path[:0] = [os.path.join(REPO, "oracle"), os.path.join(REPO, "tests"),
                os.path.join(REPO, "go1-qp-mpc-controller_amd")]
import pyoracle as po  # noqa: E402
import numpy_reference as nr  # noqa: E402
from mpcqp.balance import assemble_balance  # noqa: E402  (pure numpy record packing)
from mpcqp.records import synthetic_go1  # noqa: E402

Q_DIAG, R_W, MU, FMIN, FMAX = [1.0, 1.0, 1.0, 400.0, 400.0, 100.0], 1e-3, 0.7, 0.0, 180.0


def balance_records():
    parts = []
    for gait, seed, B in (("stance", 11, 24), ("trot", 12, 24), ("mixed", 13, 24)):
        parts.append(assemble_balance(synthetic_go1(B, seed=seed, gait=gait)))
    edge = assemble_balance(synthetic_go1(6, seed=14, gait="stance"))
    edge[0, 67:71] = 0.0                       # all swing: x = 0
    edge[1, 36 + 2], edge[1, 39 + 2] = 3.0, -3.0   # yaw error wraps (> 1.5 pi)
    edge[2, 36 + 2], edge[2, 39 + 2] = -3.0, 3.0   # yaw error wraps (< -1.5 pi)
    edge[3, 3 + 2] = 2.0                       # huge height error: fz at the 180 N bound
    edge[4, 54] = 40.0                         # heavy robot: fz bound active on every leg
    edge[5, 24:27] = [3.0, -2.0, 1.0]          # large velocity error
    parts.append(edge)
    return np.concatenate(parts)


def main():
    recs = balance_records()
    bp = po.default_balance_params()
    p = po.default_params(1)
    pc = po.default_params(1, eps_abs=1e-9, eps_rel=1e-9, max_iter=100000)
    res = po.balance_solve_batch(p, bp, recs, nthreads=8)
    resc = po.balance_solve_batch(pc, bp, recs, nthreads=8)
    for b, rec in enumerate(recs):
        P, q, l, u, A = po.balance_build_qp(bp, rec)
        H, g, C, lo, hi = nr.balance_qp(rec.copy(), Q_DIAG, R_W, MU, FMIN, FMAX)
        assert np.max(np.abs(P - H)) <= 1e-13 * np.max(np.abs(H))
        assert np.max(np.abs(q - g)) <= 1e-13 * max(np.max(np.abs(g)), 1e-300) + 1e-300
        assert np.array_equal(A, C) and np.array_equal(l, lo) and np.array_equal(u, hi)
        assert res["status"][b] == 1 and resc["status"][b] == 1
        xi = nr.ipm_qp(H, g, C, lo, hi)
        if not rec[67:71].any():  # all swing: the feasible set is {0}
            assert np.max(np.abs(resc["u0"][b])) <= 1e-6 and np.max(np.abs(xi)) <= 1e-6
            continue
        f = lambda x: 0.5 * x @ H @ x + g @ x  # noqa: E731
        scale = np.abs(g) @ np.abs(xi) + 0.5 * np.abs(xi) @ np.abs(H) @ np.abs(xi)
        assert abs(f(resc["u0"][b]) - f(xi)) <= 1e-7 * scale + 1e-9, b
    np.savez_compressed(os.path.join(HERE, "balance.npz"), records=recs, u0=res["u0"], f_body=res["f_body"],
                        status=res["status"], iters=res["iters"], rho_updates=res["rho_updates"],
                        obj_val=res["obj_val"], x_converged=resc["u0"])
    print(f"balance.npz: {len(recs)} instances, iters {res['iters'].min()}..{res['iters'].max()}")


if __name__ == "__main__":
    main()
