"""Generate tests/golden/*.npz — committed golden vectors for the GRF QP path.

The reference ships no golden vectors and cannot be built here, so the goldens are
produced by the CPU oracle (oracle/mpc_oracle.c) in THIS container and each one is independently
validated before it is written:
  * the formulation (H, g, C, l, u) against tests/numpy_reference.py (an independent restatement
    of ConvexMpc) to 1e-13 relative;
  * the converged solution (eps 1e-9) against an independent dense primal-dual interior-point
    solve of the same QP (objective within 1e-5 relative, constraint violation <= 1e-6).
Run:  python tests/golden/make_golden.py        (every set)
      python tests/golden/make_golden.py r03    (the horizon-20 and interval-100 sets only)
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
from mpcqp import records  # noqa: E402  (host record assembly; pure numpy, no GPU)


def make_set(name, recs, q, r, N=10, interval=25):
    p = po.default_params(N, q=list(q), r=list(r), adaptive_rho_interval=interval)
    pc = po.default_params(N, q=list(q), r=list(r), eps_abs=1e-9, eps_rel=1e-9, max_iter=50000)
    B = recs.shape[0]
    res, sol = po.solve_batch(p, recs, nthreads=8, want_solution=True)
    resc, solc = po.solve_batch(pc, recs, nthreads=8, want_solution=True)
    hsum = np.zeros(B); gsum = np.zeros(B)
    for b in range(B):
        P, g, l, u, A = po.build_qp(p, recs[b])
        H2, g2, C2, l2, u2 = nr.condensed_qp(recs[b], N, np.asarray(q), np.asarray(r))
        assert np.max(np.abs(P - H2)) <= 1e-13 * np.max(np.abs(H2)), (name, b)
        assert np.max(np.abs(g - g2)) <= 1e-13 * max(np.max(np.abs(g2)), 1e-300) + 1e-300, (name, b)
        assert np.array_equal(A, C2) and np.array_equal(l, l2) and np.array_equal(u, u2)
        # independent certificate: a dense primal-dual interior-point solve of the same QP
        # (at N = 20, cond(H) ~ 2.5e6: the IPM's own stop at 1e-10 lands on a worse point through
        # roundoff in its reduced KKT solve; 1e-9 is where it agrees with the OSQP restatement)
        xi = nr.ipm_qp(H2, g2, C2, l2, u2, tol=1e-10 if N <= 10 else 1e-9)
        f = lambda x: 0.5 * x @ H2 @ x + g2 @ x  # noqa: E731
        fscale = np.abs(g2) @ np.abs(xi) + 0.5 * np.abs(xi) @ np.abs(H2) @ np.abs(xi) + 1e-300
        assert abs(f(solc[b]) - f(xi)) <= 1e-5 * fscale + 1e-8, (name, b, f(solc[b]), f(xi))
        Cx = C2 @ solc[b]
        viol = max(0.0, float(np.max(np.maximum(l2 - Cx, Cx - u2))))
        assert viol <= 1e-6 * max(1.0, np.max(np.abs(solc[b]))), (name, b, viol)
        hsum[b] = P.sum(); gsum[b] = g.sum()
    out = os.path.join(HERE, f"{name}.npz")
    np.savez_compressed(out, records=recs, q_weights=np.asarray(q), r_weights=np.asarray(r),
                        u0=res["u0"], f_body=res["f_body"], x=sol, status=res["status"],
                        iters=res["iters"], rho_updates=res["rho_updates"], obj_val=res["obj_val"],
                        x_converged=solc, status_converged=resc["status"],
                        hessian_sum=hsum, gradient_sum=gsum, horizon=N, adaptive_rho_interval=interval)
    print(f"{out}: {B} instances, iters {res['iters'].min()}..{res['iters'].max()}, "
          f"status {np.unique(res['status'])}")


def main(only=None):
    if only == "r03":
        return main_r03()
    rec, q, r = records.assemble_test_mpc(10)
    make_set("test_mpc", rec[None], q, r)
    st = records.synthetic_go1(32, seed=1001, gait="trot")
    make_set("go1_trot", records.assemble_compute_grf(st, 10), records.GO1_Q, records.GO1_R)
    st = records.synthetic_go1(32, seed=5001, gait="mixed", mixed_mu=True)
    make_set("go1_mixed", records.assemble_compute_grf(st, 10), records.GO1_Q, records.GO1_R)
    # edge cases: all swing, all stance, yaw = +-pi, fz pinned at the 180 bound, heavy robot
    st = records.synthetic_go1(6, seed=77, gait="stance")
    st.contacts[0] = False
    st.root_euler[2, 2] = np.pi
    st.root_euler[3, 2] = -np.pi
    st.root_pos_d[4, 2] = 5.0
    st.robot_mass = np.array([13.0, 13.0, 13.0, 13.0, 13.0, 40.0])
    make_set("edge", records.assemble_compute_grf(st, 10), records.GO1_Q, records.GO1_R)
    # ill-conditioned secondary weight set (src/a1_cpp/config/gazebo_a1_mpc.yaml:6-72, r = 1e-7)
    qg = [20.0, 10.0, 1.0, 0.0, 0.0, 420.0, 0.05, 0.05, 0.05, 30.0, 30.0, 10.0, 0.0]
    rg = [1e-7] * 12
    st = records.synthetic_go1(16, seed=9001, gait="trot")
    st.robot_mass = np.full(16, 12.0)
    make_set("gazebo_weights", records.assemble_compute_grf(st, 10), qg, rg)
    main_r03()


def main_r03():
    """Round-3 sets: horizon 20 (config C4) and OSQP 0.6's non-profiling adaptive-rho interval."""
    rec, q, r = records.assemble_test_mpc(20)
    make_set("test_mpc_n20", rec[None], q, r, N=20)
    st = records.synthetic_go1(16, seed=2001, gait="trot")
    make_set("go1_trot_n20", records.assemble_compute_grf(st, 20), records.GO1_Q, records.GO1_R, N=20)
    st = records.synthetic_go1(16, seed=2002, gait="mixed", mixed_mu=True)
    make_set("go1_mixed_n20", records.assemble_compute_grf(st, 20), records.GO1_Q, records.GO1_R, N=20)
    # OSQP 0.6 built without profiling: adaptive_rho_interval = 4 x check_termination = 100
    st = records.synthetic_go1(32, seed=1001, gait="trot")
    make_set("go1_trot_interval100", records.assemble_compute_grf(st, 10), records.GO1_Q, records.GO1_R,
             interval=100)
    st = records.synthetic_go1(32, seed=5001, gait="mixed", mixed_mu=True)
    make_set("go1_mixed_interval100", records.assemble_compute_grf(st, 10), records.GO1_Q, records.GO1_R,
             interval=100)


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else None)
