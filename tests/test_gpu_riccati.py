"""Horizons 11..20 on the product path, and the workgroup Riccati cross-check solver (debug library), vs the CPU oracle.

The Riccati path runs the same OSQP 0.6 iteration as the dense path; only the reduced-KKT solve
(P~ + sigma I + A~' rho A~) x~ = rhs is computed differently (block-tridiagonal LQR recursion
instead of an explicit inverse), so rounding differs from the oracle's LDL' solve.  Gates
(SURVEY §8(c) P1):
  ||du0||_inf / max(||u0||_inf, 1) <= 1e-4, status identical, iteration count within +-25
  (one termination-check interval) and identical for >= 99 % of the instances (the measured
  fraction is printed; round 3's bench saw 256 / 256 identical at N = 20).
"""
import numpy as np
import pytest

import mpcqp
from gpu_helpers import build_qp_gpu, rel_err_u0, solve_gpu

pytestmark = pytest.mark.gpu

TOL_P1 = 1e-4
ITER_TOL = 25


def _oracle_params(oracle, p):
    return oracle.default_params(
        p.horizon, q=list(p.q_weights), r=list(p.r_weights), max_iter=p.max_iter,
        eps_abs=p.eps_abs, eps_rel=p.eps_rel, adaptive_rho_interval=p.adaptive_rho_interval)


def _check_p1_riccati(oracle, solver, recs, label, min_iter_equal=0.99):
    op = _oracle_params(oracle, solver.params)
    ref, ref_sol = oracle.solve_batch(op, recs, nthreads=8, want_solution=True)
    got, sol, _ = solve_gpu(solver, recs)
    err = rel_err_u0(got["u0"], ref["u0"])
    bad = np.nonzero(~(err <= TOL_P1))[0]
    assert bad.size == 0, (f"{label}: {bad.size} instances over {TOL_P1}: worst {np.nanmax(err)} at {bad[:8]}; "
                           f"iters gpu {got['iters'][bad[:8]]} ref {ref['iters'][bad[:8]]}")
    np.testing.assert_array_equal(got["status"], ref["status"], err_msg=label)
    di = np.abs(got["iters"].astype(int) - ref["iters"].astype(int))
    assert di.max() <= ITER_TOL, f"{label}: iteration drift {di.max()}"
    print(f"{label}: iteration-equal fraction {np.mean(di == 0):.4f} of {di.size}")
    assert np.mean(di == 0) >= min_iter_equal, f"{label}: only {np.mean(di == 0):.2f} identical iteration counts"
    fb = np.max(np.abs(got["f_body"] - ref["f_body"]), axis=1) / np.maximum(np.max(np.abs(ref["f_body"]), axis=1), 1)
    assert np.all(fb <= TOL_P1), label
    return got, ref, err


@pytest.fixture(scope="module")
def n20_solver():
    s = mpcqp.MpcQpSolver(mpcqp.default_params(20))
    yield s
    s.close()


def test_formulation_p0_n20(oracle, n20_solver):
    st = mpcqp.synthetic_go1(8, seed=70, gait="mixed", mixed_mu=True)
    recs = mpcqp.assemble_compute_grf(st, 20)
    P, g, l, u = build_qp_gpu(n20_solver, recs)
    op = _oracle_params(oracle, n20_solver.params)
    for b in range(recs.shape[0]):
        P0, g0, l0, u0, _ = oracle.build_qp(op, recs[b])
        assert np.max(np.abs(P[b] - P0)) <= 1e-12 * np.max(np.abs(P0)), b
        assert np.max(np.abs(g[b] - g0)) <= 1e-12 * np.max(np.abs(g0)), b
        np.testing.assert_array_equal(l[b], l0)
        np.testing.assert_array_equal(u[b], u0)


@pytest.mark.parametrize("gait", ["trot", "stance", "mixed"])
def test_n20_p1(oracle, n20_solver, gait):
    st = mpcqp.synthetic_go1(64, seed=211, gait=gait, mixed_mu=(gait == "mixed"))
    recs = mpcqp.assemble_compute_grf(st, 20)
    _check_p1_riccati(oracle, n20_solver, recs, f"N=20 {gait}")


def test_n20_test_mpc_case(oracle):
    rec, q, r = mpcqp.assemble_test_mpc(20)
    p = mpcqp.default_params(20, q_weights=q, r_weights=r)
    with mpcqp.MpcQpSolver(p) as s:
        _check_p1_riccati(oracle, s, rec[None], "test_mpc N=20", min_iter_equal=1.0)


def test_n20_edge_cases(oracle, n20_solver):
    st = mpcqp.synthetic_go1(8, seed=4, gait="stance")
    st.contacts[0] = False
    st.contacts[1] = True
    st.root_euler[2, 2] = np.pi
    st.root_euler[3, 2] = -np.pi
    st.root_pos_d[4, 2] = 5.0
    st.robot_mass = np.full(8, 13.0)
    st.robot_mass[5] = 40.0
    recs = mpcqp.assemble_compute_grf(st, 20)
    got, _, _ = _check_p1_riccati(oracle, n20_solver, recs, "edge N=20", min_iter_equal=0.75)
    assert np.all(np.abs(got["u0"][0]) <= 1e-6), "all-swing robot must get zero forces"


@pytest.mark.parametrize("N", [12, 16])
def test_intermediate_horizons(oracle, N):
    st = mpcqp.synthetic_go1(16, seed=300 + N, gait="trot")
    recs = mpcqp.assemble_compute_grf(st, N)
    with mpcqp.MpcQpSolver(mpcqp.default_params(N)) as s:
        _check_p1_riccati(oracle, s, recs, f"N={N}", min_iter_equal=0.75)


@pytest.mark.parametrize("N", [1, 10])
def test_forced_riccati_small_horizons(oracle, N):
    """The Riccati path on horizons the dense path serves: cross-check both against the oracle."""
    st = mpcqp.synthetic_go1(64, seed=400 + N, gait="mixed", mixed_mu=True)
    recs = mpcqp.assemble_compute_grf(st, N)
    with mpcqp.MpcQpSolver(mpcqp.default_params(N), debug=True) as s:
        s.set_solver(mpcqp._lib.SOLVER_RICCATI)
        _check_p1_riccati(oracle, s, recs, f"riccati N={N}")
        s.set_solver(mpcqp._lib.SOLVER_DENSE)
        dense, _, _ = solve_gpu(s, recs)
        s.set_solver(mpcqp._lib.SOLVER_RICCATI)
        ric, _, _ = solve_gpu(s, recs)
    assert np.all(rel_err_u0(ric["u0"], dense["u0"]) <= TOL_P1)


def test_dense_rejected_above_10():
    with mpcqp.MpcQpSolver(mpcqp.default_params(20), debug=True) as s:
        with pytest.raises(mpcqp.MpcQpError):
            s.set_solver(mpcqp._lib.SOLVER_DENSE)


@pytest.mark.parametrize("path", [1, 2, 4, 5])
def test_product_library_has_only_the_wave_path(path):
    """libmpcqp.so ships only scale_kernel + wave_kernel; the cross-check solvers live in
    libmpcqp_debug.so and paths 4 / 5 no longer exist."""
    with mpcqp.MpcQpSolver(mpcqp.default_params(10)) as s:
        with pytest.raises(mpcqp.MpcQpError):
            s.set_solver(path)
        s.set_solver(mpcqp._lib.SOLVER_WAVE)


def test_n20_converged_p2(oracle):
    p = mpcqp.default_params(20, eps_abs=1e-9, eps_rel=1e-9, max_iter=20000)
    st = mpcqp.synthetic_go1(16, seed=6, gait="trot")
    recs = mpcqp.assemble_compute_grf(st, 20)
    with mpcqp.MpcQpSolver(p) as s:
        got, _, _ = solve_gpu(s, recs)
    ref = oracle.solve_batch(_oracle_params(oracle, p), recs, nthreads=8)
    assert np.all(rel_err_u0(got["u0"], ref["u0"]) <= 1e-4)
    assert np.all(got["status"] == mpcqp._lib.STATUS_SOLVED)


def test_n20_nan_input_flagged(n20_solver):
    st = mpcqp.synthetic_go1(4, seed=1)
    recs = mpcqp.assemble_compute_grf(st, 20)
    recs[1, 7] = np.inf
    got, _, _ = solve_gpu(n20_solver, recs)
    assert got["status"][1] == mpcqp._lib.STATUS_NAN_INPUT
    assert got["nan_legs"][1] == 0xF and np.all(got["f_body"][1] == 0)
    assert np.all(got["status"][[0, 2, 3]] == mpcqp._lib.STATUS_SOLVED)


def test_n20_trace_close_to_oracle(oracle, n20_solver):
    """Check trace (iter, pri_res, dua_res, rho): same check iterations, residuals to 1e-6."""
    st = mpcqp.synthetic_go1(4, seed=22, gait="trot")
    recs = mpcqp.assemble_compute_grf(st, 20)
    _, _, tr = solve_gpu(n20_solver, recs, trace=True)
    op = _oracle_params(oracle, n20_solver.params)
    for b in range(4):
        _, _, otr = oracle.solve(op, recs[b], trace=True)
        g = tr[b][~np.isnan(tr[b][:, 0])]
        k = min(len(g), len(otr))
        assert abs(len(g) - len(otr)) <= 1
        for (it, pr, du, rho), o in zip(g[:k], otr[:k]):
            assert it == o[0]
            assert abs(pr - o[2]) <= 1e-6 * max(abs(o[2]), 1e-9)
            assert abs(du - o[3]) <= 1e-6 * max(abs(o[3]), 1e-9)
