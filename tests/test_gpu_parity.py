"""HIP path vs CPU oracle, through the C ABI (SURVEY §8(c) parity modes P0/P1/P2).

Tolerances (binary64 on both sides):
  P0 formulation   H, g, l, u relative to max|.|            <= 1e-12
  P1 schedule-identical (reference settings, fixed rho interval 25, cold start):
                   ||du0||_inf / max(||u0||_inf, 1)        <= 1e-4  (north_star gate)
                   status and iteration count identical
  P2 converged (eps 1e-9 on both sides)                       <= 1e-4
"""
import numpy as np
import pytest

import mpcqp
from gpu_helpers import build_qp_gpu, rel_err_u0, sentinel, solve_gpu

pytestmark = pytest.mark.gpu

TOL_P1 = 1e-4
# regression sentinels at the achieved accuracy (binary64 on both sides: ~1e-10 at the Go1 weights)
SENT = {"trot": 1e-8, "mixed": 1e-8, "stance": 1e-6}


@pytest.fixture(scope="module")
def go1_solver():
    s = mpcqp.MpcQpSolver(mpcqp.default_params(10))
    yield s
    s.close()


def _oracle_params(oracle, p):
    return oracle.default_params(
        p.horizon, q=list(p.q_weights), r=list(p.r_weights), max_iter=p.max_iter,
        eps_abs=p.eps_abs, eps_rel=p.eps_rel, adaptive_rho_interval=p.adaptive_rho_interval)


def _check_p1(oracle, solver, recs, label, max_rel=TOL_P1, sent=1e-8):
    op = _oracle_params(oracle, solver.params)
    ref, ref_sol = oracle.solve_batch(op, recs, nthreads=8, want_solution=True)
    got, sol, _ = solve_gpu(solver, recs)
    err = rel_err_u0(got["u0"], ref["u0"])
    bad = np.nonzero(~(err <= max_rel))[0]
    assert bad.size == 0, f"{label}: {bad.size} instances over {max_rel}: worst {np.nanmax(err)} at {bad[:8]}"
    np.testing.assert_array_equal(got["status"], ref["status"], err_msg=label)
    np.testing.assert_array_equal(got["iters"], ref["iters"], err_msg=label)
    np.testing.assert_array_equal(got["rho_updates"], ref["rho_updates"], err_msg=label)
    fb = np.max(np.abs(got["f_body"] - ref["f_body"]), axis=1) / np.maximum(np.max(np.abs(ref["f_body"]), axis=1), 1)
    assert np.all(fb <= max_rel), label
    full = np.max(np.abs(sol - ref_sol), axis=1) / np.maximum(np.max(np.abs(ref_sol), axis=1), 1)
    assert np.all(full <= max_rel), f"{label}: full-horizon solution worst {full.max()}"
    sentinel(err, sent, f"parity {label}")
    return err


def test_formulation_p0_test_mpc(oracle):
    rec, q, r = mpcqp.assemble_test_mpc(10)
    p = mpcqp.default_params(10, q_weights=q, r_weights=r)
    with mpcqp.MpcQpSolver(p) as s:
        P, g, l, u = build_qp_gpu(s, rec[None])
    op = _oracle_params(oracle, p)
    P0, g0, l0, u0, _ = oracle.build_qp(op, rec)
    assert np.max(np.abs(P[0] - P0)) <= 1e-12 * np.max(np.abs(P0))
    assert np.max(np.abs(g[0] - g0)) <= 1e-12 * max(np.max(np.abs(g0)), 1e-300)
    np.testing.assert_array_equal(l[0], l0)
    np.testing.assert_array_equal(u[0], u0)


def test_formulation_p0_synthetic(oracle, go1_solver):
    st = mpcqp.synthetic_go1(32, seed=7, gait="mixed", mixed_mu=True)
    recs = mpcqp.assemble_compute_grf(st, 10)
    P, g, l, u = build_qp_gpu(go1_solver, recs)
    op = _oracle_params(oracle, go1_solver.params)
    for b in range(recs.shape[0]):
        P0, g0, l0, u0, _ = oracle.build_qp(op, recs[b])
        assert np.max(np.abs(P[b] - P0)) <= 1e-12 * np.max(np.abs(P0)), b
        assert np.max(np.abs(g[b] - g0)) <= 1e-12 * np.max(np.abs(g0)), b
        np.testing.assert_array_equal(l[b], l0)
        np.testing.assert_array_equal(u[b], u0)


def test_test_mpc_case_p1(oracle):
    """The reference's only harness (test_mpc.cpp) reproduced on the GPU."""
    rec, q, r = mpcqp.assemble_test_mpc(10)
    p = mpcqp.default_params(10, q_weights=q, r_weights=r)
    with mpcqp.MpcQpSolver(p) as s:
        _check_p1(oracle, s, rec[None], "test_mpc")


@pytest.mark.parametrize("gait", ["trot", "stance", "mixed"])
def test_synthetic_p1(oracle, go1_solver, gait):
    st = mpcqp.synthetic_go1(64, seed=11, gait=gait, mixed_mu=(gait == "mixed"))
    recs = mpcqp.assemble_compute_grf(st, 10)
    _check_p1(oracle, go1_solver, recs, gait, sent=SENT[gait])


def test_edge_cases_p1(oracle, go1_solver):
    st = mpcqp.synthetic_go1(8, seed=3, gait="stance")
    st.contacts[0] = False           # all swing -> u == 0 (equality rows everywhere)
    st.contacts[1] = True            # all stance
    st.root_euler[2, 2] = np.pi      # yaw = +pi
    st.root_euler[3, 2] = -np.pi     # yaw = -pi
    st.root_pos_d[4, 2] = 5.0        # demands far beyond fz_max -> fz pinned at 180
    st.robot_mass = np.full(8, 13.0)
    st.robot_mass[5] = 40.0          # heavy robot, bound-active
    recs = mpcqp.assemble_compute_grf(st, 10)
    err = _check_p1(oracle, go1_solver, recs, "edge", sent=1e-6)
    got, sol, _ = solve_gpu(go1_solver, recs)
    assert np.all(np.abs(got["u0"][0]) <= 1e-6), "all-swing robot must get zero forces"


@pytest.mark.parametrize("N", [1, 4, 7])
def test_other_horizons_p1(oracle, N):
    st = mpcqp.synthetic_go1(16, seed=100 + N, gait="trot")
    recs = mpcqp.assemble_compute_grf(st, N)
    with mpcqp.MpcQpSolver(mpcqp.default_params(N)) as s:
        _check_p1(oracle, s, recs, f"N={N}")


@pytest.mark.parametrize("N", [2, 3, 5, 6, 8, 9, 10])
def test_every_schur_horizon_mixed_p1(oracle, N):
    """Every Schur-form horizon, mixed gait (more rho updates, so more factorizations): the
    matrix-core Gauss-Jordan runs with 1 (N <= 2), 2 (3..5), 3 (6..8) and 4 (9, 10) block rows, the
    last short (6N mod 16 real rows) except at N = 8."""
    st = mpcqp.synthetic_go1(32, seed=300 + N, gait="mixed", mixed_mu=True)
    recs = mpcqp.assemble_compute_grf(st, N)
    with mpcqp.MpcQpSolver(mpcqp.default_params(N)) as s:
        _check_p1(oracle, s, recs, f"N={N} mixed")


def test_converged_p2(oracle):
    """Converged mode: both sides run to eps 1e-9; robust to rho-schedule details."""
    p = mpcqp.default_params(10, eps_abs=1e-9, eps_rel=1e-9, max_iter=20000)
    st = mpcqp.synthetic_go1(16, seed=5, gait="trot")
    recs = mpcqp.assemble_compute_grf(st, 10)
    with mpcqp.MpcQpSolver(p) as s:
        got, _, _ = solve_gpu(s, recs)
    op = _oracle_params(oracle, p)
    ref = oracle.solve_batch(op, recs, nthreads=8)
    assert np.all(rel_err_u0(got["u0"], ref["u0"]) <= 1e-4)
    assert np.all(got["status"] == mpcqp._lib.STATUS_SOLVED)


def test_nan_input_flagged(go1_solver):
    st = mpcqp.synthetic_go1(4, seed=1)
    recs = mpcqp.assemble_compute_grf(st, 10)
    recs[2, 5] = np.nan
    got, sol, _ = solve_gpu(go1_solver, recs)
    assert got["status"][2] == mpcqp._lib.STATUS_NAN_INPUT
    assert got["nan_legs"][2] == 0xF and np.all(got["f_body"][2] == 0)
    assert np.all(got["status"][[0, 1, 3]] == mpcqp._lib.STATUS_SOLVED)


def test_trace_matches_oracle(oracle, go1_solver):
    """Termination-check trace (iter, pri_res, dua_res, rho) identical to the oracle's."""
    st = mpcqp.synthetic_go1(4, seed=21, gait="trot")
    recs = mpcqp.assemble_compute_grf(st, 10)
    _, _, tr = solve_gpu(go1_solver, recs, trace=True)
    op = _oracle_params(oracle, go1_solver.params)
    for b in range(4):
        _, _, otr = oracle.solve(op, recs[b], trace=True)
        g = tr[b][~np.isnan(tr[b][:, 0])]
        assert len(g) == len(otr)
        for (it, pr, du, rho), o in zip(g, otr):
            assert it == o[0]
            assert abs(pr - o[2]) <= 1e-9 * max(abs(o[2]), 1e-12) + 1e-15
            assert abs(du - o[3]) <= 1e-9 * max(abs(o[3]), 1e-12) + 1e-15
            assert abs(rho - o[6]) <= 1e-9 * o[6]
