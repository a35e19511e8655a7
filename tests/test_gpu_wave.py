"""One-wavefront-per-robot Riccati path (mpcqp_wave.hip) vs the CPU oracle.

Same OSQP 0.6 iteration as the dense path; the reduced-KKT solve is the LQR recursion (as the
workgroup Riccati path) and the Ruiz column norms of P~ come from an fp32 copy of |H| (the scaling
vectors D, E agree with the oracle's to ~1e-7 relative).  Gates:
  ||du0||_inf / max(||u0||_inf, 1) <= 1e-4, status identical, iteration count within +-25
  (one termination-check interval) and identical for the large majority of instances.
"""
import numpy as np
import pytest
import torch

import mpcqp
from gpu_helpers import rel_err_u0, solve_gpu
from test_gpu_riccati import _check_p1_riccati, _oracle_params, TOL_P1

pytestmark = pytest.mark.gpu


def _wave_solver(params):
    s = mpcqp.MpcQpSolver(params)
    s.set_solver(mpcqp._lib.SOLVER_WAVE)
    return s


@pytest.fixture(scope="module")
def n10_wave():
    s = _wave_solver(mpcqp.default_params(10))
    yield s
    s.close()


def test_selftest_cross_lane_primitives():
    L = mpcqp.load()
    out = torch.zeros(6 * 64, dtype=torch.float64, device="cuda")
    assert L.mpcqp_debug_wave_selftest(out.data_ptr(), torch.cuda.current_stream().cuda_stream) == 0
    torch.cuda.synchronize()
    o = out.cpu().numpy().reshape(6, 64)
    lane = np.arange(64)
    row, li = lane >> 4, lane & 15
    x = 100.0 * row + li
    c = li % 12
    src = 4 * (c // 3) + c % 3
    np.testing.assert_array_equal(o[0], 100.0 * row + src)          # mv12: row_newbcast lanes
    np.testing.assert_array_equal(o[1][row == 1], x[row == 0])      # rmove<0,1>
    np.testing.assert_array_equal(o[2][row == 0], x[row == 1])      # rmove<1,0>
    np.testing.assert_array_equal(o[3][row == 2], x[row == 0])      # rmove<0,2>
    np.testing.assert_array_equal(o[4][row == 1], x[row == 3])      # rmove<3,1>
    np.testing.assert_array_equal(o[5][row == 2], x[row == 3])      # rmove<3,2>


def test_wave_test_mpc_case(oracle):
    rec, q, r = mpcqp.assemble_test_mpc(10)
    p = mpcqp.default_params(10, q_weights=q, r_weights=r)
    with _wave_solver(p) as s:
        _check_p1_riccati(oracle, s, rec[None], "wave test_mpc", min_iter_equal=1.0)


@pytest.mark.parametrize("gait", ["trot", "stance", "mixed"])
def test_wave_p1(oracle, n10_wave, gait):
    st = mpcqp.synthetic_go1(256, seed=511, gait=gait, mixed_mu=(gait == "mixed"))
    recs = mpcqp.assemble_compute_grf(st, 10)
    _check_p1_riccati(oracle, n10_wave, recs, f"wave N=10 {gait}")


def test_wave_edge_cases(oracle, n10_wave):
    st = mpcqp.synthetic_go1(8, seed=4, gait="stance")
    st.contacts[0] = False
    st.contacts[1] = True
    st.root_euler[2, 2] = np.pi
    st.root_euler[3, 2] = -np.pi
    st.root_pos_d[4, 2] = 5.0
    st.robot_mass = np.full(8, 13.0)
    st.robot_mass[5] = 40.0
    recs = mpcqp.assemble_compute_grf(st, 10)
    got, _, _ = _check_p1_riccati(oracle, n10_wave, recs, "wave edge", min_iter_equal=0.75)
    assert np.all(np.abs(got["u0"][0]) <= 1e-6), "all-swing robot must get zero forces"


@pytest.mark.parametrize("N", [1, 2, 3, 4, 5, 7, 8])
def test_wave_other_horizons(oracle, N):
    st = mpcqp.synthetic_go1(32, seed=600 + N, gait="mixed", mixed_mu=True)
    recs = mpcqp.assemble_compute_grf(st, N)
    with _wave_solver(mpcqp.default_params(N)) as s:
        _check_p1_riccati(oracle, s, recs, f"wave N={N}", min_iter_equal=0.8)


def test_wave_matches_dense(n10_wave):
    st = mpcqp.synthetic_go1(128, seed=77, gait="mixed", mixed_mu=True)
    recs = mpcqp.assemble_compute_grf(st, 10)
    wave, _, _ = solve_gpu(n10_wave, recs)
    with mpcqp.MpcQpSolver(mpcqp.default_params(10), debug=True) as s:
        s.set_solver(mpcqp._lib.SOLVER_DENSE)
        dense, _, _ = solve_gpu(s, recs)
    assert np.all(rel_err_u0(wave["u0"], dense["u0"]) <= TOL_P1)


def test_wave_nan_input_flagged(n10_wave):
    st = mpcqp.synthetic_go1(4, seed=1)
    recs = mpcqp.assemble_compute_grf(st, 10)
    recs[2, 5] = np.nan
    got, sol, _ = solve_gpu(n10_wave, recs)
    assert got["status"][2] == mpcqp._lib.STATUS_NAN_INPUT
    assert got["nan_legs"][2] == 0xF and np.all(got["f_body"][2] == 0) and np.all(np.isnan(sol[2]))
    assert np.all(got["status"][[0, 1, 3]] == mpcqp._lib.STATUS_SOLVED)


def test_wave_full_solution_and_objective(oracle, n10_wave):
    st = mpcqp.synthetic_go1(16, seed=91, gait="trot")
    recs = mpcqp.assemble_compute_grf(st, 10)
    got, sol, _ = solve_gpu(n10_wave, recs)
    ref, ref_sol = oracle.solve_batch(_oracle_params(oracle, n10_wave.params), recs, nthreads=8,
                                      want_solution=True)
    scale = np.maximum(np.max(np.abs(ref_sol), axis=1), 1.0)
    assert np.all(np.max(np.abs(sol - ref_sol), axis=1) / scale <= 1e-4)
    np.testing.assert_allclose(got["obj_val"], ref["obj_val"], rtol=1e-4, atol=1e-6)
    np.testing.assert_array_equal(got["u0"], sol[:, :12])


def test_wave_trace_close_to_oracle(oracle, n10_wave):
    st = mpcqp.synthetic_go1(4, seed=22, gait="trot")
    recs = mpcqp.assemble_compute_grf(st, 10)
    _, _, tr = solve_gpu(n10_wave, recs, trace=True)
    op = _oracle_params(oracle, n10_wave.params)
    for b in range(4):
        _, _, otr = oracle.solve(op, recs[b], trace=True)
        g = tr[b][~np.isnan(tr[b][:, 0])]
        k = min(len(g), len(otr))
        assert abs(len(g) - len(otr)) <= 1
        for (it, pr, du, rho), o in zip(g[:k], otr[:k]):
            assert it == o[0]
            assert abs(pr - o[2]) <= 1e-5 * max(abs(o[2]), 1e-9)
            assert abs(du - o[3]) <= 1e-5 * max(abs(o[3]), 1e-9)
