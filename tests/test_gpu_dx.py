"""Register-resident explicit K^-1 solver (mpcqp_dx.hip, path 5) vs the CPU oracle.

Same OSQP 0.6 iteration; the reduced KKT matrix K = P~ + sigma I + A~' diag(rho) A~ is inverted
by an in-register Gauss-Jordan sweep once per rho and every ADMM iteration is one dense mat-vec.
Gates as the other paths: u0 within 1e-4 relative of the oracle, status
identical, iterations within one check interval.
"""
import glob
import os

import numpy as np
import pytest
import torch

import mpcqp
from gpu_helpers import rel_err_u0, solve_gpu
from test_gpu_riccati import _check_p1_riccati, _oracle_params, TOL_P1

pytestmark = pytest.mark.gpu


def _dx_solver(params):
    s = mpcqp.MpcQpSolver(params)
    s.set_solver(mpcqp._lib.SOLVER_DX)
    return s


@pytest.fixture(scope="module")
def n10_dx():
    s = _dx_solver(mpcqp.default_params(10))
    yield s
    s.close()


def test_dx_selftest_primitives():
    L = mpcqp.load()
    out = torch.zeros(6 * 64, dtype=torch.float64, device="cuda")
    assert L.mpcqp_debug_dx_selftest(out.data_ptr(), torch.cuda.current_stream().cuda_stream) == 0
    torch.cuda.synchronize()
    o = out.cpu().numpy().reshape(6, 64)
    lane = np.arange(64)
    row, li = lane >> 4, lane & 15
    x = 100.0 * row + li
    m1, m2 = li <= 14, li <= 13
    np.testing.assert_array_equal(o[0][m1], x[m1] + 1)          # row_shl:1 reads lane + 1
    np.testing.assert_array_equal(o[1][m2], x[m2] + 2)          # row_shl:2
    np.testing.assert_array_equal(o[2][li >= 1], x[li >= 1] - 1)  # row_shr:1 reads lane - 1
    np.testing.assert_array_equal(o[3][li >= 2], x[li >= 2] - 2)  # row_shr:2
    np.testing.assert_array_equal(o[4], 5.0 + 100.0 * row + 5)   # R[5] += x(lane 5 of the row)
    np.testing.assert_array_equal(o[5], 120.0 + 16 * (100.0 * row) + 120.0)  # sum_c (c + x(lane c))


def test_dx_test_mpc_case(oracle):
    rec, q, r = mpcqp.assemble_test_mpc(10)
    p = mpcqp.default_params(10, q_weights=q, r_weights=r)
    with _dx_solver(p) as s:
        _check_p1_riccati(oracle, s, rec[None], "dx test_mpc", min_iter_equal=1.0)


@pytest.mark.parametrize("gait", ["trot", "stance", "mixed"])
def test_dx_p1(oracle, n10_dx, gait):
    st = mpcqp.synthetic_go1(256, seed=511, gait=gait, mixed_mu=(gait == "mixed"))
    recs = mpcqp.assemble_compute_grf(st, 10)
    _check_p1_riccati(oracle, n10_dx, recs, f"dx N=10 {gait}")


@pytest.mark.parametrize("N", [1, 2, 3, 4, 5, 6, 7, 8, 9])
def test_dx_other_horizons(oracle, N):
    st = mpcqp.synthetic_go1(32, seed=600 + N, gait="mixed", mixed_mu=True)
    recs = mpcqp.assemble_compute_grf(st, N)
    with _dx_solver(mpcqp.default_params(N)) as s:
        _check_p1_riccati(oracle, s, recs, f"dx N={N}", min_iter_equal=0.8)


def test_dx_edge_cases(oracle, n10_dx):
    st = mpcqp.synthetic_go1(8, seed=4, gait="stance")
    st.contacts[0] = False
    st.contacts[1] = True
    st.root_euler[2, 2] = np.pi
    st.root_euler[3, 2] = -np.pi
    st.root_pos_d[4, 2] = 5.0
    st.robot_mass = np.full(8, 13.0)
    st.robot_mass[5] = 40.0
    recs = mpcqp.assemble_compute_grf(st, 10)
    got, _, _ = _check_p1_riccati(oracle, n10_dx, recs, "dx edge", min_iter_equal=0.75)
    assert np.all(np.abs(got["u0"][0]) <= 1e-6), "all-swing robot must get zero forces"


def test_dx_matches_wave():
    st = mpcqp.synthetic_go1(256, seed=77, gait="mixed", mixed_mu=True)
    recs = mpcqp.assemble_compute_grf(st, 10)
    out = {}
    for path in (mpcqp._lib.SOLVER_WAVE, mpcqp._lib.SOLVER_DX):
        with mpcqp.MpcQpSolver(mpcqp.default_params(10)) as s:
            s.set_solver(path)
            out[path] = solve_gpu(s, recs)[0]
    a, b = out[mpcqp._lib.SOLVER_WAVE], out[mpcqp._lib.SOLVER_DX]
    assert np.all(rel_err_u0(a["u0"], b["u0"]) <= TOL_P1)
    np.testing.assert_array_equal(a["status"], b["status"])
    assert np.mean(a["iters"] == b["iters"]) >= 0.95


def test_dx_nan_input_flagged(n10_dx):
    st = mpcqp.synthetic_go1(4, seed=1)
    recs = mpcqp.assemble_compute_grf(st, 10)
    recs[2, 5] = np.nan
    got, sol, _ = solve_gpu(n10_dx, recs)
    assert got["status"][2] == mpcqp._lib.STATUS_NAN_INPUT
    assert got["nan_legs"][2] == 0xF and np.all(got["f_body"][2] == 0) and np.all(np.isnan(sol[2]))
    assert np.all(got["status"][[0, 1, 3]] == mpcqp._lib.STATUS_SOLVED)


def test_dx_full_solution_and_objective(oracle, n10_dx):
    st = mpcqp.synthetic_go1(16, seed=91, gait="trot")
    recs = mpcqp.assemble_compute_grf(st, 10)
    got, sol, _ = solve_gpu(n10_dx, recs)
    ref, ref_sol = oracle.solve_batch(_oracle_params(oracle, n10_dx.params), recs, nthreads=8,
                                      want_solution=True)
    scale = np.maximum(np.max(np.abs(ref_sol), axis=1), 1.0)
    assert np.all(np.max(np.abs(sol - ref_sol), axis=1) / scale <= 1e-4)
    np.testing.assert_allclose(got["obj_val"], ref["obj_val"], rtol=1e-4, atol=1e-6)
    np.testing.assert_array_equal(got["u0"], sol[:, :12])


def test_dx_warm_sequence(oracle):
    T, B, N = 10, 64, 10
    ticks = mpcqp.records.synthetic_go1_ticks(B, T, seed=31, gait="trot", swing_ticks=5)
    recs_t = np.stack([mpcqp.assemble_compute_grf(s, N) for s in ticks])
    p = mpcqp.default_params(N)
    op = oracle.default_params(N, q=list(p.q_weights), r=list(p.r_weights))
    ref = oracle.solve_sequence(op, recs_t, nthreads=8)
    with _dx_solver(p) as s:
        d_state = torch.zeros((B, s.warm_state_size), dtype=torch.float64, device="cuda")
        d_res = torch.zeros((B, mpcqp._lib.RESULT_DOUBLES), dtype=torch.float64, device="cuda")
        stream = torch.cuda.current_stream().cuda_stream
        for t in range(T):
            d_rec = torch.from_numpy(np.ascontiguousarray(recs_t[t])).cuda()
            s.solve_warm_device(d_rec.data_ptr(), B, d_state.data_ptr(), d_res.data_ptr(), 0, stream)
            torch.cuda.synchronize()
            got = np.frombuffer(d_res.cpu().numpy().tobytes(), dtype=mpcqp.RESULT_DTYPE)
            np.testing.assert_array_equal(got["status"], ref[t]["status"], err_msg=f"tick {t}")
            assert np.all(rel_err_u0(got["u0"], ref[t]["u0"]) <= 1e-4), f"tick {t}"
            di = np.abs(got["iters"].astype(int) - ref[t]["iters"].astype(int))
            assert di.max() <= 25 and np.mean(di == 0) >= 0.9, f"tick {t}"


GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
SETS = sorted(p for p in glob.glob(os.path.join(GOLDEN, "*.npz")) if not p.endswith("balance.npz"))


@pytest.mark.parametrize("path", SETS, ids=[os.path.basename(p) for p in SETS])
def test_dx_matches_golden(path):
    """The committed golden vectors (incl. the ill-conditioned gazebo weights, r = 1e-7): the
    explicit inverse rounds differently from the oracle's Cholesky, so iterations are gated like
    the other P1 checks (within one check interval, identical for >= 90 %)."""
    d = np.load(path)
    p = mpcqp.default_params(10, q_weights=d["q_weights"], r_weights=d["r_weights"])
    with _dx_solver(p) as s:
        got, sol, _ = solve_gpu(s, d["records"])
    assert np.all(rel_err_u0(got["u0"], d["u0"]) <= 1e-4)
    np.testing.assert_array_equal(got["status"], d["status"])
    di = np.abs(got["iters"].astype(int) - d["iters"].astype(int))
    assert di.max() <= 25 and np.mean(di == 0) >= 0.9
    full = np.max(np.abs(sol - d["x"]), axis=1) / np.maximum(np.max(np.abs(d["x"]), axis=1), 1.0)
    assert np.all(full <= 1e-4)
