"""Single-step QP balance controller (A1RobotControl.cpp:321-332, :377-444):
CPU oracle vs the committed golden vectors, formulation vs an independent numpy restatement,
converged solution vs an interior-point solve, host record packing, ABI symbols."""
import os

import numpy as np
import pytest

import mpcqp
import numpy_reference as nr
from mpcqp import balance as bal

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "balance.npz")
Q_DIAG, R_W, MU, FMIN, FMAX = [1.0, 1.0, 1.0, 400.0, 400.0, 100.0], 1e-3, 0.7, 0.0, 180.0


def test_oracle_reproduces_balance_golden(oracle):
    d = np.load(GOLDEN)
    res = oracle.balance_solve_batch(oracle.default_params(1), oracle.default_balance_params(), d["records"], 4)
    np.testing.assert_array_equal(res["status"], d["status"])
    np.testing.assert_array_equal(res["iters"], d["iters"])
    np.testing.assert_array_equal(res["rho_updates"], d["rho_updates"])
    np.testing.assert_allclose(res["u0"], d["u0"], rtol=0, atol=1e-9 * np.abs(d["u0"]).max())


def test_balance_formulation_matches_restatement(oracle):
    d = np.load(GOLDEN)
    bp = oracle.default_balance_params()
    for rec in d["records"][::5]:
        P, q, l, u, A = oracle.balance_build_qp(bp, rec)
        H, g, C, lo, hi = nr.balance_qp(rec.copy(), Q_DIAG, R_W, MU, FMIN, FMAX)
        assert np.max(np.abs(P - H)) <= 1e-13 * np.max(np.abs(H))
        assert np.max(np.abs(q - g)) <= 1e-13 * np.max(np.abs(g))
        np.testing.assert_array_equal(A, C)
        np.testing.assert_array_equal(l, lo)
        np.testing.assert_array_equal(u, hi)


def test_balance_converged_matches_interior_point():
    d = np.load(GOLDEN)
    for b in (1, 30, 55):
        rec = d["records"][b]
        H, g, C, lo, hi = nr.balance_qp(rec.copy(), Q_DIAG, R_W, MU, FMIN, FMAX)
        xi = nr.ipm_qp(H, g, C, lo, hi)
        f = lambda x: 0.5 * x @ H @ x + g @ x  # noqa: E731
        scale = np.abs(g) @ np.abs(xi) + 0.5 * np.abs(xi) @ np.abs(H) @ np.abs(xi)
        assert abs(f(d["x_converged"][b]) - f(xi)) <= 1e-7 * scale + 1e-9


def test_balance_physics():
    """Stance legs carry the weight (sum fz ~ m g within the PD terms), swing legs carry nothing,
    every solution is inside the friction pyramid up to OSQP's tolerance."""
    d = np.load(GOLDEN)
    for rec, x in zip(d["records"], d["u0"]):
        f = x.reshape(4, 3)
        c = rec[bal.BAL_CONTACTS:bal.BAL_CONTACTS + 4] != 0
        tol = 0.25
        assert np.all(np.abs(f[~c]) <= tol)
        assert np.all(np.abs(f[:, 0]) <= MU * f[:, 2] + tol) and np.all(np.abs(f[:, 1]) <= MU * f[:, 2] + tol)
        assert np.all(f[:, 2] <= FMAX * c + tol)
    # an all-stance robot with small errors carries about m g
    st = d["records"][0]
    assert abs(d["u0"][0].reshape(4, 3)[:, 2].sum() - st[bal.BAL_MASS] * 9.8) < 0.5 * st[bal.BAL_MASS] * 9.8


def test_balance_nan_record(oracle):
    d = np.load(GOLDEN)
    rec = d["records"][:2].copy()
    rec[1, bal.BAL_FEET + 4] = np.nan
    res = oracle.balance_solve_batch(oracle.default_params(1), oracle.default_balance_params(), rec)
    assert res["status"][1] == mpcqp._lib.STATUS_NAN_INPUT and res["nan_legs"][1] == 0xF
    assert np.all(np.isnan(res["u0"][1])) and res["status"][0] == 1


def test_assemble_balance_layout():
    st = mpcqp.synthetic_go1(3, seed=2, gait="trot")
    rec = bal.assemble_balance(st)
    assert rec.shape == (3, bal.BAL_SIZE)
    np.testing.assert_array_equal(rec[:, bal.BAL_ROT:bal.BAL_ROT + 9], st.root_rot_mat.reshape(3, 9))
    yaw = st.root_euler[:, 2]
    np.testing.assert_allclose(rec[:, bal.BAL_ROT_Z], np.cos(yaw))
    np.testing.assert_allclose(rec[:, bal.BAL_ROT_Z + 1], -np.sin(yaw))
    np.testing.assert_array_equal(rec[:, bal.BAL_CONTACTS:bal.BAL_CONTACTS + 4], st.contacts.astype(float))
    np.testing.assert_array_equal(rec[:, bal.BAL_FEET:bal.BAL_FEET + 12], st.foot_pos_abs.reshape(3, 12))
    assert np.all(rec[:, bal.BAL_SIZE - 1] == 0)


def test_balance_symbols_and_defaults():
    L = mpcqp.load()
    for s in ("mpcqp_balance_default_params", "mpcqp_balance_solve_device"):
        assert hasattr(L, s)
    bp = mpcqp._lib.default_balance_params()
    assert list(bp.q_diag) == Q_DIAG and (bp.r, bp.mu, bp.f_min, bp.f_max) == (R_W, MU, FMIN, FMAX)
