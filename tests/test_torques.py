"""Torque map: the oracle's compute_joint_torques restatement
(oracle/mpc_oracle.c orc_joint_torques, A1RobotControl.cpp:289-319) against an independent numpy
statement of the same formulas, and the host-side record assembly.  CPU only."""
import numpy as np

import mpcqp
from mpcqp import _lib


def torque_inputs(B, seed, swing_frac=0.5):
    """Random leg Jacobians (well conditioned, with row permutations that force LU pivoting),
    swing-leg PD forces, GRFs and contact masks."""
    rng = np.random.default_rng(seed)
    J = rng.normal(0.0, 0.3, (B, 4, 3, 3)) + np.eye(3) * rng.choice([-0.4, 0.4], (B, 4, 1, 1))
    perm = rng.permuted(np.tile(np.arange(3), (B, 4, 1)), axis=2)
    J = np.take_along_axis(J, perm[..., None], axis=2)
    fkin = rng.normal(0.0, 20.0, (B, 3, 4))
    contacts = rng.random((B, 4)) >= swing_frac
    f_grf = rng.normal(0.0, 40.0, (B, 12))
    return J, fkin, contacts, f_grf


def numpy_torques(J, fkin, contacts, f_grf, km, grav):
    B = J.shape[0]
    tau = np.zeros((B, 12))
    for b in range(B):
        for leg in range(4):
            if contacts[b, leg]:
                t = J[b, leg].T @ -f_grf[b, 3 * leg:3 * leg + 3]
            else:
                t = np.linalg.solve(J[b, leg], km * fkin[b, :, leg])
            tau[b, 3 * leg:3 * leg + 3] = t + grav[3 * leg:3 * leg + 3]
    return tau


def test_record_layout_matches_header():
    assert (_lib.TQ_JFOOT, _lib.TQ_FKIN, _lib.TQ_KM, _lib.TQ_GRAV, _lib.TQ_CONTACTS, _lib.TQ_SIZE) == \
        (0, 36, 48, 51, 63, 68)
    J, fkin, contacts, _ = torque_inputs(3, 0)
    rec = mpcqp.assemble_torque_records(J, fkin, contacts)
    np.testing.assert_array_equal(rec[:, :36].reshape(3, 4, 3, 3), J)
    np.testing.assert_array_equal(rec[:, 36:48].reshape(3, 4, 3), fkin.transpose(0, 2, 1))
    # block-diagonal 12x12 j_foot (A1CtrlStates.h:410) is accepted as well
    jf = np.zeros((3, 12, 12))
    for i in range(4):
        jf[:, 3 * i:3 * i + 3, 3 * i:3 * i + 3] = J[:, i]
    np.testing.assert_array_equal(mpcqp.assemble_torque_records(jf, fkin, contacts), rec)


def test_oracle_matches_numpy_statement(oracle):
    B = 64
    J, fkin, contacts, f_grf = torque_inputs(B, 1)
    km = np.array([0.1, 0.1, 0.04])
    grav = mpcqp.torques.DEFAULT_TORQUES_GRAVITY
    rec = mpcqp.assemble_torque_records(J, fkin, contacts, km_foot=km)
    counters = np.full(B, 9, dtype=np.int32)  # the 10th call is the first that outputs torques
    tau = np.zeros((B, 12))
    oracle.joint_torques(rec, f_grf, counters, tau)
    assert np.all(counters == 10)
    ref = numpy_torques(J, fkin, contacts, f_grf, km, grav)
    np.testing.assert_allclose(tau, ref, rtol=1e-12, atol=1e-12)


def test_first_nine_ticks_output_zero(oracle):
    J, fkin, contacts, f_grf = torque_inputs(4, 2)
    rec = mpcqp.assemble_torque_records(J, fkin, contacts)
    counters = np.zeros(4, dtype=np.int32)
    tau = np.full((4, 12), 7.0)
    for tick in range(1, 12):
        oracle.joint_torques(rec, f_grf, counters, tau)
        assert np.all(counters == tick)
        assert np.all(tau == 0.0) == (tick < 10)


def test_nan_entries_keep_previous_torque(oracle):
    J, fkin, contacts, f_grf = torque_inputs(2, 3)
    contacts[:] = [True, False, True, False]
    f_grf[0, 0:3] = np.nan           # stance leg 0 of robot 0: all three torques NaN
    J[1, 1] = 0.0                    # singular swing Jacobian of robot 1: inf/NaN from the LU
    rec = mpcqp.assemble_torque_records(J, fkin, contacts)
    counters = np.full(2, 20, dtype=np.int32)
    prev = np.arange(24, dtype=np.float64).reshape(2, 12)
    tau = prev.copy()
    oracle.joint_torques(rec, f_grf, counters, tau)
    np.testing.assert_array_equal(tau[0, 0:3], prev[0, 0:3])
    assert np.all(np.isfinite(tau[0, 3:]))
    # an all-zero J: zero pivots; x2 = b2 / 0 = inf (kept: the guard is isnan only), then
    # x1, x0 = NaN -> their previous values stay
    np.testing.assert_array_equal(tau[1, 3:5], prev[1, 3:5])
    assert np.isinf(tau[1, 5])
    assert np.all(np.isfinite(tau[1, [0, 1, 2, 6, 7, 8, 9, 10, 11]]))
