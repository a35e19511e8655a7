"""Raw robot-state rows for the on-device input assembly (SURVEY §8(f) rank 2,
A1RobotControl.cpp:452-514): the MPCQP_ST_* layout mirrors the oracle's orc_robot_state field by
field, and the oracle's assembly of a packed row equals the host assemble_compute_grf record."""
import ctypes

import numpy as np

import mpcqp
from mpcqp import _lib as L


def state_struct(oracle, row):
    """pyoracle.RobotState from one MPCQP_ST row (test helper)."""
    s = oracle.RobotState()
    for name, off, cnt in (("root_euler", L.ST_EULER, 3), ("root_pos", L.ST_POS, 3),
                           ("root_ang_vel", L.ST_ANG_VEL, 3), ("root_lin_vel", L.ST_LIN_VEL, 3),
                           ("root_rot_mat", L.ST_ROT, 9), ("root_euler_d", L.ST_EULER_D, 3),
                           ("root_pos_d", L.ST_POS_D, 3), ("root_ang_vel_d", L.ST_ANG_VEL_D, 3),
                           ("root_lin_vel_d", L.ST_LIN_VEL_D, 3), ("foot_pos_abs", L.ST_FEET, 12),
                           ("trunk_inertia", L.ST_INERTIA, 9)):
        arr = getattr(s, name)
        for i in range(cnt):
            arr[i] = row[off + i]
    s.robot_mass, s.mu, s.fz_min, s.fz_max, s.mpc_dt = (row[L.ST_MASS], row[L.ST_MU], row[L.ST_FZMIN],
                                                         row[L.ST_FZMAX], row[L.ST_DT])
    for i in range(4):
        s.contacts[i] = int(row[L.ST_CONTACTS + i] != 0)
    return s


def test_state_layout_mirrors_oracle_struct(oracle):
    R = oracle.RobotState
    for name, off in (("root_euler", L.ST_EULER), ("root_pos", L.ST_POS), ("root_ang_vel", L.ST_ANG_VEL),
                      ("root_lin_vel", L.ST_LIN_VEL), ("root_rot_mat", L.ST_ROT), ("root_euler_d", L.ST_EULER_D),
                      ("root_pos_d", L.ST_POS_D), ("root_ang_vel_d", L.ST_ANG_VEL_D),
                      ("root_lin_vel_d", L.ST_LIN_VEL_D), ("foot_pos_abs", L.ST_FEET), ("robot_mass", L.ST_MASS),
                      ("trunk_inertia", L.ST_INERTIA), ("mu", L.ST_MU), ("fz_min", L.ST_FZMIN),
                      ("fz_max", L.ST_FZMAX), ("mpc_dt", L.ST_DT), ("contacts", L.ST_CONTACTS)):
        assert getattr(R, name).offset == 8 * off, name


def test_packed_state_assembles_to_host_record(oracle):
    st = mpcqp.synthetic_go1(16, seed=31, gait="mixed", mixed_mu=True)
    rows = mpcqp.pack_states(st)
    for N in (1, 10, 20):
        host = mpcqp.assemble_compute_grf(st, N)
        for b in range(16):
            ref = oracle.assemble_compute_grf(state_struct(oracle, rows[b]), N)
            np.testing.assert_allclose(ref, host[b], rtol=1e-15, atol=1e-15)
