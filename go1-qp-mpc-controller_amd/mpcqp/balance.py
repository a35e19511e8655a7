"""Single-step QP balance controller records.

The reference's ``stance_leg_control_type == 0`` branch of ``A1RobotControl::compute_grf``
(A1RobotControl.cpp:321-332 euler error, :377-444 QP) solves one 12-variable, 20-row QP per tick
with a fresh OsqpEigen solver.  ``assemble_balance`` packs the ``*CtrlStates`` fields that branch
reads into the MPCQP_BAL_* record of include/mpcqp.h; the root acceleration, H, g, bounds and the
OSQP solve all run on the device (``MpcQpSolver.balance_solve_device``).
"""
import numpy as np

from ._lib import default_balance_params  # noqa: F401  (re-export)
from .records import GO1_MASS, RobotStates

BAL_POS, BAL_POS_D, BAL_ROT, BAL_ROT_Z = 0, 3, 6, 15
BAL_LIN_VEL, BAL_LIN_VEL_D, BAL_ANG_VEL, BAL_ANG_VEL_D = 24, 27, 30, 33
BAL_EULER, BAL_EULER_D = 36, 39
BAL_KP_LIN, BAL_KD_LIN, BAL_KP_ANG, BAL_KD_ANG = 42, 45, 48, 51
BAL_MASS, BAL_FEET, BAL_CONTACTS, BAL_SIZE = 54, 55, 67, 72

# Go1 gains: the _nh.param defaults of Go1CtrlStates.hpp:276-307 (config/parameters.yaml sets none)
GO1_KP_LINEAR = np.array([100.0, 100.0, 300.0])
GO1_KD_LINEAR = np.array([70.0, 70.0, 120.0])
GO1_KP_ANGULAR = np.array([150.0, 150.0, 1.0])
GO1_KD_ANGULAR = np.array([4.5, 4.5, 30.0])


def rot_z(yaw):
    """root_rot_mat_z = AngleAxisd(yaw, UnitZ) (GazeboA1ROS.cpp:269), batched [B,3,3]."""
    c, s = np.cos(yaw), np.sin(yaw)
    z, o = np.zeros_like(yaw), np.ones_like(yaw)
    return np.stack([np.stack([c, -s, z], -1), np.stack([s, c, z], -1), np.stack([z, z, o], -1)], -2)


def assemble_balance(s: RobotStates, kp_linear=GO1_KP_LINEAR, kd_linear=GO1_KD_LINEAR,
                     kp_angular=GO1_KP_ANGULAR, kd_angular=GO1_KD_ANGULAR, mass=GO1_MASS,
                     root_rot_mat_z=None):
    """[B][72] binary64 balance records from batched robot states (per-robot or shared gains)."""
    B = s.root_pos.shape[0]
    rec = np.zeros((B, BAL_SIZE))
    rz = rot_z(s.root_euler[:, 2]) if root_rot_mat_z is None else np.asarray(root_rot_mat_z)
    rec[:, BAL_POS:BAL_POS + 3] = s.root_pos
    rec[:, BAL_POS_D:BAL_POS_D + 3] = s.root_pos_d
    rec[:, BAL_ROT:BAL_ROT + 9] = np.asarray(s.root_rot_mat).reshape(B, 9)
    rec[:, BAL_ROT_Z:BAL_ROT_Z + 9] = rz.reshape(B, 9)
    rec[:, BAL_LIN_VEL:BAL_LIN_VEL + 3] = s.root_lin_vel
    rec[:, BAL_LIN_VEL_D:BAL_LIN_VEL_D + 3] = s.root_lin_vel_d
    rec[:, BAL_ANG_VEL:BAL_ANG_VEL + 3] = s.root_ang_vel
    rec[:, BAL_ANG_VEL_D:BAL_ANG_VEL_D + 3] = s.root_ang_vel_d
    rec[:, BAL_EULER:BAL_EULER + 3] = s.root_euler
    rec[:, BAL_EULER_D:BAL_EULER_D + 3] = s.root_euler_d
    rec[:, BAL_KP_LIN:BAL_KP_LIN + 3] = kp_linear
    rec[:, BAL_KD_LIN:BAL_KD_LIN + 3] = kd_linear
    rec[:, BAL_KP_ANG:BAL_KP_ANG + 3] = kp_angular
    rec[:, BAL_KD_ANG:BAL_KD_ANG + 3] = kd_angular
    rec[:, BAL_MASS] = mass
    rec[:, BAL_FEET:BAL_FEET + 12] = np.asarray(s.foot_pos_abs).reshape(B, 12)
    rec[:, BAL_CONTACTS:BAL_CONTACTS + 4] = np.asarray(s.contacts, dtype=np.float64)
    return rec
