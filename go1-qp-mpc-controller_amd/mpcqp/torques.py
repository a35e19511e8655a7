"""Downstream torque map of the GRF solve (host side of mpcqp_joint_torques_device).

``JointTorqueMap`` ≙ ``A1RobotControl::compute_joint_torques`` (src/a1_cpp/src/A1RobotControl.cpp:
289-319) for a batch of robots: it owns each robot's ``mpc_init_counter`` and ``joint_torques`` on
the device, and maps the solve's body-frame forces (``mpcqp_result.f_body`` = ``foot_forces_grf``)
to joint torques without the forces leaving the device.
"""
import numpy as np

from . import _lib
from ._lib import TQ_CONTACTS, TQ_FKIN, TQ_GRAV, TQ_JFOOT, TQ_KM, TQ_SIZE, check, load

# A1CtrlStates.h:122,129 / Go1CtrlStates.hpp:126,133 defaults
DEFAULT_KM_FOOT = np.array([0.1, 0.1, 0.1])
DEFAULT_TORQUES_GRAVITY = np.array([0.80, 0, 0, -0.80, 0, 0, 0.80, 0, 0, -0.80, 0, 0])


def assemble_torque_records(j_foot, foot_forces_kin, contacts, km_foot=DEFAULT_KM_FOOT,
                            torques_gravity=DEFAULT_TORQUES_GRAVITY):
    """Batched MPCQP_TQ_* records.

    j_foot: [B,4,3,3] per-leg Jacobian blocks (or [B,12,12] block-diagonal j_foot);
    foot_forces_kin: [B,3,4] (the reference's Matrix<double,3,4>) or [B,4,3];
    contacts: [B,4]; km_foot: [3] or [B,3]; torques_gravity: [12] or [B,12].
    """
    j = np.asarray(j_foot, dtype=np.float64)
    B = j.shape[0]
    if j.shape[1:] == (12, 12):
        j = np.stack([j[:, 3 * i:3 * i + 3, 3 * i:3 * i + 3] for i in range(4)], 1)
    fk = np.asarray(foot_forces_kin, dtype=np.float64)
    if fk.shape[1:] == (3, 4):
        fk = fk.transpose(0, 2, 1)
    rec = np.zeros((B, TQ_SIZE))
    rec[:, TQ_JFOOT:TQ_JFOOT + 36] = j.reshape(B, 36)
    rec[:, TQ_FKIN:TQ_FKIN + 12] = fk.reshape(B, 12)
    rec[:, TQ_KM:TQ_KM + 3] = np.broadcast_to(np.asarray(km_foot, dtype=np.float64), (B, 3))
    rec[:, TQ_GRAV:TQ_GRAV + 12] = np.broadcast_to(np.asarray(torques_gravity, dtype=np.float64), (B, 12))
    rec[:, TQ_CONTACTS:TQ_CONTACTS + 4] = np.asarray(contacts, dtype=bool).astype(np.float64)
    return rec


def joint_torques_device(d_records, d_results, batch, d_counter, d_joint_torques, stream=0):
    """mpcqp_joint_torques_device on device pointers (ints)."""
    check(load().mpcqp_joint_torques_device(d_records, d_results, int(batch), d_counter, d_joint_torques,
                                            stream or None), None, "mpcqp_joint_torques_device")
