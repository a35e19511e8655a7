"""mpcqp — MI355X-native batched convex-MPC QP engine (host-side Python plumbing).

The compute path is libmpcqp.so (hand-written gfx950 HIP kernels behind the C ABI in
include/mpcqp.h); this package only packs records, owns handles and calls the ABI.
"""
from . import _lib
from ._lib import (assemble_records_device, EXPORTED, LIB_PATH, RESULT_DTYPE, MpcQpError, Params, Result, default_params,
                   load, rec_feet, rec_size, status_str)
from .records import (GO1_Q, GO1_R, RobotStates, assemble_compute_grf, assemble_test_mpc,
                      pack_states, synthetic_go1)
from .robot_control import Go1RobotControl, RobotControl
from .solver import MpcQpSolver
from .torques import assemble_torque_records, joint_torques_device

__all__ = [
    "EXPORTED", "LIB_PATH", "RESULT_DTYPE", "MpcQpError", "Params", "Result", "default_params", "load",
    "rec_feet", "rec_size", "status_str", "GO1_Q", "GO1_R", "RobotStates", "assemble_compute_grf",
    "assemble_test_mpc", "synthetic_go1", "Go1RobotControl", "RobotControl", "MpcQpSolver",
    "assemble_torque_records", "joint_torques_device", "pack_states", "assemble_records_device",
]
