"""Python mirror of the reference call surface for the GRF solve (host side of the boundary).

``RobotControl.compute_grf(states)`` ≙ ``A1RobotControl::compute_grf(state, dt)`` MPC branch
(src/a1_cpp/src/A1RobotControl.cpp:446-562) and the undefined Go1 hook
``Go1RLController::update_foot_forces_grf`` (src/go1_rl_ctrl_cpp/src/Go1RLController.hpp:39),
batched over robots.  Returns the body-frame 3x4 force matrices ``foot_forces_grf``.

Like the reference it mutates the states' MPC bookkeeping (``mpc_states``,
``mpc_states_d``, ``root_lin_vel_d_world``: A1RobotControl.cpp:452-488) when those attributes
exist on the state object.  Terrain adaptation (:335-376) is upstream of the solve and is not
performed here: pass the adapted ``root_euler_d``.
"""
import numpy as np

from . import _lib
from .records import GO1_Q, GO1_R, RobotStates, assemble_compute_grf
from .solver import MpcQpSolver


class RobotControl:
    """Holds one device solver (the reference's persistent ``OsqpEigen::Solver solver``)."""

    def __init__(self, q_weights=GO1_Q, r_weights=GO1_R, horizon=10, device=0, **settings):
        self.params = _lib.default_params(horizon, q_weights=q_weights, r_weights=r_weights, **settings)
        self.solver = MpcQpSolver(self.params, device=device)
        self.horizon = horizon
        self.last_results = None

    def compute_grf(self, states: RobotStates):
        recs = assemble_compute_grf(states, self.horizon)
        res = self.solver.solve_host(recs)
        self.last_results = res
        B = states.batch
        # foot_forces_grf.block<3,1>(0,i) = R^T u0[3i:3i+3]  (NaN legs left 0, res['nan_legs'])
        f = res["f_body"].reshape(B, 4, 3).transpose(0, 2, 1)  # [B, 3, 4] like Matrix<double,3,4>
        for name, sl in (("mpc_states", slice(0, 13)),):
            if hasattr(states, name):
                setattr(states, name, recs[:, sl].copy())
        return f

    def close(self):
        self.solver.close()


# Go1 twin of A1RobotControl (the call site commented out at MainGazebo.cpp:77)
Go1RobotControl = RobotControl
