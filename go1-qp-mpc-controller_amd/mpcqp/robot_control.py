"""Python mirror of the reference call surface for the GRF solve (host side of the boundary).

``RobotControl.compute_grf(states, dt)`` ≙ ``A1RobotControl::compute_grf(state, dt)`` MPC branch
(src/a1_cpp/src/A1RobotControl.h:44, A1RobotControl.cpp:446-562) and the undefined Go1 hook
``Go1RLController::update_foot_forces_grf`` (src/go1_rl_ctrl_cpp/src/Go1RLController.hpp:39),
batched over robots.  Returns the body-frame 3x4 force matrices ``foot_forces_grf`` [B, 3, 4].

Like the reference controller it owns a persistent, warm-started solver (A1RobotControl.h:67,
setWarmStart(true) at A1RobotControl.cpp:524): robot b keeps device warm-start slot b from call
to call (a change of the batch size re-initialises every slot); ``warm_start=False`` gives the
fresh cold solve of test_mpc.cpp:131-133.  Like the reference it writes the states' MPC
bookkeeping: ``mpc_states`` [B, 13], ``mpc_states_d`` [B, 13N] and ``root_lin_vel_d_world``
[B, 3] (A1RobotControl.cpp:452-488).  Terrain adaptation (:335-376) is upstream of the solve and
is not performed here: pass the adapted ``root_euler_d``.
"""
import ctypes
import dataclasses

import numpy as np

from . import _lib
from .records import GO1_Q, GO1_R, MPC_DT, RobotStates, assemble_compute_grf
from .solver import MpcQpSolver


class RobotControl:
    """Holds one device solver and its warm-start slots (the reference's ``OsqpEigen::Solver``)."""

    def __init__(self, q_weights=GO1_Q, r_weights=GO1_R, horizon=10, device=0, warm_start=True, **settings):
        self.params = _lib.default_params(horizon, q_weights=q_weights, r_weights=r_weights, **settings)
        self.solver = MpcQpSolver(self.params, device=device)
        self.horizon = horizon
        self.device = device
        self.warm_start = warm_start
        self.use_sim_time = False  # A1RobotControl.cpp:63, :464-467
        self.mpc_dt = MPC_DT       # :462
        self.last_results = None
        self._slots = None

    def _ensure_slots(self, B):
        import torch  # device memory only (plumbing)
        if self._slots is None or self._slots.shape[0] != B:
            self._slots = torch.zeros((B, self.solver.warm_state_size), dtype=torch.float64,
                                      device=f"cuda:{self.device}")
        return self._slots

    def reset_warm_start(self):
        if self._slots is not None:
            self._slots.zero_()

    def compute_grf(self, states: RobotStates, dt=None):
        if self.use_sim_time:
            if dt is None or not np.isfinite(dt) or dt <= 0:
                raise ValueError("use_sim_time needs the caller's dt (finite, > 0)")
            hdt = float(dt)
        else:
            hdt = self.mpc_dt
        recs = assemble_compute_grf(dataclasses.replace(states, mpc_dt=hdt), self.horizon)
        B = states.batch
        if self.warm_start:
            slots = self._ensure_slots(B)
            res = np.zeros(B, dtype=_lib.RESULT_DTYPE)
            r2 = np.ascontiguousarray(recs)
            _lib.check(self.solver._L.mpcqp_solve_batch_warm_host(
                self.solver._h, r2.ctypes.data_as(ctypes.POINTER(ctypes.c_double)), B, slots.data_ptr(),
                res.ctypes.data, None), self.solver._h, "mpcqp_solve_batch_warm_host", self.solver._L)
        else:
            res = self.solver.solve_host(recs)
        self.last_results = res
        N = self.horizon
        states.mpc_states = recs[:, _lib.REC_X0:_lib.REC_X0 + 13].copy()
        states.mpc_states_d = recs[:, _lib.REC_XREF:_lib.REC_XREF + 13 * N].copy()
        R = np.asarray(states.root_rot_mat, dtype=np.float64).reshape(B, 3, 3)
        states.root_lin_vel_d_world = np.einsum("bij,bj->bi", R, states.root_lin_vel_d)
        # foot_forces_grf.block<3,1>(0,i) = R^T u0[3i:3i+3]  (NaN legs left 0, res['nan_legs'])
        return res["f_body"].reshape(B, 4, 3).transpose(0, 2, 1).copy()

    def close(self):
        self._slots = None
        self.solver.close()


# Go1 twin of A1RobotControl (the call site commented out at MainGazebo.cpp:77)
Go1RobotControl = RobotControl
