"""Python mirror of the reference call surface for the GRF solve (host side of the boundary).

``RobotControl.compute_grf(states, dt)`` ≙ ``A1RobotControl::compute_grf(state, dt)``
(src/a1_cpp/src/A1RobotControl.h:44) and the undefined Go1 hook
``Go1RLController::update_foot_forces_grf`` (src/go1_rl_ctrl_cpp/src/Go1RLController.hpp:39),
batched over robots.  Each robot takes the branch its ``stance_leg_control_type`` selects: 1 (or
the field left None) the MPC branch (A1RobotControl.cpp:446-562), 0 the single-step QP balance
controller (:377-444, a fresh solve each tick, gains from the controller's ``balance_gains``).
Returns the body-frame 3x4 force matrices ``foot_forces_grf`` [B, 3, 4].

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

import warnings

from . import _lib
from .balance import GO1_KD_ANGULAR, GO1_KD_LINEAR, GO1_KP_ANGULAR, GO1_KP_LINEAR, assemble_balance
from .records import GO1_MASS, GO1_Q, GO1_R, MPC_DT, RobotStates, assemble_compute_grf
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
        # stance_leg_control_type == 0 branch: Go1CtrlStates.hpp:276-307 gains, A1RobotControl.cpp:11-15
        self.balance_gains = dict(kp_linear=GO1_KP_LINEAR, kd_linear=GO1_KD_LINEAR,
                                  kp_angular=GO1_KP_ANGULAR, kd_angular=GO1_KD_ANGULAR)
        self.balance_params = _lib.default_balance_params()

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
        B = states.batch
        types = states.stance_leg_control_type
        types = np.ones(B, dtype=np.int64) if types is None else np.broadcast_to(np.asarray(types), (B,))
        if not np.all((types == 0) | (types == 1)):
            raise ValueError("stance_leg_control_type must be 0 (QP) or 1 (MPC)")
        res = np.zeros(B, dtype=_lib.RESULT_DTYPE)
        mpc = np.flatnonzero(types == 1)
        qp = np.flatnonzero(types == 0)
        if mpc.size:
            res[mpc] = self._compute_mpc(states, dt, mpc)
        if qp.size:
            sq = _take(states, qp)
            rb = assemble_balance(sq, mass=GO1_MASS if sq.robot_mass is None else sq.robot_mass,
                                  **self.balance_gains)
            r2 = np.zeros(qp.size, dtype=_lib.RESULT_DTYPE)
            _lib.check(self.solver._L.mpcqp_balance_solve_host(
                self.solver._h, ctypes.byref(self.balance_params),
                np.ascontiguousarray(rb).ctypes.data_as(ctypes.POINTER(ctypes.c_double)), int(qp.size),
                r2.ctypes.data), self.solver._h, "mpcqp_balance_solve_host", self.solver._L)
            res[qp] = r2
        self.last_results = res
        # foot_forces_grf.block<3,1>(0,i) = R^T u0[3i:3i+3]  (NaN legs left 0, res['nan_legs'])
        return res["f_body"].reshape(B, 4, 3).transpose(0, 2, 1).copy()

    def _compute_mpc(self, states, dt, idx):
        """MPC branch for robots idx (their warm slots idx of this controller's slot array)."""
        if self.use_sim_time:
            if dt is None or not np.isfinite(dt) or dt <= 0:
                raise ValueError("use_sim_time needs the caller's dt (finite, > 0)")
            hdt = float(dt)
        else:
            hdt = self.mpc_dt
        if states.mpc_dt != MPC_DT and states.mpc_dt != hdt:
            # (the reference's compute_grf fixes mpc_dt = 0.0025, or dt under use_sim_time, :462-467;
            # RobotStates.mpc_dt is not an input of this call)
            warnings.warn(f"RobotStates.mpc_dt = {states.mpc_dt} is ignored by RobotControl.compute_grf "
                          f"(horizon step {hdt}: set RobotControl.mpc_dt or use_sim_time instead)")
        B = states.batch
        sub = states if idx.size == B else _take(states, idx)
        recs = assemble_compute_grf(dataclasses.replace(sub, mpc_dt=hdt), self.horizon)
        nb = idx.size
        if self.warm_start:
            import torch
            slots = self._ensure_slots(B)
            part = slots if nb == B else slots[torch.as_tensor(idx, device=slots.device)].contiguous()
            # (the host wrapper's stream is ordered after torch's default-stream zeroing / gather)
            torch.cuda.current_stream(slots.device).synchronize()
            res = np.zeros(nb, dtype=_lib.RESULT_DTYPE)
            r2 = np.ascontiguousarray(recs)
            _lib.check(self.solver._L.mpcqp_solve_batch_warm_host(
                self.solver._h, r2.ctypes.data_as(ctypes.POINTER(ctypes.c_double)), nb, part.data_ptr(),
                res.ctypes.data, None), self.solver._h, "mpcqp_solve_batch_warm_host", self.solver._L)
            if nb != B:
                slots[torch.as_tensor(idx, device=slots.device)] = part
        else:
            res = self.solver.solve_host(recs)
        N = self.horizon
        mpc_states = recs[:, _lib.REC_X0:_lib.REC_X0 + 13].copy()
        mpc_states_d = recs[:, _lib.REC_XREF:_lib.REC_XREF + 13 * N].copy()
        R = np.asarray(sub.root_rot_mat, dtype=np.float64).reshape(nb, 3, 3)
        vdw = np.einsum("bij,bj->bi", R, sub.root_lin_vel_d)
        if nb == B:
            states.mpc_states, states.mpc_states_d, states.root_lin_vel_d_world = mpc_states, mpc_states_d, vdw
        else:  # (robots of the QP branch keep their previous bookkeeping, like the reference)
            for name, val, width in (("mpc_states", mpc_states, 13), ("mpc_states_d", mpc_states_d, 13 * N),
                                     ("root_lin_vel_d_world", vdw, 3)):
                cur = getattr(states, name, None)
                cur = np.zeros((B, width)) if cur is None or np.shape(cur) != (B, width) else np.array(cur)
                cur[idx] = val
                setattr(states, name, cur)
        return res

    def close(self):
        self._slots = None
        self.solver.close()


def _take(s: RobotStates, idx):
    """The robots idx of a batched RobotStates (per-robot arrays indexed, scalars kept)."""
    B = s.batch
    kw = {}
    for f in dataclasses.fields(s):
        v = getattr(s, f.name)
        kw[f.name] = np.asarray(v)[idx] if (v is not None and np.ndim(v) >= 1 and np.shape(v)[0] == B) else v
    return RobotStates(**kw)


# Go1 twin of A1RobotControl (the call site commented out at MainGazebo.cpp:77)
Go1RobotControl = RobotControl
