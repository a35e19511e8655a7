"""Host-side assembly of problem records (include/mpcqp.h record layout), batched with numpy.

* ``assemble_compute_grf`` — the input assembly of A1RobotControl::compute_grf's MPC branch
  (src/a1_cpp/src/A1RobotControl.cpp:446-514): x0 = mpc_states, x_ref = mpc_states_d over the
  horizon, A_c from root_euler, the same foot_pos_abs for every horizon step.
* ``assemble_test_mpc`` — the hand-set stance of src/a1_cpp/src/test/test_mpc.cpp:15-122
  (A_c from the horizon-average euler, feet shifted by -v_d*dt per step).
* ``synthetic_go1`` — the seeded synthetic Go1 workload of SURVEY §8(d) (benchmark configs).
"""
from dataclasses import dataclass, field

import numpy as np

from ._lib import (REC_CONTACTS, REC_DT, REC_EULER, REC_FZMAX, REC_FZMIN, REC_INERTIA, REC_MASS,
                   REC_MU, REC_ROT, REC_X0, REC_XREF, rec_feet, rec_size)

# Go1 physical defaults (src/go1_rl_ctrl_cpp/src/Go1CtrlStates.hpp:145-195)
GO1_MASS = 13.0
GO1_INERTIA = np.diag([0.0168352186, 0.0656071082, 0.0742720659])
GO1_DEFAULT_FOOT_POS = np.array([[0.17, 0.15, -0.35], [0.17, -0.15, -0.35],
                                 [-0.17, 0.15, -0.35], [-0.17, -0.15, -0.35]])  # [leg][xyz]
GO1_Q = np.array([80.0, 80.0, 1.0, 0.0, 0.0, 270.0, 1.0, 1.0, 20.0, 20.0, 20.0, 20.0, 0.0])
GO1_R = np.array([1e-5, 1e-5, 1e-6] * 4)
MPC_DT = 0.0025  # A1RobotControl.cpp:462


@dataclass
class RobotStates:
    """Batched view of the A1CtrlStates / Go1CtrlStates fields compute_grf reads (B robots).

    Matrices are row-major; ``foot_pos_abs`` is [B][leg][xyz] (the reference's 3x4 column per leg).
    """
    root_euler: np.ndarray       # [B,3]
    root_pos: np.ndarray         # [B,3]
    root_ang_vel: np.ndarray     # [B,3] world frame
    root_lin_vel: np.ndarray     # [B,3] world frame
    root_rot_mat: np.ndarray     # [B,3,3]
    root_euler_d: np.ndarray     # [B,3] (after terrain adaptation, A1RobotControl.cpp:335-376)
    root_pos_d: np.ndarray       # [B,3]
    root_ang_vel_d: np.ndarray   # [B,3]
    root_lin_vel_d: np.ndarray   # [B,3] body frame
    foot_pos_abs: np.ndarray     # [B,4,3]
    contacts: np.ndarray         # [B,4] bool
    robot_mass: np.ndarray = None     # [B] (default Go1 13.0)
    trunk_inertia: np.ndarray = None  # [B,3,3] (default Go1)
    mu: np.ndarray = None             # [B] (ConvexMpc.cpp:8: 0.3)
    fz_min: float = 0.0               # ConvexMpc.cpp:223
    fz_max: float = 180.0             # ConvexMpc.cpp:224
    mpc_dt: float = MPC_DT            # (RobotControl.compute_grf uses its own mpc_dt / dt, see there)
    stance_leg_control_type: np.ndarray = None  # [B] or scalar: 0 QP balance, 1 MPC (None: all MPC)

    @property
    def batch(self):
        return self.root_euler.shape[0]


def assemble_compute_grf(s: RobotStates, N=10):
    """A1RobotControl.cpp:452-514 → records [B, rec_size(N)] (float64)."""
    B = s.batch
    rec = np.zeros((B, rec_size(N)))
    rec[:, REC_X0:REC_X0 + 3] = s.root_euler
    rec[:, REC_X0 + 3:REC_X0 + 6] = s.root_pos
    rec[:, REC_X0 + 6:REC_X0 + 9] = s.root_ang_vel
    rec[:, REC_X0 + 9:REC_X0 + 12] = s.root_lin_vel
    rec[:, REC_X0 + 12] = -9.8
    dt = s.mpc_dt
    R = np.asarray(s.root_rot_mat, dtype=np.float64).reshape(B, 3, 3)
    vdw = np.einsum("bij,bj->bi", R, s.root_lin_vel_d)  # root_lin_vel_d_world (:470)
    steps = (np.arange(N) + 1.0)
    xr = rec[:, REC_XREF:REC_XREF + 13 * N].reshape(B, N, 13)
    xr[:, :, 0] = s.root_euler_d[:, 0:1]
    xr[:, :, 1] = s.root_euler_d[:, 1:2]
    xr[:, :, 2] = s.root_euler[:, 2:3] + s.root_ang_vel_d[:, 2:3] * dt * steps
    xr[:, :, 3] = s.root_pos[:, 0:1] + vdw[:, 0:1] * dt * steps
    xr[:, :, 4] = s.root_pos[:, 1:2] + vdw[:, 1:2] * dt * steps
    xr[:, :, 5] = s.root_pos_d[:, 2:3]
    xr[:, :, 6:9] = s.root_ang_vel_d[:, None, :]
    xr[:, :, 9] = vdw[:, 0:1]
    xr[:, :, 10] = vdw[:, 1:2]
    xr[:, :, 11] = 0.0
    xr[:, :, 12] = -9.8
    rec[:, REC_EULER:REC_EULER + 3] = s.root_euler
    rec[:, REC_ROT:REC_ROT + 9] = R.reshape(B, 9)
    inertia = GO1_INERTIA[None] if s.trunk_inertia is None else np.asarray(s.trunk_inertia)
    rec[:, REC_INERTIA:REC_INERTIA + 9] = np.broadcast_to(inertia.reshape(-1, 9), (B, 9))
    rec[:, REC_MASS] = GO1_MASS if s.robot_mass is None else s.robot_mass
    rec[:, REC_MU] = 0.3 if s.mu is None else s.mu
    rec[:, REC_FZMIN] = s.fz_min
    rec[:, REC_FZMAX] = s.fz_max
    rec[:, REC_DT] = dt
    rec[:, REC_CONTACTS:REC_CONTACTS + 4] = np.asarray(s.contacts, dtype=bool).astype(np.float64)
    feet = np.asarray(s.foot_pos_abs, dtype=np.float64).reshape(B, 1, 12)
    rec[:, rec_feet(N):rec_feet(N) + 12 * N] = np.broadcast_to(feet, (B, N, 12)).reshape(B, 12 * N)
    return rec


def pack_states(s: RobotStates):
    """Raw robot-state rows [B, ST_SIZE] (include/mpcqp.h MPCQP_ST_*) for the on-device assembly
    (mpcqp_assemble_records_device), which then produces exactly assemble_compute_grf's records."""
    from . import _lib as L
    B = s.batch
    st = np.zeros((B, L.ST_SIZE))
    st[:, L.ST_EULER:L.ST_EULER + 3] = s.root_euler
    st[:, L.ST_POS:L.ST_POS + 3] = s.root_pos
    st[:, L.ST_ANG_VEL:L.ST_ANG_VEL + 3] = s.root_ang_vel
    st[:, L.ST_LIN_VEL:L.ST_LIN_VEL + 3] = s.root_lin_vel
    st[:, L.ST_ROT:L.ST_ROT + 9] = np.asarray(s.root_rot_mat, dtype=np.float64).reshape(B, 9)
    st[:, L.ST_EULER_D:L.ST_EULER_D + 3] = s.root_euler_d
    st[:, L.ST_POS_D:L.ST_POS_D + 3] = s.root_pos_d
    st[:, L.ST_ANG_VEL_D:L.ST_ANG_VEL_D + 3] = s.root_ang_vel_d
    st[:, L.ST_LIN_VEL_D:L.ST_LIN_VEL_D + 3] = s.root_lin_vel_d
    st[:, L.ST_FEET:L.ST_FEET + 12] = np.asarray(s.foot_pos_abs, dtype=np.float64).reshape(B, 12)
    st[:, L.ST_MASS] = GO1_MASS if s.robot_mass is None else s.robot_mass
    inertia = GO1_INERTIA[None] if s.trunk_inertia is None else np.asarray(s.trunk_inertia)
    st[:, L.ST_INERTIA:L.ST_INERTIA + 9] = np.broadcast_to(inertia.reshape(-1, 9), (B, 9))
    st[:, L.ST_MU] = 0.3 if s.mu is None else s.mu
    st[:, L.ST_FZMIN] = s.fz_min
    st[:, L.ST_FZMAX] = s.fz_max
    st[:, L.ST_DT] = s.mpc_dt
    st[:, L.ST_CONTACTS:L.ST_CONTACTS + 4] = np.asarray(s.contacts, dtype=bool).astype(np.float64)
    return st


def assemble_test_mpc(N=10):
    """test_mpc.cpp:15-122 → (record [rec_size(N)], q_weights, r_weights)."""
    dt = 0.0025
    euler = np.zeros(3)
    pos = np.array([0.0, 0.0, 0.15])
    ang_vel_d = np.zeros(3)
    lin_vel_d = np.zeros(3)
    R = np.eye(3)
    rel = np.array([[0.17, 0.15, -0.35], [0.17, -0.15, -0.35], [-0.17, 0.15, -0.35], [-0.17, -0.15, -0.35]])
    q = np.array([1.0, 1.0, 1.0, 0.0, 0.0, 50.0, 0.0, 0.0, 1.0, 1.0, 1.0, 1.0, 0.0])
    r = np.full(12, 1e-6)
    rec = np.zeros(rec_size(N))
    rec[REC_X0:REC_X0 + 3] = euler
    rec[REC_X0 + 3:REC_X0 + 6] = pos
    rec[REC_X0 + 12] = -9.8
    vdw = R @ lin_vel_d
    for i in range(N):
        xr = rec[REC_XREF + 13 * i: REC_XREF + 13 * i + 13]
        xr[2] = euler[2] + ang_vel_d[2] * dt * (i + 1)
        xr[3] = pos[0] + vdw[0] * dt * (i + 1)
        xr[4] = pos[1] + vdw[1] * dt * (i + 1)
        xr[5] = pos[2] + vdw[1] * dt * (i + 1)  # test_mpc.cpp:83 (sic: v_dw,y)
        xr[9], xr[10], xr[11] = vdw
        xr[12] = -9.8
    rec[REC_EULER:REC_EULER + 3] = (euler + euler + ang_vel_d * dt * N) / (N + 1)  # :94-101
    rec[REC_ROT:REC_ROT + 9] = R.reshape(9)
    rec[REC_INERTIA:REC_INERTIA + 9] = np.diag([0.0158533, 0.0377999, 0.0456542]).reshape(9)
    rec[REC_MASS] = 15.0
    rec[REC_MU] = 0.3
    rec[REC_FZMIN], rec[REC_FZMAX] = 0.0, 180.0
    rec[REC_DT] = dt
    rec[REC_CONTACTS:REC_CONTACTS + 4] = [1, 0, 1, 0]
    feet = rel.copy()
    for i in range(N):
        rec[rec_feet(N) + 12 * i: rec_feet(N) + 12 * i + 12] = feet.reshape(12)
        feet = feet - lin_vel_d * dt  # :112-115
    return rec, q, r


def rot_zyx(roll, pitch, yaw):
    """R = Rz(yaw) Ry(pitch) Rx(roll), batched → [B,3,3]."""
    cr, sr = np.cos(roll), np.sin(roll)
    cp, sp = np.cos(pitch), np.sin(pitch)
    cy, sy = np.cos(yaw), np.sin(yaw)
    R = np.empty(roll.shape + (3, 3))
    R[..., 0, 0] = cy * cp
    R[..., 0, 1] = cy * sp * sr - sy * cr
    R[..., 0, 2] = cy * sp * cr + sy * sr
    R[..., 1, 0] = sy * cp
    R[..., 1, 1] = sy * sp * sr + cy * cr
    R[..., 1, 2] = sy * sp * cr - cy * sr
    R[..., 2, 0] = -sp
    R[..., 2, 1] = cp * sr
    R[..., 2, 2] = cp * cr
    return R


def synthetic_go1(batch, seed=0, gait="trot", mixed_mu=False):
    """Seeded synthetic Go1 robot states.

    gait: "trot" (contacts alternate {1,0,0,1} / {0,1,1,0} by instance parity, FL+RR phase of
    A1CtrlStates.h:323-327), "stance" (all four), or "mixed" (Bernoulli(0.5) per leg, config C5).
    mixed_mu: mu ~ U(0.3, 0.9) per instance (config C5), else 0.3 (ConvexMpc.cpp:8).
    """
    rng = np.random.Generator(np.random.PCG64(seed))
    B = batch
    yaw = rng.uniform(-np.pi, np.pi, B)
    roll = rng.uniform(-0.2, 0.2, B)
    pitch = rng.uniform(-0.2, 0.2, B)
    R = rot_zyx(roll, pitch, yaw)
    pos = np.stack([rng.uniform(-1, 1, B), rng.uniform(-1, 1, B), rng.uniform(0.25, 0.35, B)], 1)
    v = rng.normal(0.0, 0.3, (B, 3))
    w = rng.normal(0.0, 0.3, (B, 3))
    feet_body = GO1_DEFAULT_FOOT_POS[None] + rng.uniform(-0.03, 0.03, (B, 4, 3))
    feet_abs = np.einsum("bij,blj->bli", R, feet_body)
    vd = np.stack([rng.uniform(-0.6, 0.6, B), rng.uniform(-0.6, 0.6, B), np.zeros(B)], 1)
    wd = np.stack([np.zeros(B), np.zeros(B), rng.uniform(-0.7, 0.7, B)], 1)
    pzd = rng.uniform(0.1, 0.32, B)
    if gait == "trot":
        ph = (np.arange(B) % 2).astype(bool)
        contacts = np.stack([~ph, ph, ph, ~ph], 1)
    elif gait == "stance":
        contacts = np.ones((B, 4), dtype=bool)
    elif gait == "mixed":
        contacts = rng.random((B, 4)) < 0.5
    else:
        raise ValueError(gait)
    mu = rng.uniform(0.3, 0.9, B) if mixed_mu else np.full(B, 0.3)
    return RobotStates(
        root_euler=np.stack([roll, pitch, yaw], 1), root_pos=pos, root_ang_vel=w, root_lin_vel=v,
        root_rot_mat=R, root_euler_d=np.zeros((B, 3)),
        root_pos_d=np.stack([np.zeros(B), np.zeros(B), pzd], 1), root_ang_vel_d=wd,
        root_lin_vel_d=vd, foot_pos_abs=feet_abs, contacts=contacts, mu=mu)


def synthetic_go1_ticks(batch, ticks, seed=0, gait="trot", period=0.0025, swing_ticks=40):
    """Seeded closed-loop-like trajectories for warm-start tests: ``ticks`` consecutive control
    ticks of ``batch`` robots (list of RobotStates, one per tick).

    From synthetic_go1's states, each tick integrates the pose with the current velocities over
    ``period``, relaxes the velocities toward the command with a small random walk, keeps the
    body-frame feet fixed, and (gait "trot") switches the FL+RR / FR+RL stance pair every
    ``swing_ticks`` ticks with a per-robot phase offset; "stance" keeps all four feet down.
    """
    base = synthetic_go1(batch, seed=seed, gait="stance")
    rng = np.random.Generator(np.random.PCG64(seed + 7919))
    B = batch
    euler = base.root_euler.copy()
    pos = base.root_pos.copy()
    v = base.root_lin_vel.copy()
    w = base.root_ang_vel.copy()
    R0 = base.root_rot_mat
    feet_body = np.einsum("bji,blj->bli", R0, base.foot_pos_abs)  # R^T feet_abs
    phase0 = rng.integers(0, 2 * swing_ticks, B)
    out = []
    for t in range(ticks):
        R = rot_zyx(euler[:, 0], euler[:, 1], euler[:, 2])
        feet_abs = np.einsum("bij,blj->bli", R, feet_body)
        if gait == "trot":
            ph = (((t + phase0) // swing_ticks) % 2).astype(bool)
            contacts = np.stack([~ph, ph, ph, ~ph], 1)
        elif gait == "stance":
            contacts = np.ones((B, 4), dtype=bool)
        else:
            raise ValueError(gait)
        out.append(RobotStates(
            root_euler=euler.copy(), root_pos=pos.copy(), root_ang_vel=w.copy(), root_lin_vel=v.copy(),
            root_rot_mat=R, root_euler_d=base.root_euler_d, root_pos_d=base.root_pos_d,
            root_ang_vel_d=base.root_ang_vel_d, root_lin_vel_d=base.root_lin_vel_d,
            foot_pos_abs=feet_abs, contacts=contacts, mu=base.mu))
        vd_world = np.einsum("bij,bj->bi", R, base.root_lin_vel_d)
        pos = pos + v * period
        euler = euler + np.stack([w[:, 0], w[:, 1], w[:, 2]], 1) * period
        euler[:, :2] = np.clip(euler[:, :2], -0.2, 0.2)
        v = v + 0.05 * (vd_world - v) + rng.normal(0.0, 0.01, (B, 3))
        w = w + 0.05 * (base.root_ang_vel_d - w) + rng.normal(0.0, 0.01, (B, 3))
    return out
