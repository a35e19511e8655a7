"""TEST INFRASTRUCTURE ONLY — ctypes binding of the CPU parity oracle (oracle/mpc_oracle.c).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this module.
The product path (go1-qp-mpc-controller_amd/) never does.
"""
import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "build", "libmpc_oracle.so")

STATE_DIM, NUM_LEG, NUM_DOF, CONSTRAINT_DIM = 13, 4, 12, 20
REC_X0, REC_EULER, REC_ROT, REC_INERTIA = 0, 13, 16, 25
REC_MASS, REC_MU, REC_FZMIN, REC_FZMAX, REC_DT, REC_CONTACTS, REC_XREF = 34, 35, 36, 37, 38, 39, 44


def rec_feet(N):
    return REC_XREF + 13 * N


def rec_size(N):
    return REC_XREF + 25 * N + (N & 1)


class Params(ctypes.Structure):
    """Mirror of mpcqp_params (include/mpcqp.h)."""
    _fields_ = [
        ("horizon", ctypes.c_int32), ("max_iter", ctypes.c_int32), ("scaling", ctypes.c_int32),
        ("check_termination", ctypes.c_int32), ("adaptive_rho", ctypes.c_int32),
        ("adaptive_rho_interval", ctypes.c_int32), ("scaled_termination", ctypes.c_int32),
        ("warm_start", ctypes.c_int32),
        ("q_weights", ctypes.c_double * 13), ("r_weights", ctypes.c_double * 12),
        ("rho", ctypes.c_double), ("sigma", ctypes.c_double), ("alpha", ctypes.c_double),
        ("eps_abs", ctypes.c_double), ("eps_rel", ctypes.c_double),
        ("eps_prim_inf", ctypes.c_double), ("eps_dual_inf", ctypes.c_double),
        ("adaptive_rho_tolerance", ctypes.c_double),
    ]


class Result(ctypes.Structure):
    """Mirror of mpcqp_result (include/mpcqp.h)."""
    _fields_ = [
        ("u0", ctypes.c_double * 12), ("f_body", ctypes.c_double * 12),
        ("obj_val", ctypes.c_double), ("pri_res", ctypes.c_double), ("dua_res", ctypes.c_double),
        ("rho", ctypes.c_double), ("status", ctypes.c_int32), ("iters", ctypes.c_int32),
        ("rho_updates", ctypes.c_int32), ("nan_legs", ctypes.c_int32),
    ]


RESULT_DTYPE = np.dtype([
    ("u0", "f8", 12), ("f_body", "f8", 12), ("obj_val", "f8"), ("pri_res", "f8"),
    ("dua_res", "f8"), ("rho", "f8"), ("status", "i4"), ("iters", "i4"),
    ("rho_updates", "i4"), ("nan_legs", "i4"),
])
assert RESULT_DTYPE.itemsize == ctypes.sizeof(Result)


class RobotState(ctypes.Structure):
    """Mirror of orc_robot_state (oracle/mpc_oracle.h)."""
    _fields_ = [
        ("root_euler", ctypes.c_double * 3), ("root_pos", ctypes.c_double * 3),
        ("root_ang_vel", ctypes.c_double * 3), ("root_lin_vel", ctypes.c_double * 3),
        ("root_rot_mat", ctypes.c_double * 9),
        ("root_euler_d", ctypes.c_double * 3), ("root_pos_d", ctypes.c_double * 3),
        ("root_ang_vel_d", ctypes.c_double * 3), ("root_lin_vel_d", ctypes.c_double * 3),
        ("foot_pos_abs", ctypes.c_double * 12),
        ("robot_mass", ctypes.c_double), ("trunk_inertia", ctypes.c_double * 9),
        ("mu", ctypes.c_double), ("fz_min", ctypes.c_double), ("fz_max", ctypes.c_double),
        ("mpc_dt", ctypes.c_double), ("contacts", ctypes.c_int32 * 4),
    ]


class TraceEntry(ctypes.Structure):
    _fields_ = [("iter", ctypes.c_int32), ("rho_updated", ctypes.c_int32),
                ("pri_res", ctypes.c_double), ("dua_res", ctypes.c_double),
                ("eps_prim", ctypes.c_double), ("eps_dual", ctypes.c_double),
                ("rho", ctypes.c_double)]


# Go1 defaults (src/go1_rl_ctrl_cpp/src/Go1CtrlStates.hpp:203-249)
GO1_Q = [80.0, 80.0, 1.0, 0.0, 0.0, 270.0, 1.0, 1.0, 20.0, 20.0, 20.0, 20.0, 0.0]
GO1_R = [1e-5, 1e-5, 1e-6] * 4


def default_params(N=10, q=None, r=None, **over):
    """OSQP 0.6 defaults + reference overrides (A1RobotControl.cpp:522-524)."""
    p = Params()
    p.horizon, p.max_iter, p.scaling, p.check_termination = N, 4000, 10, 25
    p.adaptive_rho, p.adaptive_rho_interval, p.scaled_termination, p.warm_start = 1, 25, 0, 0
    for i, v in enumerate(GO1_Q if q is None else q):
        p.q_weights[i] = v
    for i, v in enumerate(GO1_R if r is None else r):
        p.r_weights[i] = v
    p.rho, p.sigma, p.alpha = 0.1, 1e-6, 1.6
    p.eps_abs = p.eps_rel = 1e-3
    p.eps_prim_inf = p.eps_dual_inf = 1e-4
    p.adaptive_rho_tolerance = 5.0
    for k, v in over.items():
        setattr(p, k, v)
    return p


_lib = None


def build():
    subprocess.run(["make", "-s", "-C", _HERE], check=True)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        L = ctypes.CDLL(_LIB_PATH)
        dp = ctypes.POINTER(ctypes.c_double)
        L.orc_assemble_compute_grf.argtypes = [ctypes.POINTER(RobotState), ctypes.c_int32, dp]
        L.orc_assemble_test_mpc.argtypes = [ctypes.c_int32, dp, dp, dp]
        L.orc_build_qp.argtypes = [ctypes.POINTER(Params), dp, dp, dp, dp, dp, dp]
        L.orc_build_qp.restype = ctypes.c_int32
        L.orc_solve.argtypes = [ctypes.POINTER(Params), dp, ctypes.POINTER(Result), dp,
                                ctypes.POINTER(TraceEntry), ctypes.c_int32,
                                ctypes.POINTER(ctypes.c_int32)]
        L.orc_solve.restype = ctypes.c_int32
        L.orc_solve_batch.argtypes = [ctypes.POINTER(Params), dp, ctypes.c_int32,
                                      ctypes.c_void_p, dp, ctypes.c_int32]
        L.orc_solve_batch.restype = ctypes.c_int32
        L.orc_solver_new.argtypes = [ctypes.POINTER(Params)]
        L.orc_solver_new.restype = ctypes.c_void_p
        L.orc_solver_free.argtypes = [ctypes.c_void_p]
        L.orc_solver_free.restype = None
        L.orc_solver_reset.argtypes = [ctypes.c_void_p]
        L.orc_solver_reset.restype = None
        L.orc_solver_step.argtypes = [ctypes.c_void_p, dp, ctypes.POINTER(Result), dp,
                                      ctypes.POINTER(TraceEntry), ctypes.c_int32,
                                      ctypes.POINTER(ctypes.c_int32)]
        L.orc_solver_step.restype = ctypes.c_int32
        L.orc_solve_sequence.argtypes = [ctypes.POINTER(Params), dp, ctypes.c_int32, ctypes.c_int32,
                                         ctypes.c_void_p, ctypes.c_int32]
        L.orc_solve_sequence.restype = ctypes.c_int32
        L.orc_joint_torques.argtypes = [dp, dp, ctypes.POINTER(ctypes.c_int32), dp]
        L.orc_joint_torques.restype = None
        L.orc_balance_build_qp.argtypes = [ctypes.POINTER(BalanceParams), dp, dp, dp, dp, dp, dp]
        L.orc_balance_build_qp.restype = None
        L.orc_balance_solve_batch.argtypes = [ctypes.POINTER(Params), ctypes.POINTER(BalanceParams), dp,
                                              ctypes.c_int32, ctypes.c_void_p, ctypes.c_int32]
        L.orc_balance_solve_batch.restype = ctypes.c_int32
        L.orc_scale_image.argtypes = [ctypes.POINTER(Params), dp, dp, dp, dp, dp]
        L.orc_scale_image.restype = ctypes.c_int32
        L.orc_solver_step_image.argtypes = [ctypes.c_void_p, dp, ctypes.c_void_p, dp, dp, dp, dp,
                                            ctypes.POINTER(ctypes.c_int32)]
        L.orc_solver_step_image.restype = ctypes.c_int32
        _lib = L
    return _lib


def _dp(a):
    return a.ctypes.data_as(ctypes.POINTER(ctypes.c_double))


def assemble_test_mpc(N=10):
    rec = np.zeros(rec_size(N))
    q = np.zeros(13)
    r = np.zeros(12)
    lib().orc_assemble_test_mpc(N, _dp(rec), _dp(q), _dp(r))
    return rec, q, r


def assemble_compute_grf(state: RobotState, N=10):
    rec = np.zeros(rec_size(N))
    lib().orc_assemble_compute_grf(ctypes.byref(state), N, _dp(rec))
    return rec


def build_qp(params, rec):
    N = params.horizon
    n, m = 12 * N, 20 * N
    P = np.zeros((n, n)); q = np.zeros(n); l = np.zeros(m); u = np.zeros(m); A = np.zeros((m, n))
    rec = np.ascontiguousarray(rec, dtype=np.float64)
    rc = lib().orc_build_qp(ctypes.byref(params), _dp(rec), _dp(P), _dp(q), _dp(l), _dp(u), _dp(A))
    assert rc == 0
    return P, q, l, u, A


def solve(params, rec, trace=False):
    N = params.horizon
    res = Result()
    sol = np.zeros(12 * N)
    rec = np.ascontiguousarray(rec, dtype=np.float64)
    ntr = ctypes.c_int32(0)
    tr = (TraceEntry * 512)() if trace else None
    rc = lib().orc_solve(ctypes.byref(params), _dp(rec), ctypes.byref(res), _dp(sol),
                         tr, 512 if trace else 0, ctypes.byref(ntr))
    assert rc == 0
    out = np.frombuffer(bytearray(res), dtype=RESULT_DTYPE)[0]
    if trace:
        return out, sol, [(e.iter, e.rho_updated, e.pri_res, e.dua_res, e.eps_prim, e.eps_dual, e.rho)
                          for e in tr[:ntr.value]]
    return out, sol


def solve_batch(params, recs, nthreads=1, want_solution=False):
    recs = np.ascontiguousarray(recs, dtype=np.float64)
    B = recs.shape[0]
    res = np.zeros(B, dtype=RESULT_DTYPE)
    sols = np.zeros((B, 12 * params.horizon)) if want_solution else None
    rc = lib().orc_solve_batch(ctypes.byref(params), _dp(recs), B, res.ctypes.data,
                               _dp(sols) if sols is not None else None, nthreads)
    assert rc == 0
    return (res, sols) if want_solution else res


def scale_image(params, rec):
    """TEST ONLY: OSQP setup's scaled data for rec: {D [12N], E [20N], q (= c D q) [12N], c}."""
    N = params.horizon
    out = {"D": np.zeros(12 * N), "E": np.zeros(20 * N), "q": np.zeros(12 * N)}
    c = np.zeros(1)
    rec = np.ascontiguousarray(rec, dtype=np.float64)
    rc = lib().orc_scale_image(ctypes.byref(params), _dp(rec), _dp(out["D"]), _dp(out["E"]), _dp(out["q"]), _dp(c))
    assert rc == 0
    out["c"] = float(c[0])
    return out


class WarmSolver:
    """Persistent per-robot OSQP restatement (warm start across control ticks, orc_solver_*)."""

    def __init__(self, params):
        self.params = params
        self._s = lib().orc_solver_new(ctypes.byref(params))

    def step(self, rec):
        N = self.params.horizon
        res = Result()
        sol = np.zeros(12 * N)
        rec = np.ascontiguousarray(rec, dtype=np.float64)
        rc = lib().orc_solver_step(self._s, _dp(rec), ctypes.byref(res), _dp(sol), None, 0, None)
        assert rc == 0
        return np.frombuffer(bytearray(res), dtype=RESULT_DTYPE)[0], sol

    def step_image(self, rec):
        """step() that also returns the scaled data the tick's ADMM started from:
        {D, E, q (= c D q), c, mode (0 initSolver, 1 osqp_update_P, 2 re-init)}."""
        N = self.params.horizon
        res = Result()
        img = {"D": np.zeros(12 * N), "E": np.zeros(20 * N), "q": np.zeros(12 * N)}
        c = ctypes.c_double()
        mode = ctypes.c_int32()
        rec = np.ascontiguousarray(rec, dtype=np.float64)
        rc = lib().orc_solver_step_image(self._s, _dp(rec), ctypes.byref(res), _dp(img["D"]), _dp(img["E"]),
                                         _dp(img["q"]), ctypes.cast(ctypes.byref(c), ctypes.POINTER(ctypes.c_double)),
                                         ctypes.byref(mode))
        assert rc == 0
        img["c"], img["mode"] = c.value, mode.value
        return np.frombuffer(bytearray(res), dtype=RESULT_DTYPE)[0], img

    def reset(self):
        lib().orc_solver_reset(self._s)

    def close(self):
        if self._s:
            lib().orc_solver_free(self._s)
            self._s = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def solve_sequence(params, recs, nthreads=1):
    """recs [T][B][rec]: each robot b solved over T ticks by its own warm-started solver."""
    recs = np.ascontiguousarray(recs, dtype=np.float64)
    T, B = recs.shape[0], recs.shape[1]
    res = np.zeros((T, B), dtype=RESULT_DTYPE)
    rc = lib().orc_solve_sequence(ctypes.byref(params), _dp(recs), T, B, res.ctypes.data, nthreads)
    assert rc == 0
    return res


TQ_SIZE = 68


def joint_torques(tq_recs, f_grf, counters, tau):
    """orc_joint_torques per robot: tq_recs [B,68], f_grf [B,12]; counters [B] int32 and
    tau [B,12] are updated in place (compute_joint_torques, A1RobotControl.cpp:289-319)."""
    tq_recs = np.ascontiguousarray(tq_recs, dtype=np.float64)
    f_grf = np.ascontiguousarray(f_grf, dtype=np.float64)
    assert counters.dtype == np.int32 and tau.dtype == np.float64 and tau.flags.c_contiguous
    for b in range(tq_recs.shape[0]):
        c = ctypes.c_int32(int(counters[b]))
        row = tau[b]
        lib().orc_joint_torques(_dp(tq_recs[b]), _dp(f_grf[b]), ctypes.byref(c), _dp(row))
        counters[b] = c.value


# ---- single-step QP balance controller (A1RobotControl.cpp:7-48, :321-332, :377-444) ----------
BAL_SIZE = 72


class BalanceParams(ctypes.Structure):
    """Mirror of mpcqp_balance_params (include/mpcqp.h)."""
    _fields_ = [("q_diag", ctypes.c_double * 6), ("r", ctypes.c_double), ("mu", ctypes.c_double),
                ("f_min", ctypes.c_double), ("f_max", ctypes.c_double)]


def default_balance_params():
    bp = BalanceParams()
    for i, v in enumerate([1.0, 1.0, 1.0, 400.0, 400.0, 100.0]):
        bp.q_diag[i] = v
    bp.r, bp.mu, bp.f_min, bp.f_max = 1e-3, 0.7, 0.0, 180.0
    return bp


def balance_build_qp(bp, rec):
    P = np.zeros((12, 12)); q = np.zeros(12); l = np.zeros(20); u = np.zeros(20); A = np.zeros((20, 12))
    rec = np.ascontiguousarray(rec, dtype=np.float64)
    lib().orc_balance_build_qp(ctypes.byref(bp), _dp(rec), _dp(P), _dp(q), _dp(l), _dp(u), _dp(A))
    return P, q, l, u, A


def balance_solve_batch(params, bp, recs, nthreads=1):
    """Fresh OSQP solve per robot of the balance QP (params: OSQP settings; horizon ignored)."""
    recs = np.ascontiguousarray(recs, dtype=np.float64).reshape(-1, BAL_SIZE)
    res = np.zeros(recs.shape[0], dtype=RESULT_DTYPE)
    rc = lib().orc_balance_solve_batch(ctypes.byref(params), ctypes.byref(bp), _dp(recs), recs.shape[0],
                                       res.ctypes.data, nthreads)
    assert rc == 0
    return res
