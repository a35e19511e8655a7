"""ctypes view of libmpcqp.so (include/mpcqp.h, include/mpcqp_debug.h).

The shared library is built in-tree (go1-qp-mpc-controller_amd/lib/libmpcqp.so) by
``make -C go1-qp-mpc-controller_amd`` / ``__graft_entry__.build()``.  There is no fallback:
if the library is missing or has no HIP device, the call fails loudly.  ``load(debug=True)``
opens lib/libmpcqp_debug.so instead: the same ABI plus the cross-check solvers (tests only).
"""
import ctypes
import os

import numpy as np

PKG_ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# MPCQP_LIB overrides the in-tree library (A/B kernel experiments only).
LIB_PATH = os.environ.get("MPCQP_LIB") or os.path.join(PKG_ROOT, "lib", "libmpcqp.so")
DEBUG_LIB_PATH = os.path.join(PKG_ROOT, "lib", "libmpcqp_debug.so")

STATE_DIM, NUM_LEG, NUM_DOF, CONSTRAINT_DIM = 13, 4, 12, 20
MAX_HORIZON = 20
DENSE_MAX_HORIZON = 10  # the dense K^-1 path (debug selection) serves horizons up to this
SOLVER_AUTO, SOLVER_DENSE, SOLVER_RICCATI, SOLVER_WAVE = 0, 1, 2, 3  # 1, 2: debug library only
OSQP_INFTY = 1e30

# record layout (include/mpcqp.h MPCQP_REC_*)
REC_X0, REC_EULER, REC_ROT, REC_INERTIA = 0, 13, 16, 25
REC_MASS, REC_MU, REC_FZMIN, REC_FZMAX, REC_DT, REC_CONTACTS, REC_XREF = 34, 35, 36, 37, 38, 39, 44


# raw robot-state row (include/mpcqp.h MPCQP_ST_*)
ST_EULER, ST_POS, ST_ANG_VEL, ST_LIN_VEL, ST_ROT = 0, 3, 6, 9, 12
ST_EULER_D, ST_POS_D, ST_ANG_VEL_D, ST_LIN_VEL_D, ST_FEET = 21, 24, 27, 30, 33
ST_MASS, ST_INERTIA, ST_MU, ST_FZMIN, ST_FZMAX, ST_DT, ST_CONTACTS, ST_SIZE = 45, 46, 55, 56, 57, 58, 59, 64
# torque-map record layout (include/mpcqp.h MPCQP_TQ_*)
TQ_JFOOT, TQ_FKIN, TQ_KM, TQ_GRAV, TQ_CONTACTS, TQ_SIZE = 0, 36, 48, 51, 63, 68


def rec_feet(N):
    return REC_XREF + 13 * N


def rec_size(N):
    return REC_XREF + 25 * N + (N & 1)


# OSQP 0.6 status values
STATUS_SOLVED = 1
STATUS_SOLVED_INACCURATE = 2
STATUS_PRIMAL_INFEASIBLE_INACCURATE = 3
STATUS_DUAL_INFEASIBLE_INACCURATE = 4
STATUS_MAX_ITER_REACHED = -2
STATUS_PRIMAL_INFEASIBLE = -3
STATUS_DUAL_INFEASIBLE = -4
STATUS_NON_CVX = -7
STATUS_NAN_INPUT = -100
STATUS_UNSOLVED = -10

ERR_OK, ERR_INVALID_ARG, ERR_HIP, ERR_NO_DEVICE, ERR_ALLOC = 0, 1, 2, 3, 4


class Params(ctypes.Structure):
    """mpcqp_params."""
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


class BalanceParams(ctypes.Structure):
    """mpcqp_balance_params."""
    _fields_ = [("q_diag", ctypes.c_double * 6), ("r", ctypes.c_double), ("mu", ctypes.c_double),
                ("f_min", ctypes.c_double), ("f_max", ctypes.c_double)]


class Result(ctypes.Structure):
    """mpcqp_result."""
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
RESULT_DOUBLES = RESULT_DTYPE.itemsize // 8  # 30

# every symbol declared by include/mpcqp.h and include/mpcqp_debug.h
EXPORTED = [
    "mpcqp_default_params", "mpcqp_record_size", "mpcqp_create", "mpcqp_destroy", "mpcqp_reserve",
    "mpcqp_solve_batch_device", "mpcqp_solve_batch_host", "mpcqp_build_qp_device",
    "mpcqp_status_str", "mpcqp_error_str", "mpcqp_last_error",
    "mpcqp_debug_solve_trace_device", "mpcqp_abi_sizes", "mpcqp_handle_slots", "mpcqp_solve_threads",
    "mpcqp_debug_set_solver", "mpcqp_debug_wave_selftest", "mpcqp_joint_torques_device",
    "mpcqp_warm_state_size", "mpcqp_solve_batch_warm_device",
    "mpcqp_balance_default_params", "mpcqp_balance_solve_device", "mpcqp_assemble_records_device",
    "mpcqp_balance_solve_host", "mpcqp_solve_batch_warm_host",
    "mpcqp_debug_scale_image_doubles", "mpcqp_debug_scale_image_device", "mpcqp_copy_warm_slots_device",
    "mpcqp_handoff_counts",
    "mpcqp_debug_set_split", "mpcqp_debug_split_parts",
]

_libs = {}


class MpcQpError(RuntimeError):
    pass


def load(debug=False):
    """Load libmpcqp.so, or libmpcqp_debug.so with debug=True (raises if it has not been built)."""
    if debug in _libs:
        return _libs[debug]
    path = DEBUG_LIB_PATH if debug else LIB_PATH
    if not os.path.exists(path):
        raise MpcQpError(f"{path} not built: run `make -C {PKG_ROOT}` (or __graft_entry__.build())")
    L = ctypes.CDLL(path)
    vp, dp, i32 = ctypes.c_void_p, ctypes.POINTER(ctypes.c_double), ctypes.c_int32
    L.mpcqp_default_params.argtypes = [ctypes.POINTER(Params), i32]
    L.mpcqp_default_params.restype = None
    L.mpcqp_record_size.argtypes = [i32]
    L.mpcqp_record_size.restype = i32
    L.mpcqp_create.argtypes = [ctypes.POINTER(Params), i32, ctypes.POINTER(vp)]
    L.mpcqp_create.restype = i32
    L.mpcqp_destroy.argtypes = [vp]
    L.mpcqp_destroy.restype = i32
    L.mpcqp_reserve.argtypes = [vp, i32]
    L.mpcqp_reserve.restype = i32
    L.mpcqp_solve_batch_device.argtypes = [vp, vp, i32, vp, vp, vp]
    L.mpcqp_solve_batch_device.restype = i32
    L.mpcqp_solve_batch_host.argtypes = [vp, dp, i32, vp, dp]
    L.mpcqp_solve_batch_host.restype = i32
    L.mpcqp_build_qp_device.argtypes = [vp, vp, i32, vp, vp, vp, vp, vp]
    L.mpcqp_build_qp_device.restype = i32
    L.mpcqp_status_str.argtypes = [i32]
    L.mpcqp_status_str.restype = ctypes.c_char_p
    L.mpcqp_error_str.argtypes = [i32]
    L.mpcqp_error_str.restype = ctypes.c_char_p
    L.mpcqp_last_error.argtypes = [vp]
    L.mpcqp_last_error.restype = ctypes.c_char_p
    L.mpcqp_debug_solve_trace_device.argtypes = [vp, vp, i32, vp, vp, vp, i32, vp]
    L.mpcqp_debug_solve_trace_device.restype = i32
    L.mpcqp_abi_sizes.argtypes = [ctypes.POINTER(i32), ctypes.POINTER(i32)]
    L.mpcqp_abi_sizes.restype = i32
    L.mpcqp_handle_slots.argtypes = [vp]
    L.mpcqp_handle_slots.restype = i32
    L.mpcqp_solve_threads.argtypes = [i32]
    L.mpcqp_solve_threads.restype = i32
    L.mpcqp_debug_set_solver.argtypes = [vp, i32]
    L.mpcqp_debug_set_solver.restype = i32
    L.mpcqp_debug_wave_selftest.argtypes = [vp, vp]
    L.mpcqp_debug_wave_selftest.restype = i32
    if hasattr(L, "mpcqp_debug_scale_image_device"):  # (absent from older experiment builds)
        L.mpcqp_debug_scale_image_doubles.argtypes = [i32]
        L.mpcqp_debug_scale_image_doubles.restype = i32
        L.mpcqp_debug_scale_image_device.argtypes = [vp, vp, i32, vp, vp, vp]
        L.mpcqp_debug_scale_image_device.restype = i32
    L.mpcqp_joint_torques_device.argtypes = [vp, vp, i32, vp, vp, vp]
    L.mpcqp_joint_torques_device.restype = i32
    L.mpcqp_warm_state_size.argtypes = [i32]
    L.mpcqp_warm_state_size.restype = i32
    L.mpcqp_solve_batch_warm_device.argtypes = [vp, vp, i32, vp, vp, vp, vp]
    L.mpcqp_solve_batch_warm_device.restype = i32
    L.mpcqp_solve_batch_warm_host.argtypes = [vp, dp, i32, vp, vp, dp]
    L.mpcqp_solve_batch_warm_host.restype = i32
    L.mpcqp_balance_default_params.argtypes = [ctypes.POINTER(BalanceParams)]
    L.mpcqp_balance_default_params.restype = None
    L.mpcqp_balance_solve_device.argtypes = [vp, ctypes.POINTER(BalanceParams), vp, i32, vp, vp]
    L.mpcqp_balance_solve_device.restype = i32
    L.mpcqp_balance_solve_host.argtypes = [vp, ctypes.POINTER(BalanceParams), dp, i32, vp]
    L.mpcqp_balance_solve_host.restype = i32
    L.mpcqp_assemble_records_device.argtypes = [i32, vp, i32, vp, vp]
    L.mpcqp_assemble_records_device.restype = i32
    L.mpcqp_copy_warm_slots_device.argtypes = [i32, vp, vp, vp, vp, i32, vp]
    L.mpcqp_copy_warm_slots_device.restype = i32
    L.mpcqp_handoff_counts.argtypes = [vp, ctypes.POINTER(ctypes.c_int32)]
    L.mpcqp_handoff_counts.restype = i32
    L.mpcqp_debug_set_split.argtypes = [vp, i32]
    L.mpcqp_debug_set_split.restype = i32
    L.mpcqp_debug_split_parts.argtypes = [vp, i32]
    L.mpcqp_debug_split_parts.restype = i32
    ps, rs = i32(0), i32(0)
    L.mpcqp_abi_sizes(ctypes.byref(ps), ctypes.byref(rs))
    if ps.value != ctypes.sizeof(Params) or rs.value != ctypes.sizeof(Result):
        raise MpcQpError(f"ABI mismatch: C sizes {ps.value}/{rs.value} vs ctypes "
                         f"{ctypes.sizeof(Params)}/{ctypes.sizeof(Result)}")
    _libs[debug] = L
    return L


def default_params(horizon=10, **over):
    """mpcqp_default_params + keyword overrides (q_weights/r_weights accept sequences)."""
    p = Params()
    load().mpcqp_default_params(ctypes.byref(p), horizon)
    for k, v in over.items():
        if k in ("q_weights", "r_weights"):
            arr = getattr(p, k)
            for i, x in enumerate(v):
                arr[i] = float(x)
        else:
            setattr(p, k, v)
    return p


def assemble_records_device(horizon, d_states, batch, d_records, stream=0):
    """mpcqp_assemble_records_device: raw-state rows [batch][ST_SIZE] -> MPC records, on the device."""
    check(load().mpcqp_assemble_records_device(int(horizon), d_states, int(batch), d_records, stream or None),
          None, "mpcqp_assemble_records_device")


def copy_warm_slots_device(horizon, d_src, d_src_idx, d_dst, d_dst_idx, count, stream=None):
    """mpcqp_copy_warm_slots_device: slot d_dst[dst_idx[i]] = slot d_src[src_idx[i]] (device int32
    index arrays, None = identity), i < count."""
    check(load().mpcqp_copy_warm_slots_device(int(horizon), d_src, d_src_idx or None, d_dst, d_dst_idx or None,
                                                int(count), stream or None), None, "mpcqp_copy_warm_slots_device")


def default_balance_params(**over):
    """mpcqp_balance_default_params (A1RobotControl.cpp:11-15) + keyword overrides."""
    bp = BalanceParams()
    load().mpcqp_balance_default_params(ctypes.byref(bp))
    for k, v in over.items():
        if k == "q_diag":
            for i, x in enumerate(v):
                bp.q_diag[i] = float(x)
        else:
            setattr(bp, k, v)
    return bp


def check(rc, handle=None, what="mpcqp", lib=None):
    if rc != ERR_OK:
        L = lib or load()
        msg = L.mpcqp_error_str(rc).decode()
        if handle:
            msg += ": " + L.mpcqp_last_error(handle).decode()
        raise MpcQpError(f"{what} failed ({rc}): {msg}")


def status_str(s):
    return load().mpcqp_status_str(int(s)).decode()
