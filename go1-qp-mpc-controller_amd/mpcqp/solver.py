"""Handle-level Python API over libmpcqp (mirrors the C ABI one to one).

``MpcQpSolver`` plays the role of the reference's long-lived ``OsqpEigen::Solver`` member
(A1RobotControl.h:67) for a whole batch of robots.  Device buffers are passed as raw pointers
(e.g. ``torch.Tensor.data_ptr()``) and streams as integer hipStream_t handles
(``torch.cuda.current_stream().cuda_stream``); torch is plumbing only and never imported here.
"""
import ctypes

import numpy as np

from . import _lib
from ._lib import RESULT_DTYPE, Params, check, load, rec_size


class MpcQpSolver:
    def __init__(self, params: Params = None, horizon=10, device=0, debug=False):
        """debug=True: the handle lives in libmpcqp_debug.so (adds the cross-check solvers)."""
        L = load(debug)
        self.params = params if params is not None else _lib.default_params(horizon)
        self.horizon = self.params.horizon
        self.n = 12 * self.horizon
        self.m = 20 * self.horizon
        self.rec_size = rec_size(self.horizon)
        h = ctypes.c_void_p()
        check(L.mpcqp_create(ctypes.byref(self.params), int(device), ctypes.byref(h)), None, "mpcqp_create")
        self._h = h
        self._L = L

    # -- lifecycle -------------------------------------------------------------------------------
    def close(self):
        if getattr(self, "_h", None):
            self._L.mpcqp_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    @property
    def slots(self):
        return self._L.mpcqp_handle_slots(self._h)

    def set_solver(self, path):
        """mpcqp_debug_set_solver: 0 auto, 3 Riccati wave; debug handles also 1 dense K^-1 (N <= 10),
        2 Riccati workgroup."""
        check(self._L.mpcqp_debug_set_solver(self._h, int(path)), self._h, "mpcqp_debug_set_solver", self._L)

    def reserve(self, batch):
        check(self._L.mpcqp_reserve(self._h, int(batch)), self._h, "mpcqp_reserve", self._L)

    def set_split(self, parts):
        """mpcqp_debug_set_split: parts a solve is split into over the handle's internal streams
        (0 auto, 1 one launch, up to 8).  Returns the previous setting."""
        old = int(self._L.mpcqp_debug_set_split(self._h, int(parts)))
        if old < 0:
            raise ValueError("mpcqp_debug_set_split: parts must be 0..8")
        return old

    def split_parts(self, batch):
        """mpcqp_debug_split_parts: parts a solve of `batch` robots is split into."""
        return int(self._L.mpcqp_debug_split_parts(self._h, int(batch)))

    def handoff_counts(self):
        """mpcqp_handoff_counts: robots of the last Schur-form solve that the Riccati form solved in
        their own wave, as (rank-deficient feet, S_max x cancellation above SCHUR_AMP, S_max above the
        SCHUR_SMAX cap).
        Synchronizes the device."""
        import ctypes
        c = (ctypes.c_int32 * 3)()
        check(self._L.mpcqp_handoff_counts(self._h, c), self._h, "mpcqp_handoff_counts", self._L)
        return tuple(int(v) for v in c)

    # -- device-pointer API ------------------------------------------------------------------------
    def solve_device(self, d_records, batch, d_results, d_solution=0, stream=0):
        """mpcqp_solve_batch_device: records/results/solution are device pointers (ints)."""
        check(self._L.mpcqp_solve_batch_device(self._h, d_records, int(batch), d_results,
                                               d_solution or None, stream or None),
              self._h, "mpcqp_solve_batch_device", self._L)

    def balance_solve_device(self, bp, d_records, batch, d_results, stream=0):
        """Single-step QP balance controller (mpcqp_balance_solve_device): records [batch][72]."""
        check(self._L.mpcqp_balance_solve_device(self._h, ctypes.byref(bp), d_records, int(batch),
                                                 d_results, stream or None), self._h, "mpcqp_balance_solve_device", self._L)

    @property
    def warm_state_size(self):
        """Doubles per robot of the warm-start slot (mpcqp_warm_state_size)."""
        return self._L.mpcqp_warm_state_size(self.horizon)

    def solve_warm_device(self, d_records, batch, d_state, d_results, d_solution=0, stream=0):
        """mpcqp_solve_batch_warm_device: the reference's persistent, warm-started solver per robot
        (A1RobotControl.cpp:522-540); d_state [batch][warm_state_size] doubles, zeroed at first."""
        check(self._L.mpcqp_solve_batch_warm_device(self._h, d_records, int(batch), d_state, d_results,
                                                    d_solution or None, stream or None),
              self._h, "mpcqp_solve_batch_warm_device", self._L)

    @property
    def scale_image_size(self):
        return int(self._L.mpcqp_debug_scale_image_doubles(self.params.horizon))

    def scale_image_device(self, d_records, batch, d_state, d_img, stream=0):
        """Debug library: scale_kernel's image alone (include/mpcqp_debug.h); d_state 0 = cold."""
        check(self._L.mpcqp_debug_scale_image_device(self._h, d_records, int(batch), d_state or None, d_img,
                                                     stream or None), self._h, "mpcqp_debug_scale_image_device",
              self._L)

    def solve_device_trace(self, d_records, batch, d_results, d_solution, d_trace, trace_cap, stream=0):
        check(self._L.mpcqp_debug_solve_trace_device(self._h, d_records, int(batch), d_results,
                                                     d_solution or None, d_trace, int(trace_cap),
                                                     stream or None),
              self._h, "mpcqp_debug_solve_trace_device", self._L)

    def build_qp_device(self, d_records, batch, d_P, d_q, d_l, d_u, stream=0):
        check(self._L.mpcqp_build_qp_device(self._h, d_records, int(batch), d_P, d_q, d_l, d_u,
                                            stream or None),
              self._h, "mpcqp_build_qp_device", self._L)

    # -- host convenience --------------------------------------------------------------------------
    def solve_host(self, records, want_solution=False):
        """mpcqp_solve_batch_host on numpy records [B, rec_size]; returns structured results."""
        recs = np.ascontiguousarray(records, dtype=np.float64).reshape(-1, self.rec_size)
        B = recs.shape[0]
        res = np.zeros(B, dtype=RESULT_DTYPE)
        sol = np.zeros((B, self.n)) if want_solution else None
        dp = ctypes.POINTER(ctypes.c_double)
        check(self._L.mpcqp_solve_batch_host(
            self._h, recs.ctypes.data_as(dp), B, res.ctypes.data,
            sol.ctypes.data_as(dp) if sol is not None else None), self._h, "mpcqp_solve_batch_host", self._L)
        return (res, sol) if want_solution else res

    def solve_host_ptr(self, h_records, batch, h_results, h_solution=0):
        """mpcqp_solve_batch_host on raw host pointers (ints).  Pinned (hipHostMalloc'd / torch
        pin_memory) buffers go by one DMA each way; pageable ones through the handle's staging."""
        dp = ctypes.POINTER(ctypes.c_double)
        check(self._L.mpcqp_solve_batch_host(self._h, ctypes.cast(h_records, dp), int(batch), h_results,
                                             ctypes.cast(h_solution, dp) if h_solution else None),
              self._h, "mpcqp_solve_batch_host", self._L)
