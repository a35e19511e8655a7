"""Helpers for -m gpu tests: run the HIP path through the C ABI on torch-allocated buffers."""
import numpy as np
import torch

import mpcqp


def solve_gpu(solver: mpcqp.MpcQpSolver, recs: np.ndarray, trace=False):
    """Returns (results structured array, solution [B,n], trace [B,64,4] or None)."""
    recs = np.ascontiguousarray(recs, dtype=np.float64).reshape(-1, solver.rec_size)
    B = recs.shape[0]
    d_rec = torch.from_numpy(recs).cuda()
    d_res = torch.zeros((B, mpcqp._lib.RESULT_DOUBLES), dtype=torch.float64, device="cuda")
    d_sol = torch.zeros((B, solver.n), dtype=torch.float64, device="cuda")
    stream = torch.cuda.current_stream().cuda_stream
    tr = None
    if trace:
        d_tr = torch.full((B, 64, 4), float("nan"), dtype=torch.float64, device="cuda")
        solver.solve_device_trace(d_rec.data_ptr(), B, d_res.data_ptr(), d_sol.data_ptr(),
                                  d_tr.data_ptr(), B, stream)
    else:
        solver.solve_device(d_rec.data_ptr(), B, d_res.data_ptr(), d_sol.data_ptr(), stream)
    torch.cuda.synchronize()
    res = np.frombuffer(d_res.cpu().numpy().tobytes(), dtype=mpcqp.RESULT_DTYPE).copy()
    if trace:
        tr = d_tr.cpu().numpy()
    return res, d_sol.cpu().numpy(), tr


def build_qp_gpu(solver: mpcqp.MpcQpSolver, recs: np.ndarray):
    recs = np.ascontiguousarray(recs, dtype=np.float64).reshape(-1, solver.rec_size)
    B = recs.shape[0]
    n, m = solver.n, solver.m
    d_rec = torch.from_numpy(recs).cuda()
    P = torch.zeros((B, n, n), dtype=torch.float64, device="cuda")
    q = torch.zeros((B, n), dtype=torch.float64, device="cuda")
    l = torch.zeros((B, m), dtype=torch.float64, device="cuda")
    u = torch.zeros((B, m), dtype=torch.float64, device="cuda")
    solver.build_qp_device(d_rec.data_ptr(), B, P.data_ptr(), q.data_ptr(), l.data_ptr(), u.data_ptr(),
                           torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    return P.cpu().numpy(), q.cpu().numpy(), l.cpu().numpy(), u.cpu().numpy()


def rel_err_u0(a, b):
    """‖Δu0‖∞ / max(‖u0_ref‖∞, 1) per instance (SURVEY §8(c) parity gate)."""
    a = np.asarray(a).reshape(-1, 12)
    b = np.asarray(b).reshape(-1, 12)
    return np.max(np.abs(a - b), axis=1) / np.maximum(np.max(np.abs(b), axis=1), 1.0)


def sentinel(err, bound, label):
    """Regression sentinel at the accuracy the engine achieves (the SURVEY §8(c) 1e-4 gate stays in
    each test as well): prints the measured maximum, appends it to $MPCQP_SENTINEL_LOG (JSON lines)
    when set, and fails above `bound` unless $MPCQP_SENTINEL_CALIBRATE is set."""
    import json
    import os
    m = float(np.max(err)) if np.size(err) else 0.0
    print(f"[sentinel] {label}: max u0 rel err {m:.3e} (sentinel {bound:.0e})")
    log = os.environ.get("MPCQP_SENTINEL_LOG")
    if log:
        with open(log, "a") as f:
            f.write(json.dumps({"label": label, "max_rel_err_u0": m, "sentinel": bound}) + "\n")
    if not os.environ.get("MPCQP_SENTINEL_CALIBRATE"):
        assert m <= bound, f"{label}: u0 error {m:.3e} above the regression sentinel {bound:.0e}"
    return m


def note(label, **values):
    """Prints a measurement and appends it to $MPCQP_SENTINEL_LOG (JSON lines) when set."""
    import json
    import os
    print(f"[note] {label}: {values}")
    log = os.environ.get("MPCQP_SENTINEL_LOG")
    if log:
        with open(log, "a") as f:
            f.write(json.dumps({"label": label, **values}) + "\n")
