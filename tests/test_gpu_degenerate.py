"""Degenerate foot geometry (mpcqp_schur.h): the Schur-form KKT solve factors
G_k = B6_k R'^-1 B6_k', which is singular when the feet are coincident (e.g. all foot_pos_abs zero
before the first kinematics update) or collinear — B6_k then has rank 3 or 5.  The reference QP is
still strictly convex (R > 0) and OSQP solves it; scale_kernel screens every step's B6_k (Gram
pivot ratio) and the engine hands such robots to the Riccati form (in the same wave).  Gates: status and iteration count identical to the oracle, u0 within 1e-4
relative, every force finite, and the non-degenerate robots of a mixed batch bit-identical to
solving them without the degenerate ones."""
import numpy as np
import pytest
import torch

import mpcqp
from gpu_helpers import rel_err_u0, solve_gpu

pytestmark = pytest.mark.gpu

N = 10


def _degenerate(recs, N=N):
    """Four kinds of rank-deficient feet, cycling over the given records."""
    F = mpcqp._lib.rec_feet(N)
    out = recs.copy()
    line_x = np.array([[0.17, 0.0, -0.3], [0.05, 0.0, -0.3], [-0.05, 0.0, -0.3], [-0.17, 0.0, -0.3]])
    diag = np.array([[0.17, 0.15, -0.3], [0.06, 0.053, -0.3], [-0.06, -0.053, -0.3], [-0.17, -0.15, -0.3]])
    for b in range(out.shape[0]):
        kind = b % 4
        if kind == 0:    # all feet at the body origin
            feet = np.zeros((4, 3))
        elif kind == 1:  # one point below the body
            feet = np.tile([0.02, -0.01, -0.3], (4, 1))
        elif kind == 2:  # collinear along x
            feet = line_x
        else:            # collinear along a diagonal, rotated with the body
            R = out[b, mpcqp._lib.REC_ROT:mpcqp._lib.REC_ROT + 9].reshape(3, 3)
            feet = diag @ R.T
        out[b, F:F + 12 * N] = np.tile(feet.reshape(12), N)
    return out


@pytest.mark.parametrize("gait", ["trot", "stance", "mixed"])
@pytest.mark.parametrize("N", [1, 3, 5, 10])
def test_degenerate_feet_match_oracle(oracle, gait, N):
    """Every Schur horizon (at N <= 5 the screen's wave did not exist)."""
    st = mpcqp.synthetic_go1(32, seed=911, gait=gait, mixed_mu=(gait == "mixed"))
    recs = _degenerate(mpcqp.assemble_compute_grf(st, N), N)
    with mpcqp.MpcQpSolver(mpcqp.default_params(N)) as s:
        got, sol, _ = solve_gpu(s, recs)
    ref = oracle.solve_batch(oracle.default_params(N), recs, nthreads=8)
    assert np.all(np.isfinite(got["u0"])) and np.all(np.isfinite(got["f_body"]))
    np.testing.assert_array_equal(got["status"], ref["status"])
    np.testing.assert_array_equal(got["iters"], ref["iters"])
    assert np.all(rel_err_u0(got["u0"], ref["u0"]) <= 1e-4)


@pytest.mark.parametrize("N", [1, 2, 5, 6, 10])
def test_degenerate_flag_in_scale_image(oracle, N):
    """The screen flags exactly the rank-deficient robots (debug library image, slot 56N + 2) at
    every Schur horizon, the one-wave scale launches (N <= 5) included."""
    st = mpcqp.synthetic_go1(16, seed=912, gait="trot")
    recs = mpcqp.assemble_compute_grf(st, N)
    recs[::2] = _degenerate(recs[::2], N)
    with mpcqp.MpcQpSolver(mpcqp.default_params(N), debug=True) as s:
        d_rec = torch.from_numpy(recs).cuda()
        d_img = torch.zeros((16, s.scale_image_size), dtype=torch.float64, device="cuda")
        s.scale_image_device(d_rec.data_ptr(), 16, 0, d_img.data_ptr(), torch.cuda.current_stream().cuda_stream)
        torch.cuda.synchronize()
        flag = d_img.cpu().numpy()[:, 56 * N + 2]
    np.testing.assert_array_equal(flag, np.tile([1.0, 0.0], 8))


def test_degenerate_robots_in_a_large_batch(oracle):
    """A 4096-robot C2 batch with 37 degenerate robots scattered through it: the screen
    catches exactly those, the rest are untouched (bitwise equal to the batch without them)."""
    st = mpcqp.synthetic_go1(4096, seed=1000, gait="trot")
    recs = mpcqp.assemble_compute_grf(st, N)
    idx = np.unique(np.linspace(5, 4090, 37).astype(np.int64))
    mixed = recs.copy()
    mixed[idx] = _degenerate(recs[idx])
    with mpcqp.MpcQpSolver(mpcqp.default_params(N)) as s:
        clean, _, _ = solve_gpu(s, recs)
        assert s.handoff_counts()[0] == 0
        got, _, _ = solve_gpu(s, mixed)
        handed = s.handoff_counts()[0]
    # the robots the screen flags (debug image slot 56N + 2) are exactly those the Riccati form took
    with mpcqp.MpcQpSolver(mpcqp.default_params(N), debug=True) as s:
        d_rec = torch.from_numpy(mixed).cuda()
        d_img = torch.zeros((4096, s.scale_image_size), dtype=torch.float64, device="cuda")
        s.scale_image_device(d_rec.data_ptr(), 4096, 0, d_img.data_ptr(), torch.cuda.current_stream().cuda_stream)
        torch.cuda.synchronize()
        flagged = np.nonzero(d_img.cpu().numpy()[:, 56 * N + 2] == 1.0)[0]
    assert set(flagged) <= set(idx) and handed == flagged.size and flagged.size >= 0.9 * idx.size
    keep = np.setdiff1d(np.arange(4096), idx)
    for k in ("u0", "iters", "status", "rho_updates"):
        np.testing.assert_array_equal(got[k][keep], clean[k][keep])
    ref = oracle.solve_batch(oracle.default_params(N), mixed[idx], nthreads=8)
    np.testing.assert_array_equal(got["status"][idx], ref["status"])
    np.testing.assert_array_equal(got["iters"][idx], ref["iters"])
    assert np.all(rel_err_u0(got["u0"][idx], ref["u0"]) <= 1e-4)


def test_degenerate_feet_warm_ticks(oracle):
    """Warm-started ticks that start with zero feet (before the first kinematics update) and then
    get real feet: the Riccati form carries the warm slot like the Schur form does."""
    T, B = 5, 16
    ticks = mpcqp.records.synthetic_go1_ticks(B, T, seed=61, gait="trot", swing_ticks=3)
    recs_t = np.stack([mpcqp.assemble_compute_grf(s, N) for s in ticks])
    recs_t[0:2] = _degenerate(recs_t[0:2].reshape(-1, recs_t.shape[-1])).reshape(2, B, -1)
    p = mpcqp.default_params(N)
    out = np.zeros((T, B), dtype=mpcqp.RESULT_DTYPE)
    with mpcqp.MpcQpSolver(p) as s:
        d_state = torch.zeros((B, s.warm_state_size), dtype=torch.float64, device="cuda")
        d_res = torch.zeros((B, mpcqp._lib.RESULT_DOUBLES), dtype=torch.float64, device="cuda")
        stream = torch.cuda.current_stream().cuda_stream
        for t in range(T):
            d_rec = torch.from_numpy(np.ascontiguousarray(recs_t[t])).cuda()
            s.solve_warm_device(d_rec.data_ptr(), B, d_state.data_ptr(), d_res.data_ptr(), 0, stream)
            torch.cuda.synchronize()
            out[t] = np.frombuffer(d_res.cpu().numpy().tobytes(), dtype=mpcqp.RESULT_DTYPE)
    ref = oracle.solve_sequence(oracle.default_params(N), recs_t, nthreads=8)
    for t in range(T):
        np.testing.assert_array_equal(out[t]["status"], ref[t]["status"], err_msg=f"tick {t}")
        assert np.mean(out[t]["iters"] == ref[t]["iters"]) >= 0.99, f"tick {t}"
        assert np.all(rel_err_u0(out[t]["u0"], ref[t]["u0"]) <= 1e-4), f"tick {t}"
