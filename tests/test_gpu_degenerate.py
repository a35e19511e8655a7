"""Degenerate foot geometry (mpcqp_schur.h): the Schur-form KKT solve factors
G_k = B6_k R'^-1 B6_k', which is singular when the feet are coincident (e.g. all foot_pos_abs zero
before the first kinematics update) or collinear — B6_k then has rank 3 or 5.  The reference QP is
still strictly convex (R > 0) and OSQP solves it; scale_kernel screens every step's B6_k (Gram
pivot ratio below SCHUR_GRAM_TOL = 1e-6) and the engine hands such robots to the Riccati form (in
the same wave).

Contract: the screen flags exactly the robots whose Gram pivot ratio (host
restatement, tests/degenerate_cases.gram_ratio) is below the threshold — every exactly rank-deficient
robot, and near-degenerate ones by their ratio — and every robot, flagged or not, is solved to the
accuracy the engine reaches elsewhere: status and iteration count identical to the oracle, u0 within
the 1e-8 regression sentinel (the SURVEY §8(c) 1e-4 gate stays as well), every force finite.  The
near-collinear sweep shows what the Schur form does just above the threshold."""
import numpy as np
import pytest
import torch

import mpcqp
from degenerate_cases import SCHUR_GRAM_TOL, degenerate, gram_ratio, near_degenerate
from gpu_helpers import note, rel_err_u0, sentinel, solve_gpu

pytestmark = pytest.mark.gpu

N = 10
SENTINEL = 1e-8


def _flags(recs, N):
    """scale_kernel's hand-off flag per robot (debug library image, slot 56N + 2)."""
    B = recs.shape[0]
    with mpcqp.MpcQpSolver(mpcqp.default_params(N), debug=True) as s:
        d_rec = torch.from_numpy(np.ascontiguousarray(recs)).cuda()
        d_img = torch.zeros((B, s.scale_image_size), dtype=torch.float64, device="cuda")
        s.scale_image_device(d_rec.data_ptr(), B, 0, d_img.data_ptr(), torch.cuda.current_stream().cuda_stream)
        torch.cuda.synchronize()
        return d_img.cpu().numpy()[:, 56 * N + 2] == 1.0


def _predicted(recs, N):
    """(must be flagged, may be flagged): ratios within 1 % of the threshold may go either way."""
    g = gram_ratio(recs, N)
    return g < SCHUR_GRAM_TOL / 1.01, g < SCHUR_GRAM_TOL * 1.01


@pytest.mark.parametrize("gait", ["trot", "stance", "mixed"])
@pytest.mark.parametrize("N", [1, 3, 5, 10])
def test_degenerate_feet_match_oracle(oracle, gait, N):
    """Every Schur horizon (at N <= 5 the screen's wave did not exist)."""
    st = mpcqp.synthetic_go1(32, seed=911, gait=gait, mixed_mu=(gait == "mixed"))
    recs = degenerate(mpcqp.assemble_compute_grf(st, N), N)
    with mpcqp.MpcQpSolver(mpcqp.default_params(N)) as s:
        got, sol, _ = solve_gpu(s, recs)
    ref = oracle.solve_batch(oracle.default_params(N), recs, nthreads=8)
    assert np.all(np.isfinite(got["u0"])) and np.all(np.isfinite(got["f_body"]))
    np.testing.assert_array_equal(got["status"], ref["status"])
    np.testing.assert_array_equal(got["iters"], ref["iters"])
    err = rel_err_u0(got["u0"], ref["u0"])
    assert np.all(err <= 1e-4)
    sentinel(err, SENTINEL, f"degenerate {gait} N={N}")


@pytest.mark.parametrize("N", [1, 2, 5, 6, 10])
def test_degenerate_flag_in_scale_image(N):
    """The screen flags exactly the robots the host restatement predicts at every Schur horizon (the
    one-wave scale launches, N <= 5, included), and every exactly rank-deficient kind (0-2)."""
    st = mpcqp.synthetic_go1(16, seed=912, gait="trot")
    recs = mpcqp.assemble_compute_grf(st, N)
    recs[::2] = degenerate(recs[::2], N)
    flag = _flags(recs, N)
    must, may = _predicted(recs, N)
    assert np.all(flag[must]) and not np.any(flag[~may])
    kinds = np.full(16, -1)
    kinds[::2] = np.arange(8) % 4
    assert np.all(flag[(kinds >= 0) & (kinds <= 2)])
    assert not np.any(flag[1::2])


def test_degenerate_robots_in_a_large_batch(oracle):
    """A 4096-robot C2 batch with 37 degenerate robots scattered through it.  The screen flags exactly
    the planted robots whose Gram ratio is below the threshold: all of kinds 0-2 and those of the
    near-collinear kind 3 below it (35 of 37; robots 799 and 3522 sit at 3.8e-6 and 9.6e-6 and are
    solved by the Schur form, round 6: u0 within 4e-13).  Both routes meet the sentinel; the clean
    robots are bitwise unchanged."""
    st = mpcqp.synthetic_go1(4096, seed=1000, gait="trot")
    recs = mpcqp.assemble_compute_grf(st, N)
    idx = np.unique(np.linspace(5, 4090, 37).astype(np.int64))
    mixed = recs.copy()
    mixed[idx] = degenerate(recs[idx], N)
    with mpcqp.MpcQpSolver(mpcqp.default_params(N)) as s:
        clean, _, _ = solve_gpu(s, recs)
        assert s.handoff_counts()[0] == 0
        got, _, _ = solve_gpu(s, mixed)
        handed = s.handoff_counts()[0]
    flag = _flags(mixed, N)
    must, may = _predicted(mixed, N)
    assert np.all(flag[must]) and not np.any(flag[~may])
    flagged = np.nonzero(flag)[0]
    assert set(flagged) <= set(idx) and handed == flagged.size
    assert np.all(flag[idx[np.arange(idx.size) % 4 <= 2]])  # every exactly rank-deficient robot
    keep = np.setdiff1d(np.arange(4096), idx)
    for k in ("u0", "iters", "status", "rho_updates"):
        np.testing.assert_array_equal(got[k][keep], clean[k][keep])
    ref = oracle.solve_batch(oracle.default_params(N), mixed[idx], nthreads=8)
    np.testing.assert_array_equal(got["status"][idx], ref["status"])
    np.testing.assert_array_equal(got["iters"][idx], ref["iters"])
    err = rel_err_u0(got["u0"][idx], ref["u0"])
    assert np.all(err <= 1e-4)
    esc = ~flag[idx]
    g = gram_ratio(mixed[idx], N)
    note("degenerate large batch", planted=int(idx.size), flagged=int(flagged.size),
         escaped=[int(r) for r in idx[esc]], escaped_gram_ratio=[float(x) for x in g[esc]],
         escaped_u0_rel_err=[float(x) for x in err[esc]])
    sentinel(err[~esc], SENTINEL, "degenerate large batch: screened robots (Riccati form)")
    sentinel(err[esc] if esc.any() else np.zeros(1), SENTINEL, "degenerate large batch: robots above the threshold (Schur form)")


@pytest.mark.parametrize("kind", ["inplane", "outplane", "point"])
@pytest.mark.parametrize("eps", [1e-2, 1e-4, 1e-6, 1e-8])
@pytest.mark.parametrize("N", [1, 5, 10])
def test_near_degenerate_sweep(oracle, N, eps, kind):
    """Feet that are exactly rank deficient at eps = 0 (collinear with one foot moved eps in or out of
    the line's plane, or four coincident feet spread by eps): Gram ratios from ~1e-2 down to ~0.  The
    screen count equals the host prediction, and every robot — screened to the Riccati form or solved
    by the Schur form just above the threshold — meets the sentinel."""
    parts = []
    for gi, gait in enumerate(("trot", "stance", "mixed")):
        st = mpcqp.synthetic_go1(16, seed=7000 + 100 * N + 10 * gi, gait=gait, mixed_mu=(gait == "mixed"))
        parts.append(mpcqp.assemble_compute_grf(st, N))
    recs = near_degenerate(np.concatenate(parts), N, eps, kind)
    with mpcqp.MpcQpSolver(mpcqp.default_params(N)) as s:
        got, _, _ = solve_gpu(s, recs)
        counts = s.handoff_counts()
    must, may = _predicted(recs, N)
    assert int(np.sum(must)) <= counts[0] <= int(np.sum(may))
    ref = oracle.solve_batch(oracle.default_params(N), recs, nthreads=8)
    assert np.all(np.isfinite(got["u0"]))
    np.testing.assert_array_equal(got["status"], ref["status"])
    np.testing.assert_array_equal(got["iters"], ref["iters"])
    err = rel_err_u0(got["u0"], ref["u0"])
    assert np.all(err <= 1e-4)
    g = gram_ratio(recs, N)
    note(f"near-degenerate N={N} {kind} eps={eps:.0e}", gram_ratio_min=float(g.min()), gram_ratio_max=float(g.max()),
         screened=int(counts[0]), conditioning_handoffs=int(counts[1] + counts[2]), max_u0_rel_err=float(err.max()))
    sentinel(err, SENTINEL, f"near-degenerate N={N} {kind} eps={eps:.0e}")


def test_degenerate_feet_warm_ticks(oracle):
    """Warm-started ticks that start with zero feet (before the first kinematics update) and then
    get real feet: the Riccati form carries the warm slot like the Schur form does."""
    T, B = 5, 16
    ticks = mpcqp.records.synthetic_go1_ticks(B, T, seed=61, gait="trot", swing_ticks=3)
    recs_t = np.stack([mpcqp.assemble_compute_grf(s, N) for s in ticks])
    recs_t[0:2] = degenerate(recs_t[0:2].reshape(-1, recs_t.shape[-1]), N).reshape(2, B, -1)
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
    errs = []
    for t in range(T):
        np.testing.assert_array_equal(out[t]["status"], ref[t]["status"], err_msg=f"tick {t}")
        assert np.mean(out[t]["iters"] == ref[t]["iters"]) >= 0.99, f"tick {t}"
        e = rel_err_u0(out[t]["u0"], ref[t]["u0"])
        assert np.all(e <= 1e-4), f"tick {t}"
        errs.append(e)
    sentinel(np.concatenate(errs), SENTINEL, "degenerate warm ticks")
