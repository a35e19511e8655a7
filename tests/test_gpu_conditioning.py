"""Ill-conditioned Schur cores (mpcqp_schur.h, the hand-off): with four feet in contact and state
weights a few times the Go1 defaults, S = I + L'CL gets large and the push-through identity
R'^-1 w - B'(I - S^-1)B w loses digits (u0 off the oracle by up to 1e-3 at x 100, round-4 fuzz,
profiles/r04/smax).  A robot leaves the Schur form at a check when the latest factorization's max S_ii
times that iteration's observed cancellation (schur_solve's amp = max|R'^-1 w| / max|u|) exceeds
SCHUR_AMP = 5e4, or S_max exceeds SCHUR_SMAX = 1e4, and is solved again by the Riccati form in its
own wave (wave_kernel).
Gates: status and iterations equal to the oracle, u0 within SURVEY §8(c)'s 1e-4, and a regression
sentinel at the accuracy the hand-off achieves."""
import numpy as np
import pytest
import torch

import mpcqp
from gpu_helpers import note, rel_err_u0, sentinel, solve_gpu

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("scale", [1.0, 5.0, 100.0])
@pytest.mark.parametrize("gait", ["stance", "mixed"])
def test_heavy_state_weights_match_oracle(oracle, gait, scale):
    N, B = 10, 512
    st = mpcqp.synthetic_go1(B, seed=7000 + 97 * 5 + N, gait=gait, mixed_mu=(gait == "mixed"))
    recs = mpcqp.assemble_compute_grf(st, N)
    p0 = mpcqp.default_params(N)
    p = mpcqp.default_params(N, q_weights=[w * scale for w in p0.q_weights])
    with mpcqp.MpcQpSolver(p) as s:
        got, _, _ = solve_gpu(s, recs)
        counts = s.handoff_counts()
    note(f"hand-offs {gait} x{scale:g}", counts=list(counts))
    ref = oracle.solve_batch(oracle.default_params(N, q=list(p.q_weights), r=list(p.r_weights)), recs, nthreads=8)
    np.testing.assert_array_equal(got["status"], ref["status"])
    np.testing.assert_array_equal(got["iters"], ref["iters"])
    err = rel_err_u0(got["u0"], ref["u0"])
    assert np.all(err <= 1e-4), float(err.max())
    # regression sentinel: the hand-off (S_max * amp > 5e4 or S_max > 1e4) keeps these within ~2.5e-9
    # (without it 1.4e-5 at x1 stance, 5e-5 at x5, 1e-3 at x100; profiles/r06/cancel)
    sentinel(err, 1e-8, f"conditioning {gait} x{scale:g}")
    if gait == "stance":
        assert counts[1] + counts[2] > 0  # the hand-off is exercised here


@pytest.mark.parametrize("N", [3, 6, 10])
def test_heavy_weights_shorter_horizons(oracle, N):
    """The Schur form serves every N <= 10: the hand-off at shorter horizons."""
    B = 256
    st = mpcqp.synthetic_go1(B, seed=7100 + N, gait="stance")
    recs = mpcqp.assemble_compute_grf(st, N)
    p0 = mpcqp.default_params(N)
    p = mpcqp.default_params(N, q_weights=[w * 20.0 for w in p0.q_weights])
    with mpcqp.MpcQpSolver(p) as s:
        got, _, _ = solve_gpu(s, recs)
        counts = s.handoff_counts()
    note(f"hand-offs N={N} stance x20", counts=list(counts))
    ref = oracle.solve_batch(oracle.default_params(N, q=list(p.q_weights), r=list(p.r_weights)), recs, nthreads=8)
    np.testing.assert_array_equal(got["status"], ref["status"])
    np.testing.assert_array_equal(got["iters"], ref["iters"])
    err = rel_err_u0(got["u0"], ref["u0"])
    assert np.all(err <= 1e-4), float(err.max())
    sentinel(err, 1e-8, f"conditioning N={N} stance x20")


def test_heavy_weights_warm_ticks(oracle):
    """Warm-started ticks with heavy weights: robots handed to the Riccati form part-way through a
    sequence keep their warm slot (the Schur form writes nothing before it hands over; the Riccati
    form reads the previous tick's slot and writes this tick's)."""
    N, T, B = 10, 6, 48
    ticks = mpcqp.records.synthetic_go1_ticks(B, T, seed=7200, gait="trot", swing_ticks=3)
    recs_t = np.stack([mpcqp.assemble_compute_grf(s, N) for s in ticks])
    recs_t[:, :, mpcqp._lib.REC_CONTACTS:mpcqp._lib.REC_CONTACTS + 4] = 1.0  # four feet down
    p0 = mpcqp.default_params(N)
    p = mpcqp.default_params(N, q_weights=[w * 100.0 for w in p0.q_weights])
    out = np.zeros((T, B), dtype=mpcqp.RESULT_DTYPE)
    handed = 0
    with mpcqp.MpcQpSolver(p) as s:
        d_state = torch.zeros((B, s.warm_state_size), dtype=torch.float64, device="cuda")
        d_res = torch.zeros((B, mpcqp._lib.RESULT_DOUBLES), dtype=torch.float64, device="cuda")
        stream = torch.cuda.current_stream().cuda_stream
        for t in range(T):
            d_rec = torch.from_numpy(np.ascontiguousarray(recs_t[t])).cuda()
            s.solve_warm_device(d_rec.data_ptr(), B, d_state.data_ptr(), d_res.data_ptr(), 0, stream)
            torch.cuda.synchronize()
            out[t] = np.frombuffer(d_res.cpu().numpy().tobytes(), dtype=mpcqp.RESULT_DTYPE)
            c = s.handoff_counts()
            handed += c[1] + c[2]
    note("hand-offs warm ticks stance x100", handed=handed, ticks=T, robots=B)
    op = oracle.default_params(N, q=list(p.q_weights), r=list(p.r_weights))
    ref = oracle.solve_sequence(op, recs_t, nthreads=8)
    worst = 0.0
    for t in range(T):
        np.testing.assert_array_equal(out[t]["status"], ref[t]["status"], err_msg=f"tick {t}")
        assert np.mean(out[t]["iters"] == ref[t]["iters"]) >= 0.97, f"tick {t}"
        err = rel_err_u0(out[t]["u0"], ref[t]["u0"])
        assert np.all(err <= 1e-4), f"tick {t}"
        worst = max(worst, float(err.max()))
    # (warm-started ticks keep the previous tick's adapted rho: round 6 measured 2.2e-7 here with the
    # S_max * amp hand-off, as with round 5's S_max bound; the cold heavy-weight cases above reach 1e-9)
    sentinel(np.array([worst]), 1e-6, "conditioning warm ticks x100")
    assert handed > 0
