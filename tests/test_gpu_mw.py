"""One-wave-per-horizon-round solver (mpcqp_wave_mw.hip, debug path 4) vs the CPU oracle.

Same algorithm and lane layout as the wave kernel with the R = ceil(N/4) register rounds spread
over R waves of one workgroup (chains in wave 0, a_k / h_k / s_k / x_k exchanged through LDS).
Experimental: slower than path 3 at the bench batch, kept parity-tested because
its per-robot latency is lower.  Gates as the other Riccati paths.
"""
import numpy as np
import pytest

import mpcqp
from test_gpu_riccati import _check_p1_riccati

pytestmark = pytest.mark.gpu


def _mw_solver(params):
    s = mpcqp.MpcQpSolver(params)
    s.set_solver(mpcqp._lib.SOLVER_WAVE_MW)
    return s


@pytest.mark.parametrize("N", [1, 2, 4, 7, 10, 20])
@pytest.mark.parametrize("gait", ["trot", "mixed"])
def test_mw_p1(oracle, N, gait):
    st = mpcqp.synthetic_go1(64, seed=300 + N, gait=gait, mixed_mu=(gait == "mixed"))
    recs = mpcqp.assemble_compute_grf(st, N)
    with _mw_solver(mpcqp.default_params(N)) as s:
        _check_p1_riccati(oracle, s, recs, f"mw N={N} {gait}", min_iter_equal=1.0)


def test_mw_test_mpc_case(oracle):
    rec, q, r = mpcqp.assemble_test_mpc(10)
    p = mpcqp.default_params(10, q_weights=q, r_weights=r)
    with _mw_solver(p) as s:
        _check_p1_riccati(oracle, s, rec[None], "mw test_mpc", min_iter_equal=1.0)


def test_mw_matches_wave_solution():
    """Paths 3 and 4 differ only in rounding (accumulation order of a few mat-vecs)."""
    st = mpcqp.synthetic_go1(128, seed=77, gait="trot")
    recs = mpcqp.assemble_compute_grf(st, 10)
    from gpu_helpers import solve_gpu
    out = {}
    for path in (mpcqp._lib.SOLVER_WAVE, mpcqp._lib.SOLVER_WAVE_MW):
        with mpcqp.MpcQpSolver(mpcqp.default_params(10)) as s:
            s.set_solver(path)
            r, sol, _ = solve_gpu(s, recs)
        out[path] = (r, sol)
    r3, s3 = out[mpcqp._lib.SOLVER_WAVE]
    r4, s4 = out[mpcqp._lib.SOLVER_WAVE_MW]
    assert np.mean(r3["iters"] == r4["iters"]) >= 0.95
    np.testing.assert_array_equal(r3["status"], r4["status"])
    same = r3["iters"] == r4["iters"]
    assert np.max(np.abs(s3[same] - s4[same])) <= 1e-8 * max(1.0, np.max(np.abs(s3)))
