"""Two-phase cold solve (mpcqp_debug_set_park / MPCQP_PARK; csrc/mpcqp_wave.hip ParkLayout,
order_kernel): robots still running at the update_info iteration `cut` save their state, are
sorted by dua_res / eps_dual of that check and resumed longest-first by a second launch.  Resuming
restores exactly what the loop carries, so results, full solutions and check traces are bitwise
those of the one-phase solve — for trot, mixed gaits with random mu, heavy weights whose robots the
Schur form hands to the Riccati form (before and after the cut), degenerate feet, and short
horizons."""
import numpy as np
import pytest
import torch

import mpcqp
from degenerate_cases import degenerate

pytestmark = pytest.mark.gpu

RD = mpcqp._lib.RESULT_DOUBLES


def _solve(s, recs, cut):
    B = recs.shape[0]
    s.set_park(cut)
    d_rec = torch.from_numpy(np.ascontiguousarray(recs)).cuda()
    res = torch.zeros((B, RD), dtype=torch.float64, device="cuda")
    sol = torch.full((B, s.n), float("nan"), dtype=torch.float64, device="cuda")
    tr = torch.full((B, 64, 4), -1.0, dtype=torch.float64, device="cuda")
    s.solve_device_trace(d_rec.data_ptr(), B, res.data_ptr(), sol.data_ptr(), tr.data_ptr(), B,
                         torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    return [x.cpu().numpy().view(np.uint64).copy() for x in (res, sol, tr)], s.handoff_counts()


def _cases():
    out = []
    st = mpcqp.synthetic_go1(4096, seed=1000, gait="trot")
    out.append(("c2_trot", 10, mpcqp.default_params(10), mpcqp.assemble_compute_grf(st, 10)))
    st = mpcqp.synthetic_go1(2048, seed=5, gait="mixed", mixed_mu=True)
    out.append(("c5_mixed", 10, mpcqp.default_params(10), mpcqp.assemble_compute_grf(st, 10)))
    p0 = mpcqp.default_params(10)
    heavy = mpcqp.default_params(10, q_weights=[w * 100.0 for w in p0.q_weights])
    st = mpcqp.synthetic_go1(1024, seed=6, gait="stance")
    out.append(("stance_heavy", 10, heavy, mpcqp.assemble_compute_grf(st, 10)))
    st = mpcqp.synthetic_go1(512, seed=7, gait="trot")
    recs = mpcqp.assemble_compute_grf(st, 10)
    recs[::9] = degenerate(recs[::9], 10)
    out.append(("degenerate", 10, mpcqp.default_params(10), recs))
    for N in (1, 5):
        st = mpcqp.synthetic_go1(1024, seed=8 + N, gait="mixed", mixed_mu=True)
        out.append((f"mixed_N{N}", N, mpcqp.default_params(N), mpcqp.assemble_compute_grf(st, N)))
    return out


@pytest.mark.parametrize("case", _cases(), ids=lambda c: c[0])
def test_park_is_bitwise_one_phase(case):
    name, N, params, recs = case
    with mpcqp.MpcQpSolver(params) as s:
        ref, c_ref = _solve(s, recs, 0)
        for cut in (25, 50, 100):
            got, c_got = _solve(s, recs, cut)
            for a, b, what in zip(got, ref, ("results", "solution", "trace")):
                assert np.array_equal(a, b), f"{name} cut={cut}: {what}"
            assert c_got == c_ref, f"{name} cut={cut}: hand-off counts {c_got} vs {c_ref}"


def test_park_repeated_solves_and_batch_changes():
    """Park slots and the resume order are reused across solves of different batches: no robot of an
    earlier solve is resumed by a later one."""
    st = mpcqp.synthetic_go1(3000, seed=21, gait="trot")
    big = mpcqp.assemble_compute_grf(st, 10)
    small = big[:700].copy()
    small[::5] = degenerate(small[::5], 10)  # robots that return before the loop
    with mpcqp.MpcQpSolver(mpcqp.default_params(10)) as s:
        ref_small, _ = _solve(s, small, 0)
        ref_big, _ = _solve(s, big, 0)
        for _ in range(2):
            assert all(np.array_equal(a, b) for a, b in zip(_solve(s, big, 50)[0], ref_big))
            assert all(np.array_equal(a, b) for a, b in zip(_solve(s, small, 50)[0], ref_small))
