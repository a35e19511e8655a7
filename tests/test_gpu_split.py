"""The wave-path batch split (mpcqp_debug_set_split): a batch solved as K parts on the handle's
internal streams gives bitwise the results of one launch, for cold solves, warm-started ticks and
robots the Schur form hands to the Riccati form, and the hand-off counters sum over the parts."""
import numpy as np
import pytest

torch = pytest.importorskip("torch")

import mpcqp  # noqa: E402

pytestmark = pytest.mark.gpu

RD = mpcqp._lib.RESULT_DOUBLES


def _solve(s, recs, parts, state=None):
    s.set_split(parts)
    d_rec = torch.from_numpy(recs).cuda()
    res = torch.zeros((recs.shape[0], RD), dtype=torch.float64, device="cuda")
    stream = torch.cuda.current_stream().cuda_stream
    if state is None:
        s.solve_device(d_rec.data_ptr(), recs.shape[0], res.data_ptr(), 0, stream)
    else:
        s.solve_warm_device(d_rec.data_ptr(), recs.shape[0], state.data_ptr(), res.data_ptr(), 0, stream)
    torch.cuda.synchronize()
    return res.cpu().numpy().view(np.uint64).copy()


@pytest.mark.parametrize("horizon,gait,batch", [(10, "trot", 4096), (10, "mixed", 3001), (20, "trot", 2048)])
def test_split_is_bitwise_one_launch(horizon, gait, batch):
    st = mpcqp.synthetic_go1(batch, seed=77, gait=gait, mixed_mu=gait == "mixed")
    recs = mpcqp.assemble_compute_grf(st, horizon)
    with mpcqp.MpcQpSolver(mpcqp.default_params(horizon)) as s:
        s.reserve(batch)
        ref = _solve(s, recs, 1)
        for parts in (0, 2, 3, 4, 7, 8):
            got = _solve(s, recs, parts)
            assert np.array_equal(got, ref), f"parts={parts}"


def test_split_handoff_counts_sum_over_parts():
    # stance robots with heavy state weights cross the Schur form's conditioning bound after a rho
    # update (tests/test_gpu_conditioning.py); the counts must not depend on the split
    st = mpcqp.synthetic_go1(4096, seed=5, gait="stance")
    recs = mpcqp.assemble_compute_grf(st, 10)
    p0 = mpcqp.default_params(10)
    p = mpcqp.default_params(10, q_weights=[w * 100.0 for w in p0.q_weights])
    with mpcqp.MpcQpSolver(p) as s:
        s.reserve(4096)
        ref = _solve(s, recs, 1)
        c1 = s.handoff_counts()
        for parts in (4, 8):
            got = _solve(s, recs, parts)
            assert np.array_equal(got, ref)
            assert s.handoff_counts() == c1
    assert c1[1] + c1[2] > 0


def test_split_warm_ticks_bitwise():
    horizon, batch = 10, 4096
    ticks = [mpcqp.assemble_compute_grf(mpcqp.synthetic_go1(batch, seed=300 + t, gait="trot"), horizon)
             for t in range(3)]
    outs = {}
    for parts in (1, 4):
        with mpcqp.MpcQpSolver(mpcqp.default_params(horizon)) as s:
            s.reserve(batch)
            ws = s.warm_state_size
            state = torch.zeros((batch, ws), dtype=torch.float64, device="cuda")
            outs[parts] = [_solve(s, r, parts, state) for r in ticks]
            outs[parts].append(state.cpu().numpy().view(np.uint64).copy())
    for a, b in zip(outs[1], outs[4]):
        assert np.array_equal(a, b)


def _solve_full(s, recs, parts, trace_cap):
    """Results, full-horizon solutions and check traces (the per-part offsets of the
    solution and trace pointers, and trace_cap - b0, at every part boundary)."""
    B = recs.shape[0]
    s.set_split(parts)
    d_rec = torch.from_numpy(recs).cuda()
    res = torch.zeros((B, RD), dtype=torch.float64, device="cuda")
    sol = torch.full((B, s.n), float("nan"), dtype=torch.float64, device="cuda")
    tr = torch.full((B, 64, 4), -1.0, dtype=torch.float64, device="cuda")
    s.solve_device_trace(d_rec.data_ptr(), B, res.data_ptr(), sol.data_ptr(), tr.data_ptr(), trace_cap,
                         torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    return [x.cpu().numpy().view(np.uint64).copy() for x in (res, sol, tr)]


def test_split_solution_and_trace_offsets():
    batch, trace_cap = 3001, 1700  # the cap ends inside part 1 of 3, inside part 3 of 7
    st = mpcqp.synthetic_go1(batch, seed=78, gait="mixed", mixed_mu=True)
    recs = mpcqp.assemble_compute_grf(st, 10)
    with mpcqp.MpcQpSolver(mpcqp.default_params(10)) as s:
        s.reserve(batch)
        ref = _solve_full(s, recs, 1, trace_cap)
        for parts in (3, 7):
            got = _solve_full(s, recs, parts, trace_cap)
            for a, b, what in zip(got, ref, ("results", "solution", "trace")):
                assert np.array_equal(a, b), f"parts={parts}: {what}"
    # robots past the cap keep the untouched trace (-1.0)
    assert np.all(ref[2].reshape(batch, -1)[trace_cap:] == np.float64(-1.0).view(np.uint64))
    assert not np.any(np.isnan(ref[1].view(np.float64)))


def test_weighted_split_bitwise(monkeypatch):
    """MPCQP_SPLIT_W (read at handle creation) sizes the parts unevenly: part 0 a quarter, part 1
    three quarters of the batch."""
    batch = 4096
    st = mpcqp.synthetic_go1(batch, seed=79, gait="trot")
    recs = mpcqp.assemble_compute_grf(st, 10)
    with mpcqp.MpcQpSolver(mpcqp.default_params(10)) as s:
        ref = _solve_full(s, recs, 1, batch)
    monkeypatch.setenv("MPCQP_SPLIT_W", "1,3")
    with mpcqp.MpcQpSolver(mpcqp.default_params(10)) as s:
        got = _solve_full(s, recs, 2, batch)
    for a, b, what in zip(got, ref, ("results", "solution", "trace")):
        assert np.array_equal(a, b), what
