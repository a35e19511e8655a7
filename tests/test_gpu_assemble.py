"""On-device input assembly (mpcqp_assemble_records_device) vs the oracle's
orc_assemble_compute_grf: bitwise-equal records for horizons 1..20, and the chained
assemble -> solve on one stream gives the oracle's solve of the same robots."""
import numpy as np
import pytest
import torch

import mpcqp
from test_assemble import state_struct

pytestmark = pytest.mark.gpu


def assemble_gpu(rows, N):
    B = rows.shape[0]
    d_st = torch.from_numpy(np.ascontiguousarray(rows)).cuda()
    d_rec = torch.full((B, mpcqp.rec_size(N)), np.nan, dtype=torch.float64, device="cuda")
    mpcqp.assemble_records_device(N, d_st.data_ptr(), B, d_rec.data_ptr(), torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    return d_rec


@pytest.mark.parametrize("N", [1, 7, 10, 20])
def test_device_records_bitwise_oracle(oracle, N):
    st = mpcqp.synthetic_go1(129, seed=40 + N, gait="mixed", mixed_mu=True)
    rows = mpcqp.pack_states(st)
    got = assemble_gpu(rows, N).cpu().numpy()
    for b in range(rows.shape[0]):
        ref = oracle.assemble_compute_grf(state_struct(oracle, rows[b]), N)
        np.testing.assert_array_equal(got[b], ref)


def test_assemble_then_solve(oracle):
    B = 2048
    st = mpcqp.synthetic_go1(B, seed=99, gait="trot")
    rows = mpcqp.pack_states(st)
    d_rec = assemble_gpu(rows, 10)
    with mpcqp.MpcQpSolver(mpcqp.default_params(10)) as s:
        d_res = torch.zeros((B, mpcqp._lib.RESULT_DOUBLES), dtype=torch.float64, device="cuda")
        s.solve_device(d_rec.data_ptr(), B, d_res.data_ptr(), 0, torch.cuda.current_stream().cuda_stream)
        torch.cuda.synchronize()
    got = np.frombuffer(d_res.cpu().numpy().tobytes(), dtype=mpcqp.RESULT_DTYPE)
    sub = slice(0, 256)
    ref = oracle.solve_batch(oracle.default_params(10), d_rec.cpu().numpy()[sub], nthreads=8)
    np.testing.assert_array_equal(got["status"][sub], ref["status"])
    np.testing.assert_array_equal(got["iters"][sub], ref["iters"])
    err = np.abs(got["u0"][sub] - ref["u0"]).max(1) / np.maximum(np.abs(ref["u0"]).max(1), 1.0)
    assert err.max() <= 1e-4
