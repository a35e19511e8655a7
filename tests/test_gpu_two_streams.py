"""Two handles on two streams solving independent batches concurrently (the
caller-side remedy for a batch's dispatch tail): every result bitwise equal to the same batch
solved alone on one stream, for cold and warm-started solves."""
import numpy as np
import pytest
import torch

import mpcqp

pytestmark = pytest.mark.gpu


def _rows(t):
    return np.frombuffer(t.cpu().numpy().tobytes(), dtype=mpcqp.RESULT_DTYPE).copy()


def test_two_handles_two_streams_bitwise_equal():
    N, B = 10, 2048
    rec_a = mpcqp.assemble_compute_grf(mpcqp.synthetic_go1(B, seed=5, gait="trot"), N)
    rec_b = mpcqp.assemble_compute_grf(mpcqp.synthetic_go1(B, seed=6, gait="mixed", mixed_mu=True), N)
    RD = mpcqp._lib.RESULT_DOUBLES
    p = mpcqp.default_params(N)
    with mpcqp.MpcQpSolver(p) as s1, mpcqp.MpcQpSolver(p) as s2:
        da, db = torch.from_numpy(rec_a).cuda(), torch.from_numpy(rec_b).cuda()
        ra1 = torch.zeros((B, RD), dtype=torch.float64, device="cuda")
        rb1 = torch.zeros_like(ra1)
        cur = torch.cuda.current_stream().cuda_stream
        s1.solve_device(da.data_ptr(), B, ra1.data_ptr(), 0, cur)  # alone, one stream
        s1.solve_device(db.data_ptr(), B, rb1.data_ptr(), 0, cur)
        torch.cuda.synchronize()
        sa, sb = torch.cuda.Stream(), torch.cuda.Stream()
        ra2, rb2 = torch.zeros_like(ra1), torch.zeros_like(ra1)
        for _ in range(3):  # overlapping launches, each handle on its own stream
            s1.solve_device(da.data_ptr(), B, ra2.data_ptr(), 0, sa.cuda_stream)
            s2.solve_device(db.data_ptr(), B, rb2.data_ptr(), 0, sb.cuda_stream)
        torch.cuda.synchronize()
        assert _rows(ra2).tobytes() == _rows(ra1).tobytes()
        assert _rows(rb2).tobytes() == _rows(rb1).tobytes()
        # warm-started ticks, two fleets interleaved on the two streams
        wa = torch.zeros((B, s1.warm_state_size), dtype=torch.float64, device="cuda")
        wb = torch.zeros_like(wa)
        wa1, wb1 = torch.zeros_like(wa), torch.zeros_like(wa)
        for t in range(3):
            s1.solve_warm_device(da.data_ptr(), B, wa1.data_ptr(), ra1.data_ptr(), 0, cur)
            s1.solve_warm_device(db.data_ptr(), B, wb1.data_ptr(), rb1.data_ptr(), 0, cur)
        torch.cuda.synchronize()
        for t in range(3):
            s1.solve_warm_device(da.data_ptr(), B, wa.data_ptr(), ra2.data_ptr(), 0, sa.cuda_stream)
            s2.solve_warm_device(db.data_ptr(), B, wb.data_ptr(), rb2.data_ptr(), 0, sb.cuda_stream)
        torch.cuda.synchronize()
        assert _rows(ra2).tobytes() == _rows(ra1).tobytes()
        assert _rows(rb2).tobytes() == _rows(rb1).tobytes()
        assert wa.cpu().numpy().tobytes() == wa1.cpu().numpy().tobytes()
