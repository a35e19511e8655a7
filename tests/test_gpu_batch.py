"""Batch-shape properties of the default solve path (scale_kernel -> wave_kernel).

Every robot's QP is solved by its own wavefront from its own record, so a robot's result cannot
depend on which batch it is in or where: the same record gives bitwise the same u0, solution,
status and iteration count in a batch of 1, in a ragged batch, and at any offset of a large one.
Empty batches are a no-op that succeeds (mpcqp.h: batch 0 returns MPCQP_OK without a launch).
"""
import numpy as np
import pytest
import torch

import mpcqp
from gpu_helpers import solve_gpu

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def big():
    st = mpcqp.synthetic_go1(4100, seed=901, gait="mixed", mixed_mu=True)
    recs = mpcqp.assemble_compute_grf(st, 10)
    with mpcqp.MpcQpSolver(mpcqp.default_params(10)) as s:
        res, sol, _ = solve_gpu(s, recs)
    return recs, res, sol


def test_empty_batch_is_ok():
    with mpcqp.MpcQpSolver(mpcqp.default_params(10)) as s:
        d = torch.zeros(1, dtype=torch.float64, device="cuda")
        s.solve_device(d.data_ptr(), 0, d.data_ptr(), 0, torch.cuda.current_stream().cuda_stream)
        torch.cuda.synchronize()


@pytest.mark.parametrize("offset,count", [(0, 1), (4099, 1), (17, 33), (1000, 1025), (3, 4097)])
def test_batch_invariance(big, offset, count):
    recs, res, sol = big
    with mpcqp.MpcQpSolver(mpcqp.default_params(10)) as s:
        r2, s2, _ = solve_gpu(s, recs[offset:offset + count])
    sl = slice(offset, offset + count)
    np.testing.assert_array_equal(r2["status"], res["status"][sl])
    np.testing.assert_array_equal(r2["iters"], res["iters"][sl])
    np.testing.assert_array_equal(r2["u0"], res["u0"][sl])
    np.testing.assert_array_equal(s2, sol[sl])


def test_repeat_solves_are_bitwise_identical(big):
    recs, res, sol = big
    with mpcqp.MpcQpSolver(mpcqp.default_params(10)) as s:
        for _ in range(2):
            r2, s2, _ = solve_gpu(s, recs[:777])
            np.testing.assert_array_equal(r2["u0"], res["u0"][:777])
            np.testing.assert_array_equal(s2, sol[:777])
