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


@pytest.mark.parametrize("world", [2, 8])
def test_sharded_solve_equals_single_solve(world):
    """C3's sharding on one device: the global 8192-robot batch solved as world contiguous
    shard_range shards (what each rank of bench.py --gpus world solves) and concatenated in rank
    order (what allgather_forces returns) is bitwise the single-launch solve (bench.py --gpus 1
    --batch 8192)."""
    from mpcqp.distributed import shard_range
    total = 8192
    st = mpcqp.synthetic_go1(total, seed=1000, gait="trot")
    recs = mpcqp.assemble_compute_grf(st, 10)
    with mpcqp.MpcQpSolver(mpcqp.default_params(10)) as s:
        whole, _, _ = solve_gpu(s, recs)
        parts = [solve_gpu(s, recs[b:e])[0] for b, e in (shard_range(total, world, r) for r in range(world))]
    cat = np.concatenate(parts)
    np.testing.assert_array_equal(cat["u0"], whole["u0"])
    np.testing.assert_array_equal(cat["iters"], whole["iters"])
    np.testing.assert_array_equal(cat["status"], whole["status"])


@pytest.mark.parametrize("pinned", [False, True])
def test_host_wrapper_equals_device_path(big, pinned):
    """mpcqp_solve_batch_host (records 9.6 MB and solutions 3.9 MB: several 2-MiB staging chunks
    each way when pageable, one DMA each way when pinned) returns bitwise the device path's
    results, on repeated calls."""
    recs, res, sol = big
    B = 4096
    with mpcqp.MpcQpSolver(mpcqp.default_params(10)) as s:
        for _ in range(2):
            if pinned:
                h_rec = torch.from_numpy(np.ascontiguousarray(recs[:B])).pin_memory()
                h_res = torch.zeros((B, mpcqp._lib.RESULT_DOUBLES), dtype=torch.float64).pin_memory()
                h_sol = torch.zeros((B, s.n), dtype=torch.float64).pin_memory()
                s.solve_host_ptr(h_rec.data_ptr(), B, h_res.data_ptr(), h_sol.data_ptr())
                r2 = np.frombuffer(h_res.numpy().tobytes(), dtype=mpcqp.RESULT_DTYPE)
                s2 = h_sol.numpy()
            else:
                r2, s2 = s.solve_host(recs[:B], want_solution=True)
            np.testing.assert_array_equal(r2["u0"], res["u0"][:B])
            np.testing.assert_array_equal(r2["iters"], res["iters"][:B])
            np.testing.assert_array_equal(s2, sol[:B])
