"""Balance QP on the device (mpcqp_balance_solve_device) vs the CPU oracle: same status, same
iteration and rho-update counts, u0 / f_body within 1e-9 of the oracle (both binary64, same
operation order with contraction off), on the golden set, on full-size seeded batches and on
edge cases (NaN record, max_iter, all swing)."""
import numpy as np
import pytest
import torch

import mpcqp
from mpcqp import balance as bal

pytestmark = pytest.mark.gpu
GOLDEN = "tests/golden/balance.npz"


def run_gpu(recs, params=None, bp=None):
    B = recs.shape[0]
    params = params or mpcqp.default_params(1)
    bp = bp or mpcqp._lib.default_balance_params()
    with mpcqp.MpcQpSolver(params) as s:
        d_rec = torch.from_numpy(np.ascontiguousarray(recs)).cuda()
        d_res = torch.zeros((B, mpcqp._lib.RESULT_DOUBLES), dtype=torch.float64, device="cuda")
        s.balance_solve_device(bp, d_rec.data_ptr(), B, d_res.data_ptr(), torch.cuda.current_stream().cuda_stream)
        torch.cuda.synchronize()
    return np.frombuffer(d_res.cpu().numpy().tobytes(), dtype=mpcqp.RESULT_DTYPE)


def assert_parity(got, ref, tol=1e-9):
    np.testing.assert_array_equal(got["status"], ref["status"])
    np.testing.assert_array_equal(got["iters"], ref["iters"])
    np.testing.assert_array_equal(got["rho_updates"], ref["rho_updates"])
    np.testing.assert_array_equal(got["nan_legs"], ref["nan_legs"])
    ok = ~np.isnan(ref["u0"]).any(1)
    scale = np.maximum(np.abs(ref["u0"][ok]).max(1, keepdims=True), 1.0)
    assert np.all(np.abs(got["u0"][ok] - ref["u0"][ok]) <= tol * scale)
    assert np.all(np.abs(got["f_body"][ok] - ref["f_body"][ok]) <= tol * scale)
    assert np.all(np.isnan(got["u0"][~ok]))


def test_balance_golden():
    d = np.load(GOLDEN)
    got = run_gpu(d["records"])
    np.testing.assert_array_equal(got["status"], d["status"])
    np.testing.assert_array_equal(got["iters"], d["iters"])
    scale = np.maximum(np.abs(d["u0"]).max(1, keepdims=True), 1.0)
    assert np.all(np.abs(got["u0"] - d["u0"]) <= 1e-9 * scale)


@pytest.mark.parametrize("B,gait,seed", [(1, "stance", 3), (300, "trot", 4), (4096, "mixed", 5)])
def test_balance_vs_oracle(oracle, B, gait, seed):
    recs = bal.assemble_balance(mpcqp.synthetic_go1(B, seed=seed, gait=gait))
    got = run_gpu(recs)
    ref = oracle.balance_solve_batch(oracle.default_params(1), oracle.default_balance_params(), recs, 8)
    assert_parity(got, ref)


def test_balance_edge_cases(oracle):
    recs = bal.assemble_balance(mpcqp.synthetic_go1(4, seed=9, gait="stance"))
    recs[1, bal.BAL_POS] = np.inf
    recs[2, bal.BAL_CONTACTS:bal.BAL_CONTACTS + 4] = 0.0
    got = run_gpu(recs)
    ref = oracle.balance_solve_batch(oracle.default_params(1), oracle.default_balance_params(), recs)
    assert_parity(got, ref)
    assert got["status"][1] == mpcqp._lib.STATUS_NAN_INPUT
    # max_iter below convergence, other weights / friction
    p = mpcqp.default_params(1, max_iter=10)
    bp = mpcqp._lib.default_balance_params(mu=0.4, r=1e-4, q_diag=[2, 2, 5, 300, 300, 50])
    op = oracle.default_params(1, max_iter=10)
    obp = oracle.default_balance_params()
    obp.mu, obp.r = 0.4, 1e-4
    for i, v in enumerate([2, 2, 5, 300, 300, 50]):
        obp.q_diag[i] = v
    assert_parity(run_gpu(recs, p, bp), oracle.balance_solve_batch(op, obp, recs))
