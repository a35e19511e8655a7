"""Device torque map (mpcqp_joint_torques_device) vs the oracle's compute_joint_torques
restatement: bit-identical (same operation order, contraction off), over ticks that cross the
10-tick start-up window, and fused behind the GRF solve (forces never leave the device)."""
import numpy as np
import pytest
import torch

import mpcqp
from gpu_helpers import solve_gpu
from test_torques import torque_inputs

pytestmark = pytest.mark.gpu


def _run_device(rec, f_body_results, counters, tau, ticks):
    d_rec = torch.from_numpy(np.ascontiguousarray(rec)).cuda()
    d_res = torch.from_numpy(np.ascontiguousarray(f_body_results).view(np.float64).reshape(len(rec), -1)).cuda()
    d_cnt = torch.from_numpy(counters.copy()).cuda()
    d_tau = torch.from_numpy(tau.copy()).cuda()
    stream = torch.cuda.current_stream().cuda_stream
    for _ in range(ticks):
        mpcqp.joint_torques_device(d_rec.data_ptr(), d_res.data_ptr(), len(rec), d_cnt.data_ptr(),
                                   d_tau.data_ptr(), stream)
    torch.cuda.synchronize()
    return d_cnt.cpu().numpy(), d_tau.cpu().numpy()


@pytest.mark.parametrize("B,ticks", [(1, 12), (257, 10), (4096, 11)])
def test_torques_bit_identical_to_oracle(oracle, B, ticks):
    J, fkin, contacts, f_grf = torque_inputs(B, 10 + B)
    if B > 1:
        f_grf[1, 3] = np.nan          # a NaN stance force
        contacts[1, 1] = True
        J[2, 0] = 0.0                 # a singular swing Jacobian
        contacts[2, 0] = False
    rec = mpcqp.assemble_torque_records(J, fkin, contacts, km_foot=[0.1, 0.1, 0.04])
    res = np.zeros(B, dtype=mpcqp.RESULT_DTYPE)
    res["f_body"] = f_grf
    counters = np.random.default_rng(B).integers(0, 3, B).astype(np.int32)
    tau0 = np.random.default_rng(B + 1).normal(0.0, 1.0, (B, 12))
    got_c, got_t = _run_device(rec, res, counters, tau0, ticks)
    ref_c, ref_t = counters.copy(), tau0.copy()
    for _ in range(ticks):
        oracle.joint_torques(rec, f_grf, ref_c, ref_t)
    np.testing.assert_array_equal(got_c, ref_c)
    np.testing.assert_array_equal(got_t, ref_t)


def test_torques_fused_after_solve(oracle):
    """solve -> torque map on the device; the map reads mpcqp_result.f_body in place."""
    B = 512
    st = mpcqp.synthetic_go1(B, seed=77, gait="mixed", mixed_mu=True)
    recs = mpcqp.assemble_compute_grf(st, 10)
    J, fkin, _, _ = torque_inputs(B, 5)
    tq = mpcqp.assemble_torque_records(J, fkin, st.contacts)
    with mpcqp.MpcQpSolver(mpcqp.default_params(10)) as s:
        d_rec = torch.from_numpy(recs).cuda()
        d_res = torch.zeros((B, mpcqp._lib.RESULT_DOUBLES), dtype=torch.float64, device="cuda")
        d_tq = torch.from_numpy(tq).cuda()
        d_cnt = torch.full((B,), 9, dtype=torch.int32, device="cuda")
        d_tau = torch.zeros((B, 12), dtype=torch.float64, device="cuda")
        stream = torch.cuda.current_stream().cuda_stream
        s.solve_device(d_rec.data_ptr(), B, d_res.data_ptr(), 0, stream)
        mpcqp.joint_torques_device(d_tq.data_ptr(), d_res.data_ptr(), B, d_cnt.data_ptr(), d_tau.data_ptr(),
                                   stream)
        torch.cuda.synchronize()
        res = np.frombuffer(d_res.cpu().numpy().tobytes(), dtype=mpcqp.RESULT_DTYPE)
        tau = d_tau.cpu().numpy()
    ref_c = np.full(B, 9, dtype=np.int32)
    ref_t = np.zeros((B, 12))
    oracle.joint_torques(tq, res["f_body"], ref_c, ref_t)
    np.testing.assert_array_equal(tau, ref_t)
    # and the forces themselves are the oracle's to the parity gate
    ref = oracle.solve_batch(oracle.default_params(10), recs, nthreads=8)
    err = np.max(np.abs(res["f_body"] - ref["f_body"]), axis=1) / np.maximum(np.max(np.abs(ref["f_body"]), axis=1), 1)
    assert np.all(err <= 1e-4)
