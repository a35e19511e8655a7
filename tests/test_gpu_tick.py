"""Fused control tick (assemble -> warm solve -> torque map) on one stream, eager and as a captured
HIP graph: the graph replays bitwise what the eager ticks produce, and the first tick's forces
equal the oracle's cold solve of the host-assembled records."""
import numpy as np
import pytest
import torch

import mpcqp
from mpcqp.records import synthetic_go1_ticks
from mpcqp.tick import ControlTick
from test_torques import torque_inputs

pytestmark = pytest.mark.gpu


def _drive(tick, states_t, tq, use_graph):
    outs = []
    tick.tq_records.copy_(torch.from_numpy(tq))
    for t, st in enumerate(states_t):
        tick.states.copy_(torch.from_numpy(mpcqp.pack_states(st)))
        if use_graph:
            if tick.graph is None:
                tick.capture()
            tick.replay()
        else:
            tick.step()
        torch.cuda.synchronize()
        res = np.frombuffer(tick.results.cpu().numpy().tobytes(), dtype=mpcqp.RESULT_DTYPE).copy()
        outs.append((res, tick.torques.cpu().numpy().copy(), tick.counter.cpu().numpy().copy()))
    return outs


def test_tick_graph_matches_eager_and_oracle(oracle):
    B, T = 512, 14
    states_t = synthetic_go1_ticks(B, T, seed=8, gait="trot")
    J, fkin, _, _ = torque_inputs(B, 3)
    tq = mpcqp.assemble_torque_records(J, fkin, states_t[0].contacts)
    a, b = ControlTick(B), ControlTick(B)
    try:
        eager = _drive(a, states_t, tq, use_graph=False)
        graph = _drive(b, states_t, tq, use_graph=True)
    finally:
        a.close()
        b.close()
    for (ra, ta, ca), (rb, tb, cb) in zip(eager, graph):
        np.testing.assert_array_equal(ra["u0"], rb["u0"])
        np.testing.assert_array_equal(ra["iters"], rb["iters"])
        np.testing.assert_array_equal(ta, tb)
        np.testing.assert_array_equal(ca, cb)
    assert eager[-1][2].min() == T and np.abs(eager[-1][1]).max() > 0  # past the 10-tick start-up
    ref = oracle.solve_batch(oracle.default_params(10), mpcqp.assemble_compute_grf(states_t[0], 10), nthreads=8)
    r0 = eager[0][0]
    np.testing.assert_array_equal(r0["status"], ref["status"])
    err = np.abs(r0["u0"] - ref["u0"]).max(1) / np.maximum(np.abs(ref["u0"]).max(1), 1.0)
    assert err.max() <= 1e-4
