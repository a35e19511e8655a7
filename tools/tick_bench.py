"""Per-tick time of the fused control tick (mpcqp.tick.ControlTick: assemble -> warm solve ->
torque map) for a fleet of robots, eager launches vs one HIP-graph replay (HIP events).
usage: python tools/tick_bench.py [--batch 4096] [--ticks 40]"""
import argparse
import json
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "go1-qp-mpc-controller_amd"), os.path.join(REPO, "tests")]
import mpcqp  # noqa: E402
from mpcqp.records import synthetic_go1_ticks  # noqa: E402
from mpcqp.tick import ControlTick  # noqa: E402
from test_torques import torque_inputs  # noqa: E402  (synthetic Jacobians)


def timed(tick, states, use_graph):
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    tot = 0.0
    for st in states:
        tick.states.copy_(st)
        ev[0].record()
        tick.replay() if use_graph else tick.step()
        ev[1].record()
        torch.cuda.synchronize()
        tot += ev[0].elapsed_time(ev[1])
    return tot / len(states)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=4096)
    ap.add_argument("--ticks", type=int, default=40)
    a = ap.parse_args()
    B = a.batch
    sts = [torch.from_numpy(mpcqp.pack_states(s)).cuda() for s in synthetic_go1_ticks(B, a.ticks, seed=3)]
    J, fkin, _, _ = torque_inputs(B, 1)
    out = {"batch": B, "ticks": a.ticks}
    for mode in ("eager", "graph"):
        t = ControlTick(B)
        t.tq_records.copy_(torch.from_numpy(mpcqp.assemble_torque_records(J, fkin, sts[0][:, 59:63].cpu().numpy() != 0)))
        if mode == "graph":
            t.capture()
        out[f"{mode}_ms_per_tick"] = timed(t, sts, mode == "graph")
        res = t.results.cpu().numpy()
        t.close()
    out["robots_per_s_graph"] = B / (out["graph_ms_per_tick"] * 1e-3)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
