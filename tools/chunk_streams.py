"""Experiment: one 4096-robot solve vs the same robots as K chunks on K streams (separate handles),
to measure how much of scale_kernel and of the wave kernel's dispatch tail concurrent launches hide."""
import sys, time, os
import numpy as np, torch
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "go1-qp-mpc-controller_amd"))
import mpcqp
B, N = 4096, 10
dev = torch.device("cuda:0")
st = mpcqp.synthetic_go1(B, seed=1000, gait="trot")
recs = torch.from_numpy(mpcqp.assemble_compute_grf(st, N)).to(dev)
res = torch.zeros((B, mpcqp._lib.RESULT_DOUBLES), dtype=torch.float64, device=dev)
for K in (1, 2, 4, 8):
    solvers = [mpcqp.MpcQpSolver(mpcqp.default_params(N)) for _ in range(K)]
    streams = [torch.cuda.Stream(dev) for _ in range(K)]
    cb = B // K
    for s in solvers:
        s.reserve(cb)
    def run():
        main = torch.cuda.current_stream(dev)
        ev = torch.cuda.Event()
        ev.record(main)
        for i in range(K):
            streams[i].wait_event(ev)
            solvers[i].solve_device(recs[i * cb].data_ptr(), cb, res[i * cb].data_ptr(), 0, streams[i].cuda_stream)
        for i in range(K):
            e2 = torch.cuda.Event(); e2.record(streams[i]); main.wait_event(e2)
    for _ in range(3): run()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(20): run()
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t0) / 20 * 1e3
    print(f"K={K} chunks: {ms:.3f} ms per solve, {B / ms * 1e3:.0f} QP/s", flush=True)
    for s in solvers: s.close()
