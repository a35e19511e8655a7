"""Per-iteration and per-factorization cost of a solve path: fixed iteration counts (termination
checks and adaptive rho off), 4096 trot robots, N = 10.  usage: dx_timing.py [path ...]"""
import os, sys
import numpy as np
import torch
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "go1-qp-mpc-controller_amd"))
import mpcqp

paths = [int(a) for a in sys.argv[1:]] or [3, 5]
B, N = 4096, 10
st = mpcqp.synthetic_go1(B, seed=1, gait="trot")
recs = torch.from_numpy(mpcqp.assemble_compute_grf(st, N)).cuda()
res = torch.zeros((B, mpcqp._lib.RESULT_DOUBLES), dtype=torch.float64, device="cuda")
stream = torch.cuda.current_stream().cuda_stream
for path in paths:
    row = []
    for it in (1, 26, 51, 101):
        p = mpcqp.default_params(N)
        p.max_iter = it
        p.check_termination = 0
        p.adaptive_rho = 0
        with mpcqp.MpcQpSolver(p) as s:
            s.set_solver(path)
            for _ in range(2):
                s.solve_device(recs.data_ptr(), B, res.data_ptr(), 0, stream)
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(5):
                s.solve_device(recs.data_ptr(), B, res.data_ptr(), 0, stream)
            e1.record()
            torch.cuda.synchronize()
            row.append((it, e0.elapsed_time(e1) / 5))
    its = np.array([r[0] for r in row]); ms = np.array([r[1] for r in row])
    slope = np.polyfit(its, ms, 1)[0]
    print(f"path {path}: " + "  ".join(f"{i} it {m:.3f} ms" for i, m in row) +
          f"  | per iteration {slope * 1e3:.2f} us/batch, 1-iteration solve {ms[0]:.3f} ms", flush=True)
