"""scale_kernel time vs the number of Ruiz passes (p.scaling): per-pass cost and fixed cost.
Run under rocprofv3 --kernel-trace --stats once per value (argv[1])."""
import sys, os
import torch
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "go1-qp-mpc-controller_amd"))
import mpcqp
B, N = 4096, 10
sc = int(sys.argv[1])
dev = torch.device("cuda:0")
st = mpcqp.synthetic_go1(B, seed=1000, gait="trot")
recs = torch.from_numpy(mpcqp.assemble_compute_grf(st, N)).to(dev)
res = torch.zeros((B, mpcqp._lib.RESULT_DOUBLES), dtype=torch.float64, device=dev)
s = mpcqp.MpcQpSolver(mpcqp.default_params(N, scaling=sc, max_iter=1))
s.reserve(B)
for _ in range(10):
    s.solve_device(recs.data_ptr(), B, res.data_ptr(), 0, torch.cuda.current_stream().cuda_stream)
torch.cuda.synchronize()
