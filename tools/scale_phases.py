#!/usr/bin/env python3
"""scale_kernel phase timing: run a library built with -DMPCQP_SCALE_TIMING (tools/build_variant.sh
OUT.so 10 -DMPCQP_SCALE_TIMING, selected with MPCQP_LIB; MPCQP_N=20 for another horizon); thread 0 of each robot writes {id,
s_memtime} pairs over its own record.  Reports median shader-clock cycles per phase: 0 -> 1 record
load + B_w + gradient sweeps, 1 -> 2 column init, 2 -> 3 first column pass (H columns generated),
3 -> 4 Ruiz pass 0, 4 -> 5 passes 1..9, 5 -> 6 image write; and the robot's whole span; 7 = kernel
entry (before the record load), 8 = wave 0's gradient sweeps done."""
import json
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "go1-qp-mpc-controller_amd"))
import mpcqp  # noqa: E402

B = 4096
NH = int(os.environ.get("MPCQP_N", "10"))  # horizon (the variant library must be built for it)
st = mpcqp.synthetic_go1(B, seed=1000, gait="trot")
recs = mpcqp.assemble_compute_grf(st, NH)
with mpcqp.MpcQpSolver(mpcqp.default_params(NH, max_iter=1)) as s:
    d_res = torch.zeros((B, mpcqp._lib.RESULT_DOUBLES), dtype=torch.float64, device="cuda")
    for _ in range(3):
        d_rec = torch.from_numpy(recs).cuda()
        s.solve_device(d_rec.data_ptr(), B, d_res.data_ptr(), 0, torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    m = d_rec.cpu().numpy()[:, :18].reshape(B, 9, 2)
names = ["bw_gradient", "column_init", "first_colmax", "pass0", "passes1_9", "image_write"]
out = {}
for i, nm in enumerate(names):
    out[nm] = float(np.median(m[:, i + 1, 1] - m[:, i, 1]))
out["span"] = float(np.median(m[:, 6, 1] - m[:, 0, 1]))
out["entry_to_0"] = float(np.median(m[:, 0, 1] - m[:, 7, 1]))  # record load and finiteness test
out["sweep_end"] = float(np.median(m[:, 8, 1] - m[:, 0, 1]))   # wave 0: B_w rows, forward / backward sweeps
out["entry_span"] = float(np.median(m[:, 6, 1] - m[:, 7, 1]))
print(json.dumps(out, indent=1))
if len(sys.argv) > 1:
    json.dump(out, open(sys.argv[1], "w"), indent=1)
