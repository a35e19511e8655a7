"""A/B of warm-started tick sequences between two builds of libmpcqp (MPCQP_LIB) and the oracle:
per tick, status / iterations / rho updates of the first robots.
usage: MPCQP_LIB=... python tools/ab_warm.py [--robots 8] [--ticks 4]"""
import argparse
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "go1-qp-mpc-controller_amd"), os.path.join(REPO, "oracle")]
import mpcqp  # noqa: E402
import pyoracle  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--robots", type=int, default=8)
    ap.add_argument("--ticks", type=int, default=4)
    a = ap.parse_args()
    B, T = a.robots, a.ticks
    ticks = mpcqp.records.synthetic_go1_ticks(B, T, seed=41, gait="trot", swing_ticks=5)
    recs_t = np.stack([mpcqp.assemble_compute_grf(s, 10) for s in ticks])
    ref = pyoracle.solve_sequence(pyoracle.default_params(10), recs_t, nthreads=4)
    p = mpcqp.default_params(10)
    with mpcqp.MpcQpSolver(p) as s:
        st = torch.zeros((B, s.warm_state_size), dtype=torch.float64, device="cuda")
        res = torch.zeros((B, mpcqp._lib.RESULT_DOUBLES), dtype=torch.float64, device="cuda")
        for t in range(T):
            d = torch.from_numpy(np.ascontiguousarray(recs_t[t])).cuda()
            s.solve_warm_device(d.data_ptr(), B, st.data_ptr(), res.data_ptr(), 0, torch.cuda.current_stream().cuda_stream)
            torch.cuda.synchronize()
            g = np.frombuffer(res.cpu().numpy().tobytes(), dtype=mpcqp.RESULT_DTYPE)
            print(f"tick {t} gpu iters {g['iters'].tolist()} rho_up {g['rho_updates'].tolist()} rho {np.round(g['rho'], 5).tolist()}")
            print(f"tick {t} ref iters {ref[t]['iters'].tolist()} rho_up {ref[t]['rho_updates'].tolist()} rho {np.round(ref[t]['rho'], 5).tolist()}")
            err = np.max(np.abs(g["u0"] - ref[t]["u0"]), axis=1)
            print(f"tick {t} |du0| {np.array2string(err, precision=2)}")
            if t == 0:
                np.save(os.environ.get("AB_SLOT_OUT", "/tmp/slot.npy"), st.cpu().numpy())
        w = st.cpu().numpy()
        print("slot flag/rho/c/mu", w[:, :4].tolist())


if __name__ == "__main__":
    main()
