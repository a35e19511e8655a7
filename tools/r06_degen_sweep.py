"""Round-6 degenerate-feet investigation (VERDICT r05 "do this" 1), on the GPU.

1. The 37-robot batch of tests/test_gpu_degenerate.py::test_degenerate_robots_in_a_large_batch:
   which planted robots pass scale_kernel's Gram screen, their host Gram pivot ratios and their u0
   error against the oracle.
2. A near-degenerate sweep: feet families that are exactly rank deficient at eps = 0
   (tests/degenerate_cases.near_degenerate: "inplane", "outplane", "point"), eps = 1e-1 .. 1e-9, at
   N = 1, 5, 10, 16 robots each of trot / stance / mixed gait (random mu): per group the host Gram
   ratio range, the hand-off counts [screen, -, S_ii], status / iteration equality and the worst u0
   error against the oracle, for the library under test (MPCQP_LIB: the product, a build without the
   screen (-DMPCQP_SCHUR_GRAM_TOL=0: the Schur form's own error down to rank deficiency) or the
   Riccati form alone (-DMPCQP_WAVE_RICCATI_ONLY)).

usage: python tools/r06_degen_sweep.py OUT.json [--no-large]
"""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(REPO, "go1-qp-mpc-controller_amd"), os.path.join(REPO, "oracle"), os.path.join(REPO, "tests")):
    sys.path.insert(0, p)

import numpy as np  # noqa: E402
import torch  # noqa: E402

import mpcqp  # noqa: E402
import pyoracle  # noqa: E402
from degenerate_cases import degenerate, gram_ratio, near_degenerate  # noqa: E402
from gpu_helpers import rel_err_u0, solve_gpu  # noqa: E402

EPS = [1e-1, 1e-2, 1e-3, 1e-4, 1e-5, 1e-6, 1e-7, 1e-8, 1e-9]
KINDS = ["inplane", "outplane", "point"]


def large_batch():
    N = 10
    st = mpcqp.synthetic_go1(4096, seed=1000, gait="trot")
    recs = mpcqp.assemble_compute_grf(st, N)
    idx = np.unique(np.linspace(5, 4090, 37).astype(np.int64))
    mixed = recs.copy()
    mixed[idx] = degenerate(recs[idx], N)
    with mpcqp.MpcQpSolver(mpcqp.default_params(N), debug=True) as s:
        d_rec = torch.from_numpy(mixed).cuda()
        d_img = torch.zeros((4096, s.scale_image_size), dtype=torch.float64, device="cuda")
        s.scale_image_device(d_rec.data_ptr(), 4096, 0, d_img.data_ptr(), torch.cuda.current_stream().cuda_stream)
        torch.cuda.synchronize()
        flag = d_img.cpu().numpy()[idx, 56 * N + 2]
    with mpcqp.MpcQpSolver(mpcqp.default_params(N)) as s:
        got, _, _ = solve_gpu(s, mixed)
        counts = s.handoff_counts()
    ref = pyoracle.solve_batch(pyoracle.default_params(N), mixed[idx], nthreads=8)
    err = rel_err_u0(got["u0"][idx], ref["u0"])
    ratio = gram_ratio(mixed[idx], N)
    esc = [int(i) for i, f in zip(idx, flag) if f != 1.0]
    out = {"planted": int(idx.size), "flagged": int(np.sum(flag == 1.0)), "handoff_counts": counts,
           "escaped": [{"robot": r, "kind": int(np.nonzero(idx == r)[0][0] % 4),
                        "gram_ratio": float(ratio[np.nonzero(idx == r)[0][0]]),
                        "u0_rel_err": float(err[np.nonzero(idx == r)[0][0]])} for r in esc],
           "max_u0_rel_err_planted": float(err.max()),
           "iters_equal": bool(np.array_equal(got["iters"][idx], ref["iters"])),
           "status_equal": bool(np.array_equal(got["status"][idx], ref["status"]))}
    print("large batch:", json.dumps(out))
    return out


def sweep():
    rows = []
    for N in (1, 5, 10):
        groups = []
        for kind in KINDS:
            for eps in EPS:
                parts = []
                for gi, gait in enumerate(("trot", "stance", "mixed")):
                    st = mpcqp.synthetic_go1(16, seed=7000 + 100 * N + 10 * gi, gait=gait, mixed_mu=(gait == "mixed"))
                    parts.append(mpcqp.assemble_compute_grf(st, N))
                recs = near_degenerate(np.concatenate(parts), N, eps, kind)
                groups.append((kind, eps, recs))
        allrecs = np.concatenate([g[2] for g in groups])
        ref = pyoracle.solve_batch(pyoracle.default_params(N), allrecs, nthreads=16)
        off = 0
        for kind, eps, recs in groups:
            B = recs.shape[0]
            rr = ref[off:off + B]
            off += B
            row = {"N": N, "kind": kind, "eps": eps}
            gr = gram_ratio(recs, N)
            row["gram_ratio_min"] = float(np.nanmin(gr))
            row["gram_ratio_max"] = float(np.nanmax(gr))
            for label in ("lib",):
                with mpcqp.MpcQpSolver(mpcqp.default_params(N)) as s:
                    got, _, _ = solve_gpu(s, recs)
                    counts = s.handoff_counts()
                err = rel_err_u0(got["u0"], rr["u0"])
                row[label] = {"handoff": counts, "max_u0_rel_err": float(np.max(err)),
                              "worst_robot": int(np.argmax(err)),
                              "iters_equal": int(np.sum(got["iters"] == rr["iters"])),
                              "status_equal": int(np.sum(got["status"] == rr["status"])), "robots": B,
                              "finite": bool(np.all(np.isfinite(got["u0"])))}
            rows.append(row)
            print(f"N={N:2d} {kind:8s} eps={eps:.0e} gram [{row['gram_ratio_min']:.1e},{row['gram_ratio_max']:.1e}] "
                  f"lib handoff={row['lib']['handoff']} err={row['lib']['max_u0_rel_err']:.2e} "
                  f"it_eq={row['lib']['iters_equal']}/{B} st_eq={row['lib']['status_equal']}/{B}",
                  flush=True)
    return rows


def main():
    out_path = sys.argv[1]
    pyoracle.build()
    res = {"lib": os.environ.get("MPCQP_LIB", "product")}
    if "--no-large" not in sys.argv:
        res["large_batch"] = large_batch()
    res["sweep"] = sweep()
    with open(out_path, "w") as f:
        json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
