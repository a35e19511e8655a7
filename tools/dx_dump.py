"""Debug: K and K^-1 of path 5's first factorization (variant built with -DDXE_DUMP) vs numpy."""
import os, sys
import numpy as np
import torch
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "go1-qp-mpc-controller_amd"))
sys.path.insert(0, os.path.join(REPO, "oracle"))
import mpcqp, pyoracle
N = int(sys.argv[1]) if len(sys.argv) > 1 else 10
n, m = 12 * N, 20 * N
B = 4
st = mpcqp.synthetic_go1(B, seed=5, gait="trot")
recs = mpcqp.assemble_compute_grf(st, N)
p = mpcqp.default_params(N)
STEPS = int(sys.argv[2]) if len(sys.argv) > 2 else 4000
p.max_iter = STEPS
sz = 2 * n * n + n + m + 2
with mpcqp.MpcQpSolver(p) as s:
    s.set_solver(5)
    d_rec = torch.from_numpy(recs).cuda()
    d_res = torch.zeros((B, mpcqp._lib.RESULT_DOUBLES), dtype=torch.float64, device="cuda")
    d_sol = torch.zeros((B, sz), dtype=torch.float64, device="cuda")
    s.solve_device(d_rec.data_ptr(), B, d_res.data_ptr(), d_sol.data_ptr(), torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    out = d_sol.cpu().numpy()
op = pyoracle.default_params(N)


def gj_steps(K, k):
    a = K.copy()
    for p in range(k):
        piv = 1.0 / a[p, p]
        col = a[:, p].copy()
        rowp = a[p, :] * piv
        a -= np.outer(col, rowp)
        a[p, :] = rowp
        a[:, p] = -col * piv
        a[p, p] = piv
    return a

for b in range(B):
    K = out[b, :n * n].reshape(n, n)
    Ki = out[b, n * n:2 * n * n].reshape(n, n)
    D = out[b, 2 * n * n:2 * n * n + n]
    E = out[b, 2 * n * n + n:2 * n * n + n + m]
    c, rho = out[b, -2], out[b, -1]
    ref = gj_steps(K, min(STEPS, n))
    err = np.abs(Ki - ref) / np.max(np.abs(ref))
    bad = np.argwhere(err > 1e-8)
    print(f"  after {min(STEPS, n)} steps: max rel err {err.max():.3g}, {len(bad)} bad entries; first bad (row, col): {bad[:12].tolist()}")
    if STEPS == 1 and b == 0:
        rows_bad = sorted(set(bad[:, 0].tolist()))
        cols_bad = sorted(set(bad[:, 1].tolist()))
        print("  bad rows", rows_bad[:10], "...", len(rows_bad), " bad cols", cols_bad[:5], "...", len(cols_bad))
        print("  got  Ki[1,60:64]", Ki[1, 60:64], " K", K[1, 60:64])
        print("  ref     [1,60:64]", ref[1, 60:64])
        piv = 1 / K[0, 0]
        for name, rp in [("rowp half0", K[0, 0:4]), ("rowp 60", K[0, 60:64]), ("col 60", K[60:64, 0])]:
            print("  hyp", name, K[1, 60:64] - K[1, 0] * piv * rp)
        print("  delta/(K10 piv)", (Ki[1, 60:64] - K[1, 60:64]) / (-K[1, 0] * piv))
        print("  delta row 70", (Ki[70, 60:64] - K[70, 60:64]) / (-K[70, 0] * piv), "ref", K[0, 60:64])
    P, q, l, u, _ = pyoracle.build_qp(op, recs[b])
    A = np.zeros((m, n))
    mu = recs[b][mpcqp._lib.REC_MU] if hasattr(mpcqp._lib, "REC_MU") else None
    print(f"robot {b}: c={c:.4g} rho={rho} sym={np.max(np.abs(K - K.T)):.3g} |K|={np.max(np.abs(K)):.3g} "
          f"|K Ki - I|={np.max(np.abs(K @ Ki - np.eye(n))):.3g} |Ki - inv(K)|/|Ki|={np.max(np.abs(Ki - np.linalg.inv(K))) / np.max(np.abs(Ki)):.3g}")
    Pt = c * (D[:, None] * P * D[None, :])
    dK = K - Pt - 1e-6 * np.eye(n)
    # off the 3x3 foot blocks K must equal c D H D exactly
    mask = np.ones((n, n), bool)
    for f in range(n // 3):
        mask[3 * f:3 * f + 3, 3 * f:3 * f + 3] = False
    print(f"   off-block |K - cDHD|={np.max(np.abs(dK[mask])):.3g}  foot-block residual max {np.max(np.abs(dK[~mask])):.3g} "
          f"D range {D.min():.3g}..{D.max():.3g} E range {E.min():.3g}..{E.max():.3g}")
    np.set_printoptions(precision=4, suppress=True, linewidth=150)
    print("   foot block 0 of K - cDHD - sigma I:\n", dK[:3, :3])
