"""Foot geometries that make B6_k rank deficient or nearly so, and the host restatement of
scale_kernel's Gram screen (csrc/mpcqp_wave.hip, "Degenerate-foot screen").  Pure numpy: the GPU
tests (test_gpu_degenerate.py), the CPU tests and tools/r06_degen_sweep.py share it.

B6_k (rows 6-11 of B_d(k), ConvexMpc.cpp:132-143, Utils.cpp:35-41): rows 0-2 = I_w^-1 [r_l]x dt per
leg l, rows 3-5 = dt/m I per leg.  The screen takes the Cholesky pivots of the Gram matrix
B6_k B6_k' relative to its diagonal; collinear feet give rank 5 (one pivot ratio ~0), coincident feet
rank 3."""
import numpy as np

import mpcqp

# scale_kernel's screen threshold (csrc/mpcqp_wave_common.h MPCQP_SCHUR_GRAM_TOL; a CPU test checks
# the two agree).  Round 6 measured the Schur form's accuracy below it (profiles/r06/degenerate):
# u0 within 1.2e-9 of the oracle down to Gram ratios ~1e-12 without the screen, so the threshold
# leaves five to six orders of margin.
SCHUR_GRAM_TOL = 1e-6

# feet (body frame) on a line along x (rank 5), and a near-collinear diagonal
LINE_X = np.array([[0.17, 0.0, -0.3], [0.05, 0.0, -0.3], [-0.05, 0.0, -0.3], [-0.17, 0.0, -0.3]])
DIAG = np.array([[0.17, 0.15, -0.3], [0.06, 0.053, -0.3], [-0.06, -0.053, -0.3], [-0.17, -0.15, -0.3]])
POINT = np.array([0.02, -0.01, -0.3])


def _rot(recs, b):
    return recs[b, mpcqp._lib.REC_ROT:mpcqp._lib.REC_ROT + 9].reshape(3, 3)


def degenerate(recs, N):
    """Four kinds of rank-deficient (or nearly so) feet, cycling over the records: 0 all feet at the
    body origin, 1 one point below the body, 2 collinear along x, 3 the near-collinear diagonal
    (DIAG: foot 1 sits 6e-5 off the line of feet 0 and 3), rotated with the body."""
    F = mpcqp._lib.rec_feet(N)
    out = recs.copy()
    for b in range(out.shape[0]):
        kind = b % 4
        if kind == 0:
            feet = np.zeros((4, 3))
        elif kind == 1:
            feet = np.tile(POINT, (4, 1))
        elif kind == 2:
            feet = LINE_X
        else:
            feet = DIAG @ _rot(out, b).T
        out[b, F:F + 12 * N] = np.tile(feet.reshape(12), N)
    return out


def near_degenerate(recs, N, eps, kind):
    """Every record's feet (world-aligned, rotated with the body) moved to a family that is exactly
    rank deficient at eps = 0: "inplane" LINE_X with foot 1 moved eps along body y, "outplane" the
    same along body z, "point" all four feet at POINT spread by eps (foot l moved eps along axis l,
    foot 3 along the diagonal)."""
    F = mpcqp._lib.rec_feet(N)
    out = recs.copy()
    if kind == "inplane":
        fb = LINE_X.copy()
        fb[1, 1] += eps
    elif kind == "outplane":
        fb = LINE_X.copy()
        fb[1, 2] += eps
    elif kind == "point":
        fb = np.tile(POINT, (4, 1))
        fb[0, 0] += eps
        fb[1, 1] += eps
        fb[2, 2] += eps
        fb[3] += eps / np.sqrt(3.0)
    else:
        raise ValueError(kind)
    for b in range(out.shape[0]):
        feet = fb @ _rot(out, b).T
        out[b, F:F + 12 * N] = np.tile(feet.reshape(12), N)
    return out


def gram_ratio(recs, N):
    """Per robot, the smallest Cholesky pivot ratio s_c / G_cc of G_k = B6_k B6_k' over the steps
    (the quantity scale_kernel compares with SCHUR_GRAM_TOL; numpy, not bitwise the kernel's)."""
    F = mpcqp._lib.rec_feet(N)
    out = np.empty(recs.shape[0])
    for b in range(recs.shape[0]):
        r = recs[b]
        R = r[mpcqp._lib.REC_ROT:mpcqp._lib.REC_ROT + 9].reshape(3, 3)
        Ib = r[mpcqp._lib.REC_INERTIA:mpcqp._lib.REC_INERTIA + 9].reshape(3, 3)
        dt, mass = r[mpcqp._lib.REC_DT], r[mpcqp._lib.REC_MASS]
        Iwinv = np.linalg.inv(R @ Ib @ R.T)
        worst = np.inf
        for k in range(N):
            feet = r[F + 12 * k:F + 12 * k + 12].reshape(4, 3)
            B6 = np.zeros((6, 12))
            for l in range(4):
                x, y, z = feet[l]
                sk = np.array([[0.0, -z, y], [z, 0.0, -x], [-y, x, 0.0]])
                B6[0:3, 3 * l:3 * l + 3] = Iwinv @ sk * dt
                B6[3:6, 3 * l:3 * l + 3] = np.eye(3) * (dt / mass)
            G = B6 @ B6.T
            L = np.zeros((6, 6))
            for c in range(6):
                s = G[c, c] - L[c, :c] @ L[c, :c]
                # (the kernel's test !(s > tol G_cc) flags a zero diagonal: ratio 0 here)
                worst = min(worst, s / G[c, c] if G[c, c] > 0 else 0.0)
                d = np.sqrt(max(s, 0.0))
                L[c, c] = d
                for r2 in range(c + 1, 6):
                    L[r2, c] = (G[r2, c] - L[r2, :c] @ L[c, :c]) / d if d > 0 else 0.0
        out[b] = worst
    return out
