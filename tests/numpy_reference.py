"""TEST INFRASTRUCTURE — an independent numpy restatement of ConvexMpc's formulation and a KKT
verifier for the QP.  Written separately from oracle/mpc_oracle.c so the two cross-check each
other (the reference itself cannot be compiled here: Eigen/OSQP/ROS absent).

Formulation: src/a1_cpp/src/ConvexMpc.cpp:7-245 (A_c :110-130, B_c :132-143, Euler
discretization :145-156, A_qp/B_qp :184-202, H :207-211, gradient :215-217, bounds :223-245).
"""
import numpy as np

REC_X0, REC_EULER, REC_ROT, REC_INERTIA = 0, 13, 16, 25
REC_MASS, REC_MU, REC_FZMIN, REC_FZMAX, REC_DT, REC_CONTACTS, REC_XREF = 34, 35, 36, 37, 38, 39, 44
INF = 1e30


def skew(v):
    return np.array([[0, -v[2], v[1]], [v[2], 0, -v[0]], [-v[1], v[0], 0]])


def condensed_qp(rec, N, q_w, r_w):
    dt = rec[REC_DT]
    yaw = rec[REC_EULER + 2]
    Ac = np.zeros((13, 13))
    Ac[0:3, 6:9] = [[np.cos(yaw), np.sin(yaw), 0], [-np.sin(yaw), np.cos(yaw), 0], [0, 0, 1]]
    Ac[3:6, 9:12] = np.eye(3)
    Ac[11, 12] = 1.0
    Ad = np.eye(13) + Ac * dt
    R = rec[REC_ROT:REC_ROT + 9].reshape(3, 3)
    Ib = rec[REC_INERTIA:REC_INERTIA + 9].reshape(3, 3)
    Iw_inv = np.linalg.inv(R @ Ib @ R.T)
    mass = rec[REC_MASS]
    feet = rec[REC_XREF + 13 * N: REC_XREF + 25 * N].reshape(N, 4, 3)
    Bd = []
    for i in range(N):
        Bc = np.zeros((13, 12))
        for leg in range(4):
            Bc[6:9, 3 * leg:3 * leg + 3] = Iw_inv @ skew(feet[i, leg])
            Bc[9:12, 3 * leg:3 * leg + 3] = np.eye(3) / mass
        Bd.append(Bc * dt)
    Aqp = np.zeros((13 * N, 13))
    Bqp = np.zeros((13 * N, 12 * N))
    P = np.eye(13)
    for i in range(N):
        P = P @ Ad
        Aqp[13 * i:13 * i + 13] = P
        for j in range(i + 1):
            Bqp[13 * i:13 * i + 13, 12 * j:12 * j + 12] = np.linalg.matrix_power(Ad, i - j) @ Bd[j]
    Q = np.diag(2 * np.tile(q_w, N))
    Rm = np.diag(2 * np.tile(r_w, N))
    H = Bqp.T @ Q @ Bqp + Rm
    x0 = rec[REC_X0:REC_X0 + 13]
    xref = rec[REC_XREF:REC_XREF + 13 * N]
    g = Bqp.T @ Q @ (Aqp @ x0 - xref)
    mu = rec[REC_MU]
    C = np.zeros((20 * N, 12 * N))
    blk = np.array([[1, 0, mu], [1, 0, -mu], [0, 1, mu], [0, 1, -mu], [0, 0, 1]])
    lo, hi = [], []
    for f in range(4 * N):
        C[5 * f:5 * f + 5, 3 * f:3 * f + 3] = blk
        c = 1.0 if rec[REC_CONTACTS + f % 4] != 0 else 0.0
        lo += [0, -INF, 0, -INF, rec[REC_FZMIN] * c]
        hi += [INF, 0, INF, 0, rec[REC_FZMAX] * c]
    return H, g, C, np.array(lo), np.array(hi)


def kkt_residuals(H, g, C, lo, hi, x, tol_active=1e-6):
    """Return (stationarity, primal violation) for x using a nonnegative-LS multiplier fit."""
    from scipy.optimize import lsq_linear
    Cx = C @ x
    prim = max(0.0, float(np.max(np.maximum(lo - Cx, Cx - hi))))
    # multipliers y with sign constraints: y_i >= 0 at upper-active, <= 0 at lower-active, 0 else
    act_lo = (Cx - lo) <= tol_active * np.maximum(1.0, np.abs(lo))
    act_hi = (hi - Cx) <= tol_active * np.maximum(1.0, np.abs(hi))
    lb = np.where(act_lo & ~act_hi, -np.inf, 0.0)
    ub = np.where(act_hi & ~act_lo, np.inf, 0.0)
    both = act_lo & act_hi
    lb[both], ub[both] = -np.inf, np.inf
    fr = (lb != 0) | (ub != 0)
    r = -(H @ x + g)
    if fr.any():
        sol = lsq_linear(C[fr].T, r, bounds=(lb[fr], ub[fr]))
        stat = float(np.max(np.abs(C[fr].T @ sol.x - r)))
    else:
        stat = float(np.max(np.abs(r)))
    return stat, prim


def ipm_qp(H, g, C, lo, hi, tol=1e-10, max_iter=200):
    """Independent dense primal-dual interior-point solver (Mehrotra predictor-corrector) for
        min 1/2 x'Hx + g'x  s.t.  lo <= Cx <= hi
    Rows with lo == hi become equalities; +-1e30 bounds are dropped.  Returns x."""
    n = H.shape[0]
    eq = np.isclose(lo, hi, rtol=0, atol=0)
    Ae, be = C[eq], lo[eq]
    up = (~eq) & (hi < INF / 10)
    dn = (~eq) & (lo > -INF / 10)
    G = np.vstack([C[up], -C[dn]])
    h = np.concatenate([hi[up], -lo[dn]])
    p, me = G.shape[0], Ae.shape[0]
    x = np.zeros(n)
    s = np.maximum(h - G @ x, 1.0)
    z = np.ones(p)
    yv = np.zeros(me)
    for _ in range(max_iter):
        rd = H @ x + g + G.T @ z + Ae.T @ yv
        rp = G @ x + s - h
        re = Ae @ x - be
        mu = s @ z / p
        # scale-aware stop: iterating past this point only accumulates roundoff (W = z/s spans
        # ~1e20 at the end and the reduced KKT solve loses accuracy)
        dscale = 1.0 + np.max(np.abs(g)) + np.max(np.abs(H)) * np.max(np.abs(x))
        pscale = 1.0 + np.max(np.abs(h)) + np.max(np.abs(G)) * np.max(np.abs(x))
        if (np.max(np.abs(rd)) < tol * dscale and np.max(np.abs(rp)) < tol * pscale
                and (not me or np.max(np.abs(re)) < tol * pscale) and mu < tol * dscale):
            break

        def solve(rc):
            # Newton on H dx + G'dz + Ae'dy = -rd, G dx + ds = -rp, Ae dx = -re, Z ds + S dz = -rc.
            # Eliminating ds, dz: (H + G'WG) dx + Ae'dy = -rd - G'((z rp - rc)/s),  W = Z/S
            W = z / s
            K = np.block([[H + G.T @ (W[:, None] * G), Ae.T], [Ae, np.zeros((me, me))]])
            rhs = np.concatenate([-rd - G.T @ ((z * rp - rc) / s), -re])
            sol = np.linalg.solve(K, rhs)
            dx, dy = sol[:n], sol[n:]
            ds = -rp - G @ dx
            dz = -(rc + z * ds) / s
            return dx, dy, ds, dz

        def step_len(v, dv):
            neg = dv < 0
            return min(1.0, float(np.min(-v[neg] / dv[neg]))) if neg.any() else 1.0

        dx, dy, ds, dz = solve(s * z)           # affine: rc = s*z  (target s*z -> 0)
        a = min(step_len(s, ds), step_len(z, dz))
        mu_aff = (s + a * ds) @ (z + a * dz) / p
        sigma = (mu_aff / mu) ** 3
        dx, dy, ds, dz = solve(s * z + ds * dz - sigma * mu)
        a = 0.99 * min(step_len(s, ds), step_len(z, dz))
        x, yv, s, z = x + a * dx, yv + a * dy, s + a * ds, z + a * dz
    return x


def balance_qp(rec, q_diag, r, mu, f_min, f_max):
    """Independent numpy restatement of the single-step QP balance controller
    (A1RobotControl.cpp:321-332, :377-414; constraint rows of the ctor :27-44).
    rec is one MPCQP_BAL record (include/mpcqp.h). Returns H, g, C, lo, hi."""
    R = rec[6:15].reshape(3, 3)
    Rz = rec[15:24].reshape(3, 3)
    ee = rec[39:42] - rec[36:39]
    if ee[2] > 3.1415926 * 1.5:
        ee[2] = rec[41] - 3.1415926 * 2 - rec[38]
    elif ee[2] < -3.1415926 * 1.5:
        ee[2] = rec[41] + 3.1415926 * 2 - rec[38]
    acc = np.zeros(6)
    acc[:3] = rec[42:45] * (rec[3:6] - rec[0:3]) + R @ (rec[45:48] * (rec[27:30] - R.T @ rec[24:27]))
    acc[3:] = rec[48:51] * ee + rec[51:54] * (rec[33:36] - R.T @ rec[30:33])
    acc[2] += rec[54] * 9.8
    M = np.zeros((6, 12))
    for i in range(4):
        M[:3, 3 * i:3 * i + 3] = np.eye(3)
        M[3:, 3 * i:3 * i + 3] = Rz.T @ skew(rec[55 + 3 * i:58 + 3 * i])
    Q = np.diag(q_diag)
    H = r * np.eye(12) + M.T @ Q @ M
    g = -M.T @ Q @ acc
    C = np.zeros((20, 12))
    lo = np.zeros(20)
    hi = np.zeros(20)
    for i in range(4):
        c = 1.0 if rec[67 + i] != 0 else 0.0
        C[i, 3 * i + 2] = 1.0
        lo[i], hi[i] = c * f_min, c * f_max
        for k, (col, sgn) in enumerate([(0, 1.0), (0, -1.0), (1, 1.0), (1, -1.0)]):
            C[4 + 4 * i + k, 3 * i + col] = sgn
            C[4 + 4 * i + k, 3 * i + 2] = -mu
            lo[4 + 4 * i + k] = -1e30
    return H, g, C, lo, hi
