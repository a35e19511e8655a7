"""CPU oracle (oracle/mpc_oracle.c) pinned against the committed golden vectors, an independent
numpy restatement of ConvexMpc, and an independent interior-point QP solve (no GPU needed)."""
import glob
import os

import numpy as np
import pytest

import mpcqp
import numpy_reference as nr

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
# balance.npz is the balance controller's set (tests/test_balance.py, tests/test_gpu_balance.py)
SETS = sorted(p for p in glob.glob(os.path.join(GOLDEN, "*.npz")) if not p.endswith("balance.npz"))


def _meta(d):
    """(horizon, adaptive-rho interval) of a golden set (sets from before round 3: 10, 25)."""
    return (int(d["horizon"]) if "horizon" in d else 10,
            int(d["adaptive_rho_interval"]) if "adaptive_rho_interval" in d else 25)


def test_golden_sets_present():
    names = {os.path.basename(p)[:-4] for p in SETS}
    assert {"test_mpc", "go1_trot", "go1_mixed", "edge", "gazebo_weights", "test_mpc_n20", "go1_trot_n20",
            "go1_mixed_n20", "go1_trot_interval100", "go1_mixed_interval100"} <= names


@pytest.mark.parametrize("path", SETS, ids=[os.path.basename(p) for p in SETS])
def test_oracle_reproduces_golden(oracle, path):
    d = np.load(path)
    N, interval = _meta(d)
    p = oracle.default_params(N, q=list(d["q_weights"]), r=list(d["r_weights"]), adaptive_rho_interval=interval)
    res, sol = oracle.solve_batch(p, d["records"], nthreads=4, want_solution=True)
    np.testing.assert_array_equal(res["status"], d["status"])
    np.testing.assert_array_equal(res["iters"], d["iters"])
    np.testing.assert_array_equal(res["rho_updates"], d["rho_updates"])
    np.testing.assert_allclose(sol, d["x"], rtol=0, atol=1e-9 * max(1.0, np.abs(d["x"]).max()))
    np.testing.assert_allclose(res["f_body"], d["f_body"], rtol=0, atol=1e-9 * 180)


@pytest.mark.parametrize("path", SETS, ids=[os.path.basename(p) for p in SETS])
def test_formulation_matches_independent_restatement(oracle, path):
    d = np.load(path)
    N, _ = _meta(d)
    p = oracle.default_params(N, q=list(d["q_weights"]), r=list(d["r_weights"]))
    for b in range(min(4, d["records"].shape[0])):
        P, g, l, u, A = oracle.build_qp(p, d["records"][b])
        H2, g2, C2, l2, u2 = nr.condensed_qp(d["records"][b], N, d["q_weights"], d["r_weights"])
        assert np.max(np.abs(P - H2)) <= 1e-13 * np.max(np.abs(H2))
        assert np.max(np.abs(g - g2)) <= 1e-13 * max(np.max(np.abs(g2)), 1e-300) + 1e-300
        np.testing.assert_array_equal(A, C2)
        np.testing.assert_array_equal(l, l2)
        np.testing.assert_array_equal(u, u2)
        assert abs(P.sum() - d["hessian_sum"][b]) <= 1e-12 * np.abs(P).sum()


def test_converged_matches_interior_point(oracle):
    """P2 pin: OSQP restatement at eps 1e-9 vs an independent primal-dual IPM (objective)."""
    d = np.load(os.path.join(GOLDEN, "go1_mixed.npz"))
    for b in range(6):
        H, g, C, l, u = nr.condensed_qp(d["records"][b], 10, d["q_weights"], d["r_weights"])
        xi = nr.ipm_qp(H, g, C, l, u)
        xa = d["x_converged"][b]
        f = lambda x: 0.5 * x @ H @ x + g @ x  # noqa: E731
        fs = np.abs(g) @ np.abs(xi) + 0.5 * np.abs(xi) @ np.abs(H) @ np.abs(xi)
        assert abs(f(xa) - f(xi)) <= 1e-5 * fs + 1e-8


def test_solution_respects_friction_pyramid(oracle):
    """Default-tolerance solutions stay inside the friction pyramid up to OSQP's eps."""
    d = np.load(os.path.join(GOLDEN, "go1_mixed.npz"))
    for b in range(d["records"].shape[0]):
        rec = d["records"][b]
        mu = rec[mpcqp._lib.REC_MU]
        x = d["x"][b].reshape(-1, 3)
        c = np.tile(rec[mpcqp._lib.REC_CONTACTS:mpcqp._lib.REC_CONTACTS + 4] != 0, 10)
        tol = 0.25  # OSQP primal tolerance: eps_abs + eps_rel * max|Ax| = 1e-3 + 1e-3 * ~180 N
        assert np.all(np.abs(x[:, 0]) <= mu * x[:, 2] + tol)
        assert np.all(np.abs(x[:, 1]) <= mu * x[:, 2] + tol)
        assert np.all(x[:, 2] >= -tol) and np.all(x[:, 2] <= 180 * c + tol)


def test_warm_mu_change_uses_new_cone(oracle):
    """The persistent solver re-initializes when a robot's mu changes: the warm-started solve of a
    later tick obeys the new, tighter friction cone (with mu latched it would keep the old one)."""
    T, B, N = 6, 32, 10
    ticks = mpcqp.records.synthetic_go1_ticks(B, T, seed=17, gait="stance")
    recs = np.stack([mpcqp.assemble_compute_grf(s, N) for s in ticks])
    p = oracle.default_params(N)
    ratios = {}
    for mu_late in (0.9, 0.3):
        recs[:, :, mpcqp._lib.REC_MU] = 0.9
        recs[3:, :, mpcqp._lib.REC_MU] = mu_late
        res = oracle.solve_sequence(p, recs, nthreads=4)
        assert np.all(res["status"] == 1)
        u = res[4]["u0"].reshape(-1, 4, 3)
        big = u[:, :, 2] > 10.0
        ratios[mu_late] = (np.abs(u[:, :, :2]).max(-1)[big] / u[:, :, 2][big]).max()
    assert ratios[0.9] > 0.8  # the cone binds for these states, so the test can see mu
    assert ratios[0.3] <= 0.3 * (1 + 1e-2)


def test_all_swing_gives_zero_forces():
    d = np.load(os.path.join(GOLDEN, "edge.npz"))
    assert np.all(np.abs(d["u0"][0]) <= 1e-6)


def test_nan_record_is_flagged(oracle):
    rec, q, r = mpcqp.assemble_test_mpc(10)
    rec = rec.copy()
    rec[3] = np.inf
    res, sol = oracle.solve(oracle.default_params(10, q=list(q), r=list(r)), rec)
    assert res["status"] == mpcqp._lib.STATUS_NAN_INPUT and res["nan_legs"] == 0xF
    assert np.all(np.isnan(sol))


def test_max_iter_status(oracle):
    """max_iter below convergence -> OSQP_MAX_ITER_REACHED (or SOLVED_INACCURATE)."""
    rec, q, r = mpcqp.assemble_test_mpc(10)
    res, _ = oracle.solve(oracle.default_params(10, q=list(q), r=list(r), max_iter=10), rec)
    assert res["status"] in (mpcqp._lib.STATUS_MAX_ITER_REACHED, mpcqp._lib.STATUS_SOLVED_INACCURATE)
    assert res["iters"] == 10


def test_test_mpc_forces_physical(oracle):
    """test_mpc.cpp stance: FL and RL in contact carry the load, swing legs carry nothing."""
    d = np.load(os.path.join(GOLDEN, "test_mpc.npz"))
    f = d["u0"][0].reshape(4, 3)
    assert f[0, 2] > 10 and f[2, 2] > 10
    assert np.all(np.abs(f[[1, 3]]) < 1e-3)
    assert d["status"][0] == 1


def test_interval100_changes_the_schedule():
    """The interval-100 sets (OSQP 0.6 without profiling) are not the interval-25 schedule: the
    same records give different iteration counts for most robots."""
    a = np.load(os.path.join(GOLDEN, "go1_trot.npz"))
    b = np.load(os.path.join(GOLDEN, "go1_trot_interval100.npz"))
    np.testing.assert_array_equal(a["records"], b["records"])
    assert np.mean(a["iters"] != b["iters"]) > 0.5
    assert np.all(b["status"] == 1)
