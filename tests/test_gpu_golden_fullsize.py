"""GPU path vs committed golden vectors, and size-independent properties at the BASELINE sizes
(C2: 4096 trot, C5: 8192 mixed gait + random mu, C3 shard: 8192 per GPU)."""
import glob
import os

import numpy as np
import pytest

import mpcqp
from gpu_helpers import rel_err_u0, sentinel, solve_gpu

pytestmark = pytest.mark.gpu
GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
# balance.npz is the balance controller's set (tests/test_balance.py, tests/test_gpu_balance.py)
SETS = sorted(p for p in glob.glob(os.path.join(GOLDEN, "*.npz")) if not p.endswith("balance.npz"))
# regression sentinels at the achieved accuracy per set (default 1e-8; the SURVEY gate stays 1e-4)
SENT = {"edge.npz": 1e-6, "gazebo_weights.npz": 1e-6}


@pytest.mark.parametrize("path", SETS, ids=[os.path.basename(p) for p in SETS])
def test_gpu_matches_golden(path):
    d = np.load(path)
    N = int(d["horizon"]) if "horizon" in d else 10
    interval = int(d["adaptive_rho_interval"]) if "adaptive_rho_interval" in d else 25
    p = mpcqp.default_params(N, q_weights=d["q_weights"], r_weights=d["r_weights"], adaptive_rho_interval=interval)
    with mpcqp.MpcQpSolver(p) as s:
        got, sol, _ = solve_gpu(s, d["records"])
    err = rel_err_u0(got["u0"], d["u0"])
    assert np.all(err <= 1e-4)
    np.testing.assert_array_equal(got["status"], d["status"])
    np.testing.assert_array_equal(got["iters"], d["iters"])
    np.testing.assert_array_equal(got["rho_updates"], d["rho_updates"])
    sentinel(err, SENT.get(os.path.basename(path), 1e-8), f"golden {os.path.basename(path)}")
    full = np.max(np.abs(sol - d["x"]), axis=1) / np.maximum(np.max(np.abs(d["x"]), axis=1), 1.0)
    assert np.all(full <= 1e-4)


def _pyramid_violation(recs, sol, N=10):
    """max over rows of dist(Ax, [l, u]) per robot (friction pyramid + fz bounds)."""
    B = recs.shape[0]
    mu = recs[:, mpcqp._lib.REC_MU][:, None]
    c = np.tile(recs[:, mpcqp._lib.REC_CONTACTS:mpcqp._lib.REC_CONTACTS + 4] != 0, (1, N))
    x = sol.reshape(B, -1, 3)
    fx, fy, fz = x[..., 0], x[..., 1], x[..., 2]
    v = np.stack([-(fx + mu * fz), fx - mu * fz, -(fy + mu * fz), fy - mu * fz, -fz, fz - 180 * c])
    return np.max(np.maximum(v, 0.0), axis=(0, 2))


@pytest.mark.parametrize("B,gait,mixed_mu,seed", [(4096, "trot", False, 1000), (8192, "mixed", True, 4000),
                                                  (8192, "trot", False, 2000)])
def test_fullsize_properties(oracle, B, gait, mixed_mu, seed):
    st = mpcqp.synthetic_go1(B, seed=seed, gait=gait, mixed_mu=mixed_mu)
    recs = mpcqp.assemble_compute_grf(st, 10)
    with mpcqp.MpcQpSolver(mpcqp.default_params(10)) as s:
        got, sol, _ = solve_gpu(s, recs)
        got2, sol2, _ = solve_gpu(s, recs)
    # idempotence / determinism: identical bits on a re-run
    np.testing.assert_array_equal(sol, sol2)
    np.testing.assert_array_equal(got["iters"], got2["iters"])
    # every robot solved; friction pyramid / fz bounds hold up to the robot's own primal residual
    # (z is projected onto [l, u], so dist(Ax, [l, u]) <= ||Ax - z||_inf = pri_res < eps_prim)
    assert np.all(got["status"] == mpcqp._lib.STATUS_SOLVED)
    assert np.all(_pyramid_violation(recs, sol) <= got["pri_res"] + 1e-9)
    # swing legs carry no force at step 0 (|f| <= (1 + mu) pri_res)
    swing = recs[:, mpcqp._lib.REC_CONTACTS:mpcqp._lib.REC_CONTACTS + 4] == 0
    bound = ((1 + recs[:, mpcqp._lib.REC_MU]) * got["pri_res"] + 1e-9)[:, None, None]
    assert np.all((np.abs(got["u0"].reshape(B, 4, 3)) <= bound)[swing])
    # f_body = R^T u0 per leg
    R = recs[:, mpcqp._lib.REC_ROT:mpcqp._lib.REC_ROT + 9].reshape(B, 3, 3)
    fb = np.einsum("bji,blj->bli", R, got["u0"].reshape(B, 4, 3)).reshape(B, 12)
    np.testing.assert_allclose(got["f_body"], fb, rtol=0, atol=1e-9)
    # a random subset against the oracle (schedule-identical parity)
    idx = np.random.default_rng(seed).choice(B, 96, replace=False)
    ref = oracle.solve_batch(oracle.default_params(10), recs[idx], nthreads=8)
    err = rel_err_u0(got["u0"][idx], ref["u0"])
    assert np.all(err <= 1e-4)
    np.testing.assert_array_equal(got["iters"][idx], ref["iters"])
    sentinel(err, 1e-8, f"fullsize {B} {gait}")


def test_batch_order_independence():
    """Results do not depend on batch composition / workgroup placement."""
    st = mpcqp.synthetic_go1(512, seed=8, gait="mixed", mixed_mu=True)
    recs = mpcqp.assemble_compute_grf(st, 10)
    perm = np.random.default_rng(0).permutation(512)
    with mpcqp.MpcQpSolver(mpcqp.default_params(10)) as s:
        a, sa, _ = solve_gpu(s, recs)
        b, sb, _ = solve_gpu(s, recs[perm])
        c, sc, _ = solve_gpu(s, recs[:1])
    np.testing.assert_array_equal(sa[perm], sb)
    np.testing.assert_array_equal(sa[:1], sc)


def test_c4_fullsize_properties(oracle):
    """Config C4 at its full size: 4096 trot robots at horizon 20 (n = 240, m = 400).  Every robot
    solved, deterministic on a re-run, friction pyramid within the robot's primal residual, and a
    96-robot subset schedule-identical with the oracle."""
    B, N = 4096, 20
    st = mpcqp.synthetic_go1(B, seed=3000, gait="trot")
    recs = mpcqp.assemble_compute_grf(st, N)
    with mpcqp.MpcQpSolver(mpcqp.default_params(N)) as s:
        got, sol, _ = solve_gpu(s, recs)
        got2, sol2, _ = solve_gpu(s, recs)
    np.testing.assert_array_equal(sol, sol2)
    np.testing.assert_array_equal(got["iters"], got2["iters"])
    assert np.all(got["status"] == mpcqp._lib.STATUS_SOLVED)
    assert np.all(_pyramid_violation(recs, sol, N) <= got["pri_res"] + 1e-9)
    idx = np.random.default_rng(3).choice(B, 96, replace=False)
    ref = oracle.solve_batch(oracle.default_params(N), recs[idx], nthreads=8)
    err = rel_err_u0(got["u0"][idx], ref["u0"])
    assert np.all(err <= 1e-4)
    sentinel(err, 1e-8, "C4 fullsize sample")
    np.testing.assert_array_equal(got["status"][idx], ref["status"])
    frac = np.mean(got["iters"][idx] == ref["iters"])
    print(f"full-size sample: iteration-equal fraction {frac:.4f}")
    assert frac >= 0.99


@pytest.mark.parametrize("gait", ["trot", "mixed"])
def test_interval100_schedule_on_gpu(oracle, gait):
    """OSQP 0.6's adaptive-rho interval without profiling (4 x check_termination = 100) on the
    device vs the oracle at the same interval, on a fresh 256-robot batch."""
    st = mpcqp.synthetic_go1(256, seed=4100, gait=gait, mixed_mu=(gait == "mixed"))
    recs = mpcqp.assemble_compute_grf(st, 10)
    p = mpcqp.default_params(10, adaptive_rho_interval=100)
    with mpcqp.MpcQpSolver(p) as s:
        got, _, _ = solve_gpu(s, recs)
    ref = oracle.solve_batch(oracle.default_params(10, adaptive_rho_interval=100), recs, nthreads=8)
    assert np.all(rel_err_u0(got["u0"], ref["u0"]) <= 1e-4)
    np.testing.assert_array_equal(got["status"], ref["status"])
    np.testing.assert_array_equal(got["iters"], ref["iters"])
    np.testing.assert_array_equal(got["rho_updates"], ref["rho_updates"])
