"""Host-side logic and the C-ABI library, without a GPU: record assembly (the compute_grf input
mirror) vs the oracle's C restatement, reference default settings, and that libmpcqp.so loads and
exports every symbol declared in include/*.h."""
import ctypes
import os
import re
import subprocess

import numpy as np
import pytest

import mpcqp
from mpcqp import _lib

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _to_oracle_state(oracle, st, b):
    s = oracle.RobotState()
    for f in ["root_euler", "root_pos", "root_ang_vel", "root_lin_vel", "root_euler_d", "root_pos_d",
              "root_ang_vel_d", "root_lin_vel_d"]:
        getattr(s, f)[:] = [float(v) for v in getattr(st, f)[b]]
    s.root_rot_mat[:] = [float(v) for v in st.root_rot_mat[b].reshape(9)]
    s.foot_pos_abs[:] = [float(v) for v in st.foot_pos_abs[b].reshape(12)]
    s.robot_mass = 13.0 if st.robot_mass is None else float(st.robot_mass[b])
    s.trunk_inertia[:] = [float(v) for v in mpcqp.records.GO1_INERTIA.reshape(9)]
    s.mu = float(st.mu[b])
    s.fz_min, s.fz_max, s.mpc_dt = st.fz_min, st.fz_max, st.mpc_dt
    s.contacts[:] = [int(c) for c in st.contacts[b]]
    return s


@pytest.mark.parametrize("gait", ["trot", "mixed", "stance"])
def test_compute_grf_assembly_matches_oracle(oracle, gait):
    st = mpcqp.synthetic_go1(16, seed=3, gait=gait, mixed_mu=gait == "mixed")
    for N in (10, 4):
        recs = mpcqp.assemble_compute_grf(st, N)
        for b in range(16):
            ref = oracle.assemble_compute_grf(_to_oracle_state(oracle, st, b), N)
            np.testing.assert_array_equal(recs[b], ref)


def test_test_mpc_assembly_matches_oracle(oracle):
    rec, q, r = mpcqp.assemble_test_mpc(10)
    rec2, q2, r2 = oracle.assemble_test_mpc(10)
    np.testing.assert_array_equal(rec, rec2)
    np.testing.assert_array_equal(q, q2)
    np.testing.assert_array_equal(r, r2)


def test_record_layout():
    L = _lib.load()
    for N in range(1, 21):
        assert L.mpcqp_record_size(N) == _lib.rec_size(N) == 44 + 25 * N + (N & 1)
    assert L.mpcqp_record_size(0) == 0
    assert L.mpcqp_solve_threads(21) == 0 and L.mpcqp_solve_threads(20) > 0


def test_default_params_are_reference_settings():
    p = mpcqp.default_params(10)
    # OSQP 0.6 osqp_set_default_settings (reference sets only verbose/warm_start)
    assert (p.max_iter, p.scaling, p.check_termination, p.adaptive_rho) == (4000, 10, 25, 1)
    assert (p.rho, p.sigma, p.alpha) == (0.1, 1e-6, 1.6)
    assert (p.eps_abs, p.eps_rel, p.eps_prim_inf, p.eps_dual_inf) == (1e-3, 1e-3, 1e-4, 1e-4)
    assert p.adaptive_rho_tolerance == 5.0 and p.scaled_termination == 0 and p.warm_start == 0
    assert p.adaptive_rho_interval == 25  # frozen (OSQP's 0 = wall-clock derived)
    # Go1CtrlStates.hpp:203-249
    assert list(p.q_weights) == [80.0, 80.0, 1.0, 0.0, 0.0, 270.0, 1.0, 1.0, 20.0, 20.0, 20.0, 20.0, 0.0]
    assert list(p.r_weights) == [1e-5, 1e-5, 1e-6] * 4


def _declared_functions():
    names = set()
    for h in ("mpcqp.h", "mpcqp_debug.h"):
        src = open(os.path.join(REPO, "include", h)).read()
        src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
        for m in re.finditer(r"^\s*(?:const\s+)?\w[\w\s\*]*?\b(mpcqp_\w+)\s*\(", src, flags=re.M):
            names.add(m.group(1))
    return names


def test_library_exports_every_declared_symbol():
    L = _lib.load()
    declared = _declared_functions()
    assert len(declared) >= 14
    assert declared == set(_lib.EXPORTED)
    for name in declared:
        assert hasattr(L, name), name
    out = subprocess.run(["nm", "-D", "--defined-only", _lib.LIB_PATH], capture_output=True, text=True).stdout
    exported = {line.split()[-1] for line in out.splitlines() if " T " in line}
    assert declared <= exported


def test_abi_struct_sizes():
    L = _lib.load()
    ps, rs = ctypes.c_int32(), ctypes.c_int32()
    L.mpcqp_abi_sizes(ctypes.byref(ps), ctypes.byref(rs))
    assert ps.value == ctypes.sizeof(_lib.Params) == 296
    assert rs.value == ctypes.sizeof(_lib.Result) == _lib.RESULT_DTYPE.itemsize == 240


def test_invalid_params_rejected_before_device():
    L = _lib.load()
    h = ctypes.c_void_p()
    for bad in (dict(horizon=0), dict(horizon=21), dict(adaptive_rho_interval=0), dict(alpha=2.5),
                dict(rho=-1.0), dict(scaled_termination=1)):
        p = mpcqp.default_params(10)
        for k, v in bad.items():
            setattr(p, k, v)
        assert L.mpcqp_create(ctypes.byref(p), 0, ctypes.byref(h)) == _lib.ERR_INVALID_ARG, bad
    assert L.mpcqp_create(None, 0, ctypes.byref(h)) == _lib.ERR_INVALID_ARG


def test_status_and_error_strings():
    assert mpcqp.status_str(1) == "solved"
    assert mpcqp.status_str(-2) == "maximum iterations reached"
    assert mpcqp.status_str(-100) == "non-finite input"
    assert _lib.load().mpcqp_error_str(2) == b"HIP runtime error"


def test_no_device_is_reported_not_crashed():
    from conftest import has_gpu
    if has_gpu():
        pytest.skip("GPU present")
    with pytest.raises(_lib.MpcQpError, match="no HIP device|HIP"):
        mpcqp.MpcQpSolver(mpcqp.default_params(10))


def test_synthetic_generator_is_seeded_and_in_range():
    a = mpcqp.synthetic_go1(256, seed=9, gait="mixed", mixed_mu=True)
    b = mpcqp.synthetic_go1(256, seed=9, gait="mixed", mixed_mu=True)
    np.testing.assert_array_equal(mpcqp.assemble_compute_grf(a, 10), mpcqp.assemble_compute_grf(b, 10))
    assert np.all(np.abs(a.root_euler[:, :2]) <= 0.2) and np.all(np.abs(a.root_euler[:, 2]) <= np.pi)
    assert np.all((a.mu >= 0.3) & (a.mu <= 0.9))
    R = a.root_rot_mat
    np.testing.assert_allclose(np.einsum("bij,bkj->bik", R, R), np.broadcast_to(np.eye(3), R.shape), atol=1e-12)
    t = mpcqp.synthetic_go1(4, seed=0, gait="trot")
    assert t.contacts.tolist() == [[True, False, False, True], [False, True, True, False]] * 2


def test_product_library_ships_only_the_default_solve():
    """libmpcqp.so holds the wave path's kernels and none of the cross-check solvers (those are
    in libmpcqp_debug.so, which exports the same ABI)."""
    def kernels(path):
        out = subprocess.run(["nm", "-C", "--defined-only", path], capture_output=True, text=True).stdout
        return out
    prod = kernels(_lib.LIB_PATH)
    dbg = kernels(_lib.DEBUG_LIB_PATH)
    # horizon 10: the Schur-form solve (KS = 1) and the Riccati form (KS = 0, negative weights);
    # horizon 20: Riccati only
    for k in ("mpcqp::wv::wave_kernel<10, 1>", "mpcqp::wv::wave_kernel<10, 0>", "mpcqp::wv::wave_kernel<20, 0>",
              "mpcqp::wv::scale_kernel<10>", "mpcqp::wv::scale_kernel<20>"):
        assert k in prod, k
    assert "mpcqp::wv::wave_kernel<20, 1>" not in prod
    for name in ("mpcqp::solve_kernel<", "mpcqp::ric::ric_solve_kernel<", "mw_kernel", "dx_kernel"):
        assert name not in prod, name
    assert "mpcqp::solve_kernel<10>" in dbg and "mpcqp::ric::ric_solve_kernel<10>" in dbg
    out = subprocess.run(["nm", "-D", "--defined-only", _lib.DEBUG_LIB_PATH], capture_output=True, text=True).stdout
    exported = {line.split()[-1] for line in out.splitlines() if " T " in line}
    assert _declared_functions() <= exported


def test_bench_traffic_matches_the_launched_kernels(tmp_path, monkeypatch):
    """bench.py's roofline.traffic comes from a PMC pass of exactly the kernels it times: the
    Schur-form launch (wave_kernel<10, 1>) matches the committed pass, another instantiation or
    configuration reports null rather than a stale number."""
    import importlib.util
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(repo, "bench.py"))
    bench = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(bench)
    name = "mpcqp::wv::scale_kernel<10> + mpcqp::wv::wave_kernel<10, 1>"
    t = bench.load_traffic("N10_B4096_trot", name)
    assert t is not None and t > 0
    assert bench.load_traffic("N10_B4096_trot", name.replace("<10, 1>", "<10, 0>")) is None
    assert bench.load_traffic("N20_B4096_trot", name) is None
