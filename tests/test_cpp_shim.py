"""The C++ drop-in shim (include/mpcqp_robot_control.hpp) running the reference's own harness
(test_mpc.cpp, ported in tests/cpp/test_mpc_gpu.cpp) on the GPU, checked against the oracle."""
import os
import subprocess

import numpy as np
import pytest

import mpcqp

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EXE = os.path.join(REPO, "tests", "cpp", "build", "test_mpc_gpu")


@pytest.mark.gpu
def test_cpp_test_mpc_harness(oracle):
    if not os.path.exists(EXE):
        subprocess.run(["make", "-C", os.path.join(REPO, "tests", "cpp")], check=True)
    out = subprocess.run([EXE], check=True, capture_output=True, text=True, timeout=120).stdout
    kv = {}
    rows, grf, grf_sim = [], [], []
    for line in out.splitlines():
        parts = line.split()
        if parts[0] in ("RECOVERED_FEET", "RECORD", "A_MAT_D", "LIN_CON"):
            kv[parts[0]] = np.array([float(x) for x in parts[1:]])
        elif parts[0] in ("A_QP", "B_QP"):
            kv[parts[0]] = np.array([float(x) for x in parts[3:]]).reshape(int(parts[1]), int(parts[2]))
        elif parts[0].startswith("LAZY_"):
            kv[parts[0]] = [int(x) for x in parts[1:]]
        elif parts[0] == "STAGING_DEVICE":
            kv["staging_device"], kv["handle_device"] = int(parts[1]), int(parts[3])
        elif parts[0] == "ROW":
            rows.append([float(x) for x in parts[1:]])
        elif parts[0] == "GRF":
            grf.append([float(x) for x in parts[1:]])
        elif parts[0] == "GRFSIM":
            grf_sim.append([float(x) for x in parts[1:]])
        elif parts[0] == "STATUS":
            kv["status"], kv["iters"], kv["rho_updates"] = int(parts[1]), int(parts[3]), int(parts[5])
        else:
            kv[parts[0]] = float(parts[1])
    rec, q, r = mpcqp.assemble_test_mpc(10)
    op = oracle.default_params(10, q=list(q), r=list(r))
    P, g, l, u, A = oracle.build_qp(op, rec)
    assert abs(kv["HESSIAN_SUM"] - P.sum()) <= 1e-12 * np.abs(P).sum()
    assert abs(kv["HESSIAN_MAX"] - P.max()) <= 1e-12 * np.abs(P).max()
    assert abs(kv["GRADIENT_SUM"] - g.sum()) <= 1e-12 * max(np.abs(g).sum(), 1e-300) + 1e-18
    ref, _ = oracle.solve(op, rec)
    u0 = np.array(rows).T.reshape(12)  # [leg][xyz]
    assert np.max(np.abs(u0 - ref["u0"])) <= 1e-4 * max(np.max(np.abs(ref["u0"])), 1)
    assert (kv["status"], kv["iters"], kv["rho_updates"]) == (int(ref["status"]), int(ref["iters"]), int(ref["rho_updates"]))
    # lazy members: nothing produced by calculate_qp_mats itself; one device round trip fills
    # hessian and gradient together, the host-side members stay unproduced until read
    assert kv["LAZY_BEFORE"] == [0, 0, 0, 0, 0]
    assert kv["LAZY_AFTER_H"] == [1, 1, 0, 0, 0]
    # A_qp / B_qp (ConvexMpc.cpp:184-202): A_qp block i = A_d^(i+1), B_qp lower block-triangular,
    # and the reference's H = B_qp' Q B_qp + R, g = B_qp' Q (A_qp x0 - x_ref) (:207-217) with
    # Q = diag(2 q), R = diag(2 r) (ConvexMpc.cpp:20, :42) reproduce the oracle's P and q
    Ad = kv["A_MAT_D"].reshape(13, 13)
    Aqp, Bqp = kv["A_QP"], kv["B_QP"]
    assert Aqp.shape == (130, 13) and Bqp.shape == (130, 120)
    M = np.eye(13)
    for i in range(10):
        M = M @ Ad
        np.testing.assert_allclose(Aqp[13 * i:13 * i + 13], M, rtol=0, atol=1e-12 * max(1, np.abs(M).max()))
        assert np.all(Bqp[13 * i:13 * i + 13, 12 * (i + 1):] == 0)
    Qd = np.tile(2 * np.asarray(q, dtype=np.float64), 10)
    Rd = np.tile(2 * np.asarray(r, dtype=np.float64), 10)
    H2 = Bqp.T @ (Qd[:, None] * Bqp) + np.diag(Rd)
    np.testing.assert_allclose(H2, P, rtol=0, atol=1e-10 * np.abs(P).max())
    x0 = rec[mpcqp._lib.REC_X0:mpcqp._lib.REC_X0 + 13]
    xr = rec[mpcqp._lib.REC_XREF:mpcqp._lib.REC_XREF + 130]
    g2 = Bqp.T @ (Qd * (Aqp @ x0 - xr))
    np.testing.assert_allclose(g2, g, rtol=0, atol=1e-10 * max(np.abs(g).max(), 1e-12))
    assert int(kv["LIN_CON"][0]) == A.size
    np.testing.assert_array_equal(kv["LIN_CON"][1:].reshape(A.shape), A)
    # the formulation's device staging is on the handle's device
    assert kv["staging_device"] == kv["handle_device"]
    # B_mat_d_list block 3 replaced by a B_d of feet moved +0.01 in x: read back through I_w
    feet3 = rec[mpcqp.rec_feet(10) + 36: mpcqp.rec_feet(10) + 48].reshape(4, 3).copy()
    feet3[:, 0] += 0.01
    np.testing.assert_allclose(kv["RECOVERED_FEET"].reshape(4, 3), feet3, rtol=0, atol=1e-12)
    rec_mod = kv["RECORD"]
    P2, _, _, _, _ = oracle.build_qp(op, rec_mod)
    assert abs(kv["RECOVERED_HESSIAN_SUM"] - P2.sum()) <= 1e-12 * np.abs(P2).sum()
    assert abs(P2.sum() - P.sum()) > 1e-9 * np.abs(P).sum()  # the moved feet changed H
    # compute_grf (production assembly) on the same stance
    s = oracle.RobotState()
    s.root_pos[:] = [0, 0, 0.15]
    s.root_rot_mat[:] = [1, 0, 0, 0, 1, 0, 0, 0, 1]
    s.root_pos_d[:] = [0, 0, 0.15]
    s.foot_pos_abs[:] = [0.17, 0.15, -0.35, 0.17, -0.15, -0.35, -0.17, 0.15, -0.35, -0.17, -0.15, -0.35]
    s.robot_mass = 15
    s.trunk_inertia[:] = [0.0158533, 0, 0, 0, 0.0377999, 0, 0, 0, 0.0456542]
    s.mu, s.fz_min, s.fz_max, s.mpc_dt = 0.3, 0.0, 180.0, 0.0025
    s.contacts[:] = [1, 0, 1, 0]
    rec2 = oracle.assemble_compute_grf(s, 10)
    ref2, _ = oracle.solve(op, rec2)
    f = np.array(grf)  # 3x4 body frame
    fr = np.array(ref2["f_body"]).reshape(4, 3).T
    assert np.max(np.abs(f - fr)) <= 1e-4 * max(np.max(np.abs(fr)), 1)
    # use_sim_time: the horizon step is the caller's dt (0.004), not mpc_dt
    s.mpc_dt = 0.004
    ref3, _ = oracle.solve(op, oracle.assemble_compute_grf(s, 10))
    fs = np.array(grf_sim)
    fr3 = np.array(ref3["f_body"]).reshape(4, 3).T
    assert np.max(np.abs(fs - fr3)) <= 1e-4 * max(np.max(np.abs(fr3)), 1)
    assert np.max(np.abs(fr3 - fr)) > 1e-3  # dt matters, so the check can see it


@pytest.mark.gpu
def test_cpp_balance_branch(oracle):
    """compute_grf_qp (stance_leg_control_type == 0) through the C++ shim == oracle balance solve."""
    exe = os.path.join(REPO, "tests", "cpp", "build", "test_balance_gpu")
    if not os.path.exists(exe):
        subprocess.run(["make", "-C", os.path.join(REPO, "tests", "cpp")], check=True)
    out = subprocess.run([exe], check=True, capture_output=True, text=True, timeout=120).stdout
    grf, rec, st = [], None, None
    for line in out.splitlines():
        parts = line.split()
        if parts[0] == "REC":
            rec = np.array([float(x) for x in parts[1:]])
        elif parts[0] == "GRF":
            grf.append([float(x) for x in parts[1:]])
        elif parts[0] == "STATUS":
            st = (int(parts[1]), int(parts[3]))
    ref = oracle.balance_solve_batch(oracle.default_params(1), oracle.default_balance_params(), rec[None])[0]
    assert st == (int(ref["status"]), int(ref["iters"]))
    fr = np.array(ref["f_body"]).reshape(4, 3).T
    np.testing.assert_array_equal(np.array(grf), fr)
    assert fr[2, 0] > 20 and fr[2, 3] > 20 and np.all(np.abs(fr[:, 1:3]) < 0.05)  # swing legs: 0 within OSQP eps


@pytest.mark.gpu
def test_cpp_warm_ticks_match_oracle_sequence(oracle, tmp_path):
    """24 production ticks through the C++ drop-in: per-robot controllers calling
    `foot_forces_grf = compute_grf(state, dt)` (persistent warm-started solver, A1RobotControl.h:67)
    and one batched controller, against the oracle's persistent solver tick by tick (ws_update:
    initSolver, then update_P / re-init and a warm solve): status, iterations, u0 within 1e-4."""
    exe = os.path.join(REPO, "tests", "cpp", "build", "test_warm_ticks_gpu")
    if not os.path.exists(exe):
        subprocess.run(["make", "-C", os.path.join(REPO, "tests", "cpp")], check=True)
    T, B = 24, 6
    ticks = mpcqp.records.synthetic_go1_ticks(B, T, seed=41, gait="trot", swing_ticks=5)
    rows = np.stack([mpcqp.pack_states(st) for st in ticks])  # [T][B][ST_SIZE]
    path = tmp_path / "states.bin"
    np.ascontiguousarray(rows, dtype=np.float64).tofile(path)
    out = subprocess.run([exe, str(path), str(T), str(B)], check=True, capture_output=True, text=True,
                         timeout=120).stdout
    got = {"TICK": {}, "BATCH": {}}
    grf = {}
    for line in out.splitlines():
        p = line.split()
        if p[0] in got:
            got[p[0]][(int(p[1]), int(p[2]))] = (int(p[3]), int(p[4]), int(p[5]), np.array([float(x) for x in p[6:]]))
        elif p[0] == "GRF":
            grf[(int(p[1]), int(p[2]))] = np.array([float(x) for x in p[3:]]).reshape(3, 4)
    recs_t = np.stack([mpcqp.assemble_compute_grf(st, 10) for st in ticks])
    ref = oracle.solve_sequence(oracle.default_params(10), recs_t, nthreads=4)
    warm_iters = []
    for tag in ("TICK", "BATCH"):
        assert len(got[tag]) == T * B, tag
        for t in range(T):
            for b in range(B):
                st, it, ru, u0 = got[tag][(t, b)]
                r = ref[t][b]
                assert st == int(r["status"]), (tag, t, b)
                assert it == int(r["iters"]), (tag, t, b, it, int(r["iters"]))
                err = np.max(np.abs(u0 - r["u0"])) / max(np.max(np.abs(r["u0"])), 1.0)
                assert err <= 1e-4, (tag, t, b, err)
                if tag == "TICK":
                    warm_iters.append(it if t else None)
                    fb = np.array(r["f_body"]).reshape(4, 3).T
                    assert np.max(np.abs(grf[(t, b)] - fb)) <= 1e-4 * max(np.max(np.abs(fb)), 1.0)
    cold = oracle.solve_batch(oracle.default_params(10), recs_t[1:].reshape(-1, recs_t.shape[-1]), nthreads=4)
    warm = np.array([w for w in warm_iters if w is not None])
    assert warm.mean() < 0.6 * cold["iters"].mean()  # the warm start is really in effect


@pytest.mark.gpu
def test_cpp_compute_grf_dispatches_on_stance_leg_control_type(oracle, tmp_path):
    """One compute_grf(state, dt) entry point, the branch chosen per tick by
    state.stance_leg_control_type (A1RobotControl.cpp:377 QP, :446 MPC).  Every robot switches
    between the branches mid-sequence (per-robot controllers, and one batched controller that gets
    mixed-mode batches).  QP ticks == the oracle's fresh balance solve of the printed record (bitwise);
    MPC ticks == the oracle's persistent solver run over that robot's MPC ticks only (the QP branch
    never touches the member solver, so its warm start carries across the QP ticks)."""
    exe = os.path.join(REPO, "tests", "cpp", "build", "test_mode_switch_gpu")
    if not os.path.exists(exe):
        subprocess.run(["make", "-C", os.path.join(REPO, "tests", "cpp")], check=True)
    T, B = 16, 4
    ticks = mpcqp.records.synthetic_go1_ticks(B, T, seed=43, gait="trot", swing_ticks=5)
    rows = np.stack([mpcqp.pack_states(st) for st in ticks])
    path = tmp_path / "states.bin"
    np.ascontiguousarray(rows, dtype=np.float64).tofile(path)
    out = subprocess.run([exe, str(path), str(T), str(B)], check=True, capture_output=True, text=True,
                         timeout=120).stdout
    got = {"TICK": {}, "BATCH": {}}
    grf, balrec = {}, {}
    for line in out.splitlines():
        p = line.split()
        if p[0] in got:
            got[p[0]][(int(p[1]), int(p[2]))] = (int(p[3]), int(p[4]), int(p[5]), int(p[6]),
                                                  np.array([float(x) for x in p[7:]]))
        elif p[0] == "GRF":
            grf[(int(p[1]), int(p[2]))] = np.array([float(x) for x in p[3:]]).reshape(3, 4)
        elif p[0] == "BALREC":
            balrec[(int(p[1]), int(p[2]))] = np.array([float(x) for x in p[3:]])
    assert "BADTYPE rejected" in out

    def mode(t, b):
        return 0 if (t + b) % 8 in (3, 4) else 1
    recs_t = np.stack([mpcqp.assemble_compute_grf(st, 10) for st in ticks])  # [T][B][rec]
    op = oracle.default_params(10)
    bp = oracle.default_balance_params()
    n_qp = n_mpc = 0
    for b in range(B):
        mts = [t for t in range(T) if mode(t, b) == 1]
        ref_m = oracle.solve_sequence(op, np.ascontiguousarray(recs_t[mts, b:b + 1]), nthreads=1)
        ref_of = {t: ref_m[i][0] for i, t in enumerate(mts)}
        for t in range(T):
            for tag in ("TICK", "BATCH"):
                ty, st, it, ru, u0 = got[tag][(t, b)]
                assert ty == mode(t, b)
                if ty == 1:
                    r = ref_of[t]
                    assert (st, it) == (int(r["status"]), int(r["iters"])), (tag, t, b)
                    err = np.max(np.abs(u0 - r["u0"])) / max(np.max(np.abs(r["u0"])), 1.0)
                    assert err <= 1e-4, (tag, t, b, err)
                    n_mpc += 1
                else:
                    r = oracle.balance_solve_batch(op, bp, balrec[(t, b)][None])[0]
                    assert (st, it) == (int(r["status"]), int(r["iters"])), (tag, t, b)
                    np.testing.assert_array_equal(u0, r["u0"])
                    n_qp += 1
                if tag == "TICK":
                    fb = np.array(r["f_body"]).reshape(4, 3).T
                    assert np.max(np.abs(grf[(t, b)] - fb)) <= 1e-4 * max(np.max(np.abs(fb)), 1.0)
    assert n_qp > 0 and n_mpc > 0


@pytest.mark.gpu
def test_cpp_terrain_adaptation_behind_compute_grf(oracle, tmp_path):
    """Terrain adaptation behind the same compute_grf call (A1RobotControl.cpp:334-376): with the
    shim's terrain_angle_of hook set, MPC ticks clamp the filtered angle to +-0.5 (0 when
    root_pos[2] <= 0.1, where the hook is not called), set root_euler_d[1] by the front/rear
    recent-contact height difference and terrain_pitch_angle; the adapted pitch reaches x_ref, so
    u0 matches the oracle's persistent solver on records assembled from the adapted states."""
    exe = os.path.join(REPO, "tests", "cpp", "build", "test_mode_switch_gpu")
    if not os.path.exists(exe):
        subprocess.run(["make", "-C", os.path.join(REPO, "tests", "cpp")], check=True)
    T, B = 14, 4
    ticks = mpcqp.records.synthetic_go1_ticks(B, T, seed=47, gait="trot", swing_ticks=5)
    for st in ticks:  # (the generator shares some arrays between ticks; each tick gets its own here)
        st.root_euler_d = st.root_euler_d.copy()
        st.root_pos = st.root_pos.copy()
    for t in (2, 3, 9):  # a low body: no terrain sample (:341-345)
        ticks[t].root_pos[1, 2] = 0.08
    rows = np.stack([mpcqp.pack_states(st) for st in ticks])
    path = tmp_path / "states.bin"
    np.ascontiguousarray(rows, dtype=np.float64).tofile(path)
    out = subprocess.run([exe, str(path), str(T), str(B), "terrain"], check=True, capture_output=True, text=True,
                         timeout=120).stdout
    got = {"TICK": {}, "BATCH": {}}
    terr = {"TICK": {}, "BATCH": {}}
    calls = {}
    for line in out.splitlines():
        p = line.split()
        if p[0] in got:
            # TICK / BATCH t b type status iters rho_updates u0[12]
            got[p[0]][(int(p[1]), int(p[2]))] = (int(p[4]), int(p[5]), int(p[6]), np.array([float(x) for x in p[7:]]))
        elif p[0] == "TERRAIN":
            terr[p[1]][(int(p[2]), int(p[3]))] = (float(p[4]), float(p[5]))
        elif p[0] == "HOOKCALLS":
            calls[p[1]] = int(p[2])

    def mode(t, b):
        return 0 if (t + b) % 8 in (3, 4) else 1

    def recent_z(t, b, l):
        return -0.3 + 0.04 * ((3 * t + b + l) % 4)
    expect_calls = 0
    n_neg = n_clamped = 0
    for t in range(T):
        for b in range(B):
            if mode(t, b) != 1:
                assert (t, b) not in terr["TICK"]
                continue
            high = ticks[t].root_pos[b, 2] > 0.1
            expect_calls += int(high)
            ang = 0.7 * np.sin(0.9 * t + 1.7 * b) if high else 0.0
            n_clamped += int(abs(ang) > 0.5)
            ang = min(max(ang, -0.5), 0.5)
            frd = recent_z(t, b, 0) + recent_z(t, b, 1) - recent_z(t, b, 2) - recent_z(t, b, 3)
            e1 = -ang if frd > 0.05 else ang
            n_neg += int(frd > 0.05 and ang != 0.0)
            for tag in ("TICK", "BATCH"):
                g1, gp = terr[tag][(t, b)]
                assert abs(gp - ang) <= 1e-15 and abs(g1 - e1) <= 1e-15, (tag, t, b, g1, e1, gp, ang)
            assert terr["TICK"][(t, b)] == terr["BATCH"][(t, b)]
            ticks[t].root_euler_d[b, 1] = terr["TICK"][(t, b)][0]  # the adapted state, bit for bit
    assert calls == {"TICK": expect_calls, "BATCH": expect_calls}
    assert n_neg > 0 and n_clamped > 0 and expect_calls < sum(mode(t, b) for t in range(T) for b in range(B))
    recs_t = np.stack([mpcqp.assemble_compute_grf(st, 10) for st in ticks])
    op = oracle.default_params(10)
    moved = 0.0
    for b in range(B):
        mts = [t for t in range(T) if mode(t, b) == 1]
        ref_m = oracle.solve_sequence(op, np.ascontiguousarray(recs_t[mts, b:b + 1]), nthreads=1)
        for i, t in enumerate(mts):
            r = ref_m[i][0]
            for tag in ("TICK", "BATCH"):
                st, it, ru, u0 = got[tag][(t, b)]
                assert (st, it) == (int(r["status"]), int(r["iters"])), (tag, t, b)
                err = np.max(np.abs(u0 - r["u0"])) / max(np.max(np.abs(r["u0"])), 1.0)
                assert err <= 1e-4, (tag, t, b, err)
            # x_ref's pitch row is the adapted one
            xr = recs_t[t, b, mpcqp._lib.REC_XREF:mpcqp._lib.REC_XREF + 130].reshape(10, 13)
            assert np.all(xr[:, 1] == terr["TICK"][(t, b)][0])
        plain = [mpcqp.assemble_compute_grf(st, 10)[b] for st in mpcqp.records.synthetic_go1_ticks(
            B, T, seed=47, gait="trot", swing_ticks=5)]
        ref_p = oracle.solve_sequence(op, np.ascontiguousarray(np.stack([plain[t] for t in mts])[:, None]), nthreads=1)
        moved = max(moved, max(np.max(np.abs(ref_p[i][0]["u0"] - got["TICK"][(t, b)][3])) for i, t in enumerate(mts)))
    assert moved > 1e-3  # the adaptation changes the forces, so the comparison above can see it
