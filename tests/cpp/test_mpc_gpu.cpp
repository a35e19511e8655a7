// C++ port of the reference harness src/a1_cpp/src/test/test_mpc.cpp:14-162, driven through the
// drop-in shim (include/mpcqp_robot_control.hpp) instead of Eigen/OsqpEigen.  Same hand-set
// stance, same call sequence (ConvexMpc ctor/reset, A_c from the horizon-average euler, B per step
// with shifted feet, calculate_qp_mats), then the GPU solve.  Prints machine-readable lines that
// tests/test_cpp_shim.py compares with the CPU oracle.
#include <cstdio>
#include <cstring>

#include "../../include/mpcqp_robot_control.hpp"

struct Vec {  // Eigen::VectorXd stand-in for the test (operator[])
  double v[300] = {0};
  double& operator[](int i) { return v[i]; }
  const double& operator[](int i) const { return v[i]; }
};
struct Mat {  // Eigen::Matrix<double,3,4> / Matrix3d stand-in (operator()(r,c)), row-major up to 3x4
  double a[3][4] = {{0}};
  double& operator()(int r, int c) { return a[r][c]; }
  const double& operator()(int r, int c) const { return a[r][c]; }
};
struct State {  // the A1CtrlStates fields test_mpc touches
  double robot_mass = 0;
  Mat a1_trunk_inertia, root_rot_mat, foot_pos_rel, foot_pos_abs_mpc, foot_pos_abs;
  Vec root_euler, root_pos, root_ang_vel, root_lin_vel, root_euler_d, root_pos_d, root_ang_vel_d, root_lin_vel_d,
      root_lin_vel_d_world, mpc_states, mpc_states_d;
  bool contacts[4] = {false, false, false, false};
};

int main() {
  constexpr int PLAN_HORIZON = 10;
  State state;
  state.robot_mass = 15;  // :18
  state.a1_trunk_inertia(0, 0) = 0.0158533;
  state.a1_trunk_inertia(1, 1) = 0.0377999;
  state.a1_trunk_inertia(2, 2) = 0.0456542;
  for (int i = 0; i < 3; ++i) state.root_rot_mat(i, i) = 1.0;  // :25-30, all-zero angles
  state.root_pos[2] = 0.15;                                     // :32
  const double fx[4] = {0.17, 0.17, -0.17, -0.17}, fy[4] = {0.15, -0.15, 0.15, -0.15};
  for (int l = 0; l < 4; ++l) {  // :39-41
    state.foot_pos_rel(0, l) = fx[l];
    state.foot_pos_rel(1, l) = fy[l];
    state.foot_pos_rel(2, l) = -0.35;
  }
  state.contacts[0] = true;  // :43-46
  state.contacts[2] = true;
  const double dt = 0.0025;
  Vec q_weights, r_weights;  // :50-60
  const double q[13] = {1.0, 1.0, 1.0, 0.0, 0.0, 50.0, 0.0, 0.0, 1.0, 1.0, 1.0, 1.0, 0.0};
  for (int i = 0; i < 13; ++i) q_weights[i] = q[i];
  for (int i = 0; i < 12; ++i) r_weights[i] = 1e-6;
  mpcqp_cpp::ConvexMpc<PLAN_HORIZON> mpc_solver(q_weights, r_weights);
  mpc_solver.reset();
  const double x0[13] = {state.root_euler[0], state.root_euler[1], state.root_euler[2], state.root_pos[0],
                         state.root_pos[1], state.root_pos[2], state.root_ang_vel[0], state.root_ang_vel[1],
                         state.root_ang_vel[2], state.root_lin_vel[0], state.root_lin_vel[1], state.root_lin_vel[2],
                         -9.8};
  for (int k = 0; k < 13; ++k) state.mpc_states[k] = x0[k];
  for (int r = 0; r < 3; ++r) {  // :73
    double acc = 0;
    for (int c = 0; c < 3; ++c) acc += state.root_rot_mat(r, c) * state.root_lin_vel_d[c];
    state.root_lin_vel_d_world[r] = acc;
  }
  for (int i = 0; i < PLAN_HORIZON; ++i) {  // :75-91
    const double xr[13] = {state.root_euler_d[0], state.root_euler_d[1],
                           state.root_euler[2] + state.root_ang_vel_d[2] * dt * (i + 1),
                           state.root_pos[0] + state.root_lin_vel_d_world[0] * dt * (i + 1),
                           state.root_pos[1] + state.root_lin_vel_d_world[1] * dt * (i + 1),
                           state.root_pos[2] + state.root_lin_vel_d_world[1] * dt * (i + 1),
                           state.root_ang_vel_d[0], state.root_ang_vel_d[1], state.root_ang_vel_d[2],
                           state.root_lin_vel_d_world[0], state.root_lin_vel_d_world[1],
                           state.root_lin_vel_d_world[2], -9.8};
    for (int k = 0; k < 13; ++k) state.mpc_states_d[13 * i + k] = xr[k];
  }
  Vec avg;  // :94-101
  for (int k = 0; k < 3; ++k)
    avg[k] = (state.root_euler[k] + state.root_euler[k] + state.root_ang_vel_d[k] * dt * PLAN_HORIZON) /
             (PLAN_HORIZON + 1);
  mpc_solver.calculate_A_mat_c(avg);
  state.foot_pos_abs_mpc = state.foot_pos_rel;  // :105
  for (int i = 0; i < PLAN_HORIZON; i++) {      // :106-122
    mpc_solver.calculate_B_mat_c(state.robot_mass, state.a1_trunk_inertia, state.root_rot_mat,
                                 state.foot_pos_abs_mpc);
    for (int l = 0; l < 4; ++l)
      for (int r = 0; r < 3; ++r) state.foot_pos_abs_mpc(r, l) -= state.root_lin_vel_d[r] * dt;
    mpc_solver.state_space_discretization(dt);
    mpc_solver.B_mat_d_list.block<13, 12>(i * 13, 0) = mpc_solver.B_mat_d;  // :121, verbatim
  }
  mpc_solver.calculate_qp_mats(state);  // :125
  // the large members are produced on first read (nothing has been read yet)
  std::printf("LAZY_BEFORE %d %d %d %d %d\n", (int)mpc_solver.hessian.computed(), (int)mpc_solver.gradient.computed(),
              (int)mpc_solver.linear_constraints.computed(), (int)mpc_solver.A_qp.computed(),
              (int)mpc_solver.B_qp.computed());
  double hsum = 0, hmax = 0, gsum = 0;
  for (double v : mpc_solver.hessian) { hsum += v; hmax = v > hmax ? v : hmax; }
  for (double v : mpc_solver.gradient) gsum += v;
  std::printf("HESSIAN_SUM %.17g\nHESSIAN_MAX %.17g\nGRADIENT_SUM %.17g\n", hsum, hmax, gsum);
  std::printf("HESSIAN_00 %.17g\n", mpc_solver.hessian[0]);
  std::printf("LAZY_AFTER_H %d %d %d %d %d\n", (int)mpc_solver.hessian.computed(), (int)mpc_solver.gradient.computed(),
              (int)mpc_solver.linear_constraints.computed(), (int)mpc_solver.A_qp.computed(),
              (int)mpc_solver.B_qp.computed());
  // A_qp (13N x 13) and B_qp (13N x 12N) of ConvexMpc.cpp:184-202, read like the Eigen members
  std::printf("A_QP %d %d", (int)mpc_solver.A_qp.rows(), (int)mpc_solver.A_qp.cols());
  for (int i = 0; i < mpc_solver.A_qp.rows(); ++i)
    for (int j = 0; j < mpc_solver.A_qp.cols(); ++j) std::printf(" %.17g", mpc_solver.A_qp(i, j));
  std::printf("\nB_QP %d %d", (int)mpc_solver.B_qp.rows(), (int)mpc_solver.B_qp.cols());
  for (int i = 0; i < mpc_solver.B_qp.rows(); ++i)
    for (int j = 0; j < mpc_solver.B_qp.cols(); ++j) std::printf(" %.17g", mpc_solver.B_qp(i, j));
  std::printf("\nA_MAT_D");
  for (int i = 0; i < 13; ++i)
    for (int j = 0; j < 13; ++j) std::printf(" %.17g", mpc_solver.A_mat_d(i, j));
  std::printf("\nLIN_CON %d", (int)mpc_solver.linear_constraints.size());
  for (double v : mpc_solver.linear_constraints) std::printf(" %.17g", v);
  std::printf("\n");

  // :131-151 solve (fresh solver, cold start) through the C ABI
  mpcqp_result res;
  mpcqp_cpp::throw_on(mpcqp_solve_batch_host(mpc_solver.handle(), mpc_solver.record().data(), 1, &res, nullptr),
                      mpc_solver.handle(), "solve");
  std::printf("STATUS %d ITERS %d RHO_UPDATES %d\n", res.status, res.iters, res.rho_updates);
  // :153-157 print the 3x4 world-frame forces
  for (int r = 0; r < 3; ++r) {
    std::printf("ROW");
    for (int l = 0; l < 4; ++l) std::printf(" %.17g", res.u0[3 * l + r]);
    std::printf("\n");
  }

  // the formulation's device staging lives on the handle's device
  hipPointerAttribute_t at;
  mpcqp_cpp::hip_ok(hipPointerGetAttributes(&at, mpc_solver.staging()), "hipPointerGetAttributes");
  std::printf("STAGING_DEVICE %d HANDLE_DEVICE %d\n", at.device, mpc_solver.device());

  // B_mat_d_list is an input: a block the caller computed elsewhere (here: feet of step 3 moved by
  // +0.01 in x through a second ConvexMpc) is read back into the formulation through I_w.
  {
    mpcqp_cpp::ConvexMpc<PLAN_HORIZON> other(q_weights, r_weights);
    Mat moved = state.foot_pos_rel;
    for (int l = 0; l < 4; ++l)
      for (int r = 0; r < 3; ++r) moved(r, l) -= 3 * state.root_lin_vel_d[r] * dt;
    for (int l = 0; l < 4; ++l) moved(0, l) += 0.01;
    other.calculate_A_mat_c(avg);
    other.calculate_B_mat_c(state.robot_mass, state.a1_trunk_inertia, state.root_rot_mat, moved);
    other.state_space_discretization(dt);
    mpc_solver.B_mat_d_list.block<13, 12>(3 * 13, 0) = other.B_mat_d;
    mpc_solver.calculate_qp_mats(state);
    std::printf("RECOVERED_FEET");
    for (int k = 0; k < 12; ++k) std::printf(" %.17g", mpc_solver.record()[MPCQP_REC_FEET(PLAN_HORIZON) + 36 + k]);
    double hs = 0;
    for (double v : mpc_solver.hessian) hs += v;
    std::printf("\nRECOVERED_HESSIAN_SUM %.17g\n", hs);
    std::printf("RECORD");
    for (double v : mpc_solver.record()) std::printf(" %.17g", v);
    std::printf("\n");
  }

  // compute_grf (A1RobotControl.h:44, A1RobotControl.cpp:446-561) on the same stance, production
  // assembly: `foot_forces_grf = compute_grf(state, dt)` with the 3x4 return value
  state.foot_pos_abs = state.foot_pos_rel;
  state.root_pos_d[2] = 0.15;
  mpcqp_cpp::A1RobotControl ctrl(q_weights, r_weights);
  Mat forces = ctrl.compute_grf(state, dt);
  for (int r = 0; r < 3; ++r) {
    std::printf("GRF");
    for (int l = 0; l < 4; ++l) std::printf(" %.17g", forces(r, l));
    std::printf("\n");
  }
  // Gazebo: use_sim_time makes the horizon step the caller's dt (A1RobotControl.cpp:464-467)
  mpcqp_cpp::A1RobotControl ctrl_sim(q_weights, r_weights);
  ctrl_sim.use_sim_time = true;
  Mat forces_sim;
  ctrl_sim.compute_grf(state, 0.004, forces_sim);
  for (int r = 0; r < 3; ++r) {
    std::printf("GRFSIM");
    for (int l = 0; l < 4; ++l) std::printf(" %.17g", forces_sim(r, l));
    std::printf("\n");
  }
  return 0;
}
