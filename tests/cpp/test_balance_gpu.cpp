// The QP balance branch of A1RobotControl::compute_grf (stance_leg_control_type == 0,
// A1RobotControl.cpp:377-444) driven through the drop-in shim's compute_grf_qp on a Go1-like
// state with A1CtrlStates field names.  Prints the record it assembled and the forces, which
// tests/test_cpp_shim.py solves again on the CPU oracle.
#include <cmath>
#include <cstdio>

#include "../../include/mpcqp_robot_control.hpp"

struct Vec {
  double v[16] = {0};
  double& operator[](int i) { return v[i]; }
  const double& operator[](int i) const { return v[i]; }
};
struct Mat {
  double a[3][4] = {{0}};
  double& operator()(int r, int c) { return a[r][c]; }
  const double& operator()(int r, int c) const { return a[r][c]; }
};
struct State {  // the A1CtrlStates fields the QP branch reads
  double robot_mass = 13.0;
  Mat go1_trunk_inertia, root_rot_mat, root_rot_mat_z, foot_pos_abs;
  Vec root_euler, root_pos, root_ang_vel, root_lin_vel, root_euler_d, root_pos_d, root_ang_vel_d, root_lin_vel_d;
  Vec kp_linear, kd_linear, kp_angular, kd_angular;
  bool contacts[4] = {true, false, false, true};
};

int main() {
  State s;
  const double yaw = 0.4, c = std::cos(yaw), sn = std::sin(yaw);
  const double Rz[3][3] = {{c, -sn, 0}, {sn, c, 0}, {0, 0, 1}};
  for (int r = 0; r < 3; ++r)
    for (int k = 0; k < 3; ++k) s.root_rot_mat(r, k) = s.root_rot_mat_z(r, k) = Rz[r][k];
  s.root_euler[2] = yaw;
  s.root_euler_d[2] = yaw + 0.05;
  s.root_pos[2] = 0.27;
  s.root_pos_d[2] = 0.30;
  s.root_lin_vel[0] = 0.2;
  s.root_lin_vel_d[0] = 0.4;
  s.root_ang_vel[2] = 0.1;
  const double fx[4] = {0.17, 0.17, -0.17, -0.17}, fy[4] = {0.15, -0.15, 0.15, -0.15};
  for (int l = 0; l < 4; ++l) {
    const double b[3] = {fx[l], fy[l], -0.30};
    for (int r = 0; r < 3; ++r) s.foot_pos_abs(r, l) = Rz[r][0] * b[0] + Rz[r][1] * b[1] + Rz[r][2] * b[2];
  }
  const double kp[3] = {100, 100, 300}, kd[3] = {70, 70, 120}, kpa[3] = {150, 150, 1}, kda[3] = {4.5, 4.5, 30};
  for (int k = 0; k < 3; ++k) {  // Go1CtrlStates.hpp:276-307 defaults
    s.kp_linear[k] = kp[k];
    s.kd_linear[k] = kd[k];
    s.kp_angular[k] = kpa[k];
    s.kd_angular[k] = kda[k];
  }
  double q[13] = {0}, r[12] = {0};
  mpcqp_cpp::Go1RobotControl ctrl(q, r);
  Mat forces;
  mpcqp_result res;
  double f[12];
  ctrl.compute_grf_qp_batch(&s, 1, f, &res);
  ctrl.compute_grf_qp(s, forces);
  double rec[MPCQP_BAL_SIZE];
  mpcqp_cpp::Go1RobotControl::assemble_balance(s, rec);
  std::printf("REC");
  for (int k = 0; k < MPCQP_BAL_SIZE; ++k) std::printf(" %.17g", rec[k]);
  std::printf("\nSTATUS %d ITERS %d\n", res.status, res.iters);
  for (int rr = 0; rr < 3; ++rr) {
    std::printf("GRF");
    for (int l = 0; l < 4; ++l) std::printf(" %.17g", forces(rr, l));
    std::printf("\n");
  }
  return 0;
}
