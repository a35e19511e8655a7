// compute_grf's mode dispatch through the drop-in shim: the reference's single entry point
// A1RobotControl::compute_grf(state, dt) takes the QP balance branch when
// state.stance_leg_control_type == 0 (A1RobotControl.cpp:377-444, a fresh local solver) and the MPC
// branch when it is 1 (:446-562, the member solver, warm-started).  Every robot here switches mode
// mid-sequence; per-robot controllers call `foot_forces_grf = compute_grf(state, dt)` and a second,
// batched controller takes mixed-mode batches.  Input: robot-state rows (MPCQP_ST_*) as a raw binary64
// file [ticks][robots][MPCQP_ST_SIZE]; the mode schedule is type(t, b) = 0 iff (t + b) % 8 is 3 or 4.
// Output lines (checked against the oracle by tests/test_cpp_shim.py):
//   TICK t b type status iters rho_updates u0[12]   (per-robot controllers)
//   GRF t b f[3x4 row-major]                        (returned matrix of the per-robot call)
//   BATCH t b type status iters rho_updates u0[12]  (batched controller, mixed modes)
//   BALREC t b rec[MPCQP_BAL_SIZE]                  (the balance record a QP tick solved)
// With a fourth argument "terrain" both controllers also run the terrain adaptation of
// A1RobotControl.cpp:334-376 through the shim's terrain_angle_of hook (a deterministic filtered
// angle per tick and robot, terrain_in below; foot_pos_recent_contact z from recent_z below) and
// print, per MPC robot after the call,
//   TERRAIN tag t b root_euler_d[1] terrain_pitch_angle
// and at the end HOOKCALLS tag n (the hook runs only where root_pos[2] > 0.1).
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

#include "../../include/mpcqp_robot_control.hpp"

struct Vec {
  double v[13 * 10] = {0};
  double& operator[](int i) { return v[i]; }
  const double& operator[](int i) const { return v[i]; }
};
struct Mat {
  double a[3][4] = {{0}};
  double& operator()(int r, int c) { return a[r][c]; }
  const double& operator()(int r, int c) const { return a[r][c]; }
};
struct State {  // the A1CtrlStates fields both branches of compute_grf read and write
  int stance_leg_control_type = 1;
  double robot_mass = 0;
  Mat a1_trunk_inertia, root_rot_mat, root_rot_mat_z, foot_pos_abs, foot_forces_grf;
  Vec root_euler, root_pos, root_ang_vel, root_lin_vel, root_euler_d, root_pos_d, root_ang_vel_d, root_lin_vel_d,
      root_lin_vel_d_world, mpc_states, mpc_states_d;
  Vec kp_linear, kd_linear, kp_angular, kd_angular;
  bool contacts[4] = {false, false, false, false};
  int use_terrain_adapt = 1;  // terrain fields (A1CtrlStates.h:332, :370)
  double terrain_pitch_angle = 0;
  Mat foot_pos_recent_contact;
};

// the terrain inputs the test feeds (tests/test_cpp_shim.py mirrors both)
static double terrain_in(int t, int b) { return 0.7 * std::sin(0.9 * t + 1.7 * b); }
static double recent_z(int t, int b, int l) { return -0.3 + 0.04 * ((3 * t + b + l) % 4); }

static int mode_of(int t, int b) { return ((t + b) % 8 == 3 || (t + b) % 8 == 4) ? 0 : 1; }

static void load(State& s, const double* row, int type) {
  s.stance_leg_control_type = type;
  for (int k = 0; k < 3; ++k) {
    s.root_euler[k] = row[MPCQP_ST_EULER + k];
    s.root_pos[k] = row[MPCQP_ST_POS + k];
    s.root_ang_vel[k] = row[MPCQP_ST_ANG_VEL + k];
    s.root_lin_vel[k] = row[MPCQP_ST_LIN_VEL + k];
    s.root_euler_d[k] = row[MPCQP_ST_EULER_D + k];
    s.root_pos_d[k] = row[MPCQP_ST_POS_D + k];
    s.root_ang_vel_d[k] = row[MPCQP_ST_ANG_VEL_D + k];
    s.root_lin_vel_d[k] = row[MPCQP_ST_LIN_VEL_D + k];
  }
  for (int r = 0; r < 3; ++r)
    for (int c = 0; c < 3; ++c) {
      s.root_rot_mat(r, c) = row[MPCQP_ST_ROT + 3 * r + c];
      s.a1_trunk_inertia(r, c) = row[MPCQP_ST_INERTIA + 3 * r + c];
    }
  // root_rot_mat_z = AngleAxisd(yaw, UnitZ) (GazeboA1ROS.cpp:269)
  const double yaw = s.root_euler[2], cy = std::cos(yaw), sy = std::sin(yaw);
  const double Rz[3][3] = {{cy, -sy, 0}, {sy, cy, 0}, {0, 0, 1}};
  for (int r = 0; r < 3; ++r)
    for (int c = 0; c < 3; ++c) s.root_rot_mat_z(r, c) = Rz[r][c];
  for (int l = 0; l < 4; ++l) {
    for (int r = 0; r < 3; ++r) s.foot_pos_abs(r, l) = row[MPCQP_ST_FEET + 3 * l + r];
    s.contacts[l] = row[MPCQP_ST_CONTACTS + l] != 0.0;
  }
  s.robot_mass = row[MPCQP_ST_MASS];
  s.use_terrain_adapt = 1;
  s.terrain_pitch_angle = 0;
  const double kp[3] = {100, 100, 300}, kd[3] = {70, 70, 120}, kpa[3] = {150, 150, 1}, kda[3] = {4.5, 4.5, 30};
  for (int k = 0; k < 3; ++k) {  // Go1CtrlStates.hpp:276-307 defaults
    s.kp_linear[k] = kp[k];
    s.kd_linear[k] = kd[k];
    s.kp_angular[k] = kpa[k];
    s.kd_angular[k] = kda[k];
  }
}

static void print(const char* tag, int t, int b, int type, const mpcqp_result& r) {
  std::printf("%s %d %d %d %d %d %d", tag, t, b, type, r.status, r.iters, r.rho_updates);
  for (int k = 0; k < 12; ++k) std::printf(" %.17g", r.u0[k]);
  std::printf("\n");
}

int main(int argc, char** argv) {
  if (argc != 4 && argc != 5) {
    std::fprintf(stderr, "usage: %s states.bin ticks robots [terrain]\n", argv[0]);
    return 2;
  }
  const int T = std::atoi(argv[2]), B = std::atoi(argv[3]);
  const bool terrain = argc == 5 && std::string(argv[4]) == "terrain";
  std::vector<double> rows((size_t)T * B * MPCQP_ST_SIZE);
  FILE* f = std::fopen(argv[1], "rb");
  if (!f || std::fread(rows.data(), sizeof(double), rows.size(), f) != rows.size()) {
    std::fprintf(stderr, "cannot read %s\n", argv[1]);
    return 2;
  }
  std::fclose(f);
  const double q[13] = {80.0, 80.0, 1.0, 0.0, 0.0, 270.0, 1.0, 1.0, 20.0, 20.0, 20.0, 20.0, 0.0};
  const double r[12] = {1e-5, 1e-5, 1e-6, 1e-5, 1e-5, 1e-6, 1e-5, 1e-5, 1e-6, 1e-5, 1e-5, 1e-6};
  std::vector<std::unique_ptr<mpcqp_cpp::A1RobotControl>> ctrl;
  for (int b = 0; b < B; ++b) ctrl.emplace_back(new mpcqp_cpp::A1RobotControl(q, r));
  mpcqp_cpp::A1RobotControl batch(q, r);
  std::vector<State> states(B), bstates(B);
  std::vector<double> forces((size_t)B * 12);
  std::vector<mpcqp_result> res(B);
  const double dt = 0.002;
  int cur_t = 0, calls_tick = 0, calls_batch = 0;
  if (terrain) {
    for (int b = 0; b < B; ++b)
      ctrl[b]->terrain_angle_of = [&cur_t, &calls_tick, b](int i) {
        if (i != 0) std::abort();  // a single-robot call is robot 0 of its batch
        ++calls_tick;
        return terrain_in(cur_t, b);
      };
    batch.terrain_angle_of = [&cur_t, &calls_batch](int i) {
      ++calls_batch;
      return terrain_in(cur_t, i);
    };
  }
  auto set_recent = [&](State& s, int t, int b) {
    for (int l = 0; l < 4; ++l) {
      for (int r = 0; r < 2; ++r) s.foot_pos_recent_contact(r, l) = s.foot_pos_abs(r, l);
      s.foot_pos_recent_contact(2, l) = recent_z(t, b, l);
    }
  };
  for (int t = 0; t < T; ++t) {
    cur_t = t;
    for (int b = 0; b < B; ++b) {
      State& s = states[b];
      const int ty = mode_of(t, b);
      load(s, &rows[((size_t)t * B + b) * MPCQP_ST_SIZE], ty);
      set_recent(s, t, b);
      s.foot_forces_grf = ctrl[b]->compute_grf(s, dt);
      print("TICK", t, b, ty, ctrl[b]->last_result());
      if (terrain && ty == 1) std::printf("TERRAIN TICK %d %d %.17g %.17g\n", t, b, s.root_euler_d[1], s.terrain_pitch_angle);
      std::printf("GRF %d %d", t, b);
      for (int rr = 0; rr < 3; ++rr)
        for (int l = 0; l < 4; ++l) std::printf(" %.17g", s.foot_forces_grf(rr, l));
      std::printf("\n");
      if (ty == 0) {
        double rec[MPCQP_BAL_SIZE];
        mpcqp_cpp::A1RobotControl::assemble_balance(s, rec);
        std::printf("BALREC %d %d", t, b);
        for (double v : rec) std::printf(" %.17g", v);
        std::printf("\n");
      }
      load(bstates[b], &rows[((size_t)t * B + b) * MPCQP_ST_SIZE], ty);
      set_recent(bstates[b], t, b);
    }
    batch.compute_grf_batch(bstates.data(), B, forces.data(), res.data(), dt);
    for (int b = 0; b < B; ++b) {
      print("BATCH", t, b, mode_of(t, b), res[b]);
      if (terrain && mode_of(t, b) == 1)
        std::printf("TERRAIN BATCH %d %d %.17g %.17g\n", t, b, bstates[b].root_euler_d[1],
                    bstates[b].terrain_pitch_angle);
    }
  }
  if (terrain) std::printf("HOOKCALLS TICK %d\nHOOKCALLS BATCH %d\n", calls_tick, calls_batch);
  // an unknown control type is rejected, not silently solved
  State bad;
  load(bad, &rows[0], 2);
  try {
    ctrl[0]->compute_grf(bad, dt);
    std::printf("BADTYPE accepted\n");
  } catch (const std::invalid_argument&) {
    std::printf("BADTYPE rejected\n");
  }
  return 0;
}
