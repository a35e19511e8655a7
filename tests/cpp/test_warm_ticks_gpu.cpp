// Production tick sequence through the drop-in shim: the reference's GRF thread calls
// A1RobotControl::compute_grf(state, dt) once per tick on a controller that owns a persistent,
// warm-started OsqpEigen solver (A1RobotControl.h:44,67; A1RobotControl.cpp:446-562).  Here every
// robot has its own mpcqp_cpp::A1RobotControl (warm_start on, its default), driven tick by tick
// with `state.foot_forces_grf = ctrl.compute_grf(state, dt)`; a second, batched controller runs
// all robots per tick through compute_grf_batch.  Input: the robot-state rows of
// include/mpcqp.h (MPCQP_ST_*) as a raw binary64 file [ticks][robots][MPCQP_ST_SIZE].
// Output lines (compared with the oracle's persistent solver by tests/test_cpp_shim.py):
//   TICK t b status iters rho_updates u0[12]       (per-robot controllers)
//   BATCH t b status iters rho_updates u0[12]      (batched controller)
//   GRF t b f[3x4 row-major]                       (returned matrix of the per-robot call)
#include <cstdio>
#include <cstdlib>
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
struct State {  // the A1CtrlStates fields compute_grf reads and writes
  double robot_mass = 0;
  Mat a1_trunk_inertia, root_rot_mat, foot_pos_abs, foot_forces_grf;
  Vec root_euler, root_pos, root_ang_vel, root_lin_vel, root_euler_d, root_pos_d, root_ang_vel_d, root_lin_vel_d,
      root_lin_vel_d_world, mpc_states, mpc_states_d;
  bool contacts[4] = {false, false, false, false};
};

static void load(State& s, const double* row) {
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
  for (int l = 0; l < 4; ++l) {
    for (int r = 0; r < 3; ++r) s.foot_pos_abs(r, l) = row[MPCQP_ST_FEET + 3 * l + r];
    s.contacts[l] = row[MPCQP_ST_CONTACTS + l] != 0.0;
  }
  s.robot_mass = row[MPCQP_ST_MASS];
}

static void print(const char* tag, int t, int b, const mpcqp_result& r) {
  std::printf("%s %d %d %d %d %d", tag, t, b, r.status, r.iters, r.rho_updates);
  for (int k = 0; k < 12; ++k) std::printf(" %.17g", r.u0[k]);
  std::printf("\n");
}

int main(int argc, char** argv) {
  if (argc != 4) {
    std::fprintf(stderr, "usage: %s states.bin ticks robots\n", argv[0]);
    return 2;
  }
  const int T = std::atoi(argv[2]), B = std::atoi(argv[3]);
  std::vector<double> rows((size_t)T * B * MPCQP_ST_SIZE);
  FILE* f = std::fopen(argv[1], "rb");
  if (!f || std::fread(rows.data(), sizeof(double), rows.size(), f) != rows.size()) {
    std::fprintf(stderr, "cannot read %s\n", argv[1]);
    return 2;
  }
  std::fclose(f);
  // Go1 weights (Go1CtrlStates.hpp:203-249), the same as mpcqp_default_params
  const double q[13] = {80.0, 80.0, 1.0, 0.0, 0.0, 270.0, 1.0, 1.0, 20.0, 20.0, 20.0, 20.0, 0.0};
  const double r[12] = {1e-5, 1e-5, 1e-6, 1e-5, 1e-5, 1e-6, 1e-5, 1e-5, 1e-6, 1e-5, 1e-5, 1e-6};
  std::vector<std::unique_ptr<mpcqp_cpp::A1RobotControl>> ctrl;
  for (int b = 0; b < B; ++b) ctrl.emplace_back(new mpcqp_cpp::A1RobotControl(q, r));
  mpcqp_cpp::A1RobotControl batch(q, r);
  std::vector<State> states(B), bstates(B);
  std::vector<double> forces((size_t)B * 12);
  std::vector<mpcqp_result> res(B);
  const double dt = 0.002;  // the thread's period; the horizon step stays mpc_dt = 0.0025
  for (int t = 0; t < T; ++t) {
    for (int b = 0; b < B; ++b) {
      State& s = states[b];
      load(s, &rows[((size_t)t * B + b) * MPCQP_ST_SIZE]);
      s.foot_forces_grf = ctrl[b]->compute_grf(s, dt);
      print("TICK", t, b, ctrl[b]->last_result());
      std::printf("GRF %d %d", t, b);
      for (int rr = 0; rr < 3; ++rr)
        for (int l = 0; l < 4; ++l) std::printf(" %.17g", s.foot_forces_grf(rr, l));
      std::printf("\n");
      load(bstates[b], &rows[((size_t)t * B + b) * MPCQP_ST_SIZE]);
    }
    batch.compute_grf_batch(bstates.data(), B, forces.data(), res.data(), dt);
    for (int b = 0; b < B; ++b) print("BATCH", t, b, res[b]);
  }
  return 0;
}
