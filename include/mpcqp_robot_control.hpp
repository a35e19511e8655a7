// mpcqp_robot_control.hpp — header-only C++ drop-in for the reference's GRF call surface,
// implemented over the C ABI in mpcqp.h (link with libmpcqp.so).
//
//   mpcqp_cpp::ConvexMpc<N>          ≙ class ConvexMpc (src/a1_cpp/src/ConvexMpc.h:22-94)
//   mpcqp_cpp::A1RobotControl        ≙ A1RobotControl::compute_grf MPC branch
//                                       (src/a1_cpp/src/A1RobotControl.cpp:446-562)
//   mpcqp_cpp::Go1RobotControl       ≙ the declared-but-undefined Go1 hook
//                                       (src/go1_rl_ctrl_cpp/src/Go1RLController.hpp:38-40)
//
// Eigen-agnostic: state types are templates; anything with operator[] for 3-vectors,
// operator()(r,c) for matrices and a bool contacts[4] works (Eigen::Vector3d / Matrix3d /
// Matrix<double,3,4> included), so A1CtrlStates / Go1CtrlStates plug in unchanged.
#pragma once

#include <cmath>
#include <cstring>
#include <stdexcept>
#include <string>
#include <vector>

#include "mpcqp.h"

namespace mpcqp_cpp {

inline void throw_on(int32_t rc, mpcqp_handle* h, const char* what) {
  if (rc != MPCQP_OK) {
    std::string msg = std::string(what) + ": " + mpcqp_error_str(rc);
    if (h) msg += std::string(" (") + mpcqp_last_error(h) + ")";
    throw std::runtime_error(msg);
  }
}

// ---------------------------------------------------------------------------------------------
// ConvexMpc: same method names and call order as the reference; calculate_qp_mats() runs the
// formulation on the GPU (mpcqp_build_qp_device) and fills the public members.
// ---------------------------------------------------------------------------------------------
template <int N = 10>
class ConvexMpc {
 public:
  static constexpr int n = MPCQP_NUM_DOF * N;
  static constexpr int m = MPCQP_CONSTRAINT_DIM * N;

  template <class VecQ, class VecR>
  ConvexMpc(const VecQ& q_weights_, const VecR& r_weights_, int device = 0) : mu(0.3), fz_min(0), fz_max(0) {
    mpcqp_default_params(&params_, N);
    for (int i = 0; i < MPCQP_STATE_DIM; ++i) params_.q_weights[i] = q_weights_[i];
    for (int i = 0; i < MPCQP_NUM_DOF; ++i) params_.r_weights[i] = r_weights_[i];
    throw_on(mpcqp_create(&params_, device, &h_), nullptr, "mpcqp_create");
    hessian.assign((size_t)n * n, 0.0);
    gradient.assign(n, 0.0);
    lb.assign(m, 0.0);
    ub.assign(m, 0.0);
    linear_constraints.assign((size_t)m * n, 0.0);
    reset();
  }
  ~ConvexMpc() {
    free_device();
    if (h_) mpcqp_destroy(h_);
  }
  ConvexMpc(const ConvexMpc&) = delete;
  ConvexMpc& operator=(const ConvexMpc&) = delete;

  void reset() {  // ConvexMpc.cpp:70-108
    rec_.assign(MPCQP_REC_SIZE(N), 0.0);
    step_ = 0;
    std::fill(gradient.begin(), gradient.end(), 0.0);
    std::fill(lb.begin(), lb.end(), 0.0);
    std::fill(ub.begin(), ub.end(), 0.0);
  }

  template <class Vec3>
  void calculate_A_mat_c(const Vec3& root_euler) {  // ConvexMpc.cpp:110-130 (yaw only)
    for (int k = 0; k < 3; ++k) rec_[MPCQP_REC_EULER + k] = root_euler[k];
  }

  // ConvexMpc.cpp:132-143: the body inertia, rotation and feet of the NEXT horizon step.
  template <class Mat3a, class Mat3b, class Mat34>
  void calculate_B_mat_c(double robot_mass, const Mat3a& trunk_inertia, const Mat3b& root_rot_mat,
                         const Mat34& foot_pos) {
    rec_[MPCQP_REC_MASS] = robot_mass;
    for (int r = 0; r < 3; ++r)
      for (int c = 0; c < 3; ++c) {
        rec_[MPCQP_REC_INERTIA + 3 * r + c] = trunk_inertia(r, c);
        rec_[MPCQP_REC_ROT + 3 * r + c] = root_rot_mat(r, c);
      }
    for (int leg = 0; leg < MPCQP_NUM_LEG; ++leg)
      for (int r = 0; r < 3; ++r) pending_feet_[3 * leg + r] = foot_pos(r, leg);
  }

  // ConvexMpc.cpp:145-156; also commits the step's B_d into the horizon (the caller's
  // `B_mat_d_list.block<13,12>(i*13,0) = B_mat_d` line, A1RobotControl.cpp:513).
  void state_space_discretization(double dt) {
    rec_[MPCQP_REC_DT] = dt;
    if (step_ < N) {
      std::memcpy(&rec_[MPCQP_REC_FEET(N) + 12 * step_], pending_feet_, sizeof(pending_feet_));
      ++step_;
    }
  }

  // ConvexMpc.cpp:158-245.  State needs mpc_states (13), mpc_states_d (13N) and contacts[4].
  template <class State>
  void calculate_qp_mats(const State& state) {
    for (int i = step_; i < N; ++i)  // steps never discretized reuse the last feet
      std::memcpy(&rec_[MPCQP_REC_FEET(N) + 12 * i], pending_feet_, sizeof(pending_feet_));
    for (int k = 0; k < MPCQP_STATE_DIM; ++k) rec_[MPCQP_REC_X0 + k] = state.mpc_states[k];
    for (int k = 0; k < MPCQP_STATE_DIM * N; ++k) rec_[MPCQP_REC_XREF + k] = state.mpc_states_d[k];
    for (int l = 0; l < MPCQP_NUM_LEG; ++l) rec_[MPCQP_REC_CONTACTS + l] = state.contacts[l] ? 1.0 : 0.0;
    fz_min = 0;
    fz_max = 180;
    rec_[MPCQP_REC_MU] = mu;
    rec_[MPCQP_REC_FZMIN] = fz_min;
    rec_[MPCQP_REC_FZMAX] = fz_max;
    build_on_device();
    for (int f = 0; f < MPCQP_NUM_LEG * N; ++f) {  // ConvexMpc.cpp:46-58
      double* A = linear_constraints.data();
      A[(size_t)(5 * f + 0) * n + 3 * f + 0] = 1;
      A[(size_t)(5 * f + 1) * n + 3 * f + 0] = 1;
      A[(size_t)(5 * f + 2) * n + 3 * f + 1] = 1;
      A[(size_t)(5 * f + 3) * n + 3 * f + 1] = 1;
      A[(size_t)(5 * f + 4) * n + 3 * f + 2] = 1;
      A[(size_t)(5 * f + 0) * n + 3 * f + 2] = mu;
      A[(size_t)(5 * f + 1) * n + 3 * f + 2] = -mu;
      A[(size_t)(5 * f + 2) * n + 3 * f + 2] = mu;
      A[(size_t)(5 * f + 3) * n + 3 * f + 2] = -mu;
    }
  }

  // the record handed to the solve path (inputs of calculate_qp_mats + the solve)
  const std::vector<double>& record() const { return rec_; }
  mpcqp_handle* handle() const { return h_; }

  double mu, fz_min, fz_max;
  std::vector<double> hessian;             // dense row-major n x n (reference: sparseView of it)
  std::vector<double> gradient;            // n
  std::vector<double> lb, ub;              // m
  std::vector<double> linear_constraints;  // dense row-major m x n

 private:
  void build_on_device();
  void free_device();
  mpcqp_params params_{};
  mpcqp_handle* h_ = nullptr;
  // device staging of build_on_device, allocated on first use and owned by the object
  double *d_rec_ = nullptr, *d_P_ = nullptr, *d_q_ = nullptr, *d_l_ = nullptr, *d_u_ = nullptr;
  std::vector<double> rec_;
  double pending_feet_[12] = {0};
  int step_ = 0;
};

}  // namespace mpcqp_cpp

#include <hip/hip_runtime_api.h>

namespace mpcqp_cpp {

template <int N>
void ConvexMpc<N>::free_device() {
  (void)hipFree(d_rec_);
  (void)hipFree(d_P_);
  (void)hipFree(d_q_);
  (void)hipFree(d_l_);
  (void)hipFree(d_u_);
  d_rec_ = d_P_ = d_q_ = d_l_ = d_u_ = nullptr;
}

template <int N>
void ConvexMpc<N>::build_on_device() {
  auto ok = [&](hipError_t e) {
    if (e != hipSuccess) throw std::runtime_error(std::string("HIP: ") + hipGetErrorString(e));
  };
  if (!d_u_) {  // first call: all five buffers or none (a failed allocation frees the others)
    try {
      ok(hipMalloc(&d_rec_, sizeof(double) * rec_.size()));
      ok(hipMalloc(&d_P_, sizeof(double) * hessian.size()));
      ok(hipMalloc(&d_q_, sizeof(double) * n));
      ok(hipMalloc(&d_l_, sizeof(double) * m));
      ok(hipMalloc(&d_u_, sizeof(double) * m));
    } catch (...) {
      free_device();
      throw;
    }
  }
  ok(hipMemcpy(d_rec_, rec_.data(), sizeof(double) * rec_.size(), hipMemcpyHostToDevice));
  throw_on(mpcqp_build_qp_device(h_, d_rec_, 1, d_P_, d_q_, d_l_, d_u_, nullptr), h_, "mpcqp_build_qp_device");
  ok(hipMemcpy(hessian.data(), d_P_, sizeof(double) * hessian.size(), hipMemcpyDeviceToHost));
  ok(hipMemcpy(gradient.data(), d_q_, sizeof(double) * n, hipMemcpyDeviceToHost));
  ok(hipMemcpy(lb.data(), d_l_, sizeof(double) * m, hipMemcpyDeviceToHost));
  ok(hipMemcpy(ub.data(), d_u_, sizeof(double) * m, hipMemcpyDeviceToHost));
}

// ---------------------------------------------------------------------------------------------
// compute_grf: the MPC branch of A1RobotControl::compute_grf, batched.  Inertia accessor is the
// only difference between A1CtrlStates (a1_trunk_inertia) and Go1CtrlStates (go1_trunk_inertia).
// ---------------------------------------------------------------------------------------------
struct A1InertiaOf {
  template <class S> static const auto& get(const S& s) { return s.a1_trunk_inertia; }
};
struct Go1InertiaOf {
  template <class S> static const auto& get(const S& s) { return s.go1_trunk_inertia; }
};

template <class InertiaOf, int N = 10>
class RobotControlT {
 public:
  template <class VecQ, class VecR>
  RobotControlT(const VecQ& q_weights, const VecR& r_weights, int device = 0) {
    mpcqp_default_params(&params_, N);
    for (int i = 0; i < MPCQP_STATE_DIM; ++i) params_.q_weights[i] = q_weights[i];
    for (int i = 0; i < MPCQP_NUM_DOF; ++i) params_.r_weights[i] = r_weights[i];
    throw_on(mpcqp_create(&params_, device, &h_), nullptr, "mpcqp_create");
  }
  ~RobotControlT() { if (h_) mpcqp_destroy(h_); }
  RobotControlT(const RobotControlT&) = delete;
  RobotControlT& operator=(const RobotControlT&) = delete;

  double mpc_dt = 0.0025;  // A1RobotControl.cpp:462
  // The reference's ROS param `use_sim_time` (read at A1RobotControl.cpp:63): when true, the MPC
  // horizon uses the caller's dt instead of mpc_dt (:464-467).
  bool use_sim_time = false;
  double mu = 0.3, fz_min = 0.0, fz_max = 180.0;

  // A1RobotControl.cpp:452-514: mutates state.mpc_states / mpc_states_d / root_lin_vel_d_world
  // exactly like the reference, and writes the record for the solve.
  template <class State>
  void assemble(State& s, double* rec) const {
    assemble(s, rec, mpc_dt);
  }
  template <class State>
  void assemble(State& s, double* rec, double dt) const {
    std::memset(rec, 0, sizeof(double) * MPCQP_REC_SIZE(N));
    double x0[13];
    for (int k = 0; k < 3; ++k) {
      x0[k] = s.root_euler[k];
      x0[3 + k] = s.root_pos[k];
      x0[6 + k] = s.root_ang_vel[k];
      x0[9 + k] = s.root_lin_vel[k];
    }
    x0[12] = -9.8;
    double vdw[3];
    for (int r = 0; r < 3; ++r) {
      double acc = 0.0;
      for (int c = 0; c < 3; ++c) acc += s.root_rot_mat(r, c) * s.root_lin_vel_d[c];
      vdw[r] = acc;
    }
    for (int k = 0; k < 3; ++k) s.root_lin_vel_d_world[k] = vdw[k];
    for (int k = 0; k < 13; ++k) {
      s.mpc_states[k] = x0[k];
      rec[MPCQP_REC_X0 + k] = x0[k];
    }
    for (int i = 0; i < N; ++i) {
      double xr[13] = {s.root_euler_d[0], s.root_euler_d[1], s.root_euler[2] + s.root_ang_vel_d[2] * dt * (i + 1),
                       s.root_pos[0] + vdw[0] * dt * (i + 1), s.root_pos[1] + vdw[1] * dt * (i + 1),
                       s.root_pos_d[2], s.root_ang_vel_d[0], s.root_ang_vel_d[1], s.root_ang_vel_d[2],
                       vdw[0], vdw[1], 0.0, -9.8};
      for (int k = 0; k < 13; ++k) {
        s.mpc_states_d[13 * i + k] = xr[k];
        rec[MPCQP_REC_XREF + 13 * i + k] = xr[k];
      }
    }
    for (int k = 0; k < 3; ++k) rec[MPCQP_REC_EULER + k] = s.root_euler[k];
    const auto& I = InertiaOf::get(s);
    for (int r = 0; r < 3; ++r)
      for (int c = 0; c < 3; ++c) {
        rec[MPCQP_REC_ROT + 3 * r + c] = s.root_rot_mat(r, c);
        rec[MPCQP_REC_INERTIA + 3 * r + c] = I(r, c);
      }
    rec[MPCQP_REC_MASS] = s.robot_mass;
    rec[MPCQP_REC_MU] = mu;
    rec[MPCQP_REC_FZMIN] = fz_min;
    rec[MPCQP_REC_FZMAX] = fz_max;
    rec[MPCQP_REC_DT] = dt;
    for (int l = 0; l < 4; ++l) rec[MPCQP_REC_CONTACTS + l] = s.contacts[l] ? 1.0 : 0.0;
    for (int i = 0; i < N; ++i)
      for (int l = 0; l < 4; ++l)
        for (int r = 0; r < 3; ++r) rec[MPCQP_REC_FEET(N) + 12 * i + 3 * l + r] = s.foot_pos_abs(r, l);
  }

  // Batched compute_grf: forces[b] receives foot_forces_grf (3x4, row r / leg l at [r*4+l]).
  // `dt` is the caller's thread period; it is the horizon step only when use_sim_time is set.
  template <class State>
  void compute_grf_batch(State* states, int count, double* forces, mpcqp_result* results = nullptr,
                         double dt = 0.0) {
    const double hdt = use_sim_time ? dt : mpc_dt;  // A1RobotControl.cpp:462-467
    recs_.resize((size_t)count * MPCQP_REC_SIZE(N));
    res_.resize(count);
    for (int b = 0; b < count; ++b) assemble(states[b], &recs_[(size_t)b * MPCQP_REC_SIZE(N)], hdt);
    throw_on(mpcqp_solve_batch_host(h_, recs_.data(), count, res_.data(), nullptr), h_, "mpcqp_solve_batch_host");
    for (int b = 0; b < count; ++b) {
      for (int l = 0; l < 4; ++l)
        for (int r = 0; r < 3; ++r) forces[(size_t)b * 12 + r * 4 + l] = res_[b].f_body[3 * l + r];
      if (results) results[b] = res_[b];
    }
  }

  // A1RobotControl::compute_grf(state, dt) — single robot; like the reference, the horizon step is
  // mpc_dt = 0.0025 on hardware and `dt` when use_sim_time is set (:458-467).
  template <class State, class Mat34>
  void compute_grf(State& state, double dt, Mat34& foot_forces_grf) {
    double f[12];
    compute_grf_batch(&state, 1, f, nullptr, dt);
    for (int r = 0; r < 3; ++r)
      for (int l = 0; l < 4; ++l) foot_forces_grf(r, l) = f[r * 4 + l];
  }

  // ---- stance_leg_control_type == 0: single-step QP balance controller -----------------------
  // A1RobotControl ctor constants (:11-15); a caller may edit them before the first call.
  mpcqp_balance_params balance_params = [] {
    mpcqp_balance_params p;
    mpcqp_balance_default_params(&p);
    return p;
  }();

  // A1RobotControl.cpp:321-332 + :377-414 inputs of one robot -> MPCQP_BAL record
  template <class State>
  static void assemble_balance(const State& s, double* rec) {
    std::memset(rec, 0, sizeof(double) * MPCQP_BAL_SIZE);
    for (int k = 0; k < 3; ++k) {
      rec[MPCQP_BAL_POS + k] = s.root_pos[k];
      rec[MPCQP_BAL_POS_D + k] = s.root_pos_d[k];
      rec[MPCQP_BAL_LIN_VEL + k] = s.root_lin_vel[k];
      rec[MPCQP_BAL_LIN_VEL_D + k] = s.root_lin_vel_d[k];
      rec[MPCQP_BAL_ANG_VEL + k] = s.root_ang_vel[k];
      rec[MPCQP_BAL_ANG_VEL_D + k] = s.root_ang_vel_d[k];
      rec[MPCQP_BAL_EULER + k] = s.root_euler[k];
      rec[MPCQP_BAL_EULER_D + k] = s.root_euler_d[k];
      rec[MPCQP_BAL_KP_LIN + k] = s.kp_linear[k];
      rec[MPCQP_BAL_KD_LIN + k] = s.kd_linear[k];
      rec[MPCQP_BAL_KP_ANG + k] = s.kp_angular[k];
      rec[MPCQP_BAL_KD_ANG + k] = s.kd_angular[k];
    }
    for (int r = 0; r < 3; ++r)
      for (int c = 0; c < 3; ++c) {
        rec[MPCQP_BAL_ROT + 3 * r + c] = s.root_rot_mat(r, c);
        rec[MPCQP_BAL_ROT_Z + 3 * r + c] = s.root_rot_mat_z(r, c);
      }
    rec[MPCQP_BAL_MASS] = s.robot_mass;
    for (int l = 0; l < 4; ++l) {
      for (int r = 0; r < 3; ++r) rec[MPCQP_BAL_FEET + 3 * l + r] = s.foot_pos_abs(r, l);
      rec[MPCQP_BAL_CONTACTS + l] = s.contacts[l] ? 1.0 : 0.0;
    }
  }

  // Batched QP branch of compute_grf: forces[b] = foot_forces_grf (row r / leg l at [r*4+l]).
  template <class State>
  void compute_grf_qp_batch(const State* states, int count, double* forces, mpcqp_result* results = nullptr) {
    bal_recs_.resize((size_t)count * MPCQP_BAL_SIZE);
    res_.resize(count);
    for (int b = 0; b < count; ++b) assemble_balance(states[b], &bal_recs_[(size_t)b * MPCQP_BAL_SIZE]);
    throw_on(mpcqp_balance_solve_host(h_, &balance_params, bal_recs_.data(), count, res_.data()), h_,
             "mpcqp_balance_solve_host");
    for (int b = 0; b < count; ++b) {
      for (int l = 0; l < 4; ++l)
        for (int r = 0; r < 3; ++r) forces[(size_t)b * 12 + r * 4 + l] = res_[b].f_body[3 * l + r];
      if (results) results[b] = res_[b];
    }
  }

  // A1RobotControl::compute_grf with state.stance_leg_control_type == 0 (:377-444)
  template <class State, class Mat34>
  void compute_grf_qp(const State& state, Mat34& foot_forces_grf) {
    double f[12];
    compute_grf_qp_batch(&state, 1, f);
    for (int r = 0; r < 3; ++r)
      for (int l = 0; l < 4; ++l) foot_forces_grf(r, l) = f[r * 4 + l];
  }

  mpcqp_handle* handle() const { return h_; }

 private:
  mpcqp_params params_{};
  mpcqp_handle* h_ = nullptr;
  std::vector<double> recs_;
  std::vector<double> bal_recs_;
  std::vector<mpcqp_result> res_;
};

using A1RobotControl = RobotControlT<A1InertiaOf>;
using Go1RobotControl = RobotControlT<Go1InertiaOf>;

}  // namespace mpcqp_cpp
