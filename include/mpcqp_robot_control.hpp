// mpcqp_robot_control.hpp — header-only C++ drop-in for the reference's GRF call surface,
// implemented over the C ABI in mpcqp.h (link with libmpcqp.so).
//
//   mpcqp_cpp::ConvexMpc<N>          ≙ class ConvexMpc (src/a1_cpp/src/ConvexMpc.h:22-94)
//   mpcqp_cpp::A1RobotControl        ≙ A1RobotControl::compute_grf (src/a1_cpp/src/A1RobotControl.h:44,
//                                       MPC branch A1RobotControl.cpp:446-562, QP branch :377-444)
//   mpcqp_cpp::Go1RobotControl       ≙ the declared-but-undefined Go1 hook
//                                       (src/go1_rl_ctrl_cpp/src/Go1RLController.hpp:38-40)
//
// Eigen-agnostic: state types are templates; anything with operator[] for vectors,
// operator()(r,c) for matrices and a bool contacts[4] works (Eigen::Vector3d / Matrix3d /
// Matrix<double,3,4> included), so A1CtrlStates / Go1CtrlStates plug in unchanged.  The matrices
// the shim owns are mpcqp_cpp::Mat<R, C>, which speaks the Eigen spellings the reference's caller
// uses (m(r, c), m.block<R, C>(i, j) = other) and converts implicitly to any matrix type with
// operator()(r, c), so `state.foot_forces_grf = ctrl.compute_grf(state, dt);` compiles with an
// Eigen::Matrix<double, 3, 4> on the left.
#pragma once

#include <hip/hip_runtime_api.h>

#include <cmath>
#include <cstring>
#include <functional>
#include <memory>
#include <mutex>
#include <stdexcept>
#include <string>
#include <type_traits>
#include <utility>
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
inline void hip_ok(hipError_t e, const char* what) {
  if (e != hipSuccess) throw std::runtime_error(std::string(what) + ": " + hipGetErrorString(e));
}

// Makes `device` current for a scope and restores the caller's current device (device
// buffers of a handle must be allocated on the handle's device, whatever the caller's selection).
class DeviceScope {
 public:
  explicit DeviceScope(int device) {
    if (hipGetDevice(&prev_) != hipSuccess) prev_ = -1;
    hip_ok(hipSetDevice(device), "hipSetDevice");
  }
  ~DeviceScope() {
    if (prev_ >= 0) (void)hipSetDevice(prev_);
  }
  DeviceScope(const DeviceScope&) = delete;
  DeviceScope& operator=(const DeviceScope&) = delete;

 private:
  int prev_ = -1;
};

// ---------------------------------------------------------------------------------------------
// Mat<R, C>: fixed-size row-major binary64 matrix with the Eigen member spellings of the caller.
// ---------------------------------------------------------------------------------------------
template <class M, class = void>
struct is_matrix_like : std::false_type {};
template <class M>
struct is_matrix_like<M, std::void_t<decltype(std::declval<M&>()(0, 0) = 0.0)>> : std::true_type {};

template <int R, int C>
struct Mat {
  double a[R * C] = {};
  static constexpr int rows() { return R; }
  static constexpr int cols() { return C; }
  double& operator()(int r, int c) { return a[r * C + c]; }
  const double& operator()(int r, int c) const { return a[r * C + c]; }
  double* data() { return a; }
  const double* data() const { return a; }
  void setZero() { std::memset(a, 0, sizeof(a)); }
  static Mat Zero() { return Mat(); }

  template <int BR, int BC>
  struct Block {  // Eigen's m.block<BR, BC>(r0, c0): read, write, assign from any matrix-like
    Mat* m;
    int r0, c0;
    double& operator()(int r, int c) { return (*m)(r0 + r, c0 + c); }
    template <class O>
    Block& operator=(const O& o) {
      for (int r = 0; r < BR; ++r)
        for (int c = 0; c < BC; ++c) (*m)(r0 + r, c0 + c) = o(r, c);
      return *this;
    }
    operator Mat<BR, BC>() const {
      Mat<BR, BC> o;
      for (int r = 0; r < BR; ++r)
        for (int c = 0; c < BC; ++c) o(r, c) = (*m)(r0 + r, c0 + c);
      return o;
    }
  };
  template <int BR, int BC>
  Block<BR, BC> block(int r0, int c0) {
    static_assert(BR <= R && BC <= C, "block larger than the matrix");
    if (r0 < 0 || c0 < 0 || r0 + BR > R || c0 + BC > C) throw std::out_of_range("Mat::block");
    return Block<BR, BC>{this, r0, c0};
  }
  template <int BR, int BC>
  Mat<BR, BC> block(int r0, int c0) const {
    return const_cast<Mat*>(this)->template block<BR, BC>(r0, c0);
  }
  // assignment from / conversion to any other matrix-like type (e.g. Eigen::Matrix<double, R, C>)
  template <class O, class = std::enable_if_t<is_matrix_like<O>::value && !std::is_same<O, Mat>::value>>
  Mat& operator=(const O& o) {
    for (int r = 0; r < R; ++r)
      for (int c = 0; c < C; ++c) (*this)(r, c) = o(r, c);
    return *this;
  }
  template <class O, class = std::enable_if_t<is_matrix_like<O>::value && !std::is_same<O, Mat>::value &&
                                              std::is_default_constructible<O>::value>>
  operator O() const {
    O o;
    for (int r = 0; r < R; ++r)
      for (int c = 0; c < C; ++c) o(r, c) = (*this)(r, c);
    return o;
  }
};
using Matrix34 = Mat<3, MPCQP_NUM_LEG>;

// Heap-backed row-major binary64 matrix for the large formulation members (B_qp is 13N x 12N).
struct DMat {
  int r = 0, c = 0;
  std::vector<double> a;
  DMat() = default;
  DMat(int rows_, int cols_) : r(rows_), c(cols_), a((size_t)rows_ * cols_, 0.0) {}
  int rows() const { return r; }
  int cols() const { return c; }
  double& operator()(int i, int j) { return a[(size_t)i * c + j]; }
  const double& operator()(int i, int j) const { return a[(size_t)i * c + j]; }
  double* data() { return a.data(); }
  const double* data() const { return a.data(); }
};

// A public data member of the reference's ConvexMpc whose value is produced on first read after
// calculate_qp_mats (ConvexMpc.h:77-92): the shim computes hessian / gradient on the device and
// A_qp / B_qp / linear_constraints on the host only when the caller actually reads them, so a tick
// that only needs the solve moves no dense matrix across PCIe.  Reads look like the member's
// (v[i], v.size(), range-for, v.data(), implicit conversion to the value type).
template <class T>
class Lazy {
 public:
  using value_type = T;
  const T& get() const {
    if (!valid_) {
      if (!fill_) throw std::logic_error("ConvexMpc: member read before calculate_qp_mats");
      fill_(val_);
      valid_ = true;
    }
    return val_;
  }
  operator const T&() const { return get(); }
  // (member templates: each exists only for value types that have the operation)
  template <class U = T>
  auto operator[](size_t i) const -> decltype(std::declval<const U&>()[i]) { return get()[i]; }
  template <class U = T>
  auto operator()(int i, int j) const -> decltype(std::declval<const U&>()(i, j)) { return get()(i, j); }
  template <class U = T>
  auto size() const -> decltype(std::declval<const U&>().size()) { return get().size(); }
  const double* data() const { return get().data(); }
  template <class U = T>
  auto rows() const -> decltype(std::declval<const U&>().rows()) { return get().rows(); }
  template <class U = T>
  auto cols() const -> decltype(std::declval<const U&>().cols()) { return get().cols(); }
  template <class U = T>
  auto begin() const -> decltype(std::declval<const U&>().begin()) { return get().begin(); }
  template <class U = T>
  auto end() const -> decltype(std::declval<const U&>().end()) { return get().end(); }
  bool computed() const { return valid_; }  // tests: has this member been materialised?
  // (internal) the producer for the current formulation
  template <class F>
  void reset(T init, F&& fill) {
    val_ = std::move(init);
    valid_ = false;
    fill_ = std::forward<F>(fill);
  }

 private:
  mutable T val_{};
  mutable bool valid_ = false;
  std::function<void(T&)> fill_;
};

namespace detail {

// calculate_B_mat_c + state_space_discretization on the host (ConvexMpc.cpp:132-156, Utils.cpp:
// 35-41): B_d = B_c dt with B_c rows 6-8 = I_w^-1 [r_l]x, rows 9-11 = I / m (I_w = R I_b R',
// Eigen's cofactor 3x3 inverse).  The device recomputes the same matrices from the same inputs.
inline void iw_and_inverse(const double R[9], const double Ib[9], double Iw[9], double Iwinv[9]) {
  double t[9];
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) {
      double s = 0.0;
      for (int k = 0; k < 3; ++k) s += R[3 * i + k] * Ib[3 * k + j];
      t[3 * i + j] = s;
    }
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) {
      double s = 0.0;
      for (int k = 0; k < 3; ++k) s += t[3 * i + k] * R[3 * j + k];
      Iw[3 * i + j] = s;
    }
  auto cof = [&](int i, int j) {
    const int i1 = (i + 1) % 3, i2 = (i + 2) % 3, j1 = (j + 1) % 3, j2 = (j + 2) % 3;
    return Iw[3 * i1 + j1] * Iw[3 * i2 + j2] - Iw[3 * i1 + j2] * Iw[3 * i2 + j1];
  };
  const double invdet = 1.0 / ((cof(0, 0) * Iw[0] + cof(1, 0) * Iw[3]) + cof(2, 0) * Iw[6]);
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) Iwinv[3 * j + i] = cof(i, j) * invdet;
}
inline void b_mat_c(double mass, const double Iwinv[9], const double feet[12], Mat<13, 12>& B) {
  B.setZero();
  for (int l = 0; l < MPCQP_NUM_LEG; ++l) {
    const double* r = feet + 3 * l;
    const double sk[9] = {0.0, -r[2], r[1], r[2], 0.0, -r[0], -r[1], r[0], 0.0};
    for (int i = 0; i < 3; ++i)
      for (int j = 0; j < 3; ++j) {
        double s = 0.0;
        for (int k = 0; k < 3; ++k) s += Iwinv[3 * i + k] * sk[3 * k + j];
        B(6 + i, 3 * l + j) = s;
      }
    for (int i = 0; i < 3; ++i) B(9 + i, 3 * l + i) = 1.0 / mass;
  }
}

// One formulation handle + device staging per (device, weights), shared by every ConvexMpc
// object: the reference constructs ConvexMpc on every tick (A1RobotControl.cpp:447), which must
// not mean a handle and five device allocations per tick.  Entries live for the process (they are
// intentionally never destroyed: no HIP call from static destructors after runtime teardown).
template <int N>
struct BuildSlot {
  std::mutex mu;
  int device = 0;
  double q[MPCQP_STATE_DIM], r[MPCQP_NUM_DOF];
  mpcqp_handle* h = nullptr;
  double *d_rec = nullptr, *d_P = nullptr, *d_q = nullptr, *d_l = nullptr, *d_u = nullptr;
};
template <int N>
inline BuildSlot<N>* build_slot(int device, const double* q, const double* r) {
  static std::mutex pool_mu;
  static std::vector<BuildSlot<N>*> pool;
  std::lock_guard<std::mutex> lk(pool_mu);
  for (BuildSlot<N>* s : pool)
    if (s->device == device && !std::memcmp(s->q, q, sizeof(s->q)) && !std::memcmp(s->r, r, sizeof(s->r))) return s;
  std::unique_ptr<BuildSlot<N>> s(new BuildSlot<N>());
  s->device = device;
  std::memcpy(s->q, q, sizeof(s->q));
  std::memcpy(s->r, r, sizeof(s->r));
  mpcqp_params p;
  mpcqp_default_params(&p, N);
  std::memcpy(p.q_weights, q, sizeof(s->q));
  std::memcpy(p.r_weights, r, sizeof(s->r));
  throw_on(mpcqp_create(&p, device, &s->h), nullptr, "mpcqp_create");
  try {
    DeviceScope ds(device);
    const int n = MPCQP_NUM_DOF * N, m = MPCQP_CONSTRAINT_DIM * N;
    hip_ok(hipMalloc(&s->d_rec, sizeof(double) * MPCQP_REC_SIZE(N)), "hipMalloc");
    hip_ok(hipMalloc(&s->d_P, sizeof(double) * n * n), "hipMalloc");
    hip_ok(hipMalloc(&s->d_q, sizeof(double) * n), "hipMalloc");
    hip_ok(hipMalloc(&s->d_l, sizeof(double) * m), "hipMalloc");
    hip_ok(hipMalloc(&s->d_u, sizeof(double) * m), "hipMalloc");
  } catch (...) {
    DeviceScope ds(device);
    for (double* d : {s->d_rec, s->d_P, s->d_q, s->d_l, s->d_u}) (void)hipFree(d);
    mpcqp_destroy(s->h);
    throw;
  }
  pool.push_back(s.get());
  return s.release();
}

}  // namespace detail

// ---------------------------------------------------------------------------------------------
// ConvexMpc: same methods, call order and public members as the reference (ConvexMpc.h:22-94).
// calculate_qp_mats() reads B_mat_d_list (what the caller stored, A1RobotControl.cpp:513) and
// runs the formulation on the GPU (mpcqp_build_qp_device) to fill hessian / gradient / lb / ub.
// ---------------------------------------------------------------------------------------------
template <int N = 10>
class ConvexMpc {
 public:
  static constexpr int n = MPCQP_NUM_DOF * N;
  static constexpr int m = MPCQP_CONSTRAINT_DIM * N;

  template <class VecQ, class VecR>
  ConvexMpc(const VecQ& q_weights_, const VecR& r_weights_, int device = 0)
      : mu(0.3), fz_min(0), fz_max(0), device_(device) {
    double q[MPCQP_STATE_DIM], r[MPCQP_NUM_DOF];
    for (int i = 0; i < MPCQP_STATE_DIM; ++i) q[i] = q_weights_[i];
    for (int i = 0; i < MPCQP_NUM_DOF; ++i) r[i] = r_weights_[i];
    slot_ = detail::build_slot<N>(device, q, r);
    reset();
  }
  ConvexMpc(const ConvexMpc&) = delete;
  ConvexMpc& operator=(const ConvexMpc&) = delete;

  void reset() {  // ConvexMpc.cpp:70-108
    rec_.assign(MPCQP_REC_SIZE(N), 0.0);
    step_ = 0;
    have_body_ = false;
    A_mat_c.setZero();
    B_mat_c.setZero();
    A_mat_d.setZero();
    B_mat_d.setZero();
    B_mat_d_list.setZero();
    lb.assign(m, 0.0);
    ub.assign(m, 0.0);
    const auto zeros = [](size_t k) { return [k](std::vector<double>& v) { v.assign(k, 0.0); }; };
    hessian.reset({}, zeros((size_t)n * n));  // the reference's zero-filled members (:70-108)
    gradient.reset({}, zeros(n));
    linear_constraints.reset({}, zeros((size_t)m * n));
    A_qp.reset(DMat(), [](DMat& d) { d = DMat(13 * N, 13); });
    B_qp.reset(DMat(), [](DMat& d) { d = DMat(13 * N, MPCQP_NUM_DOF * N); });
  }

  template <class Vec3>
  void calculate_A_mat_c(const Vec3& root_euler) {  // ConvexMpc.cpp:110-130 (yaw only)
    for (int k = 0; k < 3; ++k) rec_[MPCQP_REC_EULER + k] = root_euler[k];
    const double cy = std::cos(root_euler[2]), sy = std::sin(root_euler[2]);
    A_mat_c.setZero();
    A_mat_c(0, 6) = cy;
    A_mat_c(0, 7) = sy;
    A_mat_c(1, 6) = -sy;
    A_mat_c(1, 7) = cy;
    A_mat_c(2, 8) = 1.0;
    for (int i = 0; i < 3; ++i) A_mat_c(3 + i, 9 + i) = 1.0;
    A_mat_c(11, 12) = 1.0;
  }

  // ConvexMpc.cpp:132-143.  The record holds ONE mass / inertia / rotation for the horizon (what
  // both reference callers pass); feet may differ per horizon step.
  template <class Mat3a, class Mat3b, class Mat34>
  void calculate_B_mat_c(double robot_mass, const Mat3a& trunk_inertia, const Mat3b& root_rot_mat,
                         const Mat34& foot_pos) {
    double R[9], Ib[9];
    for (int r = 0; r < 3; ++r)
      for (int c = 0; c < 3; ++c) {
        Ib[3 * r + c] = trunk_inertia(r, c);
        R[3 * r + c] = root_rot_mat(r, c);
      }
    if (have_body_ && (robot_mass != rec_[MPCQP_REC_MASS] || std::memcmp(Ib, &rec_[MPCQP_REC_INERTIA], sizeof(Ib)) ||
                       std::memcmp(R, &rec_[MPCQP_REC_ROT], sizeof(R))))
      throw std::invalid_argument("ConvexMpc: mass, inertia and rotation must be the same for every horizon step");
    have_body_ = true;
    rec_[MPCQP_REC_MASS] = robot_mass;
    std::memcpy(&rec_[MPCQP_REC_INERTIA], Ib, sizeof(Ib));
    std::memcpy(&rec_[MPCQP_REC_ROT], R, sizeof(R));
    detail::iw_and_inverse(R, Ib, Iw_, Iwinv_);
    for (int leg = 0; leg < MPCQP_NUM_LEG; ++leg)
      for (int r = 0; r < 3; ++r) pending_feet_[3 * leg + r] = foot_pos(r, leg);
    detail::b_mat_c(robot_mass, Iwinv_, pending_feet_, B_mat_c);
  }

  // ConvexMpc.cpp:145-156 (forward Euler).  Remembers the feet behind this call's B_mat_d so that
  // calculate_qp_mats can recognise the block the caller stores from it.
  void state_space_discretization(double dt) {
    rec_[MPCQP_REC_DT] = dt;
    for (int i = 0; i < 13; ++i)
      for (int j = 0; j < 13; ++j) A_mat_d(i, j) = (i == j ? 1.0 : 0.0) + A_mat_c(i, j) * dt;
    for (int i = 0; i < 13; ++i)
      for (int j = 0; j < 12; ++j) B_mat_d(i, j) = B_mat_c(i, j) * dt;
    if (step_ < N) std::memcpy(seen_feet_[step_], pending_feet_, sizeof(pending_feet_));
    if (step_ < N) std::memcpy(seen_bd_[step_].a, B_mat_d.a, sizeof(B_mat_d.a));
    ++step_;
  }

  // ConvexMpc.cpp:158-245.  State needs mpc_states (13), mpc_states_d (13N) and contacts[4].  The
  // record for the solve is complete on return and lb / ub are filled; hessian and gradient (device
  // formulation, mpcqp_build_qp_device), A_qp / B_qp and linear_constraints (host) are produced
  // when first read.
  template <class State>
  void calculate_qp_mats(const State& state) {
    for (int i = 0; i < N; ++i) feet_of_block(i, &rec_[MPCQP_REC_FEET(N) + 12 * i]);
    for (int k = 0; k < MPCQP_STATE_DIM; ++k) rec_[MPCQP_REC_X0 + k] = state.mpc_states[k];
    for (int k = 0; k < MPCQP_STATE_DIM * N; ++k) rec_[MPCQP_REC_XREF + k] = state.mpc_states_d[k];
    for (int l = 0; l < MPCQP_NUM_LEG; ++l) rec_[MPCQP_REC_CONTACTS + l] = state.contacts[l] ? 1.0 : 0.0;
    fz_min = 0;
    fz_max = 180;
    rec_[MPCQP_REC_MU] = mu;
    rec_[MPCQP_REC_FZMIN] = fz_min;
    rec_[MPCQP_REC_FZMAX] = fz_max;
    for (int i = 0; i < N; ++i)  // ConvexMpc.cpp:223-245 (the current contacts over the horizon)
      for (int l = 0; l < MPCQP_NUM_LEG; ++l) {
        const double c = rec_[MPCQP_REC_CONTACTS + l];
        double* lo = &lb[MPCQP_CONSTRAINT_DIM * i + 5 * l];
        double* up = &ub[MPCQP_CONSTRAINT_DIM * i + 5 * l];
        lo[0] = 0; lo[1] = -MPCQP_OSQP_INFTY; lo[2] = 0; lo[3] = -MPCQP_OSQP_INFTY; lo[4] = fz_min * c;
        up[0] = MPCQP_OSQP_INFTY; up[1] = 0; up[2] = MPCQP_OSQP_INFTY; up[3] = 0; up[4] = fz_max * c;
      }
    // one device round trip fills both device members, whichever is read first
    auto dev = std::make_shared<std::vector<double>>();
    auto fetch = [this, dev, rec = rec_](int which, std::vector<double>& out) {
      if (dev->empty()) {  // (the record as of this call: later setters do not leak into it)
        std::vector<double> H((size_t)n * n), g(n);
        build_on_device(rec, H.data(), g.data());
        dev->swap(H);
        dev->insert(dev->end(), g.begin(), g.end());
      }
      if (which == 0) out.assign(dev->begin(), dev->begin() + (size_t)n * n);
      else out.assign(dev->begin() + (size_t)n * n, dev->end());
    };
    hessian.reset({}, [fetch](std::vector<double>& v) { fetch(0, v); });
    gradient.reset({}, [fetch](std::vector<double>& v) { fetch(1, v); });
    const double mu_ = mu;
    linear_constraints.reset({}, [mu_](std::vector<double>& A) {  // ConvexMpc.cpp:46-58, dense
      A.assign((size_t)m * n, 0.0);
      for (int f = 0; f < MPCQP_NUM_LEG * N; ++f) {
        A[(size_t)(5 * f + 0) * n + 3 * f + 0] = 1;
        A[(size_t)(5 * f + 1) * n + 3 * f + 0] = 1;
        A[(size_t)(5 * f + 2) * n + 3 * f + 1] = 1;
        A[(size_t)(5 * f + 3) * n + 3 * f + 1] = 1;
        A[(size_t)(5 * f + 4) * n + 3 * f + 2] = 1;
        A[(size_t)(5 * f + 0) * n + 3 * f + 2] = mu_;
        A[(size_t)(5 * f + 1) * n + 3 * f + 2] = -mu_;
        A[(size_t)(5 * f + 2) * n + 3 * f + 2] = mu_;
        A[(size_t)(5 * f + 3) * n + 3 * f + 2] = -mu_;
      }
    });
    // A_qp / B_qp by the reference's recurrence (ConvexMpc.cpp:184-202), from A_mat_d and the
    // B_mat_d_list the caller stored
    const Mat<13, 13> Ad = A_mat_d;
    const Mat<13 * N, 12> Bl = B_mat_d_list;
    auto aqp = std::make_shared<DMat>();
    auto make_aqp = [aqp, Ad]() -> const DMat& {
      if (aqp->rows() == 0) {
        *aqp = DMat(13 * N, 13);
        for (int i = 0; i < N; ++i)
          for (int r = 0; r < 13; ++r)
            for (int c = 0; c < 13; ++c) {
              if (i == 0) { (*aqp)(r, c) = Ad(r, c); continue; }
              double s = 0.0;
              for (int k = 0; k < 13; ++k) s += (*aqp)(13 * (i - 1) + r, k) * Ad(k, c);
              (*aqp)(13 * i + r, c) = s;
            }
      }
      return *aqp;
    };
    A_qp.reset(DMat(), [make_aqp](DMat& d) { d = make_aqp(); });
    B_qp.reset(DMat(), [make_aqp, Bl](DMat& d) {
      const DMat& Aq = make_aqp();
      d = DMat(13 * N, MPCQP_NUM_DOF * N);
      for (int i = 0; i < N; ++i)
        for (int j = 0; j <= i; ++j)
          for (int r = 0; r < 13; ++r)
            for (int c = 0; c < 12; ++c) {
              double s;
              if (i == j) {
                s = Bl(13 * j + r, c);
              } else {
                s = 0.0;
                for (int k = 0; k < 13; ++k) s += Aq(13 * (i - j - 1) + r, k) * Bl(13 * j + k, c);
              }
              d(13 * i + r, 12 * j + c) = s;
            }
    });
  }

  // the record handed to the solve path (inputs of calculate_qp_mats + the solve)
  const std::vector<double>& record() const { return rec_; }
  mpcqp_handle* handle() const { return slot_->h; }
  int device() const { return device_; }
  // device staging of the formulation (tests check it lives on device())
  const double* staging() const { return slot_->d_P; }

  double mu, fz_min, fz_max;
  Mat<13, 13> A_mat_c, A_mat_d;
  Mat<13, 12> B_mat_c, B_mat_d;
  Mat<13 * N, 12> B_mat_d_list;                  // block i: B_d of horizon step i (written by the caller)
  Lazy<DMat> A_qp;                               // 13N x 13 (ConvexMpc.h:77)
  Lazy<DMat> B_qp;                               // 13N x 12N (ConvexMpc.h:78)
  Lazy<std::vector<double>> hessian;             // dense row-major n x n (reference: sparseView of it)
  Lazy<std::vector<double>> gradient;            // n
  std::vector<double> lb, ub;                    // m
  Lazy<std::vector<double>> linear_constraints;  // dense row-major m x n

 private:
  // Feet of horizon step i from B_mat_d_list block i.  The block the reference's loop stores is the
  // B_mat_d of one of this object's discretizations: its feet are taken as they were given.  Any
  // other block with the physical structure (rows 0-5, 12 zero; rows 9-11 dt/m I; rows 6-8
  // I_w^-1 [r]x dt) gives its feet back through I_w; anything else is rejected.
  void feet_of_block(int i, double* feet) const {
    const Mat<13, 12> blk = B_mat_d_list.template block<13, 12>(13 * i, 0);
    for (int s = 0; s < step_ && s < N; ++s)
      if (!std::memcmp(blk.a, seen_bd_[s].a, sizeof(blk.a))) {
        std::memcpy(feet, seen_feet_[s], sizeof(seen_feet_[s]));
        return;
      }
    const double dt = rec_[MPCQP_REC_DT], dtm = (1.0 / rec_[MPCQP_REC_MASS]) * dt;
    bool ok = have_body_ && dt > 0;
    for (int r = 0; r < 13 && ok; ++r)
      for (int c = 0; c < 12 && ok; ++c) {
        const double v = blk(r, c);
        if (r < 6 || r == 12) ok = v == 0.0;
        else if (r >= 9) ok = std::fabs(v - (c % 3 == r - 9 ? dtm : 0.0)) <= 1e-12 * dtm;
      }
    if (!ok)
      throw std::invalid_argument("ConvexMpc: B_mat_d_list block " + std::to_string(i) +
                                  " is not a single-rigid-body B_d of this robot");
    for (int l = 0; l < MPCQP_NUM_LEG; ++l) {  // [r]x = I_w B_d[6:9, 3l:3l+3] / dt
      double S[9];
      for (int a = 0; a < 3; ++a)
        for (int b = 0; b < 3; ++b) {
          double s = 0.0;
          for (int k = 0; k < 3; ++k) s += Iw_[3 * a + k] * blk(6 + k, 3 * l + b);
          S[3 * a + b] = s / dt;
        }
      feet[3 * l + 0] = 0.5 * (S[7] - S[5]);
      feet[3 * l + 1] = 0.5 * (S[2] - S[6]);
      feet[3 * l + 2] = 0.5 * (S[3] - S[1]);
    }
    // rows 6-8 must be exactly what those feet give with this robot's I_w (a block built with
    // another rotation / inertia, or not skew-symmetric through I_w, is rejected, not re-read)
    Mat<13, 12> Bc;
    detail::b_mat_c(rec_[MPCQP_REC_MASS], Iwinv_, feet, Bc);
    double scale = 0.0;
    for (int r = 6; r < 9; ++r)
      for (int c = 0; c < 12; ++c) scale = std::fmax(scale, std::fabs(blk(r, c)));
    for (int r = 6; r < 9; ++r)
      for (int c = 0; c < 12; ++c)
        if (std::fabs(Bc(r, c) * dt - blk(r, c)) > 1e-9 * scale + 1e-300)
          throw std::invalid_argument("ConvexMpc: B_mat_d_list block " + std::to_string(i) +
                                      " rows 6-8 are not I_w^-1 [r]x dt of this robot for any feet r");
  }
  void build_on_device(const std::vector<double>& rec, double* H, double* g) const;

  int device_ = 0;
  detail::BuildSlot<N>* slot_ = nullptr;
  std::vector<double> rec_;
  double pending_feet_[12] = {0};
  double seen_feet_[N][12] = {};
  Mat<13, 12> seen_bd_[N];
  double Iw_[9] = {0}, Iwinv_[9] = {0};
  bool have_body_ = false;
  int step_ = 0;
};

// The formulation of one record on the device (shared staging of the weights' BuildSlot, held for
// the round trip): H (n x n) and g (n) to the host.
template <int N>
void ConvexMpc<N>::build_on_device(const std::vector<double>& rec, double* H, double* g) const {
  detail::BuildSlot<N>& s = *slot_;
  std::lock_guard<std::mutex> lk(s.mu);
  DeviceScope ds(s.device);
  hip_ok(hipMemcpy(s.d_rec, rec.data(), sizeof(double) * rec.size(), hipMemcpyHostToDevice), "hipMemcpy");
  throw_on(mpcqp_build_qp_device(s.h, s.d_rec, 1, s.d_P, s.d_q, s.d_l, s.d_u, nullptr), s.h, "mpcqp_build_qp_device");
  hip_ok(hipMemcpy(H, s.d_P, sizeof(double) * n * n, hipMemcpyDeviceToHost), "hipMemcpy");
  hip_ok(hipMemcpy(g, s.d_q, sizeof(double) * n, hipMemcpyDeviceToHost), "hipMemcpy");
}

// ---------------------------------------------------------------------------------------------
// compute_grf: the MPC branch of A1RobotControl::compute_grf, batched.  Like the reference's
// controller (A1RobotControl.h:67 member OsqpEigen::Solver, setWarmStart(true) at
// A1RobotControl.cpp:524) it owns a persistent solver: one device warm-start slot per robot, the
// first tick an initSolver, later ticks update + warm solve (mpcqp_solve_batch_warm_host).  Inertia
// accessor is the only difference between A1CtrlStates (a1_trunk_inertia) and Go1CtrlStates
// (go1_trunk_inertia).
// ---------------------------------------------------------------------------------------------
struct A1InertiaOf {
  template <class S> static const auto& get(const S& s) { return s.a1_trunk_inertia; }
};
struct Go1InertiaOf {
  template <class S> static const auto& get(const S& s) { return s.go1_trunk_inertia; }
};

// state.stance_leg_control_type (A1CtrlStates.h / Go1CtrlStates.hpp: 0 = QP balance, 1 = MPC), or
// 1 for a state type without the field (an MPC-only caller)
template <class S, class = void>
struct has_control_type : std::false_type {};
template <class S>
struct has_control_type<S, std::void_t<decltype(std::declval<const S&>().stance_leg_control_type)>>
    : std::true_type {};
template <class S>
int control_type_of(const S& s) {
  if constexpr (has_control_type<S>::value) return (int)s.stance_leg_control_type;
  else return 1;
}

// state types carrying the terrain-adaptation fields (A1CtrlStates.h:332, :370; Go1CtrlStates.hpp:337,
// :375): use_terrain_adapt, terrain_pitch_angle, foot_pos_recent_contact (3x4)
template <class S, class = void>
struct has_terrain_fields : std::false_type {};
template <class S>
struct has_terrain_fields<S, std::void_t<decltype(std::declval<const S&>().use_terrain_adapt),
                                         decltype(std::declval<S&>().terrain_pitch_angle = 0.0),
                                         decltype(std::declval<const S&>().foot_pos_recent_contact(2, 0) + 0.0)>>
    : std::true_type {};

template <class InertiaOf, int N = 10>
class RobotControlT {
 public:
  template <class VecQ, class VecR>
  RobotControlT(const VecQ& q_weights, const VecR& r_weights, int device = 0) : device_(device) {
    mpcqp_default_params(&params_, N);
    for (int i = 0; i < MPCQP_STATE_DIM; ++i) params_.q_weights[i] = q_weights[i];
    for (int i = 0; i < MPCQP_NUM_DOF; ++i) params_.r_weights[i] = r_weights[i];
    throw_on(mpcqp_create(&params_, device, &h_), nullptr, "mpcqp_create");
  }
  ~RobotControlT() {
    if (d_state_ || d_gather_) {
      DeviceScope ds(device_);
      (void)hipFree(d_state_);
      (void)hipFree(d_gather_);
      (void)hipFree(d_idx_);
    }
    if (h_) mpcqp_destroy(h_);
  }
  RobotControlT(const RobotControlT&) = delete;
  RobotControlT& operator=(const RobotControlT&) = delete;

  double mpc_dt = 0.0025;  // A1RobotControl.cpp:462
  // The reference's ROS param `use_sim_time` (read at A1RobotControl.cpp:63): when true, the MPC
  // horizon uses the caller's dt instead of mpc_dt (:464-467).
  bool use_sim_time = false;
  // Persistent warm-started solver per robot (production, A1RobotControl.cpp:524).  false: every
  // call is a fresh cold solve (test_mpc.cpp:131-133).
  bool warm_start = true;
  double mu = 0.3, fz_min = 0.0, fz_max = 180.0;

  // Terrain adaptation (A1RobotControl.cpp:334-376), on MPC ticks only (:335).  When this hook is
  // set, compute_grf / compute_grf_batch apply the reference's state mutation to each MPC robot b
  // before its record is assembled, so x_ref carries the adapted pitch (:475-476):
  //   terrain_angle = root_pos[2] > 0.1 ? terrain_angle_of(b) : 0, clamped to [-0.5, 0.5];
  //   F_R_diff = z(FL) + z(FR) - z(RL) - z(RR) of foot_pos_recent_contact;
  //   if use_terrain_adapt: root_euler_d[1] = F_R_diff > 0.05 ? -terrain_angle : terrain_angle;
  //   terrain_pitch_angle = terrain_angle.
  // The hook returns the reference's filtered dihedral angle,
  //   terrain_angle_filter.CalculateAverage(Utils::cal_dihedral_angle(flat_ground_coef,
  //                                                                 compute_walking_surface(state)))
  // and is called exactly where the reference updates that filter (only when root_pos[2] > 0.1), so
  // the caller's filter sees the same sequence of samples; the plane fit and the filter stay with the
  // caller.  Unset: no terrain adaptation (pass an adapted root_euler_d yourself).  The
  // state type must carry use_terrain_adapt, terrain_pitch_angle and foot_pos_recent_contact.
  std::function<double(int)> terrain_angle_of;

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
  // Each robot takes the branch its state.stance_leg_control_type selects (A1RobotControl.cpp:377,
  // :446): 0 -> the single-step QP balance controller (fresh solve), 1 -> the MPC (this
  // controller's persistent warm-started solver); states without the field are MPC.  `dt` is the
  // caller's thread period; it is the horizon step only when use_sim_time is set.  Robot b keeps
  // MPC warm-start slot b from call to call (a change of `count` re-initialises all); a QP tick
  // leaves the robot's MPC solver state untouched, as the reference's QP branch leaves the member
  // solver (it builds a local one, :416).
  template <class State>
  void compute_grf_batch(State* states, int count, double* forces, mpcqp_result* results = nullptr,
                         double dt = 0.0) {
    mpc_idx_.clear();
    qp_idx_.clear();
    for (int b = 0; b < count; ++b) {
      const int ty = control_type_of(states[b]);
      if (ty == 1) mpc_idx_.push_back(b);
      else if (ty == 0) qp_idx_.push_back(b);
      else throw std::invalid_argument("compute_grf: stance_leg_control_type must be 0 (QP) or 1 (MPC)");
    }
    res_.resize(count);
    if (!mpc_idx_.empty()) {
      if (use_sim_time && !(std::isfinite(dt) && dt > 0.0))
        throw std::invalid_argument("compute_grf: use_sim_time needs the caller's dt (finite, > 0)");
      const double hdt = use_sim_time ? dt : mpc_dt;  // A1RobotControl.cpp:462-467
      const int nm = (int)mpc_idx_.size();
      recs_.resize((size_t)nm * MPCQP_REC_SIZE(N));
      sub_res_.resize(nm);
      if (terrain_angle_of)
        for (int i = 0; i < nm; ++i) adapt_terrain(states[mpc_idx_[i]], mpc_idx_[i]);
      for (int i = 0; i < nm; ++i) assemble(states[mpc_idx_[i]], &recs_[(size_t)i * MPCQP_REC_SIZE(N)], hdt);
      if (warm_start) {
        ensure_slots(count);
        if (nm == count) {
          throw_on(mpcqp_solve_batch_warm_host(h_, recs_.data(), nm, d_state_, sub_res_.data(), nullptr), h_,
                   "mpcqp_solve_batch_warm_host");
        } else {  // the MPC robots' slots, gathered and scattered back around the solve
          // (one indexed-copy kernel each way on the legacy NULL stream, which the handle's
          // blocking stream waits for; the index list is uploaded only when it changes)
          DeviceScope ds(device_);
          ensure_gather(nm);
          if (mpc_idx_ != dev_idx_) {
            hip_ok(hipMemcpy(d_idx_, mpc_idx_.data(), sizeof(int) * nm, hipMemcpyHostToDevice), "hipMemcpy");
            dev_idx_ = mpc_idx_;
          }
          throw_on(mpcqp_copy_warm_slots_device(N, d_state_, d_idx_, d_gather_, nullptr, nm, nullptr), nullptr,
                   "mpcqp_copy_warm_slots_device");
          throw_on(mpcqp_solve_batch_warm_host(h_, recs_.data(), nm, d_gather_, sub_res_.data(), nullptr), h_,
                   "mpcqp_solve_batch_warm_host");
          throw_on(mpcqp_copy_warm_slots_device(N, d_gather_, nullptr, d_state_, d_idx_, nm, nullptr), nullptr,
                   "mpcqp_copy_warm_slots_device");
          hip_ok(hipStreamSynchronize(nullptr), "hipStreamSynchronize");
        }
      } else {
        throw_on(mpcqp_solve_batch_host(h_, recs_.data(), nm, sub_res_.data(), nullptr), h_, "mpcqp_solve_batch_host");
      }
      for (int i = 0; i < nm; ++i) res_[mpc_idx_[i]] = sub_res_[i];
    }
    if constexpr (has_control_type<State>::value) {  // (a state type without the field is MPC only)
     if (!qp_idx_.empty()) {
      const int nq = (int)qp_idx_.size();
      bal_recs_.resize((size_t)nq * MPCQP_BAL_SIZE);
      sub_res_.resize(nq);
      for (int i = 0; i < nq; ++i) assemble_balance(states[qp_idx_[i]], &bal_recs_[(size_t)i * MPCQP_BAL_SIZE]);
      throw_on(mpcqp_balance_solve_host(h_, &balance_params, bal_recs_.data(), nq, sub_res_.data()), h_,
               "mpcqp_balance_solve_host");
      for (int i = 0; i < nq; ++i) res_[qp_idx_[i]] = sub_res_[i];
     }
    }
    for (int b = 0; b < count; ++b) {
      for (int l = 0; l < 4; ++l)
        for (int r = 0; r < 3; ++r) forces[(size_t)b * 12 + r * 4 + l] = res_[b].f_body[3 * l + r];
      if (results) results[b] = res_[b];
    }
  }

  // A1RobotControl::compute_grf(A1CtrlStates& state, double dt) -> Eigen::Matrix<double,3,NUM_LEG>
  // (A1RobotControl.h:44): single robot, the branch of state.stance_leg_control_type (0: QP balance,
  // :377-444; 1: MPC warm-started from this controller's previous MPC call, :446-562).  Like the
  // reference, the MPC horizon step is mpc_dt = 0.0025 and `dt` only with use_sim_time (:458-467).
  // A leg whose MPC solution norm is NaN keeps a zero column (the reference leaves it uninitialised).
  // Terrain adaptation (:335-376): set terrain_angle_of (above), or pass an adapted root_euler_d.
  template <class State>
  Matrix34 compute_grf(State& state, double dt) {
    double f[12];
    compute_grf_batch(&state, 1, f, nullptr, dt);
    Matrix34 out;
    for (int r = 0; r < 3; ++r)
      for (int l = 0; l < 4; ++l) out(r, l) = f[r * 4 + l];
    return out;
  }
  // out-parameter form of the same call
  template <class State, class Mat34>
  void compute_grf(State& state, double dt, Mat34& foot_forces_grf) {
    const Matrix34 f = compute_grf(state, dt);
    for (int r = 0; r < 3; ++r)
      for (int l = 0; l < 4; ++l) foot_forces_grf(r, l) = f(r, l);
  }
  // status / iterations / residuals of the last compute_grf call (robot b of a batch)
  const mpcqp_result& last_result(int b = 0) const { return res_.at(b); }
  // forget the warm-start state (the next call is an initSolver again)
  void reset_warm_start() {
    if (d_state_) {
      DeviceScope ds(device_);
      hip_ok(hipMemset(d_state_, 0, sizeof(double) * slot_doubles() * slots_), "hipMemset");
    }
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

  // The state mutation of A1RobotControl.cpp:340-375 for MPC robot b (terrain_angle_of set).
  template <class State>
  void adapt_terrain(State& s, int b) const {
    if constexpr (has_terrain_fields<State>::value) {
      double terrain_angle = 0;
      if (s.root_pos[2] > 0.1) terrain_angle = terrain_angle_of(b);  // the filter samples only here
      if (terrain_angle > 0.5) terrain_angle = 0.5;
      if (terrain_angle < -0.5) terrain_angle = -0.5;
      const double f_r_diff = s.foot_pos_recent_contact(2, 0) + s.foot_pos_recent_contact(2, 1) -
                              s.foot_pos_recent_contact(2, 2) - s.foot_pos_recent_contact(2, 3);
      if (s.use_terrain_adapt) s.root_euler_d[1] = f_r_diff > 0.05 ? -terrain_angle : terrain_angle;
      s.terrain_pitch_angle = terrain_angle;
    } else {
      (void)s;
      (void)b;
      throw std::invalid_argument(
          "compute_grf: terrain_angle_of is set but the state type has no use_terrain_adapt / "
          "terrain_pitch_angle / foot_pos_recent_contact");
    }
  }

  mpcqp_handle* handle() const { return h_; }
  int device() const { return device_; }
  const double* warm_slots() const { return d_state_; }

 private:
  static size_t slot_doubles() { return (size_t)mpcqp_warm_state_size(N); }
  void ensure_slots(int count) {
    if (count == slots_ && d_state_) return;
    DeviceScope ds(device_);
    if (d_state_) hip_ok(hipFree(d_state_), "hipFree");
    d_state_ = nullptr;
    slots_ = 0;
    hip_ok(hipMalloc(&d_state_, sizeof(double) * slot_doubles() * count), "hipMalloc");
    hip_ok(hipMemset(d_state_, 0, sizeof(double) * slot_doubles() * count), "hipMemset");  // = not initialised
    slots_ = count;
  }
  void ensure_gather(int count) {
    if (count <= gather_cap_ && d_gather_) return;
    DeviceScope ds(device_);
    if (d_gather_) hip_ok(hipFree(d_gather_), "hipFree");
    if (d_idx_) hip_ok(hipFree(d_idx_), "hipFree");
    d_gather_ = nullptr;
    d_idx_ = nullptr;
    dev_idx_.clear();
    gather_cap_ = 0;
    hip_ok(hipMalloc(&d_gather_, sizeof(double) * slot_doubles() * count), "hipMalloc");
    hip_ok(hipMalloc(&d_idx_, sizeof(int) * count), "hipMalloc");
    gather_cap_ = count;
  }

  mpcqp_params params_{};
  mpcqp_handle* h_ = nullptr;
  int device_ = 0;
  double* d_state_ = nullptr;
  int slots_ = 0;
  double* d_gather_ = nullptr;  // mixed-mode batches: the MPC robots' slots, compacted
  int gather_cap_ = 0;
  int* d_idx_ = nullptr;         // device copy of mpc_idx_ (gather / scatter index list)
  std::vector<int> dev_idx_;     // what d_idx_ holds
  std::vector<int> mpc_idx_, qp_idx_;
  std::vector<mpcqp_result> sub_res_;
  std::vector<double> recs_;
  std::vector<double> bal_recs_;
  std::vector<mpcqp_result> res_;
};

using A1RobotControl = RobotControlT<A1InertiaOf>;
using Go1RobotControl = RobotControlT<Go1InertiaOf>;

}  // namespace mpcqp_cpp
