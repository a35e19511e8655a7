// mpcqp_balance.hip — the single-step QP balance controller, batched on the device
// (SURVEY §8(f) rank 3): the stance_leg_control_type == 0 branch of A1RobotControl::compute_grf
// (src/a1_cpp/src/A1RobotControl.cpp:321-332 euler error, :377-444 QP; ctor constants :7-48).
//
// Per robot: root_acc from the PD gains, M = [I; Rz^T skew(foot_i)] (6 x 12),
// H = r I + M'QM, g = -M'Q root_acc, 4 fz rows + 16 friction-pyramid rows, then a fresh OSQP 0.6
// setup + solve (Ruiz scaling, rho vector, KKT factorisation, ADMM, termination checks every
// check_termination iterations, adaptive rho at the fixed interval, infeasibility tests) and
// foot_forces_grf = R^T x per leg.
//
// Layout: one thread per robot; the whole 12-variable / 20-row OSQP workspace lives in that
// thread's registers (scratch where the compiler spills).  Every loop has compile-time bounds and
// is unrolled, and the constraint matrix is touched only at its 36 structural nonzeros (`anz`),
// so nothing is indexed at run time.  The arithmetic follows oracle/mpc_oracle.c
// (orc_balance_build_qp / ws_setup_dense / ws_admm) operation by operation with contraction off,
// so the GPU reproduces the oracle's iterate sequence.  The QP is 12 x 20: per-robot work is
// ~100 kFLOP (setup) + ~1.5 kFLOP per ADMM iteration, latency-bound, nowhere near HBM.
#include "mpcqp_device.h"

#pragma clang fp contract(off)

namespace mpcqp {
namespace bal {

constexpr int n = MPCQP_NUM_DOF;         // 12
constexpr int m = MPCQP_CONSTRAINT_DIM;  // 20
constexpr double INF = MPCQP_OSQP_INFTY;
constexpr double RHO_MIN_ = 1e-6, RHO_MAX_ = 1e6, RHO_EQ = 1e3, RHO_TOL_ = 1e-4;
constexpr double DIV_TOL = 1.0 / MPCQP_OSQP_INFTY;

// Structural nonzeros of the constraint matrix (ctor, A1RobotControl.cpp:27-44): row i < 4 is
// F_zi (col 3i+2); row 4+4i+k has +-1 at col 3i+(k>>1) and -mu at col 3i+2.
__host__ __device__ constexpr bool anz(int r, int c) {
  return r < 4 ? c == 3 * r + 2 : (c == 3 * ((r - 4) / 4) + 2 || c == 3 * ((r - 4) / 4) + (((r - 4) % 4) >> 1));
}

struct Ws {
  double P[n][n];  // scaled Hessian, upper triangle (i <= j) only
  double A[m][n];  // scaled constraints, structural nonzeros only
  double L[n][n];  // KKT Cholesky factor, lower triangle
  double q[n], l[m], u[m], D[n], E[m];
  double c, cinv, rho;
  int ctype[m];
  double x[n], z[m], y[m], xp[n], zp[m], xt[n], zt[m], dx[n], dy[m];
  double Ax[m], Px[n], Aty[n];
  double pri_res, dua_res, obj_val;
  int status, iter, rho_updates;
  double sigma, alpha;
};

__device__ __forceinline__ double rho_of(const Ws& w, int r) {
  return w.ctype[r] == -1 ? RHO_MIN_ : (w.ctype[r] == 1 ? RHO_EQ * w.rho : w.rho);
}

// K = P + sigma I + A' diag(rho) A, dense Cholesky (oracle factor_kkt, same accumulation order)
__device__ __forceinline__ int factor(Ws& w) {
  double K[n][n];
#pragma unroll
  for (int j = 0; j < n; ++j)
#pragma unroll
    for (int k = 0; k <= j; ++k) K[j][k] = 0.0;
#pragma unroll
  for (int j = 0; j < n; ++j)
#pragma unroll
    for (int i = 0; i <= j; ++i) K[j][i] += w.P[i][j];  // lower (j, i) of the symmetric P
#pragma unroll
  for (int i = 0; i < n; ++i) K[i][i] += w.sigma;
#pragma unroll
  for (int j = 0; j < n; ++j)
#pragma unroll
    for (int r = 0; r < m; ++r) {
      if (!anz(r, j)) continue;
#pragma unroll
      for (int k = 0; k <= j; ++k)
        if (anz(r, k)) K[j][k] += w.A[r][j] * rho_of(w, r) * w.A[r][k];
    }
  int bad = 0;
#pragma unroll
  for (int j = 0; j < n; ++j) {
    double s = K[j][j];
#pragma unroll
    for (int k = 0; k < j; ++k) s -= w.L[j][k] * w.L[j][k];
    bad |= !(s > 0.0);
    const double d = __builtin_sqrt(s);
    w.L[j][j] = d;
#pragma unroll
    for (int i = j + 1; i < n; ++i) {
      double t = K[i][j];
#pragma unroll
      for (int k = 0; k < j; ++k) t -= w.L[i][k] * w.L[j][k];
      w.L[i][j] = t / d;
    }
  }
  return bad;
}

__device__ __forceinline__ void kkt_solve(const Ws& w, double (&b)[n]) {
#pragma unroll
  for (int i = 0; i < n; ++i) {
    double s = b[i];
#pragma unroll
    for (int k = 0; k < i; ++k) s -= w.L[i][k] * b[k];
    b[i] = s / w.L[i][i];
  }
#pragma unroll
  for (int i = n - 1; i >= 0; --i) {
    double s = b[i];
#pragma unroll
    for (int k = i + 1; k < n; ++k) s -= w.L[k][i] * b[k];
    b[i] = s / w.L[i][i];
  }
}

// y = A x (CSC column order)
__device__ __forceinline__ void a_mul(const Ws& w, const double (&x)[n], double (&y)[m]) {
#pragma unroll
  for (int r = 0; r < m; ++r) y[r] = 0.0;
#pragma unroll
  for (int j = 0; j < n; ++j)
#pragma unroll
    for (int r = 0; r < m; ++r)
      if (anz(r, j)) y[r] += w.A[r][j] * x[j];
}
// y (+)= A' v
__device__ __forceinline__ void at_mul(const Ws& w, const double (&v)[m], double (&y)[n], bool plus) {
#pragma unroll
  for (int j = 0; j < n; ++j) {
    double s = plus ? y[j] : 0.0;
#pragma unroll
    for (int r = 0; r < m; ++r)
      if (anz(r, j)) s += w.A[r][j] * v[r];
    y[j] = s;
  }
}
// y = P x with P symmetric from its upper triangle (mat_vec, then mat_tpose_vec skipping the diagonal)
__device__ __forceinline__ void p_mul(const Ws& w, const double (&x)[n], double (&y)[n]) {
#pragma unroll
  for (int i = 0; i < n; ++i) y[i] = 0.0;
#pragma unroll
  for (int j = 0; j < n; ++j)
#pragma unroll
    for (int i = 0; i <= j; ++i) y[i] += w.P[i][j] * x[j];
#pragma unroll
  for (int j = 0; j < n; ++j)
#pragma unroll
    for (int i = 0; i <= j; ++i) y[j] += i == j ? 0.0 : w.P[i][j] * x[i];
}

template <int K>
__device__ __forceinline__ double norm_inf(const double (&v)[K]) {
  double mx = 0.0;
#pragma unroll
  for (int i = 0; i < K; ++i) mx = dabs(v[i]) > mx ? dabs(v[i]) : mx;
  return mx;
}
template <int K>
__device__ __forceinline__ double scaled_norm_inf(const double (&s)[K], const double (&v)[K], bool inv) {
  double mx = 0.0;
#pragma unroll
  for (int i = 0; i < K; ++i) {
    const double a = dabs((inv ? 1.0 / s[i] : s[i]) * v[i]);
    mx = a > mx ? a : mx;
  }
  return mx;
}

__device__ __forceinline__ void update_info(Ws& w, const mpcqp_params& p, int iter) {
  w.iter = iter;
  a_mul(w, w.x, w.Ax);
#pragma unroll
  for (int r = 0; r < m; ++r) w.zp[r] = w.Ax[r] + -1.0 * w.z[r];
  w.pri_res = p.scaling && !p.scaled_termination ? scaled_norm_inf<m>(w.E, w.zp, true) : norm_inf<m>(w.zp);
  p_mul(w, w.x, w.Px);
  at_mul(w, w.y, w.Aty, false);
#pragma unroll
  for (int j = 0; j < n; ++j) w.xp[j] = (w.q[j] + 1.0 * w.Px[j]) + 1.0 * w.Aty[j];
  w.dua_res = p.scaling && !p.scaled_termination ? w.cinv * scaled_norm_inf<n>(w.D, w.xp, true) : norm_inf<n>(w.xp);
}

__device__ __forceinline__ bool primal_infeasible(Ws& w, const mpcqp_params& p, double eps) {
  const bool sc = p.scaling && !p.scaled_termination;
#pragma unroll
  for (int r = 0; r < m; ++r) {
    if (w.u[r] > INF * MIN_SCALING)
      w.dy[r] = w.l[r] < -INF * MIN_SCALING ? 0.0 : dmin(w.dy[r], 0.0);
    else if (w.l[r] < -INF * MIN_SCALING)
      w.dy[r] = dmax(w.dy[r], 0.0);
  }
  double nrm = 0.0;
#pragma unroll
  for (int r = 0; r < m; ++r) {
    const double a = dabs(sc ? w.dy[r] * w.E[r] : w.dy[r]);
    nrm = a > nrm ? a : nrm;
  }
  if (nrm > DIV_TOL) {
    double lhs = 0.0;
#pragma unroll
    for (int r = 0; r < m; ++r) lhs += w.u[r] * dmax(w.dy[r], 0) + w.l[r] * dmin(w.dy[r], 0);
    if (lhs < eps * nrm) {
      double t[n];
      at_mul(w, w.dy, t, false);
      double mx = 0.0;
#pragma unroll
      for (int j = 0; j < n; ++j) {
        const double a = dabs(sc ? t[j] * (1.0 / w.D[j]) : t[j]);
        mx = a > mx ? a : mx;
      }
      return mx < eps * nrm;
    }
  }
  return false;
}

__device__ __forceinline__ bool dual_infeasible(const Ws& w, const mpcqp_params& p, double eps) {
  const bool sc = p.scaling && !p.scaled_termination;
  const double nrm = sc ? scaled_norm_inf<n>(w.D, w.dx, false) : norm_inf<n>(w.dx);
  const double cs = sc ? w.c : 1.0;
  if (nrm > DIV_TOL) {
    double qd = 0.0;
#pragma unroll
    for (int j = 0; j < n; ++j) qd += w.q[j] * w.dx[j];
    if (qd < cs * eps * nrm) {
      double t[n];
      p_mul(w, w.dx, t);
      double mx = 0.0;
#pragma unroll
      for (int j = 0; j < n; ++j) {
        const double a = dabs(sc ? t[j] * (1.0 / w.D[j]) : t[j]);
        mx = a > mx ? a : mx;
      }
      if (mx < cs * eps * nrm) {
        double ad[m];
        a_mul(w, w.dx, ad);
        bool ok = true;
#pragma unroll
        for (int r = 0; r < m; ++r) {
          const double v = sc ? ad[r] * (1.0 / w.E[r]) : ad[r];
          if (((w.u[r] < INF * MIN_SCALING) && (v > eps * nrm)) || ((w.l[r] > -INF * MIN_SCALING) && (v < -eps * nrm)))
            ok = false;
        }
        return ok;
      }
    }
  }
  return false;
}

__device__ __forceinline__ int check_termination(Ws& w, const mpcqp_params& p, bool approximate) {
  if ((w.pri_res > INF) || (w.dua_res > INF)) {
    w.status = MPCQP_STATUS_NON_CVX;
    w.obj_val = __builtin_nan("");
    return 1;
  }
  double eps_abs = p.eps_abs, eps_rel = p.eps_rel, eps_pinf = p.eps_prim_inf, eps_dinf = p.eps_dual_inf;
  if (approximate) {
    eps_abs *= 10;
    eps_rel *= 10;
    eps_pinf *= 10;
    eps_dinf *= 10;
  }
  const bool sc = p.scaling && !p.scaled_termination;
  bool prim_ok = false, dual_ok = false, prim_inf = false, dual_inf = false;
  {
    double mx = sc ? dmax(scaled_norm_inf<m>(w.E, w.z, true), scaled_norm_inf<m>(w.E, w.Ax, true))
                   : dmax(norm_inf<m>(w.z), norm_inf<m>(w.Ax));
    const double eps_prim = eps_abs + eps_rel * mx;
    if (w.pri_res < eps_prim)
      prim_ok = true;
    else
      prim_inf = primal_infeasible(w, p, eps_pinf);
  }
  {
    double mx;
    if (sc) {
      mx = scaled_norm_inf<n>(w.D, w.q, true);
      mx = dmax(mx, scaled_norm_inf<n>(w.D, w.Aty, true));
      mx = dmax(mx, scaled_norm_inf<n>(w.D, w.Px, true));
      mx *= w.cinv;
    } else {
      mx = dmax(dmax(norm_inf<n>(w.q), norm_inf<n>(w.Aty)), norm_inf<n>(w.Px));
    }
    const double eps_dual = eps_abs + eps_rel * mx;
    if (w.dua_res < eps_dual)
      dual_ok = true;
    else
      dual_inf = dual_infeasible(w, p, eps_dinf);
  }
  if (prim_ok && dual_ok) {
    w.status = approximate ? MPCQP_STATUS_SOLVED_INACCURATE : MPCQP_STATUS_SOLVED;
    return 1;
  }
  if (prim_inf) {
    w.status = approximate ? MPCQP_STATUS_PRIMAL_INFEASIBLE_INACCURATE : MPCQP_STATUS_PRIMAL_INFEASIBLE;
    w.obj_val = INF;
    return 1;
  }
  if (dual_inf) {
    w.status = approximate ? MPCQP_STATUS_DUAL_INFEASIBLE_INACCURATE : MPCQP_STATUS_DUAL_INFEASIBLE;
    w.obj_val = -INF;
    return 1;
  }
  return 0;
}

// compute_rho_estimate + adapt_rho (refactors on a change); returns the factorisation failure flag
__device__ __forceinline__ int adapt_rho(Ws& w, const mpcqp_params& p) {
  double pri = norm_inf<m>(w.zp);
  double dua = norm_inf<n>(w.xp);
  const double pn = dmax(norm_inf<m>(w.z), norm_inf<m>(w.Ax));
  pri /= (pn + DIV_TOL);
  const double dn = dmax(dmax(norm_inf<n>(w.q), norm_inf<n>(w.Aty)), norm_inf<n>(w.Px));
  dua /= (dn + DIV_TOL);
  double est = w.rho * __builtin_sqrt(pri / (dua + DIV_TOL));
  est = dmin(dmax(est, RHO_MIN_), RHO_MAX_);
  if ((est > w.rho * p.adaptive_rho_tolerance) || (est < w.rho / p.adaptive_rho_tolerance)) {
    w.rho_updates += 1;
    if (est <= 0) return 1;
    w.rho = dmin(dmax(est, RHO_MIN_), RHO_MAX_);
    return factor(w);
  }
  return 0;
}

__device__ __forceinline__ bool has_solution(int s) {
  return (s != MPCQP_STATUS_PRIMAL_INFEASIBLE) && (s != MPCQP_STATUS_PRIMAL_INFEASIBLE_INACCURATE) &&
         (s != MPCQP_STATUS_DUAL_INFEASIBLE) && (s != MPCQP_STATUS_DUAL_INFEASIBLE_INACCURATE) &&
         (s != MPCQP_STATUS_NON_CVX);
}

// orc_balance_build_qp: H (upper), g, l, u, A from one record (A1RobotControl.cpp:321-414)
__device__ __forceinline__ void build(Ws& w, const mpcqp_balance_params& bp, const double* rec) {
  double R[9], Rz[9];
#pragma unroll
  for (int k = 0; k < 9; ++k) {
    R[k] = rec[MPCQP_BAL_ROT + k];
    Rz[k] = rec[MPCQP_BAL_ROT_Z + k];
  }
  double ee[3];
#pragma unroll
  for (int k = 0; k < 3; ++k) ee[k] = rec[MPCQP_BAL_EULER_D + k] - rec[MPCQP_BAL_EULER + k];
  if (ee[2] > 3.1415926 * 1.5)
    ee[2] = rec[MPCQP_BAL_EULER_D + 2] - 3.1415926 * 2 - rec[MPCQP_BAL_EULER + 2];
  else if (ee[2] < -3.1415926 * 1.5)
    ee[2] = rec[MPCQP_BAL_EULER_D + 2] + 3.1415926 * 2 - rec[MPCQP_BAL_EULER + 2];
  double acc[6], tv[3], tw[3];
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    double sv = 0.0, sw = 0.0;
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      sv += R[k * 3 + i] * rec[MPCQP_BAL_LIN_VEL + k];
      sw += R[k * 3 + i] * rec[MPCQP_BAL_ANG_VEL + k];
    }
    tv[i] = rec[MPCQP_BAL_KD_LIN + i] * (rec[MPCQP_BAL_LIN_VEL_D + i] - sv);
    tw[i] = sw;
  }
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    double s = 0.0;
#pragma unroll
    for (int k = 0; k < 3; ++k) s += R[i * 3 + k] * tv[k];
    acc[i] = rec[MPCQP_BAL_KP_LIN + i] * (rec[MPCQP_BAL_POS_D + i] - rec[MPCQP_BAL_POS + i]) + s;
    acc[3 + i] = rec[MPCQP_BAL_KP_ANG + i] * ee[i] + rec[MPCQP_BAL_KD_ANG + i] * (rec[MPCQP_BAL_ANG_VEL_D + i] - tw[i]);
  }
  acc[2] += rec[MPCQP_BAL_MASS] * 9.8;
  double M[6][n];
#pragma unroll
  for (int leg = 0; leg < 4; ++leg) {
    const double f0 = rec[MPCQP_BAL_FEET + 3 * leg], f1 = rec[MPCQP_BAL_FEET + 3 * leg + 1],
                 f2 = rec[MPCQP_BAL_FEET + 3 * leg + 2];
    const double S[9] = {0.0, -f2, f1, f2, 0.0, -f0, -f1, f0, 0.0};  // Utils.cpp:35-41
#pragma unroll
    for (int a = 0; a < 3; ++a)
#pragma unroll
      for (int b = 0; b < 3; ++b) {
        M[a][3 * leg + b] = a == b ? 1.0 : 0.0;
        double s = 0.0;
#pragma unroll
        for (int k = 0; k < 3; ++k) s += Rz[k * 3 + a] * S[k * 3 + b];
        M[3 + a][3 * leg + b] = s;
      }
  }
#pragma unroll
  for (int j = 0; j < n; ++j) {
#pragma unroll
    for (int i = 0; i <= j; ++i) {
      double s = 0.0;
#pragma unroll
      for (int k = 0; k < 6; ++k) s += (M[k][i] * bp.q_diag[k]) * M[k][j];
      w.P[i][j] = (i == j ? bp.r : 0.0) + s;
    }
    double g = 0.0;
#pragma unroll
    for (int k = 0; k < 6; ++k) g += (-M[k][j] * bp.q_diag[k]) * acc[k];
    w.q[j] = g;
  }
#pragma unroll
  for (int leg = 0; leg < 4; ++leg) {
    const double c = rec[MPCQP_BAL_CONTACTS + leg] != 0.0 ? 1.0 : 0.0;
    w.A[leg][3 * leg + 2] = 1.0;
    w.l[leg] = c * bp.f_min;
    w.u[leg] = c * bp.f_max;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int row = 4 + 4 * leg + k;
      w.A[row][3 * leg + (k >> 1)] = (k & 1) ? -1.0 : 1.0;
      w.A[row][3 * leg + 2] = -bp.mu;
      w.l[row] = -INF;
      w.u[row] = 0.0;
    }
  }
}

// OSQP 0.6 scale_data (10 Ruiz passes + cost scaling) on the dense structured data
__device__ __forceinline__ void scale(Ws& w, const mpcqp_params& p) {
  w.c = 1.0;
#pragma unroll
  for (int j = 0; j < n; ++j) w.D[j] = 1.0;
#pragma unroll
  for (int r = 0; r < m; ++r) w.E[r] = 1.0;
  for (int it = 0; it < p.scaling; ++it) {
    double Dt[n], Et[m];
#pragma unroll
    for (int j = 0; j < n; ++j) Dt[j] = 0.0;
#pragma unroll
    for (int j = 0; j < n; ++j)
#pragma unroll
      for (int i = 0; i <= j; ++i) {
        const double ax = dabs(w.P[i][j]);
        Dt[j] = dmax(ax, Dt[j]);
        if (i != j) Dt[i] = dmax(ax, Dt[i]);
      }
#pragma unroll
    for (int j = 0; j < n; ++j) {
      double a = 0.0;
#pragma unroll
      for (int r = 0; r < m; ++r)
        if (anz(r, j)) a = dmax(dabs(w.A[r][j]), a);
      Dt[j] = dmax(Dt[j], a);
    }
#pragma unroll
    for (int r = 0; r < m; ++r) {
      double a = 0.0;
#pragma unroll
      for (int j = 0; j < n; ++j)
        if (anz(r, j)) a = dmax(dabs(w.A[r][j]), a);
      Et[r] = a;
    }
#pragma unroll
    for (int j = 0; j < n; ++j) Dt[j] = 1.0 / __builtin_sqrt(limit_scaling(Dt[j]));
#pragma unroll
    for (int r = 0; r < m; ++r) Et[r] = 1.0 / __builtin_sqrt(limit_scaling(Et[r]));
#pragma unroll
    for (int j = 0; j < n; ++j)
#pragma unroll
      for (int i = 0; i <= j; ++i) w.P[i][j] = (w.P[i][j] * Dt[i]) * Dt[j];
#pragma unroll
    for (int r = 0; r < m; ++r)
#pragma unroll
      for (int j = 0; j < n; ++j)
        if (anz(r, j)) w.A[r][j] = (w.A[r][j] * Et[r]) * Dt[j];
#pragma unroll
    for (int j = 0; j < n; ++j) {
      w.q[j] = w.q[j] * Dt[j];
      w.D[j] = Dt[j] * w.D[j];
    }
#pragma unroll
    for (int r = 0; r < m; ++r) w.E[r] = Et[r] * w.E[r];
    // cost normalisation
    double cn[n];
#pragma unroll
    for (int j = 0; j < n; ++j) cn[j] = 0.0;
#pragma unroll
    for (int j = 0; j < n; ++j)
#pragma unroll
      for (int i = 0; i <= j; ++i) {
        const double ax = dabs(w.P[i][j]);
        cn[j] = dmax(ax, cn[j]);
        if (i != j) cn[i] = dmax(ax, cn[i]);
      }
    double s = 0.0;
#pragma unroll
    for (int j = 0; j < n; ++j) s += cn[j];
    double ct = s / n;
    const double qn = limit_scaling(norm_inf<n>(w.q));
    ct = limit_scaling(dmax(ct, qn));
    ct = 1. / ct;
#pragma unroll
    for (int j = 0; j < n; ++j)
#pragma unroll
      for (int i = 0; i <= j; ++i) w.P[i][j] *= ct;
#pragma unroll
    for (int j = 0; j < n; ++j) w.q[j] *= ct;
    w.c *= ct;
  }
  w.cinv = 1. / w.c;
#pragma unroll
  for (int r = 0; r < m; ++r) {
    w.l[r] = w.l[r] * w.E[r];
    w.u[r] = w.u[r] * w.E[r];
  }
}

__global__ void __launch_bounds__(64) balance_kernel(const double* __restrict__ recs, int batch,
                                                     mpcqp_balance_params bp, mpcqp_params p,
                                                     mpcqp_result* __restrict__ out) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= batch) return;
  const double* rec = recs + (size_t)MPCQP_BAL_SIZE * b;
  mpcqp_result* res = out + b;
  bool finite = true;
#pragma unroll
  for (int k = 0; k < MPCQP_BAL_SIZE - 1; ++k) finite &= __builtin_isfinite(rec[k]);
  if (!finite) {
#pragma unroll
    for (int k = 0; k < n; ++k) res->u0[k] = res->f_body[k] = __builtin_nan("");
    res->obj_val = res->pri_res = res->dua_res = res->rho = 0.0;
    res->status = MPCQP_STATUS_NAN_INPUT;
    res->iters = res->rho_updates = 0;
    res->nan_legs = 0xF;
    return;
  }
  Ws w;
  w.sigma = p.sigma;
  w.alpha = p.alpha;
  w.pri_res = w.dua_res = w.obj_val = 0.0;
  w.iter = 0;
  w.rho_updates = 0;
  build(w, bp, rec);
#pragma unroll
  for (int r = 0; r < m; ++r) {
    w.l[r] = dmax(w.l[r], -INF);
    w.u[r] = dmin(w.u[r], INF);
  }
  if (p.scaling) {
    scale(w, p);
  } else {
    w.c = w.cinv = 1.0;
#pragma unroll
    for (int j = 0; j < n; ++j) w.D[j] = 1.0;
#pragma unroll
    for (int r = 0; r < m; ++r) w.E[r] = 1.0;
  }
  // set_rho_vec
  w.rho = dmin(dmax(p.rho, RHO_MIN_), RHO_MAX_);
#pragma unroll
  for (int r = 0; r < m; ++r)
    w.ctype[r] = (w.l[r] < -INF * MIN_SCALING && w.u[r] > INF * MIN_SCALING) ? -1 : (w.u[r] - w.l[r] < RHO_TOL_ ? 1 : 0);
#pragma unroll
  for (int j = 0; j < n; ++j) w.x[j] = 0.0;
#pragma unroll
  for (int r = 0; r < m; ++r) w.z[r] = w.y[r] = 0.0;
  int fail = factor(w);

  // ws_admm
  w.status = MPCQP_STATUS_UNSOLVED;
  const double a = w.alpha, a1 = (double)1.0 - w.alpha;
  int iter = 0;
  bool can_check = false;
  if (!fail) {
    for (iter = 1; iter <= p.max_iter; ++iter) {
#pragma unroll
      for (int j = 0; j < n; ++j) w.xp[j] = w.x[j];
#pragma unroll
      for (int r = 0; r < m; ++r) w.zp[r] = w.z[r];
      // (P + sigma I + A' rho A) x~ = (sigma x - q) + A' (rho z - y);  z~ = A x~
#pragma unroll
      for (int j = 0; j < n; ++j) w.xt[j] = w.sigma * w.xp[j] - w.q[j];
      {
        double t[m];
#pragma unroll
        for (int r = 0; r < m; ++r) t[r] = rho_of(w, r) * w.zp[r] - w.y[r];
        at_mul(w, t, w.xt, true);
      }
      kkt_solve(w, w.xt);
      a_mul(w, w.xt, w.zt);
#pragma unroll
      for (int j = 0; j < n; ++j) {
        w.x[j] = a * w.xt[j] + a1 * w.xp[j];
        w.dx[j] = w.x[j] - w.xp[j];
      }
#pragma unroll
      for (int r = 0; r < m; ++r) {
        const double rv = rho_of(w, r);
        const double zr = a * w.zt[r] + a1 * w.zp[r] + (1. / rv) * w.y[r];
        w.z[r] = dmin(dmax(zr, w.l[r]), w.u[r]);
        w.dy[r] = rv * (a * w.zt[r] + a1 * w.zp[r] - w.z[r]);
        w.y[r] += w.dy[r];
      }
      can_check = p.check_termination && (iter % p.check_termination == 0);
      int done = 0;
      if (can_check) {
        update_info(w, p, iter);
        done = check_termination(w, p, false);
      }
      if (!done && p.adaptive_rho && p.adaptive_rho_interval && (iter % p.adaptive_rho_interval == 0)) {
        if (!can_check) update_info(w, p, iter);
        if (adapt_rho(w, p)) fail = 1;
      }
      if (done || fail) break;
    }
    if (!can_check && !fail) {
      update_info(w, p, iter - 1);
      check_termination(w, p, false);
    }
    if (w.status == MPCQP_STATUS_UNSOLVED && !fail) {
      if (!check_termination(w, p, true)) w.status = MPCQP_STATUS_MAX_ITER_REACHED;
    }
  }
  if (fail) w.status = MPCQP_STATUS_NON_CVX;
  const bool sol = has_solution(w.status);
  if (sol) {  // compute_obj_val
    double qf = 0.0;
#pragma unroll
    for (int j = 0; j < n; ++j)
#pragma unroll
      for (int i = 0; i <= j; ++i)
        if (w.P[i][j] != 0.0) qf += i == j ? .5 * w.P[i][j] * w.x[i] * w.x[i] : w.P[i][j] * w.x[i] * w.x[j];
    double qx = 0.0;
#pragma unroll
    for (int j = 0; j < n; ++j) qx += w.q[j] * w.x[j];
    double obj = qf + qx;
    if (p.scaling) obj *= w.cinv;
    w.obj_val = obj;
  }
  // getSolution + foot_forces_grf = R^T x per leg (A1RobotControl.cpp:438-443)
  double xs[n];
#pragma unroll
  for (int j = 0; j < n; ++j) xs[j] = sol ? w.D[j] * w.x[j] : __builtin_nan("");
  int nan_legs = 0;
#pragma unroll
  for (int leg = 0; leg < 4; ++leg) {
    const double f0 = xs[3 * leg], f1 = xs[3 * leg + 1], f2 = xs[3 * leg + 2];
    if (__builtin_isnan(f0 + f1 + f2)) nan_legs |= 1 << leg;
#pragma unroll
    for (int r = 0; r < 3; ++r) {
      double s = 0.0;
      s += rec[MPCQP_BAL_ROT + r] * f0;
      s += rec[MPCQP_BAL_ROT + 3 + r] * f1;
      s += rec[MPCQP_BAL_ROT + 6 + r] * f2;
      res->f_body[3 * leg + r] = s;
    }
  }
#pragma unroll
  for (int j = 0; j < n; ++j) res->u0[j] = xs[j];
  res->obj_val = w.obj_val;
  res->pri_res = w.pri_res;
  res->dua_res = w.dua_res;
  res->rho = w.rho;
  res->status = w.status;
  res->iters = w.iter;
  res->rho_updates = w.rho_updates;
  res->nan_legs = nan_legs;
}

}  // namespace bal

hipError_t launch_balance(const mpcqp_balance_params& bp, const mpcqp_params& p, const double* recs, int batch,
                          mpcqp_result* out, void* stream) {
  hipLaunchKernelGGL(bal::balance_kernel, dim3((batch + 63) / 64), dim3(64), 0, (hipStream_t)stream, recs, batch, bp,
                     p, out);
  return hipGetLastError();
}

}  // namespace mpcqp
