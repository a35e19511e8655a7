/*
 * mpc_oracle.c — TEST INFRASTRUCTURE ONLY (parity checker + CPU baseline "port").
 *
 * CPU binary64 restatement of the reference hot path:
 *   - input assembly of A1RobotControl::compute_grf's MPC branch
 *       (src/a1_cpp/src/A1RobotControl.cpp:446-514) and of test_mpc (src/a1_cpp/src/test/test_mpc.cpp:15-125)
 *   - ConvexMpc (src/a1_cpp/src/ConvexMpc.cpp:7-245): A_c, B_c, forward-Euler discretization,
 *     A_qp/B_qp, dense H = B_qp' Q B_qp + R, gradient, friction-pyramid C, l/u
 *   - OSQP 0.6.x ADMM as driven by OsqpEigen 0.6.3 (A1RobotControl.cpp:522-555): Ruiz scaling,
 *     rho vector, reduced-KKT solve, alpha relaxation, projection, termination every
 *     check_termination iterations, primal/dual infeasibility tests, adaptive rho with a FIXED
 *     interval (OSQP's wall-clock interval is not reproducible), approximate check at max_iter,
 *     unscaling, NaN-guarded force extraction (A1RobotControl.cpp:555-561).
 *
 * The OSQP functions below keep OSQP's names (scale_data, set_rho_vec, update_xz_tilde, ...) and
 * their operation order.  OSQP's QDLDL factorization of the quasi-definite KKT matrix is replaced
 * by a dense Cholesky of the equivalent reduced matrix P + sigma I + A' diag(rho) A (identical in
 * exact arithmetic; differs at rounding level).
 *
 * Parity: formulation pinned to the reference's formulas; OSQP iterate sequence "parity unpinned"
 * (OSQP not vendored/buildable here, no reference golden vectors) — see DESIGN.md.
 * Built with -ffp-contract=off so results are deterministic on any x86-64 host.
 */
#include "mpc_oracle.h"

#include <math.h>
#include <pthread.h>
#include <stdlib.h>
#include <string.h>

#define SD 13
#define NL 4
#define ND 12
#define CD 20
#define OSQP_INFTY MPCQP_OSQP_INFTY
#define OSQP_NAN (NAN)
#define MIN_SCALING 1e-4
#define MAX_SCALING 1e4
#define RHO_MIN 1e-6
#define RHO_MAX 1e6
#define RHO_EQ_OVER_RHO_INEQ 1e3
#define RHO_TOL 1e-4
#define OSQP_DIVISION_TOL (1.0 / OSQP_INFTY)

static inline double c_max(double a, double b) { return a > b ? a : b; }
static inline double c_min(double a, double b) { return a < b ? a : b; }
static inline double c_absval(double a) { return a < 0 ? -a : a; }

/* ============================================================================================
 * Input assembly
 * ========================================================================================== */

static void mat3_mul(const double* A, const double* B, double* C) {
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) {
      double s = 0.0;
      for (int k = 0; k < 3; ++k) s += A[i * 3 + k] * B[k * 3 + j];
      C[i * 3 + j] = s;
    }
}

/* A1RobotControl.cpp:452-514 (MPC branch of compute_grf). */
void orc_assemble_compute_grf(const orc_robot_state* s, int32_t N, double* rec) {
  memset(rec, 0, sizeof(double) * (size_t)MPCQP_REC_SIZE(N));
  double* x0 = rec + MPCQP_REC_X0;
  /* :452-456 */
  for (int k = 0; k < 3; ++k) {
    x0[k] = s->root_euler[k];
    x0[3 + k] = s->root_pos[k];
    x0[6 + k] = s->root_ang_vel[k];
    x0[9 + k] = s->root_lin_vel[k];
  }
  x0[12] = -9.8;
  const double dt = s->mpc_dt; /* :462 (0.0025) */
  /* :470 root_lin_vel_d_world = root_rot_mat * root_lin_vel_d */
  double vdw[3];
  for (int r = 0; r < 3; ++r) {
    double acc = 0.0;
    for (int c = 0; c < 3; ++c) acc += s->root_rot_mat[r * 3 + c] * s->root_lin_vel_d[c];
    vdw[r] = acc;
  }
  /* :472-488 */
  for (int i = 0; i < N; ++i) {
    double* xr = rec + MPCQP_REC_XREF + 13 * i;
    xr[0] = s->root_euler_d[0];
    xr[1] = s->root_euler_d[1];
    xr[2] = s->root_euler[2] + s->root_ang_vel_d[2] * dt * (i + 1);
    xr[3] = s->root_pos[0] + vdw[0] * dt * (i + 1);
    xr[4] = s->root_pos[1] + vdw[1] * dt * (i + 1);
    xr[5] = s->root_pos_d[2];
    xr[6] = s->root_ang_vel_d[0];
    xr[7] = s->root_ang_vel_d[1];
    xr[8] = s->root_ang_vel_d[2];
    xr[9] = vdw[0];
    xr[10] = vdw[1];
    xr[11] = 0.0;
    xr[12] = -9.8;
  }
  /* :492 calculate_A_mat_c(state.root_euler) */
  for (int k = 0; k < 3; ++k) rec[MPCQP_REC_EULER + k] = s->root_euler[k];
  for (int k = 0; k < 9; ++k) {
    rec[MPCQP_REC_ROT + k] = s->root_rot_mat[k];
    rec[MPCQP_REC_INERTIA + k] = s->trunk_inertia[k];
  }
  rec[MPCQP_REC_MASS] = s->robot_mass;
  rec[MPCQP_REC_MU] = s->mu;
  rec[MPCQP_REC_FZMIN] = s->fz_min;
  rec[MPCQP_REC_FZMAX] = s->fz_max;
  rec[MPCQP_REC_DT] = dt;
  for (int l = 0; l < 4; ++l) rec[MPCQP_REC_CONTACTS + l] = s->contacts[l] ? 1.0 : 0.0;
  /* :498-514 production: the same foot_pos_abs for every horizon step (shift commented out) */
  for (int i = 0; i < N; ++i)
    for (int k = 0; k < 12; ++k) rec[MPCQP_REC_FEET(N) + 12 * i + k] = s->foot_pos_abs[k];
}

/* test_mpc.cpp:15-122 */
void orc_assemble_test_mpc(int32_t N, double* rec, double q_weights[13], double r_weights[12]) {
  memset(rec, 0, sizeof(double) * (size_t)MPCQP_REC_SIZE(N));
  const double dt = 0.0025;                               /* :48 */
  const double euler[3] = {0.0, 0.0, 0.0};                /* :23 */
  const double pos[3] = {0.0, 0.0, 0.15};                 /* :32 */
  const double euler_d[3] = {0, 0, 0}, ang_vel_d[3] = {0, 0, 0}, lin_vel_d[3] = {0, 0, 0};
  const double R[9] = {1, 0, 0, 0, 1, 0, 0, 0, 1};        /* :25-30 with all-zero angles */
  /* :39-41 foot_pos_rel (rows x,y,z; cols FL FR RL RR) */
  const double fx[4] = {0.17, 0.17, -0.17, -0.17}, fy[4] = {0.15, -0.15, 0.15, -0.15},
               fz[4] = {-0.35, -0.35, -0.35, -0.35};
  const int contacts[4] = {1, 0, 1, 0}; /* :43-46 */
  const double qw[13] = {1.0, 1.0, 1.0, 0.0, 0.0, 50.0, 0.0, 0.0, 1.0, 1.0, 1.0, 1.0, 0.0};
  if (q_weights) memcpy(q_weights, qw, sizeof(qw));
  if (r_weights)
    for (int k = 0; k < 12; ++k) r_weights[k] = 1e-6; /* :57-60 */
  double* x0 = rec + MPCQP_REC_X0;
  for (int k = 0; k < 3; ++k) {
    x0[k] = euler[k];
    x0[3 + k] = pos[k];
  }
  x0[12] = -9.8;
  double vdw[3];
  for (int r = 0; r < 3; ++r) {
    double acc = 0.0;
    for (int c = 0; c < 3; ++c) acc += R[r * 3 + c] * lin_vel_d[c];
    vdw[r] = acc;
  }
  for (int i = 0; i < N; ++i) { /* :75-91 (note pz_ref uses v_dw,y and vz_ref = v_dw,z) */
    double* xr = rec + MPCQP_REC_XREF + 13 * i;
    xr[0] = euler_d[0];
    xr[1] = euler_d[1];
    xr[2] = euler[2] + ang_vel_d[2] * dt * (i + 1);
    xr[3] = pos[0] + vdw[0] * dt * (i + 1);
    xr[4] = pos[1] + vdw[1] * dt * (i + 1);
    xr[5] = pos[2] + vdw[1] * dt * (i + 1);
    xr[6] = ang_vel_d[0];
    xr[7] = ang_vel_d[1];
    xr[8] = ang_vel_d[2];
    xr[9] = vdw[0];
    xr[10] = vdw[1];
    xr[11] = vdw[2];
    xr[12] = -9.8;
  }
  /* :94-101 average euler over the horizon (only yaw enters A_c) */
  for (int k = 0; k < 3; ++k)
    rec[MPCQP_REC_EULER + k] = (euler[k] + euler[k] + ang_vel_d[k] * dt * N) / (N + 1);
  for (int k = 0; k < 9; ++k) rec[MPCQP_REC_ROT + k] = R[k];
  rec[MPCQP_REC_INERTIA + 0] = 0.0158533; /* :19-21 */
  rec[MPCQP_REC_INERTIA + 4] = 0.0377999;
  rec[MPCQP_REC_INERTIA + 8] = 0.0456542;
  rec[MPCQP_REC_MASS] = 15;               /* :18 */
  rec[MPCQP_REC_MU] = 0.3;                /* ConvexMpc.cpp:8 */
  rec[MPCQP_REC_FZMIN] = 0.0;             /* ConvexMpc.cpp:223 */
  rec[MPCQP_REC_FZMAX] = 180.0;           /* ConvexMpc.cpp:224 */
  rec[MPCQP_REC_DT] = dt;
  for (int l = 0; l < 4; ++l) rec[MPCQP_REC_CONTACTS + l] = contacts[l];
  /* :105-122 foot_pos_abs_mpc = foot_pos_rel, shifted by -root_lin_vel_d*dt after each step */
  double feet[12];
  for (int l = 0; l < 4; ++l) {
    feet[3 * l + 0] = fx[l];
    feet[3 * l + 1] = fy[l];
    feet[3 * l + 2] = fz[l];
  }
  for (int i = 0; i < N; ++i) {
    for (int k = 0; k < 12; ++k) rec[MPCQP_REC_FEET(N) + 12 * i + k] = feet[k];
    for (int l = 0; l < 4; ++l)
      for (int c = 0; c < 3; ++c) feet[3 * l + c] = feet[3 * l + c] - lin_vel_d[c] * dt;
  }
}

/* ============================================================================================
 * ConvexMpc restatement
 * ========================================================================================== */

/* Eigen's 3x3 inverse (cofactor / determinant), Eigen/src/LU/InverseImpl.h. */
static double cof3(const double* m, int i, int j) {
  int i1 = (i + 1) % 3, i2 = (i + 2) % 3, j1 = (j + 1) % 3, j2 = (j + 2) % 3;
  return m[i1 * 3 + j1] * m[i2 * 3 + j2] - m[i1 * 3 + j2] * m[i2 * 3 + j1];
}
static void mat3_inverse(const double* m, double* inv) {
  double c0 = cof3(m, 0, 0), c1 = cof3(m, 1, 0), c2 = cof3(m, 2, 0);
  double det = (c0 * m[0] + c1 * m[3]) + c2 * m[6];
  double invdet = 1.0 / det;
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) inv[j * 3 + i] = cof3(m, i, j) * invdet;
}

/* calculate_A_mat_c (ConvexMpc.cpp:110-130) + discretization A_d = I + A_c dt (:150). */
static void build_A_d(double yaw, double dt, double* Ad /*13x13 row-major*/) {
  double Ac[SD * SD];
  memset(Ac, 0, sizeof(Ac));
  double cy = cos(yaw), sy = sin(yaw);
  Ac[0 * SD + 6] = cy;
  Ac[0 * SD + 7] = sy;
  Ac[1 * SD + 6] = -sy;
  Ac[1 * SD + 7] = cy;
  Ac[2 * SD + 8] = 1.0;
  Ac[3 * SD + 9] = 1.0;
  Ac[4 * SD + 10] = 1.0;
  Ac[5 * SD + 11] = 1.0;
  Ac[11 * SD + ND] = 1.0;
  for (int i = 0; i < SD; ++i)
    for (int j = 0; j < SD; ++j) Ad[i * SD + j] = (i == j ? 1.0 : 0.0) + Ac[i * SD + j] * dt;
}

/* calculate_B_mat_c (ConvexMpc.cpp:132-143) + B_d = B_c dt (:151). */
static void build_B_d(const double* R, const double* Ib, double mass, const double* feet, double dt,
                      double* Bd /*13x12 row-major*/) {
  double tmp[9], Rt[9], Iw[9], Iwinv[9];
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) Rt[i * 3 + j] = R[j * 3 + i];
  mat3_mul(R, Ib, tmp);
  mat3_mul(tmp, Rt, Iw);
  mat3_inverse(Iw, Iwinv);
  double Bc[SD * ND];
  memset(Bc, 0, sizeof(Bc));
  for (int l = 0; l < NL; ++l) {
    const double* r = feet + 3 * l;
    double sk[9] = {0.0, -r[2], r[1], r[2], 0.0, -r[0], -r[1], r[0], 0.0}; /* Utils.cpp:35-41 */
    double blk[9];
    mat3_mul(Iwinv, sk, blk);
    for (int i = 0; i < 3; ++i)
      for (int j = 0; j < 3; ++j) {
        Bc[(6 + i) * ND + 3 * l + j] = blk[i * 3 + j];
        Bc[(9 + i) * ND + 3 * l + j] = (i == j ? (1.0 / mass) : 0.0);
      }
  }
  for (int k = 0; k < SD * ND; ++k) Bd[k] = Bc[k] * dt;
}

int32_t orc_build_qp(const mpcqp_params* prm, const double* rec, double* P, double* q, double* l,
                     double* u, double* Acon) {
  const int N = prm->horizon;
  if (N < 1) return MPCQP_ERR_INVALID_ARG;
  const int n = ND * N, m = CD * N, ns = SD * N;
  const double dt = rec[MPCQP_REC_DT];
  double Ad[SD * SD];
  build_A_d(rec[MPCQP_REC_EULER + 2], dt, Ad);

  double* Bdl = (double*)malloc(sizeof(double) * SD * ND * N);        /* B_mat_d_list */
  double* Aqp = (double*)malloc(sizeof(double) * SD * SD * N);        /* A_qp blocks */
  double* Bqp = (double*)calloc((size_t)ns * n, sizeof(double));      /* B_qp dense */
  for (int i = 0; i < N; ++i)
    build_B_d(rec + MPCQP_REC_ROT, rec + MPCQP_REC_INERTIA, rec[MPCQP_REC_MASS],
              rec + MPCQP_REC_FEET(N) + 12 * i, dt, Bdl + SD * ND * i);

  /* ConvexMpc.cpp:184-202 */
  for (int i = 0; i < N; ++i) {
    double* Ai = Aqp + SD * SD * i;
    if (i == 0) {
      memcpy(Ai, Ad, sizeof(Ad));
    } else {
      const double* Ap = Aqp + SD * SD * (i - 1);
      for (int r = 0; r < SD; ++r)
        for (int c = 0; c < SD; ++c) {
          double s = 0.0;
          for (int k = 0; k < SD; ++k) s += Ap[r * SD + k] * Ad[k * SD + c];
          Ai[r * SD + c] = s;
        }
    }
    for (int j = 0; j < i + 1; ++j) {
      const double* Bd = Bdl + SD * ND * j;
      for (int r = 0; r < SD; ++r)
        for (int c = 0; c < ND; ++c) {
          double v;
          if (i - j == 0) {
            v = Bd[r * ND + c];
          } else {
            const double* Apow = Aqp + SD * SD * (i - j - 1);
            double s = 0.0;
            for (int k = 0; k < SD; ++k) s += Apow[r * SD + k] * Bd[k * ND + c];
            v = s;
          }
          Bqp[(size_t)(SD * i + r) * n + ND * j + c] = v;
        }
    }
  }
  /* Q = diag(2 q tiled), R = diag(2 r tiled) (ConvexMpc.cpp:16-23, 37-44) */
  /* :209-210  dense_hessian = B_qp' * Q * B_qp; += R */
  double* W = (double*)malloc(sizeof(double) * (size_t)n * ns); /* W = B_qp' Q, [n][ns] */
  for (int a = 0; a < n; ++a)
    for (int r = 0; r < ns; ++r) W[(size_t)a * ns + r] = Bqp[(size_t)r * n + a] * (2 * prm->q_weights[r % SD]);
  for (int a = 0; a < n; ++a)
    for (int b = 0; b < n; ++b) {
      double s = 0.0;
      for (int r = 0; r < ns; ++r) s += W[(size_t)a * ns + r] * Bqp[(size_t)r * n + b];
      P[(size_t)a * n + b] = s;
    }
  for (int a = 0; a < n; ++a) P[(size_t)a * n + a] += 2 * prm->r_weights[a % ND];
  /* :215-217  gradient = B_qp' * Q * (A_qp * x0 - x_ref) */
  double* tmp = (double*)malloc(sizeof(double) * ns);
  const double* x0 = rec + MPCQP_REC_X0;
  for (int i = 0; i < N; ++i)
    for (int r = 0; r < SD; ++r) {
      double s = 0.0;
      for (int k = 0; k < SD; ++k) s += Aqp[SD * SD * i + r * SD + k] * x0[k];
      tmp[SD * i + r] = s;
    }
  for (int r = 0; r < ns; ++r) tmp[r] -= rec[MPCQP_REC_XREF + r];
  for (int a = 0; a < n; ++a) {
    double s = 0.0;
    for (int r = 0; r < ns; ++r) s += W[(size_t)a * ns + r] * tmp[r];
    q[a] = s;
  }
  /* :223-245 bounds */
  const double fz_min = rec[MPCQP_REC_FZMIN], fz_max = rec[MPCQP_REC_FZMAX];
  for (int i = 0; i < N; ++i)
    for (int leg = 0; leg < NL; ++leg) {
      double c = rec[MPCQP_REC_CONTACTS + leg] != 0.0 ? 1.0 : 0.0; /* bool contacts[i] */
      int b = CD * i + 5 * leg;
      l[b + 0] = 0;
      l[b + 1] = -OSQP_INFTY;
      l[b + 2] = 0;
      l[b + 3] = -OSQP_INFTY;
      l[b + 4] = fz_min * c;
      u[b + 0] = OSQP_INFTY;
      u[b + 1] = 0;
      u[b + 2] = OSQP_INFTY;
      u[b + 3] = 0;
      u[b + 4] = fz_max * c;
    }
  /* :46-58 friction pyramid (ConvexMpc ctor), mu per record */
  if (Acon) {
    const double mu = rec[MPCQP_REC_MU];
    memset(Acon, 0, sizeof(double) * (size_t)m * n);
    for (int f = 0; f < NL * N; ++f) {
      Acon[(size_t)(5 * f + 0) * n + 3 * f + 0] = 1;
      Acon[(size_t)(5 * f + 1) * n + 3 * f + 0] = 1;
      Acon[(size_t)(5 * f + 2) * n + 3 * f + 1] = 1;
      Acon[(size_t)(5 * f + 3) * n + 3 * f + 1] = 1;
      Acon[(size_t)(5 * f + 4) * n + 3 * f + 2] = 1;
      Acon[(size_t)(5 * f + 0) * n + 3 * f + 2] = mu;
      Acon[(size_t)(5 * f + 1) * n + 3 * f + 2] = -mu;
      Acon[(size_t)(5 * f + 2) * n + 3 * f + 2] = mu;
      Acon[(size_t)(5 * f + 3) * n + 3 * f + 2] = -mu;
    }
  }
  free(Bdl);
  free(Aqp);
  free(Bqp);
  free(W);
  free(tmp);
  return MPCQP_OK;
}

/* ============================================================================================
 * OSQP 0.6 restatement (CSC storage like OSQP; dense Cholesky for the KKT solve)
 * ========================================================================================== */

typedef struct {
  int m, n;
  int* p;
  int* i;
  double* x;
} csc;

typedef struct {
  int n, m;
  csc P, A; /* P: upper triangle */
  double *q, *l, *u;
  /* scaling */
  double *D, *Dinv, *E, *Einv, c, cinv;
  /* rho */
  double *rho_vec, *rho_inv_vec;
  int* constr_type;
  double rho;
  /* iterates & work vectors */
  double *x, *y, *z, *xz_tilde, *x_prev, *z_prev, *Ax, *Px, *Aty, *delta_y, *Atdelta_y, *delta_x,
      *Pdelta_x, *Adelta_x, *D_temp, *D_temp_A, *E_temp;
  /* KKT */
  double *K, *L;
  double* pool; /* backing store of the vectors above */
  /* settings */
  const mpcqp_params* st;
  /* info */
  int iter, status, rho_updates;
  double pri_res, dua_res, obj_val;
  double mu; /* friction coefficient of the constraint matrix A latched by the last setup */
  int last_update_mode; /* ws_update's branch: 1 osqp_update_P, 2 OsqpEigen re-init */
} osqp_ws;

static csc dense_to_csc_upper(const double* M, int n) {
  csc C;
  C.m = n;
  C.n = n;
  C.p = (int*)malloc(sizeof(int) * (n + 1));
  int nnz = 0;
  for (int j = 0; j < n; ++j)
    for (int i = 0; i <= j; ++i)
      if (M[(size_t)i * n + j] != 0.0) ++nnz;
  C.i = (int*)malloc(sizeof(int) * (nnz > 0 ? nnz : 1));
  C.x = (double*)malloc(sizeof(double) * (nnz > 0 ? nnz : 1));
  int k = 0;
  for (int j = 0; j < n; ++j) {
    C.p[j] = k;
    for (int i = 0; i <= j; ++i) {
      double v = M[(size_t)i * n + j];
      if (v != 0.0) { /* Eigen sparseView(): drops exact zeros only */
        C.i[k] = i;
        C.x[k] = v;
        ++k;
      }
    }
  }
  C.p[n] = k;
  return C;
}

static csc dense_to_csc(const double* M, int m, int n) {
  csc C;
  C.m = m;
  C.n = n;
  C.p = (int*)malloc(sizeof(int) * (n + 1));
  int nnz = 0;
  for (int j = 0; j < n; ++j)
    for (int i = 0; i < m; ++i)
      if (M[(size_t)i * n + j] != 0.0) ++nnz;
  C.i = (int*)malloc(sizeof(int) * (nnz > 0 ? nnz : 1));
  C.x = (double*)malloc(sizeof(double) * (nnz > 0 ? nnz : 1));
  int k = 0;
  for (int j = 0; j < n; ++j) {
    C.p[j] = k;
    for (int i = 0; i < m; ++i) {
      double v = M[(size_t)i * n + j];
      if (v != 0.0) {
        C.i[k] = i;
        C.x[k] = v;
        ++k;
      }
    }
  }
  C.p[n] = k;
  return C;
}

static void csc_free(csc* C) {
  free(C->p);
  free(C->i);
  free(C->x);
}

/* lin_alg.c */
static void vec_set_scalar(double* a, double sc, int n) {
  for (int i = 0; i < n; ++i) a[i] = sc;
}
static void vec_ew_sqrt(double* a, int n) {
  for (int i = 0; i < n; ++i) a[i] = sqrt(a[i]);
}
static void vec_ew_recipr(const double* a, double* b, int n) {
  for (int i = 0; i < n; ++i) b[i] = 1.0 / a[i];
}
static void vec_ew_prod(const double* a, const double* b, double* c, int n) {
  for (int i = 0; i < n; ++i) c[i] = b[i] * a[i];
}
static void vec_ew_max_vec(const double* a, const double* b, double* c, int n) {
  for (int i = 0; i < n; ++i) c[i] = c_max(a[i], b[i]);
}
static double vec_mean(const double* a, int n) {
  double s = 0.0;
  for (int i = 0; i < n; ++i) s += a[i];
  return s / n;
}
static double vec_norm_inf(const double* v, int l) {
  double mx = 0.0;
  for (int i = 0; i < l; ++i) {
    double a = c_absval(v[i]);
    if (a > mx) mx = a;
  }
  return mx;
}
static double vec_scaled_norm_inf(const double* S, const double* v, int l) {
  double mx = 0.0;
  for (int i = 0; i < l; ++i) {
    double a = c_absval(S[i] * v[i]);
    if (a > mx) mx = a;
  }
  return mx;
}
static double vec_prod(const double* a, const double* b, int n) {
  double s = 0.0;
  for (int i = 0; i < n; ++i) s += a[i] * b[i];
  return s;
}
static void vec_add_scaled(double* c, const double* a, const double* b, int n, double sc) {
  for (int i = 0; i < n; ++i) c[i] = a[i] + sc * b[i];
}
static void vec_mult_scalar(double* a, double sc, int n) {
  for (int i = 0; i < n; ++i) a[i] *= sc;
}
static void mat_mult_scalar(csc* A, double sc) {
  for (int i = 0; i < A->p[A->n]; ++i) A->x[i] *= sc;
}
static void mat_premult_diag(csc* A, const double* d) {
  for (int j = 0; j < A->n; ++j)
    for (int i = A->p[j]; i < A->p[j + 1]; ++i) A->x[i] *= d[A->i[i]];
}
static void mat_postmult_diag(csc* A, const double* d) {
  for (int j = 0; j < A->n; ++j)
    for (int i = A->p[j]; i < A->p[j + 1]; ++i) A->x[i] *= d[j];
}
static void mat_vec(const csc* A, const double* x, double* y, int plus_eq) {
  if (!plus_eq)
    for (int i = 0; i < A->m; ++i) y[i] = 0;
  for (int j = 0; j < A->n; ++j)
    for (int i = A->p[j]; i < A->p[j + 1]; ++i) y[A->i[i]] += A->x[i] * x[j];
}
static void mat_tpose_vec(const csc* A, const double* x, double* y, int plus_eq, int skip_diag) {
  if (!plus_eq)
    for (int i = 0; i < A->n; ++i) y[i] = 0;
  if (skip_diag) {
    for (int j = 0; j < A->n; ++j)
      for (int k = A->p[j]; k < A->p[j + 1]; ++k) {
        int i = A->i[k];
        y[j] += i == j ? 0 : A->x[k] * x[i];
      }
  } else {
    for (int j = 0; j < A->n; ++j)
      for (int k = A->p[j]; k < A->p[j + 1]; ++k) y[j] += A->x[k] * x[A->i[k]];
  }
}
static void mat_inf_norm_cols(const csc* M, double* E) {
  for (int j = 0; j < M->n; ++j) E[j] = 0.;
  for (int j = 0; j < M->n; ++j)
    for (int p = M->p[j]; p < M->p[j + 1]; ++p) E[j] = c_max(c_absval(M->x[p]), E[j]);
}
static void mat_inf_norm_rows(const csc* M, double* E) {
  for (int j = 0; j < M->m; ++j) E[j] = 0.;
  for (int j = 0; j < M->n; ++j)
    for (int p = M->p[j]; p < M->p[j + 1]; ++p) {
      int i = M->i[p];
      E[i] = c_max(c_absval(M->x[p]), E[i]);
    }
}
static void mat_inf_norm_cols_sym_triu(const csc* M, double* E) {
  for (int j = 0; j < M->n; ++j) E[j] = 0.;
  for (int j = 0; j < M->n; ++j)
    for (int p = M->p[j]; p < M->p[j + 1]; ++p) {
      int i = M->i[p];
      double ax = c_absval(M->x[p]);
      E[j] = c_max(ax, E[j]);
      if (i != j) E[i] = c_max(ax, E[i]);
    }
}

/* scaling.c */
static void limit_scaling(double* D, int n) {
  for (int i = 0; i < n; ++i) {
    D[i] = D[i] < MIN_SCALING ? 1.0 : D[i];
    D[i] = D[i] > MAX_SCALING ? MAX_SCALING : D[i];
  }
}
static void compute_inf_norm_cols_KKT(const csc* P, const csc* A, double* D, double* D_temp_A,
                                      double* E, int n) {
  mat_inf_norm_cols_sym_triu(P, D);
  mat_inf_norm_cols(A, D_temp_A);
  vec_ew_max_vec(D, D_temp_A, D, n);
  mat_inf_norm_rows(A, E);
}
static void scale_data(osqp_ws* w) {
  const int n = w->n, m = w->m;
  w->c = 1.0;
  vec_set_scalar(w->D, 1., n);
  vec_set_scalar(w->Dinv, 1., n);
  vec_set_scalar(w->E, 1., m);
  vec_set_scalar(w->Einv, 1., m);
  for (int i = 0; i < w->st->scaling; ++i) {
    compute_inf_norm_cols_KKT(&w->P, &w->A, w->D_temp, w->D_temp_A, w->E_temp, n);
    limit_scaling(w->D_temp, n);
    limit_scaling(w->E_temp, m);
    vec_ew_sqrt(w->D_temp, n);
    vec_ew_sqrt(w->E_temp, m);
    vec_ew_recipr(w->D_temp, w->D_temp, n);
    vec_ew_recipr(w->E_temp, w->E_temp, m);
    mat_premult_diag(&w->P, w->D_temp);
    mat_postmult_diag(&w->P, w->D_temp);
    mat_premult_diag(&w->A, w->E_temp);
    mat_postmult_diag(&w->A, w->D_temp);
    vec_ew_prod(w->D_temp, w->q, w->q, n);
    vec_ew_prod(w->D, w->D_temp, w->D, n);
    vec_ew_prod(w->E, w->E_temp, w->E, m);
    /* cost normalization */
    mat_inf_norm_cols_sym_triu(&w->P, w->D_temp);
    double c_temp = vec_mean(w->D_temp, n);
    double inf_norm_q = vec_norm_inf(w->q, n);
    limit_scaling(&inf_norm_q, 1);
    c_temp = c_max(c_temp, inf_norm_q);
    limit_scaling(&c_temp, 1);
    c_temp = 1. / c_temp;
    mat_mult_scalar(&w->P, c_temp);
    vec_mult_scalar(w->q, c_temp, n);
    w->c *= c_temp;
  }
  w->cinv = 1. / w->c;
  vec_ew_recipr(w->D, w->Dinv, n);
  vec_ew_recipr(w->E, w->Einv, m);
  vec_ew_prod(w->E, w->l, w->l, m);
  vec_ew_prod(w->E, w->u, w->u, m);
}

/* auxil.c */
static void set_rho_vec(osqp_ws* w) {
  w->rho = c_min(c_max(w->rho, RHO_MIN), RHO_MAX);
  for (int i = 0; i < w->m; ++i) {
    if ((w->l[i] < -OSQP_INFTY * MIN_SCALING) && (w->u[i] > OSQP_INFTY * MIN_SCALING)) {
      w->constr_type[i] = -1;
      w->rho_vec[i] = RHO_MIN;
    } else if (w->u[i] - w->l[i] < RHO_TOL) {
      w->constr_type[i] = 1;
      w->rho_vec[i] = RHO_EQ_OVER_RHO_INEQ * w->rho;
    } else {
      w->constr_type[i] = 0;
      w->rho_vec[i] = w->rho;
    }
    w->rho_inv_vec[i] = 1. / w->rho_vec[i];
  }
}

/* KKT "factorization": K = P + sigma I + A' diag(rho) A, dense Cholesky K = L L'. */
static int factor_kkt(osqp_ws* w) {
  const int n = w->n;
  double* K = w->K;
  memset(K, 0, sizeof(double) * (size_t)n * n);
  for (int j = 0; j < n; ++j)
    for (int p = w->P.p[j]; p < w->P.p[j + 1]; ++p) {
      int i = w->P.i[p];
      K[(size_t)i * n + j] += w->P.x[p];
      if (i != j) K[(size_t)j * n + i] += w->P.x[p];
    }
  for (int i = 0; i < n; ++i) K[(size_t)i * n + i] += w->st->sigma;
  /* A' diag(rho) A: for each pair of entries sharing a row */
  for (int j = 0; j < n; ++j)
    for (int p = w->A.p[j]; p < w->A.p[j + 1]; ++p) {
      int r = w->A.i[p];
      for (int k = 0; k < n; ++k)
        for (int p2 = w->A.p[k]; p2 < w->A.p[k + 1]; ++p2)
          if (w->A.i[p2] == r) K[(size_t)j * n + k] += w->A.x[p] * w->rho_vec[r] * w->A.x[p2];
    }
  double* L = w->L;
  memset(L, 0, sizeof(double) * (size_t)n * n);
  for (int j = 0; j < n; ++j) {
    double s = K[(size_t)j * n + j];
    for (int k = 0; k < j; ++k) s -= L[(size_t)j * n + k] * L[(size_t)j * n + k];
    if (!(s > 0.0)) return 1;
    double d = sqrt(s);
    L[(size_t)j * n + j] = d;
    for (int i = j + 1; i < n; ++i) {
      double t = K[(size_t)i * n + j];
      for (int k = 0; k < j; ++k) t -= L[(size_t)i * n + k] * L[(size_t)j * n + k];
      L[(size_t)i * n + j] = t / d;
    }
  }
  return 0;
}

static void kkt_solve(osqp_ws* w, double* b /* in: rhs of x part; out: solution */) {
  const int n = w->n;
  const double* L = w->L;
  for (int i = 0; i < n; ++i) {
    double s = b[i];
    for (int k = 0; k < i; ++k) s -= L[(size_t)i * n + k] * b[k];
    b[i] = s / L[(size_t)i * n + i];
  }
  for (int i = n - 1; i >= 0; --i) {
    double s = b[i];
    for (int k = i + 1; k < n; ++k) s -= L[(size_t)k * n + i] * b[k];
    b[i] = s / L[(size_t)i * n + i];
  }
}

/* osqp.c / auxil.c ADMM steps */
static void compute_rhs(osqp_ws* w) {
  for (int i = 0; i < w->n; ++i) w->xz_tilde[i] = w->st->sigma * w->x_prev[i] - w->q[i];
  for (int i = 0; i < w->m; ++i) w->xz_tilde[i + w->n] = w->z_prev[i] - w->rho_inv_vec[i] * w->y[i];
}
static void update_xz_tilde(osqp_ws* w) {
  const int n = w->n, m = w->m;
  compute_rhs(w);
  /* reduced form of the KKT solve:
   *   (P + sigma I + A' rho A) x~ = (sigma x - q) + A' rho (z - y/rho);   z~ = A x~ */
  double* b = w->xz_tilde;
  double* t = w->Adelta_x; /* scratch (overwritten before any other use) */
  for (int i = 0; i < m; ++i) t[i] = w->rho_vec[i] * w->z_prev[i] - w->y[i];
  mat_tpose_vec(&w->A, t, b, 1, 0);
  kkt_solve(w, b);
  mat_vec(&w->A, b, b + n, 0);
}
static void update_x(osqp_ws* w) {
  for (int i = 0; i < w->n; ++i)
    w->x[i] = w->st->alpha * w->xz_tilde[i] + ((double)1.0 - w->st->alpha) * w->x_prev[i];
  for (int i = 0; i < w->n; ++i) w->delta_x[i] = w->x[i] - w->x_prev[i];
}
static void project(osqp_ws* w, double* z) {
  for (int i = 0; i < w->m; ++i) z[i] = c_min(c_max(z[i], w->l[i]), w->u[i]);
}
static void update_z(osqp_ws* w) {
  for (int i = 0; i < w->m; ++i)
    w->z[i] = w->st->alpha * w->xz_tilde[i + w->n] + ((double)1.0 - w->st->alpha) * w->z_prev[i] +
              w->rho_inv_vec[i] * w->y[i];
  project(w, w->z);
}
static void update_y(osqp_ws* w) {
  for (int i = 0; i < w->m; ++i) {
    w->delta_y[i] = w->rho_vec[i] * (w->st->alpha * w->xz_tilde[i + w->n] +
                                     ((double)1.0 - w->st->alpha) * w->z_prev[i] - w->z[i]);
    w->y[i] += w->delta_y[i];
  }
}
static double compute_obj_val(osqp_ws* w, const double* x) {
  /* quad_form(P, x) on the upper triangle + q'x, unscaled by cinv */
  double qf = 0.0;
  for (int j = 0; j < w->n; ++j)
    for (int p = w->P.p[j]; p < w->P.p[j + 1]; ++p) {
      int i = w->P.i[p];
      if (i == j)
        qf += .5 * w->P.x[p] * x[i] * x[i];
      else
        qf += w->P.x[p] * x[i] * x[j];
    }
  double obj = qf + vec_prod(w->q, x, w->n);
  if (w->st->scaling) obj *= w->cinv;
  return obj;
}
static double compute_pri_res(osqp_ws* w, const double* x, const double* z) {
  mat_vec(&w->A, x, w->Ax, 0);
  vec_add_scaled(w->z_prev, w->Ax, z, w->m, -1);
  if (w->st->scaling && !w->st->scaled_termination)
    return vec_scaled_norm_inf(w->Einv, w->z_prev, w->m);
  return vec_norm_inf(w->z_prev, w->m);
}
static double compute_pri_tol(osqp_ws* w, double eps_abs, double eps_rel) {
  double max_rel_eps, temp_rel_eps;
  if (w->st->scaling && !w->st->scaled_termination) {
    max_rel_eps = vec_scaled_norm_inf(w->Einv, w->z, w->m);
    temp_rel_eps = vec_scaled_norm_inf(w->Einv, w->Ax, w->m);
    max_rel_eps = c_max(max_rel_eps, temp_rel_eps);
  } else {
    max_rel_eps = vec_norm_inf(w->z, w->m);
    temp_rel_eps = vec_norm_inf(w->Ax, w->m);
    max_rel_eps = c_max(max_rel_eps, temp_rel_eps);
  }
  return eps_abs + eps_rel * max_rel_eps;
}
static double compute_dua_res(osqp_ws* w, const double* x, const double* y) {
  memcpy(w->x_prev, w->q, sizeof(double) * w->n);
  mat_vec(&w->P, x, w->Px, 0);
  mat_tpose_vec(&w->P, x, w->Px, 1, 1);
  vec_add_scaled(w->x_prev, w->x_prev, w->Px, w->n, 1);
  mat_tpose_vec(&w->A, y, w->Aty, 0, 0);
  vec_add_scaled(w->x_prev, w->x_prev, w->Aty, w->n, 1);
  if (w->st->scaling && !w->st->scaled_termination)
    return w->cinv * vec_scaled_norm_inf(w->Dinv, w->x_prev, w->n);
  return vec_norm_inf(w->x_prev, w->n);
}
static double compute_dua_tol(osqp_ws* w, double eps_abs, double eps_rel) {
  double max_rel_eps, temp_rel_eps;
  if (w->st->scaling && !w->st->scaled_termination) {
    max_rel_eps = vec_scaled_norm_inf(w->Dinv, w->q, w->n);
    temp_rel_eps = vec_scaled_norm_inf(w->Dinv, w->Aty, w->n);
    max_rel_eps = c_max(max_rel_eps, temp_rel_eps);
    temp_rel_eps = vec_scaled_norm_inf(w->Dinv, w->Px, w->n);
    max_rel_eps = c_max(max_rel_eps, temp_rel_eps);
    max_rel_eps *= w->cinv;
  } else {
    max_rel_eps = vec_norm_inf(w->q, w->n);
    temp_rel_eps = vec_norm_inf(w->Aty, w->n);
    max_rel_eps = c_max(max_rel_eps, temp_rel_eps);
    temp_rel_eps = vec_norm_inf(w->Px, w->n);
    max_rel_eps = c_max(max_rel_eps, temp_rel_eps);
  }
  return eps_abs + eps_rel * max_rel_eps;
}
static int is_primal_infeasible(osqp_ws* w, double eps_prim_inf) {
  double norm_delta_y, ineq_lhs = 0.0;
  for (int i = 0; i < w->m; ++i) {
    if (w->u[i] > OSQP_INFTY * MIN_SCALING) {
      if (w->l[i] < -OSQP_INFTY * MIN_SCALING)
        w->delta_y[i] = 0.0;
      else
        w->delta_y[i] = c_min(w->delta_y[i], 0.0);
    } else if (w->l[i] < -OSQP_INFTY * MIN_SCALING) {
      w->delta_y[i] = c_max(w->delta_y[i], 0.0);
    }
  }
  if (w->st->scaling && !w->st->scaled_termination) {
    vec_ew_prod(w->E, w->delta_y, w->Adelta_x, w->m);
    norm_delta_y = vec_norm_inf(w->Adelta_x, w->m);
  } else {
    norm_delta_y = vec_norm_inf(w->delta_y, w->m);
  }
  if (norm_delta_y > OSQP_DIVISION_TOL) {
    for (int i = 0; i < w->m; ++i)
      ineq_lhs += w->u[i] * c_max(w->delta_y[i], 0) + w->l[i] * c_min(w->delta_y[i], 0);
    if (ineq_lhs < eps_prim_inf * norm_delta_y) {
      mat_tpose_vec(&w->A, w->delta_y, w->Atdelta_y, 0, 0);
      if (w->st->scaling && !w->st->scaled_termination)
        vec_ew_prod(w->Dinv, w->Atdelta_y, w->Atdelta_y, w->n);
      return vec_norm_inf(w->Atdelta_y, w->n) < eps_prim_inf * norm_delta_y;
    }
  }
  return 0;
}
static int is_dual_infeasible(osqp_ws* w, double eps_dual_inf) {
  double norm_delta_x, cost_scaling;
  if (w->st->scaling && !w->st->scaled_termination) {
    norm_delta_x = vec_scaled_norm_inf(w->D, w->delta_x, w->n);
    cost_scaling = w->c;
  } else {
    norm_delta_x = vec_norm_inf(w->delta_x, w->n);
    cost_scaling = 1.0;
  }
  if (norm_delta_x > OSQP_DIVISION_TOL) {
    if (vec_prod(w->q, w->delta_x, w->n) < cost_scaling * eps_dual_inf * norm_delta_x) {
      mat_vec(&w->P, w->delta_x, w->Pdelta_x, 0);
      mat_tpose_vec(&w->P, w->delta_x, w->Pdelta_x, 1, 1);
      if (w->st->scaling && !w->st->scaled_termination)
        vec_ew_prod(w->Dinv, w->Pdelta_x, w->Pdelta_x, w->n);
      if (vec_norm_inf(w->Pdelta_x, w->n) < cost_scaling * eps_dual_inf * norm_delta_x) {
        mat_vec(&w->A, w->delta_x, w->Adelta_x, 0);
        if (w->st->scaling && !w->st->scaled_termination)
          vec_ew_prod(w->Einv, w->Adelta_x, w->Adelta_x, w->m);
        for (int i = 0; i < w->m; ++i) {
          if (((w->u[i] < OSQP_INFTY * MIN_SCALING) && (w->Adelta_x[i] > eps_dual_inf * norm_delta_x)) ||
              ((w->l[i] > -OSQP_INFTY * MIN_SCALING) && (w->Adelta_x[i] < -eps_dual_inf * norm_delta_x)))
            return 0;
        }
        return 1;
      }
    }
  }
  return 0;
}
static void update_info(osqp_ws* w, int iter) {
  w->iter = iter;
  w->pri_res = (w->m == 0) ? 0. : compute_pri_res(w, w->x, w->z);
  w->dua_res = compute_dua_res(w, w->x, w->y);
}
static int check_termination(osqp_ws* w, int approximate, double* eps_prim_out, double* eps_dual_out) {
  int exitflag = 0, prim_res_check = 0, dual_res_check = 0, prim_inf_check = 0, dual_inf_check = 0;
  double eps_abs = w->st->eps_abs, eps_rel = w->st->eps_rel;
  double eps_prim_inf = w->st->eps_prim_inf, eps_dual_inf = w->st->eps_dual_inf;
  double eps_prim = 0, eps_dual = 0;
  if ((w->pri_res > OSQP_INFTY) || (w->dua_res > OSQP_INFTY)) {
    w->status = MPCQP_STATUS_NON_CVX;
    w->obj_val = OSQP_NAN;
    return 1;
  }
  if (approximate) {
    eps_abs *= 10;
    eps_rel *= 10;
    eps_prim_inf *= 10;
    eps_dual_inf *= 10;
  }
  if (w->m == 0) {
    prim_res_check = 1;
  } else {
    eps_prim = compute_pri_tol(w, eps_abs, eps_rel);
    if (w->pri_res < eps_prim)
      prim_res_check = 1;
    else
      prim_inf_check = is_primal_infeasible(w, eps_prim_inf);
  }
  eps_dual = compute_dua_tol(w, eps_abs, eps_rel);
  if (w->dua_res < eps_dual)
    dual_res_check = 1;
  else
    dual_inf_check = is_dual_infeasible(w, eps_dual_inf);
  if (eps_prim_out) *eps_prim_out = eps_prim;
  if (eps_dual_out) *eps_dual_out = eps_dual;
  if (prim_res_check && dual_res_check) {
    w->status = approximate ? MPCQP_STATUS_SOLVED_INACCURATE : MPCQP_STATUS_SOLVED;
    exitflag = 1;
  } else if (prim_inf_check) {
    w->status = approximate ? MPCQP_STATUS_PRIMAL_INFEASIBLE_INACCURATE : MPCQP_STATUS_PRIMAL_INFEASIBLE;
    if (w->st->scaling && !w->st->scaled_termination) vec_ew_prod(w->E, w->delta_y, w->delta_y, w->m);
    w->obj_val = OSQP_INFTY;
    exitflag = 1;
  } else if (dual_inf_check) {
    w->status = approximate ? MPCQP_STATUS_DUAL_INFEASIBLE_INACCURATE : MPCQP_STATUS_DUAL_INFEASIBLE;
    if (w->st->scaling && !w->st->scaled_termination) vec_ew_prod(w->D, w->delta_x, w->delta_x, w->n);
    w->obj_val = -OSQP_INFTY;
    exitflag = 1;
  }
  return exitflag;
}
static double compute_rho_estimate(osqp_ws* w) {
  const int n = w->n, m = w->m;
  double pri_res = vec_norm_inf(w->z_prev, m);
  double dua_res = vec_norm_inf(w->x_prev, n);
  double pri_res_norm = vec_norm_inf(w->z, m);
  double temp = vec_norm_inf(w->Ax, m);
  pri_res_norm = c_max(pri_res_norm, temp);
  pri_res /= (pri_res_norm + OSQP_DIVISION_TOL);
  double dua_res_norm = vec_norm_inf(w->q, n);
  temp = vec_norm_inf(w->Aty, n);
  dua_res_norm = c_max(dua_res_norm, temp);
  temp = vec_norm_inf(w->Px, n);
  dua_res_norm = c_max(dua_res_norm, temp);
  dua_res /= (dua_res_norm + OSQP_DIVISION_TOL);
  double rho_estimate = w->rho * sqrt(pri_res / (dua_res + OSQP_DIVISION_TOL));
  return c_min(c_max(rho_estimate, RHO_MIN), RHO_MAX);
}
static int osqp_update_rho(osqp_ws* w, double rho_new) {
  if (rho_new <= 0) return 1;
  w->rho = c_min(c_max(rho_new, RHO_MIN), RHO_MAX);
  for (int i = 0; i < w->m; ++i) {
    if (w->constr_type[i] == 0) {
      w->rho_vec[i] = w->rho;
      w->rho_inv_vec[i] = 1. / w->rho;
    } else if (w->constr_type[i] == 1) {
      w->rho_vec[i] = RHO_EQ_OVER_RHO_INEQ * w->rho;
      w->rho_inv_vec[i] = 1. / w->rho_vec[i];
    }
  }
  return factor_kkt(w);
}
static int adapt_rho(osqp_ws* w) {
  double rho_new = compute_rho_estimate(w);
  int exitflag = 0;
  if ((rho_new > w->rho * w->st->adaptive_rho_tolerance) ||
      (rho_new < w->rho / w->st->adaptive_rho_tolerance)) {
    exitflag = osqp_update_rho(w, rho_new);
    w->rho_updates += 1;
  }
  return exitflag;
}
static int has_solution(int s) {
  return (s != MPCQP_STATUS_PRIMAL_INFEASIBLE) && (s != MPCQP_STATUS_PRIMAL_INFEASIBLE_INACCURATE) &&
         (s != MPCQP_STATUS_DUAL_INFEASIBLE) && (s != MPCQP_STATUS_DUAL_INFEASIBLE_INACCURATE) &&
         (s != MPCQP_STATUS_NON_CVX);
}

static int record_has_nonfinite(const double* rec, int N) {
  for (int k = 0; k < MPCQP_REC_SIZE(N); ++k)
    if (!isfinite(rec[k])) return 1;
  return 0;
}

/* ---- workspace lifetime ------------------------------------------------------------------- */
static void ws_alloc(osqp_ws* w, const mpcqp_params* prm) {
  const int N = prm->horizon, n = ND * N, m = CD * N;
  memset(w, 0, sizeof(*w));
  w->n = n;
  w->m = m;
  w->st = prm;
  w->q = (double*)malloc(sizeof(double) * n);
  w->l = (double*)malloc(sizeof(double) * m);
  w->u = (double*)malloc(sizeof(double) * m);
  double* pool = (double*)calloc((size_t)(15 * n + 12 * m + 2 * (n + m)), sizeof(double));
  w->pool = pool;
  double* pp = pool;
#define TAKE(ptr, cnt) \
  ptr = pp;            \
  pp += (cnt)
  TAKE(w->D, n);
  TAKE(w->Dinv, n);
  TAKE(w->E, m);
  TAKE(w->Einv, m);
  TAKE(w->rho_vec, m);
  TAKE(w->rho_inv_vec, m);
  TAKE(w->x, n);
  TAKE(w->y, m);
  TAKE(w->z, m);
  TAKE(w->xz_tilde, n + m);
  TAKE(w->x_prev, n);
  TAKE(w->z_prev, m);
  TAKE(w->Ax, m);
  TAKE(w->Px, n);
  TAKE(w->Aty, n);
  TAKE(w->delta_y, m);
  TAKE(w->Atdelta_y, n);
  TAKE(w->delta_x, n);
  TAKE(w->Pdelta_x, n);
  TAKE(w->Adelta_x, m);
  TAKE(w->D_temp, n);
  TAKE(w->D_temp_A, n);
  TAKE(w->E_temp, m);
#undef TAKE
  w->constr_type = (int*)calloc(m, sizeof(int));
  w->K = (double*)malloc(sizeof(double) * (size_t)n * n);
  w->L = (double*)malloc(sizeof(double) * (size_t)n * n);
  w->rho = prm->rho;
  w->status = MPCQP_STATUS_UNSOLVED;
}
static void ws_free(osqp_ws* w) {
  csc_free(&w->P);
  csc_free(&w->A);
  free(w->q);
  free(w->l);
  free(w->u);
  free(w->pool);
  free(w->constr_type);
  free(w->K);
  free(w->L);
  memset(w, 0, sizeof(*w));
}

/* osqp_setup on the QP of `rec` (OsqpEigen::Solver::initSolver, A1RobotControl.cpp:521-531):
 * data copy, bound clipping, scale_data, set_rho_vec, KKT factorization; x = z = y = 0. */
static int ws_setup_dense(osqp_ws* w, double* Pd, double* Ad);
static int ws_setup(osqp_ws* w, const double* rec) {
  w->mu = rec[MPCQP_REC_MU];
  const int n = w->n, m = w->m;
  double* Pd = (double*)malloc(sizeof(double) * (size_t)n * n);
  double* Ad = (double*)malloc(sizeof(double) * (size_t)m * n);
  orc_build_qp(w->st, rec, Pd, w->q, w->l, w->u, Ad);
  return ws_setup_dense(w, Pd, Ad);
}
/* osqp_setup from dense P (full symmetric) and A (row-major) with q, l, u already in `w`;
 * frees Pd and Ad. */
static int ws_setup_dense(osqp_ws* w, double* Pd, double* Ad) {
  const int n = w->n, m = w->m;
  /* OsqpEigen::Data::setHessianMatrix keeps triangularView<Upper> of hessian.sparseView() */
  csc_free(&w->P);
  csc_free(&w->A);
  w->P = dense_to_csc_upper(Pd, n);
  w->A = dense_to_csc(Ad, m, n);
  free(Pd);
  free(Ad);
  for (int i = 0; i < m; ++i) { /* osqp_setup clips bounds to +-OSQP_INFTY */
    w->l[i] = c_max(w->l[i], -OSQP_INFTY);
    w->u[i] = c_min(w->u[i], OSQP_INFTY);
  }
  w->rho = w->st->rho;
  if (w->st->scaling)
    scale_data(w);
  else {
    w->c = w->cinv = 1.0;
    vec_set_scalar(w->D, 1., n);
    vec_set_scalar(w->Dinv, 1., n);
    vec_set_scalar(w->E, 1., m);
    vec_set_scalar(w->Einv, 1., m);
  }
  set_rho_vec(w);
  vec_set_scalar(w->x, 0., n);
  vec_set_scalar(w->z, 0., m);
  vec_set_scalar(w->y, 0., m);
  return factor_kkt(w);
}

/* OSQP 0.6 osqp_solve main loop + post-loop checks, from the iterates currently in `w` (zero
 * after ws_setup = cold start; the previous solution = warm start). */
static int ws_admm(osqp_ws* w, int fail, orc_trace_entry* trace, int32_t max_trace, int32_t* n_trace) {
  const mpcqp_params* prm = w->st;
  int ntr = 0;
  int iter = 0, can_check_termination = 0;
  w->status = MPCQP_STATUS_UNSOLVED;
  w->rho_updates = 0; /* reset_info */
  if (!fail) {
    for (iter = 1; iter <= prm->max_iter; iter++) {
      double* t;
      t = w->x; w->x = w->x_prev; w->x_prev = t; /* swap_vectors */
      t = w->z; w->z = w->z_prev; w->z_prev = t;
      update_xz_tilde(w);
      update_x(w);
      update_z(w);
      update_y(w);
      can_check_termination = prm->check_termination && (iter % prm->check_termination == 0);
      double ep = 0, ed = 0;
      int done = 0;
      if (can_check_termination) {
        update_info(w, iter);
        done = check_termination(w, 0, &ep, &ed);
      }
      int rho_upd = 0;
      if (!done && prm->adaptive_rho && prm->adaptive_rho_interval &&
          (iter % prm->adaptive_rho_interval == 0)) {
        if (!can_check_termination) update_info(w, iter);
        int before = w->rho_updates;
        if (adapt_rho(w)) {
          fail = 1;
        }
        rho_upd = w->rho_updates != before;
      }
      if (trace && can_check_termination && ntr < max_trace) {
        orc_trace_entry* e = &trace[ntr++];
        e->iter = iter;
        e->rho_updated = rho_upd;
        e->pri_res = w->pri_res;
        e->dua_res = w->dua_res;
        e->eps_prim = ep;
        e->eps_dual = ed;
        e->rho = w->rho;
      }
      if (done || fail) break;
    }
    if (!can_check_termination && !fail) {
      update_info(w, iter - 1);
      check_termination(w, 0, NULL, NULL);
    }
    if (w->status == MPCQP_STATUS_UNSOLVED && !fail) {
      if (!check_termination(w, 1, NULL, NULL)) w->status = MPCQP_STATUS_MAX_ITER_REACHED;
    }
  }
  if (fail) w->status = MPCQP_STATUS_NON_CVX;
  if (has_solution(w->status)) w->obj_val = compute_obj_val(w, w->x);
  if (n_trace) *n_trace = ntr;
  return fail;
}

/* store_solution + unscale_solution (x = D x) and compute_grf's extraction
 * (A1RobotControl.cpp:555-561). */
static void ws_extract(const osqp_ws* w, const double* rec, mpcqp_result* res, double* sol) {
  const int n = w->n;
  double* xs = (double*)malloc(sizeof(double) * n);
  if (has_solution(w->status)) {
    for (int i = 0; i < n; ++i) xs[i] = w->st->scaling ? w->D[i] * w->x[i] : w->x[i];
  } else {
    for (int i = 0; i < n; ++i) xs[i] = OSQP_NAN;
  }
  const double* R = rec + MPCQP_REC_ROT;
  for (int k = 0; k < ND; ++k) res->u0[k] = xs[k];
  for (int leg = 0; leg < NL; ++leg) {
    const double* f = xs + 3 * leg;
    double nrm = sqrt(f[0] * f[0] + f[1] * f[1] + f[2] * f[2]);
    if (isnan(nrm)) {
      res->nan_legs |= 1 << leg;
      for (int r = 0; r < 3; ++r) res->f_body[3 * leg + r] = 0.0;
    } else {
      for (int r = 0; r < 3; ++r) {
        double s = 0.0;
        for (int c = 0; c < 3; ++c) s += R[c * 3 + r] * f[c];
        res->f_body[3 * leg + r] = s;
      }
    }
  }
  if (sol) memcpy(sol, xs, sizeof(double) * n);
  res->obj_val = w->obj_val;
  res->pri_res = w->pri_res;
  res->dua_res = w->dua_res;
  res->rho = w->rho;
  res->status = w->status;
  res->iters = w->iter;
  res->rho_updates = w->rho_updates;
  free(xs);
}

int32_t orc_solve(const mpcqp_params* prm, const double* rec, mpcqp_result* res, double* sol,
                  orc_trace_entry* trace, int32_t max_trace, int32_t* n_trace) {
  const int N = prm->horizon;
  if (N < 1 || !res) return MPCQP_ERR_INVALID_ARG;
  const int n = ND * N;
  memset(res, 0, sizeof(*res));
  if (n_trace) *n_trace = 0;
  if (record_has_nonfinite(rec, N)) {
    res->status = MPCQP_STATUS_NAN_INPUT;
    res->nan_legs = 0xF;
    if (sol)
      for (int i = 0; i < n; ++i) sol[i] = OSQP_NAN;
    return MPCQP_OK;
  }
  osqp_ws w;
  ws_alloc(&w, prm);
  int fail = ws_setup(&w, rec);
  ws_admm(&w, fail, trace, max_trace, n_trace);
  ws_extract(&w, rec, res, sol);
  ws_free(&w);
  return MPCQP_OK;
}

/* ============================================================================================
 * Warm start across control ticks: the persistent solver of A1RobotControl.h:67 driven as in
 * A1RobotControl.cpp:520-540 (OsqpEigen 0.6.3 on OSQP 0.6).
 * ========================================================================================== */

/* OSQP 0.6 unscale_data (scaling.c) */
static void unscale_data(osqp_ws* w) {
  const int n = w->n, m = w->m;
  mat_mult_scalar(&w->P, w->cinv);
  mat_premult_diag(&w->P, w->Dinv);
  mat_postmult_diag(&w->P, w->Dinv);
  vec_mult_scalar(w->q, w->cinv, n);
  vec_ew_prod(w->Dinv, w->q, w->q, n);
  mat_premult_diag(&w->A, w->Einv);
  mat_postmult_diag(&w->A, w->Dinv);
  vec_ew_prod(w->Einv, w->l, w->l, m);
  vec_ew_prod(w->Einv, w->u, w->u, m);
}

/* OSQP 0.6 update_rho_vec (auxil.c), called by osqp_update_{lower,upper}_bound: a constraint
 * whose type changed gets the current settings rho, and the KKT matrix is refactored. */
static int update_rho_vec(osqp_ws* w) {
  int changed = 0;
  for (int i = 0; i < w->m; ++i) {
    int t;
    if ((w->l[i] < -OSQP_INFTY * MIN_SCALING) && (w->u[i] > OSQP_INFTY * MIN_SCALING))
      t = -1;
    else if (w->u[i] - w->l[i] < RHO_TOL)
      t = 1;
    else
      t = 0;
    if (t == w->constr_type[i]) continue;
    w->constr_type[i] = t;
    w->rho_vec[i] = t == -1 ? RHO_MIN : t == 1 ? RHO_EQ_OVER_RHO_INEQ * w->rho : w->rho;
    w->rho_inv_vec[i] = 1. / w->rho_vec[i];
    changed = 1;
  }
  return changed ? factor_kkt(w) : 0;
}

/* OSQP 0.6 osqp_update_{lower,upper}_bound: replace, scale by E, check l <= u (a violation
 * returns before update_rho_vec and is ignored by the reference), update_rho_vec. */
static int update_bound(osqp_ws* w, double* dst, const double* src) {
  const int m = w->m;
  memcpy(dst, src, sizeof(double) * m);
  if (w->st->scaling) vec_ew_prod(w->E, dst, dst, m);
  for (int i = 0; i < m; ++i)
    if (w->l[i] > w->u[i]) return 1;
  return update_rho_vec(w);
}

/* OsqpEigen 0.6.3 Solver::updateHessianMatrix + updateGradient + updateLowerBound +
 * updateUpperBound (A1RobotControl.cpp:532-535) on the QP of `rec`. */
static int ws_update(osqp_ws* w, const double* rec) {
  const int n = w->n, m = w->m;
  double* Pd = (double*)malloc(sizeof(double) * (size_t)n * n);
  double* qn = (double*)malloc(sizeof(double) * n);
  double* ln = (double*)malloc(sizeof(double) * m);
  double* un = (double*)malloc(sizeof(double) * m);
  orc_build_qp(w->st, rec, Pd, qn, ln, un, NULL);
  int fail = 0;
  csc Pn = dense_to_csc_upper(Pd, n);
  /* The reference sets the constraint matrix once, at initSolver (A1RobotControl.cpp:526-530), with
   * ConvexMpc's fixed mu = 0.3 (ConvexMpc.cpp:8).  mu is a per-record input here, so a changed mu
   * is treated like a changed Hessian pattern: the solver is re-initialized with the new A (the
   * update_P branch would otherwise keep the old, latched cone). */
  int same = Pn.p[n] == w->P.p[n] && rec[MPCQP_REC_MU] == w->mu;
  for (int j = 0; same && j <= n; ++j) same = Pn.p[j] == w->P.p[j];
  for (int k = 0; same && k < Pn.p[n]; ++k) same = Pn.i[k] == w->P.i[k];
  if (same) {
    /* osqp_update_P: unscale_data, new P values, scale_data (q, l, u and A are the old data,
     * unscaled: the cost scaling c of this tick depends on the previous gradient), refactor */
    if (w->st->scaling) unscale_data(w);
    memcpy(w->P.x, Pn.x, sizeof(double) * Pn.p[n]);
    if (w->st->scaling) scale_data(w);
    fail |= factor_kkt(w);
    w->last_update_mode = 1;
  } else {
    /* sparsity changed: OsqpEigen re-initializes the solver and restores the unscaled primal
     * and dual variables through osqp_warm_start_x / _y */
    double* xu = (double*)malloc(sizeof(double) * n);
    double* yu = (double*)malloc(sizeof(double) * m);
    for (int i = 0; i < n; ++i) xu[i] = w->st->scaling ? w->D[i] * w->x[i] : w->x[i];
    for (int i = 0; i < m; ++i) yu[i] = w->st->scaling ? (w->E[i] * w->y[i]) * w->cinv : w->y[i];
    fail |= ws_setup(w, rec);
    for (int i = 0; i < n; ++i) w->x[i] = w->st->scaling ? w->Dinv[i] * xu[i] : xu[i];
    mat_vec(&w->A, w->x, w->z, 0);
    for (int i = 0; i < m; ++i) w->y[i] = w->st->scaling ? w->c * (w->Einv[i] * yu[i]) : yu[i];
    free(xu);
    free(yu);
    w->last_update_mode = 2;
  }
  csc_free(&Pn);
  /* osqp_update_lin_cost */
  memcpy(w->q, qn, sizeof(double) * n);
  if (w->st->scaling) {
    vec_ew_prod(w->D, w->q, w->q, n);
    vec_mult_scalar(w->q, w->c, n);
  }
  /* osqp_update_lower_bound, then osqp_update_upper_bound (no clipping on update) */
  fail |= update_bound(w, w->l, ln);
  fail |= update_bound(w, w->u, un);
  free(Pd);
  free(qn);
  free(ln);
  free(un);
  return fail;
}

struct orc_solver {
  osqp_ws w;
  int initialized;
  mpcqp_params prm;
  int last_mode; /* branch of the last step: 0 setup (initSolver), 1 osqp_update_P, 2 re-init */
  /* TEST ONLY (orc_solver_step_image): where the next step copies its scaled data */
  double *img_D, *img_E, *img_q, *img_c;
  int32_t* img_mode;
};

orc_solver* orc_solver_new(const mpcqp_params* prm) {
  orc_solver* s = (orc_solver*)calloc(1, sizeof(orc_solver));
  s->prm = *prm;
  return s;
}
void orc_solver_free(orc_solver* s) {
  if (!s) return;
  if (s->initialized) ws_free(&s->w);
  free(s);
}
void orc_solver_reset(orc_solver* s) {
  if (s->initialized) ws_free(&s->w);
  s->initialized = 0;
}

int32_t orc_solver_step(orc_solver* s, const double* rec, mpcqp_result* res, double* sol,
                        orc_trace_entry* trace, int32_t max_trace, int32_t* n_trace) {
  const int N = s->prm.horizon;
  memset(res, 0, sizeof(*res));
  if (n_trace) *n_trace = 0;
  if (record_has_nonfinite(rec, N)) { /* engine contract: state untouched, NaN result */
    res->status = MPCQP_STATUS_NAN_INPUT;
    res->nan_legs = 0xF;
    if (sol)
      for (int i = 0; i < ND * N; ++i) sol[i] = OSQP_NAN;
    return MPCQP_OK;
  }
  int fail;
  if (!s->initialized) {
    ws_alloc(&s->w, &s->prm);
    fail = ws_setup(&s->w, rec);
    s->initialized = 1;
    s->last_mode = 0;
  } else {
    fail = ws_update(&s->w, rec);
    s->last_mode = s->w.last_update_mode;
  }
  if (s->img_D) { /* TEST ONLY: the scaled data this tick's ADMM starts from */
    memcpy(s->img_D, s->w.D, sizeof(double) * s->w.n);
    memcpy(s->img_E, s->w.E, sizeof(double) * s->w.m);
    memcpy(s->img_q, s->w.q, sizeof(double) * s->w.n);
    *s->img_c = s->w.c;
    *s->img_mode = s->last_mode;
    s->img_D = NULL;
  }
  ws_admm(&s->w, fail, trace, max_trace, n_trace);
  ws_extract(&s->w, rec, res, sol);
  return MPCQP_OK;
}

/* T ticks of `batch` independent robots: recs [T][batch][rec], res [T][batch]. */
typedef struct {
  const mpcqp_params* prm;
  const double* recs;
  mpcqp_result* res;
  int T, batch, begin, end, rec_size;
} seq_arg;
static void* seq_worker(void* p) {
  seq_arg* a = (seq_arg*)p;
  for (int b = a->begin; b < a->end; ++b) {
    orc_solver* s = orc_solver_new(a->prm);
    for (int t = 0; t < a->T; ++t)
      orc_solver_step(s, a->recs + ((size_t)t * a->batch + b) * a->rec_size, &a->res[(size_t)t * a->batch + b],
                      NULL, NULL, 0, NULL);
    orc_solver_free(s);
  }
  return NULL;
}
int32_t orc_solve_sequence(const mpcqp_params* prm, const double* recs, int32_t T, int32_t batch,
                           mpcqp_result* res, int32_t nthreads) {
  if (T < 0 || batch < 0 || nthreads < 1) return MPCQP_ERR_INVALID_ARG;
  if (nthreads > batch) nthreads = batch > 0 ? batch : 1;
  pthread_t* th = (pthread_t*)malloc(sizeof(pthread_t) * nthreads);
  seq_arg* args = (seq_arg*)malloc(sizeof(seq_arg) * nthreads);
  for (int t = 0; t < nthreads; ++t) {
    args[t].prm = prm;
    args[t].recs = recs;
    args[t].res = res;
    args[t].T = T;
    args[t].batch = batch;
    args[t].begin = (int)((long long)batch * t / nthreads);
    args[t].end = (int)((long long)batch * (t + 1) / nthreads);
    args[t].rec_size = MPCQP_REC_SIZE(prm->horizon);
    pthread_create(&th[t], NULL, seq_worker, &args[t]);
  }
  for (int t = 0; t < nthreads; ++t) pthread_join(th[t], NULL);
  free(th);
  free(args);
  return MPCQP_OK;
}

/* ============================================================================================
 * Downstream torque map: A1RobotControl::compute_joint_torques (A1RobotControl.cpp:289-319)
 * ========================================================================================== */

/* Eigen PartialPivLU<Matrix3d>::solve: column-wise partial pivoting (first maximal |a_ik|,
 * rows swapped whole), unit-lower forward and upper backward substitution. */
static void lu3_solve(const double* J, const double* b, double* x) {
  double a[9], y[3];
  int perm[3] = {0, 1, 2};
  memcpy(a, J, sizeof(a));
  for (int k = 0; k < 3; ++k) {
    int p = k;
    double best = c_absval(a[3 * k + k]);
    for (int i = k + 1; i < 3; ++i)
      if (c_absval(a[3 * i + k]) > best) {
        best = c_absval(a[3 * i + k]);
        p = i;
      }
    if (p != k) {
      for (int j = 0; j < 3; ++j) {
        double t = a[3 * k + j];
        a[3 * k + j] = a[3 * p + j];
        a[3 * p + j] = t;
      }
      int t = perm[k];
      perm[k] = perm[p];
      perm[p] = t;
    }
    if (best != 0.0)
      for (int i = k + 1; i < 3; ++i) a[3 * i + k] /= a[3 * k + k];
    for (int i = k + 1; i < 3; ++i)
      for (int j = k + 1; j < 3; ++j) a[3 * i + j] -= a[3 * i + k] * a[3 * k + j];
  }
  for (int i = 0; i < 3; ++i) y[i] = b[perm[i]];
  for (int i = 1; i < 3; ++i)
    for (int j = 0; j < i; ++j) y[i] -= a[3 * i + j] * y[j];
  for (int i = 2; i >= 0; --i) {
    double s = y[i];
    for (int j = i + 1; j < 3; ++j) s -= a[3 * i + j] * x[j];
    x[i] = s / a[3 * i + i];
  }
}

void orc_joint_torques(const double* tq, const double* f_grf, int32_t* counter, double* tau) {
  double jt[12];
  *counter += 1;                 /* mpc_init_counter++ (:292) */
  if (*counter < 10) {           /* first ticks: zero torques (:294-295) */
    for (int k = 0; k < 12; ++k) tau[k] = 0.0;
    return;
  }
  for (int leg = 0; leg < NL; ++leg) {
    const double* J = tq + MPCQP_TQ_JFOOT + 9 * leg; /* j_foot.block<3,3>(3i,3i), row-major */
    double* t = jt + 3 * leg;
    if (tq[MPCQP_TQ_CONTACTS + leg] != 0.0) {        /* stance: tau = J' (-f_grf) (:303) */
      for (int c = 0; c < 3; ++c) {
        double s = 0.0;
        for (int r = 0; r < 3; ++r) s += J[3 * r + c] * -f_grf[3 * leg + r];
        t[c] = s;
      }
    } else {                                         /* swing: J tau = km .* f_kin (:306-307) */
      double ft[3];
      for (int r = 0; r < 3; ++r) ft[r] = tq[MPCQP_TQ_KM + r] * tq[MPCQP_TQ_FKIN + 3 * leg + r];
      lu3_solve(J, ft, t);
    }
  }
  for (int k = 0; k < 12; ++k) {
    double v = jt[k] + tq[MPCQP_TQ_GRAV + k];        /* += torques_gravity (:311) */
    if (!isnan(v)) tau[k] = v;                       /* NaN guard (:313-317) */
  }
}

/* ============================================================================================
 * Single-step QP balance controller (stance_leg_control_type == 0)
 * ========================================================================================== */

/* A1RobotControl.cpp:321-332 (euler error, yaw wrapped at 1.5 pi with the literal 3.1415926),
 * :379-392 (root_acc), :394-407 (inertia_inv, H, g), ctor :27-44 (constraint rows), :410-414
 * (fz bounds from contacts).  OsqpEigen::INFTY lower bounds on the 16 friction rows (:31-43),
 * upper bounds 0 (setZero, :21). */
void orc_balance_build_qp(const mpcqp_balance_params* bp, const double* rec, double* P, double* q,
                          double* l, double* u, double* A) {
  const double* R = rec + MPCQP_BAL_ROT;
  const double* Rz = rec + MPCQP_BAL_ROT_Z;
  double ee[3];
  for (int k = 0; k < 3; ++k) ee[k] = rec[MPCQP_BAL_EULER_D + k] - rec[MPCQP_BAL_EULER + k];
  if (ee[2] > 3.1415926 * 1.5)
    ee[2] = rec[MPCQP_BAL_EULER_D + 2] - 3.1415926 * 2 - rec[MPCQP_BAL_EULER + 2];
  else if (ee[2] < -3.1415926 * 1.5)
    ee[2] = rec[MPCQP_BAL_EULER_D + 2] + 3.1415926 * 2 - rec[MPCQP_BAL_EULER + 2];
  double acc[6], tv[3], tw[3];
  for (int i = 0; i < 3; ++i) { /* R^T v */
    double sv = 0.0, sw = 0.0;
    for (int k = 0; k < 3; ++k) {
      sv += R[k * 3 + i] * rec[MPCQP_BAL_LIN_VEL + k];
      sw += R[k * 3 + i] * rec[MPCQP_BAL_ANG_VEL + k];
    }
    tv[i] = rec[MPCQP_BAL_KD_LIN + i] * (rec[MPCQP_BAL_LIN_VEL_D + i] - sv);
    tw[i] = sw;
  }
  for (int i = 0; i < 3; ++i) {
    double s = 0.0;
    for (int k = 0; k < 3; ++k) s += R[i * 3 + k] * tv[k];
    acc[i] = rec[MPCQP_BAL_KP_LIN + i] * (rec[MPCQP_BAL_POS_D + i] - rec[MPCQP_BAL_POS + i]) + s;
    acc[3 + i] = rec[MPCQP_BAL_KP_ANG + i] * ee[i] +
                 rec[MPCQP_BAL_KD_ANG + i] * (rec[MPCQP_BAL_ANG_VEL_D + i] - tw[i]);
  }
  acc[2] += rec[MPCQP_BAL_MASS] * 9.8;
  /* inertia_inv M (6 x 12): [I_3; Rz^T skew(foot_i)] per leg */
  double M[6][12];
  for (int leg = 0; leg < NL; ++leg) {
    const double* f = rec + MPCQP_BAL_FEET + 3 * leg;
    const double S[9] = {0.0, -f[2], f[1], f[2], 0.0, -f[0], -f[1], f[0], 0.0}; /* Utils.cpp:35-41 */
    for (int a = 0; a < 3; ++a)
      for (int b = 0; b < 3; ++b) {
        M[a][3 * leg + b] = a == b ? 1.0 : 0.0;
        double s = 0.0;
        for (int k = 0; k < 3; ++k) s += Rz[k * 3 + a] * S[k * 3 + b];
        M[3 + a][3 * leg + b] = s;
      }
  }
  for (int i = 0; i < ND; ++i) {
    for (int j = 0; j < ND; ++j) {
      double s = 0.0;
      for (int k = 0; k < 6; ++k) s += (M[k][i] * bp->q_diag[k]) * M[k][j];
      P[i * ND + j] = (i == j ? bp->r : 0.0) + s;
    }
    double g = 0.0;
    for (int k = 0; k < 6; ++k) g += (-M[k][i] * bp->q_diag[k]) * acc[k];
    q[i] = g;
  }
  memset(A, 0, sizeof(double) * CD * ND);
  for (int leg = 0; leg < NL; ++leg) {
    const double c = rec[MPCQP_BAL_CONTACTS + leg] != 0.0 ? 1.0 : 0.0;
    A[leg * ND + 3 * leg + 2] = 1.0;
    l[leg] = c * bp->f_min;
    u[leg] = c * bp->f_max;
    for (int r = 0; r < 4; ++r) {
      const int row = NL + 4 * leg + r;
      A[row * ND + 3 * leg + (r >> 1)] = (r & 1) ? -1.0 : 1.0;
      A[row * ND + 3 * leg + 2] = -bp->mu;
      l[row] = -OSQP_INFTY;
      u[row] = 0.0;
    }
  }
}

int32_t orc_balance_solve(const mpcqp_params* prm, const mpcqp_balance_params* bp, const double* rec,
                          mpcqp_result* res) {
  if (!prm || !bp || !rec || !res) return MPCQP_ERR_INVALID_ARG;
  memset(res, 0, sizeof(*res));
  for (int k = 0; k < MPCQP_BAL_SIZE - 1; ++k)
    if (!isfinite(rec[k])) {
      res->status = MPCQP_STATUS_NAN_INPUT;
      res->nan_legs = 0xF;
      for (int i = 0; i < ND; ++i) res->u0[i] = res->f_body[i] = OSQP_NAN;
      return MPCQP_OK;
    }
  mpcqp_params p1 = *prm; /* a new OsqpEigen::Solver per tick, warm start off (:416-421) */
  p1.horizon = 1;
  p1.warm_start = 0;
  osqp_ws w;
  ws_alloc(&w, &p1);
  double* Pd = (double*)malloc(sizeof(double) * ND * ND);
  double* Ad = (double*)malloc(sizeof(double) * CD * ND);
  orc_balance_build_qp(bp, rec, Pd, w.q, w.l, w.u, Ad);
  int fail = ws_setup_dense(&w, Pd, Ad);
  ws_admm(&w, fail, NULL, 0, NULL);
  /* getSolution (NaN unless a solution exists) and foot_forces_grf = R^T x per leg (:440-443) */
  const double* R = rec + MPCQP_BAL_ROT;
  double xs[ND];
  for (int i = 0; i < ND; ++i) xs[i] = has_solution(w.status) ? w.D[i] * w.x[i] : OSQP_NAN;
  for (int leg = 0; leg < NL; ++leg) {
    const double* f = xs + 3 * leg;
    if (isnan(f[0] + f[1] + f[2])) res->nan_legs |= 1 << leg;
    for (int r = 0; r < 3; ++r) {
      double s = 0.0;
      for (int c = 0; c < 3; ++c) s += R[c * 3 + r] * f[c];
      res->f_body[3 * leg + r] = s;
    }
  }
  memcpy(res->u0, xs, sizeof(xs));
  res->obj_val = w.obj_val;
  res->pri_res = w.pri_res;
  res->dua_res = w.dua_res;
  res->rho = w.rho;
  res->status = w.status;
  res->iters = w.iter;
  res->rho_updates = w.rho_updates;
  ws_free(&w);
  return MPCQP_OK;
}

/* ============================================================================================
 * Batch over host threads (CPU baseline)
 * ========================================================================================== */

typedef struct {
  const mpcqp_params* prm;
  const double* recs;
  mpcqp_result* res;
  double* sols;
  int begin, end, rec_size, n;
} batch_arg;

static void* batch_worker(void* p) {
  batch_arg* a = (batch_arg*)p;
  for (int b = a->begin; b < a->end; ++b)
    orc_solve(a->prm, a->recs + (size_t)b * a->rec_size, &a->res[b],
              a->sols ? a->sols + (size_t)b * a->n : NULL, NULL, 0, NULL);
  return NULL;
}

int32_t orc_solve_batch(const mpcqp_params* prm, const double* recs, int32_t batch,
                        mpcqp_result* res, double* sols, int32_t nthreads) {
  if (batch < 0 || nthreads < 1) return MPCQP_ERR_INVALID_ARG;
  if (nthreads > batch) nthreads = batch > 0 ? batch : 1;
  pthread_t* th = (pthread_t*)malloc(sizeof(pthread_t) * nthreads);
  batch_arg* args = (batch_arg*)malloc(sizeof(batch_arg) * nthreads);
  const int rs = MPCQP_REC_SIZE(prm->horizon);
  for (int t = 0; t < nthreads; ++t) {
    args[t].prm = prm;
    args[t].recs = recs;
    args[t].res = res;
    args[t].sols = sols;
    args[t].begin = (int)((long long)batch * t / nthreads);
    args[t].end = (int)((long long)batch * (t + 1) / nthreads);
    args[t].rec_size = rs;
    args[t].n = ND * prm->horizon;
    pthread_create(&th[t], NULL, batch_worker, &args[t]);
  }
  for (int t = 0; t < nthreads; ++t) pthread_join(th[t], NULL);
  free(th);
  free(args);
  return MPCQP_OK;
}

typedef struct {
  const mpcqp_params* prm;
  const mpcqp_balance_params* bp;
  const double* recs;
  mpcqp_result* res;
  int begin, end;
} bal_arg;

static void* bal_worker(void* p) {
  bal_arg* a = (bal_arg*)p;
  for (int b = a->begin; b < a->end; ++b)
    orc_balance_solve(a->prm, a->bp, a->recs + (size_t)b * MPCQP_BAL_SIZE, &a->res[b]);
  return NULL;
}

int32_t orc_balance_solve_batch(const mpcqp_params* prm, const mpcqp_balance_params* bp, const double* recs,
                                int32_t batch, mpcqp_result* res, int32_t nthreads) {
  if (batch < 0 || !prm || !bp) return MPCQP_ERR_INVALID_ARG;
  if (nthreads < 1) nthreads = 1;
  if (nthreads > batch) nthreads = batch > 0 ? batch : 1;
  pthread_t th[256];
  bal_arg args[256];
  if (nthreads > 256) nthreads = 256;
  for (int t = 0; t < nthreads; ++t) {
    args[t] = (bal_arg){prm, bp, recs, res, (int)((int64_t)batch * t / nthreads),
                        (int)((int64_t)batch * (t + 1) / nthreads)};
    if (nthreads == 1)
      bal_worker(&args[t]);
    else
      pthread_create(&th[t], NULL, bal_worker, &args[t]);
  }
  if (nthreads > 1)
    for (int t = 0; t < nthreads; ++t) pthread_join(th[t], NULL);
  return MPCQP_OK;
}

/* TEST ONLY — the scaled problem data an OSQP solve of `rec` starts from (osqp_setup: bound
 * clipping, scale_data): D [n], E [m], the scaled gradient q~ = c D q [n] and the cost scale c.
 * Checks the device scale_kernel's image (tests/test_gpu_scale_image.py). */
int32_t orc_scale_image(const mpcqp_params* prm, const double* rec, double* D, double* E, double* q, double* c) {
  const int N = prm->horizon;
  if (N < 1 || record_has_nonfinite(rec, N)) return MPCQP_ERR_INVALID_ARG;
  osqp_ws w;
  ws_alloc(&w, prm);
  ws_setup(&w, rec);
  memcpy(D, w.D, sizeof(double) * w.n);
  memcpy(E, w.E, sizeof(double) * w.m);
  memcpy(q, w.q, sizeof(double) * w.n);
  *c = w.c;
  ws_free(&w);
  return MPCQP_OK;
}

/* TEST ONLY — orc_solver_step that also reports the scaled data the tick's ADMM starts from (after
 * initSolver / osqp_update_P / re-init and osqp_update_lin_cost) and the branch taken. */
int32_t orc_solver_step_image(orc_solver* s, const double* rec, mpcqp_result* res, double* D, double* E, double* q,
                              double* c, int32_t* mode) {
  s->img_D = D;
  s->img_E = E;
  s->img_q = q;
  s->img_c = c;
  s->img_mode = mode;
  const int32_t rc = orc_solver_step(s, rec, res, NULL, NULL, 0, NULL);
  s->img_D = NULL;
  return rc;
}
