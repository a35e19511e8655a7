/*
 * mpcqp.h — C ABI of the MI355X-native batched convex-MPC QP engine.
 *
 * Drop-in boundary for the per-control-cycle ground-reaction-force (GRF) solve of
 * zerenluo123/Go1-QP-MPC-Controller.  The reference performs, per robot and per tick:
 *
 *   ConvexMpc ctor/reset                      src/a1_cpp/src/ConvexMpc.cpp:7-108
 *   calculate_A_mat_c / calculate_B_mat_c     src/a1_cpp/src/ConvexMpc.cpp:110-143
 *   state_space_discretization                src/a1_cpp/src/ConvexMpc.cpp:145-156
 *   calculate_qp_mats (A_qp, B_qp, H, g, l/u) src/a1_cpp/src/ConvexMpc.cpp:158-245
 *   OsqpEigen setup + solve (OSQP 0.6.x)      src/a1_cpp/src/A1RobotControl.cpp:522-555
 *   extraction f_i = R^T u[3i:3i+3]           src/a1_cpp/src/A1RobotControl.cpp:555-561
 *
 * Every entry point below replaces one of those interfaces for a whole *batch* of robots.
 * The header is plain C: no HIP, Eigen or torch types.  Streams are passed as opaque
 * `void*` (a hipStream_t; NULL = the default stream).
 *
 * Arithmetic is IEEE binary64 (the reference computes in double everywhere).
 *
 * Threading: a handle is bound to one device and is not thread-safe; use one handle per
 * host thread / stream.  Inputs are read once per call (snapshot semantics).
 * Errors never throw across this boundary: every function returns an mpcqp_error code.
 */
#ifndef MPCQP_H_
#define MPCQP_H_

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- dimensions (reference: src/a1_cpp/src/A1Params.h:26-34) ------------------------ */
#define MPCQP_STATE_DIM 13      /* MPC_STATE_DIM: [rpy, p, w, v, g]                       */
#define MPCQP_NUM_LEG 4         /* NUM_LEG (FL, FR, RL, RR)                               */
#define MPCQP_NUM_DOF 12        /* NUM_DOF: 3 GRF components x 4 legs per horizon step     */
#define MPCQP_CONSTRAINT_DIM 20 /* MPC_CONSTRAINT_DIM: 5 friction-pyramid rows x 4 legs    */
#define MPCQP_MAX_HORIZON 20    /* 1..20: one wavefront per robot (Schur form N<=10, Riccati N>10) */
#define MPCQP_OSQP_INFTY 1e30   /* OsqpEigen::INFTY == OSQP_INFTY (OSQP 0.6 constants.h)  */

/* ---- per-instance problem record (all binary64, contiguous) ----------------------------
 * One record describes exactly the inputs ConvexMpc::calculate_qp_mats and the MPC branch
 * of A1RobotControl::compute_grf consume.  Offsets are in doubles.                        */
#define MPCQP_REC_X0 0        /* [13] mpc_states x0 (A1RobotControl.cpp:452-456)                 */
#define MPCQP_REC_EULER 13    /* [3]  euler given to calculate_A_mat_c (only yaw is used, :116)  */
#define MPCQP_REC_ROT 16      /* [9]  root_rot_mat, row-major (calculate_B_mat_c arg)            */
#define MPCQP_REC_INERTIA 25  /* [9]  trunk inertia, body frame, row-major                       */
#define MPCQP_REC_MASS 34     /* robot_mass                                                       */
#define MPCQP_REC_MU 35       /* friction coefficient (ConvexMpc.cpp:8 hard-codes 0.3)            */
#define MPCQP_REC_FZMIN 36    /* fz_min (ConvexMpc.cpp:223: 0)                                    */
#define MPCQP_REC_FZMAX 37    /* fz_max (ConvexMpc.cpp:224: 180)                                  */
#define MPCQP_REC_DT 38       /* mpc_dt used by state_space_discretization (A1RobotControl:462)  */
#define MPCQP_REC_CONTACTS 39 /* [4]  contacts[i] as 0.0 / 1.0 (bounds, ConvexMpc.cpp:225-241)    */
#define MPCQP_REC_XREF 44     /* [13N] mpc_states_d                                               */
/* feet: [N][4][3] foot_pos used for B_c at horizon step i (foot_pos_abs in compute_grf, the
 * per-step shifted foot_pos_abs_mpc in test_mpc.cpp:105-115), at MPCQP_REC_XREF + 13N           */
#define MPCQP_REC_FEET(N) (MPCQP_REC_XREF + 13 * (N))
#define MPCQP_REC_SIZE(N) (MPCQP_REC_XREF + 25 * (N) + ((N)&1))

/* ---- solver settings: OSQP 0.6 defaults + the reference's overrides -------------------
 * (A1RobotControl.cpp:522-538 sets only verbosity=false and warm_start; everything else
 * is osqp_set_default_settings).  adaptive_rho_interval: OSQP's 0 means "derive from
 * wall-clock" (non-reproducible); the engine requires a fixed interval (default 25).      */
typedef struct mpcqp_params {
  int32_t horizon;                /* N, 1..MPCQP_MAX_HORIZON (PLAN_HORIZON = 10)            */
  int32_t max_iter;               /* 4000                                                   */
  int32_t scaling;                /* 10 Ruiz passes                                          */
  int32_t check_termination;      /* 25                                                      */
  int32_t adaptive_rho;           /* 1                                                       */
  int32_t adaptive_rho_interval;  /* 25 (fixed; see above)                                   */
  int32_t scaled_termination;     /* 0                                                       */
  int32_t warm_start;             /* 0: cold start every solve (test_mpc.cpp:133)            */
  double q_weights[MPCQP_STATE_DIM]; /* ConvexMpc ctor arg; Q = diag(2 q) tiled (:16-23)    */
  double r_weights[MPCQP_NUM_DOF];   /* ConvexMpc ctor arg; R = diag(2 r) tiled (:37-44)    */
  double rho;                     /* 0.1                                                     */
  double sigma;                   /* 1e-6                                                    */
  double alpha;                   /* 1.6                                                     */
  double eps_abs, eps_rel;        /* 1e-3, 1e-3                                              */
  double eps_prim_inf, eps_dual_inf; /* 1e-4, 1e-4                                           */
  double adaptive_rho_tolerance;  /* 5                                                       */
} mpcqp_params;

/* ---- per-instance result --------------------------------------------------------------- */
typedef struct mpcqp_result {
  double u0[MPCQP_NUM_DOF];     /* solution.segment(0,12): world-frame GRF of horizon step 0 */
  double f_body[MPCQP_NUM_DOF]; /* compute_grf output: R^T u0[3i:3i+3] per leg (leg-major);
                                   legs whose norm is NaN are left 0 and flagged in nan_legs  */
  double obj_val;               /* unscaled objective 1/2 x'Px + q'x (OSQP info->obj_val)     */
  double pri_res, dua_res;      /* unscaled residuals at the last termination check          */
  double rho;                   /* final rho                                                  */
  int32_t status;               /* MPCQP_STATUS_* (numerically equal to OSQP 0.6 status_val)  */
  int32_t iters;                /* OSQP info->iter                                            */
  int32_t rho_updates;          /* OSQP info->rho_updates                                     */
  int32_t nan_legs;             /* bit i set: leg i solution had a NaN norm                   */
} mpcqp_result;

/* OSQP 0.6 status values (constants.h) */
enum {
  MPCQP_STATUS_SOLVED = 1,
  MPCQP_STATUS_SOLVED_INACCURATE = 2,
  MPCQP_STATUS_PRIMAL_INFEASIBLE_INACCURATE = 3,
  MPCQP_STATUS_DUAL_INFEASIBLE_INACCURATE = 4,
  MPCQP_STATUS_MAX_ITER_REACHED = -2,
  MPCQP_STATUS_PRIMAL_INFEASIBLE = -3,
  MPCQP_STATUS_DUAL_INFEASIBLE = -4,
  MPCQP_STATUS_NON_CVX = -7,
  MPCQP_STATUS_NAN_INPUT = -100, /* engine-specific: a NaN/inf in the instance's record      */
  MPCQP_STATUS_UNSOLVED = -10
};

/* call-level error codes */
enum {
  MPCQP_OK = 0,
  MPCQP_ERR_INVALID_ARG = 1,
  MPCQP_ERR_HIP = 2,
  MPCQP_ERR_NO_DEVICE = 3,
  MPCQP_ERR_ALLOC = 4
};

typedef struct mpcqp_handle mpcqp_handle;

/* Fill *p with the reference's settings for horizon N (OSQP 0.6 defaults, Go1 weights from
 * src/go1_rl_ctrl_cpp/src/Go1CtrlStates.hpp:203-249, fixed adaptive-rho interval 25). */
void mpcqp_default_params(mpcqp_params* p, int32_t horizon);

/* Number of doubles in one problem record for horizon N. */
int32_t mpcqp_record_size(int32_t horizon);

/* Replaces the ConvexMpc ctor + OsqpEigen::Solver construction (ConvexMpc.cpp:7-68,
 * A1RobotControl.h:67): uploads weights/settings to `device`. */
int32_t mpcqp_create(const mpcqp_params* params, int32_t device, mpcqp_handle** out);
int32_t mpcqp_destroy(mpcqp_handle* h);

/* Pre-size the handle's device workspace — the scaling image scale_kernel hands to wave_kernel,
 * 56N + 3 binary64 per robot (3.5 KB at N = 10) — and create the internal streams a solve of `batch`
 * robots splits over, so that later mpcqp_solve_batch_device calls with batch <= `batch` neither
 * allocate nor create streams (hipGraph-capture safe). */
int32_t mpcqp_reserve(mpcqp_handle* h, int32_t batch);

/* Replaces calculate_A/B_mat_c + discretization + calculate_qp_mats + OSQP initSolver/solve
 * + extraction (A1RobotControl.cpp:446-561) for `batch` robots.  All pointers are DEVICE
 * pointers; asynchronous on `stream`.
 *   d_records  [batch][mpcqp_record_size(N)]
 *   d_results  [batch] mpcqp_result
 *   d_solution [batch][12N] full unscaled primal solution, or NULL                       */
int32_t mpcqp_solve_batch_device(mpcqp_handle* h, const double* d_records, int32_t batch,
                                 mpcqp_result* d_results, double* d_solution, void* stream);

/* Warm start across control ticks: the reference keeps one OsqpEigen::Solver per controller
 * (A1RobotControl.h:67) with setWarmStart(true) (A1RobotControl.cpp:524); its first tick runs
 * initSolver, later ticks updateHessianMatrix / updateGradient / updateLowerBound /
 * updateUpperBound and solve from the previous x, z, y and adapted rho (:522-540).  The engine
 * keeps that solver state per robot in a caller-owned DEVICE buffer
 *   d_state [batch][mpcqp_warm_state_size(N)] binary64, zero-filled = "not initialized yet",
 * so a robot's slot must follow it from tick to tick (same batch index).  Robots whose record
 * is non-finite leave their slot untouched.  Default (wave) solver path only. */
int32_t mpcqp_warm_state_size(int32_t horizon);
int32_t mpcqp_solve_batch_warm_device(mpcqp_handle* h, const double* d_records, int32_t batch, double* d_state,
                                      mpcqp_result* d_results, double* d_solution, void* stream);

/* Indexed copy of warm-start slots between DEVICE buffers, for callers whose solved robots are a
 * subset of their slots (a mixed-mode batch: the MPC robots' slots gathered into a compact buffer
 * for the warm solve and scattered back after it, as the reference's controller keeps its member
 * solver untouched on QP ticks, A1RobotControl.cpp:377-444).  For i < count:
 *   slot d_dst[d_dst_idx ? d_dst_idx[i] : i] = slot d_src[d_src_idx ? d_src_idx[i] : i],
 * slots of mpcqp_warm_state_size(horizon) doubles, index arrays DEVICE int32 (NULL = identity).
 * Destination slots must be distinct.  Async on `stream`. */
int32_t mpcqp_copy_warm_slots_device(int32_t horizon, const double* d_src, const int32_t* d_src_idx, double* d_dst,
                                     const int32_t* d_dst_idx, int32_t count, void* stream);

/* Host-pointer convenience wrapper (copies in, solves, copies out, synchronizes) on a stream of the
 * handle's own.  That stream is a blocking stream: it waits for work queued before the call on the
 * legacy NULL stream (zeroing warm slots with hipMemset(..) / on torch's default stream is ordered
 * before the solve), but NOT for work on other non-blocking streams — synchronize those first.  One
 * handle must not run a device-pointer solve on another stream concurrently with a host-wrapper
 * call (they share the handle's workspace).  Pinned host buffers (hipHostMalloc / registered) move by one DMA each way;
 * pageable ones through two pinned 2-MiB staging chunks of the handle, host copies overlapping the
 * DMA.  Not for concurrent use of one handle from several threads. */
int32_t mpcqp_solve_batch_host(mpcqp_handle* h, const double* h_records, int32_t batch,
                               mpcqp_result* h_results, double* h_solution);

/* Host-pointer variant of the warm-started solve: records and results on the host (as in
 * mpcqp_solve_batch_host), the solver slots d_state in DEVICE memory (as in
 * mpcqp_solve_batch_warm_device).  This is the per-tick call of a persistent controller-owned
 * solver (A1RobotControl.h:67 member OsqpEigen::Solver, warm start on: A1RobotControl.cpp:522-540);
 * synchronous. */
int32_t mpcqp_solve_batch_warm_host(mpcqp_handle* h, const double* h_records, int32_t batch, double* d_state,
                                    mpcqp_result* h_results, double* h_solution);

/* Formulation only (ConvexMpc::calculate_qp_mats): dense Hessian (full symmetric, row-major
 * [12N][12N]), gradient [12N], bounds l/u [20N] per instance.  DEVICE pointers. */
int32_t mpcqp_build_qp_device(mpcqp_handle* h, const double* d_records, int32_t batch,
                              double* d_P, double* d_q, double* d_l, double* d_u, void* stream);

/* ---- on-device input assembly from raw robot state --------------------
 * One binary64 record per robot holding the A1CtrlStates / Go1CtrlStates fields the MPC branch of
 * compute_grf reads (A1RobotControl.cpp:446-514); matrices row-major, vectors world frame unless
 * noted.  Offsets in doubles.                                                                  */
#define MPCQP_ST_EULER 0      /* [3] root_euler                                                  */
#define MPCQP_ST_POS 3        /* [3] root_pos                                                    */
#define MPCQP_ST_ANG_VEL 6    /* [3] root_ang_vel (world)                                        */
#define MPCQP_ST_LIN_VEL 9    /* [3] root_lin_vel (world)                                        */
#define MPCQP_ST_ROT 12       /* [9] root_rot_mat                                                */
#define MPCQP_ST_EULER_D 21   /* [3] root_euler_d (after terrain adaptation, :335-376)           */
#define MPCQP_ST_POS_D 24     /* [3] root_pos_d                                                  */
#define MPCQP_ST_ANG_VEL_D 27 /* [3] root_ang_vel_d                                              */
#define MPCQP_ST_LIN_VEL_D 30 /* [3] root_lin_vel_d (body frame; :470 rotates it to world)       */
#define MPCQP_ST_FEET 33      /* [4][3] foot_pos_abs column i                                     */
#define MPCQP_ST_MASS 45      /* robot_mass                                                      */
#define MPCQP_ST_INERTIA 46   /* [9] trunk_inertia                                               */
#define MPCQP_ST_MU 55        /* friction coefficient (ConvexMpc.cpp:8: 0.3)                      */
#define MPCQP_ST_FZMIN 56     /* 0                                                               */
#define MPCQP_ST_FZMAX 57     /* 180                                                             */
#define MPCQP_ST_DT 58        /* mpc_dt (:462, 0.0025)                                           */
#define MPCQP_ST_CONTACTS 59  /* [4] contacts[i] as 0.0 / 1.0                                    */
#define MPCQP_ST_SIZE 64      /* 63 used, padded to a multiple of 4 doubles                      */

/* Replaces the host-side x0 / x_ref / horizon-feet assembly of compute_grf (A1RobotControl.cpp:
 * 452-514: mpc_states, root_lin_vel_d_world, mpc_states_d, B_mat_d_list feet) for `batch` robots:
 * d_states [batch][MPCQP_ST_SIZE] -> d_records [batch][mpcqp_record_size(horizon)], DEVICE
 * pointers, async on `stream`.  Chain it before mpcqp_solve_batch_device on the same stream. */
int32_t mpcqp_assemble_records_device(int32_t horizon, const double* d_states, int32_t batch, double* d_records,
                                      void* stream);

/* ---- downstream torque map: A1RobotControl::compute_joint_torques (A1RobotControl.cpp:289-319)
 * One binary64 record per robot (offsets in doubles); FL, FR, RL, RR leg order.             */
#define MPCQP_TQ_JFOOT 0      /* [4][9] j_foot.block<3,3>(3i,3i), row-major (A1CtrlStates.h:410) */
#define MPCQP_TQ_FKIN 36      /* [4][3] foot_forces_kin column i (swing-leg PD force, :220-286)  */
#define MPCQP_TQ_KM 48        /* [3]    km_foot                                                    */
#define MPCQP_TQ_GRAV 51      /* [12]   torques_gravity                                            */
#define MPCQP_TQ_CONTACTS 63  /* [4]    contacts[i] as 0.0 / 1.0                                   */
#define MPCQP_TQ_SIZE 68      /* 67 used, padded to a multiple of 4 doubles                       */

/* Replaces compute_joint_torques for `batch` robots (DEVICE pointers, async on `stream`):
 *   d_counter[b] += 1 (mpc_init_counter); while it is < 10 the robot's torques are zeroed;
 *   otherwise stance legs get tau = J^T (-f_grf), swing legs J tau = km .* f_kin (Eigen
 *   PartialPivLU), plus torques_gravity, and non-NaN entries overwrite d_joint_torques[b][12].
 * f_grf is taken from d_grf[b].f_body — the solve's output, so the MPC result never leaves the
 * device (a NaN leg's f_body is 0 there; the reference leaves that column uninitialised). */
int32_t mpcqp_joint_torques_device(const double* d_tq_records, const mpcqp_result* d_grf, int32_t batch,
                                   int32_t* d_counter, double* d_joint_torques, void* stream);

/* ---- single-step QP balance controller: the stance_leg_control_type == 0 branch of
 * A1RobotControl::compute_grf (A1RobotControl.cpp:321-332 euler error, :377-444 QP), constants
 * from the A1RobotControl ctor (:7-48).  12 variables (world-frame GRF), 20 rows (4 fz bounds,
 * 16 friction-pyramid rows), a fresh OsqpEigen::Solver every tick (warm start off, :420).
 * One binary64 record per robot (offsets in doubles; matrices row-major).                    */
#define MPCQP_BAL_POS 0        /* [3] root_pos (world)                                       */
#define MPCQP_BAL_POS_D 3      /* [3] root_pos_d                                             */
#define MPCQP_BAL_ROT 6        /* [9] root_rot_mat                                           */
#define MPCQP_BAL_ROT_Z 15     /* [9] root_rot_mat_z (yaw-only rotation)                     */
#define MPCQP_BAL_LIN_VEL 24   /* [3] root_lin_vel (world)                                   */
#define MPCQP_BAL_LIN_VEL_D 27 /* [3] root_lin_vel_d (body, as :382 reads it)                */
#define MPCQP_BAL_ANG_VEL 30   /* [3] root_ang_vel (world)                                   */
#define MPCQP_BAL_ANG_VEL_D 33 /* [3] root_ang_vel_d (body)                                  */
#define MPCQP_BAL_EULER 36     /* [3] root_euler                                             */
#define MPCQP_BAL_EULER_D 39   /* [3] root_euler_d                                           */
#define MPCQP_BAL_KP_LIN 42    /* [3] kp_linear                                              */
#define MPCQP_BAL_KD_LIN 45    /* [3] kd_linear                                              */
#define MPCQP_BAL_KP_ANG 48    /* [3] kp_angular                                             */
#define MPCQP_BAL_KD_ANG 51    /* [3] kd_angular                                             */
#define MPCQP_BAL_MASS 54      /* robot_mass                                                 */
#define MPCQP_BAL_FEET 55      /* [4][3] foot_pos_abs column i (world-aligned, body origin)   */
#define MPCQP_BAL_CONTACTS 67  /* [4] contacts[i] as 0.0 / 1.0                               */
#define MPCQP_BAL_SIZE 72      /* 71 used, padded to a multiple of 4 doubles                 */

typedef struct mpcqp_balance_params {
  double q_diag[6]; /* Q.diagonal() = 1, 1, 1, 400, 400, 100 (A1RobotControl.cpp:11)   */
  double r;         /* R = 1e-3 (:12)                                                    */
  double mu;        /* 0.7 (:13)                                                         */
  double f_min;     /* F_min = 0 (:14)                                                   */
  double f_max;     /* F_max = 180 (:15)                                                 */
} mpcqp_balance_params;

void mpcqp_balance_default_params(mpcqp_balance_params* p);

/* Replaces the QP branch of compute_grf for `batch` robots (DEVICE pointers, async on `stream`):
 * root_acc, H = R I + M'QM, g = -M'Q root_acc, bounds from contacts, OSQP setup + solve with the
 * handle's OSQP settings (warm_start ignored: the reference builds a new solver each tick).
 * d_results[b].u0 = QPSolution (world), .f_body = root_rot_mat^T QPSolution per leg (no NaN
 * guard in this branch, :440-443: a NaN solution stays NaN and sets nan_legs). */
int32_t mpcqp_balance_solve_device(mpcqp_handle* h, const mpcqp_balance_params* bp, const double* d_records,
                                   int32_t batch, mpcqp_result* d_results, void* stream);
/* Host-pointer convenience wrapper of the above (copies in, solves, copies out, synchronizes). */
int32_t mpcqp_balance_solve_host(mpcqp_handle* h, const mpcqp_balance_params* bp, const double* h_records,
                                 int32_t batch, mpcqp_result* h_results);

const char* mpcqp_status_str(int32_t status);
const char* mpcqp_error_str(int32_t err);
/* Last HIP error string recorded by the handle (for MPCQP_ERR_HIP). */
const char* mpcqp_last_error(mpcqp_handle* h);

#ifdef __cplusplus
}
#endif
#endif /* MPCQP_H_ */
