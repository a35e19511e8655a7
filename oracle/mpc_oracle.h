/*
 * mpc_oracle.h — TEST INFRASTRUCTURE ONLY.
 *
 * CPU (binary64) restatement of the reference hot path, used as the parity checker by tests/,
 * __graft_entry__.smoke() and as bench.py's cpu_baseline ("port").  The product path never
 * links or calls this code.
 *
 * Parity status: the formulation follows src/a1_cpp/src/ConvexMpc.cpp and
 * src/a1_cpp/src/A1RobotControl.cpp line by line.  The QP solver restates OSQP 0.6.x
 * (third-party, cloned unpinned in docker/Dockerfile:74-98, not vendored in the reference and
 * not buildable here).  No reference test pins results at that boundary, so the OSQP iterate
 * sequence is "parity unpinned" (see DESIGN.md §Oracle).
 */
#ifndef MPC_ORACLE_H_
#define MPC_ORACLE_H_

#include "../include/mpcqp.h"

#ifdef __cplusplus
extern "C" {
#endif

/* Robot-state view of A1CtrlStates / Go1CtrlStates fields read by compute_grf's MPC branch
 * (A1RobotControl.cpp:446-514).  Matrices are row-major; foot_pos_abs is [leg][xyz]. */
typedef struct orc_robot_state {
  double root_euler[3], root_pos[3], root_ang_vel[3], root_lin_vel[3];
  double root_rot_mat[9];
  double root_euler_d[3], root_pos_d[3], root_ang_vel_d[3], root_lin_vel_d[3];
  double foot_pos_abs[12];
  double robot_mass, trunk_inertia[9];
  double mu, fz_min, fz_max, mpc_dt;
  int32_t contacts[4];
} orc_robot_state;

/* Per-check trace of one solve (iteration, residuals, rho) for parity diagnostics. */
typedef struct orc_trace_entry {
  int32_t iter, rho_updated;
  double pri_res, dua_res, eps_prim, eps_dual, rho;
} orc_trace_entry;

/* compute_grf MPC-branch input assembly (A1RobotControl.cpp:446-514) → problem record.
 * `rec` must hold mpcqp_record_size(N) doubles. */
void orc_assemble_compute_grf(const orc_robot_state* s, int32_t N, double* rec);

/* test_mpc.cpp:15-122 hand-set stance → problem record (feet shift by -v_d*dt per step). */
void orc_assemble_test_mpc(int32_t N, double* rec, double q_weights[13], double r_weights[12]);

/* ConvexMpc::calculate_qp_mats restatement.  P is full symmetric row-major [n][n],
 * q [n], l/u [m], Acon row-major dense constraint matrix [m][n] (may be NULL). */
int32_t orc_build_qp(const mpcqp_params* prm, const double* rec, double* P, double* q,
                     double* l, double* u, double* Acon);

/* OSQP 0.6 restatement on the QP built from `rec`; cold start.  sol: [12N] or NULL.
 * trace: optional array of max_trace entries; *n_trace receives the count. */
int32_t orc_solve(const mpcqp_params* prm, const double* rec, mpcqp_result* res, double* sol,
                  orc_trace_entry* trace, int32_t max_trace, int32_t* n_trace);

/* Warm start across control ticks: one persistent OSQP solver per robot, driven like the
 * reference's member solver (A1RobotControl.h:67, A1RobotControl.cpp:520-540): the first step
 * is initSolver + solve, later steps updateHessianMatrix / updateGradient / updateLowerBound /
 * updateUpperBound + solve with warm_start (previous x, z, y and the adapted rho persist). */
typedef struct orc_solver orc_solver;
orc_solver* orc_solver_new(const mpcqp_params* prm);
void orc_solver_free(orc_solver* s);
void orc_solver_reset(orc_solver* s);
int32_t orc_solver_step(orc_solver* s, const double* rec, mpcqp_result* res, double* sol,
                        orc_trace_entry* trace, int32_t max_trace, int32_t* n_trace);
/* T ticks x `batch` robots, each robot its own persistent solver: recs [T][batch][rec],
 * res [T][batch]; robots partitioned over `nthreads` POSIX threads. */
int32_t orc_solve_sequence(const mpcqp_params* prm, const double* recs, int32_t T, int32_t batch,
                           mpcqp_result* res, int32_t nthreads);

/* A1RobotControl::compute_joint_torques (A1RobotControl.cpp:289-319) for one robot: `tq` is an
 * MPCQP_TQ_SIZE record (include/mpcqp.h), `f_grf` the 12 body-frame GRFs (foot_forces_grf
 * columns, = mpcqp_result.f_body), `counter` the controller's mpc_init_counter (incremented),
 * `tau` the robot's joint_torques (updated in place; NaN entries keep the previous value). */
/* TEST ONLY: scaled problem data (D, E, q~ = c D q, c) a cold solve / a persistent solver's next
 * tick starts from; mode = 0 initSolver, 1 osqp_update_P, 2 OsqpEigen re-init. */
int32_t orc_scale_image(const mpcqp_params* prm, const double* rec, double* D, double* E, double* q, double* c);
int32_t orc_solver_step_image(orc_solver* s, const double* rec, mpcqp_result* res, double* D, double* E, double* q,
                              double* c, int32_t* mode);
void orc_joint_torques(const double* tq, const double* f_grf, int32_t* counter, double* tau);

/* Batch over `nthreads` POSIX threads (static contiguous partition).  sols may be NULL. */
int32_t orc_solve_batch(const mpcqp_params* prm, const double* recs, int32_t batch,
                        mpcqp_result* res, double* sols, int32_t nthreads);

/* Single-step QP balance controller (A1RobotControl.cpp:7-48, :321-332, :377-444): dense
 * H [12][12] full symmetric, g [12], l/u [20], A [20][12] row-major from one MPCQP_BAL record. */
void orc_balance_build_qp(const mpcqp_balance_params* bp, const double* rec, double* P, double* q,
                          double* l, double* u, double* A);
/* Fresh OSQP 0.6 solve of that QP with prm's settings (horizon / warm_start ignored). */
int32_t orc_balance_solve(const mpcqp_params* prm, const mpcqp_balance_params* bp, const double* rec,
                          mpcqp_result* res);
int32_t orc_balance_solve_batch(const mpcqp_params* prm, const mpcqp_balance_params* bp, const double* recs,
                                int32_t batch, mpcqp_result* res, int32_t nthreads);

#ifdef __cplusplus
}
#endif
#endif
