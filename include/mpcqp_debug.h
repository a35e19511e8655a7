/*
 * mpcqp_debug.h — diagnostic entry points of libmpcqp (not needed by a drop-in caller).
 */
#ifndef MPCQP_DEBUG_H_
#define MPCQP_DEBUG_H_

#include <stdint.h>

#include "mpcqp.h"

#ifdef __cplusplus
extern "C" {
#endif

/* Same as mpcqp_solve_batch_device, and additionally records, for the first `trace_cap`
 * instances, up to 64 termination checks each as {iter, pri_res, dua_res, rho} into
 * d_trace[trace_cap][64][4] (device pointer; pre-fill with NaN to see the count). */
int32_t mpcqp_debug_solve_trace_device(mpcqp_handle* h, const double* d_records, int32_t batch,
                                       mpcqp_result* d_results, double* d_solution,
                                       double* d_trace, int32_t trace_cap, void* stream);

/* sizeof(mpcqp_params), sizeof(mpcqp_result) as compiled (ABI check for bindings). */
int32_t mpcqp_abi_sizes(int32_t* params_size, int32_t* result_size);

/* Persistent-grid size (resident workgroups) chosen for the handle's device. */
int32_t mpcqp_handle_slots(mpcqp_handle* h);

/* Robots of the handle's last Schur-form (N <= 10) wave solve that the Riccati form solved in their
 * own wave: counts[0] rank-deficient feet (scale_kernel's screen), counts[1] a check whose KKT solve
 * cancelled too much for its core (max S_ii times the push-through identity's observed cancellation
 * above SCHUR_AMP), counts[2] a core whose max S_ii crossed the cap SCHUR_SMAX (each left the Schur
 * form at that check).  Synchronizes the device. */
int32_t mpcqp_handoff_counts(mpcqp_handle* h, int32_t counts[3]);

/* Parts a wave-path solve is split into (solved concurrently on the handle's internal streams,
 * forked from and joined to the caller's stream; results are bitwise those of one launch):
 * 0 = auto (3 parts from 3072 robots, 2 from 2048), 1 = one launch, up to 8.  The environment
 * variable MPCQP_SPLIT sets the initial value at mpcqp_create.  Returns the previous setting, or
 * -MPCQP_ERR_INVALID_ARG. */
int32_t mpcqp_debug_set_split(mpcqp_handle* h, int32_t parts);

/* Parts a solve of `batch` robots on this handle is split into under its current setting. */
int32_t mpcqp_debug_split_parts(mpcqp_handle* h, int32_t batch);

/* Threads per robot workgroup of the solve kernel the default path uses for horizon N. */
int32_t mpcqp_solve_threads(int32_t horizon);

/* Select the linear-system path of a handle: 0 auto (= 3), 3 the product path, one wavefront per
 * robot (impulse-space Schur form for N <= 10 with the Riccati form for robots whose feet are
 * degenerate; Riccati form for N > 10).  The debug build libmpcqp_debug.so adds two cross-check solvers:
 * 1 dense K^-1 with one workgroup per robot (N <= 10), 2 Riccati with one workgroup per robot.
 * All paths run the same OSQP iteration; the selection exists to cross-check them on the same
 * inputs.  The product libmpcqp.so returns MPCQP_ERR_INVALID_ARG for 1 and 2. */
int32_t mpcqp_debug_set_solver(mpcqp_handle* h, int32_t path);

/* The scaling image scale_kernel hands to wave_kernel (OSQP scale_data of the robot's QP, and for
 * warm slots the update_P / re-init branch): per robot mpcqp_debug_scale_image_doubles(N) doubles
 *   [0, 12N) D, [12N, 32N) E, [32N, 44N) q~ (cold / re-init: c D q; update_P: the previous tick's
 *   scaled gradient re-scaled), [44N, 56N) this tick's raw gradient q (warm slots), [56N] c,
 *   [56N + 1] branch (0 cold, 1 osqp_update_P, 2 OsqpEigen re-init), [56N + 2] 1 if some step's
 *   B6_k is rank deficient (collinear / coincident feet: the robot is solved by the Riccati form).
 *   (During a solve the Schur-form wave kernel reuses slot 56N + 2, after reading the flag, for
 *   max S_ii of its latest factorization: 1.0, or 2 SCHUR_SMAX when that exceeded SCHUR_SMAX and the
 *   robot is handed to the Riccati form.  This entry point runs scale_kernel alone.)
 * d_state: warm slots as for mpcqp_solve_batch_warm_device, or NULL (cold).  Note that the pass
 * records H's zero pattern into the slots (as the solve's own pass does): run it on a copy.
 * libmpcqp_debug.so only (the product library returns MPCQP_ERR_INVALID_ARG). */
int32_t mpcqp_debug_scale_image_doubles(int32_t horizon);
int32_t mpcqp_debug_scale_image_device(mpcqp_handle* h, const double* d_records, int32_t batch, double* d_state,
                                       double* d_img, void* stream);

/* Cross-lane primitive self-test of the wave path: writes 6 x 64 doubles to d_out (device). */
int32_t mpcqp_debug_wave_selftest(double* d_out, void* stream);

#ifdef __cplusplus
}
#endif
#endif
