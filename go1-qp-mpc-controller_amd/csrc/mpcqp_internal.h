// mpcqp_internal.h — shared between the kernels and the C-ABI layer (not installed).
#pragma once
#include <hip/hip_runtime.h>

#include "../../include/mpcqp.h"

#define MPCQP_TRACE_LEN 64  // termination-check records kept per instance by the debug trace

namespace mpcqp {


struct LaunchArgs {
  const double* recs;
  int batch;
  mpcqp_result* results;
  double* solution;
  double* work;
  double* trace;
  int trace_cap;
  double* wstate;  // warm-start slots [batch][warm_state_doubles(N)] (wave path) or nullptr
  int* fallback;   // wave path: 4 hand-off counters (handle-owned): [0] rank-deficient feet,
                   // [2] ill-conditioned Schur core after a rho update ([1], [3] unused)
  int grid;
  void* stream;
  mpcqp_params p;
};

// Formulation only (mpcqp_build.hip): ConvexMpc::calculate_qp_mats, horizons 1..20
hipError_t launch_build_any(const LaunchArgs& a, double* P, double* q, double* l, double* u);

// The solve: scale_kernel + one-wave-per-robot Riccati wave_kernel (mpcqp_wave.hip), horizons
// 1..WAVE_MAX_HORIZON
hipError_t launch_wave_any(const LaunchArgs& a);
hipError_t occupancy_wave_any(const mpcqp_params& p, int* blocks);
hipError_t wave_selftest(double* d_out, void* stream);
hipError_t launch_scale_any(const LaunchArgs& a);  // scale_kernel alone (the image in a.work)
constexpr int WAVE_MAX_HORIZON = 20;

#ifdef MPCQP_DEBUG_PATHS
// Cross-check solvers, built only into libmpcqp_debug.so (mpcqp_debug_set_solver 1, 2):
// dense K^-1 workgroup (mpcqp_kernels.hip, N <= DENSE_MAX_HORIZON) and workgroup Riccati
// (mpcqp_riccati.hip).
hipError_t launch_solve_any(const LaunchArgs& a);
hipError_t occupancy_any(int horizon, int* blocks);
size_t workspace_doubles(int horizon);  // per robot
hipError_t launch_riccati_any(const LaunchArgs& a);
hipError_t occupancy_riccati_any(int horizon, int* blocks);
size_t riccati_workspace_doubles(int horizon);  // per robot
#endif
constexpr int DENSE_MAX_HORIZON = 10;
// doubles per robot of the warm-start slot (mpcqp_wave.hip WarmLayout)
__host__ __device__ constexpr int warm_state_doubles(int N) {
  return 4 + 3 * 12 * N + 5 * 20 * N + ((12 * N + 63) / 64) * 12 * N;
}

// doubles per robot of the scaling image scale_kernel hands to wave_kernel (mpcqp_wave.hip ScaleImg)
__host__ __device__ constexpr int scale_image_doubles(int N) { return 3 * 12 * N + 20 * N + 3; }

// Downstream torque map (mpcqp_torque.hip)
hipError_t launch_torques(const double* recs, const mpcqp_result* grf, int batch, int* counter, double* tau,
                          void* stream);

// Input assembly from raw robot state (mpcqp_assemble.hip)
hipError_t launch_assemble(int horizon, const double* states, int batch, double* recs, void* stream);
// Indexed copy of fixed-size slots (warm-start slots of mixed-mode batches; mpcqp_assemble.hip)
hipError_t launch_copy_slots(const double* src, const int* sidx, double* dst, const int* didx, int count, int slot,
                             void* stream);

// Single-step QP balance controller (mpcqp_balance.hip)
hipError_t launch_balance(const mpcqp_balance_params& bp, const mpcqp_params& p, const double* recs, int batch,
                          mpcqp_result* out, void* stream);

}  // namespace mpcqp
