// mpcqp_torque.hip — the downstream torque map of the GRF solve, batched on the device:
// A1RobotControl::compute_joint_torques (src/a1_cpp/src/A1RobotControl.cpp:289-319).
//
// One thread per (robot, leg); the four legs of a robot are adjacent lanes of one wave.  Stance
// legs map the solve's body-frame force through the foot Jacobian, tau = J^T (-f_grf) (:303);
// swing legs solve J tau = km .* f_kin with Eigen's partial-pivot LU (:306-307); gravity
// compensation is added (:311) and NaN entries keep the previous torque (:313-317).  The first
// nine ticks of a controller output zero torque (mpc_init_counter, :292-296).
//
// Element-wise and HBM-bound (~0.7 KB moved per robot).  Contraction is off so the result is
// bitwise the oracle's (oracle/mpc_oracle.c orc_joint_torques, same operation order).
#include "mpcqp_device.h"

namespace mpcqp {
namespace tq {

__device__ __forceinline__ void swap_if(bool s, double& x, double& y) {
  const double t = x;
  x = s ? y : x;
  y = s ? t : y;
}

// Eigen PartialPivLU<Matrix3d>(J).solve(b): pivot on the first maximal |a_ik|, swap whole rows
// (L part included), unit-lower forward and upper backward substitution.  Swaps are selects so
// nothing is indexed at run time.
__device__ __forceinline__ void lu3_solve(double (&a)[9], double (&b)[3], double (&x)[3]) {
#pragma clang fp contract(off)
  {  // column 0
    const double m0 = dabs(a[0]), m1 = dabs(a[3]), m2 = dabs(a[6]);
    const bool p1 = m1 > m0;
    double best = p1 ? m1 : m0;
    const bool p2 = m2 > best;
    best = p2 ? m2 : best;
#pragma unroll
    for (int j = 0; j < 3; ++j) {
      swap_if(p2, a[j], a[6 + j]);
      swap_if(!p2 && p1, a[j], a[3 + j]);
    }
    swap_if(p2, b[0], b[2]);
    swap_if(!p2 && p1, b[0], b[1]);
    if (best != 0.0) {
      a[3] /= a[0];
      a[6] /= a[0];
    }
    a[4] -= a[3] * a[1];
    a[5] -= a[3] * a[2];
    a[7] -= a[6] * a[1];
    a[8] -= a[6] * a[2];
  }
  {  // column 1
    const double m1 = dabs(a[4]), m2 = dabs(a[7]);
    const bool q = m2 > m1;
    const double best = q ? m2 : m1;
#pragma unroll
    for (int j = 0; j < 3; ++j) swap_if(q, a[3 + j], a[6 + j]);
    swap_if(q, b[1], b[2]);
    if (best != 0.0) a[7] /= a[4];
    a[8] -= a[7] * a[5];
  }
  const double y0 = b[0], y1 = b[1] - a[3] * y0, y2 = (b[2] - a[6] * y0) - a[7] * y1;
  x[2] = y2 / a[8];
  x[1] = (y1 - a[5] * x[2]) / a[4];
  x[0] = ((y0 - a[1] * x[1]) - a[2] * x[2]) / a[0];
}

__global__ __launch_bounds__(256) void torque_kernel(const double* __restrict__ recs,
                                                     const mpcqp_result* __restrict__ grf, int batch,
                                                     int* __restrict__ counter, double* __restrict__ tau) {
#pragma clang fp contract(off)
  const int gid = blockIdx.x * blockDim.x + threadIdx.x;
  const int b = gid >> 2, leg = gid & 3;
  if (b >= batch) return;
  const int c = counter[b] + 1;  // mpc_init_counter++ (the four legs read before leg 0 writes)
  if (leg == 0) counter[b] = c;
  double* t = tau + (size_t)12 * b + 3 * leg;
  if (c < 10) {
    t[0] = 0.0;
    t[1] = 0.0;
    t[2] = 0.0;
    return;
  }
  const double* r = recs + (size_t)MPCQP_TQ_SIZE * b;
  double J[9], v[3];
#pragma unroll
  for (int e = 0; e < 9; ++e) J[e] = r[MPCQP_TQ_JFOOT + 9 * leg + e];
  if (r[MPCQP_TQ_CONTACTS + leg] != 0.0) {  // stance: tau = J^T (-f_grf)
    const double* f = grf[b].f_body + 3 * leg;
    const double f0 = -f[0], f1 = -f[1], f2 = -f[2];
#pragma unroll
    for (int k = 0; k < 3; ++k) v[k] = ((0.0 + J[k] * f0) + J[3 + k] * f1) + J[6 + k] * f2;
  } else {  // swing: J tau = km .* f_kin
    double ft[3];
#pragma unroll
    for (int k = 0; k < 3; ++k) ft[k] = r[MPCQP_TQ_KM + k] * r[MPCQP_TQ_FKIN + 3 * leg + k];
    lu3_solve(J, ft, v);
  }
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    const double s = v[k] + r[MPCQP_TQ_GRAV + 3 * leg + k];
    if (!isnan(s)) t[k] = s;
  }
}

}  // namespace tq

hipError_t launch_torques(const double* recs, const mpcqp_result* grf, int batch, int* counter, double* tau,
                          void* stream) {
  const int threads = 4 * batch;
  hipLaunchKernelGGL(tq::torque_kernel, dim3((threads + 255) / 256), dim3(256), 0, (hipStream_t)stream, recs, grf,
                     batch, counter, tau);
  return hipGetLastError();
}

}  // namespace mpcqp
