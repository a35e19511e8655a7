// mpcqp_build.hip — formulation-only kernel: ConvexMpc::calculate_qp_mats for a batch of robots
// (src/a1_cpp/src/ConvexMpc.cpp:158-245) -> dense Hessian (both triangles, row-major n x n),
// gradient, unscaled bounds l / u.  Serves the C++ ConvexMpc shim (include/mpcqp_robot_control.hpp,
// whose public `hessian`, `gradient`, `lb`, `ub` members the reference's caller reads at
// A1RobotControl.cpp:527-537) and the P0 formulation parity tests.  One 256-thread workgroup per
// robot running the block condensation of mpcqp_device.h (condense()).
#include "mpcqp_device.h"

namespace mpcqp {

template <int N>
struct BuildSmem {
  using Dm = Dim<N>;
  double rec[Dm::rec];
  double lo[Dm::m], hi[Dm::m];
  double qt[Dm::n];
  union U {
    CondScratch<N> c;
  } u;
};

template <int N>
__global__ __launch_bounds__(256) void build_qp_kernel(const double* __restrict__ recs, int batch,
                                                       double* __restrict__ P, double* __restrict__ q,
                                                       double* __restrict__ l, double* __restrict__ u,
                                                       mpcqp_params p) {
  using Dm = Dim<N>;
  __shared__ BuildSmem<N> sm;
  const int inst = blockIdx.x;
  if (inst >= batch) return;
  const int t = threadIdx.x;
  for (int e = t; e < Dm::rec; e += 256) sm.rec[e] = recs[(size_t)inst * Dm::rec + e];
  __syncthreads();
  condense<N, 256>(sm, p, P + (size_t)inst * Dm::n * Dm::n, Dm::n);
  if (t < Dm::n) q[(size_t)inst * Dm::n + t] = sm.qt[t];
  for (int e = t; e < Dm::m; e += 256) {
    l[(size_t)inst * Dm::m + e] = sm.lo[e];
    u[(size_t)inst * Dm::m + e] = sm.hi[e];
  }
}

template <int N>
static hipError_t launch_build(const LaunchArgs& a, double* P, double* q, double* l, double* u) {
  hipLaunchKernelGGL((build_qp_kernel<N>), dim3(a.batch), dim3(256), 0, (hipStream_t)a.stream, a.recs,
                     a.batch, P, q, l, u, a.p);
  return hipGetLastError();
}

hipError_t launch_build_any(const LaunchArgs& a, double* P, double* q, double* l, double* u) {
  switch (a.p.horizon) {
#define CASE(K) \
  case K: return launch_build<K>(a, P, q, l, u);
    CASE(1) CASE(2) CASE(3) CASE(4) CASE(5) CASE(6) CASE(7) CASE(8) CASE(9) CASE(10)
    CASE(11) CASE(12) CASE(13) CASE(14) CASE(15) CASE(16) CASE(17) CASE(18) CASE(19) CASE(20)
#undef CASE
    default: return hipErrorInvalidValue;
  }
}

}  // namespace mpcqp
