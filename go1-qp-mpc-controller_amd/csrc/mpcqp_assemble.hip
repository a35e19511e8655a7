// mpcqp_assemble.hip — on-device input assembly of the MPC problem record from raw robot state
// (SURVEY §8(f) rank 2): the x0 / x_ref / horizon-feet part of A1RobotControl::compute_grf
// (src/a1_cpp/src/A1RobotControl.cpp:452-514), so a batched simulator hands its robot states to
// the solve without host packing.
//
// Grid: one thread per (robot, record chunk).  A robot's record is REC_SIZE(N) doubles
// (334 at N = 10); it is written by 64 lanes of one wave, each lane computing the doubles at
// offsets lane, lane + 64, ...: consecutive lanes write consecutive doubles, so the stores are
// fully coalesced, and the 64-double state row is read once per lane from L1/L2.  HBM-bound:
// 512 B read + 8 * REC_SIZE(N) B written per robot.  Contraction is off and every value is
// computed in the oracle's operation order (oracle/mpc_oracle.c orc_assemble_compute_grf), so the
// record is bitwise the oracle's.
#include "mpcqp_device.h"

#pragma clang fp contract(off)

namespace mpcqp {
namespace as {

template <int N>
__device__ __forceinline__ double record_value(const double* __restrict__ s, int k) {
  constexpr int feet0 = MPCQP_REC_FEET(N);
  if (k < MPCQP_REC_EULER) {  // x0 = [euler, pos, w, v, -9.8] (:452-456)
    return k == 12 ? -9.8 : s[MPCQP_ST_EULER + k];
  }
  if (k < MPCQP_REC_ROT) return s[MPCQP_ST_EULER + k - MPCQP_REC_EULER];        // calculate_A_mat_c arg (:492)
  if (k < MPCQP_REC_INERTIA) return s[MPCQP_ST_ROT + k - MPCQP_REC_ROT];
  if (k < MPCQP_REC_MASS) return s[MPCQP_ST_INERTIA + k - MPCQP_REC_INERTIA];
  if (k == MPCQP_REC_MASS) return s[MPCQP_ST_MASS];
  if (k == MPCQP_REC_MU) return s[MPCQP_ST_MU];
  if (k == MPCQP_REC_FZMIN) return s[MPCQP_ST_FZMIN];
  if (k == MPCQP_REC_FZMAX) return s[MPCQP_ST_FZMAX];
  if (k == MPCQP_REC_DT) return s[MPCQP_ST_DT];
  if (k < MPCQP_REC_CONTACTS + 4) return s[MPCQP_ST_CONTACTS + k - MPCQP_REC_CONTACTS] != 0.0 ? 1.0 : 0.0;
  if (k < MPCQP_REC_XREF) return 0.0;
  if (k < feet0) {  // x_ref step i (:472-488)
    const int i = (k - MPCQP_REC_XREF) / 13, e = (k - MPCQP_REC_XREF) % 13;
    const double dt = s[MPCQP_ST_DT];
    const double* R = s + MPCQP_ST_ROT;
    const double* vd = s + MPCQP_ST_LIN_VEL_D;
    auto vdw = [&](int r) {  // root_lin_vel_d_world = root_rot_mat * root_lin_vel_d (:470)
      double acc = 0.0;
      acc += R[r * 3 + 0] * vd[0];
      acc += R[r * 3 + 1] * vd[1];
      acc += R[r * 3 + 2] * vd[2];
      return acc;
    };
    const double step = (double)(i + 1);
    switch (e) {
      case 0: return s[MPCQP_ST_EULER_D + 0];
      case 1: return s[MPCQP_ST_EULER_D + 1];
      case 2: return s[MPCQP_ST_EULER + 2] + s[MPCQP_ST_ANG_VEL_D + 2] * dt * step;
      case 3: return s[MPCQP_ST_POS + 0] + vdw(0) * dt * step;
      case 4: return s[MPCQP_ST_POS + 1] + vdw(1) * dt * step;
      case 5: return s[MPCQP_ST_POS_D + 2];
      case 6: return s[MPCQP_ST_ANG_VEL_D + 0];
      case 7: return s[MPCQP_ST_ANG_VEL_D + 1];
      case 8: return s[MPCQP_ST_ANG_VEL_D + 2];
      case 9: return vdw(0);
      case 10: return vdw(1);
      case 11: return 0.0;
      default: return -9.8;
    }
  }
  if (k < feet0 + 12 * N) return s[MPCQP_ST_FEET + (k - feet0) % 12];  // same feet every step (:498-514)
  return 0.0;  // padding
}

template <int N>
__global__ void __launch_bounds__(256) assemble_kernel(const double* __restrict__ states, int batch,
                                                       double* __restrict__ recs) {
  constexpr int RS = MPCQP_REC_SIZE(N);
  const int b = (int)((blockIdx.x * blockDim.x + threadIdx.x) >> 6);
  const int lane = threadIdx.x & 63;
  if (b >= batch) return;
  const double* s = states + (size_t)MPCQP_ST_SIZE * b;
  double* r = recs + (size_t)RS * b;
  for (int k = lane; k < RS; k += 64) r[k] = record_value<N>(s, k);
}

template <int N>
hipError_t launch_n(const double* states, int batch, double* recs, void* stream) {
  const long threads = 64L * batch;
  hipLaunchKernelGGL(assemble_kernel<N>, dim3((unsigned)((threads + 255) / 256)), dim3(256), 0, (hipStream_t)stream,
                     states, batch, recs);
  return hipGetLastError();
}

template <int... Ns>
hipError_t dispatch(int horizon, const double* states, int batch, double* recs, void* stream,
                    std::integer_sequence<int, Ns...>) {
  hipError_t e = hipErrorInvalidValue;
  ((horizon == Ns + 1 ? (e = launch_n<Ns + 1>(states, batch, recs, stream), 0) : 0), ...);
  return e;
}

}  // namespace as

hipError_t launch_assemble(int horizon, const double* states, int batch, double* recs, void* stream) {
  return as::dispatch(horizon, states, batch, recs, stream, std::make_integer_sequence<int, MPCQP_MAX_HORIZON>{});
}

namespace as {
// Indexed slot copy: dst[dst_idx[i]] = src[src_idx[i]] (identity where an index array is null), one
// 256-thread block per slot, coalesced along the slot.
__global__ void __launch_bounds__(256) copy_slots_kernel(const double* __restrict__ src, const int* __restrict__ sidx,
                                                         double* __restrict__ dst, const int* __restrict__ didx,
                                                         int count, int slot) {
  const int i = blockIdx.x;
  if (i >= count) return;
  const double* s = src + (size_t)slot * (sidx ? sidx[i] : i);
  double* d = dst + (size_t)slot * (didx ? didx[i] : i);
  for (int e = threadIdx.x; e < slot; e += 256) d[e] = s[e];
}
}  // namespace as

hipError_t launch_copy_slots(const double* src, const int* sidx, double* dst, const int* didx, int count, int slot,
                             void* stream) {
  if (count <= 0) return hipSuccess;
  hipLaunchKernelGGL(as::copy_slots_kernel, dim3((unsigned)count), dim3(256), 0, (hipStream_t)stream, src, sidx, dst,
                     didx, count, slot);
  return hipGetLastError();
}

}  // namespace mpcqp
