// mpcqp_device.h — device-side pieces shared by the dense (mpcqp_kernels.hip) and Riccati
// (mpcqp_riccati.hip) solve kernels: OSQP constants, dimensions, cross-lane reductions and the
// ConvexMpc condensation.  Not installed.
#pragma once
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>

#include <type_traits>

#include "../../include/mpcqp.h"
#include "mpcqp_internal.h"

namespace mpcqp {

constexpr int SD = 13, ND = 12, CD = 20;
constexpr double OSQP_INF = 1e30;
constexpr double MIN_SCALING = 1e-4, MAX_SCALING = 1e4;
constexpr double RHO_MIN = 1e-6, RHO_MAX = 1e6, RHO_EQ_OVER_RHO_INEQ = 1e3, RHO_TOL = 1e-4;
constexpr double DIV_TOL = 1.0 / OSQP_INF;

template <int N>
struct Dim {
  static constexpr int n = ND * N, m = CD * N, nf = 4 * N, ns = SD * N;
  static constexpr int rec = MPCQP_REC_SIZE(N);
  static constexpr int feet = MPCQP_REC_FEET(N);
  static constexpr int GL = 8;                                   // lanes per foot group
  static constexpr int BC = 3 * ((n + 3 * GL - 1) / (3 * GL));   // tile columns per lane (multiple of 3)
  static constexpr int NP = GL * BC;                             // padded column count
  static constexpr int NT = ((GL * nf + 63) / 64) * 64;          // threads (whole waves)
  static constexpr int NG = NT / GL;                             // groups, idle ones included
  static constexpr int NW = NT / 64;                             // waves
  static constexpr int SPL = BC / 3;                             // feet whose columns one lane holds
};

// LDS scratch of condense() (union member of every kernel's LDS image).
template <int N>
struct CondScratch {
  double S[N][SD * SD];
  double Bq[N][SD * ND];
  double G[SD * ND];
  double Ad[SD * SD];
  double T[SD * SD];
  double Iwinv[9];
  double a[SD];
  double w[SD];
};

// Returns v unchanged but opaque to the optimizer, so values derived from it are recomputed in
// the loop instead of being hoisted (and held live) across the whole ADMM loop.
__device__ __forceinline__ int opaque(int v) {
  asm volatile("" : "+v"(v));
  return v;
}
// Pins a value read from LDS into a register: the asm hides where it came from, so the compiler
// cannot rematerialize it later by reloading LDS that has been reused in between.
__device__ __forceinline__ void keep(double& v) { asm volatile("" : "+v"(v)); }
// arr[i] for a per-lane i in [0, K): a select chain over the wave-uniform elements.  (Indexing the
// kernel's by-value parameters with a per-lane index makes the compiler copy them to scratch memory
// and load from there: a store and a load round trip through the memory pipe per robot.)
template <int K>
__device__ __forceinline__ double lane_pick(const double (&arr)[K], int i) {
  double v = arr[0];
#pragma unroll
  for (int k = 1; k < K; ++k) v = i == k ? arr[k] : v;
  return v;
}
__device__ __forceinline__ double dmax(double a, double b) { return a > b ? a : b; }
__device__ __forceinline__ double dmin(double a, double b) { return a < b ? a : b; }
__device__ __forceinline__ double dabs(double a) { return __builtin_fabs(a); }
// Three-way select on values (a select of lvalues can become a select of addresses, which
// forces the operands out of registers into scratch).
__device__ __forceinline__ double sel3(int k, double a, double b, double c) {
  return k == 0 ? a : (k == 1 ? b : c);
}
__device__ __forceinline__ double limit_scaling(double d) {
  d = d < MIN_SCALING ? 1.0 : d;
  return d > MAX_SCALING ? MAX_SCALING : d;
}

// ---- cross-lane helpers ----------------------------------------------------------------------
// DPP move of a double inside a 16-lane row.  CTRL: 0x140 row_mirror (i <-> 15-i),
// 0x141 row_half_mirror (i <-> 7-i in each half), 0x4E quad_perm xor 2, 0xB1 quad_perm xor 1.
// (mov_dpp: no "old" operand to materialize; every control used here reads an in-row lane)
template <int CTRL>
__device__ __forceinline__ double dpp(double v) {
  const int lo = __builtin_amdgcn_mov_dpp(__double2loint(v), CTRL, 0xF, 0xF, true);
  const int hi = __builtin_amdgcn_mov_dpp(__double2hiint(v), CTRL, 0xF, 0xF, true);
  return __hiloint2double(hi, lo);
}
// 16-lane all-reduce; the four pairings generate the whole group and every step adds the same two
// operands on both partners, so all 16 lanes end with bitwise-identical results.
__device__ __forceinline__ double g16_sum(double v) {
  v = v + dpp<0x140>(v);
  v = v + dpp<0x141>(v);
  v = v + dpp<0x4E>(v);
  v = v + dpp<0xB1>(v);
  return v;
}
__device__ __forceinline__ double g16_max(double v) {
  v = dmax(v, dpp<0x140>(v));
  v = dmax(v, dpp<0x141>(v));
  v = dmax(v, dpp<0x4E>(v));
  v = dmax(v, dpp<0xB1>(v));
  return v;
}
// 8-lane (foot group) all-reduce, same bitwise-symmetric pairing argument as g16_*.
__device__ __forceinline__ double g8_sum(double v) {
  v = v + dpp<0x141>(v);
  v = v + dpp<0x4E>(v);
  v = v + dpp<0xB1>(v);
  return v;
}
__device__ __forceinline__ double g8_max(double v) {
  v = dmax(v, dpp<0x141>(v));
  v = dmax(v, dpp<0x4E>(v));
  v = dmax(v, dpp<0xB1>(v));
  return v;
}
// Orders LDS traffic between lanes of one wave (LDS executes a wave's operations in order; this
// keeps the compiler from moving memory operations across the hand-off).
__device__ __forceinline__ void wave_sync() {
  __builtin_amdgcn_wave_barrier();
  asm volatile("" ::: "memory");
}
// Partner of every lane in the other DPP row of its pair (lane ^ 16) / other row pair (lane ^ 32),
// through the gfx950 row-swap permutes (no LDS round trip, unlike ds_bpermute).
__device__ __forceinline__ double xor16(double v) {
  const unsigned lo = (unsigned)__double2loint(v), hi = (unsigned)__double2hiint(v);
  const auto l2 = __builtin_amdgcn_permlane16_swap(lo, lo, false, false);
  const auto h2 = __builtin_amdgcn_permlane16_swap(hi, hi, false, false);
  // even rows: the odd partner moved into src; odd rows: the even partner moved into vdst
  const bool odd = (threadIdx.x >> 4) & 1;
  return __hiloint2double((int)(odd ? h2[0] : h2[1]), (int)(odd ? l2[0] : l2[1]));
}
__device__ __forceinline__ double xor32(double v) {
  const unsigned lo = (unsigned)__double2loint(v), hi = (unsigned)__double2hiint(v);
  const auto l2 = __builtin_amdgcn_permlane32_swap(lo, lo, false, false);
  const auto h2 = __builtin_amdgcn_permlane32_swap(hi, hi, false, false);
  const bool upper = (threadIdx.x >> 5) & 1;
  return __hiloint2double((int)(upper ? h2[0] : h2[1]), (int)(upper ? l2[0] : l2[1]));
}
// Row-pair / row-half combine for commutative all-reduces: permlane16_swap(v, v) leaves rows
// [r0 r0 r2 r2] in one copy and [r1 r1 r3 r3] in the other (permlane32_swap likewise for the halves),
// so op(copy0, copy1) is the pair's result in every lane with no lane select, bitwise the same in
// both partners.
template <class Op>
__device__ __forceinline__ double swap16_reduce(double v, Op op) {
  const unsigned lo = (unsigned)__double2loint(v), hi = (unsigned)__double2hiint(v);
  const auto l2 = __builtin_amdgcn_permlane16_swap(lo, lo, false, false);
  const auto h2 = __builtin_amdgcn_permlane16_swap(hi, hi, false, false);
  return op(__hiloint2double((int)h2[0], (int)l2[0]), __hiloint2double((int)h2[1], (int)l2[1]));
}
template <class Op>
__device__ __forceinline__ double swap32_reduce(double v, Op op) {
  const unsigned lo = (unsigned)__double2loint(v), hi = (unsigned)__double2hiint(v);
  const auto l2 = __builtin_amdgcn_permlane32_swap(lo, lo, false, false);
  const auto h2 = __builtin_amdgcn_permlane32_swap(hi, hi, false, false);
  return op(__hiloint2double((int)h2[0], (int)l2[0]), __hiloint2double((int)h2[1], (int)l2[1]));
}
__device__ __forceinline__ double wave_max(double v) {
  auto op = [](double a, double b) __attribute__((always_inline)) { return dmax(a, b); };
  v = g16_max(v);
  v = swap16_reduce(v, op);
  return swap32_reduce(v, op);
}
__device__ __forceinline__ double wave_sum(double v) {
  auto op = [](double a, double b) __attribute__((always_inline)) { return a + b; };
  v = g16_sum(v);
  v = swap16_reduce(v, op);
  return swap32_reduce(v, op);
}
// max of two non-negative, non-NaN doubles (norms of absolute values), where fmax equals dmax
// bitwise: one v_max_f64, without the IEEE-mode canonicalization the compiler wraps around fmax
__device__ __forceinline__ double nmax(double a, double b) {
  double r;
  asm("v_max_f64 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
  return r;
}
__device__ __forceinline__ double wave_nmax(double v) {
  auto op = [](double a, double b) __attribute__((always_inline)) { return nmax(a, b); };
  v = nmax(v, dpp<0x140>(v));
  v = nmax(v, dpp<0x141>(v));
  v = nmax(v, dpp<0x4E>(v));
  v = nmax(v, dpp<0xB1>(v));
  v = swap16_reduce(v, op);
  return swap32_reduce(v, op);
}

// KM max-reductions (non-negative operands, as wave_nmax) and KS sum-reductions (as wave_sum) of one
// wave, level by level: every value takes exactly the operations of its single reduction, in the same
// order (bitwise the same results), but the values of a level are independent, so each DPP read of a
// value comes several instructions after the VALU write that made it (no wait states, which a lone
// chain needs at every level: 2 states = s_nop 1, 8.4 cycles).
template <int KM, int KS>
__device__ __forceinline__ void wave_reduce_batch(double (&mx)[KM], double (&sm)[KS]) {
  auto level = [&](auto CTRL) __attribute__((always_inline)) {
    constexpr int ctrl = decltype(CTRL)::value;
#pragma unroll
    for (int k = 0; k < KM; ++k) mx[k] = nmax(mx[k], dpp<ctrl>(mx[k]));
#pragma unroll
    for (int k = 0; k < KS; ++k) sm[k] = sm[k] + dpp<ctrl>(sm[k]);
  };
  level(std::integral_constant<int, 0x140>{});
  level(std::integral_constant<int, 0x141>{});
  level(std::integral_constant<int, 0x4E>{});
  level(std::integral_constant<int, 0xB1>{});
  auto mop = [](double a, double b) __attribute__((always_inline)) { return nmax(a, b); };
  auto sop = [](double a, double b) __attribute__((always_inline)) { return a + b; };
#pragma unroll
  for (int k = 0; k < KM; ++k) mx[k] = swap16_reduce(mx[k], mop);
#pragma unroll
  for (int k = 0; k < KS; ++k) sm[k] = swap16_reduce(sm[k], sop);
#pragma unroll
  for (int k = 0; k < KM; ++k) mx[k] = swap32_reduce(mx[k], mop);
#pragma unroll
  for (int k = 0; k < KS; ++k) sm[k] = swap32_reduce(sm[k], sop);
}

// ---- condensation: ConvexMpc.cpp:110-245 ----------------------------------------------------
// Writes the dense Hessian (both triangles) to Pout[ld], the gradient to sm.qt and the unscaled
// bounds to sm.lo / sm.hi.
template <int N, int NT, class SM>
__device__ __forceinline__ void condense(SM& sm, const mpcqp_params& p, double* __restrict__ Pout, int ld) {
  using Dm = Dim<N>;
  const int t = threadIdx.x;
  auto& C = sm.u.c;
  const double* rec = sm.rec;
  const double dt = rec[MPCQP_REC_DT];
  // calculate_A_mat_c (:110-130) + A_d = I + A_c dt (:150); S_{N-1} = Q
  for (int e = t; e < SD * SD; e += NT) {
    const int i = e / SD, j = e % SD;
    const double yaw = rec[MPCQP_REC_EULER + 2];
    const double cy = cos(yaw), sy = sin(yaw);
    double ac = 0.0;
    if (i == 0 && j == 6) ac = cy;
    if (i == 0 && j == 7) ac = sy;
    if (i == 1 && j == 6) ac = -sy;
    if (i == 1 && j == 7) ac = cy;
    if (i == 2 && j == 8) ac = 1.0;
    if (i >= 3 && i <= 5 && j == i + 6) ac = 1.0;
    if (i == 11 && j == ND) ac = 1.0;
    C.Ad[e] = (i == j ? 1.0 : 0.0) + ac * dt;
    C.S[N - 1][e] = (i == j) ? 2 * p.q_weights[i] : 0.0;
  }
  if (t == NT - 1) {
    // I_w = R I_b R' and its inverse (Eigen cofactor form), calculate_B_mat_c (:132-138)
    const double* R = rec + MPCQP_REC_ROT;
    const double* Ib = rec + MPCQP_REC_INERTIA;
    double tmp[9], Iw[9];
    for (int i = 0; i < 3; ++i)
      for (int j = 0; j < 3; ++j) {
        double s = 0.0;
        for (int k = 0; k < 3; ++k) s += R[i * 3 + k] * Ib[k * 3 + j];
        tmp[i * 3 + j] = s;
      }
    for (int i = 0; i < 3; ++i)
      for (int j = 0; j < 3; ++j) {
        double s = 0.0;
        for (int k = 0; k < 3; ++k) s += tmp[i * 3 + k] * R[j * 3 + k];
        Iw[i * 3 + j] = s;
      }
    auto cof = [&](int i, int j) {
      int i1 = (i + 1) % 3, i2 = (i + 2) % 3, j1 = (j + 1) % 3, j2 = (j + 2) % 3;
      return Iw[i1 * 3 + j1] * Iw[i2 * 3 + j2] - Iw[i1 * 3 + j2] * Iw[i2 * 3 + j1];
    };
    const double det = (cof(0, 0) * Iw[0] + cof(1, 0) * Iw[3]) + cof(2, 0) * Iw[6];
    const double invdet = 1.0 / det;
    for (int i = 0; i < 3; ++i)
      for (int j = 0; j < 3; ++j) C.Iwinv[j * 3 + i] = cof(i, j) * invdet;
  }
  __syncthreads();
  // S_k = Q + A_d' S_{k+1} A_d  (S_k = sum_{i>=k} (A^{i-k})' Q A^{i-k})
  for (int k = N - 2; k >= 0; --k) {
    for (int e = t; e < SD * SD; e += NT) {
      const int i = e / SD, j = e % SD;
      double s = 0.0;
      for (int u = 0; u < SD; ++u) s += C.S[k + 1][i * SD + u] * C.Ad[u * SD + j];
      C.T[e] = s;
    }
    __syncthreads();
    for (int e = t; e < SD * SD; e += NT) {
      const int i = e / SD, j = e % SD;
      double s = 0.0;
      for (int u = 0; u < SD; ++u) s += C.Ad[u * SD + i] * C.T[u * SD + j];
      C.S[k][e] = (i == j ? 2 * p.q_weights[i] : 0.0) + s;
    }
    __syncthreads();
  }
  // forward over horizon steps k: B_qp row-block k, G_k = S_k B_d(k), block column k of H
  constexpr int BQ = SD * ND;
  constexpr int EI = (N * BQ + NT - 1) / NT;
  double g_acc = 0.0;
  const double mass = rec[MPCQP_REC_MASS];
  for (int k = 0; k < N; ++k) {
    double val[EI];
#pragma unroll
    for (int q = 0; q < EI; ++q) {
      const int e = t + q * NT;
      val[q] = 0.0;
      if (e < (k + 1) * BQ) {
        const int j = e / BQ, rc = e % BQ, r = rc / ND, c = rc % ND;
        if (j < k) {
          double s = 0.0;
          for (int u = 0; u < SD; ++u) s += C.Ad[r * SD + u] * C.Bq[j][u * ND + c];
          val[q] = s;
        } else if (r >= 6 && r < 9) {
          // B_c[6:9, 3l:3l+3] = I_w^-1 skew(foot_l)  (Utils.cpp:35-41), B_d = B_c dt
          const int leg = c / 3, cc = c % 3;
          const double* fp = rec + Dm::feet + 12 * k + 3 * leg;
          // column cc of skew(v) = [[0,-v2,v1],[v2,0,-v0],[-v1,v0,0]]
          const double sk0 = cc == 0 ? 0.0 : cc == 1 ? -fp[2] : fp[1];
          const double sk1 = cc == 0 ? fp[2] : cc == 1 ? 0.0 : -fp[0];
          const double sk2 = cc == 0 ? -fp[1] : cc == 1 ? fp[0] : 0.0;
          const double* iw = C.Iwinv + (r - 6) * 3;
          double s = 0.0;
          s += iw[0] * sk0;
          s += iw[1] * sk1;
          s += iw[2] * sk2;
          val[q] = s * dt;
        } else if (r >= 9 && r < 12) {
          val[q] = ((r - 9) == (c % 3)) ? (1.0 / mass) * dt : 0.0;
        }
      }
    }
    double anew = 0.0;
    if (t < SD) {  // A_qp x0 row-block k = A_d^{k+1} x0
      const double* prev = (k == 0) ? rec + MPCQP_REC_X0 : C.a;
      for (int u = 0; u < SD; ++u) anew += C.Ad[t * SD + u] * prev[u];
    }
    __syncthreads();
#pragma unroll
    for (int q = 0; q < EI; ++q) {
      const int e = t + q * NT;
      if (e < (k + 1) * BQ) C.Bq[e / BQ][e % BQ] = val[q];
    }
    if (t < SD) {
      C.a[t] = anew;
      C.w[t] = 2 * p.q_weights[t] * (anew - rec[MPCQP_REC_XREF + SD * k + t]);
    }
    __syncthreads();
    for (int e = t; e < BQ; e += NT) {
      const int s = e / ND, b = e % ND;
      double acc = 0.0;
      for (int u = 0; u < SD; ++u) acc += C.S[k][s * SD + u] * C.Bq[k][u * ND + b];
      C.G[e] = acc;
    }
    if (t < ND * (k + 1)) {  // gradient: g_j += B_qp(k,j)' Q (A_qp x0 - x_ref)_k
      const int j = t / ND, a = t % ND;
      double acc = 0.0;
      for (int s = 0; s < SD; ++s) acc += C.Bq[j][s * ND + a] * C.w[s];
      g_acc += acc;
    }
    __syncthreads();
    // H entries (rows 0..12(k+1)-1, block column k)
    constexpr int EP = (N * ND * ND + NT - 1) / NT;
#pragma unroll
    for (int q = 0; q < EP; ++q) {
      const int e = t + q * NT;
      // diagonal block (j == k): only a <= cc, mirrored, so each location has exactly one writer
      // (the two triangles of B_k' S_k B_k round differently)
      if (e < ND * ND * (k + 1) && !((e / ND) / ND == k && (e / ND) % ND > e % ND)) {
        const int rr = e / ND, cc = e % ND;
        const int j = rr / ND, a = rr % ND;
        double s = 0.0;
        for (int u = 0; u < SD; ++u) s += C.Bq[j][u * ND + a] * C.G[u * ND + cc];
        const int col = ND * k + cc;
        if (rr == col) s += 2 * p.r_weights[cc];
        Pout[(size_t)rr * ld + col] = s;
        if (rr != col) Pout[(size_t)col * ld + rr] = s;
      }
    }
    // (next step's first barrier orders these reads of Bq/G before they are overwritten)
  }
  __syncthreads();
  if (t < Dm::n) sm.qt[t] = g_acc;
  // bounds (:223-245): per leg, identical for every horizon step
  for (int r = t; r < Dm::m; r += NT) {
    const int leg = (r % CD) / 5, row = r % 5;
    const double c = rec[MPCQP_REC_CONTACTS + leg] != 0.0 ? 1.0 : 0.0;
    double l, u;
    switch (row) {
      case 0: l = 0; u = OSQP_INF; break;
      case 1: l = -OSQP_INF; u = 0; break;
      case 2: l = 0; u = OSQP_INF; break;
      case 3: l = -OSQP_INF; u = 0; break;
      default: l = rec[MPCQP_REC_FZMIN] * c; u = rec[MPCQP_REC_FZMAX] * c; break;
    }
    sm.lo[r] = l;
    sm.hi[r] = u;
  }
  __syncthreads();
}

}  // namespace mpcqp
