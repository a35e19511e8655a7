// mpcqp_kernels.hip — CDNA4 (gfx950) kernels of the batched convex-MPC QP engine.
//
// One 512-thread workgroup (8 waves, 2 per SIMD) solves one robot instance; the hardware
// dispatcher back-fills CUs as instances finish (iteration counts differ).  Per instance:
//
//   1. condensation (ConvexMpc::calculate_qp_mats, src/a1_cpp/src/ConvexMpc.cpp:158-245)
//        S_k = Q + A_d' S_{k+1} A_d  (backward),  B_qp(k,j) = A_d B_qp(k-1,j)  (forward),
//        H[block j][block k] = B_qp(k,j)' S_k B_d(k)  (j <= k),  g_j = sum_k B_qp(k,j)' Q e_k,
//      written once to a per-instance HBM/L2 workspace (H is needed again at every rho refactor);
//   2. OSQP 0.6 Ruiz equilibration (scaling.c) on H held in REGISTERS: every thread owns a
//      4x8 tile of the 128x128 (padded) matrix, tiles row-reduced with 16-lane shuffles;
//   3. K = P~ + sigma I + A~' diag(rho) A~ and its inverse by in-register Gauss-Jordan
//      (pivot row/column broadcast through a double-buffered LDS line, one barrier per pivot);
//   4. ADMM (osqp.c) with x~ = K^-1 rhs as a register-tile mat-vec + 16-lane reduce-scatter;
//      the friction-pyramid rows are handled per foot (5 rows x 3 vars) by wave 0, with
//      termination checks / adaptive rho every 25 iterations exactly as OSQP 0.6.
//
// Arithmetic is binary64 throughout (the reference is double everywhere).
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>

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
};

// LDS image of one instance.
template <int N>
struct Smem {
  using Dm = Dim<N>;
  double rec[Dm::rec];
  double qt[Dm::n], D[Dm::n], Dinv[Dm::n], E[Dm::m], Einv[Dm::m], lo[Dm::m], hi[Dm::m];
  double A9[Dm::nf][9];  // A~ per foot: {ax0, az0, ax1, az1, ay2, az2, ay3, az3, az4}
  double BD[Dm::nf][9];  // (A~' diag(rho) A~) 3x3 block per foot, row-major
  double rho_v[Dm::m], rho_inv[Dm::m];
  int ctype[Dm::m];
  alignas(16) double rhs[NP];
  alignas(16) double xt[NP];
  double X[Dm::n], Z[Dm::m], Y[Dm::m], PX[Dm::n];
  alignas(16) double gj[2][2][NP];
  double cst[8];  // 0: c, 1: cinv, 2: rho, 3: c_temp
  int ctl[8];     // 0: instance, 1: done flag, 2: refactor flag, 3: status
  union U {
    struct C {
      double S[N][SD * SD];
      double Bq[N][SD * ND];
      double G[SD * ND];
      double Ad[SD * SD];
      double T[SD * SD];
      double Iwinv[9];
      double a[SD];
      double w[SD];
    } c;
    struct R {
      alignas(16) double Dt[NP];
      double Et[Dm::m];
      double colP[NP];
      double red[64];
    } r;
  } u;
};

// Returns v unchanged but opaque to the optimizer: values derived from it are recomputed where
// used instead of being hoisted out of the ADMM loop (which exhausts the VGPR file).
__device__ __forceinline__ int opaque(int v) {
  asm volatile("" : "+v"(v));
  return v;
}

__device__ __forceinline__ double dmax(double a, double b) { return a > b ? a : b; }
__device__ __forceinline__ double dmin(double a, double b) { return a < b ? a : b; }
__device__ __forceinline__ double dabs(double a) { return a < 0 ? -a : a; }
__device__ __forceinline__ double limit_scaling(double d) {
  d = d < MIN_SCALING ? 1.0 : d;
  return d > MAX_SCALING ? MAX_SCALING : d;
}

// ---- 16-lane reductions (a lane group shares one tile row: t = tr*16 + tc) ------------------
// Reduce-scatter: returns the reduction of v[row] for row = tc >> (4 - log2 BR) (lane groups
// of 16/BR lanes hold the same row).
template <int BR, bool MAX>
__device__ __forceinline__ double rs16(double (&v)[BR], int tc) {
  static_assert(BR == 1 || BR == 2 || BR == 4 || BR == 8, "BR must be a power of two <= 8");
  constexpr int L = BR == 1 ? 0 : BR == 2 ? 1 : BR == 4 ? 2 : 3;
  double a[BR];
#pragma unroll
  for (int i = 0; i < BR; ++i) a[i] = v[i];
#pragma unroll
  for (int s = 0; s < L; ++s) {
    const int mask = 8 >> s;
    const int half = BR >> (s + 1);
    const bool up = (tc & mask) != 0;
#pragma unroll
    for (int i = 0; i < half; ++i) {
      double send = up ? a[i] : a[i + half];
      double keep = up ? a[i + half] : a[i];
      double got = __shfl_xor(send, mask);
      a[i] = MAX ? dmax(keep, got) : keep + got;
    }
  }
  double r = a[0];
#pragma unroll
  for (int mask = 8 >> L; mask >= 1; mask >>= 1) {
    double got = __shfl_xor(r, mask);
    r = MAX ? dmax(r, got) : r + got;
  }
  return r;
}

// wave-wide (64-lane) all-reduce
__device__ __forceinline__ double wave_max(double v) {
#pragma unroll
  for (int mask = 32; mask >= 1; mask >>= 1) v = dmax(v, __shfl_xor(v, mask));
  return v;
}
__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
  for (int mask = 32; mask >= 1; mask >>= 1) v += __shfl_xor(v, mask);
  return v;
}

// ---- condensation: ConvexMpc.cpp:110-245 ----------------------------------------------------
// Writes the dense Hessian (both triangles) to Pout[ld] and leaves the gradient in sm.qt and
// the unscaled bounds in sm.lo / sm.hi.
template <int N, int NT>
__device__ void condense(Smem<N>& sm, const mpcqp_params& p, double* __restrict__ Pout, int ld) {
  using Dm = Dim<N>;
  const int t = threadIdx.x;
  auto& C = sm.u.c;
  const double* rec = sm.rec;
  const double dt = rec[MPCQP_REC_DT];
  // calculate_A_mat_c (:110-130) + A_d = I + A_c dt (:150); S_{N-1} = Q
  if (t < SD * SD) {
    const int i = t / SD, j = t % SD;
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
    C.Ad[t] = (i == j ? 1.0 : 0.0) + ac * dt;
    C.S[N - 1][t] = (i == j) ? 2 * p.q_weights[i] : 0.0;
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
    if (t < SD * SD) {
      const int i = t / SD, j = t % SD;
      double s = 0.0;
      for (int u = 0; u < SD; ++u) s += C.S[k + 1][i * SD + u] * C.Ad[u * SD + j];
      C.T[t] = s;
    }
    __syncthreads();
    if (t < SD * SD) {
      const int i = t / SD, j = t % SD;
      double s = 0.0;
      for (int u = 0; u < SD; ++u) s += C.Ad[u * SD + i] * C.T[u * SD + j];
      C.S[k][t] = (i == j ? 2 * p.q_weights[i] : 0.0) + s;
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
    if (t < BQ) {
      const int s = t / ND, b = t % ND;
      double acc = 0.0;
      for (int u = 0; u < SD; ++u) acc += C.S[k][s * SD + u] * C.Bq[k][u * ND + b];
      C.G[t] = acc;
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
  if (t < Dm::m) {
    const int leg = (t % CD) / 5, row = t % 5;
    const double c = rec[MPCQP_REC_CONTACTS + leg] != 0.0 ? 1.0 : 0.0;
    double l, u;
    switch (row) {
      case 0: l = 0; u = OSQP_INF; break;
      case 1: l = -OSQP_INF; u = 0; break;
      case 2: l = 0; u = OSQP_INF; break;
      case 3: l = -OSQP_INF; u = 0; break;
      default: l = rec[MPCQP_REC_FZMIN] * c; u = rec[MPCQP_REC_FZMAX] * c; break;
    }
    sm.lo[t] = l;
    sm.hi[t] = u;
  }
  __syncthreads();
}

// ---- register tile helpers -----------------------------------------------------------------
template <int BR>
__device__ __forceinline__ void load_tile(double (&M)[BR][BC], const double* __restrict__ P, int n,
                                          int tr, int tc) {
#pragma unroll
  for (int i = 0; i < BR; ++i) {
    const int r = tr * BR + i;
#pragma unroll
    for (int j = 0; j < BC; ++j) {
      const int c = tc * BC + j;
      M[i][j] = (r < n && c < n) ? P[(size_t)r * NP + c] : 0.0;
    }
  }
}
template <int BR>
__device__ __forceinline__ void store_tile(const double (&M)[BR][BC], double* __restrict__ P, int n,
                                           int tr, int tc) {
#pragma unroll
  for (int i = 0; i < BR; ++i) {
    const int r = tr * BR + i;
#pragma unroll
    for (int j = 0; j < BC; ++j) {
      const int c = tc * BC + j;
      if (r < n && c < n) P[(size_t)r * NP + c] = M[i][j];
    }
  }
}

// K = P~ + sigma I + A~' rho A~ (padded diagonal = 1), then in-place Gauss-Jordan inverse.
template <int N, int BR>
__device__ void build_and_invert(double (&M)[BR][BC], Smem<N>& sm, double sigma, int tr, int tc) {
  using Dm = Dim<N>;
  constexpr int n = Dm::n;
#pragma unroll
  for (int i = 0; i < BR; ++i) {
    const int r = tr * BR + i;
#pragma unroll
    for (int j = 0; j < BC; ++j) {
      const int c = tc * BC + j;
      if (r < n && c < n) {
        double v = M[i][j];
        if (r == c) v += sigma;
        if (r / 3 == c / 3) v += sm.BD[r / 3][(r % 3) * 3 + (c % 3)];
        M[i][j] = v;
      } else {
        M[i][j] = (r == c) ? 1.0 : 0.0;
      }
    }
  }
  // Gauss-Jordan: pivot k = kb*BC + ki (ki unrolled so every register index is static)
  constexpr int KB = (n + BC - 1) / BC;
  for (int kb = 0; kb < KB; ++kb) {
#pragma unroll
    for (int ki = 0; ki < BC; ++ki) {
      const int k = kb * BC + ki;
      if (k < n) {
        double* rowb = sm.gj[k & 1][0];
        double* colb = sm.gj[k & 1][1];
        const bool own_row = tr == kb * (BC / BR) + ki / BR;
        const bool own_col = tc == kb;
        if (own_row) {
#pragma unroll
          for (int j = 0; j < BC; ++j) rowb[tc * BC + j] = M[ki % BR][j];
        }
        if (own_col) {
#pragma unroll
          for (int i = 0; i < BR; ++i) colb[tr * BR + i] = M[i][ki];
        }
        __syncthreads();
        const double inv = 1.0 / rowb[k];
        double rk[BC], ck[BR];
#pragma unroll
        for (int j = 0; j < BC; ++j) rk[j] = rowb[tc * BC + j] * inv;
#pragma unroll
        for (int i = 0; i < BR; ++i) ck[i] = colb[tr * BR + i];
#pragma unroll
        for (int i = 0; i < BR; ++i)
#pragma unroll
          for (int j = 0; j < BC; ++j) M[i][j] = fma(-ck[i], rk[j], M[i][j]);
        if (own_row) {
#pragma unroll
          for (int j = 0; j < BC; ++j) M[ki % BR][j] = rk[j];
        }
        if (own_col) {
#pragma unroll
          for (int i = 0; i < BR; ++i) M[i][ki] = -ck[i] * inv;
        }
        if (own_row && own_col) M[ki % BR][ki] = inv;
      }
    }
  }
  __syncthreads();
}

// set_rho_vec (auxil.c) + A~' rho A~ blocks
template <int N>
__device__ void set_rho_and_blocks(Smem<N>& sm, double rho, bool reclassify) {
  using Dm = Dim<N>;
  const int t = threadIdx.x;
  if (t < Dm::nf) {
    const int f = t;
    double rv[5];
#pragma unroll
    for (int k = 0; k < 5; ++k) {
      const int r = 5 * f + k;
      int ct;
      if (reclassify) {
        if (sm.lo[r] < -OSQP_INF * MIN_SCALING && sm.hi[r] > OSQP_INF * MIN_SCALING)
          ct = -1;
        else if (sm.hi[r] - sm.lo[r] < RHO_TOL)
          ct = 1;
        else
          ct = 0;
        sm.ctype[r] = ct;
      } else {
        ct = sm.ctype[r];
      }
      double rr;
      if (ct == -1) {
        rr = reclassify ? RHO_MIN : sm.rho_v[r];
      } else if (ct == 1) {
        rr = RHO_EQ_OVER_RHO_INEQ * rho;
      } else {
        rr = rho;
      }
      sm.rho_v[r] = rr;
      sm.rho_inv[r] = 1. / rr;
      rv[k] = rr;
    }
    const double* a = sm.A9[f];
    double* bd = sm.BD[f];
    // rows: 0:(x,z) 1:(x,z) 2:(y,z) 3:(y,z) 4:(z)
    bd[0] = a[0] * rv[0] * a[0] + a[2] * rv[1] * a[2];
    bd[1] = 0.0;
    bd[2] = a[0] * rv[0] * a[1] + a[2] * rv[1] * a[3];
    bd[3] = 0.0;
    bd[4] = a[4] * rv[2] * a[4] + a[6] * rv[3] * a[6];
    bd[5] = a[4] * rv[2] * a[5] + a[6] * rv[3] * a[7];
    bd[6] = bd[2];
    bd[7] = bd[5];
    bd[8] = a[1] * rv[0] * a[1] + a[3] * rv[1] * a[3] + a[5] * rv[2] * a[5] + a[7] * rv[3] * a[7] +
            a[8] * rv[4] * a[8];
  }
}

// ---- the solver kernel ---------------------------------------------------------------------
template <int N, int BR>
__global__ __launch_bounds__((NP / BR) * 16) void solve_kernel(
    const double* __restrict__ recs, int batch, mpcqp_result* __restrict__ results,
    double* __restrict__ solution, double* __restrict__ work,
    double* __restrict__ trace, int trace_cap, mpcqp_params p) {
  using Dm = Dim<N>;
  constexpr int NT = (NP / BR) * 16;
  constexpr int n = Dm::n, m = Dm::m, nf = Dm::nf;
  static_assert(nf <= 64, "feet must fit in wave 0");
  __shared__ Smem<N> sm;
  const int t = threadIdx.x;
  const int tr = t >> 4, tc = t & 15;
  const int lane = t & 63;
  const bool wave0 = t < 64;
  const int inst = blockIdx.x;
  if (inst >= batch) return;
  double* __restrict__ Pw = work + (size_t)inst * NP * NP;
  const double alpha = p.alpha, sigma = p.sigma;
  double M[BR][BC];
  {
    const double* rec_g = recs + (size_t)inst * Dm::rec;
    bool bad = false;
    for (int e = t; e < Dm::rec; e += NT) {
      const double v = rec_g[e];
      sm.rec[e] = v;
      bad |= !isfinite(v);
    }
    if (__syncthreads_or(bad)) {
      if (t == 0) {
        mpcqp_result r;
        for (int k = 0; k < ND; ++k) { r.u0[k] = NAN; r.f_body[k] = 0.0; }
        r.obj_val = NAN; r.pri_res = NAN; r.dua_res = NAN; r.rho = p.rho;
        r.status = MPCQP_STATUS_NAN_INPUT; r.iters = 0; r.rho_updates = 0; r.nan_legs = 0xF;
        results[inst] = r;
      }
      if (solution)
        for (int e = t; e < n; e += NT) solution[(size_t)inst * n + e] = NAN;
      return;
    }

    if (t == 0) sm.ctl[2] = 0;
    // ---- 1. condensation -> workspace (unscaled H), sm.qt (gradient), sm.lo/hi --------------
    condense<N, NT>(sm, p, Pw, NP);

    // ---- 2. OSQP scale_data (Ruiz), P in registers ------------------------------------------
    load_tile<BR>(M, Pw, n, tr, tc);
    if (t < n) { sm.D[t] = 1.0; }
    if (t < m) { sm.E[t] = 1.0; }
    if (t < nf) {
      const double mu = sm.rec[MPCQP_REC_MU];
      double* a = sm.A9[t];
      a[0] = 1; a[1] = mu; a[2] = 1; a[3] = -mu; a[4] = 1; a[5] = mu; a[6] = 1; a[7] = -mu; a[8] = 1;
    }
    if (t == 0) sm.cst[0] = 1.0;
    __syncthreads();
    auto& RS = sm.u.r;
    for (int pass = 0; pass < p.scaling; ++pass) {
      // colnorm(P) = rownorm (P symmetric, both triangles stored identically)
      {
        double pm[BR];
#pragma unroll
        for (int i = 0; i < BR; ++i) {
          double mx = 0.0;
#pragma unroll
          for (int j = 0; j < BC; ++j) mx = dmax(mx, dabs(M[i][j]));
          pm[i] = mx;
        }
        const double r = rs16<BR, true>(pm, tc);
        if ((tc & ((16 / BR) - 1)) == 0) RS.colP[tr * BR + (tc >> (4 - (BR == 1 ? 0 : BR == 2 ? 1 : BR == 4 ? 2 : 3)))] = r;
      }
      __syncthreads();
      if (t < n) {  // D_temp (compute_inf_norm_cols_KKT + limit + sqrt + recip)
        const int f = t / 3, a = t % 3;
        const double* A9 = sm.A9[f];
        double ca;
        if (a == 0) ca = dmax(dabs(A9[0]), dabs(A9[2]));
        else if (a == 1) ca = dmax(dabs(A9[4]), dabs(A9[6]));
        else ca = dmax(dmax(dmax(dmax(dabs(A9[1]), dabs(A9[3])), dabs(A9[5])), dabs(A9[7])), dabs(A9[8]));
        double d = dmax(RS.colP[t], ca);
        d = limit_scaling(d);
        RS.Dt[t] = 1.0 / sqrt(d);
      }
      if (t < m) {
        const int f = t / 5, k = t % 5;
        const double* A9 = sm.A9[f];
        double e = (k < 4) ? dmax(dabs(A9[2 * k]), dabs(A9[2 * k + 1])) : dabs(A9[8]);
        e = limit_scaling(e);
        RS.Et[t] = 1.0 / sqrt(e);
      }
      __syncthreads();
      // P <- D P D (premult by row of the upper-triangle entry, then postmult by its column)
#pragma unroll
      for (int i = 0; i < BR; ++i) {
        const int r = tr * BR + i;
#pragma unroll
        for (int j = 0; j < BC; ++j) {
          const int c = tc * BC + j;
          if (r < n && c < n) {
            const int pr = r < c ? r : c, pc = r < c ? c : r;
            M[i][j] = (M[i][j] * RS.Dt[pr]) * RS.Dt[pc];
          }
        }
      }
      if (t < m) {  // A <- E A D
        const int f = t / 5, k = t % 5;
        double* A9 = sm.A9[f];
        const double et = RS.Et[t];
        if (k < 4) {
          const int mainc = 3 * f + (k < 2 ? 0 : 1);
          A9[2 * k] = (A9[2 * k] * et) * RS.Dt[mainc];
          A9[2 * k + 1] = (A9[2 * k + 1] * et) * RS.Dt[3 * f + 2];
        } else {
          A9[8] = (A9[8] * et) * RS.Dt[3 * f + 2];
        }
        sm.E[t] *= et;
      }
      if (t < n) {
        sm.qt[t] = RS.Dt[t] * sm.qt[t];
        sm.D[t] = sm.D[t] * RS.Dt[t];
      }
      __syncthreads();
      // cost normalization
      {
        double pm[BR];
#pragma unroll
        for (int i = 0; i < BR; ++i) {
          double mx = 0.0;
#pragma unroll
          for (int j = 0; j < BC; ++j) mx = dmax(mx, dabs(M[i][j]));
          pm[i] = mx;
        }
        const double r = rs16<BR, true>(pm, tc);
        if ((tc & ((16 / BR) - 1)) == 0) RS.colP[tr * BR + (tc >> (4 - (BR == 1 ? 0 : BR == 2 ? 1 : BR == 4 ? 2 : 3)))] = r;
      }
      __syncthreads();
      if (wave0) {
        double s = 0.0, qn = 0.0;
        for (int c = lane; c < n; c += 64) {
          s += RS.colP[c];
          qn = dmax(qn, dabs(sm.qt[c]));
        }
        s = wave_sum(s);
        qn = wave_max(qn);
        double c_temp = s / n;
        qn = limit_scaling(qn);
        c_temp = dmax(c_temp, qn);
        c_temp = limit_scaling(c_temp);
        c_temp = 1. / c_temp;
        if (lane == 0) {
          sm.cst[3] = c_temp;
          sm.cst[0] *= c_temp;
        }
      }
      __syncthreads();
      const double c_temp = sm.cst[3];
#pragma unroll
      for (int i = 0; i < BR; ++i)
#pragma unroll
        for (int j = 0; j < BC; ++j) M[i][j] *= c_temp;
      if (t < n) sm.qt[t] *= c_temp;
      __syncthreads();
    }
    // cinv, Dinv, Einv, scaled bounds
    if (t == 0) sm.cst[1] = 1. / sm.cst[0];
    if (t < n) sm.Dinv[t] = 1. / sm.D[t];
    if (t < m) {
      sm.Einv[t] = 1. / sm.E[t];
      sm.lo[t] = sm.E[t] * sm.lo[t];
      sm.hi[t] = sm.E[t] * sm.hi[t];
    }
    __syncthreads();
    store_tile<BR>(M, Pw, n, tr, tc);  // scaled P~ kept for rho refactorizations
    double rho = dmin(dmax(p.rho, RHO_MIN), RHO_MAX);
    set_rho_and_blocks<N>(sm, rho, true);
    // zero iterates (cold start) and padded mat-vec lanes
    for (int e = t; e < NP; e += NT) { sm.rhs[e] = 0.0; sm.xt[e] = 0.0; }
    if (t < n) { sm.X[t] = 0.0; sm.PX[t] = 0.0; }
    if (t < m) { sm.Z[t] = 0.0; sm.Y[t] = 0.0; }
    __syncthreads();
    build_and_invert<N, BR>(M, sm, sigma, tr, tc);

    // ---- 3. ADMM ------------------------------------------------------------------------------
    const double cinv = sm.cst[1], cc = sm.cst[0];
    int status = MPCQP_STATUS_UNSOLVED, iters = 0, rho_updates = 0;
    double pri_res = 0.0, dua_res = 0.0;
    int ntrace = 0;
    for (int iter = 1; iter <= p.max_iter; ++iter) {
      const int t = opaque(threadIdx.x);
      const int tr = t >> 4, tc = t & 15;
      const int lane = t & 63;
      // (a) rhs = sigma x - q~ + A~'(rho z - y)   [compute_rhs + reduced KKT right-hand side]
      if (t < nf) {
        const int f = t;
        const double* a = sm.A9[f];
        double tt[5];
#pragma unroll
        for (int k = 0; k < 5; ++k) tt[k] = sm.rho_v[5 * f + k] * sm.Z[5 * f + k] - sm.Y[5 * f + k];
        const double bx = (sigma * sm.X[3 * f + 0] - sm.qt[3 * f + 0]);
        const double by = (sigma * sm.X[3 * f + 1] - sm.qt[3 * f + 1]);
        const double bz = (sigma * sm.X[3 * f + 2] - sm.qt[3 * f + 2]);
        sm.rhs[3 * f + 0] = (bx + a[0] * tt[0]) + a[2] * tt[1];
        sm.rhs[3 * f + 1] = (by + a[4] * tt[2]) + a[6] * tt[3];
        sm.rhs[3 * f + 2] = ((((bz + a[1] * tt[0]) + a[3] * tt[1]) + a[5] * tt[2]) + a[7] * tt[3]) + a[8] * tt[4];
      }
      __syncthreads();
      // (b) x~ = K^-1 rhs
      {
        double v[BC];
#pragma unroll
        for (int j = 0; j < BC; ++j) v[j] = sm.rhs[tc * BC + j];
        double s[BR];
#pragma unroll
        for (int i = 0; i < BR; ++i) {
          double acc = 0.0;
#pragma unroll
          for (int j = 0; j < BC; ++j) acc = fma(M[i][j], v[j], acc);
          s[i] = acc;
        }
        const double r = rs16<BR, false>(s, tc);
        if ((tc & ((16 / BR) - 1)) == 0) sm.xt[tr * BR + (tc >> (4 - (BR == 1 ? 0 : BR == 2 ? 1 : BR == 4 ? 2 : 3)))] = r;
      }
      __syncthreads();
      // (c) x, z, y updates per foot (update_x, update_z + project, update_y)
      const bool is_check = p.check_termination && (iter % p.check_termination == 0);
      const bool is_adapt = p.adaptive_rho && p.adaptive_rho_interval && (iter % p.adaptive_rho_interval == 0);
      const bool last = iter == p.max_iter;
      const bool need_info = is_check || is_adapt || last;
      double part[14];
#pragma unroll
      for (int k = 0; k < 14; ++k) part[k] = 0.0;
      double dxv[3] = {0, 0, 0}, dyv[5] = {0, 0, 0, 0, 0}, pxo[3] = {0, 0, 0}, pxn[3] = {0, 0, 0};
      if (t < nf) {
        const int f = t;
        const double* a = sm.A9[f];
        const double xt0 = sm.xt[3 * f], xt1 = sm.xt[3 * f + 1], xt2 = sm.xt[3 * f + 2];
        double zt[5];
        zt[0] = a[0] * xt0 + a[1] * xt2;
        zt[1] = a[2] * xt0 + a[3] * xt2;
        zt[2] = a[4] * xt1 + a[5] * xt2;
        zt[3] = a[6] * xt1 + a[7] * xt2;
        zt[4] = a[8] * xt2;
        const double xtv[3] = {xt0, xt1, xt2};
        const double* bd = sm.BD[f];
        double xn[3];
#pragma unroll
        for (int k = 0; k < 3; ++k) {
          const double xo = sm.X[3 * f + k];
          xn[k] = alpha * xtv[k] + (1.0 - alpha) * xo;
          dxv[k] = xn[k] - xo;
          // P~ x~ from the KKT identity: (P~ + sigma I + A~'rho A~) x~ = rhs
          const double pxt = sm.rhs[3 * f + k] - sigma * xtv[k] -
                             ((bd[3 * k] * xt0 + bd[3 * k + 1] * xt1) + bd[3 * k + 2] * xt2);
          pxo[k] = sm.PX[3 * f + k];
          pxn[k] = alpha * pxt + (1.0 - alpha) * pxo[k];
          sm.X[3 * f + k] = xn[k];
          sm.PX[3 * f + k] = pxn[k];
        }
        double zn[5], yn[5];
#pragma unroll
        for (int k = 0; k < 5; ++k) {
          const int r = 5 * f + k;
          const double zo = sm.Z[r], yo = sm.Y[r];
          const double zr = alpha * zt[k] + (1.0 - alpha) * zo;
          zn[k] = dmin(dmax(zr + sm.rho_inv[r] * yo, sm.lo[r]), sm.hi[r]);
          dyv[k] = sm.rho_v[r] * (zr - zn[k]);
          yn[k] = yo + dyv[k];
          sm.Z[r] = zn[k];
          sm.Y[r] = yn[k];
        }
        if (need_info) {
          double ax[5];
          ax[0] = a[0] * xn[0] + a[1] * xn[2];
          ax[1] = a[2] * xn[0] + a[3] * xn[2];
          ax[2] = a[4] * xn[1] + a[5] * xn[2];
          ax[3] = a[6] * xn[1] + a[7] * xn[2];
          ax[4] = a[8] * xn[2];
#pragma unroll
          for (int k = 0; k < 5; ++k) {
            const int r = 5 * f + k;
            const double pr = ax[k] + (-1.0) * zn[k];
            const double ei = sm.Einv[r];
            part[0] = dmax(part[0], dabs(ei * pr));
            part[1] = dmax(part[1], dabs(pr));
            part[2] = dmax(part[2], dabs(ei * zn[k]));
            part[3] = dmax(part[3], dabs(zn[k]));
            part[4] = dmax(part[4], dabs(ei * ax[k]));
            part[5] = dmax(part[5], dabs(ax[k]));
          }
          double aty[3];
          aty[0] = a[0] * yn[0] + a[2] * yn[1];
          aty[1] = a[4] * yn[2] + a[6] * yn[3];
          aty[2] = (((a[1] * yn[0] + a[3] * yn[1]) + a[5] * yn[2]) + a[7] * yn[3]) + a[8] * yn[4];
#pragma unroll
          for (int k = 0; k < 3; ++k) {
            const int c = 3 * f + k;
            const double di = sm.Dinv[c], q = sm.qt[c];
            const double d = (q + 1.0 * pxn[k]) + 1.0 * aty[k];
            part[6] = dmax(part[6], dabs(di * d));
            part[7] = dmax(part[7], dabs(d));
            part[8] = dmax(part[8], dabs(di * q));
            part[9] = dmax(part[9], dabs(q));
            part[10] = dmax(part[10], dabs(di * aty[k]));
            part[11] = dmax(part[11], dabs(aty[k]));
            part[12] = dmax(part[12], dabs(di * pxn[k]));
            part[13] = dmax(part[13], dabs(pxn[k]));
          }
        }
      }
      if (need_info) {
        if (wave0) {
          double mx[14];
#pragma unroll
          for (int k = 0; k < 14; ++k) mx[k] = wave_max(part[k]);
          pri_res = mx[0];
          dua_res = cinv * mx[6];
          iters = iter;
          int st = MPCQP_STATUS_UNSOLVED;
          bool done = false;
          // check_termination (approximate = 0, then 1 at max_iter)
          for (int approx = 0; approx < 2 && !done; ++approx) {
            if (approx == 1 && !last) break;
            if (!is_check && !last) break;
            double eps_abs = p.eps_abs, eps_rel = p.eps_rel, eps_pinf = p.eps_prim_inf, eps_dinf = p.eps_dual_inf;
            if (pri_res > OSQP_INF || dua_res > OSQP_INF) {
              st = MPCQP_STATUS_NON_CVX;
              done = true;
              break;
            }
            if (approx) { eps_abs *= 10; eps_rel *= 10; eps_pinf *= 10; eps_dinf *= 10; }
            const double eps_prim = eps_abs + eps_rel * dmax(mx[2], mx[4]);
            const bool prim_ok = pri_res < eps_prim;
            bool prim_inf = false, dual_inf = false;
            if (!prim_ok) {
              // is_primal_infeasible: project delta_y onto the polar of the recession cone
              double ndy = 0.0, lhs = 0.0;
              double dyp[5];
#pragma unroll
              for (int k = 0; k < 5; ++k) {
                dyp[k] = dyv[k];
                if (t < nf) {
                  const int r = 5 * t + k;
                  if (sm.hi[r] > OSQP_INF * MIN_SCALING) {
                    if (sm.lo[r] < -OSQP_INF * MIN_SCALING) dyp[k] = 0.0;
                    else dyp[k] = dmin(dyp[k], 0.0);
                  } else if (sm.lo[r] < -OSQP_INF * MIN_SCALING) {
                    dyp[k] = dmax(dyp[k], 0.0);
                  }
                  dyv[k] = dyp[k];
                  ndy = dmax(ndy, dabs(sm.E[r] * dyp[k]));
                  lhs += sm.hi[r] * dmax(dyp[k], 0.0) + sm.lo[r] * dmin(dyp[k], 0.0);
                } else {
                  dyp[k] = 0.0;
                }
              }
              ndy = wave_max(ndy);
              if (ndy > DIV_TOL) {
                lhs = wave_sum(lhs);
                if (lhs < eps_pinf * ndy) {
                  double atn = 0.0;
                  if (t < nf) {
                    const double* a = sm.A9[t];
                    const double at0 = a[0] * dyp[0] + a[2] * dyp[1];
                    const double at1 = a[4] * dyp[2] + a[6] * dyp[3];
                    const double at2 = (((a[1] * dyp[0] + a[3] * dyp[1]) + a[5] * dyp[2]) + a[7] * dyp[3]) + a[8] * dyp[4];
                    atn = dmax(dmax(dabs(sm.Dinv[3 * t] * at0), dabs(sm.Dinv[3 * t + 1] * at1)),
                               dabs(sm.Dinv[3 * t + 2] * at2));
                  }
                  atn = wave_max(atn);
                  prim_inf = atn < eps_pinf * ndy;
                }
              }
            }
            const double eps_dual = eps_abs + eps_rel * (cinv * dmax(dmax(mx[8], mx[10]), mx[12]));
            const bool dual_ok = dua_res < eps_dual;
            if (!dual_ok) {
              // is_dual_infeasible
              double ndx = 0.0, qdx = 0.0, npdx = 0.0;
              if (t < nf) {
#pragma unroll
                for (int k = 0; k < 3; ++k) {
                  const int c = 3 * t + k;
                  ndx = dmax(ndx, dabs(sm.D[c] * dxv[k]));
                  qdx += sm.qt[c] * dxv[k];
                  npdx = dmax(npdx, dabs(sm.Dinv[c] * (pxn[k] - pxo[k])));
                }
              }
              ndx = wave_max(ndx);
              if (ndx > DIV_TOL) {
                qdx = wave_sum(qdx);
                if (qdx < cc * eps_dinf * ndx) {
                  npdx = wave_max(npdx);
                  if (npdx < cc * eps_dinf * ndx) {
                    double viol = 0.0;
                    if (t < nf) {
                      const double* a = sm.A9[t];
                      double adx[5];
                      adx[0] = a[0] * dxv[0] + a[1] * dxv[2];
                      adx[1] = a[2] * dxv[0] + a[3] * dxv[2];
                      adx[2] = a[4] * dxv[1] + a[5] * dxv[2];
                      adx[3] = a[6] * dxv[1] + a[7] * dxv[2];
                      adx[4] = a[8] * dxv[2];
#pragma unroll
                      for (int k = 0; k < 5; ++k) {
                        const int r = 5 * t + k;
                        const double v = sm.Einv[r] * adx[k];
                        if ((sm.hi[r] < OSQP_INF * MIN_SCALING && v > eps_dinf * ndx) ||
                            (sm.lo[r] > -OSQP_INF * MIN_SCALING && v < -eps_dinf * ndx))
                          viol = 1.0;
                      }
                    }
                    viol = wave_max(viol);
                    dual_inf = viol == 0.0;
                  }
                }
              }
            }
            if (prim_ok && dual_ok) {
              st = approx ? MPCQP_STATUS_SOLVED_INACCURATE : MPCQP_STATUS_SOLVED;
              done = true;
            } else if (prim_inf) {
              st = approx ? MPCQP_STATUS_PRIMAL_INFEASIBLE_INACCURATE : MPCQP_STATUS_PRIMAL_INFEASIBLE;
              done = true;
            } else if (dual_inf) {
              st = approx ? MPCQP_STATUS_DUAL_INFEASIBLE_INACCURATE : MPCQP_STATUS_DUAL_INFEASIBLE;
              done = true;
            }
            if (!done && approx == 0 && is_adapt) {
              // adapt_rho (runs before the post-loop approximate check in osqp_solve)
              const double pr_n = mx[1] / (dmax(mx[3], mx[5]) + DIV_TOL);
              const double du_n = mx[7] / (dmax(dmax(mx[9], mx[11]), mx[13]) + DIV_TOL);
              double est = rho * sqrt(pr_n / (du_n + DIV_TOL));
              est = dmin(dmax(est, RHO_MIN), RHO_MAX);
              if (est > rho * p.adaptive_rho_tolerance || est < rho / p.adaptive_rho_tolerance) {
                rho = dmin(dmax(est, RHO_MIN), RHO_MAX);
                rho_updates += 1;
                if (lane == 0) sm.ctl[2] = last ? 0 : 1;
              }
            }
          }
          if (!is_check && !last && is_adapt) {
            // adapt-only iteration (adaptive_rho_interval not a multiple of check_termination)
            const double pr_n = mx[1] / (dmax(mx[3], mx[5]) + DIV_TOL);
            const double du_n = mx[7] / (dmax(dmax(mx[9], mx[11]), mx[13]) + DIV_TOL);
            double est = rho * sqrt(pr_n / (du_n + DIV_TOL));
            est = dmin(dmax(est, RHO_MIN), RHO_MAX);
            if (est > rho * p.adaptive_rho_tolerance || est < rho / p.adaptive_rho_tolerance) {
              rho = dmin(dmax(est, RHO_MIN), RHO_MAX);
              rho_updates += 1;
              if (lane == 0) sm.ctl[2] = 1;
            }
          }
          if (last && !done) st = MPCQP_STATUS_MAX_ITER_REACHED;
          if (last) done = true;
          status = st;
          if (lane == 0) {
            sm.ctl[1] = done ? 1 : 0;
            sm.ctl[3] = st;
            sm.cst[2] = rho;
            if (trace && inst < trace_cap && ntrace < MPCQP_TRACE_LEN && is_check) {
              double* tp = trace + ((size_t)inst * MPCQP_TRACE_LEN + ntrace) * 4;
              tp[0] = iter; tp[1] = pri_res; tp[2] = dua_res; tp[3] = rho;
            }
          }
          ntrace += is_check ? 1 : 0;
        }
        __syncthreads();
        const bool done = sm.ctl[1] != 0;
        rho = sm.cst[2];
        if (sm.ctl[2]) {
          // osqp_update_rho: new rho_vec, refactor K (reload P~ from the workspace)
          __syncthreads();
          if (t == 0) sm.ctl[2] = 0;
          set_rho_and_blocks<N>(sm, rho, false);
          load_tile<BR>(M, Pw, n, tr, tc);
          __syncthreads();
          build_and_invert<N, BR>(M, sm, sigma, tr, tc);
        }
        if (done) {
          status = sm.ctl[3];
          break;
        }
      }
    }
    if (t == 0) sm.ctl[2] = 0;
    // ---- 4. store_solution + unscale + compute_grf extraction -----------------------------------
    const bool has_sol = status != MPCQP_STATUS_PRIMAL_INFEASIBLE &&
                         status != MPCQP_STATUS_PRIMAL_INFEASIBLE_INACCURATE &&
                         status != MPCQP_STATUS_DUAL_INFEASIBLE &&
                         status != MPCQP_STATUS_DUAL_INFEASIBLE_INACCURATE &&
                         status != MPCQP_STATUS_NON_CVX;
    if (wave0) {
      double ob = 0.0;
      if (t < nf) {
#pragma unroll
        for (int k = 0; k < 3; ++k) {
          const int c = 3 * t + k;
          ob += 0.5 * sm.X[c] * sm.PX[c] + sm.qt[c] * sm.X[c];
        }
      }
      ob = wave_sum(ob);
      double xs[3] = {NAN, NAN, NAN};
      if (t < 4 && has_sol) {
#pragma unroll
        for (int k = 0; k < 3; ++k) xs[k] = sm.D[3 * t + k] * sm.X[3 * t + k];
      }
      if (t < 4) {
        mpcqp_result* r = results + inst;
        const double* R = sm.rec + MPCQP_REC_ROT;
        const double nrm = sqrt(xs[0] * xs[0] + xs[1] * xs[1] + xs[2] * xs[2]);
        const bool nanleg = isnan(nrm);
#pragma unroll
        for (int k = 0; k < 3; ++k) {
          r->u0[3 * t + k] = xs[k];
          double s = 0.0;
          s += R[0 * 3 + k] * xs[0];
          s += R[1 * 3 + k] * xs[1];
          s += R[2 * 3 + k] * xs[2];
          r->f_body[3 * t + k] = nanleg ? 0.0 : s;
        }
        const unsigned long long nb = __ballot(nanleg);
        if (t == 0) {
          r->nan_legs = (int)(nb & 0xFull);
          double obj;
          if (has_sol) obj = ob * cinv;
          else if (status == MPCQP_STATUS_PRIMAL_INFEASIBLE || status == MPCQP_STATUS_PRIMAL_INFEASIBLE_INACCURATE) obj = OSQP_INF;
          else if (status == MPCQP_STATUS_DUAL_INFEASIBLE || status == MPCQP_STATUS_DUAL_INFEASIBLE_INACCURATE) obj = -OSQP_INF;
          else obj = NAN;
          r->obj_val = obj;
          r->pri_res = pri_res;
          r->dua_res = dua_res;
          r->rho = rho;
          r->status = status;
          r->iters = iters;
          r->rho_updates = rho_updates;
        }
      }
    }
    if (solution) {
      for (int e = t; e < n; e += NT)
        solution[(size_t)inst * n + e] = has_sol ? sm.D[e] * sm.X[e] : NAN;
    }
  }
}

// Formulation-only kernel (P0 parity): dense H (row-major n x n), g, l, u.
template <int N>
__global__ __launch_bounds__(256) void build_qp_kernel(const double* __restrict__ recs, int batch,
                                                       double* __restrict__ P, double* __restrict__ q,
                                                       double* __restrict__ l, double* __restrict__ u,
                                                       mpcqp_params p) {
  using Dm = Dim<N>;
  __shared__ Smem<N> sm;
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

// ---- launch table --------------------------------------------------------------------------
template <int N>
static hipError_t launch_solve(const LaunchArgs& a) {
  constexpr int BR = SOLVE_BR;
  constexpr int NT = (NP / BR) * 16;
  hipLaunchKernelGGL((solve_kernel<N, BR>), dim3(a.grid), dim3(NT), 0, (hipStream_t)a.stream, a.recs,
                     a.batch, a.results, a.solution, a.work, a.trace, a.trace_cap, a.p);
  return hipGetLastError();
}
template <int N>
static hipError_t launch_build(const LaunchArgs& a, double* P, double* q, double* l, double* u) {
  hipLaunchKernelGGL((build_qp_kernel<N>), dim3(a.batch), dim3(256), 0, (hipStream_t)a.stream, a.recs,
                     a.batch, P, q, l, u, a.p);
  return hipGetLastError();
}
template <int N>
static hipError_t occupancy(int* blocks) {
  constexpr int BR = SOLVE_BR;
  constexpr int NT = (NP / BR) * 16;
  return hipOccupancyMaxActiveBlocksPerMultiprocessor(blocks, solve_kernel<N, BR>, NT, 0);
}

#ifndef MPCQP_FOR_EACH_N
#define MPCQP_FOR_EACH_N(X) X(1) X(2) X(3) X(4) X(5) X(6) X(7) X(8) X(9) X(10)
#endif

hipError_t launch_solve_any(const LaunchArgs& a) {
  switch (a.p.horizon) {
#define CASE(K) \
  case K: return launch_solve<K>(a);
    MPCQP_FOR_EACH_N(CASE)
#undef CASE
    default: return hipErrorInvalidValue;
  }
}
hipError_t launch_build_any(const LaunchArgs& a, double* P, double* q, double* l, double* u) {
  switch (a.p.horizon) {
#define CASE(K) \
  case K: return launch_build<K>(a, P, q, l, u);
    MPCQP_FOR_EACH_N(CASE)
#undef CASE
    default: return hipErrorInvalidValue;
  }
}
hipError_t occupancy_any(int horizon, int* blocks) {
  switch (horizon) {
#define CASE(K) \
  case K: return occupancy<K>(blocks);
    MPCQP_FOR_EACH_N(CASE)
#undef CASE
    default: return hipErrorInvalidValue;
  }
}
int solve_threads() { return (NP / SOLVE_BR) * 16; }

}  // namespace mpcqp
