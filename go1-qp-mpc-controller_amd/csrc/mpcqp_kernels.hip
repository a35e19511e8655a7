// mpcqp_kernels.hip — dense K^-1 cross-check solver (debug library only, mpcqp_debug_set_solver 1).
//
// One workgroup solves one robot.  Its threads form one 16-lane group per FOOT (4 per horizon
// step; 40 groups = 640 threads = 10 waves at N = 10).  Group f owns, in registers, the 3 rows of
// the KKT matrix / its inverse that belong to foot f's force (fx, fy, fz), split in 16 column
// tiles of BC = 8; lanes 0-4 of the group own the foot's 5 friction-pyramid rows, lanes 5-7 its 3
// variables.  Per robot:
//
//   1. condensation (ConvexMpc::calculate_qp_mats, src/a1_cpp/src/ConvexMpc.cpp:158-245)
//        S_k = Q + A_d' S_{k+1} A_d (backward), B_qp(k,j) = A_d B_qp(k-1,j) (forward in LDS),
//        H_jk = B_qp(k,j)' S_k B_d(k) (j <= k), g_j = sum_k B_qp(k,j)' Q (A^{k+1} x0 - x_ref_k);
//      H goes to a per-robot HBM/L2 workspace (it is re-read at every rho refactor);
//   2. OSQP 0.6 Ruiz equilibration (scaling.c) on P held in registers; column norms = row norms
//      of the symmetric tiles, reduced inside each 16-lane group with DPP;
//   3. K = P~ + sigma I + A~' diag(rho) A~ and its inverse by block Gauss-Jordan with the foot's
//      3x3 diagonal block as pivot (one barrier per foot);
//   4. ADMM (osqp.c): x~ = K^-1 rhs is a register-tile mat-vec + 16-lane DPP all-reduce that
//      lands x~ of foot f in group f, where the relaxation / projection / dual update and the
//      next right-hand side are computed lane-parallel — ONE barrier per iteration; every 25
//      iterations the termination test and adaptive rho run redundantly in every thread on
//      workgroup-reduced norms (exactly OSQP 0.6's tests, see oracle/mpc_oracle.c);
//   5. unscaling and compute_grf's extraction f_i = R^T u0[3i:3i+3] with its NaN guard.
//
// Arithmetic is binary64 throughout (the reference is double everywhere).
#include "mpcqp_device.h"

namespace mpcqp {

// LDS image of one robot.  The per-row / per-variable ADMM state lives in registers of the
// owning lanes; LDS only carries what crosses lanes.
template <int N>
struct Smem {
  using Dm = Dim<N>;
  double rec[Dm::rec];
  double lo[Dm::m], hi[Dm::m];  // condensation output: unscaled bounds
  double qt[Dm::n];             // condensation output: gradient
  double rowc[Dm::m][4];        // scaled A~ row (coefficients on fx, fy, fz) and its rho
  double BD[Dm::n][3];          // (A~' diag(rho) A~) row of each variable (3x3 block per foot)
  alignas(16) double rhs[2][Dm::NP];  // KKT right-hand side, double-buffered by iteration parity
  alignas(16) double Dt[Dm::NP];      // Ruiz D_temp
  double red[2][Dm::NW][16];          // workgroup reductions (double-buffered)
  double info[Dm::NW][16];            // per-wave maxima of the termination / rho norms
  double cst[4];                      // {cost scaling c, rho, pri_res, dua_res}
  union U {
    CondScratch<N> c;
    struct G {  // block Gauss-Jordan broadcast lines (double-buffered by pivot parity)
      alignas(16) double r[2][3][Dm::NP];  // P^-1 * pivot rows
      double ck[2][Dm::NG][9];             // every group's 3x3 block of the pivot columns
      double pinv[2][9];                   // P^-1
    } g;
  } u;
};

// Workgroup all-reduce of K values (every thread returns the same K results).  `slot` alternates
// between calls so a buffer is never rewritten before every thread has read it (the barrier of
// the following call orders the reads of the previous one).
template <int N, int K, bool MAX>
__device__ __forceinline__ void wg_reduce(Smem<N>& sm, double (&v)[K], int& slot) {
  using Dm = Dim<N>;
  static_assert(K <= 16, "");
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
#pragma unroll
  for (int k = 0; k < K; ++k) v[k] = MAX ? wave_max(v[k]) : wave_sum(v[k]);
  if (lane == 0) {
#pragma unroll
    for (int k = 0; k < K; ++k) sm.red[slot][wave][k] = v[k];
  }
  __syncthreads();
#pragma unroll
  for (int k = 0; k < K; ++k) {
    double r = sm.red[slot][0][k];
    for (int w = 1; w < Dm::NW; ++w) r = MAX ? dmax(r, sm.red[slot][w][k]) : r + sm.red[slot][w][k];
    v[k] = r;
  }
  slot ^= 1;
}

// ---- register tile: rows 3f..3f+2 (foot f's forces) x cols tc*BC .. tc*BC+BC-1 ----------------
template <int N>
__device__ __forceinline__ void load_tile(double (&M)[3][Dim<N>::BC], const double* __restrict__ P, int f,
                                          int tc) {
  using Dm = Dim<N>;
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    const int r = 3 * f + i;
#pragma unroll
    for (int j = 0; j < Dm::BC; ++j) {
      const int c = tc * Dm::BC + j;
      M[i][j] = (r < Dm::n && c < Dm::n) ? P[(size_t)r * Dm::NP + c] : 0.0;
    }
  }
}
template <int N>
__device__ __forceinline__ void store_tile(const double (&M)[3][Dim<N>::BC], double* __restrict__ P, int f,
                                           int tc) {
  using Dm = Dim<N>;
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    const int r = 3 * f + i;
#pragma unroll
    for (int j = 0; j < Dm::BC; ++j) {
      const int c = tc * Dm::BC + j;
      if (r < Dm::n && c < Dm::n) P[(size_t)r * Dm::NP + c] = M[i][j];
    }
  }
}

// Workgroup sum of s and max of mx in one round trip.
template <int N>
__device__ __forceinline__ void wg_sum_max(Smem<N>& sm, double& s, double& mx, int& slot) {
  using Dm = Dim<N>;
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  s = wave_sum(s);
  mx = wave_max(mx);
  if (lane == 0) {
    sm.red[slot][wave][0] = s;
    sm.red[slot][wave][1] = mx;
  }
  __syncthreads();
  double rs = sm.red[slot][0][0], rm = sm.red[slot][0][1];
  for (int w = 1; w < Dm::NW; ++w) {
    rs = rs + sm.red[slot][w][0];
    rm = dmax(rm, sm.red[slot][w][1]);
  }
  s = rs;
  mx = rm;
  slot ^= 1;
}

// (A~' diag(rho) A~) row of variable 3f+a from the foot's five rows (sm.rowc, written by the
// row lanes of the same group = same wave).
template <int N>
__device__ __forceinline__ void bd_row(const Smem<N>& sm, int f, int a, double& b0, double& b1, double& b2) {
  b0 = 0.0;
  b1 = 0.0;
  b2 = 0.0;
#pragma unroll
  for (int k = 0; k < 5; ++k) {
    const double* rc = sm.rowc[5 * f + k];
    const double w = sel3(a, rc[0], rc[1], rc[2]) * rc[3];
    b0 += w * rc[0];
    b1 += w * rc[1];
    b2 += w * rc[2];
  }
}

// A~'v at the variable lanes of each foot group from the row lanes' mv = (main coefficient) v and
// zv = (fz coefficient) v, with DPP row shifts, in the reference's summation order:
//   fx: m0 + m1,  fy: m2 + m3,  fz: z0 + z1 + z2 + z3 + m4   (rows 0-4 of the foot).
// Must be called with every lane of the wave active.
__device__ __forceinline__ double gather_atv(double mv, double zv, int a, double init) {
  const double m3 = dpp<0x113>(mv), m4 = dpp<0x114>(mv), m5 = dpp<0x115>(mv);
  const double z4 = dpp<0x114>(zv), z5 = dpp<0x115>(zv), z6 = dpp<0x116>(zv), z7 = dpp<0x117>(zv);
  const double s1 = sel3(a, m5, m4, z7);
  const double s2 = sel3(a, m4, m3, z6);
  const double acc = (init + s1) + s2;
  const double accz = ((acc + z5) + z4) + m3;
  return a == 2 ? accz : acc;
}

// K = P~ + sigma I + blockdiag(A~' rho A~) from the tile holding P~, then K^-1 in place by block
// Gauss-Jordan with the 3x3 diagonal block P of foot kf as pivot.  With R = the raw pivot rows
// A_k. and W_i = A_ik P^-1 (W_k = I - P^-1 for the pivot rows themselves) every group applies
// the same update  A_i. <- A_i. - W_i R,  then the pivot columns are set to -W_i (P^-1 for the
// pivot rows):
//   A_kk <- P^-1,  A_kj <- P^-1 A_kj,  A_ik <- -A_ik P^-1,  A_ij <- A_ij - A_ik P^-1 A_kj.
// Pivot kf's columns 3kf..3kf+2 are tile columns 3s..3s+2 of lane L = kf / SPL (s = kf % SPL);
// unrolling s makes them static register positions.
template <int N>
__device__ __forceinline__ void factor_and_invert(double (&M)[3][Dim<N>::BC], Smem<N>& sm, double sigma) {
  using Dm = Dim<N>;
  constexpr int BC = Dm::BC, n = Dm::n, SPL = Dm::SPL, NP = Dm::NP;
  const int t = opaque(threadIdx.x);
  const int f = t >> 3, tc = t & 7;
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    const int r = 3 * f + i;
#pragma unroll
    for (int j = 0; j < BC; ++j) {
      const int c = tc * BC + j;
      double v = M[i][j];
      if (r == c && r < n) v += sigma;
      const int d = c - 3 * f;
      if (r < n && d >= 0 && d < 3) v += sm.BD[r][d];
      M[i][j] = v;
    }
  }
  for (int L = 0; L < (Dm::nf + SPL - 1) / SPL; ++L) {
#pragma unroll
    for (int s = 0; s < SPL; ++s) {
      const int kf = L * SPL + s;
      if (kf >= Dm::nf) break;
      const int b = kf & 1;
      const bool own = f == kf;  // this group owns the pivot rows
      const bool pl = tc == L;   // this lane holds the pivot columns
      double* __restrict__ Rb = &sm.u.g.r[b][0][tc * BC];
      // ---- phase A: publish every group's pivot-column block, the raw pivot rows and P^-1 ----
      if (pl) {
#pragma unroll
        for (int i = 0; i < 3; ++i)
#pragma unroll
          for (int q = 0; q < 3; ++q) sm.u.g.ck[b][f][3 * i + q] = M[i][3 * s + q];
      }
      if (own) {  // raw pivot rows, pivot columns zeroed (those are set explicitly below)
#pragma unroll
        for (int j = 0; j < BC; ++j)
#pragma unroll
          for (int i = 0; i < 3; ++i) Rb[i * NP + j] = (pl && j >= 3 * s && j < 3 * s + 3) ? 0.0 : M[i][j];
        if (pl) {
          const double P0 = M[0][3 * s], P1 = M[0][3 * s + 1], P2 = M[0][3 * s + 2];
          const double P3 = M[1][3 * s], P4 = M[1][3 * s + 1], P5 = M[1][3 * s + 2];
          const double P6 = M[2][3 * s], P7 = M[2][3 * s + 1], P8 = M[2][3 * s + 2];
          // cofactor inverse (Eigen's 3x3 formula)
          const double c00 = P4 * P8 - P5 * P7, c01 = P5 * P6 - P3 * P8, c02 = P3 * P7 - P4 * P6;
          const double c10 = P7 * P2 - P8 * P1, c11 = P8 * P0 - P6 * P2, c12 = P6 * P1 - P7 * P0;
          const double c20 = P1 * P5 - P2 * P4, c21 = P2 * P3 - P0 * P5, c22 = P0 * P4 - P1 * P3;
          const double invdet = 1.0 / ((c00 * P0 + c10 * P3) + c20 * P6);
          double* pv = sm.u.g.pinv[b];
          pv[0] = c00 * invdet; pv[1] = c10 * invdet; pv[2] = c20 * invdet;
          pv[3] = c01 * invdet; pv[4] = c11 * invdet; pv[5] = c21 * invdet;
          pv[6] = c02 * invdet; pv[7] = c12 * invdet; pv[8] = c22 * invdet;
        }
      }
      __syncthreads();
      // ---- phase B: A_i. -= W_i R for every group, then the pivot columns ----
      double Pv[9], W[9];
#pragma unroll
      for (int e = 0; e < 9; ++e) Pv[e] = sm.u.g.pinv[b][e];
#pragma unroll
      for (int i = 0; i < 3; ++i) {
        const double C0 = sm.u.g.ck[b][f][3 * i], C1 = sm.u.g.ck[b][f][3 * i + 1], C2 = sm.u.g.ck[b][f][3 * i + 2];
#pragma unroll
        for (int q = 0; q < 3; ++q) {
          const double w = (C0 * Pv[q] + C1 * Pv[3 + q]) + C2 * Pv[6 + q];
          W[3 * i + q] = own ? (i == q ? 1.0 : 0.0) - Pv[3 * i + q] : w;
        }
      }
#pragma unroll
      for (int i = 0; i < 3; ++i)
#pragma unroll
        for (int q = 0; q < 3; ++q) {
          const double v = own ? Pv[3 * i + q] : -W[3 * i + q];
          M[i][3 * s + q] = pl ? v : M[i][3 * s + q];
        }
#pragma unroll
      for (int j = 0; j < BC; ++j) {
        const double R0 = Rb[j], R1 = Rb[NP + j], R2 = Rb[2 * NP + j];
#pragma unroll
        for (int i = 0; i < 3; ++i)
          M[i][j] = fma(-W[3 * i + 2], R2, fma(-W[3 * i + 1], R1, fma(-W[3 * i], R0, M[i][j])));
      }
    }
  }
  __syncthreads();
}

// Phase timing (debug builds with -DMPCQP_PHASE_TIMING): thread 0 of each traced robot appends
// {phase id, s_memtime, s_memrealtime (100 MHz), 0} records to the trace buffer instead of
// termination-check records.
#ifdef MPCQP_PHASE_TIMING
#define PHASE_MARK(id)                                                                     \
  do {                                                                                     \
    if (trace && threadIdx.x == 0 && inst < trace_cap && nmark < MPCQP_TRACE_LEN) {        \
      double* tm_ = trace + ((size_t)inst * MPCQP_TRACE_LEN + nmark) * 4;                   \
      tm_[0] = (id);                                                                       \
      tm_[1] = (double)__builtin_readcyclecounter();                                       \
      tm_[2] = (double)__builtin_amdgcn_s_memrealtime();                                   \
      ++nmark;                                                                             \
    }                                                                                      \
  } while (0)
#else
#define PHASE_MARK(id) \
  do {                 \
  } while (0)
#endif

// Per-robot workspace (doubles): the scaled P~ (n x NP, re-read at every rho refactorization),
// then 12 doubles per thread where a lane parks its ADMM state while the block inverts.
template <int N>
struct WS {
  static constexpr size_t PARK = (size_t)Dim<N>::n * Dim<N>::NP;
  static constexpr size_t SIZE = PARK + (size_t)12 * Dim<N>::NT;
};

// ---- the solver kernel ---------------------------------------------------------------------
template <int N>
__global__ __launch_bounds__(Dim<N>::NT) void solve_kernel(
    const double* __restrict__ recs, int batch, mpcqp_result* __restrict__ results,
    double* __restrict__ solution, double* __restrict__ work, double* __restrict__ trace, int trace_cap,
    mpcqp_params p) {
  using Dm = Dim<N>;
  constexpr int NT = Dm::NT, BC = Dm::BC, n = Dm::n, nf = Dm::nf;
  __shared__ Smem<N> sm;
  const int inst = blockIdx.x;
  if (inst >= batch) return;
  const int t0 = threadIdx.x;
  double* __restrict__ Pw = work + (size_t)inst * WS<N>::SIZE;
  const double alpha = p.alpha, sigma = p.sigma;
  double M[3][BC];
  int rslot = 0;
#ifdef MPCQP_PHASE_TIMING
  int nmark = 0;
#endif
  PHASE_MARK(0);

  // ---- 0. record -> LDS, non-finite guard --------------------------------------------------
  {
    const double* rec_g = recs + (size_t)inst * Dm::rec;
    bool bad = false;
    for (int e = t0; e < Dm::rec; e += NT) {
      const double v = rec_g[e];
      sm.rec[e] = v;
      bad |= !isfinite(v);
    }
    if (__syncthreads_or(bad)) {
      if (t0 == 0) {
        mpcqp_result r;
        for (int k = 0; k < ND; ++k) { r.u0[k] = NAN; r.f_body[k] = 0.0; }
        r.obj_val = NAN; r.pri_res = NAN; r.dua_res = NAN; r.rho = p.rho;
        r.status = MPCQP_STATUS_NAN_INPUT; r.iters = 0; r.rho_updates = 0; r.nan_legs = 0xF;
        results[inst] = r;
      }
      if (solution)
        for (int e = t0; e < n; e += NT) solution[(size_t)inst * n + e] = NAN;
      return;
    }
  }

  // ---- 1. condensation -> workspace (unscaled H), sm.qt (gradient), sm.lo/hi ----------------
  PHASE_MARK(1);
  condense<N, NT>(sm, p, Pw, Dm::NP);
  PHASE_MARK(2);

  // Lane roles inside foot group f: lanes 0-4 own the foot's friction-pyramid rows r = 5f+tc,
  // lanes 5-7 its force variables c = 3f+a.  The two roles share the state registers below.
  const int f = t0 >> 3, tc = t0 & 7;
  const bool live = f < nf;
  const bool row_lane = live && tc < 5, var_lane = live && tc >= 5;
  const int r = 5 * f + tc;
  const int a = tc - 5;
  const int c = 3 * f + (a < 0 ? 0 : a);
  double s_a = 0.0, s_b = 0.0, s_c = 0.0, s_d = 0.0, s_e = 0.0, s_f = 0.0, s_g = 0.0, s_h = 0.0;
  double k0 = 0.0, k1 = 0.0, k2 = 0.0;  // row: A~ coefficients on (fx, fy, fz); var: A~'rho A~ row
  double &z = s_a, &x = s_a;            // z / x
  double &y = s_b, &px = s_b;           // y / P~x
  double &lo = s_c, &q = s_c;           // l~ / q~
  double &hi = s_d, &xr = s_d;          // u~ / current KKT right-hand side entry
  double &rho_r = s_e, &rinv = s_f;     // rho of the row and its inverse
  double &E = s_g, &D = s_g;            // Ruiz row / column scaling
  double &Ei = s_h, &Di = s_h;          // their inverses
  int ct = 0;                           // constraint type (set_rho_vec)

  // ---- 2. OSQP scale_data (Ruiz), P in registers ---------------------------------------------
  load_tile<N>(M, Pw, f, tc);
  for (int e = n + t0; e < Dm::NP; e += NT) sm.Dt[e] = 1.0;
  if (row_lane) {  // unscaled friction pyramid row (ConvexMpc.cpp:46-58)
    const double mu = sm.rec[MPCQP_REC_MU];
    const double am = 1.0, az = tc == 4 ? 0.0 : ((tc & 1) ? -mu : mu);
    k0 = tc < 2 ? am : 0.0;
    k1 = (tc == 2 || tc == 3) ? am : 0.0;
    k2 = tc < 4 ? az : am;
    E = 1.0;
    lo = sm.lo[r];
    hi = sm.hi[r];
  }
  if (var_lane) {
    D = 1.0;
    q = sm.qt[c];
  }
  double cost_c = 1.0;
  for (int pass = 0; pass < p.scaling; ++pass) {
    // D_temp: column inf-norm of [P; A] per variable (P symmetric: row norms of the tiles)
    double pm[3];
#pragma unroll
    for (int i = 0; i < 3; ++i) {
      double mx = 0.0;
#pragma unroll
      for (int j = 0; j < BC; ++j) mx = fmax(mx, dabs(M[i][j]));
      pm[i] = g8_max(mx);
    }
    const double ca0 = g8_max(row_lane ? dabs(k0) : 0.0);
    const double ca1 = g8_max(row_lane ? dabs(k1) : 0.0);
    const double ca2 = g8_max(row_lane ? dabs(k2) : 0.0);
    if (var_lane) {
      const double pc = sel3(a, pm[0], pm[1], pm[2]);
      const double cav = sel3(a, ca0, ca1, ca2);
      sm.Dt[c] = 1.0 / sqrt(limit_scaling(dmax(pc, cav)));
    }
    double et = 1.0;
    if (row_lane) et = 1.0 / sqrt(limit_scaling(dmax(dmax(dabs(k0), dabs(k1)), dabs(k2))));
    __syncthreads();
    // P <- D P D (premultiply by the row of the upper-triangle entry, then its column)
    double drow[3];
#pragma unroll
    for (int i = 0; i < 3; ++i) drow[i] = sm.Dt[3 * f + i];
#pragma unroll
    for (int j = 0; j < BC; ++j) {
      const int cc = tc * BC + j;
      if (cc < n) {
        const double dc = sm.Dt[cc];
#pragma unroll
        for (int i = 0; i < 3; ++i) {
          const int rr = 3 * f + i;
          M[i][j] = rr <= cc ? (M[i][j] * drow[i]) * dc : (M[i][j] * dc) * drow[i];
        }
      }
    }
    if (row_lane) {  // A <- E A D
      k0 = (k0 * et) * drow[0];
      k1 = (k1 * et) * drow[1];
      k2 = (k2 * et) * drow[2];
      E *= et;
    }
    if (var_lane) {
      const double dt = sel3(a, drow[0], drow[1], drow[2]);
      q = dt * q;
      D = D * dt;
    }
    // cost normalization: mean column norm of P and inf-norm of q
#pragma unroll
    for (int i = 0; i < 3; ++i) {
      double mx = 0.0;
#pragma unroll
      for (int j = 0; j < BC; ++j) mx = fmax(mx, dabs(M[i][j]));
      pm[i] = g8_max(mx);
    }
    double sv = var_lane ? sel3(a, pm[0], pm[1], pm[2]) : 0.0;
    double qv = var_lane ? dabs(q) : 0.0;
    wg_sum_max<N>(sm, sv, qv, rslot);
    double c_temp = sv / n;
    const double inf_norm_q = limit_scaling(qv);
    c_temp = dmax(c_temp, inf_norm_q);
    c_temp = limit_scaling(c_temp);
    c_temp = 1. / c_temp;
#pragma unroll
    for (int i = 0; i < 3; ++i)
#pragma unroll
      for (int j = 0; j < BC; ++j) M[i][j] *= c_temp;
    if (var_lane) q *= c_temp;
    cost_c *= c_temp;
  }
  if (var_lane) Di = 1. / D;
  if (row_lane) {
    Ei = 1. / E;
    lo = E * lo;
    hi = E * hi;
  }
  PHASE_MARK(3);
  store_tile<N>(M, Pw, f, tc);  // scaled P~ kept for rho refactorizations
  // Uniform doubles used only at termination checks live in LDS, not in registers across the
  // loop: cst = {cost scaling c, rho, pri_res, dua_res}.
  if (t0 == 0) {
    sm.cst[0] = cost_c;
    sm.cst[1] = dmin(dmax(p.rho, RHO_MIN), RHO_MAX);
    sm.cst[2] = 0.0;
    sm.cst[3] = 0.0;
  }
  const double rho0 = dmin(dmax(p.rho, RHO_MIN), RHO_MAX);
  if (row_lane) {  // set_rho_vec (auxil.c)
    if (lo < -OSQP_INF * MIN_SCALING && hi > OSQP_INF * MIN_SCALING)
      ct = -1;
    else if (hi - lo < RHO_TOL)
      ct = 1;
    else
      ct = 0;
    rho_r = ct == -1 ? RHO_MIN : ct == 1 ? RHO_EQ_OVER_RHO_INEQ * rho0 : rho0;
    rinv = 1. / rho_r;
    sm.rowc[r][0] = k0;
    sm.rowc[r][1] = k1;
    sm.rowc[r][2] = k2;
    sm.rowc[r][3] = rho_r;
    z = 0.0;
    y = 0.0;
  }
  wave_sync();
  if (var_lane) {
    bd_row<N>(sm, f, a, k0, k1, k2);
    sm.BD[c][0] = k0;
    sm.BD[c][1] = k1;
    sm.BD[c][2] = k2;
    x = 0.0;
    px = 0.0;
  }

  // Cold per-lane values (Ruiz factors and their inverses, constraint type) are parked in the
  // workspace for the whole solve; only the termination checks and the epilogue read them.
  double* __restrict__ const park0 = Pw + WS<N>::PARK + (size_t)t0 * 12;
  park0[6] = s_g;
  park0[7] = s_h;
  park0[11] = ct;

  // ---- 3. ADMM -------------------------------------------------------------------------------
  int status = MPCQP_STATUS_UNSOLVED, iters = 0, rho_updates = 0, ntrace = 0;
  // iteration-1 right-hand side from the cold start (x = z = y = 0)
  for (int e = n + t0; e < Dm::NP; e += NT) sm.rhs[0][e] = sm.rhs[1][e] = 0.0;  // padding
  if (var_lane) {
    xr = sigma * 0.0 - q;
    sm.rhs[1][c] = xr;  // read by iteration 1
  }
  __syncthreads();
  bool need_factor = true;  // K^-1 is (re)built at the top of the iteration that needs it
  int to_check = p.check_termination, to_adapt = p.adaptive_rho_interval;  // iter % k countdowns
  for (int iter = 1; iter <= p.max_iter; ++iter) {
    const int t = opaque(threadIdx.x);
    const int f = t >> 3, tc = t & 7;
    const bool live = f < nf;
    const bool row_lane = live && tc < 5, var_lane = live && tc >= 5;
    const int a = tc - 5, c = 3 * f + (a < 0 ? 0 : a);
    const int gb = t & ~7;
    if (need_factor) {  // single inlined site: initial factorization and osqp_update_rho refactors
      // park the lane's ADMM state in the workspace so the inversion has the register file
      double* __restrict__ park = Pw + WS<N>::PARK + (size_t)t * 12;
      park[0] = s_a; park[1] = s_b; park[2] = s_c; park[3] = s_d; park[4] = s_e; park[5] = s_f;
      park[8] = k0; park[9] = k1; park[10] = k2;
      asm volatile("" ::: "memory");
      PHASE_MARK(10);
      if (iter > 1) load_tile<N>(M, Pw, f, tc);
      PHASE_MARK(11);
      factor_and_invert<N>(M, sm, sigma);
      PHASE_MARK(12);
      asm volatile("" ::: "memory");
      s_a = park[0]; s_b = park[1]; s_c = park[2]; s_d = park[3]; s_e = park[4]; s_f = park[5];
      k0 = park[8]; k1 = park[9]; k2 = park[10];
      need_factor = false;
    }
    // (b) x~ = K^-1 rhs: register-tile mat-vec, all-reduced inside the foot's 8-lane group
    double xt0, xt1, xt2;
    {
      const double* rb = sm.rhs[iter & 1] + tc * BC;
      double e0 = 0.0, e1 = 0.0, e2 = 0.0, o0 = 0.0, o1 = 0.0, o2 = 0.0;
#pragma unroll
      for (int j = 0; j < BC; j += 2) {
        const double v = rb[j];
        e0 = fma(M[0][j], v, e0);
        e1 = fma(M[1][j], v, e1);
        e2 = fma(M[2][j], v, e2);
        if (j + 1 < BC) {
          const double w = rb[j + 1];
          o0 = fma(M[0][j + 1], w, o0);
          o1 = fma(M[1][j + 1], w, o1);
          o2 = fma(M[2][j + 1], w, o2);
        }
      }
      xt0 = g8_sum(e0 + o0);
      xt1 = g8_sum(e1 + o1);
      xt2 = g8_sum(e2 + o2);
    }
    bool is_check = false, is_adapt = false;
    if (p.check_termination && --to_check == 0) {
      is_check = true;
      to_check = p.check_termination;
    }
    if (p.adaptive_rho && --to_adapt == 0) {
      is_adapt = true;
      to_adapt = p.adaptive_rho_interval;
    }
    const bool last = iter == p.max_iter;
    const bool need_info = is_check || is_adapt || last;
    // (c) update_z / update_y on row lanes, update_x (+ P~x via the KKT identity
    //     P~x~ = rhs - sigma x~ - A~'rho A~ x~) on variable lanes
    const double kd = (k0 * xt0 + k1 * xt1) + k2 * xt2;  // row: (A~x~)_r; var: (A~'rho A~ x~)_c
    const double km = tc < 2 ? k0 : tc < 4 ? k1 : k2;    // row: coefficient on its main force
    const double kz = tc < 4 ? k2 : 0.0;                 // row: coefficient on fz (rows 0-3)
    double dyv = 0.0, dxv = 0.0, pxo = 0.0;
    if (row_lane) {
      const double zr = alpha * kd + (1.0 - alpha) * z;
      const double zn = dmin(dmax(zr + rinv * y, lo), hi);
      dyv = rho_r * (zr - zn);
      y = y + dyv;
      z = zn;
    }
    if (var_lane) {
      const double xa = sel3(a, xt0, xt1, xt2);
      const double xn = alpha * xa + (1.0 - alpha) * x;
      dxv = xn - x;
      const double pxt = xr - sigma * xa - kd;
      pxo = px;
      px = alpha * pxt + (1.0 - alpha) * px;
      x = xn;
    }

    if (need_info) {
      // ---- update_info / check_termination / adapt_rho (osqp.c, auxil.c) ----
      const double* __restrict__ parkc = Pw + WS<N>::PARK + (size_t)t * 12;
      const double E = parkc[6], Ei = parkc[7];  // row lanes: E, 1/E; variable lanes: D, 1/D
      const double &D = E, &Di = Ei;
      // row lanes need the new x of their foot, variable lanes A~'y of the new y
      const double x0n = __shfl(x, gb + 5), x1n = __shfl(x, gb + 6), x2n = __shfl(x, gb + 7);
      const double ax = row_lane ? (k0 * x0n + k1 * x1n) + k2 * x2n : 0.0;
      const double atyg = gather_atv(row_lane ? km * y : 0.0, row_lane ? kz * y : 0.0, a, 0.0);
      const double aty = var_lane ? atyg : 0.0;
      double pr = 0.0, d = 0.0;
      if (row_lane) pr = ax + (-1.0) * z;
      if (var_lane) d = (q + 1.0 * px) + 1.0 * aty;
      // the 14 norms of update_info / compute_pri_tol / compute_dua_tol / compute_rho_estimate,
      // reduced one at a time straight into LDS (keeps register pressure flat)
      {
        const int lane = t & 63, wave = t >> 6;
        auto put = [&](int k, double v) {
          v = wave_max(v);
          if (lane == 0) sm.info[wave][k] = v;
          __builtin_amdgcn_sched_barrier(0);
        };
        put(0, row_lane ? dabs(Ei * pr) : 0.0);
        put(1, row_lane ? dabs(pr) : 0.0);
        put(2, row_lane ? dabs(Ei * z) : 0.0);
        put(3, row_lane ? dabs(z) : 0.0);
        put(4, row_lane ? dabs(Ei * ax) : 0.0);
        put(5, row_lane ? dabs(ax) : 0.0);
        put(6, var_lane ? dabs(Di * d) : 0.0);
        put(7, var_lane ? dabs(d) : 0.0);
        put(8, var_lane ? dabs(Di * q) : 0.0);
        put(9, var_lane ? dabs(q) : 0.0);
        put(10, var_lane ? dabs(Di * aty) : 0.0);
        put(11, var_lane ? dabs(aty) : 0.0);
        put(12, var_lane ? dabs(Di * px) : 0.0);
        put(13, var_lane ? dabs(px) : 0.0);
      }
      __syncthreads();
      // workgroup maxima read from LDS where they are used (not held across the check)
      auto mx = [&](int k) {
        double v = sm.info[0][k];
        for (int w = 1; w < Dm::NW; ++w) v = dmax(v, sm.info[w][k]);
        return v;
      };
      const double cost_c = sm.cst[0], cinv = 1. / cost_c;
      double rho = sm.cst[1];
      const double pri_res = mx(0);
      const double dua_res = cinv * mx(6);
      iters = iter;
      // check_termination (osqp.c): approx=1 is the post-loop check at max_iter (eps x 10)
      auto check = [&](bool approx) -> int {
        double eps_abs = p.eps_abs, eps_rel = p.eps_rel, eps_pinf = p.eps_prim_inf, eps_dinf = p.eps_dual_inf;
        if (pri_res > OSQP_INF || dua_res > OSQP_INF) return MPCQP_STATUS_NON_CVX;
        if (approx) { eps_abs *= 10; eps_rel *= 10; eps_pinf *= 10; eps_dinf *= 10; }
        const double eps_prim = eps_abs + eps_rel * dmax(mx(2), mx(4));
        const bool prim_ok = pri_res < eps_prim;
        bool prim_inf = false, dual_inf = false;
        if (!prim_ok) {
          // is_primal_infeasible: project delta_y onto the polar of the recession cone (in place)
          if (row_lane) {
            if (hi > OSQP_INF * MIN_SCALING) {
              if (lo < -OSQP_INF * MIN_SCALING) dyv = 0.0;
              else dyv = dmin(dyv, 0.0);
            } else if (lo < -OSQP_INF * MIN_SCALING) {
              dyv = dmax(dyv, 0.0);
            }
          }
          double nd[1] = {row_lane ? dabs(E * dyv) : 0.0};
          wg_reduce<N, 1, true>(sm, nd, rslot);
          const double ndy = nd[0];
          if (ndy > DIV_TOL) {
            double lh[1] = {row_lane ? hi * dmax(dyv, 0.0) + lo * dmin(dyv, 0.0) : 0.0};
            wg_reduce<N, 1, false>(sm, lh, rslot);
            if (lh[0] < eps_pinf * ndy) {
              const double atd = gather_atv(row_lane ? km * dyv : 0.0, row_lane ? kz * dyv : 0.0, a, 0.0);
              double an[1] = {var_lane ? dabs(Di * atd) : 0.0};
              wg_reduce<N, 1, true>(sm, an, rslot);
              prim_inf = an[0] < eps_pinf * ndy;
            }
          }
        }
        const double eps_dual = eps_abs + eps_rel * (cinv * dmax(dmax(mx(8), mx(10)), mx(12)));
        const bool dual_ok = dua_res < eps_dual;
        if (!dual_ok) {
          // is_dual_infeasible (P~ delta_x = P~x_new - P~x_old)
          double nx[1] = {var_lane ? dabs(D * dxv) : 0.0};
          wg_reduce<N, 1, true>(sm, nx, rslot);
          const double ndx = nx[0];
          if (ndx > DIV_TOL) {
            double qd[1] = {var_lane ? q * dxv : 0.0};
            wg_reduce<N, 1, false>(sm, qd, rslot);
            if (qd[0] < cost_c * eps_dinf * ndx) {
              double pd[1] = {var_lane ? dabs(Di * (px - pxo)) : 0.0};
              wg_reduce<N, 1, true>(sm, pd, rslot);
              if (pd[0] < cost_c * eps_dinf * ndx) {
                const double dx0 = __shfl(dxv, gb + 5), dx1 = __shfl(dxv, gb + 6), dx2 = __shfl(dxv, gb + 7);
                double viol = 0.0;
                if (row_lane) {
                  const double v = Ei * ((k0 * dx0 + k1 * dx1) + k2 * dx2);
                  if ((hi < OSQP_INF * MIN_SCALING && v > eps_dinf * ndx) ||
                      (lo > -OSQP_INF * MIN_SCALING && v < -eps_dinf * ndx))
                    viol = 1.0;
                }
                double vv[1] = {viol};
                wg_reduce<N, 1, true>(sm, vv, rslot);
                dual_inf = vv[0] == 0.0;
              }
            }
          }
        }
        if (prim_ok && dual_ok) return approx ? MPCQP_STATUS_SOLVED_INACCURATE : MPCQP_STATUS_SOLVED;
        if (prim_inf) return approx ? MPCQP_STATUS_PRIMAL_INFEASIBLE_INACCURATE : MPCQP_STATUS_PRIMAL_INFEASIBLE;
        if (dual_inf) return approx ? MPCQP_STATUS_DUAL_INFEASIBLE_INACCURATE : MPCQP_STATUS_DUAL_INFEASIBLE;
        return MPCQP_STATUS_UNSOLVED;
      };
      int st = MPCQP_STATUS_UNSOLVED;
      bool done = false, refactor = false;
      for (int pass = 0; pass < 2 && !done; ++pass) {
        // pass 0: in-loop check_termination; pass 1: osqp_solve's approximate check at max_iter
        if (pass == 1 && !last) break;
        if (pass == 1 || is_check || last) {
          st = check(pass == 1);
          done = st != MPCQP_STATUS_UNSOLVED;
        }
        if (pass == 1 || done || !is_adapt) continue;
        // adapt_rho / compute_rho_estimate (scaled residuals and norms); runs before the
        // post-loop approximate check of osqp_solve
        const double pr_n = mx(1) / (dmax(mx(3), mx(5)) + DIV_TOL);
        const double du_n = mx(7) / (dmax(dmax(mx(9), mx(11)), mx(13)) + DIV_TOL);
        double est = rho * sqrt(pr_n / (du_n + DIV_TOL));
        est = dmin(dmax(est, RHO_MIN), RHO_MAX);
        if (est > rho * p.adaptive_rho_tolerance || est < rho / p.adaptive_rho_tolerance) {
          rho = dmin(dmax(est, RHO_MIN), RHO_MAX);
          rho_updates += 1;
          refactor = !last;
        }
      }
      if (last && st == MPCQP_STATUS_UNSOLVED) st = MPCQP_STATUS_MAX_ITER_REACHED;
      if (last) done = true;
      status = st;
#ifdef MPCQP_PHASE_TIMING
      if (is_check) PHASE_MARK(30);
#else
      if (trace && t == 0 && inst < trace_cap && ntrace < MPCQP_TRACE_LEN && is_check) {
        double* tp = trace + ((size_t)inst * MPCQP_TRACE_LEN + ntrace) * 4;
        tp[0] = iter; tp[1] = pri_res; tp[2] = dua_res; tp[3] = rho;
      }
#endif
      ntrace += is_check ? 1 : 0;
      if (t == 0) {  // every thread holds the same values; the reads above precede a barrier
        sm.cst[1] = rho;
        sm.cst[2] = pri_res;
        sm.cst[3] = dua_res;
      }
      if (done) break;
      if (refactor) {
        // osqp_update_rho: new rho vector and A~'rho A~ blocks now; P~ reload + re-inversion at
        // the top of the next iteration
        if (row_lane) {
          const int ct = (int)parkc[11];
          rho_r = ct == -1 ? rho_r : ct == 1 ? RHO_EQ_OVER_RHO_INEQ * rho : rho;
          rinv = 1. / rho_r;
          sm.rowc[5 * f + tc][3] = rho_r;
        }
        wave_sync();
        if (var_lane) {
          bd_row<N>(sm, f, a, k0, k1, k2);
          sm.BD[c][0] = k0;
          sm.BD[c][1] = k1;
          sm.BD[c][2] = k2;
        }
        need_factor = true;
      }
    }
    // (a) next right-hand side: rhs = sigma x - q~ + A~'(rho z - y)  [compute_rhs + KKT rhs]
    {
      double mv = 0.0, zv = 0.0, init = 0.0;
      if (row_lane) {
        const double tv = rho_r * z - y;
        mv = km * tv;
        zv = kz * tv;
      }
      if (var_lane) init = sigma * x - q;
      const double rr = gather_atv(mv, zv, a, init);
      if (var_lane) {
        xr = rr;
        sm.rhs[(iter + 1) & 1][c] = xr;  // other buffer: slower waves may still read this one
      }
    }
    __syncthreads();
  }

  PHASE_MARK(20);
  // ---- 4. store_solution + unscale + compute_grf extraction (A1RobotControl.cpp:555-561) ------
  __syncthreads();
  const double cinv = 1. / sm.cst[0], rho = sm.cst[1], pri_res = sm.cst[2], dua_res = sm.cst[3];
  const bool has_sol = status != MPCQP_STATUS_PRIMAL_INFEASIBLE &&
                       status != MPCQP_STATUS_PRIMAL_INFEASIBLE_INACCURATE &&
                       status != MPCQP_STATUS_DUAL_INFEASIBLE &&
                       status != MPCQP_STATUS_DUAL_INFEASIBLE_INACCURATE && status != MPCQP_STATUS_NON_CVX;
  {
    // objective 1/2 x'P~x + q~'x (unscaled by cinv)
    double ob[1] = {var_lane ? 0.5 * x * px + q * x : 0.0};
    wg_reduce<N, 1, false>(sm, ob, rslot);
    const double xs = has_sol ? park0[6] * x : NAN;  // D x
    if (solution && var_lane) solution[(size_t)inst * n + c] = xs;
    if (f < 4) {  // horizon step 0 = feet 0..3 = legs FL, FR, RL, RR
      mpcqp_result* res = results + inst;
      const int gb = t0 & ~7;
      const double u0 = __shfl(xs, gb + 5), u1 = __shfl(xs, gb + 6), u2 = __shfl(xs, gb + 7);
      const double nrm = sqrt(u0 * u0 + u1 * u1 + u2 * u2);
      const bool nanleg = isnan(nrm);
      if (var_lane) {
        const double* R = sm.rec + MPCQP_REC_ROT;
        double s = 0.0;
        s += R[0 * 3 + a] * u0;
        s += R[1 * 3 + a] * u1;
        s += R[2 * 3 + a] * u2;
        res->u0[3 * f + a] = xs;
        res->f_body[3 * f + a] = nanleg ? 0.0 : s;
      }
      const unsigned long long nb = __ballot(nanleg && tc == 0);
      if (t0 == 0) {
        int legs = 0;
        for (int l = 0; l < 4; ++l) legs |= ((nb >> (8 * l)) & 1ull) ? (1 << l) : 0;
        res->nan_legs = legs;
        double obj;
        if (has_sol) obj = ob[0] * cinv;
        else if (status == MPCQP_STATUS_PRIMAL_INFEASIBLE || status == MPCQP_STATUS_PRIMAL_INFEASIBLE_INACCURATE) obj = OSQP_INF;
        else if (status == MPCQP_STATUS_DUAL_INFEASIBLE || status == MPCQP_STATUS_DUAL_INFEASIBLE_INACCURATE) obj = -OSQP_INF;
        else obj = NAN;
        res->obj_val = obj;
        res->pri_res = pri_res;
        res->dua_res = dua_res;
        res->rho = rho;
        res->status = status;
        res->iters = iters;
        res->rho_updates = rho_updates;
      }
    }
  }
}

// ---- launch table --------------------------------------------------------------------------
template <int N>
static hipError_t launch_solve(const LaunchArgs& a) {
  hipLaunchKernelGGL((solve_kernel<N>), dim3(a.grid), dim3(Dim<N>::NT), 0, (hipStream_t)a.stream, a.recs,
                     a.batch, a.results, a.solution, a.work, a.trace, a.trace_cap, a.p);
  return hipGetLastError();
}
template <int N>
static hipError_t occupancy(int* blocks) {
  return hipOccupancyMaxActiveBlocksPerMultiprocessor(blocks, solve_kernel<N>, Dim<N>::NT, 0);
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
hipError_t occupancy_any(int horizon, int* blocks) {
  switch (horizon) {
#define CASE(K) \
  case K: return occupancy<K>(blocks);
    MPCQP_FOR_EACH_N(CASE)
#undef CASE
    default: return hipErrorInvalidValue;
  }
}
int solve_threads(int horizon) { return ((8 * 4 * horizon + 63) / 64) * 64; }
size_t workspace_doubles(int horizon) {  // WS<N>::SIZE
  const int n = 12 * horizon;
  return (size_t)n * 8 * 3 * ((n + 23) / 24) + (size_t)12 * solve_threads(horizon);
}

}  // namespace mpcqp
