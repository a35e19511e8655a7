// mpcqp_riccati.hip — the OSQP 0.6 ADMM of solve_kernel with the KKT solve done through the
// problem's state-space structure instead of an explicit inverse; used for horizons 11..20
// (config C4, N = 20: K^-1 would be 460 KiB of binary64, more than a CU's registers).
//
// OSQP scales P = c D H D and A~ = E A D (scaling.c), so the reduced KKT matrix factors as
//   K = P~ + sigma I + A~' diag(rho) A~ = D (c B'Q̄B + R~) D,
//   R~ = c R + D^-1 (sigma I + A~' diag(rho) A~) D^-1        (3x3 block-diagonal per foot),
// where H = B'Q̄B + R is ConvexMpc's condensed Hessian (B = B_qp, Q̄ = blockdiag(Q),
// ConvexMpc.cpp:184-211).  (c B'Q̄B + R~) u = w is the normal equation of the LQR problem
//   min 1/2 sum_{k=1..N} x_k' cQ x_k + 1/2 sum_k u_k' R~_k u_k - w'u,  x_{k+1} = A_d x_k + B_d(k) u_k,
// x_0 = 0, solved by a backward Riccati recursion (factorization, O(N S^3), once per rho) and a
// backward/forward sweep per ADMM iteration (O(N S^2)).
//
// One workgroup (4 waves) per robot: setup, Ruiz and the factorization use every thread; each
// iteration's sweeps run in wave 0 (4 lanes per output row, DPP quad reductions, no barriers);
// the per-foot ADMM updates run one thread per foot.  Arithmetic is binary64.
#include "mpcqp_device.h"

namespace mpcqp {
namespace ric {

constexpr int NT = 256;
constexpr int NWV = NT / 64;

template <int N>
struct RSmem {
  using Dm = Dim<N>;
  static constexpr int n = Dm::n, m = Dm::m, nf = Dm::nf;
  double rec[Dm::rec];
  double lo[m], hi[m];  // condensation output, then l~, u~
  double qt[n];         // condensation output (gradient)
  // constraint rows
  double ak[m][3];      // A~ row: coefficients on the foot's (fx, fy, fz)
  double rho_v[m], rho_inv[m], E[m], z[m], y[m], dy[m];
  int ctype[m];
  // variables
  double D[n], q[n], x[n], px[n], rhs[n], BD[n][3], w[n], uo[n];  // w: solve input, uo: output
  double Dt[n], colmax[n];  // Ruiz scratch; during ADMM: delta x and the previous P~x
  // dynamics (A_d dense; B_d(k): rows 6-8 per step, rows 9-11 = dt/m I per leg)
  double Ad[SD * SD];
  double Bw[N][3][ND];
  double gk[N][ND];
  double sv[2][16], xv[2][16], tv[16], vv[16];
  double red[2][NWV][16];
  double info[NWV][16];
  double cst[8];  // 0 c, 1 rho, 2 pri_res, 3 dua_res, 4 dt/m
  union U {
    CondScratch<N> c;
    struct F {
      double Gi[N][ND][ND];
      double K[N][ND][SD];
      double PB[N][SD][ND];
      double P[SD][SD];
      double PA[SD][SD];
      double G[ND][ND];
      double Fm[ND][SD];
    } f;
  } u;
};

// workgroup all-reduce (sum or max) of one value
template <class SM, bool MAX>
__device__ __forceinline__ double wg_red1(SM& sm, double v, int& slot) {
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  v = MAX ? wave_max(v) : wave_sum(v);
  if (lane == 0) sm.red[slot][wave][0] = v;
  __syncthreads();
  double r = sm.red[slot][0][0];
  for (int w = 1; w < NWV; ++w) r = MAX ? dmax(r, sm.red[slot][w][0]) : r + sm.red[slot][w][0];
  slot ^= 1;
  return r;
}

// 4-lane (quad) all-reduce sum
__device__ __forceinline__ double q4_sum(double v) {
  v = v + dpp<0x4E>(v);
  v = v + dpp<0xB1>(v);
  return v;
}

// (A~' diag(rho) A~) row of variable c = 3f + a (3x3 block per foot)
template <int N>
__device__ __forceinline__ void bd_var(RSmem<N>& sm, int c) {
  const int f = c / 3, a = c % 3;
  double b0 = 0.0, b1 = 0.0, b2 = 0.0;
  for (int k = 0; k < 5; ++k) {
    const int r = 5 * f + k;
    const double wgt = sel3(a, sm.ak[r][0], sm.ak[r][1], sm.ak[r][2]) * sm.rho_v[r];
    b0 += wgt * sm.ak[r][0];
    b1 += wgt * sm.ak[r][1];
    b2 += wgt * sm.ak[r][2];
  }
  sm.BD[c][0] = b0;
  sm.BD[c][1] = b1;
  sm.BD[c][2] = b2;
}

// Riccati factorization of c B'Q̄B + R~ (cost-to-go P_N = cQ, backward over the horizon):
//   PB = P_{k+1} B_k, G = R~_k + B_k' PB, PA = P_{k+1} A, F = B_k' PA, K_k = G^-1 F,
//   P_k = cQ + A' PA - F' K_k.   Stores G^-1, K_k, PB per step.
template <int N>
__device__ void factorize(RSmem<N>& sm, const mpcqp_params& p, double sigma) {
  auto& F = sm.u.f;
  const int t = threadIdx.x;
  const double c = sm.cst[0], dtm = sm.cst[4];
  for (int e = t; e < SD * SD; e += NT) {
    const int i = e / SD, j = e % SD;
    F.P[i][j] = (i == j) ? c * (2.0 * p.q_weights[i]) : 0.0;
  }
  __syncthreads();
  for (int k = N - 1; k >= 0; --k) {
    // PB (13x12) and PA (13x13)
    for (int e = t; e < SD * ND + SD * SD; e += NT) {
      if (e < SD * ND) {
        const int r = e / ND, j = e % ND;
        double s = 0.0;
        s += F.P[r][6] * sm.Bw[k][0][j];
        s += F.P[r][7] * sm.Bw[k][1][j];
        s += F.P[r][8] * sm.Bw[k][2][j];
        s += F.P[r][9 + j % 3] * dtm;
        F.PB[k][r][j] = s;
      } else {
        const int e2 = e - SD * ND, r = e2 / SD, s2 = e2 % SD;
        double s = 0.0;
        for (int q = 0; q < SD; ++q) s += F.P[r][q] * sm.Ad[q * SD + s2];
        F.PA[r][s2] = s;
      }
    }
    __syncthreads();
    // G = R~_k + B' PB (12x12), F = B' PA (12x13)
    for (int e = t; e < ND * ND + ND * SD; e += NT) {
      if (e < ND * ND) {
        const int i = e / ND, j = e % ND;
        double s = 0.0;
        s += sm.Bw[k][0][i] * F.PB[k][6][j];
        s += sm.Bw[k][1][i] * F.PB[k][7][j];
        s += sm.Bw[k][2][i] * F.PB[k][8][j];
        s += dtm * F.PB[k][9 + i % 3][j];
        // R~ block of foot (4k + i/3): c R + D^-1 (sigma I + BD) D^-1
        double rt = 0.0;
        if (i / 3 == j / 3) {
          const int ci = ND * k + i, cj = ND * k + j;
          const double inner = (i == j ? sigma : 0.0) + sm.BD[ci][j % 3];
          rt = (i == j ? c * (2.0 * p.r_weights[i]) : 0.0) + (1.0 / sm.D[ci]) * inner * (1.0 / sm.D[cj]);
        }
        F.G[i][j] = rt + s;
      } else {
        const int e2 = e - ND * ND, i = e2 / SD, s2 = e2 % SD;
        double s = 0.0;
        s += sm.Bw[k][0][i] * F.PA[6][s2];
        s += sm.Bw[k][1][i] * F.PA[7][s2];
        s += sm.Bw[k][2][i] * F.PA[8][s2];
        s += dtm * F.PA[9 + i % 3][s2];
        F.Fm[i][s2] = s;
      }
    }
    __syncthreads();
    // G^-1 by Gauss-Jordan (SPD, no pivoting) in wave 0: lane owns columns lane % 12 of rows
    if (t < 64) {
      double* G = &F.G[0][0];
      for (int piv = 0; piv < ND; ++piv) {
        const double dinv = 1.0 / G[piv * ND + piv];
        // new pivot row / column and the rank-1 update (144 entries over 64 lanes: e = t, t+64, t+128)
        auto gj = [&](int e) __attribute__((always_inline)) {
          const int i = e / ND, j = e % ND;
          if (i == piv && j == piv) return dinv;
          if (i == piv) return G[piv * ND + j] * dinv;
          if (j == piv) return -G[i * ND + piv] * dinv;
          return G[i * ND + j] - G[i * ND + piv] * (G[piv * ND + j] * dinv);
        };
        const double u0 = gj(t), u1 = gj(t + 64);
        const double u2 = t + 128 < ND * ND ? gj(t + 128) : 0.0;
        wave_sync();
        G[t] = u0;
        G[t + 64] = u1;
        if (t + 128 < ND * ND) G[t + 128] = u2;
        wave_sync();
      }
      for (int e = t; e < ND * ND; e += 64) F.Gi[k][e / ND][e % ND] = G[e];
    }
    __syncthreads();
    // K_k = G^-1 F (12x13)
    for (int e = t; e < ND * SD; e += NT) {
      const int i = e / SD, s2 = e % SD;
      double s = 0.0;
      for (int j = 0; j < ND; ++j) s += F.Gi[k][i][j] * F.Fm[j][s2];
      F.K[k][i][s2] = s;
    }
    __syncthreads();
    // P_k = cQ + A' PA - F' K_k (only needed while k >= 1)
    if (k >= 1) {
      for (int e = t; e < SD * SD; e += NT) {
        const int r = e / SD, s2 = e % SD;
        double a = 0.0;
        for (int q = 0; q < SD; ++q) a += sm.Ad[q * SD + r] * F.PA[q][s2];
        double b = 0.0;
        for (int i = 0; i < ND; ++i) b += F.Fm[i][r] * F.K[k][i][s2];
        F.P[r][s2] = ((r == s2) ? c * (2.0 * p.q_weights[r]) : 0.0) + a - b;
      }
      __syncthreads();
    }
  }
}

// One sweep pair: sm.u = (c B'Q̄B + R~)^-1 sm.w, in wave 0 (lanes 4r + pp: output row r, part pp).
template <int N>
__device__ void riccati_solve(RSmem<N>& sm) {
  auto& F = sm.u.f;
  const int lane = threadIdx.x & 63, r = lane >> 2, pp = lane & 3;
  const double dtm = sm.cst[4];
  int sb = 0;
  if (lane < 16) sm.sv[0][lane] = 0.0;
  wave_sync();
  for (int k = N - 1; k >= 0; --k) {
    const double* s = sm.sv[sb];
    // t = w_k - B_k' s
    if (lane < ND) {
      const double bs = ((sm.Bw[k][0][lane] * s[6] + sm.Bw[k][1][lane] * s[7]) + sm.Bw[k][2][lane] * s[8]) +
                        dtm * s[9 + lane % 3];
      sm.tv[lane] = sm.w[ND * k + lane] - bs;
    }
    wave_sync();
    // g_k = G^-1 t
    {
      double acc = 0.0;
      if (r < ND)
        for (int j = pp; j < ND; j += 4) acc += F.Gi[k][r][j] * sm.tv[j];
      acc = q4_sum(acc);
      if (r < ND && pp == 0) sm.gk[k][r] = acc;
    }
    wave_sync();
    if (k >= 1) {
      // v = PB_k g + s
      {
        double acc = 0.0;
        if (r < SD)
          for (int j = pp; j < ND; j += 4) acc += F.PB[k][r][j] * sm.gk[k][j];
        acc = q4_sum(acc);
        if (r < SD && pp == 0) sm.vv[r] = acc + s[r];
      }
      wave_sync();
      // s_k = A' v
      {
        double acc = 0.0;
        if (r < SD)
          for (int q = pp; q < SD; q += 4) acc += sm.Ad[q * SD + r] * sm.vv[q];
        acc = q4_sum(acc);
        if (r < SD && pp == 0) sm.sv[sb ^ 1][r] = acc;
      }
      sb ^= 1;
      wave_sync();
    }
  }
  int xb = 0;
  if (lane < 16) sm.xv[0][lane] = 0.0;
  wave_sync();
  for (int k = 0; k < N; ++k) {
    const double* xc = sm.xv[xb];
    // u_k = g_k - K_k x
    {
      double acc = 0.0;
      if (r < ND)
        for (int s2 = pp; s2 < SD; s2 += 4) acc += F.K[k][r][s2] * xc[s2];
      acc = q4_sum(acc);
      if (r < ND && pp == 0) sm.uo[ND * k + r] = sm.gk[k][r] - acc;
    }
    wave_sync();
    if (k + 1 < N) {
      // x_{k+1} = A x + B_k u_k
      double acc = 0.0;
      if (r < SD) {
        for (int q = pp; q < SD; q += 4) acc += sm.Ad[r * SD + q] * xc[q];
        if (r >= 6 && r < 9)
          for (int j = pp; j < ND; j += 4) acc += sm.Bw[k][r - 6][j] * sm.uo[ND * k + j];
        else if (r >= 9 && r < 12 && pp == 0)
          acc += dtm * (((sm.uo[ND * k + (r - 9)] + sm.uo[ND * k + 3 + (r - 9)]) + sm.uo[ND * k + 6 + (r - 9)]) +
                        sm.uo[ND * k + 9 + (r - 9)]);
      }
      acc = q4_sum(acc);
      if (r < SD && pp == 0) sm.xv[xb ^ 1][r] = acc;
      xb ^= 1;
      wave_sync();
    }
  }
}

template <int N>
__global__ __launch_bounds__(NT) void ric_solve_kernel(const double* __restrict__ recs, int batch,
                                                       mpcqp_result* __restrict__ results,
                                                       double* __restrict__ solution, double* __restrict__ work,
                                                       double* __restrict__ trace, int trace_cap, mpcqp_params p) {
  using Dm = Dim<N>;
  constexpr int n = Dm::n, m = Dm::m, nf = Dm::nf;
  __shared__ RSmem<N> sm;
  const int inst = blockIdx.x;
  if (inst >= batch) return;
  const int t = threadIdx.x;
  double* __restrict__ Hw = work + (size_t)inst * n * n;
  const double alpha = p.alpha, sigma = p.sigma;
  int rslot = 0;

  // ---- 0. record -> LDS, non-finite guard ----
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
  }

  // ---- 1. condensation (H to the workspace, gradient, bounds) + the dynamics the factorization needs
  condense<N, NT>(sm, p, Hw, n);
  {
    auto& C = sm.u.c;
    for (int e = t; e < SD * SD; e += NT) sm.Ad[e] = C.Ad[e];
    const double dt = sm.rec[MPCQP_REC_DT];
    for (int e = t; e < N * 3 * ND; e += NT) {  // rows 6-8 of B_d(k) = I_w^-1 skew(foot) dt (Utils.cpp:35-41)
      const int k = e / (3 * ND), rr = (e / ND) % 3, cc = e % ND;
      const int leg = cc / 3, c3 = cc % 3;
      const double* fp = sm.rec + Dm::feet + 12 * k + 3 * leg;
      const double sk0 = c3 == 0 ? 0.0 : c3 == 1 ? -fp[2] : fp[1];
      const double sk1 = c3 == 0 ? fp[2] : c3 == 1 ? 0.0 : -fp[0];
      const double sk2 = c3 == 0 ? -fp[1] : c3 == 1 ? fp[0] : 0.0;
      const double* iw = C.Iwinv + rr * 3;
      double s = 0.0;
      s += iw[0] * sk0;
      s += iw[1] * sk1;
      s += iw[2] * sk2;
      sm.Bw[k][rr][cc] = s * dt;
    }
    if (t == 0) sm.cst[4] = (1.0 / sm.rec[MPCQP_REC_MASS]) * dt;
  }
  // unscaled A rows (ConvexMpc.cpp:46-58) and variables
  for (int r = t; r < m; r += NT) {
    const int k5 = r % 5;
    const double mu = sm.rec[MPCQP_REC_MU];
    const double am = 1.0, az = k5 == 4 ? 0.0 : ((k5 & 1) ? -mu : mu);
    sm.ak[r][0] = k5 < 2 ? am : 0.0;
    sm.ak[r][1] = (k5 == 2 || k5 == 3) ? am : 0.0;
    sm.ak[r][2] = k5 < 4 ? az : am;
    sm.E[r] = 1.0;
  }
  for (int c = t; c < n; c += NT) {
    sm.D[c] = 1.0;
    sm.q[c] = sm.qt[c];
  }
  __syncthreads();

  // ---- 2. OSQP scale_data with the scaling deferred: P~ = c D H D is never formed; each pass
  // reads H once for the column maxima max_i D_i |H_ij| (H symmetric: column j of P~ has inf-norm
  // (c D_j) max_i D_i |H_ij|)
  double c_s = 1.0;
  if (p.scaling > 0) {
    for (int j = t; j < n; j += NT) {
      double mx = 0.0;
      for (int i = 0; i < n; ++i) mx = fmax(mx, dabs(Hw[(size_t)i * n + j]));
      sm.colmax[j] = mx;
    }
    __syncthreads();
  }
  for (int pass = 0; pass < p.scaling; ++pass) {
    // D_temp / E_temp
    for (int j = t; j < n; j += NT) {
      const int f = j / 3, a = j % 3;
      double ca = 0.0;
      for (int k = 0; k < 5; ++k) ca = fmax(ca, dabs(sm.ak[5 * f + k][a]));
      const double pc = (c_s * sm.D[j]) * sm.colmax[j];
      sm.Dt[j] = 1.0 / sqrt(limit_scaling(fmax(pc, ca)));
    }
    __syncthreads();
    for (int r = t; r < m; r += NT) {  // A <- E A D (row lanes)
      const int f = r / 5;
      const double et = 1.0 / sqrt(limit_scaling(fmax(fmax(dabs(sm.ak[r][0]), dabs(sm.ak[r][1])), dabs(sm.ak[r][2]))));
      sm.ak[r][0] = (sm.ak[r][0] * et) * sm.Dt[3 * f];
      sm.ak[r][1] = (sm.ak[r][1] * et) * sm.Dt[3 * f + 1];
      sm.ak[r][2] = (sm.ak[r][2] * et) * sm.Dt[3 * f + 2];
      sm.E[r] *= et;
    }
    for (int j = t; j < n; j += NT) {
      sm.q[j] = sm.Dt[j] * sm.q[j];
      sm.D[j] = sm.D[j] * sm.Dt[j];
    }
    __syncthreads();
    // cost normalization on the D-scaled P: column maxima with the new D
    double sv = 0.0, qv = 0.0;
    for (int j = t; j < n; j += NT) {
      double mx = 0.0;
      for (int i = 0; i < n; ++i) mx = fmax(mx, sm.D[i] * dabs(Hw[(size_t)i * n + j]));
      sm.colmax[j] = mx;
      sv += (c_s * sm.D[j]) * mx;
      qv = fmax(qv, dabs(sm.q[j]));
    }
    sv = wg_red1<RSmem<N>, false>(sm, sv, rslot);
    qv = wg_red1<RSmem<N>, true>(sm, qv, rslot);
    double c_temp = sv / n;
    const double inf_norm_q = limit_scaling(qv);
    c_temp = dmax(c_temp, inf_norm_q);
    c_temp = limit_scaling(c_temp);
    c_temp = 1. / c_temp;
    for (int j = t; j < n; j += NT) sm.q[j] *= c_temp;
    c_s *= c_temp;
    __syncthreads();
  }
  const double rho0 = dmin(dmax(p.rho, RHO_MIN), RHO_MAX);
  for (int r = t; r < m; r += NT) {
    const double E = sm.E[r];
    const double l = E * sm.lo[r], u = E * sm.hi[r];
    sm.lo[r] = l;
    sm.hi[r] = u;
    int ct;
    if (l < -OSQP_INF * MIN_SCALING && u > OSQP_INF * MIN_SCALING) ct = -1;
    else if (u - l < RHO_TOL) ct = 1;
    else ct = 0;
    sm.ctype[r] = ct;
    sm.rho_v[r] = ct == -1 ? RHO_MIN : ct == 1 ? RHO_EQ_OVER_RHO_INEQ * rho0 : rho0;
    sm.rho_inv[r] = 1. / sm.rho_v[r];
    sm.z[r] = 0.0;
    sm.y[r] = 0.0;
  }
  if (t == 0) {
    sm.cst[0] = c_s;
    sm.cst[1] = rho0;
    sm.cst[2] = 0.0;
    sm.cst[3] = 0.0;
  }
  __syncthreads();
  for (int c = t; c < n; c += NT) {
    bd_var<N>(sm, c);
    sm.x[c] = 0.0;
    sm.px[c] = 0.0;
    const double rr = sigma * 0.0 - sm.q[c];  // cold start
    sm.rhs[c] = rr;
    sm.w[c] = (1.0 / sm.D[c]) * rr;
  }
  __syncthreads();

  // ---- 3. ADMM ----
  int status = MPCQP_STATUS_UNSOLVED, iters = 0, rho_updates = 0, ntrace = 0;
  bool need_factor = true;
  int to_check = p.check_termination, to_adapt = p.adaptive_rho_interval;
  for (int iter = 1; iter <= p.max_iter; ++iter) {
    if (need_factor) {
      factorize<N>(sm, p, sigma);
      need_factor = false;
    }
    // x~ = K^-1 rhs = D^-1 (c B'Q̄B + R~)^-1 D^-1 rhs
    if (t < 64) {
      riccati_solve<N>(sm);
      for (int c = t; c < n; c += 64) sm.uo[c] = (1.0 / sm.D[c]) * sm.uo[c];
    }
    __syncthreads();
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
    // per-foot updates: update_z / update_y (rows), update_x + P~x by the KKT identity (vars);
    // delta y, delta x and the previous P~x are kept for the infeasibility tests
    for (int f = t; f < nf; f += NT) {
      const double x0 = sm.uo[3 * f], x1 = sm.uo[3 * f + 1], x2 = sm.uo[3 * f + 2];
      for (int k = 0; k < 5; ++k) {
        const int r = 5 * f + k;
        const double ztl = (sm.ak[r][0] * x0 + sm.ak[r][1] * x1) + sm.ak[r][2] * x2;
        const double zo = sm.z[r], yo = sm.y[r];
        const double zr = alpha * ztl + (1.0 - alpha) * zo;
        const double zn = dmin(dmax(zr + sm.rho_inv[r] * yo, sm.lo[r]), sm.hi[r]);
        const double dyv = sm.rho_v[r] * (zr - zn);
        sm.z[r] = zn;
        sm.y[r] = yo + dyv;
        sm.dy[r] = dyv;
      }
      for (int a = 0; a < 3; ++a) {
        const int c = 3 * f + a;
        const double xa = sel3(a, x0, x1, x2);
        const double xo = sm.x[c];
        const double xn = alpha * xa + (1.0 - alpha) * xo;
        const double kd = (sm.BD[c][0] * x0 + sm.BD[c][1] * x1) + sm.BD[c][2] * x2;
        const double pxt = sm.rhs[c] - sigma * xa - kd;
        sm.colmax[c] = sm.px[c];  // previous P~x
        sm.Dt[c] = xn - xo;       // delta x
        sm.px[c] = alpha * pxt + (1.0 - alpha) * sm.px[c];
        sm.x[c] = xn;
      }
    }
    __syncthreads();
    if (need_info) {
      // ---- update_info / check_termination / adapt_rho (osqp.c, auxil.c), as solve_kernel ----
      const double cost_c = sm.cst[0], cinv = 1. / cost_c;
      double rho = sm.cst[1];
      double mxv[14];
      for (int k = 0; k < 14; ++k) mxv[k] = 0.0;
      for (int f = t; f < nf; f += NT) {
        const double x0 = sm.x[3 * f], x1 = sm.x[3 * f + 1], x2 = sm.x[3 * f + 2];
        double aty[3] = {0.0, 0.0, 0.0};
        for (int k = 0; k < 5; ++k) {
          const int r = 5 * f + k;
          const double ax = (sm.ak[r][0] * x0 + sm.ak[r][1] * x1) + sm.ak[r][2] * x2;
          const double z = sm.z[r], Ei = 1.0 / sm.E[r];
          const double pr = ax + (-1.0) * z;
          mxv[0] = dmax(mxv[0], dabs(Ei * pr));
          mxv[1] = dmax(mxv[1], dabs(pr));
          mxv[2] = dmax(mxv[2], dabs(Ei * z));
          mxv[3] = dmax(mxv[3], dabs(z));
          mxv[4] = dmax(mxv[4], dabs(Ei * ax));
          mxv[5] = dmax(mxv[5], dabs(ax));
          for (int a = 0; a < 3; ++a) aty[a] += sm.ak[r][a] * sm.y[r];
        }
        for (int a = 0; a < 3; ++a) {
          const int c = 3 * f + a;
          const double Di = 1.0 / sm.D[c];
          const double qv = sm.q[c], pxv = sm.px[c];
          const double d = (qv + 1.0 * pxv) + 1.0 * aty[a];
          mxv[6] = dmax(mxv[6], dabs(Di * d));
          mxv[7] = dmax(mxv[7], dabs(d));
          mxv[8] = dmax(mxv[8], dabs(Di * qv));
          mxv[9] = dmax(mxv[9], dabs(qv));
          mxv[10] = dmax(mxv[10], dabs(Di * aty[a]));
          mxv[11] = dmax(mxv[11], dabs(aty[a]));
          mxv[12] = dmax(mxv[12], dabs(Di * pxv));
          mxv[13] = dmax(mxv[13], dabs(pxv));
        }
      }
      {
        const int lane = t & 63, wave = t >> 6;
        for (int k = 0; k < 14; ++k) {
          const double v = wave_max(mxv[k]);
          if (lane == 0) sm.info[wave][k] = v;
        }
      }
      __syncthreads();
      auto mx = [&](int k) __attribute__((always_inline)) {
        double v = sm.info[0][k];
        for (int w = 1; w < NWV; ++w) v = dmax(v, sm.info[w][k]);
        return v;
      };
      const double pri_res = mx(0);
      const double dua_res = cinv * mx(6);
      iters = iter;
      // check_termination (osqp.c): approx=1 is the post-loop check at max_iter (eps x 10)
      auto check = [&](bool approx) __attribute__((always_inline)) -> int {
        double eps_abs = p.eps_abs, eps_rel = p.eps_rel, eps_pinf = p.eps_prim_inf, eps_dinf = p.eps_dual_inf;
        if (pri_res > OSQP_INF || dua_res > OSQP_INF) return MPCQP_STATUS_NON_CVX;
        if (approx) { eps_abs *= 10; eps_rel *= 10; eps_pinf *= 10; eps_dinf *= 10; }
        const double eps_prim = eps_abs + eps_rel * dmax(mx(2), mx(4));
        const bool prim_ok = pri_res < eps_prim;
        bool prim_inf = false, dual_inf = false;
        if (!prim_ok) {
          // is_primal_infeasible: project delta_y onto the polar of the recession cone (in place)
          double nd = 0.0, lh = 0.0;
          for (int r = t; r < m; r += NT) {
            double d = sm.dy[r];
            if (sm.hi[r] > OSQP_INF * MIN_SCALING) {
              if (sm.lo[r] < -OSQP_INF * MIN_SCALING) d = 0.0;
              else d = dmin(d, 0.0);
            } else if (sm.lo[r] < -OSQP_INF * MIN_SCALING) {
              d = dmax(d, 0.0);
            }
            sm.dy[r] = d;
            nd = dmax(nd, dabs(sm.E[r] * d));
            lh += sm.hi[r] * dmax(d, 0.0) + sm.lo[r] * dmin(d, 0.0);
          }
          const double ndy = wg_red1<RSmem<N>, true>(sm, nd, rslot);
          if (ndy > DIV_TOL) {
            lh = wg_red1<RSmem<N>, false>(sm, lh, rslot);
            if (lh < eps_pinf * ndy) {
              double an = 0.0;
              for (int c = t; c < n; c += NT) {
                const int f = c / 3, a = c % 3;
                double atd = 0.0;
                for (int k = 0; k < 5; ++k) atd += sm.ak[5 * f + k][a] * sm.dy[5 * f + k];
                an = dmax(an, dabs((1.0 / sm.D[c]) * atd));
              }
              an = wg_red1<RSmem<N>, true>(sm, an, rslot);
              prim_inf = an < eps_pinf * ndy;
            }
          }
        }
        const double eps_dual = eps_abs + eps_rel * (cinv * dmax(dmax(mx(8), mx(10)), mx(12)));
        const bool dual_ok = dua_res < eps_dual;
        if (!dual_ok) {
          // is_dual_infeasible (P~ delta_x = P~x_new - P~x_old)
          double nx = 0.0, qd = 0.0;
          for (int c = t; c < n; c += NT) {
            nx = dmax(nx, dabs(sm.D[c] * sm.Dt[c]));
            qd += sm.q[c] * sm.Dt[c];
          }
          const double ndx = wg_red1<RSmem<N>, true>(sm, nx, rslot);
          if (ndx > DIV_TOL) {
            qd = wg_red1<RSmem<N>, false>(sm, qd, rslot);
            if (qd < cost_c * eps_dinf * ndx) {
              double pd = 0.0;
              for (int c = t; c < n; c += NT) pd = dmax(pd, dabs((1.0 / sm.D[c]) * (sm.px[c] - sm.colmax[c])));
              pd = wg_red1<RSmem<N>, true>(sm, pd, rslot);
              if (pd < cost_c * eps_dinf * ndx) {
                double viol = 0.0;
                for (int r = t; r < m; r += NT) {
                  const int f = r / 5;
                  const double adx =
                      (sm.ak[r][0] * sm.Dt[3 * f] + sm.ak[r][1] * sm.Dt[3 * f + 1]) + sm.ak[r][2] * sm.Dt[3 * f + 2];
                  const double v = (1.0 / sm.E[r]) * adx;
                  if ((sm.hi[r] < OSQP_INF * MIN_SCALING && v > eps_dinf * ndx) ||
                      (sm.lo[r] > -OSQP_INF * MIN_SCALING && v < -eps_dinf * ndx))
                    viol = 1.0;
                }
                viol = wg_red1<RSmem<N>, true>(sm, viol, rslot);
                dual_inf = viol == 0.0;
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
        if (pass == 1 && !last) break;
        if (pass == 1 || is_check || last) {
          st = check(pass == 1);
          done = st != MPCQP_STATUS_UNSOLVED;
        }
        if (pass == 1 || done || !is_adapt) continue;
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
      if (trace && t == 0 && inst < trace_cap && ntrace < MPCQP_TRACE_LEN && is_check) {
        double* tp = trace + ((size_t)inst * MPCQP_TRACE_LEN + ntrace) * 4;
        tp[0] = iter; tp[1] = pri_res; tp[2] = dua_res; tp[3] = rho;
      }
      ntrace += is_check ? 1 : 0;
      __syncthreads();  // every mx() read precedes the writes below
      if (t == 0) {
        sm.cst[1] = rho;
        sm.cst[2] = pri_res;
        sm.cst[3] = dua_res;
      }
      if (done) break;
      if (refactor) {
        for (int r = t; r < m; r += NT) {
          const int ct = sm.ctype[r];
          sm.rho_v[r] = ct == -1 ? sm.rho_v[r] : ct == 1 ? RHO_EQ_OVER_RHO_INEQ * rho : rho;
          sm.rho_inv[r] = 1. / sm.rho_v[r];
        }
        __syncthreads();
        for (int c = t; c < n; c += NT) bd_var<N>(sm, c);
        need_factor = true;
      }
      __syncthreads();
    }
    // next rhs = sigma x - q~ + A~'(rho z - y) (per variable, rows in order), w = D^-1 rhs
    for (int f = t; f < nf; f += NT) {
      for (int a = 0; a < 3; ++a) {
        const int c = 3 * f + a;
        double acc = sigma * sm.x[c] - sm.q[c];
        for (int k = 0; k < 5; ++k) {
          const int r = 5 * f + k;
          acc += sm.ak[r][a] * (sm.rho_v[r] * sm.z[r] - sm.y[r]);
        }
        sm.rhs[c] = acc;
        sm.w[c] = (1.0 / sm.D[c]) * acc;
      }
    }
    __syncthreads();
  }

  // ---- 4. store_solution + unscale + compute_grf extraction (A1RobotControl.cpp:555-561) ----
  const double cinv = 1. / sm.cst[0], rho = sm.cst[1], pri_res = sm.cst[2], dua_res = sm.cst[3];
  const bool has_sol = status != MPCQP_STATUS_PRIMAL_INFEASIBLE &&
                       status != MPCQP_STATUS_PRIMAL_INFEASIBLE_INACCURATE &&
                       status != MPCQP_STATUS_DUAL_INFEASIBLE &&
                       status != MPCQP_STATUS_DUAL_INFEASIBLE_INACCURATE && status != MPCQP_STATUS_NON_CVX;
  double ob = 0.0;
  for (int c = t; c < n; c += NT) ob += 0.5 * sm.x[c] * sm.px[c] + sm.q[c] * sm.x[c];
  ob = wg_red1<RSmem<N>, false>(sm, ob, rslot);
  for (int c = t; c < n; c += NT) {
    const double xs = has_sol ? sm.D[c] * sm.x[c] : NAN;
    sm.uo[c] = xs;
    if (solution) solution[(size_t)inst * n + c] = xs;
  }
  __syncthreads();
  if (t == 0) {
    mpcqp_result* res = results + inst;
    const double* R = sm.rec + MPCQP_REC_ROT;
    int legs = 0;
    for (int l = 0; l < 4; ++l) {
      const double u0 = sm.uo[3 * l], u1 = sm.uo[3 * l + 1], u2 = sm.uo[3 * l + 2];
      const double nrm = sqrt(u0 * u0 + u1 * u1 + u2 * u2);
      const bool nanleg = isnan(nrm);
      legs |= nanleg ? (1 << l) : 0;
      for (int a = 0; a < 3; ++a) {
        double s = 0.0;
        s += R[0 * 3 + a] * u0;
        s += R[1 * 3 + a] * u1;
        s += R[2 * 3 + a] * u2;
        res->u0[3 * l + a] = sm.uo[3 * l + a];
        res->f_body[3 * l + a] = nanleg ? 0.0 : s;
      }
    }
    res->nan_legs = legs;
    double obj;
    if (has_sol) obj = ob * cinv;
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

}  // namespace ric
}  // namespace mpcqp

namespace mpcqp {
template <int N>
static hipError_t launch_ric(const LaunchArgs& a) {
  hipLaunchKernelGGL((ric::ric_solve_kernel<N>), dim3(a.grid), dim3(ric::NT), 0, (hipStream_t)a.stream, a.recs,
                     a.batch, a.results, a.solution, a.work, a.trace, a.trace_cap, a.p);
  return hipGetLastError();
}
template <int N>
static hipError_t occupancy_ric(int* blocks) {
  return hipOccupancyMaxActiveBlocksPerMultiprocessor(blocks, ric::ric_solve_kernel<N>, ric::NT, 0);
}

#define MPCQP_RIC_FOR_EACH_N(X) \
  X(1) X(2) X(3) X(4) X(5) X(6) X(7) X(8) X(9) X(10) X(11) X(12) X(13) X(14) X(15) X(16) X(17) X(18) X(19) X(20)

hipError_t launch_riccati_any(const LaunchArgs& a) {
  switch (a.p.horizon) {
#define CASE(K) \
  case K: return launch_ric<K>(a);
    MPCQP_RIC_FOR_EACH_N(CASE)
#undef CASE
    default: return hipErrorInvalidValue;
  }
}
hipError_t occupancy_riccati_any(int horizon, int* blocks) {
  switch (horizon) {
#define CASE(K) \
  case K: return occupancy_ric<K>(blocks);
    MPCQP_RIC_FOR_EACH_N(CASE)
#undef CASE
    default: return hipErrorInvalidValue;
  }
}
int riccati_threads(int) { return ric::NT; }
size_t riccati_workspace_doubles(int horizon) {  // the condensed Hessian, n x n
  const size_t n = 12 * (size_t)horizon;
  return n * n;
}
}  // namespace mpcqp
