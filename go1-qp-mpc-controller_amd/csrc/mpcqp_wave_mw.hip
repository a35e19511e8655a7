// mpcqp_wave_mw.hip — the OSQP 0.6 solve of ConvexMpc's QP with ONE WAVE PER HORIZON ROUND.
//
// Same algorithm, lane layout and arithmetic as wave_kernel (mpcqp_wave.hip): the KKT system is
// solved through the problem's LQR structure, horizon step k sits in DPP row gray(k & 3) of round
// k >> 2, lane 4l + a = component a of leg l.  Here the R = ceil(N/4) rounds are R waves of one
// workgroup instead of R register sets of one wave: every parallel phase (a_k = K_k'w_k, g_k, h_k,
// u_k, the ADMM updates, the termination tests) runs in all waves at once on their own four steps,
// and the two sequential Riccati chains run in wave 0, which reads each step's a_k / h_k from LDS
// and leaves s_{k+1} / x_k there (no row hand-offs).  A robot's ADMM iteration is shorter by the
// parallel phases' share, and so is the tail of a batch, which is set by its slowest robots.
//
// Reference path: A1RobotControl::compute_grf (src/a1_cpp/src/A1RobotControl.cpp:446-562) ->
// ConvexMpc (src/a1_cpp/src/ConvexMpc.cpp:7-245) -> OsqpEigen 0.6.3 / OSQP 0.6 (restated in
// oracle/mpc_oracle.c: scale_data runs in scale_kernel; set_rho_vec, update_xz_tilde,
// update_x/z/y, update_info, check_termination, adapt_rho, store_solution here).
#include "mpcqp_wave_common.h"

namespace mpcqp {
namespace mw {
using namespace wv;

template <int N>
struct MwCfg {
  static constexpr int R = (N + 3) / 4;  // rounds = waves
  static constexpr int NT = 64 * R;
  static constexpr int WPE = R <= 3 ? 3 : 2;  // waves per SIMD the register budget is sized for
};

template <int N>
struct MwMem {
  using C = Cfg<N>;
  static constexpr int NK = N > 1 ? N - 1 : 1;  // K_k stored for k = 1..N-1
  static constexpr int NA = N > 2 ? N - 2 : 1;  // Acl_k stored for k = 1..N-2
  alignas(16) double Bw[N][3][ND];  // rows 6-8 of B_d(k) = I_w^-1 skew(foot) dt (rows 9-11: dt/m I)
  alignas(16) double xa[N][16];     // per step: a_k (backward chain input), then h_k (forward)
  alignas(16) double xs[N][16];     // per step: s_{k+1} (backward chain output), then x_k (forward)
  double red[32][8];                // block reductions [slot][wave] (0-13 norms, 14-27 tests, 31 obj)
  union U {
    struct Hs {
      double rec[C::REC];
      double D[C::n], Dt[C::n], q[C::n], E[C::m];
      double lam[N][ND];
      double vec[2][16];
      double Ap[2][C::m];
      double qn[C::n];
    } h;
    struct Fs {
      alignas(16) double Gi[N][MS];
      alignas(16) double K[NK][MS];
      alignas(16) double Acl[NA][MS];
      double Rt[N][4][6];
    } f;
  } u;
};

// block-wide max / sum over the R waves: each wave's value through slot `s` of the LDS table (the
// caller keeps slots distinct between two barriers); every wave gets the same value.
template <int R>
__device__ __forceinline__ double bmax(double v, double (*red)[8], int s) {
  v = wave_max(v);
  if constexpr (R == 1) {
    return v;
  } else {
    if ((threadIdx.x & 63) == 0) red[s][threadIdx.x >> 6] = v;
    __syncthreads();
    double x = red[s][0];
#pragma unroll
    for (int i = 1; i < R; ++i) x = dmax(x, red[s][i]);
    return x;
  }
}
template <int R>
__device__ __forceinline__ double bsum(double v, double (*red)[8], int s) {
  v = wave_sum(v);
  if constexpr (R == 1) {
    return v;
  } else {
    if ((threadIdx.x & 63) == 0) red[s][threadIdx.x >> 6] = v;
    __syncthreads();
    double x = red[s][0];
#pragma unroll
    for (int i = 1; i < R; ++i) x = x + red[s][i];
    return x;
  }
}

template <int N>
__global__ __launch_bounds__(MwCfg<N>::NT, MwCfg<N>::WPE) void mw_kernel(
    const double* __restrict__ recs, int batch, mpcqp_result* __restrict__ results, double* __restrict__ solution,
    double* __restrict__ trace, int trace_cap, double* __restrict__ wstate, const double* __restrict__ img,
    mpcqp_params p) {
  using C = Cfg<N>;
  using WL = WarmLayout<N>;
  using SI = ScaleImg<N>;
  constexpr int n = C::n, m = C::m, R = MwCfg<N>::R, NT = MwCfg<N>::NT;
  __shared__ MwMem<N> sm;
  const int inst = blockIdx.x;
  if (inst >= batch) return;
  const int t = threadIdx.x;
  const int w = t >> 6, lt = t & 63;  // wave = round
  const int q = lt >> 4, li = lt & 15, leg = li >> 2, a = li & 3;
  const bool av = a < 3;
  const int idx = 3 * leg + (av ? a : 2);  // index inside a step (padding lanes alias component 2)
  const int k = 4 * w + gray(q);            // this lane's horizon step
  const bool kv = k < N, vv = kv && av;
  const int kc = kv ? k : N - 1, kk = kc > 0 ? kc - 1 : 0;  // clamped step, slot of K_k
  const double alpha = p.alpha, sigma = p.sigma;
  auto& HS = sm.u.h;
  auto& F = sm.u.f;

  // ---- 0. record -> LDS, non-finite guard -------------------------------------------------------
  {
    const double* rg = recs + (size_t)inst * C::REC;
    int bad = 0;
    for (int e = t; e < C::REC; e += NT) {
      const double v = rg[e];
      HS.rec[e] = v;
      bad |= !isfinite(v);
    }
    if (__syncthreads_or(bad)) {
      if (t == 0) {
        mpcqp_result r;
        for (int i = 0; i < ND; ++i) { r.u0[i] = NAN; r.f_body[i] = 0.0; }
        r.obj_val = NAN; r.pri_res = NAN; r.dua_res = NAN; r.rho = p.rho;
        r.status = MPCQP_STATUS_NAN_INPUT; r.iters = 0; r.rho_updates = 0; r.nan_legs = 0xF;
        results[inst] = r;
      }
      if (solution)
        for (int e = t; e < n; e += NT) solution[(size_t)inst * n + e] = NAN;
      return;
    }
  }
  const double* rec = HS.rec;
  const double dt = rec[MPCQP_REC_DT], mass = rec[MPCQP_REC_MASS], mu = rec[MPCQP_REC_MU];
  Adisc A;
  {
    const double yaw = rec[MPCQP_REC_EULER + 2];
    A.ad0 = cos(yaw) * dt;
    A.ad1 = sin(yaw) * dt;
    A.dt = dt;
  }
  const double dtm = (1.0 / mass) * dt;
  double Rot[9];
#pragma unroll
  for (int e = 0; e < 9; ++e) Rot[e] = rec[MPCQP_REC_ROT + e];
  const double cont = rec[MPCQP_REC_CONTACTS + leg] != 0.0 ? 1.0 : 0.0;
  const double fzmin = rec[MPCQP_REC_FZMIN], fzmax = rec[MPCQP_REC_FZMAX];

  // ---- 1. B_d(k) rows 6-8 (calculate_B_mat_c, Utils.cpp:35-41) --------------------------------------
  {
    double Iwinv[9];
    iw_inverse(rec, Iwinv);
    for (int e = t; e < N * 36; e += NT) {
      const int kb = e / 36, rr = (e / 12) % 3, cc = e % 12;
      const int lg = cc / 3, c3 = cc % 3;
      const double* fp = rec + MPCQP_REC_FEET(N) + 12 * kb + 3 * lg;
      const double sk0 = c3 == 0 ? 0.0 : c3 == 1 ? -fp[2] : fp[1];
      const double sk1 = c3 == 0 ? fp[2] : c3 == 1 ? 0.0 : -fp[0];
      const double sk2 = c3 == 0 ? -fp[1] : c3 == 1 ? fp[0] : 0.0;
      double s = 0.0;
      s += sel3(rr, Iwinv[0], Iwinv[3], Iwinv[6]) * sk0;
      s += sel3(rr, Iwinv[1], Iwinv[4], Iwinv[7]) * sk1;
      s += sel3(rr, Iwinv[2], Iwinv[5], Iwinv[8]) * sk2;
      sm.Bw[kb][rr][cc] = s * dt;
    }
  }

  // ---- 3. OSQP scale_data: the image scale_kernel wrote (D, E, q~, raw q, A entries, c, branch) ----
  const double* im = img + (size_t)inst * SI::SIZE;
  for (int j = t; j < n; j += NT) {
    HS.D[j] = im[SI::D + j];
    HS.q[j] = im[SI::Q + j];
    HS.qn[j] = im[SI::QN + j];
  }
  for (int r = t; r < m; r += NT) {
    HS.E[r] = im[SI::E + r];
    HS.Ap[0][r] = im[SI::AP + r];
    HS.Ap[1][r] = im[SI::AP + m + r];
  }
  const double c_s = im[SI::CS];
  const int mode = (int)im[SI::MODE];  // 0 cold, 1 osqp_update_P, 2 OsqpEigen re-init
  double* const ws = wstate ? wstate + (size_t)inst * WL::SIZE : nullptr;
  __syncthreads();
  const double cost_c = c_s, cinv = 1. / c_s;

  // ---- 4. lane registers: variable (D, q~) and rows (E, A~, bounds, rho) of this lane — set_rho_vec
  const double rho0 = mode == 1 ? ws[WL::RHO] : dmin(dmax(p.rho, RHO_MIN), RHO_MAX);
  const int ci = ND * kc + idx, ri = CD * kc + 5 * leg + a, r4 = CD * kc + 5 * leg + 4;
  const int cf = ND * kc + 3 * leg;  // the leg's three variables
  const double Dv = vv ? HS.D[ci] : 1.0;
  const double DI = 1. / Dv;
  // update_P then osqp_update_lin_cost: q~ = c (D q) of this tick's gradient
  const double Qv = vv ? (mode == 1 ? (HS.qn[ci] * Dv) * c_s : HS.q[ci]) : 0.0;
  const double Ev = kv ? HS.E[ri] : 1.0;
  const double E4 = kv ? HS.E[r4] : 1.0;
  // A~ = E A D: row a < 4 has A on fx (a < 2) / fy (a >= 2) and on fz; row 4 on fz
  const double AK0 = kv ? (HS.Ap[0][ri] * Ev) * HS.D[cf + (a >> 1)] : 0.0;
  const double AK1 = kv ? (HS.Ap[1][ri] * Ev) * HS.D[cf + 2] : 0.0;
  const double AK4 = kv ? (HS.Ap[1][r4] * E4) * HS.D[cf + 2] : 0.0;
  double L4, U4;
  {  // bounds (ConvexMpc.cpp:223-245), clipped to +-OSQP_INFTY, scaled by E
    double l4 = fzmin * cont, u4 = fzmax * cont;
    l4 = dmin(dmax(l4, -OSQP_INF), OSQP_INF);
    u4 = dmin(dmax(u4, -OSQP_INF), OSQP_INF);
    L4 = E4 * l4;
    U4 = E4 * u4;
  }
  double X = 0.0, PX = 0.0, PXO = 0.0, DX = 0.0;
  double Z = 0.0, Y = 0.0, DY = 0.0, Z4 = 0.0, Y4 = 0.0, DY4 = 0.0;
  double RHS = vv ? sigma * 0.0 - Qv : 0.0;  // cold start: compute_rhs with x = z = y = 0
  if (mode == 1) {  // warm start: the previous scaled iterates as they are
    X = vv ? ws[WL::X + ci] : 0.0;
    Z = kv ? ws[WL::Z + ri] : 0.0;
    Y = kv ? ws[WL::Y + ri] : 0.0;
    Z4 = kv ? ws[WL::Z + r4] : 0.0;
    Y4 = kv ? ws[WL::Y + r4] : 0.0;
  } else if (mode == 2) {  // re-init: x = D^-1 (D_old x_old), y = c E^-1 ((E_old y_old) c_old^-1)
    const double cinv_o = 1. / ws[WL::C];
    X = vv ? DI * (ws[WL::D + ci] * ws[WL::X + ci]) : 0.0;
    Y = kv ? c_s * ((1. / Ev) * ((ws[WL::E + ri] * ws[WL::Y + ri]) * cinv_o)) : 0.0;
    Y4 = kv ? c_s * ((1. / E4) * ((ws[WL::E + r4] * ws[WL::Y + r4]) * cinv_o)) : 0.0;
    const double xp = dpp<QP_PRIM>(X), xz = dpp<QP_B2>(X);  // z = A~ x
    Z = AK0 * xp + AK1 * xz;
    Z4 = AK4 * xz;
  }
  auto rho4_of = [&](double rho) __attribute__((always_inline)) {
    const bool loose = L4 < -OSQP_INF * MIN_SCALING && U4 > OSQP_INF * MIN_SCALING;
    const bool eq = U4 - L4 < RHO_TOL;
    return loose ? RHO_MIN : (eq ? RHO_EQ_OVER_RHO_INEQ * rho : rho);
  };
  double RHO4 = rho4_of(rho0), RI4 = 1. / RHO4;  // rho of row 4 and OSQP's rho_inv_vec entry
  if (mode != 0) {
    // P~x of the warm iterate (the loop carries P~x through the KKT identity from here):
    // P~x = c D H (D x), H v = B_qp' Q B_qp v + R v by the dynamics: x_{i+1} = A x_i + B_i v_i
    // from x_0 = 0, e_i = Q x_{i+1}, lambda_j = e_j + A' lambda_{j+1}, (H v)_j = B_j' lambda_j + R v_j.
    if (vv) HS.Dt[ci] = Dv * X;
    if (t < 16) HS.vec[0][t] = 0.0;
    __syncthreads();
    if (w == 0) {
      for (int i = 0; i < N; ++i) {
        if (t < ND) {
          const double* pv = HS.vec[i & 1];
          const double* v = HS.Dt + ND * i;
          double s;
          if (t == 0) s = (pv[0] + A.ad0 * pv[6]) + A.ad1 * pv[7];
          else if (t == 1) s = (pv[1] + (-A.ad1) * pv[6]) + A.ad0 * pv[7];
          else if (t == 2) s = pv[2] + dt * pv[8];
          else if (t <= 5) s = pv[t] + dt * pv[t + 6];
          else s = pv[t];
          double bu = 0.0;
          if (t >= 6 && t < 9) {
            const double* bw = sm.Bw[i][t - 6];
            for (int c2 = 0; c2 < ND; ++c2) bu += bw[c2] * v[c2];
          } else if (t >= 9) {
            bu = dtm * (((v[t - 9] + v[t - 6]) + v[t - 3]) + v[t]);
          }
          const double xn = s + bu;
          HS.vec[(i + 1) & 1][t] = xn;
          HS.lam[i][t] = 2 * p.q_weights[t] * xn;
        }
        wave_sync();
      }
      for (int j = N - 2; j >= 0; --j) {
        if (t < ND) HS.lam[j][t] = HS.lam[j][t] + A.atv(t, HS.lam[j + 1]);
        wave_sync();
      }
    }
    __syncthreads();
    {
      const double* lm = HS.lam[kc];
      const double hv = (((sm.Bw[kc][0][idx] * lm[6] + sm.Bw[kc][1][idx] * lm[7]) + sm.Bw[kc][2][idx] * lm[8]) +
                         dtm * lm[9 + idx % 3]) + (2 * p.r_weights[idx]) * HS.Dt[ci];
      PX = vv ? (c_s * Dv) * hv : 0.0;
      // compute_rhs from the warm x, z, y: sigma x - q~ + A~'(rho z - y)
      const double at = quad_at(rho0 * Z - Y, RHO4 * Z4 - Y4, AK0, AK1, AK4, a);
      RHS = vv ? (sigma * X - Qv) + at : 0.0;
    }
  }
  // rows 0-3: l = 0 / u = +inf (rows 0, 2) or l = -inf / u = 0 (rows 1, 3): always inequalities
  const double lo03 = (a & 1) ? Ev * -OSQP_INF : Ev * 0.0, hi03 = (a & 1) ? Ev * 0.0 : Ev * OSQP_INF;
  // the projection onto those bounds needs no E: [0, +inf) for rows 0, 2, (-inf, 0] for rows 1, 3
  const double LO03 = (a & 1) ? -INFINITY : 0.0, HI03 = (a & 1) ? 0.0 : INFINITY;
  const double dm0 = a == 0 ? dtm : 0.0, dm1 = a == 1 ? dtm : 0.0, dm2 = a == 2 ? dtm : 0.0;
  __syncthreads();  // every LDS read of the setup image precedes its reuse by the factorization

  // ---- 5. ADMM (osqp_solve) ------------------------------------------------------------------------
  double rho = rho0, rinv = 1. / rho0, pri_res = 0.0, dua_res = 0.0;
  int status = MPCQP_STATUS_UNSOLVED, iters = 0, rho_updates = 0, ntrace = 0;
  bool need_factor = true;
  int to_check = p.check_termination, to_adapt = p.adaptive_rho_interval;
  for (int iter = 1; iter <= p.max_iter; ++iter) {
    if (need_factor) {
      {  // R'_k foot blocks of this lane's step: c 2r + D^-1 (sigma I + A~' diag(rho) A~) D^-1
        const double k00 = dpp<QP_B0>(AK0), k01 = dpp<QP_B1>(AK0), k02 = dpp<QP_B2>(AK0), k03 = dpp<QP_B3>(AK0);
        const double k10 = dpp<QP_B0>(AK1), k11 = dpp<QP_B1>(AK1), k12 = dpp<QP_B2>(AK1), k13 = dpp<QP_B3>(AK1);
        const double d0 = dpp<QP_B0>(Dv), d1 = dpp<QP_B1>(Dv), d2 = dpp<QP_B2>(Dv);
        const double ak4 = AK4, r4 = RHO4;
        // rows of the foot: r0 [k00,0,k10] r1 [k01,0,k11] r2 [0,k02,k12] r3 [0,k03,k13] r4 [0,0,ak4]
        auto coef = [&](int row, int col) __attribute__((always_inline)) {
          if (row == 4) return col == 2 ? ak4 : 0.0;
          const double kp = row == 0 ? k00 : row == 1 ? k01 : row == 2 ? k02 : k03;
          const double kz = row == 0 ? k10 : row == 1 ? k11 : row == 2 ? k12 : k13;
          if (col == 2) return kz;
          return (col == (row >> 1)) ? kp : 0.0;
        };
        const double da = a == 0 ? d0 : (a == 1 ? d1 : d2);
#pragma unroll
        for (int b = 0; b < 3; ++b) {
          double s = 0.0;
#pragma unroll
          for (int row = 0; row < 5; ++row) s += (coef(row, av ? a : 2) * (row == 4 ? r4 : rho)) * coef(row, b);
          const double db = b == 0 ? d0 : (b == 1 ? d1 : d2);
          const double rt = (av && a == b ? cost_c * (2.0 * p.r_weights[idx]) : 0.0) +
                            ((1.0 / da) * ((av && a == b ? sigma : 0.0) + s)) * (1.0 / db);
          if (kv && av && b >= a) F.Rt[k][leg][sym6(a, b)] = rt;
        }
      }
      __syncthreads();
      if (w == 0) factorize_mfma<N>(sm, p, A, cost_c, dtm);
      __syncthreads();
      need_factor = false;
    }

    // ---- KKT solve: u = (c B'Q̄B + R')^-1 D^-1 rhs, x~ = D^-1 u ----
    double U;
    {
      const double W = DI * RHS;
      double cA[12], cB[12];
      ld12s(cA, &F.K[kk][idx]);  // K_k column
      ld12(cB, &F.Gi[kc][mo(idx)]);
      const double cw0 = sm.Bw[kc][0][idx], cw1 = sm.Bw[kc][1][idx], cw2 = sm.Bw[kc][2][idx];
      __builtin_amdgcn_sched_barrier(0);
      // a_k = K_k' w_k (k >= 1) -> LDS for the chain
      const double akw = mv12(W, cA);
      if (kv) sm.xa[k][li] = akw;
      __syncthreads();
      if (w == 0) {  // backward chain: s_{N-1} = -a_{N-1}; s_k = Acl_k' s_{k+1} - a_k; xs[k] = s_{k+1}
        double cur = -sm.xa[N - 1][li];
        sm.xs[N - 1][li] = 0.0;
        double cn[12], an = 0.0;
        if constexpr (N >= 3) ld12s(cn, &F.Acl[N - 3][idx]);
        if constexpr (N >= 2) an = sm.xa[N - 2][li];
        sfor<0, N - 1>([&](auto J) {
          constexpr int kb = N - 2 - decltype(J)::value;
          sm.xs[kb][li] = cur;
          if constexpr (kb >= 1) {
            double cc[12];
#pragma unroll
            for (int e = 0; e < 12; ++e) cc[e] = cn[e];
            const double ac = an;
            if constexpr (kb >= 2) {  // the next step's column and a
              ld12s(cn, &F.Acl[kb - 2][idx]);
              an = sm.xa[kb - 1][li];
            }
            __builtin_amdgcn_sched_barrier(0);
            cur = mv12a(cur, cc, -ac);
          }
        });
      }
      ld12(cA, &sm.Bw[kc][av ? a : 2][0]);  // for h_k
      __syncthreads();
      // g_k = G_k^-1 (w_k + B_k' s_{k+1}); h_k = B_k g_k (rows 6-8: B_w g on the leg-2 lanes, rows
      // 9-11: dt/m times the legs' matching force component on the leg-3 lanes, rows 0-5 zero)
      const double smv = sm.xs[kc][li];
      const double c6[6] = {cw0, cw1, cw2, dm0, dm1, dm2};
      const double tt = W + mv6(smv, c6);
      const double G = mv12(tt, cB);
      const double hb = mv12(G, cA);
      // (legsum's DPP reads other legs' lanes: evaluated by every lane, outside the select — a
      // conditional would run it with those lanes masked off and read zeros)
      const double ls = dtm * legsum(G);
      const double Hh = leg == 2 ? hb : (leg == 3 ? ls : 0.0);
      if (kv) sm.xa[k][li] = Hh;
      ld12(cB, &F.K[kk][mo(idx)]);  // for u_k
      __syncthreads();
      if (w == 0) {  // forward chain: x_1 = h_0; x_{k+1} = Acl_k x_k + h_k; xs[k] = x_k (x_0 = 0)
        double cur = sm.xa[0][li];
        sm.xs[0][li] = 0.0;
        double cn[12], hn = 0.0;
        if constexpr (N >= 3) ld12(cn, &F.Acl[0][mo(idx)]);
        if constexpr (N >= 2) hn = sm.xa[1][li];
        sfor<1, N>([&](auto K) {
          constexpr int kb = decltype(K)::value;
          sm.xs[kb][li] = cur;
          if constexpr (kb <= N - 2) {
            double cc[12];
#pragma unroll
            for (int e = 0; e < 12; ++e) cc[e] = cn[e];
            const double hc = hn;
            if constexpr (kb + 1 <= N - 2) {  // the next step's row and h
              ld12(cn, &F.Acl[kb][mo(idx)]);
              hn = sm.xa[kb + 1][li];
            }
            __builtin_amdgcn_sched_barrier(0);
            cur = mv12a(cur, cc, hc);
          }
        });
      }
      __syncthreads();
      // u_k = g_k - K_k x_k (x_0 = 0)
      const double xs = sm.xs[kc][li];
      U = G - mv12(xs, cB);
#ifdef MPCQP_DBG
      U = MPCQP_DBG == 1 ? G : MPCQP_DBG == 2 ? Hh : MPCQP_DBG == 3 ? xs : MPCQP_DBG == 4 ? smv : W;
#endif
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

    // ---- update_x / update_z / update_y, and P~x by the KKT identity P~x~ = rhs - sigma x~ - A~'rho A~x~
    {
      const double xt = DI * U;
      const double xp = dpp<QP_PRIM>(xt), xz = dpp<QP_B2>(xt);
      const double zt = AK0 * xp + AK1 * xz;
      const double zt4 = AK4 * xz;
      {  // (fmin/fmax = the reference's c_min/c_max on these non-NaN operands)
        const double zr = alpha * zt + (1.0 - alpha) * Z;
        const double zn = fmin(fmax(zr + rinv * Y, LO03), HI03);
        const double dyv = rho * (zr - zn);
        Z = zn;
        Y = Y + dyv;
        DY = dyv;
      }
      {
        const double zr = alpha * zt4 + (1.0 - alpha) * Z4;
        const double zn = fmin(fmax(zr + RI4 * Y4, L4), U4);
        const double dyv = RHO4 * (zr - zn);
        Z4 = zn;
        Y4 = Y4 + dyv;
        DY4 = dyv;
      }
      const double kd = quad_at(rho * zt, RHO4 * zt4, AK0, AK1, AK4, a);
      // every lane updates (values of padding lanes / steps past N are never read unmasked)
      const double xo = X;
      const double xn = alpha * xt + (1.0 - alpha) * xo;
      DX = xn - xo;
      X = xn;
      const double pxt = (RHS - sigma * xt) - kd;
      PXO = PX;
      PX = alpha * pxt + (1.0 - alpha) * PX;
    }

    if (need_info) {
      // ---- update_info / check_termination / adapt_rho (osqp.c, auxil.c) ----
      double mx[14];
#pragma unroll
      for (int i = 0; i < 14; ++i) mx[i] = 0.0;
      {
        const double xp = dpp<QP_PRIM>(X), xz = dpp<QP_B2>(X);
        const double ax = AK0 * xp + AK1 * xz, ax4 = AK4 * xz;
        const double aty = quad_at(Y, Y4, AK0, AK1, AK4, a);
        if (kv) {
          const double ei = 1.0 / Ev, ei4 = 1.0 / E4;
          const double pr = ax + (-1.0) * Z, pr4 = ax4 + (-1.0) * Z4;
          mx[0] = dmax(dabs(ei * pr), dabs(ei4 * pr4));
          mx[1] = dmax(dabs(pr), dabs(pr4));
          mx[2] = dmax(dabs(ei * Z), dabs(ei4 * Z4));
          mx[3] = dmax(dabs(Z), dabs(Z4));
          mx[4] = dmax(dabs(ei * ax), dabs(ei4 * ax4));
          mx[5] = dmax(dabs(ax), dabs(ax4));
        }
        if (vv) {
          const double d = (Qv + 1.0 * PX) + 1.0 * aty;
          mx[6] = dabs(DI * d);
          mx[7] = dabs(d);
          mx[8] = dabs(DI * Qv);
          mx[9] = dabs(Qv);
          mx[10] = dabs(DI * aty);
          mx[11] = dabs(aty);
          mx[12] = dabs(DI * PX);
          mx[13] = dabs(PX);
        }
      }
#pragma unroll
      for (int i = 0; i < 14; ++i) {  // one barrier for all fourteen
        mx[i] = wave_max(mx[i]);
        if (R > 1 && lt == 0) sm.red[i][w] = mx[i];
      }
      if constexpr (R > 1) {
        __syncthreads();
#pragma unroll
        for (int i = 0; i < 14; ++i) {
          double x = sm.red[i][0];
#pragma unroll
          for (int j = 1; j < R; ++j) x = dmax(x, sm.red[i][j]);
          mx[i] = x;
        }
      }
      pri_res = mx[0];
      dua_res = cinv * mx[6];
      iters = iter;
      auto check = [&](bool approx, int slot) __attribute__((always_inline)) -> int {
        double eps_abs = p.eps_abs, eps_rel = p.eps_rel, eps_pinf = p.eps_prim_inf, eps_dinf = p.eps_dual_inf;
        if (pri_res > OSQP_INF || dua_res > OSQP_INF) return MPCQP_STATUS_NON_CVX;
        if (approx) { eps_abs *= 10; eps_rel *= 10; eps_pinf *= 10; eps_dinf *= 10; }
        const double eps_prim = eps_abs + eps_rel * dmax(mx[2], mx[4]);
        const bool prim_ok = pri_res < eps_prim;
        bool prim_inf = false, dual_inf = false;
        if (!prim_ok) {
          // is_primal_infeasible: delta_y projected onto the polar of the recession cone
          auto proj = [&](double d, double lo, double hi) __attribute__((always_inline)) {
            if (hi > OSQP_INF * MIN_SCALING) {
              if (lo < -OSQP_INF * MIN_SCALING) d = 0.0;
              else d = dmin(d, 0.0);
            } else if (lo < -OSQP_INF * MIN_SCALING) {
              d = dmax(d, 0.0);
            }
            return d;
          };
          const double d = proj(DY, lo03, hi03), d4 = proj(DY4, L4, U4);
          double nd = 0.0, lh = 0.0;
          if (kv) {
            nd = dmax(dabs(Ev * d), dabs(E4 * d4));
            lh = hi03 * dmax(d, 0.0) + lo03 * dmin(d, 0.0);
            if (a == 0) lh += U4 * dmax(d4, 0.0) + L4 * dmin(d4, 0.0);
          }
          const double ndy = bmax<R>(nd, sm.red, slot + 0);
          if (ndy > DIV_TOL) {
            lh = bsum<R>(lh, sm.red, slot + 1);
            if (lh < eps_pinf * ndy) {
              const double atd = quad_at(d, d4, AK0, AK1, AK4, a);
              const double an = bmax<R>(vv ? dabs(DI * atd) : 0.0, sm.red, slot + 2);
              prim_inf = an < eps_pinf * ndy;
            }
          }
        }
        const double eps_dual = eps_abs + eps_rel * (cinv * dmax(dmax(mx[8], mx[10]), mx[12]));
        const bool dual_ok = dua_res < eps_dual;
        if (!dual_ok) {
          // is_dual_infeasible (P~ delta_x = P~x_new - P~x_old)
          const double ndx = bmax<R>(vv ? dabs(Dv * DX) : 0.0, sm.red, slot + 3);
          if (ndx > DIV_TOL) {
            const double qd = bsum<R>(vv ? Qv * DX : 0.0, sm.red, slot + 4);
            if (qd < cost_c * eps_dinf * ndx) {
              const double pd = bmax<R>(vv ? dabs(DI * (PX - PXO)) : 0.0, sm.red, slot + 5);
              if (pd < cost_c * eps_dinf * ndx) {
                const double dp = dpp<QP_PRIM>(DX), dz = dpp<QP_B2>(DX);
                const double v = (1.0 / Ev) * (AK0 * dp + AK1 * dz);
                const double v4 = (1.0 / E4) * (AK4 * dz);
                double viol = 0.0;
                if (kv) {
                  if ((hi03 < OSQP_INF * MIN_SCALING && v > eps_dinf * ndx) ||
                      (lo03 > -OSQP_INF * MIN_SCALING && v < -eps_dinf * ndx))
                    viol = 1.0;
                  if ((U4 < OSQP_INF * MIN_SCALING && v4 > eps_dinf * ndx) ||
                      (L4 > -OSQP_INF * MIN_SCALING && v4 < -eps_dinf * ndx))
                    viol = 1.0;
                }
                viol = bmax<R>(viol, sm.red, slot + 6);
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
          st = check(pass == 1, 14 + 7 * pass);  // slots 14-20 / 21-27: consecutive reductions never share one
          done = st != MPCQP_STATUS_UNSOLVED;
        }
        if (pass == 1 || done || !is_adapt) continue;
        const double pr_n = mx[1] / (dmax(mx[3], mx[5]) + DIV_TOL);
        const double du_n = mx[7] / (dmax(dmax(mx[9], mx[11]), mx[13]) + DIV_TOL);
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
      if (done) break;
      if (refactor) {
        RHO4 = rho4_of(rho);
        RI4 = 1. / RHO4;
        rinv = 1. / rho;
        need_factor = true;
      }
    }
    // ---- next right-hand side: sigma x - q~ + A~'(rho z - y) ----
    // (padding lanes and steps past N compute values nothing reads unmasked)
    const double at = quad_at(rho * Z - Y, RHO4 * Z4 - Y4, AK0, AK1, AK4, a);
    RHS = (sigma * X - Qv) + at;
  }

  if (ws) {  // the solver persists: scaling, scaled data, iterates and rho for the next tick
    if (t == 0) {
      ws[WL::FLAG] = 1.0;
      ws[WL::RHO] = rho;
      ws[WL::C] = cost_c;
      ws[WL::MU] = mu;
    }
    if (vv) {
      ws[WL::D + ci] = Dv;
      ws[WL::QT + ci] = Qv;
      ws[WL::X + ci] = X;
    }
    if (kv) {
      ws[WL::E + ri] = Ev;
      ws[WL::AK + ri] = AK0;
      ws[WL::AK + m + ri] = AK1;
      ws[WL::Z + ri] = Z;
      ws[WL::Y + ri] = Y;
      if (a == 0) {
        ws[WL::E + r4] = E4;
        ws[WL::AK + r4] = 0.0;
        ws[WL::AK + m + r4] = AK4;
        ws[WL::Z + r4] = Z4;
        ws[WL::Y + r4] = Y4;
      }
    }
  }
  // ---- 6. store_solution + unscale + compute_grf extraction (A1RobotControl.cpp:555-561) --------
  const bool has_sol = status != MPCQP_STATUS_PRIMAL_INFEASIBLE &&
                       status != MPCQP_STATUS_PRIMAL_INFEASIBLE_INACCURATE &&
                       status != MPCQP_STATUS_DUAL_INFEASIBLE &&
                       status != MPCQP_STATUS_DUAL_INFEASIBLE_INACCURATE && status != MPCQP_STATUS_NON_CVX;
  const double ob = bsum<R>(vv ? 0.5 * X * PX + Qv * X : 0.0, sm.red, 31);
  const double xs0 = has_sol ? Dv * X : NAN;
  if (solution && vv) solution[(size_t)inst * n + ci] = xs0;
  if (w == 0) {
    // u0 = step 0 = wave 0, DPP row 0 (lanes 0..15); f_i = R^T u0[3i:3i+3], NaN legs skipped
    mpcqp_result* res = results + inst;
    const double u00 = dpp<QP_B0>(xs0), u01 = dpp<QP_B1>(xs0), u02 = dpp<QP_B2>(xs0);
    const double nrm = sqrt(u00 * u00 + u01 * u01 + u02 * u02);
    const bool nanleg = isnan(nrm);
    const unsigned long long nanmask = __ballot(q == 0 && a == 0 && nanleg);
    if (q == 0 && av) {
      double s = 0.0;
      s += sel3(a, Rot[0], Rot[1], Rot[2]) * u00;
      s += sel3(a, Rot[3], Rot[4], Rot[5]) * u01;
      s += sel3(a, Rot[6], Rot[7], Rot[8]) * u02;
      res->u0[3 * leg + a] = xs0;
      res->f_body[3 * leg + a] = nanleg ? 0.0 : s;
    }
    if (t == 0) {
      int legs = 0;
      for (int l = 0; l < 4; ++l) legs |= ((nanmask >> (4 * l)) & 1ull) ? (1 << l) : 0;
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
}

}  // namespace mw

template <int N>
static hipError_t launch_mw(const LaunchArgs& a) {
  hipError_t e = launch_scale_any(a);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL((mw::mw_kernel<N>), dim3(a.batch), dim3(mw::MwCfg<N>::NT), 0, (hipStream_t)a.stream, a.recs,
                     a.batch, a.results, a.solution, a.trace, a.trace_cap, a.wstate, a.work, a.p);
  return hipGetLastError();
}
template <int N>
static hipError_t occupancy_mw(int* blocks) {
  return hipOccupancyMaxActiveBlocksPerMultiprocessor(blocks, mw::mw_kernel<N>, mw::MwCfg<N>::NT, 0);
}

#define MPCQP_MW_FOR_EACH_N(X) \
  X(1) X(2) X(3) X(4) X(5) X(6) X(7) X(8) X(9) X(10) X(11) X(12) X(13) X(14) X(15) X(16) X(17) X(18) X(19) X(20)

hipError_t launch_mw_any(const LaunchArgs& a) {
  switch (a.p.horizon) {
#define CASE(K) \
  case K: return launch_mw<K>(a);
    MPCQP_MW_FOR_EACH_N(CASE)
#undef CASE
    default: return hipErrorInvalidValue;
  }
}
hipError_t occupancy_mw_any(int horizon, int* blocks) {
  switch (horizon) {
#define CASE(K) \
  case K: return occupancy_mw<K>(blocks);
    MPCQP_MW_FOR_EACH_N(CASE)
#undef CASE
    default: return hipErrorInvalidValue;
  }
}

}  // namespace mpcqp
