// mpcqp_wave.hip — one WAVEFRONT per robot: the OSQP 0.6 solve of ConvexMpc's QP with the KKT
// system solved through the problem's state-space (LQR) structure, all of it inside one 64-lane
// wave, so that several robots share a CU (the dense path runs one 5-wave workgroup per CU).
//
// Reference path: A1RobotControl::compute_grf (src/a1_cpp/src/A1RobotControl.cpp:446-562) ->
// ConvexMpc (src/a1_cpp/src/ConvexMpc.cpp:7-245) -> OsqpEigen 0.6.3 / OSQP 0.6 (restated in
// oracle/mpc_oracle.c; the phases below follow it: scale_data, set_rho_vec, update_xz_tilde,
// update_x/z/y, update_info, check_termination, adapt_rho, store_solution).
//
// KKT structure.  OSQP scales P = c D H D, A~ = E A D (scaling.c), so its reduced KKT matrix is
//   K = P~ + sigma I + A~' diag(rho) A~ = D (c B'Q̄B + R') D,
//   R' = c R + D^-1 (sigma I + A~' diag(rho) A~) D^-1     (3x3 block-diagonal per foot),
// H = B'Q̄B + R being ConvexMpc's condensed Hessian (B = B_qp, ConvexMpc.cpp:184-211).
// (c B'Q̄B + R') u = w is the normal equation of an LQR problem with dynamics
// x_{k+1} = A x_k + B_k u_k, x_0 = 0, state cost cQ and input cost R'_k.  The gravity state never
// moves (x_0 = 0, B row 12 = 0), so the state is 12-dimensional.  Factorization (once per rho):
//   P_N = cQ, G_k = R'_k + B_k'P_{k+1}B_k, K_k = G_k^-1 B_k'P_{k+1}A, Acl_k = A - B_k K_k,
//   P_k = cQ + A'P_{k+1}A - (B_k'P_{k+1}A)'K_k.
// Solve (every ADMM iteration), with a_k = K_k'w_k, b_k = G_k^-1 w_k:
//   backward  s_{N-1} = -a_{N-1},  s_k = Acl_k' s_{k+1} - a_k         (chain of 12x12 mat-vecs)
//   parallel  g_k = b_k + G_k^-1 B_k' s_{k+1},  h_k = B_k g_k
//   forward   x_1 = h_0,  x_{k+1} = Acl_k x_k + h_k                   (chain of 12x12 mat-vecs)
//   parallel  u_k = g_k - K_k x_k.
//
// Lane layout.  A wave is 4 DPP rows of 16 lanes.  Horizon step k lives in DPP row GRAY(k & 3) of
// register "round" k >> 2; inside a row, lane 4l+a holds component a (fx, fy, fz; state triplets
// likewise) of leg l, lane 4l+3 is padding for variables.  A 12x12 mat-vec whose matrix row i sits
// in the lane of output i is 12 `v_fmac_f64_dpp ... row_newbcast:c` (input element c broadcast
// from its lane) — four horizon steps at once, one per row.  Consecutive steps sit in rows one bit
// apart, so a chain hands its vector to the next step with one v_permlane16/32_swap per dword.
// The four lanes of a leg hold the foot's constraint rows: friction-pyramid rows 0-3 (one per
// lane) and row 4 (fz bounds, replicated), so every per-foot ADMM operation (A~x, A~'y, the
// projection) is a quad-perm DPP.  No barrier exists anywhere: the workgroup is the wave.
// Arithmetic is binary64 throughout.
#include "mpcqp_schur.h"

// OSQP scale_data inside the Schur-form wave (scale_wave) instead of a scale_kernel launch before it
#ifndef MPCQP_FUSED_SCALE
#define MPCQP_FUSED_SCALE 0
#endif

namespace mpcqp {
namespace wv {

// MPCQP_SCALE_TIMING experiment builds: thread 0 of each robot overwrites the first doubles of its
// own record with {id, s_memtime} pairs (tools/scale_phases.py; the solve that follows is garbage)
#ifdef MPCQP_SCALE_TIMING
#define SC_MARK(id)                                                                     \
  do {                                                                                  \
    if (threadIdx.x == 0) {                                                             \
      double* tm_ = const_cast<double*>(recs) + (size_t)blockIdx.x * Cfg<N>::REC + 2 * (id); \
      tm_[0] = (id);                                                                    \
      tm_[1] = (double)__builtin_readcyclecounter();                                    \
    }                                                                                   \
  } while (0)
#else
#define SC_MARK(id) \
  do {              \
  } while (0)
#endif
template <int N>
__global__ __launch_bounds__(ScaleCfg<N>::NTS, ScaleCfg<N>::WPE) void scale_kernel(const double* __restrict__ recs, int batch,
                                                                 double* __restrict__ wstate,
                                                                 double* __restrict__ img, mpcqp_params p,
                                                                 int* __restrict__ fb) {
  using C = Cfg<N>;
  using SC = ScaleCfg<N>;
  using WL = WarmLayout<N>;
  using SI = ScaleImg<N>;
  constexpr int n = C::n, m = C::m, NTS = SC::NTS;
  static_assert(NTS >= 64 + N, "wave 1 screens one horizon step per lane");
  __shared__ ScaleSmem<N> sm;
  const int inst = blockIdx.x;
  if (inst >= batch) return;
  const int t = threadIdx.x;
#ifdef MPCQP_SCALE_TIMING
  const double t_entry = (double)__builtin_readcyclecounter();
#endif
  // wave_kernel's hand-off counters start at zero (stream order): [0] rank-deficient feet, [1] a KKT
  // solve that cancelled too much for its core (S_max * amp > SCHUR_AMP), [2] S_max > SCHUR_SMAX
  if (inst == 0 && t < 3) fb[t] = 0;
  {
    const double* rg = recs + (size_t)inst * C::REC;
    int bad = 0;
    for (int e = t; e < C::REC; e += NTS) {
      const double v = rg[e];
      sm.rec[e] = v;
      bad |= !isfinite(v);
    }
    if (__syncthreads_or(bad)) return;  // wave_kernel reports the non-finite record
  }
  SC_MARK(0);
#ifdef MPCQP_SCALE_TIMING
  if (t == 0) {  // kernel entry (before the record load), kept until the record's first words are read
    double* tm_ = const_cast<double*>(recs) + (size_t)blockIdx.x * Cfg<N>::REC + 14;
    tm_[0] = 7;
    tm_[1] = t_entry;
  }
#endif
  const double* rec = sm.rec;
  const double dt = rec[MPCQP_REC_DT], mass = rec[MPCQP_REC_MASS], mu = rec[MPCQP_REC_MU];
  Adisc A;
  {
    const double yaw = rec[MPCQP_REC_EULER + 2];
    A.ad0 = cos(yaw) * dt;
    A.ad1 = sin(yaw) * dt;
    A.dt = dt;
  }
  const double dtm = (1.0 / mass) * dt;
  // B_d(k) rows 6-8 (calculate_B_mat_c, Utils.cpp:35-41), gradient adjoint (ConvexMpc.cpp:215-217)
  bool any_degen;
  {
    int degen = 0;
    double Iwinv[9];
    iw_inverse(rec, Iwinv);
    for (int e = t; e < N * 36; e += NTS) {
      const int k = e / 36, rr = (e / 12) % 3, cc = e % 12;
      const int lg = cc / 3, c3 = cc % 3;
      const double* fp = rec + MPCQP_REC_FEET(N) + 12 * k + 3 * lg;
      const double sk0 = c3 == 0 ? 0.0 : c3 == 1 ? -fp[2] : fp[1];
      const double sk1 = c3 == 0 ? fp[2] : c3 == 1 ? 0.0 : -fp[0];
      const double sk2 = c3 == 0 ? -fp[1] : c3 == 1 ? fp[0] : 0.0;
      double s = 0.0;
      s += sel3(rr, Iwinv[0], Iwinv[3], Iwinv[6]) * sk0;
      s += sel3(rr, Iwinv[1], Iwinv[4], Iwinv[7]) * sk1;
      s += sel3(rr, Iwinv[2], Iwinv[5], Iwinv[8]) * sk2;
      sm.Bw[k][rr][cc] = s * dt;
    }
    // forward: a_i = A_d^{i+1} x0 (13 states), e_i = 2q (a_i - x_ref_i); backward: lambda_j = e_j + A' lambda_{j+1}
    // (sequential over the horizon: wave 0 alone, wave-synchronous; one block barrier at the end)
    if (t < 64) {
      if (t < SD) sm.vec[0][t] = rec[MPCQP_REC_X0 + t];
      // 2 q of the lane's state, loaded once (indexed by the lane, it is a memory round trip: inside
      // the sweep it was one per step)
      double q2t = 2 * p.q_weights[t < ND ? t : 0];
      keep(q2t);
      // Branch-free rows of A_d (forward) and A_d' (backward): lane t's row is
      // fma(c2, v[j2], fma(c1, v[j1], v[t])), the unused terms with a zero coefficient (exact: the
      // operands are finite).  Per-lane branches serialized the rows, each with its own LDS wait.
      const int tr = t < SD ? t : 0;
      const int fj1 = tr <= 1 ? 6 : (tr == 2 ? 8 : (tr <= 5 ? tr + 6 : (tr == 11 ? 12 : tr)));
      const double fc1 = tr == 0 ? A.ad0 : (tr == 1 ? -A.ad1 : ((tr <= 5 || tr == 11) ? dt : 0.0));
      const int fj2 = tr <= 1 ? 7 : tr;
      const double fc2 = tr == 0 ? A.ad1 : (tr == 1 ? A.ad0 : 0.0);
      const int bj1 = tr == 6 || tr == 7 ? 0 : (tr == 8 ? 2 : (tr >= 9 && tr < ND ? tr - 6 : tr));
      const double bc1 = tr == 6 ? A.ad0 : (tr == 7 ? A.ad1 : ((tr >= 8 && tr < ND) ? dt : 0.0));
      const int bj2 = tr == 6 || tr == 7 ? 1 : tr;
      const double bc2 = tr == 6 ? -A.ad1 : (tr == 7 ? A.ad0 : 0.0);
      wave_sync();
      for (int i = 0; i < N; ++i) {
        if (t < SD) {
          const double* pv = sm.vec[i & 1];
          const double s = fma(fc2, pv[fj2], fma(fc1, pv[fj1], pv[tr]));
          sm.vec[(i + 1) & 1][t] = s;
          if (t < ND) sm.lam[i][t] = q2t * (s - rec[MPCQP_REC_XREF + SD * i + t]);
        }
        wave_sync();
      }
      for (int j = N - 2; j >= 0; --j) {
        if (t < ND) {
          const double* v = sm.lam[j + 1];
          sm.lam[j][t] = sm.lam[j][t] + fma(bc2, v[bj2], fma(bc1, v[bj1], v[tr]));
        }
        wave_sync();
      }
      SC_MARK(8);
    } else if (N <= 10 && t < 64 + N) {  // (the Schur form serves N <= 10 only: no screen beyond)
      // Degenerate-foot screen for the Schur form (wave_kernel KS = 1), by wave 1 while wave 0 runs
      // the sweep: per step k the Cholesky pivots of the Gram matrix B6_k B6_k' (B6 = rows 6-11 of
      // B_d(k): I_w^-1 [r_l]x dt and dt/m sums) relative to its diagonal.  Collinear feet give rank
      // 5, coincident feet rank 3; a pivot ratio below SCHUR_GRAM_TOL sends the robot to the Riccati
      // form.  (Go1 workloads: smallest ratio ~0.12; with R'^-1 between B6 and B6' (spread <= ~1e3)
      // the Schur form then factors G_k with pivot ratios above ~1e-9.)
      const int k = t - 64;
      double bw[3][ND];
#pragma unroll
      for (int lg = 0; lg < 4; ++lg) {
        const double* fp = rec + MPCQP_REC_FEET(N) + 12 * k + 3 * lg;
#pragma unroll
        for (int rr = 0; rr < 3; ++rr) {  // (I_w^-1 [r]x)[rr][c3] = sum_e Iwinv[rr][e] skew[e][c3]
          const double i0 = Iwinv[3 * rr], i1 = Iwinv[3 * rr + 1], i2 = Iwinv[3 * rr + 2];
          bw[rr][3 * lg + 0] = (i1 * fp[2] - i2 * fp[1]) * dt;
          bw[rr][3 * lg + 1] = (i2 * fp[0] - i0 * fp[2]) * dt;
          bw[rr][3 * lg + 2] = (i0 * fp[1] - i1 * fp[0]) * dt;
        }
      }
      double G[21];  // lower triangle, row-major packed; Cholesky in place
      auto gi = [](int r1, int r2) { return r1 * (r1 + 1) / 2 + r2; };
#pragma unroll
      for (int r1 = 0; r1 < 6; ++r1)
#pragma unroll
        for (int r2 = 0; r2 <= r1; ++r2) {
          double g = 0.0;
          if (r1 < 3) {
#pragma unroll
            for (int b = 0; b < ND; ++b) g += bw[r1][b] * bw[r2][b];
          } else if (r2 < 3) {
#pragma unroll
            for (int l = 0; l < 4; ++l) g += bw[r2][3 * l + (r1 - 3)] * dtm;
          } else {
            g = r1 == r2 ? 4.0 * dtm * dtm : 0.0;
          }
          G[gi(r1, r2)] = g;
        }
#pragma unroll
      for (int c = 0; c < 6; ++c) {
        const double d0 = G[gi(c, c)];
        double sc = d0;
#pragma unroll
        for (int e = 0; e < c; ++e) sc -= G[gi(c, e)] * G[gi(c, e)];
        degen |= !(sc > SCHUR_GRAM_TOL * d0);
        const double dg = sqrt(dmax(sc, 0.0)), di = dg > 0.0 ? 1.0 / dg : 0.0;
        G[gi(c, c)] = dg;
#pragma unroll
        for (int r1 = c + 1; r1 < 6; ++r1) {
          double v = G[gi(r1, c)];
#pragma unroll
          for (int e = 0; e < c; ++e) v -= G[gi(r1, e)] * G[gi(c, e)];
          G[gi(r1, c)] = v * di;
        }
      }
    }
    // (a block-uniform flag: nothing else of the screen stays live through the Ruiz passes)
    any_degen = __syncthreads_or(degen) != 0;
  }
  // thread t: column j0 = t / 4, blocks jb .. jb+BPT-1 of it (the column's four threads are a quad)
  constexpr int BPT = SC::BPT;
  const int j0 = t / SC::TPC, jb = (t % SC::TPC) * BPT;
  SC_MARK(1);
  const bool lead = (t % SC::TPC) == 0;  // the lane that owns the column's per-column values
  // D and E of the current pass (each pass writes the other buffer: no read-before-write barrier)
  double* Dc = sm.D[0];
  double* Ec = sm.E[0];
  if (lead && j0 < n) {
    const int k = j0 / ND, ii = j0 % ND;
    const double* lm = sm.lam[k];
    const double g = ((sm.Bw[k][0][ii] * lm[6] + sm.Bw[k][1][ii] * lm[7]) + sm.Bw[k][2][ii] * lm[8]) + dtm * lm[9 + ii % 3];
    sm.q[j0] = g;
    sm.qn[j0] = g;
    Dc[j0] = 1.0;
  }
  for (int r = t; r < m; r += NTS) {
    Ec[r] = 1.0;
    const int a5 = r % 5;  // friction pyramid rows (ConvexMpc.cpp:46-58)
    sm.Ap[0][r] = a5 < 4 ? 1.0 : 0.0;
    sm.Ap[1][r] = a5 < 4 ? ((a5 & 1) ? -mu : mu) : 1.0;
  }
  __syncthreads();
  double* const ws = wstate ? wstate + (size_t)inst * WL::SIZE : nullptr;
  const bool had = ws && ws[WL::FLAG] != 0.0;
  // max_i D_i |H_ij0| over the thread's blocks, then over the quad (every lane of it gets the norm)
  double hc[SC::HREG ? 12 * BPT : 1];
  auto colmax = [&](bool first) __attribute__((always_inline)) -> double {
    double mx0 = 0.0, mx1 = 0.0;
    if (j0 < n) {
      if constexpr (SC::HREG) {
        if (first)
          gen_col<N, BPT, true>(sm, p, A, dtm, j0, jb, [&](int jj, int b, int, double hv) __attribute__((always_inline)) {
            hc[12 * jj + b] = hv;
          });
        // six independent max chains (a max is exact, so the grouping does not change the result)
        double m6[6] = {0.0, 0.0, 0.0, 0.0, 0.0, 0.0};
#pragma unroll
        for (int jj = 0; jj < BPT; ++jj) {
          const int j = jb + jj;
          if (j < N) {
            const double* dj = Dc + ND * j;
#pragma unroll
            for (int b = 0; b < 12; ++b) m6[b % 6] = fmax(m6[b % 6], dj[b] * dabs(hc[12 * jj + b]));
          }
        }
        mx0 = fmax(fmax(m6[0], m6[2]), m6[4]);
        mx1 = fmax(fmax(m6[1], m6[3]), m6[5]);
      } else {
        gen_col<N, BPT, false>(sm, p, A, dtm, j0, jb, [&](int, int b, int ri, double hv) __attribute__((always_inline)) {
          if (b & 1) mx1 = fmax(mx1, Dc[ri] * dabs(hv));
          else mx0 = fmax(mx0, Dc[ri] * dabs(hv));
        });
      }
    }
    double mx = fmax(mx0, mx1);
    if constexpr (SC::TPC >= 2) mx = fmax(mx, dpp<0xB1>(mx));  // over the column's lanes
    if constexpr (SC::TPC == 4) mx = fmax(mx, dpp<0x4E>(mx));
    return mx;
  };
  // H's zero pattern (sparseView) of column j0's upper triangle vs the previous tick's: decides
  // between osqp_update_P and OsqpEigen's re-init (oracle ws_update)
  auto pattern = [&]() __attribute__((always_inline)) -> bool {
    unsigned long long zm[WL::MW];
#pragma unroll
    for (int w = 0; w < WL::MW; ++w) zm[w] = 0ull;
    auto put = [&](int, int, int ri, double hv) __attribute__((always_inline)) {
      const unsigned long long bit = (hv == 0.0 && ri <= j0) ? (1ull << (ri & 63)) : 0ull;
#pragma unroll
      for (int w = 0; w < WL::MW; ++w) zm[w] |= (ri >> 6) == w ? bit : 0ull;
    };
    if (j0 < n) {
      if constexpr (SC::HREG) {
#pragma unroll
        for (int jj = 0; jj < BPT; ++jj)
#pragma unroll
          for (int b = 0; b < 12; ++b)
            if (jb + jj < N) put(jj, b, ND * (jb + jj) + b, hc[12 * jj + b]);
      } else {
        gen_col<N, BPT, false>(sm, p, A, dtm, j0, jb, put);
      }
    }
    bool diff = false;
#pragma unroll
    for (int w = 0; w < WL::MW; ++w) {  // OR over the column's lanes
      unsigned lo = (unsigned)zm[w], hi = (unsigned)(zm[w] >> 32);
      if constexpr (SC::TPC >= 2) {
        lo |= (unsigned)__builtin_amdgcn_update_dpp(0, (int)lo, 0xB1, 0xF, 0xF, false);
        hi |= (unsigned)__builtin_amdgcn_update_dpp(0, (int)hi, 0xB1, 0xF, 0xF, false);
      }
      if constexpr (SC::TPC == 4) {
        lo |= (unsigned)__builtin_amdgcn_update_dpp(0, (int)lo, 0x4E, 0xF, 0xF, false);
        hi |= (unsigned)__builtin_amdgcn_update_dpp(0, (int)hi, 0x4E, 0xF, 0xF, false);
      }
      zm[w] = ((unsigned long long)hi << 32) | lo;
    }
    if (lead && j0 < n) {
      double* slot = ws + WL::MASK + WL::MW * j0;
#pragma unroll
      for (int w = 0; w < WL::MW; ++w) {
        diff |= __double_as_longlong(slot[w]) != (long long)zm[w];
        slot[w] = __longlong_as_double((long long)zm[w]);
      }
    }
    return diff;
  };
  // A~ column / row norms, branch-free (every operand loaded, the case selected after: per-lane
  // branches ran the cases one after another, each with its own LDS wait)
  auto acol = [&](int j) __attribute__((always_inline)) {
    const int f = j / 3, aa = j % 3;
    const double* e = Ec + 5 * f;
    const double* a0 = sm.Ap[0] + 5 * f;
    const double* a1 = sm.Ap[1] + 5 * f;
    const double e0 = e[0], e1 = e[1], e2 = e[2], e3 = e[3], e4 = e[4];
    const double m0 = dmax(e0 * dabs(a0[0]), e1 * dabs(a0[1]));
    const double m1 = dmax(e2 * dabs(a0[2]), e3 * dabs(a0[3]));
    const double m2 = dmax(dmax(dmax(dmax(dabs(a1[0]) * e0, dabs(a1[1]) * e1), dabs(a1[2]) * e2), dabs(a1[3]) * e3),
                           e4 * dabs(a1[4]));
    return sel3(aa, m0, m1, m2) * Dc[j];
  };
  auto arow = [&](int r) __attribute__((always_inline)) {
    const int f = r / 5, k5 = r % 5;
    const double e = Ec[r];
    const double* d = Dc + 3 * f;
    const double a0r = sm.Ap[0][r], a1r = sm.Ap[1][r], dk = d[k5 < 4 ? k5 >> 1 : 0], d2 = d[2];
    const double m4 = (e * dabs(a1r)) * d2;
    const double m03 = dmax((e * dabs(a0r)) * dk, (dabs(a1r) * e) * d2);
    return k5 == 4 ? m4 : m03;
  };
  double c_s = 1.0, cm = 0.0;
  // First column pass (D = 1): the raw norms, and H's zero pattern (warm start only): same pattern
  // -> osqp_update_P (unscale with the old scaling, rescale with the previous A and q, keep iterates
  // and rho); a changed pattern or mu -> re-init (fresh scaling and rho, the previous unscaled x, y)
  bool pattern_changed = false;
  SC_MARK(2);
  // The raw norms only enter the bound-decided passes below, where an upper bound serves as well
  // (their tests then err on the side of the exact passes): for nonnegative weights H is symmetric
  // positive semidefinite, so max_i |H_ij| <= sqrt(H_jj max_i H_ii), from H's diagonal alone (one
  // block of column j instead of N; the margin covers the roundings of the computed entries).  The
  // first pass, which compares the raw norm itself with |A col j|, takes the bound only when the
  // bound already loses that comparison in every column (checked below; else the exact norms).
  bool cm_ub = true;
#ifndef MPCQP_SCALE_EXACT_CM0
  for (int i = 0; i < ND; ++i) cm_ub = cm_ub && p.q_weights[i] >= 0.0 && p.r_weights[i % MPCQP_NUM_DOF] >= 0.0;
#else
  cm_ub = false;
#endif
  auto colmax_ub = [&]() __attribute__((always_inline)) -> double {
    double hd = 0.0;
    if (lead && j0 < n) {
      const int a2 = j0 % ND;
      gen_col<N, 1, true>(sm, p, A, dtm, j0, j0 / ND, [&](int, int b, int, double hv) __attribute__((always_inline)) {
        hd = b == a2 ? hv : hd;
      });
    }
    double unused = 0.0, hm = hd;
    block_sum_max<SC::NWS>(unused, hm, sm.red);
    return sqrt(dmax(hd, 0.0) * hm) * (1.0 + 0x1p-20);
  };
  if (p.scaling > 0 || ws) {
    cm = cm_ub ? colmax_ub() : colmax(true);
    if (ws) pattern_changed = __syncthreads_or(pattern()) != 0;
  }
  // A is set once per solver init (A1RobotControl.cpp:526-530); a changed mu re-initializes
  const bool mu_changed = had && ws[WL::MU] != mu;
  const int mode = !had ? 0 : ((pattern_changed || mu_changed) ? 2 : 1);  // 0 cold, 1 update_P, 2 re-init
  if (mode == 1) {
    // unscale_data with the previous scaling: q = D^-1 (c^-1 q~), A = (E^-1 A~) D^-1
    const double cinv_o = 1. / ws[WL::C];
    if (lead && j0 < n) sm.q[j0] = (1. / ws[WL::D + j0]) * (cinv_o * ws[WL::QT + j0]);
    for (int r = t; r < m; r += NTS) {
      const int f = r / 5, k5 = r % 5;
      const double ei = 1. / ws[WL::E + r];
      const double d2 = 1. / ws[WL::D + 3 * f + 2];
      sm.Ap[0][r] = k5 < 4 ? (ws[WL::AK + r] * ei) * (1. / ws[WL::D + 3 * f + (k5 >> 1)]) : 0.0;
      sm.Ap[1][r] = (ws[WL::AK + m + r] * ei) * d2;
    }
    __syncthreads();
  }
  SC_MARK(3);
  // Ruiz passes decided by bounds.  A pass uses the column norms cm_j = max_i D_i |H_ij| of the
  // D-scaled P twice: in the cost normalization (c_temp = 1 / max(mean_j c D_j cm_j, |q|_inf)) and
  // in the next pass's fmax(c D_j cm_j, |A~ col j|).  With cm0_j = max_i |H_ij| (the raw pass,
  // D = 1) and Dmax = max_i D_i, fl(D_i |H_ij|) <= fl(Dmax cm0_j) (rounding is monotone); where
  // these bounds, with a margin for the roundings of the sums and products, already let |q|_inf win
  // the normalization and the A~ norm win every column's fmax, the exact norms cannot change a bit
  // of the result.  Such a pass is per-foot work — A is block diagonal over the feet (5 rows x 3
  // columns) — done by one thread per foot in place, plus one block reduction (sum c D_j cm0_j,
  // max |q_j|, max D_j, min_j |A~ col j| / (D_j cm0_j)).  The first pass the bounds cannot decide
  // and all after it run the exact passes below.  (Go1 workloads: every pass of every robot is
  // decided by the bounds, H's entries being far below A's unit entries.)
  if (lead && j0 < n) sm.cm0[j0] = cm;
  __syncthreads();
  if (cm_ub && p.scaling > 0) {
    // the first pass's fmax(c D_j cm_j, |A~ col j| D_j) with c = D_j = E_i = 1: the bound must lose it
    // (then the raw norm, at most the bound, loses it too and the pass is the same)
    bool wins = false;
    if (t < 4 * N) {
      const double* a0 = sm.Ap[0] + 5 * t;
      const double* a1 = sm.Ap[1] + 5 * t;
      const double* cz = sm.cm0 + 3 * t;
      const double m0 = dmax(Ec[5 * t] * dabs(a0[0]), Ec[5 * t + 1] * dabs(a0[1]));
      const double m1 = dmax(Ec[5 * t + 2] * dabs(a0[2]), Ec[5 * t + 3] * dabs(a0[3]));
      const double m2 = dmax(dmax(dmax(dmax(dabs(a1[0]) * Ec[5 * t], dabs(a1[1]) * Ec[5 * t + 1]),
                                       dabs(a1[2]) * Ec[5 * t + 2]), dabs(a1[3]) * Ec[5 * t + 3]),
                             Ec[5 * t + 4] * dabs(a1[4]));
      wins = !(cz[0] <= m0 * Dc[3 * t]) || !(cz[1] <= m1 * Dc[3 * t + 1]) || !(cz[2] <= m2 * Dc[3 * t + 2]);
    }
    if (__syncthreads_or(wins)) {
      cm = colmax(true);
      if (lead && j0 < n) sm.cm0[j0] = cm;
      __syncthreads();
    }
  }
  int pass = 0;
  bool resume = false;  // the bound passes stopped after the D, E, q update of `pass`
  {
    constexpr int NF = 4 * N;
    constexpr double EPS = 2.220446049250313e-16;
    constexpr double M1 = 1.0 + 4.0 * (n + 8) * EPS;  // sum / product margin of the normalization test
    constexpr double M2 = 1.0 + 16.0 * EPS;           // product margin of the fmax test
    double dmax_prev = 1.0;                           // Dmax of the previous pass (ub_j = Dmax cm0_j)
    for (; pass < p.scaling; ++pass) {
      if (pass == 1) SC_MARK(4);
      double s0 = 0.0, qm = 0.0, dm = 0.0, rmin = INFINITY, moved = 0.0;
      if (t < NF) {
        const int f = t;
        double e[5], a0[5], a1[5], d[3], cz[3];
#pragma unroll
        for (int i = 0; i < 5; ++i) {
          e[i] = Ec[5 * f + i];
          a0[i] = sm.Ap[0][5 * f + i];
          a1[i] = sm.Ap[1][5 * f + i];
        }
#pragma unroll
        for (int i = 0; i < 3; ++i) {
          d[i] = Dc[3 * f + i];
          cz[i] = sm.cm0[3 * f + i];
        }
        // |A~ col| of the foot's fx, fy, fz columns without D (acol above, same operations)
        auto acol3 = [&](const double (&ee)[5], double (&mc)[3]) __attribute__((always_inline)) {
          mc[0] = dmax(ee[0] * dabs(a0[0]), ee[1] * dabs(a0[1]));
          mc[1] = dmax(ee[2] * dabs(a0[2]), ee[3] * dabs(a0[3]));
          mc[2] = dmax(dmax(dmax(dmax(dabs(a1[0]) * ee[0], dabs(a1[1]) * ee[1]), dabs(a1[2]) * ee[2]),
                            dabs(a1[3]) * ee[3]),
                       ee[4] * dabs(a1[4]));
        };
        double mc[3];
        acol3(e, mc);
        double dtv[3], et[5];
#pragma unroll
        for (int i = 0; i < 3; ++i) {
          const double cmj = pass == 0 ? cz[i] : dmax_prev * cz[i];
          const double pc = (c_s * d[i]) * cmj;
          dtv[i] = limit_scaling(fmax(pc, mc[i] * d[i]));
        }
#pragma unroll
        for (int i = 0; i < 5; ++i) {  // arow above
          const double dk = d[i < 4 ? i >> 1 : 0], d2 = d[2];
          const double m4 = (e[i] * dabs(a1[i])) * d2;
          const double m03 = dmax((e[i] * dabs(a0[i])) * dk, (dabs(a1[i]) * e[i]) * d2);
          et[i] = limit_scaling(i == 4 ? m4 : m03);
        }
        // 1 / sqrt of the limited norms; 1 / sqrt(1) = 1 exactly, and on the Go1 workloads every
        // norm is 1 (unit friction-pyramid entries, D = E = 1): the wave skips the divisions then
        bool ne1 = false;
#pragma unroll
        for (int i = 0; i < 3; ++i) ne1 |= dtv[i] != 1.0;
#pragma unroll
        for (int i = 0; i < 5; ++i) ne1 |= et[i] != 1.0;
        if (__any(ne1)) {
#pragma unroll
          for (int i = 0; i < 3; ++i) dtv[i] = 1.0 / sqrt(dtv[i]);
#pragma unroll
          for (int i = 0; i < 5; ++i) et[i] = 1.0 / sqrt(et[i]);
        }
        moved = ne1 ? 1.0 : 0.0;
#pragma unroll
        for (int i = 0; i < 5; ++i) {
          e[i] = e[i] * et[i];
          Ec[5 * f + i] = e[i];
        }
#pragma unroll
        for (int i = 0; i < 3; ++i) {
          const double qj = dtv[i] * sm.q[3 * f + i];
          sm.q[3 * f + i] = qj;
          d[i] = d[i] * dtv[i];
          Dc[3 * f + i] = d[i];
          s0 += (c_s * d[i]) * cz[i];
          qm = dmax(qm, dabs(qj));
          dm = dmax(dm, d[i]);
        }
        acol3(e, mc);  // the next pass's A~ norms
#pragma unroll
        for (int i = 0; i < 3; ++i) {
          const double den = d[i] * cz[i];
          rmin = fmin(rmin, den > 0.0 ? (mc[i] * d[i]) / den : INFINITY);
        }
      }
      {  // one block reduction; partials double-buffered by pass parity (no second barrier)
        s0 = wave_sum(s0);
        qm = wave_max(qm);
        dm = wave_max(dm);
        rmin = -wave_max(-rmin);
        moved = wave_max(moved);
        double* pr = sm.red4[pass & 1];
        if ((t & 63) == 0) {
          pr[5 * (t >> 6) + 0] = s0;
          pr[5 * (t >> 6) + 1] = qm;
          pr[5 * (t >> 6) + 2] = dm;
          pr[5 * (t >> 6) + 3] = rmin;
          pr[5 * (t >> 6) + 4] = moved;
        }
        __syncthreads();
        s0 = pr[0];
        qm = pr[1];
        dm = pr[2];
        rmin = pr[3];
        moved = pr[4];
#pragma unroll
        for (int w = 1; w < SC::NWS; ++w) {
          s0 += pr[5 * w];
          qm = dmax(qm, pr[5 * w + 1]);
          dm = dmax(dm, pr[5 * w + 2]);
          rmin = fmin(rmin, pr[5 * w + 3]);
          moved = dmax(moved, pr[5 * w + 4]);
        }
      }
      const double inf_norm_q = limit_scaling(qm);
      const double c_temp = 1. / limit_scaling(inf_norm_q);
      const double c_new = c_s * c_temp;
      const bool ok1 = ((dm * s0) * M1) / n <= inf_norm_q;
      const bool ok2 = pass + 1 == p.scaling || (c_new * dm) * M2 <= rmin;
      if (!(ok1 && ok2)) {  // (block-uniform)
        resume = true;
        break;
      }
      if (t < NF) {
#pragma unroll
        for (int i = 0; i < 3; ++i) sm.q[3 * t + i] *= c_temp;
      }
      // A pass that moved nothing (every 1/sqrt factor 1, c_temp 1, the same Dmax) leaves the next
      // pass exactly the same inputs: every remaining pass is the identity.  (Go1 workloads: from
      // the second or third pass on.)
      const bool fixed = moved == 0.0 && c_temp == 1.0 && dm == dmax_prev;
      c_s = c_new;
      dmax_prev = dm;
      if (fixed) {
        pass = p.scaling;
        break;
      }
    }
  }
  // exact passes: H's columns regenerated for the norms
  for (; pass < p.scaling; ++pass) {
    if (!resume) {
      if (pass == 1) SC_MARK(4);
      // new scaling factors from the current D, E (every thread reads before anyone writes)
      double dtv = 1.0;
      if (lead && j0 < n) {
        const double pc = (c_s * Dc[j0]) * cm;
        dtv = 1.0 / sqrt(limit_scaling(fmax(pc, acol(j0))));
      }
      double et[SC::RPT];
#pragma unroll
      for (int rr = 0; rr < SC::RPT; ++rr) {
        const int r = t + NTS * rr;
        et[rr] = r < m ? 1.0 / sqrt(limit_scaling(arow(r))) : 1.0;
      }
      double* const Dn = Dc == sm.D[0] ? sm.D[1] : sm.D[0];
      double* const En = Ec == sm.E[0] ? sm.E[1] : sm.E[0];
#pragma unroll
      for (int rr = 0; rr < SC::RPT; ++rr) {
        const int r = t + NTS * rr;
        if (r < m) En[r] = Ec[r] * et[rr];
      }
      if (lead && j0 < n) {
        sm.q[j0] = dtv * sm.q[j0];
        Dn[j0] = Dc[j0] * dtv;
      }
      Dc = Dn;
      Ec = En;
    }
    resume = false;
    __syncthreads();
    cm = colmax(false);  // column norms of the D-scaled P (cost normalization)
    double sv = 0.0, qv = 0.0;
    if (lead && j0 < n) {
      sv = (c_s * Dc[j0]) * cm;
      qv = dabs(sm.q[j0]);
    }
    block_sum_max<SC::NWS>(sv, qv, sm.red);
    double c_temp = sv / n;
    const double inf_norm_q = limit_scaling(qv);
    c_temp = dmax(c_temp, inf_norm_q);
    c_temp = limit_scaling(c_temp);
    c_temp = 1. / c_temp;
    if (lead && j0 < n) sm.q[j0] *= c_temp;  // own column only: no barrier before the next pass
    c_s *= c_temp;
  }
  __syncthreads();
  SC_MARK(5);
  double* out = img + (size_t)inst * SI::SIZE;
  // (the A entries the passes used are not handed over: wave_kernel derives them from mu or the
  // warm slot as above; this tick's raw gradient only matters to osqp_update_P, i.e. warm slots)
  if (lead && j0 < n) {
    out[SI::D + j0] = Dc[j0];
    out[SI::Q + j0] = sm.q[j0];
    if (ws) out[SI::QN + j0] = sm.qn[j0];
  }
  for (int r = t; r < m; r += NTS) out[SI::E + r] = Ec[r];
  // The Schur form's hand-off flag: 1 for rank-deficient B6_k (the screen above).  (Evaluating max
  // S_ii at the initial rho here as well was measured and dropped: at rho = 0.1 no C5 or heavy-weight
  // robot crosses SCHUR_SMAX -- with OSQP's cost scaling S barely grows with the state weights; the
  // crossings come after adapt_rho lowers rho -- and it cost scale_kernel 11 %, profiles/r05.)
  const double flag = any_degen ? 1.0 : 0.0;
  if (t == 0) {
    out[SI::CS] = c_s;
    out[SI::MODE] = (double)mode;
    out[SI::DEGEN] = flag;
  }
  SC_MARK(6);
}
#undef SC_MARK

// ---- OSQP scale_data inside the robot's own wave (fused setup, N <= 10) ---------------------------
// scale_kernel's computation on the 64 lanes of the Schur-form wave instead of a separate two-wave
// launch: lane t owns columns t and t + 64 of P~ (CPT slots) and rows t + 64 r of A~; the gradient
// sweeps run on lanes 0-12, then the degenerate-feet screen on lanes 16 .. 16 + N - 1.  Every value is
// computed by the same expressions, and the two block reductions of the exact passes add the two
// column slots' wave sums in scale_kernel's wave order, so the image is bitwise scale_kernel's
// (tests/test_gpu_fused.py).  The image is still written for the checks' D / E reloads and for a
// Riccati hand-off; the setup's copies (D, q~, the raw gradient, E) are left in the LDS image.
struct FusedScale {
  double c_s;
  int mode;
  bool degen;
};
template <int N>
__device__ __forceinline__ FusedScale scale_wave(WSmem<N, 1>& sm, const mpcqp_params& p, double* __restrict__ wstate,
                                                 int inst, const Adisc& A, double dtm, double mu,
                                                 double* __restrict__ out) {
  using C = Cfg<N>;
  using WL = WarmLayout<N>;
  using SI = ScaleImg<N>;
  constexpr int n = C::n, m = C::m, CPT = (n + 63) / 64, RPT = (m + 63) / 64, BPT = N;
  auto& H = sm.u.h;
  const int t = threadIdx.x;
  const double* rec = H.rec;
  const double dt = A.dt;
  // -- gradient sweeps (scale_kernel wave 0) and the Gram screen (scale_kernel wave 1) --
  double Iwinv[9];
  iw_inverse(rec, Iwinv);
  {
    if (t < SD) H.vec[0][t] = rec[MPCQP_REC_X0 + t];
    double q2t = 2 * p.q_weights[t < ND ? t : 0];
    keep(q2t);
    const int tr = t < SD ? t : 0;
    const int fj1 = tr <= 1 ? 6 : (tr == 2 ? 8 : (tr <= 5 ? tr + 6 : (tr == 11 ? 12 : tr)));
    const double fc1 = tr == 0 ? A.ad0 : (tr == 1 ? -A.ad1 : ((tr <= 5 || tr == 11) ? dt : 0.0));
    const int fj2 = tr <= 1 ? 7 : tr;
    const double fc2 = tr == 0 ? A.ad1 : (tr == 1 ? A.ad0 : 0.0);
    const int bj1 = tr == 6 || tr == 7 ? 0 : (tr == 8 ? 2 : (tr >= 9 && tr < ND ? tr - 6 : tr));
    const double bc1 = tr == 6 ? A.ad0 : (tr == 7 ? A.ad1 : ((tr >= 8 && tr < ND) ? dt : 0.0));
    const int bj2 = tr == 6 || tr == 7 ? 1 : tr;
    const double bc2 = tr == 6 ? -A.ad1 : (tr == 7 ? A.ad0 : 0.0);
    wave_sync();
    for (int i = 0; i < N; ++i) {
      if (t < SD) {
        const double* pv = H.vec[i & 1];
        const double sv = fma(fc2, pv[fj2], fma(fc1, pv[fj1], pv[tr]));
        H.vec[(i + 1) & 1][t] = sv;
        if (t < ND) H.lam[i][t] = q2t * (sv - rec[MPCQP_REC_XREF + SD * i + t]);
      }
      wave_sync();
    }
    for (int j = N - 2; j >= 0; --j) {
      if (t < ND) {
        const double* v = H.lam[j + 1];
        H.lam[j][t] = H.lam[j][t] + fma(bc2, v[bj2], fma(bc1, v[bj1], v[tr]));
      }
      wave_sync();
    }
  }
  bool any_degen;
  {
    int degen = 0;
    if (t >= 16 && t < 16 + N) {
      const int k = t - 16;
      double bw[3][ND];
#pragma unroll
      for (int lg = 0; lg < 4; ++lg) {
        const double* fp = rec + MPCQP_REC_FEET(N) + 12 * k + 3 * lg;
#pragma unroll
        for (int rr = 0; rr < 3; ++rr) {
          const double i0 = Iwinv[3 * rr], i1 = Iwinv[3 * rr + 1], i2 = Iwinv[3 * rr + 2];
          bw[rr][3 * lg + 0] = (i1 * fp[2] - i2 * fp[1]) * dt;
          bw[rr][3 * lg + 1] = (i2 * fp[0] - i0 * fp[2]) * dt;
          bw[rr][3 * lg + 2] = (i0 * fp[1] - i1 * fp[0]) * dt;
        }
      }
      double G[21];
      auto gi = [](int r1, int r2) { return r1 * (r1 + 1) / 2 + r2; };
#pragma unroll
      for (int r1 = 0; r1 < 6; ++r1)
#pragma unroll
        for (int r2 = 0; r2 <= r1; ++r2) {
          double g = 0.0;
          if (r1 < 3) {
#pragma unroll
            for (int b = 0; b < ND; ++b) g += bw[r1][b] * bw[r2][b];
          } else if (r2 < 3) {
#pragma unroll
            for (int l = 0; l < 4; ++l) g += bw[r2][3 * l + (r1 - 3)] * dtm;
          } else {
            g = r1 == r2 ? 4.0 * dtm * dtm : 0.0;
          }
          G[gi(r1, r2)] = g;
        }
#pragma unroll
      for (int c = 0; c < 6; ++c) {
        const double d0 = G[gi(c, c)];
        double sc = d0;
#pragma unroll
        for (int e = 0; e < c; ++e) sc -= G[gi(c, e)] * G[gi(c, e)];
        degen |= !(sc > SCHUR_GRAM_TOL * d0);
        const double dg = sqrt(dmax(sc, 0.0)), di = dg > 0.0 ? 1.0 / dg : 0.0;
        G[gi(c, c)] = dg;
#pragma unroll
        for (int r1 = c + 1; r1 < 6; ++r1) {
          double v = G[gi(r1, c)];
#pragma unroll
          for (int e = 0; e < c; ++e) v -= G[gi(r1, e)] * G[gi(c, e)];
          G[gi(r1, c)] = v * di;
        }
      }
    }
    any_degen = __any(degen) != 0;
  }
  // -- columns (CPT slots per lane) and rows: gradient, D = E = 1, the friction pyramid --
  double* Dc = H.D;
  double* Ec = H.E;
#pragma unroll
  for (int c = 0; c < CPT; ++c) {
    const int j0 = t + 64 * c;
    if (j0 < n) {
      const int k = j0 / ND, ii = j0 % ND;
      const double* lm = H.lam[k];
      const double g = ((sm.Bw[k][0][ii] * lm[6] + sm.Bw[k][1][ii] * lm[7]) + sm.Bw[k][2][ii] * lm[8]) + dtm * lm[9 + ii % 3];
      H.q[j0] = g;
      H.qn[j0] = g;
      Dc[j0] = 1.0;
    }
  }
  for (int r = t; r < m; r += 64) {
    Ec[r] = 1.0;
    const int a5 = r % 5;  // friction pyramid rows (ConvexMpc.cpp:46-58)
    H.Ap[0][r] = a5 < 4 ? 1.0 : 0.0;
    H.Ap[1][r] = a5 < 4 ? ((a5 & 1) ? -mu : mu) : 1.0;
  }
  wave_sync();
  double* const ws = wstate ? wstate + (size_t)inst * WL::SIZE : nullptr;
  const bool had = ws && ws[WL::FLAG] != 0.0;
  auto colmax1 = [&](int j0, bool first) __attribute__((always_inline)) -> double {
    (void)first;
    double mx0 = 0.0, mx1 = 0.0;
    if (j0 < n)
      gen_col<N, BPT, false>(sm, p, A, dtm, j0, 0, [&](int, int b, int ri, double hv) __attribute__((always_inline)) {
        if (b & 1) mx1 = fmax(mx1, Dc[ri] * dabs(hv));
        else mx0 = fmax(mx0, Dc[ri] * dabs(hv));
      });
    return fmax(mx0, mx1);
  };
  auto pattern1 = [&](int j0) __attribute__((always_inline)) -> bool {
    unsigned long long zm[WL::MW];
#pragma unroll
    for (int w = 0; w < WL::MW; ++w) zm[w] = 0ull;
    auto put = [&](int, int, int ri, double hv) __attribute__((always_inline)) {
      const unsigned long long bit = (hv == 0.0 && ri <= j0) ? (1ull << (ri & 63)) : 0ull;
#pragma unroll
      for (int w = 0; w < WL::MW; ++w) zm[w] |= (ri >> 6) == w ? bit : 0ull;
    };
    bool diff = false;
    if (j0 < n) {
      gen_col<N, BPT, false>(sm, p, A, dtm, j0, 0, put);
      double* slot = ws + WL::MASK + WL::MW * j0;
#pragma unroll
      for (int w = 0; w < WL::MW; ++w) {
        diff |= __double_as_longlong(slot[w]) != (long long)zm[w];
        slot[w] = __longlong_as_double((long long)zm[w]);
      }
    }
    return diff;
  };
  auto acol = [&](int j) __attribute__((always_inline)) {
    const int f = j / 3, aa = j % 3;
    const double* e = Ec + 5 * f;
    const double* a0 = H.Ap[0] + 5 * f;
    const double* a1 = H.Ap[1] + 5 * f;
    const double e0 = e[0], e1 = e[1], e2 = e[2], e3 = e[3], e4 = e[4];
    const double m0 = dmax(e0 * dabs(a0[0]), e1 * dabs(a0[1]));
    const double m1 = dmax(e2 * dabs(a0[2]), e3 * dabs(a0[3]));
    const double m2 = dmax(dmax(dmax(dmax(dabs(a1[0]) * e0, dabs(a1[1]) * e1), dabs(a1[2]) * e2), dabs(a1[3]) * e3),
                           e4 * dabs(a1[4]));
    return sel3(aa, m0, m1, m2) * Dc[j];
  };
  auto arow = [&](int r) __attribute__((always_inline)) {
    const int f = r / 5, k5 = r % 5;
    const double e = Ec[r];
    const double* d = Dc + 3 * f;
    const double a0r = H.Ap[0][r], a1r = H.Ap[1][r], dk = d[k5 < 4 ? k5 >> 1 : 0], d2 = d[2];
    const double m4 = (e * dabs(a1r)) * d2;
    const double m03 = dmax((e * dabs(a0r)) * dk, (dabs(a1r) * e) * d2);
    return k5 == 4 ? m4 : m03;
  };
  double c_s = 1.0, cm[CPT];
#pragma unroll
  for (int c = 0; c < CPT; ++c) cm[c] = 0.0;
  bool pattern_changed = false;
  bool cm_ub = true;
#ifndef MPCQP_SCALE_EXACT_CM0
  for (int i = 0; i < ND; ++i) cm_ub = cm_ub && p.q_weights[i] >= 0.0 && p.r_weights[i % MPCQP_NUM_DOF] >= 0.0;
#else
  cm_ub = false;
#endif
  if (p.scaling > 0 || ws) {
    if (cm_ub) {  // colmax_ub: max_i |H_ij| <= sqrt(H_jj max_i H_ii)
      double hd[CPT], hm = 0.0;
#pragma unroll
      for (int c = 0; c < CPT; ++c) {
        const int j0 = t + 64 * c;
        hd[c] = 0.0;
        if (j0 < n) {
          const int a2 = j0 % ND;
          double h = 0.0;
          gen_col<N, 1, true>(sm, p, A, dtm, j0, j0 / ND, [&](int, int b, int, double hv) __attribute__((always_inline)) {
            h = b == a2 ? hv : h;
          });
          hd[c] = h;
        }
        hm = fmax(hm, hd[c]);
      }
      hm = wave_max(hm);
#pragma unroll
      for (int c = 0; c < CPT; ++c) cm[c] = sqrt(dmax(hd[c], 0.0) * hm) * (1.0 + 0x1p-20);
    } else {
#pragma unroll
      for (int c = 0; c < CPT; ++c) cm[c] = colmax1(t + 64 * c, true);
    }
    if (ws) {
      bool d = false;
#pragma unroll
      for (int c = 0; c < CPT; ++c) d |= pattern1(t + 64 * c);
      pattern_changed = __any(d) != 0;
    }
  }
  const bool mu_changed = had && ws[WL::MU] != mu;
  const int mode = !had ? 0 : ((pattern_changed || mu_changed) ? 2 : 1);
  if (mode == 1) {
    const double cinv_o = 1. / ws[WL::C];
#pragma unroll
    for (int c = 0; c < CPT; ++c) {
      const int j0 = t + 64 * c;
      if (j0 < n) H.q[j0] = (1. / ws[WL::D + j0]) * (cinv_o * ws[WL::QT + j0]);
    }
    for (int r = t; r < m; r += 64) {
      const int f = r / 5, k5 = r % 5;
      const double ei = 1. / ws[WL::E + r];
      const double d2 = 1. / ws[WL::D + 3 * f + 2];
      H.Ap[0][r] = k5 < 4 ? (ws[WL::AK + r] * ei) * (1. / ws[WL::D + 3 * f + (k5 >> 1)]) : 0.0;
      H.Ap[1][r] = (ws[WL::AK + m + r] * ei) * d2;
    }
    wave_sync();
  }
#pragma unroll
  for (int c = 0; c < CPT; ++c) {
    const int j0 = t + 64 * c;
    if (j0 < n) H.cm0[j0] = cm[c];
  }
  wave_sync();
  if (cm_ub && p.scaling > 0) {
    bool wins = false;
    if (t < 4 * N) {
      const double* a0 = H.Ap[0] + 5 * t;
      const double* a1 = H.Ap[1] + 5 * t;
      const double* cz = H.cm0 + 3 * t;
      const double m0 = dmax(Ec[5 * t] * dabs(a0[0]), Ec[5 * t + 1] * dabs(a0[1]));
      const double m1 = dmax(Ec[5 * t + 2] * dabs(a0[2]), Ec[5 * t + 3] * dabs(a0[3]));
      const double m2 = dmax(dmax(dmax(dmax(dabs(a1[0]) * Ec[5 * t], dabs(a1[1]) * Ec[5 * t + 1]),
                                       dabs(a1[2]) * Ec[5 * t + 2]), dabs(a1[3]) * Ec[5 * t + 3]),
                             Ec[5 * t + 4] * dabs(a1[4]));
      wins = !(cz[0] <= m0 * Dc[3 * t]) || !(cz[1] <= m1 * Dc[3 * t + 1]) || !(cz[2] <= m2 * Dc[3 * t + 2]);
    }
    if (__any(wins)) {
#pragma unroll
      for (int c = 0; c < CPT; ++c) {
        const int j0 = t + 64 * c;
        cm[c] = colmax1(j0, true);
        if (j0 < n) H.cm0[j0] = cm[c];
      }
      wave_sync();
    }
  }
  int pass = 0;
  bool resume = false;
  {
    constexpr int NF = 4 * N;
    constexpr double EPS = 2.220446049250313e-16;
    constexpr double M1 = 1.0 + 4.0 * (n + 8) * EPS;
    constexpr double M2 = 1.0 + 16.0 * EPS;
    double dmax_prev = 1.0;
    for (; pass < p.scaling; ++pass) {
      double s0 = 0.0, qm = 0.0, dm = 0.0, rmin = INFINITY, moved = 0.0;
      if (t < NF) {
        const int f = t;
        double e[5], a0[5], a1[5], d[3], cz[3];
#pragma unroll
        for (int i = 0; i < 5; ++i) {
          e[i] = Ec[5 * f + i];
          a0[i] = H.Ap[0][5 * f + i];
          a1[i] = H.Ap[1][5 * f + i];
        }
#pragma unroll
        for (int i = 0; i < 3; ++i) {
          d[i] = Dc[3 * f + i];
          cz[i] = H.cm0[3 * f + i];
        }
        auto acol3 = [&](const double (&ee)[5], double (&mc)[3]) __attribute__((always_inline)) {
          mc[0] = dmax(ee[0] * dabs(a0[0]), ee[1] * dabs(a0[1]));
          mc[1] = dmax(ee[2] * dabs(a0[2]), ee[3] * dabs(a0[3]));
          mc[2] = dmax(dmax(dmax(dmax(dabs(a1[0]) * ee[0], dabs(a1[1]) * ee[1]), dabs(a1[2]) * ee[2]),
                            dabs(a1[3]) * ee[3]),
                       ee[4] * dabs(a1[4]));
        };
        double mc[3];
        acol3(e, mc);
        double dtv[3], et[5];
#pragma unroll
        for (int i = 0; i < 3; ++i) {
          const double cmj = pass == 0 ? cz[i] : dmax_prev * cz[i];
          const double pc = (c_s * d[i]) * cmj;
          dtv[i] = limit_scaling(fmax(pc, mc[i] * d[i]));
        }
#pragma unroll
        for (int i = 0; i < 5; ++i) {
          const double dk = d[i < 4 ? i >> 1 : 0], d2 = d[2];
          const double m4 = (e[i] * dabs(a1[i])) * d2;
          const double m03 = dmax((e[i] * dabs(a0[i])) * dk, (dabs(a1[i]) * e[i]) * d2);
          et[i] = limit_scaling(i == 4 ? m4 : m03);
        }
        bool ne1 = false;
#pragma unroll
        for (int i = 0; i < 3; ++i) ne1 |= dtv[i] != 1.0;
#pragma unroll
        for (int i = 0; i < 5; ++i) ne1 |= et[i] != 1.0;
        if (__any(ne1)) {
#pragma unroll
          for (int i = 0; i < 3; ++i) dtv[i] = 1.0 / sqrt(dtv[i]);
#pragma unroll
          for (int i = 0; i < 5; ++i) et[i] = 1.0 / sqrt(et[i]);
        }
        moved = ne1 ? 1.0 : 0.0;
#pragma unroll
        for (int i = 0; i < 5; ++i) {
          e[i] = e[i] * et[i];
          Ec[5 * f + i] = e[i];
        }
#pragma unroll
        for (int i = 0; i < 3; ++i) {
          const double qj = dtv[i] * H.q[3 * f + i];
          H.q[3 * f + i] = qj;
          d[i] = d[i] * dtv[i];
          Dc[3 * f + i] = d[i];
          s0 += (c_s * d[i]) * cz[i];
          qm = dmax(qm, dabs(qj));
          dm = dmax(dm, d[i]);
        }
        acol3(e, mc);
#pragma unroll
        for (int i = 0; i < 3; ++i) {
          const double den = d[i] * cz[i];
          rmin = fmin(rmin, den > 0.0 ? (mc[i] * d[i]) / den : INFINITY);
        }
      }
      // (scale_kernel: the same wave reductions, then + the second wave's partials, all neutral: its
      // lanes hold no foot)
      s0 = wave_sum(s0) + 0.0;
      qm = dmax(wave_max(qm), 0.0);
      dm = dmax(wave_max(dm), 0.0);
      rmin = fmin(-wave_max(-rmin), INFINITY);
      moved = dmax(wave_max(moved), 0.0);
      wave_sync();
      const double inf_norm_q = limit_scaling(qm);
      const double c_temp = 1. / limit_scaling(inf_norm_q);
      const double c_new = c_s * c_temp;
      const bool ok1 = ((dm * s0) * M1) / n <= inf_norm_q;
      const bool ok2 = pass + 1 == p.scaling || (c_new * dm) * M2 <= rmin;
      if (!(ok1 && ok2)) {
        resume = true;
        break;
      }
      if (t < NF) {
#pragma unroll
        for (int i = 0; i < 3; ++i) H.q[3 * t + i] *= c_temp;
      }
      const bool fixed = moved == 0.0 && c_temp == 1.0 && dm == dmax_prev;
      c_s = c_new;
      dmax_prev = dm;
      if (fixed) {
        pass = p.scaling;
        break;
      }
    }
  }
  // exact passes: H's columns regenerated for the norms
  for (; pass < p.scaling; ++pass) {
    if (!resume) {
      double dtv[CPT];
#pragma unroll
      for (int c = 0; c < CPT; ++c) {
        const int j0 = t + 64 * c;
        dtv[c] = 1.0;
        if (j0 < n) {
          const double pc = (c_s * Dc[j0]) * cm[c];
          dtv[c] = 1.0 / sqrt(limit_scaling(fmax(pc, acol(j0))));
        }
      }
      double et[RPT];
#pragma unroll
      for (int rr = 0; rr < RPT; ++rr) {
        const int r = t + 64 * rr;
        et[rr] = r < m ? 1.0 / sqrt(limit_scaling(arow(r))) : 1.0;
      }
      double* const Dn = Dc == H.D ? H.Dx : H.D;
      double* const En = Ec == H.E ? H.Ex : H.E;
#pragma unroll
      for (int rr = 0; rr < RPT; ++rr) {
        const int r = t + 64 * rr;
        if (r < m) En[r] = Ec[r] * et[rr];
      }
#pragma unroll
      for (int c = 0; c < CPT; ++c) {
        const int j0 = t + 64 * c;
        if (j0 < n) {
          H.q[j0] = dtv[c] * H.q[j0];
          Dn[j0] = Dc[j0] * dtv[c];
        }
      }
      Dc = Dn;
      Ec = En;
    }
    resume = false;
    wave_sync();
    // cost normalization: the column slots' wave sums added in scale_kernel's wave order
    double sv = 0.0, qv = 0.0;
#pragma unroll
    for (int c = 0; c < CPT; ++c) {
      const int j0 = t + 64 * c;
      cm[c] = colmax1(j0, false);
      const double svc = j0 < n ? (c_s * Dc[j0]) * cm[c] : 0.0;
      sv = c == 0 ? wave_sum(svc) : sv + wave_sum(svc);
      qv = fmax(qv, j0 < n ? dabs(H.q[j0]) : 0.0);
    }
    if (CPT == 1) sv = sv + 0.0;  // (scale_kernel adds its second wave's zero partial)
    qv = wave_max(qv);
    double c_temp = sv / n;
    const double inf_norm_q = limit_scaling(qv);
    c_temp = dmax(c_temp, inf_norm_q);
    c_temp = limit_scaling(c_temp);
    c_temp = 1. / c_temp;
#pragma unroll
    for (int c = 0; c < CPT; ++c) {
      const int j0 = t + 64 * c;
      if (j0 < n) H.q[j0] *= c_temp;
    }
    c_s *= c_temp;
  }
  wave_sync();
  // the image (the checks reload D and E from it; a Riccati hand-off reads all of it) and, in the
  // setup image, the final D and E (the passes may have left them in the second buffers)
#pragma unroll
  for (int c = 0; c < CPT; ++c) {
    const int j0 = t + 64 * c;
    if (j0 < n) {
      const double dj = Dc[j0];
      out[SI::D + j0] = dj;
      out[SI::Q + j0] = H.q[j0];
      if (ws) out[SI::QN + j0] = H.qn[j0];
      H.D[j0] = dj;
    }
  }
  for (int r = t; r < m; r += 64) {
    const double er = Ec[r];
    out[SI::E + r] = er;
    H.E[r] = er;
  }
  if (t == 0) {
    out[SI::CS] = c_s;
    out[SI::MODE] = (double)mode;
    out[SI::DEGEN] = any_degen ? 1.0 : 0.0;
  }
  wave_sync();
  return FusedScale{c_s, mode, any_degen};
}

// Phase timing (debug builds with -DMPCQP_PHASE_TIMING): lane 0 of each traced robot appends
// {phase id, s_memtime, s_memrealtime (100 MHz), 0} to the trace buffer instead of check records.
#ifdef MPCQP_PHASE_TIMING
// MPCQP_PHASE_TIMING_ENDS: only the first and last marks (0, 20), with the wave's HW_ID register in
// the fourth word, for per-robot durations and the dispatch timeline at no cost to the solve itself
#ifdef MPCQP_PHASE_TIMING_ENDS
#define WV_MARK_ON(id) ((id) == 0 || (id) == 20)
// HW_ID (hwreg 4: wave, SIMD, CU, SE fields) + 2^32 XCC_ID (hwreg 20)
#define WV_HWID()                                                          \
  ((double)(unsigned)__builtin_amdgcn_s_getreg(4 | (0 << 6) | (31 << 11)) + \
   4294967296.0 * (double)(unsigned)__builtin_amdgcn_s_getreg(20 | (0 << 6) | (3 << 11)))
#else
#define WV_MARK_ON(id) true
#define WV_HWID() 0.0
#endif
#define WV_MARK(id) WV_MARK_AT(id, -1)
// cyc >= 0: a cycle count taken earlier (marks recorded in registers inside straight-line code)
#define WV_MARK_AT(id, cyc)                                                             \
  do {                                                                                  \
    if (WV_MARK_ON(id) && trace && threadIdx.x == 0 && inst < trace_cap && nmark < MPCQP_TRACE_LEN) { \
      double* tm_ = trace + ((size_t)inst * MPCQP_TRACE_LEN + nmark) * 4;                \
      tm_[0] = (id);                                                                    \
      tm_[1] = (cyc) >= 0 ? (double)(cyc) : (double)__builtin_readcyclecounter();       \
      tm_[2] = (double)__builtin_amdgcn_s_memrealtime();                                \
      tm_[3] = WV_HWID();                                                               \
      ++nmark;                                                                          \
    }                                                                                   \
  } while (0)
#elif defined(MPCQP_ISA_MARKS)
// static ISA accounting (tools/isa_phases.py): an assembly comment per phase mark
#define WV_MARK(id) asm volatile(";WV_MARK %0" ::"n"(id))
// (the Gauss-Jordan's internal marks are recorded after the fact only in timing builds: never here)
#define WV_MARK_AT(id, cyc) \
  do {                      \
    (void)(cyc);            \
    WV_MARK(id);            \
  } while (0)
#else
#define WV_MARK(id) \
  do {              \
  } while (0)
#define WV_MARK_AT(id, cyc) \
  do {                      \
  } while (0)
#endif

// KS: the KKT solve.  0 = Riccati recursion (chains over the horizon, factors on MFMA; every N),
// 1 = impulse-space Schur form (mpcqp_schur.h; N <= 10, nonnegative state weights).
// The solve of robot `inst` by one wave (wave_kernel: one robot per workgroup).  Returns true when a
// KS = 1 solve hands the robot to the Riccati form without having written anything: scale_kernel
// flagged it (rank-deficient B6_k), or a factorization's max S_ii crossed SCHUR_SMAX; wave_kernel
// then solves it with KS = 0 in the same wave.  fb[0] and fb[2] count the two cases.
// FUSED (KS = 1): OSQP scale_data runs in this wave (scale_wave) instead of scale_kernel's launch
template <int N, int KS, bool FUSED = false>
__device__ __forceinline__ bool wave_solve(const int inst, WSmem<N, KS>& sm, const double* __restrict__ recs,
                                           mpcqp_result* __restrict__ results, double* __restrict__ solution,
                                           double* __restrict__ trace, int trace_cap, double* __restrict__ wstate,
                                           double* __restrict__ img, const mpcqp_params& p,
                                           int* __restrict__ fb) {
  using C = Cfg<N>;
  using WL = WarmLayout<N>;
  constexpr int n = C::n, m = C::m, R = C::R;
  const int t = threadIdx.x;
  const int q = t >> 4, li = t & 15, leg = li >> 2, a = li & 3;
  const bool av = a < 3;
  const int idx = 3 * leg + (av ? a : 2);  // index inside a step (padding lanes alias component 2)
  const int ig = gray(q);                  // this lane's step in round r is 4r + ig
  const double alpha = p.alpha, sigma = p.sigma;
  int nmark = 0;
  (void)nmark;
  WV_MARK(0);

  // ---- 0. record -> LDS, non-finite guard -------------------------------------------------------
  auto& HS = sm.u.h;
  {
    const double* rg = recs + (size_t)inst * C::REC;
    bool bad = false;
    for (int e = t; e < C::REC; e += NT) {
      const double v = rg[e];
      HS.rec[e] = v;
      bad |= !isfinite(v);
    }
    if (__ballot(bad) != 0) {
      if (t == 0) {
        mpcqp_result r;
        for (int k = 0; k < ND; ++k) { r.u0[k] = NAN; r.f_body[k] = 0.0; }
        r.obj_val = NAN; r.pri_res = NAN; r.dua_res = NAN; r.rho = p.rho;
        r.status = MPCQP_STATUS_NAN_INPUT; r.iters = 0; r.rho_updates = 0; r.nan_legs = 0xF;
        results[inst] = r;
      }
      if (solution)
        for (int e = t; e < n; e += NT) solution[(size_t)inst * n + e] = NAN;
      return false;
    }
  }
  wave_sync();
  WV_MARK(1);
  const double* rec = HS.rec;
  // (record values used after the setup image is recycled are plain register copies: every LDS
  // store of the union aliases them under -fno-strict-aliasing, so no reload can be hoisted past
  // the factorization's stores — see DESIGN §5, "LDS unions and aliasing")
  const double dt = rec[MPCQP_REC_DT], mass = rec[MPCQP_REC_MASS], mu_rec = rec[MPCQP_REC_MU];
  Adisc A;
  {
    const double yaw = rec[MPCQP_REC_EULER + 2];
    A.ad0 = cos(yaw) * dt;
    A.ad1 = sin(yaw) * dt;
    A.dt = dt;
  }
  const double dtm = (1.0 / mass) * dt;
  // what the solve needs from the record after the setup image is recycled (root_rot_mat is read
  // again from HBM by the epilogue)
  const double cont = rec[MPCQP_REC_CONTACTS + leg] != 0.0 ? 1.0 : 0.0;
  const double fzmin = rec[MPCQP_REC_FZMIN], fzmax = rec[MPCQP_REC_FZMAX];

  // ---- 1. B_d(k) rows 6-8 (calculate_B_mat_c, Utils.cpp:35-41), gradient adjoint --------------------
  {
    double Iwinv[9];
    iw_inverse(rec, Iwinv);
    for (int e = t; e < N * 36; e += NT) {
      const int k = e / 36, rr = (e / 12) % 3, cc = e % 12;
      const int lg = cc / 3, c3 = cc % 3;
      const double* fp = rec + MPCQP_REC_FEET(N) + 12 * k + 3 * lg;
      const double sk0 = c3 == 0 ? 0.0 : c3 == 1 ? -fp[2] : fp[1];
      const double sk1 = c3 == 0 ? fp[2] : c3 == 1 ? 0.0 : -fp[0];
      const double sk2 = c3 == 0 ? -fp[1] : c3 == 1 ? fp[0] : 0.0;
      double s = 0.0;
      s += sel3(rr, Iwinv[0], Iwinv[3], Iwinv[6]) * sk0;
      s += sel3(rr, Iwinv[1], Iwinv[4], Iwinv[7]) * sk1;
      s += sel3(rr, Iwinv[2], Iwinv[5], Iwinv[8]) * sk2;
      sm.Bw[k][rr][cc] = s * dt;
    }
  }
  WV_MARK(2);

  WV_MARK(3);

  // ---- 3. OSQP scale_data: computed here by the robot's wave (fused setup, Schur form), or the image
  // scale_kernel wrote (D, E, q~, c, branch; raw q if warm) ---------------------------------------
  using SI = ScaleImg<N>;
  // (not const: the Schur form records max S_ii of its latest factorization in the DEGEN slot)
  double* const im = img + (size_t)inst * SI::SIZE;
  double c_s;
  int mode;  // 0 cold, 1 osqp_update_P, 2 OsqpEigen re-init
  bool degen_feet = false;
  if constexpr (KS == 1 && FUSED) {
    const FusedScale fs = scale_wave<N>(sm, p, wstate, inst, A, dtm, mu_rec, im);
    c_s = fs.c_s;
    mode = fs.mode;
    degen_feet = fs.degen;  // (D, q~, the raw gradient and E are in the setup image already)
  } else {
    c_s = im[SI::CS];
    mode = (int)im[SI::MODE];
    if (KS == 1) degen_feet = im[SI::DEGEN] != 0.0;
  }
  if (KS == 1 && degen_feet) {
    // rank-deficient B6_k (collinear / coincident feet: G_k would be singular; the reference QP is
    // still strictly convex, R > 0): the Riccati form (KS = 0) solves this robot.  Nothing of it
    // has been written yet (the fused setup wrote the image the Riccati form reads).
    if (t == 0) atomicAdd(fb, 1);
    return true;
  }
  if (!(KS == 1 && FUSED)) {
    for (int j = t; j < n; j += NT) {
      HS.D[j] = im[SI::D + j];
      HS.q[j] = im[SI::Q + j];
      if (mode != 0) HS.qn[j] = im[SI::QN + j];
    }
    for (int r = t; r < m; r += NT) HS.E[r] = im[SI::E + r];
  }
  // Warm start (A1RobotControl.h:67 member solver, :522-538): the slot of the previous tick.
  double* const ws = wstate ? wstate + (size_t)inst * WL::SIZE : nullptr;
  // The unscaled constraint entries of row ri (ConvexMpc.cpp:46-58), as scale_kernel used them:
  // [0] on fx (rows 0, 1) / fy (rows 2, 3), [1] on fz.  Set once per solver init (friction pyramid
  // of this tick's mu); osqp_update_P keeps the previous A: unscale_data of the previous A~ with the
  // previous scaling (the same expressions as scale_kernel's, so the same bits).
  auto ap_of = [&](int ri, int which) __attribute__((always_inline)) -> double {
    const int f = ri / 5, k5 = ri % 5;
    if (mode == 1) {
      const double ei = 1. / ws[WL::E + ri];
      if (which == 0) return k5 < 4 ? (ws[WL::AK + ri] * ei) * (1. / ws[WL::D + 3 * f + (k5 >> 1)]) : 0.0;
      return (ws[WL::AK + m + ri] * ei) * (1. / ws[WL::D + 3 * f + 2]);
    }
    if (which == 0) return k5 < 4 ? 1.0 : 0.0;
    return k5 < 4 ? ((k5 & 1) ? -mu_rec : mu_rec) : 1.0;
  };
  wave_sync();
  const double cost_c = c_s, cinv = 1. / c_s;
  WV_MARK(4);

  // ---- 4. lane registers: variables (D, q~) and rows (E, A~, bounds, rho) — set_rho_vec -----------
  // update_P keeps the adapted rho (settings->rho); setup and re-init start from the settings'
  const double rho0 = mode == 1 ? ws[WL::RHO] : dmin(dmax(p.rho, RHO_MIN), RHO_MAX);
  // Dv, Ev, E4 are setup-only arrays: the loop reads D and E from the image again when it needs
  // them (factorizations, termination checks, the epilogue) instead of holding them in registers
  double X[R], Qv[R], Dv[R], DI[R], PX[R], RHS[R];
  double Z[R], Y[R], Ev[R], AK0[R], AK1[R];
  double Z4[R], Y4[R], E4[R], L4[R], U4[R], AK4[R], RHO4[R];
  bool kvr[R], vvr[R];
#pragma unroll
  for (int r = 0; r < R; ++r) {
    const int k = 4 * r + ig;
    const bool kv = k < N, vv = kv && av;
    kvr[r] = kv;
    vvr[r] = vv;
    const int kc = kv ? k : 0;
    const int ci = ND * kc + idx, ri = CD * kc + 5 * leg + a, r4 = CD * kc + 5 * leg + 4;
    const int cf = ND * kc + 3 * leg;  // the leg's three variables
    Dv[r] = vv ? HS.D[ci] : 1.0;
    DI[r] = 1. / Dv[r];
    // warm ticks end with osqp_update_lin_cost (A1RobotControl.cpp:533, after updateHessianMatrix's
    // update_P or re-init): q~ = c (D q) of this tick's gradient; a cold setup scales q pass by pass
    Qv[r] = vv ? (mode != 0 ? (HS.qn[ci] * Dv[r]) * c_s : HS.q[ci]) : 0.0;
    Ev[r] = kv ? HS.E[ri] : 1.0;
    E4[r] = kv ? HS.E[r4] : 1.0;
    // A~ = E A D: row a < 4 has A on fx (a < 2) / fy (a >= 2) and on fz; row 4 on fz
    AK0[r] = kv ? (ap_of(ri, 0) * Ev[r]) * HS.D[cf + (a >> 1)] : 0.0;
    AK1[r] = kv ? (ap_of(ri, 1) * Ev[r]) * HS.D[cf + 2] : 0.0;
    AK4[r] = kv ? (ap_of(r4, 1) * E4[r]) * HS.D[cf + 2] : 0.0;
    // bounds (ConvexMpc.cpp:223-245), clipped to +-OSQP_INFTY, scaled by E
    double l4 = fzmin * cont, u4 = fzmax * cont;
    l4 = dmin(dmax(l4, -OSQP_INF), OSQP_INF);
    u4 = dmin(dmax(u4, -OSQP_INF), OSQP_INF);
    L4[r] = E4[r] * l4;
    U4[r] = E4[r] * u4;
    X[r] = 0.0; PX[r] = 0.0;
    Z[r] = 0.0; Y[r] = 0.0; Z4[r] = 0.0; Y4[r] = 0.0;
    RHS[r] = vv ? sigma * 0.0 - Qv[r] : 0.0;  // cold start: compute_rhs with x = z = y = 0
    if (mode == 1) {  // warm start: the previous scaled iterates as they are
      X[r] = vv ? ws[WL::X + ci] : 0.0;
      Z[r] = kv ? ws[WL::Z + ri] : 0.0;
      Y[r] = kv ? ws[WL::Y + ri] : 0.0;
      Z4[r] = kv ? ws[WL::Z + r4] : 0.0;
      Y4[r] = kv ? ws[WL::Y + r4] : 0.0;
    } else if (mode == 2) {  // re-init: x = D^-1 (D_old x_old), y = c E^-1 ((E_old y_old) c_old^-1)
      const double cinv_o = 1. / ws[WL::C];
      X[r] = vv ? DI[r] * (ws[WL::D + ci] * ws[WL::X + ci]) : 0.0;
      Y[r] = kv ? c_s * ((1. / Ev[r]) * ((ws[WL::E + ri] * ws[WL::Y + ri]) * cinv_o)) : 0.0;
      Y4[r] = kv ? c_s * ((1. / E4[r]) * ((ws[WL::E + r4] * ws[WL::Y + r4]) * cinv_o)) : 0.0;
    }
  }
  if (mode == 2) {  // z = A~ x
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const double xp = dpp<QP_PRIM>(X[r]), xz = dpp<QP_B2>(X[r]);
      Z[r] = AK0[r] * xp + AK1[r] * xz;
      Z4[r] = AK4[r] * xz;
    }
  }
  auto rho4_of = [&](double l4, double u4, double rho) __attribute__((always_inline)) {
    const bool loose = l4 < -OSQP_INF * MIN_SCALING && u4 > OSQP_INF * MIN_SCALING;
    const bool eq = u4 - l4 < RHO_TOL;
    return loose ? RHO_MIN : (eq ? RHO_EQ_OVER_RHO_INEQ * rho : rho);
  };
  double RI4[R];  // 1 / rho of row 4 (OSQP rho_inv_vec), refreshed with rho
#pragma unroll
  for (int r = 0; r < R; ++r) {
    RHO4[r] = rho4_of(L4[r], U4[r], rho0);
    RI4[r] = 1. / RHO4[r];
  }
  if (mode != 0) {
#pragma unroll
    for (int r = 0; r < R; ++r) {
      // compute_rhs from the warm x, z, y: sigma x - q~ + A~'(rho z - y)
      const double at = quad_at(rho0 * Z[r] - Y[r], RHO4[r] * Z4[r] - Y4[r], AK0[r], AK1[r], AK4[r], a);
      RHS[r] = vvr[r] ? (sigma * X[r] - Qv[r]) + at : 0.0;
    }
  }
  // Row 4 of every foot (the fz bounds row; its values are the same on the foot's four lanes) packed
  // four register rounds to a register: lane a of a foot's quad holds round 4p + a's value in P[p].
  // The ADMM update projects row 4 once per packed register instead of once per round, and the loop
  // carries 7 NP doubles for it instead of 7 R (NP = 1 at N <= 12): fewer registers for the
  // allocator to park in AGPRs.  unpack(P, r) is round r's value on all four lanes (a quad
  // broadcast), bitwise the value the per-round arrays held.
  constexpr int NP = (R + 3) / 4;
  auto unpack = [&](const double (&P)[NP], int r) __attribute__((always_inline)) -> double {
    const double v = P[r >> 2];
    switch (r & 3) {
      case 0: return dpp<QP_B0>(v);
      case 1: return dpp<QP_B1>(v);
      case 2: return dpp<QP_B2>(v);
      default: return dpp<QP_B3>(v);
    }
  };
  auto pack_of = [&](auto get, int pr) __attribute__((always_inline)) -> double {
    const int r0 = 4 * pr, rl = R - 1;
    const double v0 = get(r0 < rl ? r0 : rl), v1 = get(r0 + 1 < rl ? r0 + 1 : rl);
    const double v2 = get(r0 + 2 < rl ? r0 + 2 : rl), v3 = get(r0 + 3 < rl ? r0 + 3 : rl);
    return a == 0 ? v0 : (a == 1 ? v1 : (a == 2 ? v2 : v3));
  };
  // (the setup's operands through a register copy: a select among loads of one local array is
  // otherwise folded into one load at a per-lane address, which keeps the array in scratch memory)
  auto reg = [](double v) __attribute__((always_inline)) {
    asm("" : "+v"(v));
    return v;
  };
  double Z4P[NP], Y4P[NP], L4P[NP], U4P[NP], AK4P[NP], RHO4P[NP], RI4P[NP];
#pragma unroll
  for (int pr = 0; pr < NP; ++pr) {
    Z4P[pr] = pack_of([&](int r) { return reg(Z4[r]); }, pr);
    Y4P[pr] = pack_of([&](int r) { return reg(Y4[r]); }, pr);
    L4P[pr] = pack_of([&](int r) { return reg(L4[r]); }, pr);
    U4P[pr] = pack_of([&](int r) { return reg(U4[r]); }, pr);
    AK4P[pr] = pack_of([&](int r) { return reg(AK4[r]); }, pr);
    RHO4P[pr] = pack_of([&](int r) { return reg(RHO4[r]); }, pr);
    RI4P[pr] = pack_of([&](int r) { return reg(RI4[r]); }, pr);
  }
  if (KS == 0 && mode != 0) {
    // P~x of the warm iterate (the Riccati variant carries P~x through the KKT identity from here):
    // P~x = c D H (D x), H v = B_qp' Q B_qp v + R v by the dynamics: x_{i+1} = A x_i + B_i v_i
    // from x_0 = 0, e_i = Q x_{i+1}, lambda_j = e_j + A' lambda_{j+1}, (H v)_j = B_j' lambda_j + R v_j.
#pragma unroll
    for (int r = 0; r < R; ++r)
      if (vvr[r]) HS.Dt[ND * (4 * r + ig) + idx] = Dv[r] * X[r];
    if (t < 16) HS.vec[0][t] = 0.0;
    wave_sync();
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
        HS.lam[i][t] = 2 * lane_pick(p.q_weights, t) * xn;
      }
      wave_sync();
    }
    for (int j = N - 2; j >= 0; --j) {
      if (t < ND) HS.lam[j][t] = HS.lam[j][t] + A.atv(t, HS.lam[j + 1]);
      wave_sync();
    }
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const int k = vvr[r] ? 4 * r + ig : 0;
      const double* lm = HS.lam[k];
      const double hv = (((sm.Bw[k][0][idx] * lm[6] + sm.Bw[k][1][idx] * lm[7]) + sm.Bw[k][2][idx] * lm[8]) +
                         dtm * lm[9 + idx % 3]) + (2 * lane_pick(p.r_weights, idx)) * HS.Dt[ND * k + idx];
      PX[r] = vvr[r] ? (c_s * Dv[r]) * hv : 0.0;
    }
  }
  // D and E of the lane's variable / rows, reloaded from the image where they are needed (the
  // factorizations, the checks, the epilogue) instead of being held in loop-carried registers: the
  // element offset goes through an opaque copy, so the loads are neither hoisted out of the loop
  // nor merged across uses.  Plain loads, not volatile ones (each volatile load was followed by its
  // own wait for the memory round trip); unconditional, at a clamped step, the padding value
  // selected after (a load under the lane mask became a branch with its own wait).  A
  // global-address-space pointer: global_load, not flat_load, whose lgkmcnt share would also wait
  // on the LDS traffic in flight.
  using gd = const __attribute__((address_space(1))) double;
  gd* const imv = (gd*)im;
  auto img_at = [&](int e) __attribute__((always_inline)) -> double {
    asm volatile("" : "+v"(e));
    return imv[e];
  };
  auto dv_of = [&](int r) __attribute__((always_inline)) {
    const double v = img_at(SI::D + ND * min(4 * r + ig, N - 1) + idx);
    return vvr[r] ? v : 1.0;
  };
  auto ev_of = [&](int r) __attribute__((always_inline)) {
    const double v = img_at(SI::E + CD * min(4 * r + ig, N - 1) + 5 * leg + a);
    return kvr[r] ? v : 1.0;
  };
  auto e4_of = [&](int r) __attribute__((always_inline)) {
    const double v = img_at(SI::E + CD * min(4 * r + ig, N - 1) + 5 * leg + 4);
    return kvr[r] ? v : 1.0;
  };
  // rows 0-3: l = 0 / u = +inf (rows 0, 2) or l = -inf / u = 0 (rows 1, 3): always inequalities
  auto lo03 = [&](double ev) __attribute__((always_inline)) { return (a & 1) ? ev * -OSQP_INF : ev * 0.0; };
  // the projection onto those bounds needs no E: [0, +inf) for rows 0, 2, (-inf, 0] for rows 1, 3
  // (equal to clamping at E * -+OSQP_INF for every operand below 1e30 E in magnitude)
  const double LO03 = (a & 1) ? -INFINITY : 0.0, HI03 = (a & 1) ? 0.0 : INFINITY;
  auto hi03 = [&](double ev) __attribute__((always_inline)) { return (a & 1) ? ev * 0.0 : ev * OSQP_INF; };
  wave_sync();  // every LDS read of the setup image precedes its reuse by the factorization

  // ---- 5. ADMM (osqp_solve) ------------------------------------------------------------------------
  auto& F = sm.u.f;
  // per-lane weights, selected once (lane_pick: a per-lane index into the kernel parameters is a
  // scratch copy and a memory round trip): 2 r of the lane's variable component, 2 q_(6+c) of its
  // impulse component (KS = 1)
  double R2I = 2.0 * lane_pick(p.r_weights, idx), Q2C = 2.0 * lane_pick(p.q_weights, 6 + (t < 6 * N ? t : 0) % 6);
  keep(R2I);
  keep(Q2C);
  // KS = 0: 2 q_j of the MFMA column j = lane & 15 (factorize_mfma's cQ diagonal)
  double Q2J = KS == 0 ? 2.0 * lane_pick(p.q_weights, li < ND ? li : 0) : 0.0;
  keep(Q2J);
  // KS = 0 without stored Acl: the lane's coefficients of A' on states 0-5 (lane of state i: A[s][i])
  // and of A on states 6-11 (A[i][6 + s]), the off-diagonal part of the discrete A
  constexpr bool NOACL = KS == 0 && !WSmem<N, KS>::SACL;
  double CAT[NOACL ? 6 : 1], CAX[NOACL ? 6 : 1];
  if constexpr (NOACL) {
    const int si = 3 * leg + (a < 3 ? a : 0);  // the lane's state (a = 3: padding)
    const bool sv = a < 3;
#pragma unroll
    for (int e = 0; e < 6; ++e) {
      CAT[e] = sv && si >= 6 ? A.at(e, si) : 0.0;
      CAX[e] = sv && si < 6 ? A.at(si, 6 + e) : 0.0;
    }
  }
  // the LDS address of element c of the lane's row of the packed G_k^-1 in round 0 (step ig)
  unsigned GADR[NOACL ? 12 : 1];
  if constexpr (NOACL) {
    const unsigned gb = lds_off(&sm.u.f.Gp[0][0]) + (unsigned)(sizeof(double) * GPS * ig);
#pragma unroll
    for (int e = 0; e < 12; ++e)
      GADR[e] = gb + (unsigned)sizeof(double) * (unsigned)(e >= idx ? poff(idx) + e - idx : poff(e) + idx - e);
  }
  (void)GADR;
  (void)CAT;
  (void)CAX;
  // KS = 1: the lane's rows of R'^-1 (mpcqp_schur.h), set per rho
  double SRI[KS == 1 ? R : 1][3];
  (void)SRI;
  // KS = 1: P~v computed directly where the checks need it (mpcqp_schur.h schur_px)
  auto px_of = [&](const double (&v)[R], const double (&dd)[R], double (&out)[R]) __attribute__((always_inline)) {
    if constexpr (KS == 1) {
      double dvv[R];
#pragma unroll
      for (int r = 0; r < R; ++r) dvv[r] = dd[r] * v[r];
      schur_px<N, R>(sm, F, p, A, dtm, cost_c, Q2C, R2I, dvv, dd, vvr, out);
    }
  };
  double rho = rho0, rinv = 1. / rho0, pri_res = 0.0, dua_res = 0.0;
  int status = MPCQP_STATUS_UNSOLVED, iters = 0, rho_updates = 0, ntrace = 0;
  double obj_sum = 0.0;  // 1/2 x'P~x + q~'x of the final iterate (scaled), set when the loop ends
  bool need_factor = true;
  int to_check = p.check_termination, to_adapt = p.adaptive_rho_interval;
  bool amp_bad = false;  // the Schur form's cancellation bound was crossed at the last check
  for (int iter = 1; iter <= p.max_iter; ++iter) {
    if (need_factor) {
#ifdef MPCQP_REPEAT_FACTOR  // cost measurement builds: the (idempotent) factorization runs twice
     for (int rep = 0; rep < 2; ++rep) {
#endif
      WV_MARK(10);
      // R'_k foot blocks: c 2r + D^-1 (sigma I + A~' diag(rho) A~) D^-1
#pragma unroll
      for (int r = 0; r < R; ++r) {
        const double k00 = dpp<QP_B0>(AK0[r]), k01 = dpp<QP_B1>(AK0[r]), k02 = dpp<QP_B2>(AK0[r]),
                     k03 = dpp<QP_B3>(AK0[r]);
        const double k10 = dpp<QP_B0>(AK1[r]), k11 = dpp<QP_B1>(AK1[r]), k12 = dpp<QP_B2>(AK1[r]),
                     k13 = dpp<QP_B3>(AK1[r]);
        // D^-1 of the foot's three variables from the lanes' own 1 / D (the same correctly rounded
        // quotients: no reload of D, no division here)
        const double dir = DI[r];
        const double i0 = dpp<QP_B0>(dir), i1 = dpp<QP_B1>(dir), i2 = dpp<QP_B2>(dir);
        const double ak4 = unpack(AK4P, r), r4 = unpack(RHO4P, r);
        // rows of the foot: r0 [k00,0,k10] r1 [k01,0,k11] r2 [0,k02,k12] r3 [0,k03,k13] r4 [0,0,ak4]
        auto coef = [&](int row, int col) __attribute__((always_inline)) {
          if (row == 4) return col == 2 ? ak4 : 0.0;
          const double kp = row == 0 ? k00 : row == 1 ? k01 : row == 2 ? k02 : k03;
          const double kz = row == 0 ? k10 : row == 1 ? k11 : row == 2 ? k12 : k13;
          if (col == 2) return kz;
          return (col == (row >> 1)) ? kp : 0.0;
        };
        const int k = 4 * r + ig;
        const double ia = a == 0 ? i0 : (a == 1 ? i1 : i2);
#pragma unroll
        for (int b = 0; b < 3; ++b) {
          double s = 0.0;
#pragma unroll
          for (int row = 0; row < 5; ++row) s += (coef(row, av ? a : 2) * (row == 4 ? r4 : rho)) * coef(row, b);
          const double ib = b == 0 ? i0 : (b == 1 ? i1 : i2);
          const double rt = (av && a == b ? cost_c * R2I : 0.0) + (ia * ((av && a == b ? sigma : 0.0) + s)) * ib;
          if (kvr[r] && av && b >= a) {
            if constexpr (KS == 0) F.rt(k)[6 * leg + sym6(a, b)] = rt;
            else F.s.Rt[k][leg][sym6(a, b)] = rt;
          }
        }
      }
      wave_sync();
      if constexpr (KS == 0) factorize_mfma<N>(sm, p, A, cost_c, dtm, Q2J);
      else {
        double smax;
        schur_factor<N, R>(sm, F, p, A, cost_c, dtm, SRI,
                           [&](int id, long long cyc = -1) __attribute__((always_inline)) {
                             WV_MARK_AT(id, cyc);
                             (void)id;
                             (void)cyc;
                           },
                           smax);
        // The push-through identity subtracts B'(I - S^-1)B w from R'^-1 w: with S ill-conditioned
        // (large state weights, four feet in contact) the difference loses digits the Riccati form
        // keeps.  Such a robot leaves the loop at the next need_info iteration (one follows every
        // factorization before the next one; an exit right here cost 8 % of the kernel in register
        // allocation) and is handed to the Riccati form (wave_kernel: the same wave), which solves
        // it from the start; nothing of it has been written.  max S_ii of the latest factorization
        // lives in the robot's image slot, not in a loop-carried register.
        if (t == 0) im[SI::DEGEN] = smax;
      }
      wave_sync();
#ifdef MPCQP_REPEAT_FACTOR
     }
#endif
      need_factor = false;
      WV_MARK(12);
    }

    // ---- KKT solve: u = (c B'Q̄B + R')^-1 D^-1 rhs, x~ = D^-1 u ----
    double U[R];
    double amp = 1.0;  // the Schur form's cancellation at the update_info iteration (schur_solve)
    auto kkt = [&](auto INFO) __attribute__((always_inline)) {
    const bool tm_it = iter == 60;
    if (tm_it) WV_MARK(40);
    if constexpr (KS == 1) {
      double W[R];
#pragma unroll
      for (int r = 0; r < R; ++r) W[r] = DI[r] * RHS[r];
      schur_solve<N, R, decltype(INFO)::value>(F, W, SRI, vvr, U, amp);
#ifdef MPCQP_REPEAT_SOLVE  // cost measurement builds: the (idempotent) KKT solve runs twice
      {
        double W2[R];
#pragma unroll
        for (int r = 0; r < R; ++r) W2[r] = W[r] + 0.0 * U[r];  // after the first solve
        schur_solve<N, R>(F, W2, SRI, vvr, U, amp);
      }
#endif
    } else if constexpr (NOACL) {
      // Riccati form without Acl (sigma_k = -s_k):
      //   backward  t_k = w_k - B_k' sigma_{k+1},  sigma_k = K_k' t_k + A' sigma_{k+1}  (sigma_N = 0)
      //   parallel  g_k = G_k^-1 t_k
      //   forward   u_k = g_k - K_k x_k,  x_{k+1} = A x_k + B_k u_k                    (x_0 = 0)
      // (the same recursion: s_k = Acl_k' s_{k+1} - K_k' w_k, x_{k+1} = Acl_k x_k + B_k g_k)
      double W[R], TT[R], G[R];
      int kc[R], kk[R];
#pragma unroll
      for (int r = 0; r < R; ++r) {
        W[r] = DI[r] * RHS[r];
        TT[r] = 0.0;
        U[r] = 0.0;
        kc[r] = min(4 * r + ig, N - 1);
        kk[r] = max(kc[r] - 1, 0);  // slot of K_k (k >= 1)
      }
      if (tm_it) WV_MARK(41);
      {  // backward chain; a round's K_k columns (rows of K_k') serve its four steps, one per row
        double kn[12], kcur[12], bcur[6];
        ldcol(kn, &F.K[kk[(N - 1) >> 2]][idx]);
        double cur = 0.0;
        sfor<0, N>([&](auto J) {
          constexpr int k = N - 1 - decltype(J)::value;
          constexpr int r = k >> 2;
          if constexpr (k == N - 1 || (k & 3) == 3) {  // entering round r (descending)
            lds_wait<0>(kn);
#pragma unroll
            for (int e = 0; e < 12; ++e) kcur[e] = kn[e];
            if constexpr (r >= 1) ldcol(kn, &F.K[kk[r - 1]][idx]);
            bcur[0] = -sm.Bw[kc[r]][0][idx];
            bcur[1] = -sm.Bw[kc[r]][1][idx];
            bcur[2] = -sm.Bw[kc[r]][2][idx];
            bcur[3] = a == 0 ? -dtm : 0.0;
            bcur[4] = a == 1 ? -dtm : 0.0;
            bcur[5] = a == 2 ? -dtm : 0.0;
          }
          __builtin_amdgcn_sched_barrier(0);
#ifndef MPCQP_CHAIN_SPLIT
          if constexpr (k >= 1 && k < N - 1) {  // a middle step: one block (chain_bwd)
            const double m = rmove2<row_of(k + 1), row_of(k)>(cur);
            double tk = W[r], sn = m;
            chain_bwd(m, bcur, CAT, kcur, tk, sn);
            TT[r] = (q == row_of(k)) ? tk : TT[r];
            cur = sn;
            return;
          }
#endif
          double m = 0.0, tk = W[r];
          if constexpr (k < N - 1) {
            m = rmove2<row_of(k + 1), row_of(k)>(cur);
            tk = mv6a(m, bcur, W[r]);
          }
          TT[r] = (q == row_of(k)) ? tk : TT[r];
          if constexpr (k >= 1) {
            const double as = k < N - 1 ? mv6lo_a(m, CAT, m) : 0.0;
            cur = mv12a(tk, kcur, as);
          }
        });
      }
      if (tm_it) WV_MARK(42);
      // g_k = G_k^-1 t_k: row idx of the packed upper triangle, element c at (min, max) of (idx, c);
      // per-lane LDS addresses (constant) plus the round's compile-time offset
      {
        using lds_d = __attribute__((address_space(3))) const double;
        double c0[12], c1[12];
        auto ldg = [&](int r, double (&c)[12]) __attribute__((always_inline)) {
#pragma unroll
          for (int e = 0; e < 12; ++e)
            c[e] = *(lds_d*)(GADR[e] + (unsigned)(sizeof(double) * GPS * 4 * r));
        };
        ldg(0, c0);
        sfor<0, R>([&](auto RR) {
          constexpr int r = decltype(RR)::value;
          if constexpr (r + 1 < R) ldg(r + 1, (r & 1) ? c0 : c1);
          G[r] = mv12(TT[r], (r & 1) ? c1 : c0);
        });
      }
      if (tm_it) WV_MARK(43);
      {  // forward chain; a round's K_k rows and B_w rows serve its four steps
        double kn[12], kcur[12], bn[12], bcu[12];
        ld12(kn, &F.K[kk[0]][mo(idx)]);
        ld12(bn, &sm.Bw[kc[0]][av ? a : 2][0]);
        double cur = 0.0;
        sfor<0, N>([&](auto K) {
          constexpr int k = decltype(K)::value;
          constexpr int r = k >> 2;
          if constexpr ((k & 3) == 0) {  // entering round r (ascending)
#pragma unroll
            for (int e = 0; e < 12; ++e) {
              kcur[e] = kn[e];
              bcu[e] = bn[e];
            }
            if constexpr (r + 1 < R) {
              ld12(kn, &F.K[kk[r + 1]][mo(idx)]);
              ld12(bn, &sm.Bw[kc[r + 1]][av ? a : 2][0]);
            }
          }
          __builtin_amdgcn_sched_barrier(0);
#ifndef MPCQP_CHAIN_SPLIT
          if constexpr (k >= 1 && k <= N - 2) {  // a middle step: one block (chain_fwd)
            const double m = rmove2<row_of(k - 1), row_of(k)>(cur);
            double nu = -G[r], ax = m, hb = 0.0;
            chain_fwd(m, kcur, CAX, bcu, nu, ax, hb);
            U[r] = (q == row_of(k)) ? -nu : U[r];
            const double ls = dtm * legsum(nu);
            const double bnu = leg == 2 ? hb : (leg == 3 ? ls : 0.0);
            cur = ax - bnu;
            return;
          }
#endif
          double m = 0.0, nu = -G[r];  // nu = -u_k = K_k x_k - g_k
          if constexpr (k >= 1) {
            m = rmove2<row_of(k - 1), row_of(k)>(cur);
            nu = mv12a(m, kcur, -G[r]);
          }
          U[r] = (q == row_of(k)) ? -nu : U[r];
          if constexpr (k <= N - 2) {
            // B_k nu: rows 6-8 (leg-2 lanes) B_w nu, rows 9-11 (leg-3 lanes) dt/m times the legs' sum
            const double hb = mv12(nu, bcu);
            const double ls = dtm * legsum(nu);
            const double bnu = leg == 2 ? hb : (leg == 3 ? ls : 0.0);
            const double ax = k >= 1 ? mv6a(m, CAX, m) : 0.0;  // A x_k
            cur = ax - bnu;
          }
        });
      }
      if (tm_it) WV_MARK(44);
    } else {
      // LDS operands are loaded one phase ahead of their use; sched_barrier keeps the scheduler from
      // sinking a prefetch back down to its consumer (counted lgkmcnt waits then cover only it).
      double W[R], AKw[R], SMv[R], G[R], Hh[R], XS[R], tt[R];
      // Up to three rounds every phase's rows of all rounds are loaded one phase ahead (48 R VGPRs);
      // beyond, each phase streams its rounds through two 12-double buffers.
      constexpr bool PF = R <= 3;
      double cA[PF ? R : 1][12], cB[PF ? R : 1][12], cw[PF ? R : 1][3];
      // stream the rounds of a parallel phase: load(r, c) fills c with round r's rows, use(r, c)
      auto pipe = [&](auto load, auto use) __attribute__((always_inline)) {
        double c0[12], c1[12];
        load(0, c0);
        sfor<0, R>([&](auto RR) {
          constexpr int r = decltype(RR)::value;
          if constexpr (r + 1 < R) load(r + 1, (r & 1) ? c0 : c1);
          use(r, (r & 1) ? c1 : c0);
        });
      };
      int kc[R], kk[R];
#pragma unroll
      for (int r = 0; r < R; ++r) {
        W[r] = DI[r] * RHS[r];
        SMv[r] = 0.0;
        XS[r] = 0.0;
        kc[r] = min(4 * r + ig, N - 1);
        kk[r] = max(kc[r] - 1, 0);  // slot of K_k (k >= 1)
      }
      double cn[12];
      if constexpr (PF) {
#pragma unroll
        for (int r = 0; r < R; ++r) ldcol(cA[r], &F.K[kk[r]][idx]);
      }
      // The chains load Acl one ROUND at a time: DPP row q takes the matrix of step 4 rr + gray(q) of
      // round rr, the step that row computes (every chain step runs in the row of its step), so one
      // 12-double load per lane serves four chain steps.
      constexpr int NA = WSmem<N, KS>::NA;
      auto aslot = [&](int rr) __attribute__((always_inline)) { return min(max(4 * rr + ig - 1, 0), NA - 1); };
      if constexpr (N >= 3) ldcol(cn, &F.Acl[aslot((N - 2) >> 2)][idx]);
      __builtin_amdgcn_sched_barrier(0);
      // a_k = K_k' w_k (k >= 1)
      if constexpr (PF) {
#pragma unroll
        for (int r = 0; r < R; ++r) lds_wait<N >= 3 ? 12 : 0>(cA[r]);
        mv_rounds<R>(W, cA, AKw);
      } else {
        lds_wait<0>(cn);  // (the chain's first columns; the streamed loads below are compiler-tracked)
        pipe([&](int r, double (&c)[12]) __attribute__((always_inline)) { ld12s(c, &F.K[kk[r]][idx]); },
             [&](int r, const double (&c)[12]) __attribute__((always_inline)) { AKw[r] = mv12(W[r], c); });
      }
      __builtin_amdgcn_sched_barrier(0);
      if (tm_it) WV_MARK(41);
      // g_k's G_k^-1 rows and B_k' columns: issued when the backward chain enters its last round
      // (three steps before their use), so they do not hold registers through the whole chain
      auto load_g = [&]() __attribute__((always_inline)) {
        if constexpr (PF) {
#pragma unroll
          for (int r = 0; r < R; ++r) {
            ld12(cB[r], &F.Gi[kc[r]][mo(idx)]);
            cw[r][0] = sm.Bw[kc[r]][0][idx];
            cw[r][1] = sm.Bw[kc[r]][1][idx];
            cw[r][2] = sm.Bw[kc[r]][2][idx];
          }
        }
      };
      constexpr int KG = N - 2 >= 2 ? 2 : N - 2;  // the backward chain's step that issues them
      if constexpr (KG < 1) load_g();
      {  // backward chain: s_{N-1} = -a_{N-1}; s_k = Acl_k' s_{k+1} - a_k; SMv (row of k) = s_{k+1}
        double cur = -AKw[(N - 1) >> 2];
        double cc[12];
        sfor<0, N - 1>([&](auto J) {
          constexpr int k = N - 2 - decltype(J)::value;
          const double mvv = rmove2<row_of(k + 1), row_of(k)>(cur);
          SMv[k >> 2] = (q == row_of(k)) ? mvv : SMv[k >> 2];
          if constexpr (k >= 1) {
            if constexpr (k == N - 2 || (k & 3) == 3) {  // entering round k >> 2 (descending)
              lds_wait<0>(cn);
#pragma unroll
              for (int e = 0; e < 12; ++e) cc[e] = cn[e];
              if constexpr (k >= 4) ldcol(cn, &F.Acl[aslot((k >> 2) - 1)][idx]);  // the next round's columns
            }
            if constexpr (k == KG) load_g();
            __builtin_amdgcn_sched_barrier(0);
            cur = mv12a(mvv, cc, -AKw[k >> 2]);
          }
        });
      }
      if (tm_it) WV_MARK(42);
      // g_k = G_k^-1 (w_k + B_k' s_{k+1})
      auto ttr = [&](int r, double c0, double c1, double c2) __attribute__((always_inline)) {
        const double c6[6] = {c0, c1, c2, a == 0 ? dtm : 0.0, a == 1 ? dtm : 0.0, a == 2 ? dtm : 0.0};
        return W[r] + mv6(SMv[r], c6);
      };
      // h_k = B_k g_k: rows 6-8 (leg-2 lanes) B_w g, rows 9-11 (leg-3 lanes) dt/m times the sum of
      // the legs' matching force component, rows 0-5 zero
      auto hhr = [&](int r, double hb) __attribute__((always_inline)) {
        const double ls = dtm * legsum(G[r]);
        return leg == 2 ? hb : (leg == 3 ? ls : 0.0);
      };
      if constexpr (PF) {
#pragma unroll
        for (int r = 0; r < R; ++r) tt[r] = ttr(r, cw[r][0], cw[r][1], cw[r][2]);
#pragma unroll
        for (int r = 0; r < R; ++r) ld12(cA[r], &sm.Bw[kc[r]][av ? a : 2][0]);  // for h_k
        __builtin_amdgcn_sched_barrier(0);
        mv_rounds<R>(tt, cB, G);
        if constexpr (N >= 3) ld12(cn, &F.Acl[aslot(0)][mo(idx)]);
        __builtin_amdgcn_sched_barrier(0);
        double hb[R];
        mv_rounds<R>(G, cA, hb);
#pragma unroll
        for (int r = 0; r < R; ++r) Hh[r] = hhr(r, hb[r]);
      } else {
        pipe([&](int r, double (&c)[12]) __attribute__((always_inline)) { ld12(c, &F.Gi[kc[r]][mo(idx)]); },
             [&](int r, const double (&c)[12]) __attribute__((always_inline)) {
               tt[r] = ttr(r, sm.Bw[kc[r]][0][idx], sm.Bw[kc[r]][1][idx], sm.Bw[kc[r]][2][idx]);
               G[r] = mv12(tt[r], c);
             });
        pipe([&](int r, double (&c)[12]) __attribute__((always_inline)) { ld12(c, &sm.Bw[kc[r]][av ? a : 2][0]); },
             [&](int r, const double (&c)[12]) __attribute__((always_inline)) { Hh[r] = hhr(r, mv12(G[r], c)); });
        if constexpr (N >= 3) ld12(cn, &F.Acl[aslot(0)][mo(idx)]);
      }
      if (tm_it) WV_MARK(43);
      // u_k's K_k rows: issued three steps before the forward chain ends
      auto load_u = [&]() __attribute__((always_inline)) {
        if constexpr (PF) {
#pragma unroll
          for (int r = 0; r < R; ++r) ld12(cB[r], &F.K[kk[r]][mo(idx)]);
        }
      };
      constexpr int KU = N - 2 >= 1 ? (N - 3 > 1 ? N - 3 : 1) : 0;  // two steps before the end
      if constexpr (KU < 1) load_u();
      {  // forward chain: x_1 = h_0; x_{k+1} = Acl_k x_k + h_k; XS (row of k) = x_k
        double cur = Hh[0];
        double cc[12];
        sfor<1, N>([&](auto K) {
          constexpr int k = decltype(K)::value;
          const double mvv = rmove2<row_of(k - 1), row_of(k)>(cur);
          XS[k >> 2] = (q == row_of(k)) ? mvv : XS[k >> 2];
          if constexpr (k <= N - 2) {
            if constexpr (k == 1 || (k & 3) == 0) {  // entering round k >> 2 (ascending)
#pragma unroll
              for (int e = 0; e < 12; ++e) cc[e] = cn[e];
              if constexpr (4 * ((k >> 2) + 1) <= N - 2) ld12(cn, &F.Acl[aslot((k >> 2) + 1)][mo(idx)]);
            }
            if constexpr (k == KU) load_u();
            __builtin_amdgcn_sched_barrier(0);
            cur = mv12a(mvv, cc, Hh[k >> 2]);
          }
        });
      }
      if (tm_it) WV_MARK(44);
      // u_k = g_k - K_k x_k (x_0 = 0)
      if constexpr (PF) {
        double kx[R];
        mv_rounds<R>(XS, cB, kx);
#pragma unroll
        for (int r = 0; r < R; ++r) U[r] = G[r] - kx[r];
      } else {
        pipe([&](int r, double (&c)[12]) __attribute__((always_inline)) { ld12(c, &F.K[kk[r]][mo(idx)]); },
             [&](int r, const double (&c)[12]) __attribute__((always_inline)) { U[r] = G[r] - mv12(XS[r], c); });
      }
#ifdef MPCQP_DBG
      for (int r = 0; r < R; ++r)
        U[r] = MPCQP_DBG == 1 ? G[r] : MPCQP_DBG == 2 ? Hh[r] : MPCQP_DBG == 3 ? XS[r] : MPCQP_DBG == 4 ? SMv[r] : W[r];
#endif
    }
    if (tm_it) WV_MARK(45);
    };  // kkt

    // ---- update_x / update_z / update_y, and P~x by the KKT identity P~x~ = rhs - sigma x~ - A~'rho A~x~
    // this iteration's deltas, for the infeasibility tests of a need_info iteration only
    double DX[R], DY[R], DY4P[NP], PXO[R];
    auto update = [&](auto INFO) __attribute__((always_inline)) {
      constexpr bool info = decltype(INFO)::value;
      double xt[R], xz[R], zt[R];
#pragma unroll
    for (int r = 0; r < R; ++r) {
      xt[r] = DI[r] * U[r];
      const double xp = dpp<QP_PRIM>(xt[r]);
      xz[r] = dpp<QP_B2>(xt[r]);
      zt[r] = AK0[r] * xp + AK1[r] * xz[r];
      {  // (fmin/fmax = the reference's c_min/c_max on these non-NaN operands)
        const double zr = alpha * zt[r] + (1.0 - alpha) * Z[r];
        const double zn = fmin(fmax(zr + rinv * Y[r], LO03), HI03);
        const double dyv = rho * (zr - zn);
        Z[r] = zn;
        Y[r] = Y[r] + dyv;
        if constexpr (info) DY[r] = dyv;
      }
    }
      // row 4, packed: lane a projects round 4 pr + a
      double V4P[NP], T4P[NP];
#pragma unroll
    for (int pr = 0; pr < NP; ++pr) {
      const double zt4 = AK4P[pr] * pack_of([&](int r) { return xz[r]; }, pr);
      const double r4 = RHO4P[pr];
      const double zr = alpha * zt4 + (1.0 - alpha) * Z4P[pr];
      const double zn = fmin(fmax(zr + RI4P[pr] * Y4P[pr], L4P[pr]), U4P[pr]);
      const double dyv = r4 * (zr - zn);
      Z4P[pr] = zn;
      Y4P[pr] = Y4P[pr] + dyv;
      if constexpr (info) DY4P[pr] = dyv;
      V4P[pr] = RHO4P[pr] * Z4P[pr] - Y4P[pr];
      T4P[pr] = KS == 0 ? RHO4P[pr] * zt4 : 0.0;
    }
#pragma unroll
    for (int r = 0; r < R; ++r) {
      // every lane updates (values of padding lanes / steps past N are never read unmasked)
      const double xo = X[r];
      const double xn = alpha * xt[r] + (1.0 - alpha) * xo;
      if constexpr (info) DX[r] = xn - xo;
      X[r] = xn;
      const double ak4 = unpack(AK4P, r);
      if constexpr (KS == 0) {  // the Riccati variant carries P~x; the Schur form computes it at checks
        const double kd = quad_at(rho * zt[r], unpack(T4P, r), AK0[r], AK1[r], ak4, a);
        const double pxt = (RHS[r] - sigma * xt[r]) - kd;
        if constexpr (info) PXO[r] = PX[r];
        PX[r] = alpha * pxt + (1.0 - alpha) * PX[r];
      }
      // next right-hand side sigma x - q~ + A~'(rho z - y) (recomputed below when adapt_rho changes rho)
      const double at = quad_at(rho * Z[r] - Y[r], unpack(V4P, r), AK0[r], AK1[r], ak4, a);
      RHS[r] = (sigma * X[r] - Qv[r]) + at;
    }
    };

#ifndef MPCQP_SINGLE_LOOP
    // The iterations before the next one that needs update_info (a termination check, an adapt_rho
    // step or the last iteration) run in a loop of their own: the check's registers are then live
    // only outside it, and the allocator keeps the ADMM state of the inner loop in registers.
    {
      int plain = p.max_iter - iter;
      if (p.check_termination) plain = min(plain, to_check - 1);
      if (p.adaptive_rho) plain = min(plain, to_adapt - 1);
      for (int j = 0; j < plain; ++j) {
        kkt(IC<0>{});
        if (p.check_termination) --to_check;
        if (p.adaptive_rho) --to_adapt;
        update(IC<0>{});
        if (iter == 60) WV_MARK(46);
        if (iter == 60) WV_MARK(47);
        ++iter;
      }
    }
#endif
    const bool tm_it = iter == 60;
    kkt(IC<1>{});  // (with the inner loop above, always an update_info iteration)
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

    if (need_info) update(IC<1>{});
    else update(IC<0>{});

    if (tm_it) WV_MARK(46);
    const bool tm_ck = iter == 75;  // (a termination check + adapt_rho iteration, timed)
    if (tm_ck) WV_MARK(48);
    if (need_info) {
      // ---- update_info / check_termination / adapt_rho (osqp.c, auxil.c) ----
      // KS = 1: P~x of this iterate, local to the check (not carried through the loop)
      // D and E of the lane's variables / rows.  The Riccati form loads them for the whole check in
      // one batch (one memory round trip instead of one per round: C4 +1.4 %); the Schur form where
      // they are used (holding them through P~x made its check slower: C2 -2 %, profiles/r05)
      // row 4 per round (the packed registers unpacked for the check)
      double Z4[R], Y4[R], L4[R], U4[R], AK4[R], DY4[R];
#pragma unroll
      for (int r = 0; r < R; ++r) {
        Z4[r] = unpack(Z4P, r);
        Y4[r] = unpack(Y4P, r);
        L4[r] = unpack(L4P, r);
        U4[r] = unpack(U4P, r);
        AK4[r] = unpack(AK4P, r);
        DY4[r] = unpack(DY4P, r);
      }
      double DVc[R], EVc[R], E4c[R];
#pragma unroll
      for (int r = 0; r < R; ++r) {
        if constexpr (KS == 0) {
          DVc[r] = dv_of(r);
          EVc[r] = ev_of(r);
          E4c[r] = e4_of(r);
        } else {
          DVc[r] = EVc[r] = E4c[r] = 0.0;
        }
      }
      auto dvc = [&](int r) __attribute__((always_inline)) { return KS == 0 ? DVc[r] : dv_of(r); };
      auto evc = [&](int r) __attribute__((always_inline)) { return KS == 0 ? EVc[r] : ev_of(r); };
      auto e4c = [&](int r) __attribute__((always_inline)) { return KS == 0 ? E4c[r] : e4_of(r); };
      double PXl[R];
      double (&PXc)[R] = KS == 1 ? PXl : PX;
      if constexpr (KS == 1) {
        double dd[R];
#pragma unroll
        for (int r = 0; r < R; ++r) dd[r] = dvc(r);
        px_of(X, dd, PXc);
      }
      if (tm_ck) WV_MARK(50);
      // The norms of update_info / check_termination / compute_rho_estimate, and the first-level
      // quantities of both infeasibility tests (||E dy||, the support term of dy, ||D dx||, q'dx:
      // needed at nearly every check, since dua_res is rarely small before convergence), reduced
      // in one batch of independent wave reductions.  Norms that enter only as max(a, b) share a
      // slot (a max is exact in any grouping): [0] |E^-1 (A~x - z)|, [1] |A~x - z|,
      // [2] max(|E^-1 z|, |E^-1 A~x|), [3] max(|z|, |A~x|), [4] |D^-1 dual|, [5] |dual|,
      // [6] max(|D^-1 q~|, |D^-1 A~'y|, |D^-1 P~x|), [7] max(|q~|, |A~'y|, |P~x|).
      constexpr int NM = 8;
      double mx[NM];
#pragma unroll
      for (int k = 0; k < NM; ++k) mx[k] = 0.0;
      double nd = 0.0, lh = 0.0, nx = 0.0, qd = 0.0, dyp[R], dyp4[R];
      auto proj = [&](double d, double lo, double hi) __attribute__((always_inline)) {
        // delta_y projected onto the polar of the recession cone of [l, u]
        if (hi > OSQP_INF * MIN_SCALING) {
          if (lo < -OSQP_INF * MIN_SCALING) d = 0.0;
          else d = dmin(d, 0.0);
        } else if (lo < -OSQP_INF * MIN_SCALING) {
          d = dmax(d, 0.0);
        }
        return d;
      };
#pragma unroll
      for (int r = 0; r < R; ++r) {
        const double xp = dpp<QP_PRIM>(X[r]), xz = dpp<QP_B2>(X[r]);
        const double ax = AK0[r] * xp + AK1[r] * xz, ax4 = AK4[r] * xz;
        const double aty = quad_at(Y[r], Y4[r], AK0[r], AK1[r], AK4[r], a);
        const double evr = evc(r), e4r = e4c(r);
        if (kvr[r]) {
          const double ei = recip(evr), ei4 = recip(e4r);
          const double pr = ax + (-1.0) * Z[r], pr4 = ax4 + (-1.0) * Z4[r];
          mx[0] = nmax(mx[0], nmax(dabs(ei * pr), dabs(ei4 * pr4)));
          mx[1] = nmax(mx[1], nmax(dabs(pr), dabs(pr4)));
          mx[2] = nmax(mx[2], nmax(nmax(dabs(ei * Z[r]), dabs(ei4 * Z4[r])), nmax(dabs(ei * ax), dabs(ei4 * ax4))));
          mx[3] = nmax(mx[3], nmax(nmax(dabs(Z[r]), dabs(Z4[r])), nmax(dabs(ax), dabs(ax4))));
        }
        if (vvr[r]) {
          const double d = (Qv[r] + 1.0 * PXc[r]) + 1.0 * aty;
          mx[4] = nmax(mx[4], dabs(DI[r] * d));
          mx[5] = nmax(mx[5], dabs(d));
          mx[6] = nmax(mx[6], nmax(nmax(dabs(DI[r] * Qv[r]), dabs(DI[r] * aty)), dabs(DI[r] * PXc[r])));
          mx[7] = nmax(mx[7], nmax(nmax(dabs(Qv[r]), dabs(aty)), dabs(PXc[r])));
        }
        // is_primal_infeasible: ||E dy||_inf and u'max(dy, 0) + l'min(dy, 0) of the projected dy
        const double lo = lo03(evr), hi = hi03(evr);
        const double d = proj(DY[r], lo, hi), d4 = proj(DY4[r], L4[r], U4[r]);
        dyp[r] = d;
        dyp4[r] = d4;
        if (kvr[r]) {
          nd = nmax(nd, nmax(dabs(evr * d), dabs(e4r * d4)));
          lh += hi * dmax(d, 0.0) + lo * dmin(d, 0.0);
          if (a == 0) lh += U4[r] * dmax(d4, 0.0) + L4[r] * dmin(d4, 0.0);
        }
        // is_dual_infeasible: ||D dx||_inf and q~'dx
        if (vvr[r]) {
          nx = nmax(nx, dabs(dvc(r) * DX[r]));
          qd += Qv[r] * DX[r];
        }
      }
      // the 10 max- and 2 sum-reductions level by level (wave_reduce_batch: same bits, no waits)
      double rm[NM + 2], rs[2] = {lh, qd};
#pragma unroll
      for (int k = 0; k < NM; ++k) rm[k] = mx[k];
      rm[NM] = nd;
      rm[NM + 1] = nx;
      wave_reduce_batch(rm, rs);
#pragma unroll
      for (int k = 0; k < NM; ++k) mx[k] = rm[k];
      const double ndy = rm[NM], ndx = rm[NM + 1];
      lh = rs[0];
      qd = rs[1];
      pri_res = mx[0];
      dua_res = cinv * mx[4];
      iters = iter;
      if (tm_ck) WV_MARK(51);
      auto check = [&](bool approx) __attribute__((always_inline)) -> int {
        double eps_abs = p.eps_abs, eps_rel = p.eps_rel, eps_pinf = p.eps_prim_inf, eps_dinf = p.eps_dual_inf;
        if (pri_res > OSQP_INF || dua_res > OSQP_INF) return MPCQP_STATUS_NON_CVX;
        if (approx) { eps_abs *= 10; eps_rel *= 10; eps_pinf *= 10; eps_dinf *= 10; }
        const double eps_prim = eps_abs + eps_rel * mx[2];
        const bool prim_ok = pri_res < eps_prim;
        bool prim_inf = false, dual_inf = false;
        if (!prim_ok && ndy > DIV_TOL && lh < eps_pinf * ndy) {
          double an = 0.0;
#pragma unroll
          for (int r = 0; r < R; ++r) {
            const double atd = quad_at(dyp[r], dyp4[r], AK0[r], AK1[r], AK4[r], a);
            if (vvr[r]) an = nmax(an, dabs(DI[r] * atd));
          }
          an = wave_nmax(an);
          prim_inf = an < eps_pinf * ndy;
        }
        const double eps_dual = eps_abs + eps_rel * (cinv * mx[6]);
        const bool dual_ok = dua_res < eps_dual;
        if (!dual_ok && ndx > DIV_TOL && qd < cost_c * eps_dinf * ndx) {
          // is_dual_infeasible (P~ delta_x = P~x_new - P~x_old)
          double pd = 0.0, PDX[R];
          if constexpr (KS == 1) {
            double dd[R];
#pragma unroll
            for (int r = 0; r < R; ++r) dd[r] = dvc(r);
            px_of(DX, dd, PDX);
          }
#pragma unroll
          for (int r = 0; r < R; ++r) {
            if constexpr (KS == 0) PDX[r] = PX[r] - PXO[r];
            if (vvr[r]) pd = nmax(pd, dabs(DI[r] * PDX[r]));
          }
          pd = wave_nmax(pd);
          if (pd < cost_c * eps_dinf * ndx) {
            double viol = 0.0;
#pragma unroll
            for (int r = 0; r < R; ++r) {
              const double dp = dpp<QP_PRIM>(DX[r]), dz = dpp<QP_B2>(DX[r]);
              const double evr = evc(r);
              const double v = (1.0 / evr) * (AK0[r] * dp + AK1[r] * dz);
              const double v4 = (1.0 / e4c(r)) * (AK4[r] * dz);
              const double lo = lo03(evr), hi = hi03(evr);
              if (kvr[r]) {
                if ((hi < OSQP_INF * MIN_SCALING && v > eps_dinf * ndx) ||
                    (lo > -OSQP_INF * MIN_SCALING && v < -eps_dinf * ndx))
                  viol = 1.0;
                if ((U4[r] < OSQP_INF * MIN_SCALING && v4 > eps_dinf * ndx) ||
                    (L4[r] > -OSQP_INF * MIN_SCALING && v4 < -eps_dinf * ndx))
                  viol = 1.0;
              }
            }
            viol = wave_nmax(viol);
            dual_inf = viol == 0.0;
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
        const double pr_n = mx[1] / (mx[3] + DIV_TOL);
        const double du_n = mx[5] / (mx[7] + DIV_TOL);
        double est = rho * sqrt(pr_n / (du_n + DIV_TOL));
        est = dmin(dmax(est, RHO_MIN), RHO_MAX);
        if (est > rho * p.adaptive_rho_tolerance || est < rho / p.adaptive_rho_tolerance) {
          rho = dmin(dmax(est, RHO_MIN), RHO_MAX);
          rho_updates += 1;
          refactor = !last;
        }
      }
      if (tm_ck) WV_MARK(52);
      if (last && st == MPCQP_STATUS_UNSOLVED) st = MPCQP_STATUS_MAX_ITER_REACHED;
      // (an ill-conditioned factorization since the last check, or a KKT solve whose push-through
      // identity cancelled too many digits: leave now, see the factorization)
      if constexpr (KS == 1) amp_bad = !(amp * img_at(SI::DEGEN) <= SCHUR_AMP);
      if (last || (KS == 1 && (amp_bad || !(img_at(SI::DEGEN) <= SCHUR_SMAX)))) done = true;
      status = st;
#ifndef MPCQP_PHASE_TIMING
      if (trace && t == 0 && inst < trace_cap && ntrace < MPCQP_TRACE_LEN && is_check) {
        double* tp = trace + ((size_t)inst * MPCQP_TRACE_LEN + ntrace) * 4;
#ifdef MPCQP_TRACE_COND  // conditioning study builds (tools/r06_cancel.py): amp and S_max per check
        tp[0] = iter; tp[1] = amp; tp[2] = KS == 1 ? img_at(SI::DEGEN) : 0.0; tp[3] = rho;
#else
        tp[0] = iter; tp[1] = pri_res; tp[2] = dua_res; tp[3] = rho;
#endif
      }
#endif
      ntrace += is_check ? 1 : 0;
      if (done) {
        // the objective of the final iterate (every exit of the loop is a need_info iteration)
#pragma unroll
        for (int r = 0; r < R; ++r)
          if (vvr[r]) obj_sum += 0.5 * X[r] * PXc[r] + Qv[r] * X[r];
        obj_sum = wave_sum(obj_sum);
        break;
      }
      if (refactor) {
#pragma unroll
        for (int pr = 0; pr < NP; ++pr) {
          RHO4P[pr] = rho4_of(L4P[pr], U4P[pr], rho);
          RI4P[pr] = 1. / RHO4P[pr];
        }
        rinv = 1. / rho;
        need_factor = true;
        // the right-hand side with the new rho vector
#pragma unroll
        for (int r = 0; r < R; ++r) {
          const double at = quad_at(rho * Z[r] - Y[r], unpack(RHO4P, r) * Z4[r] - Y4[r], AK0[r], AK1[r], AK4[r], a);
          RHS[r] = (sigma * X[r] - Qv[r]) + at;
        }
      }
    }
    if (tm_ck) WV_MARK(49);
    if (tm_it) WV_MARK(47);
  }

  WV_MARK(20);
  if (KS == 1 && (amp_bad || !(img_at(SI::DEGEN) <= SCHUR_SMAX))) {  // the Riccati form solves it
    if (t == 0) atomicAdd(fb + (amp_bad ? 1 : 2), 1);
    return true;
  }
  if (ws) {  // the solver persists: scaling, scaled data, iterates and rho for the next tick
    if (t == 0) {
      ws[WL::FLAG] = 1.0;
      ws[WL::RHO] = rho;
      ws[WL::C] = cost_c;
      ws[WL::MU] = mu_rec;
    }
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const int k = 4 * r + ig;
      if (vvr[r]) {
        const int ci = ND * k + idx;
        ws[WL::D + ci] = dv_of(r);
        ws[WL::QT + ci] = Qv[r];
        ws[WL::X + ci] = X[r];
      }
      if (kvr[r]) {
        const int ri = CD * k + 5 * leg + a, r4 = CD * k + 5 * leg + 4;
        ws[WL::E + ri] = ev_of(r);
        ws[WL::AK + ri] = AK0[r];
        ws[WL::AK + m + ri] = AK1[r];
        ws[WL::Z + ri] = Z[r];
        ws[WL::Y + ri] = Y[r];
        const double ak4 = unpack(AK4P, r), z4 = unpack(Z4P, r), y4 = unpack(Y4P, r);
        if (a == 0) {
          ws[WL::E + r4] = e4_of(r);
          ws[WL::AK + r4] = 0.0;
          ws[WL::AK + m + r4] = ak4;
          ws[WL::Z + r4] = z4;
          ws[WL::Y + r4] = y4;
        }
      }
    }
  }
  // ---- 6. store_solution + unscale + compute_grf extraction (A1RobotControl.cpp:555-561) --------
  const bool has_sol = status != MPCQP_STATUS_PRIMAL_INFEASIBLE &&
                       status != MPCQP_STATUS_PRIMAL_INFEASIBLE_INACCURATE &&
                       status != MPCQP_STATUS_DUAL_INFEASIBLE &&
                       status != MPCQP_STATUS_DUAL_INFEASIBLE_INACCURATE && status != MPCQP_STATUS_NON_CVX;
  const double ob = obj_sum;
  double xs0 = 0.0;
#pragma unroll
  for (int r = 0; r < R; ++r) {
    const double xs = has_sol ? dv_of(r) * X[r] : NAN;
    if (r == 0) xs0 = xs;
    if (solution && vvr[r]) solution[(size_t)inst * n + ND * (4 * r + ig) + idx] = xs;
  }
  // u0 = step 0 = round 0, DPP row 0 (lanes 0..15); f_i = R^T u0[3i:3i+3], NaN legs skipped
  mpcqp_result* res = results + inst;
  const volatile double* rotv = recs + (size_t)inst * C::REC + MPCQP_REC_ROT;
  double Rot[9];
#pragma unroll
  for (int e = 0; e < 9; ++e) Rot[e] = rotv[e];
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
  return false;
}

// waves per SIMD the register allocation must allow (experiment builds: MPCQP_WAVE_WPE=2 asks the
// allocator for 256 registers, the budget of two robots per SIMD; profiles/r06/two_per_simd)
#if defined(MPCQP_WAVE_NUM_VGPR)
#define MPCQP_WAVE_BOUNDS __launch_bounds__(NT) __attribute__((amdgpu_num_vgpr(MPCQP_WAVE_NUM_VGPR)))
#elif defined(MPCQP_WAVE_WPE)
#define MPCQP_WAVE_BOUNDS __launch_bounds__(NT) __attribute__((amdgpu_waves_per_eu(MPCQP_WAVE_WPE)))
#else
#define MPCQP_WAVE_BOUNDS __launch_bounds__(NT, 1)
#endif
template <int N, int KS>
__global__ MPCQP_WAVE_BOUNDS void wave_kernel(const double* __restrict__ recs, int batch,
                                                     mpcqp_result* __restrict__ results,
                                                     double* __restrict__ solution, double* __restrict__ trace,
                                                     int trace_cap, double* __restrict__ wstate,
                                                     double* __restrict__ img, mpcqp_params p,
                                                     int* __restrict__ fb) {
  const int inst = blockIdx.x;
  if constexpr (KS == 1) {
    // The Schur form, and in the same wave the Riccati form for the robots it hands over (the two
    // forms' LDS images share one allocation: the Riccati factors fit inside the Schur core's)
    __shared__ union LdsU {
      WSmem<N, 1> s;
      WSmem<N, 0> r;
    } sm;
    if (inst >= batch) return;
    if (wave_solve<N, 1, MPCQP_FUSED_SCALE != 0>(inst, sm.s, recs, results, solution, trace, trace_cap, wstate, img,
                                                   p, fb)) {
      wave_sync();
      wave_solve<N, 0>(inst, sm.r, recs, results, solution, trace, trace_cap, wstate, img, p, nullptr);
    }
  } else {
    __shared__ WSmem<N, 0> sm;
    if (inst >= batch) return;
    wave_solve<N, 0>(inst, sm, recs, results, solution, trace, trace_cap, wstate, img, p, fb);
  }
}

// Self-test of the cross-lane primitives (mv12 broadcast lanes, rmove directions): out[64*k + lane].
__global__ void wave_selftest_kernel(double* out) {
  const int t = threadIdx.x;
  const double x = 100.0 * (t >> 4) + (t & 15);
  double c[12];
  for (int i = 0; i < 12; ++i) c[i] = (i == (t & 15) % 12) ? 1.0 : 0.0;
  out[t] = mv12(x, c);            // lane 16q+i: x of lane loff(i % 12) of row q
  out[64 + t] = rmove<0, 1>(x);   // row 1 lanes: row 0 values
  out[128 + t] = rmove<1, 0>(x);  // row 0 lanes: row 1 values
  out[192 + t] = rmove<0, 2>(x);  // row 2 lanes: row 0 values
  out[256 + t] = rmove<3, 1>(x);  // row 1 lanes: row 3 values
  out[320 + t] = rmove<3, 2>(x);  // row 2 lanes: row 3 values
}

}  // namespace wv

// The Schur-form KKT solve serves N <= 10 with nonnegative state weights (it factors Q with square
// roots); the Riccati recursion everything else.
static bool schur_ok(const mpcqp_params& p) {
  if (p.horizon > 10) return false;
  for (int i = 0; i < MPCQP_STATE_DIM; ++i)
    if (!(p.q_weights[i] >= 0.0)) return false;
#ifdef MPCQP_WAVE_RICCATI_ONLY
  return false;
#endif
  return true;
}
// experiment builds: MPCQP_WAVE_LDS_PAD bytes of dynamic LDS per wave-kernel workgroup (fewer robots
// per CU: per-robot phase costs without neighbours sharing the CU's LDS or instruction cache)
#ifndef MPCQP_WAVE_LDS_PAD
#define MPCQP_WAVE_LDS_PAD 0
#endif
template <int N>
static hipError_t launch_wave(const LaunchArgs& a) {
  if (!a.fallback) return hipErrorInvalidValue;
  hipError_t e = hipSuccess;
  if (!(MPCQP_FUSED_SCALE && N <= 10 && schur_ok(a.p))) {
    hipLaunchKernelGGL((wv::scale_kernel<N>), dim3(a.batch), dim3(wv::ScaleCfg<N>::NTS), 0, (hipStream_t)a.stream,
                       a.recs, a.batch, a.wstate, a.work, a.p, a.fallback);
    e = hipGetLastError();
  } else {  // the fused setup: wave_kernel scales; the hand-off counters start at zero (stream order)
    e = hipMemsetAsync(a.fallback, 0, 4 * sizeof(int), (hipStream_t)a.stream);
  }
  if (e != hipSuccess) return e;
  if constexpr (N <= 10) {
    if (schur_ok(a.p)) {
      hipLaunchKernelGGL((wv::wave_kernel<N, 1>), dim3(a.batch), dim3(wv::NT), MPCQP_WAVE_LDS_PAD, (hipStream_t)a.stream, a.recs,
                         a.batch, a.results, a.solution, a.trace, a.trace_cap, a.wstate, a.work, a.p, a.fallback);
      return hipGetLastError();
    }
  }
  hipLaunchKernelGGL((wv::wave_kernel<N, 0>), dim3(a.batch), dim3(wv::NT), MPCQP_WAVE_LDS_PAD, (hipStream_t)a.stream, a.recs, a.batch,
                     a.results, a.solution, a.trace, a.trace_cap, a.wstate, a.work, a.p, a.fallback);
  return hipGetLastError();
}
template <int N>
static hipError_t launch_scale(const LaunchArgs& a) {
  if (!a.fallback) return hipErrorInvalidValue;
  hipLaunchKernelGGL((wv::scale_kernel<N>), dim3(a.batch), dim3(wv::ScaleCfg<N>::NTS), 0, (hipStream_t)a.stream,
                     a.recs, a.batch, a.wstate, a.work, a.p, a.fallback);
  return hipGetLastError();
}
// occupancy of the wave kernel a handle with these parameters launches (the KS choice of launch_wave)
template <int N>
static hipError_t occupancy_wave(const mpcqp_params& p, int* blocks) {
  if constexpr (N <= 10)
    if (schur_ok(p)) return hipOccupancyMaxActiveBlocksPerMultiprocessor(blocks, wv::wave_kernel<N, 1>, wv::NT, 0);
  return hipOccupancyMaxActiveBlocksPerMultiprocessor(blocks, wv::wave_kernel<N, 0>, wv::NT, 0);
}

#ifndef MPCQP_WAVE_FOR_EACH_N
#define MPCQP_WAVE_FOR_EACH_N(X) \
  X(1) X(2) X(3) X(4) X(5) X(6) X(7) X(8) X(9) X(10) X(11) X(12) X(13) X(14) X(15) X(16) X(17) X(18) X(19) X(20)
#endif

hipError_t launch_wave_any(const LaunchArgs& a) {
  switch (a.p.horizon) {
#define CASE(K) \
  case K: return launch_wave<K>(a);
    MPCQP_WAVE_FOR_EACH_N(CASE)
#undef CASE
    default: return hipErrorInvalidValue;
  }
}
hipError_t launch_scale_any(const LaunchArgs& a) {
  switch (a.p.horizon) {
#define CASE(K) \
  case K: return launch_scale<K>(a);
    MPCQP_WAVE_FOR_EACH_N(CASE)
#undef CASE
    default: return hipErrorInvalidValue;
  }
}
hipError_t occupancy_wave_any(const mpcqp_params& p, int* blocks) {
  switch (p.horizon) {
#define CASE(K) \
  case K: return occupancy_wave<K>(p, blocks);
    MPCQP_WAVE_FOR_EACH_N(CASE)
#undef CASE
    default: return hipErrorInvalidValue;
  }
}
hipError_t wave_selftest(double* d_out, void* stream) {
  hipLaunchKernelGGL(wv::wave_selftest_kernel, dim3(1), dim3(64), 0, (hipStream_t)stream, d_out);
  return hipGetLastError();
}
}  // namespace mpcqp
