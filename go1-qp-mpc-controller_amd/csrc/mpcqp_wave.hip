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
// Setup (condensation, Ruiz) keeps |H| as fp32 in LDS for the column norms only;
// everything else is binary64.
#include "mpcqp_device.h"

namespace mpcqp {
namespace wv {

constexpr int NT = 64;
__host__ __device__ constexpr int gray(int v) { return v == 2 ? 3 : (v == 3 ? 2 : v); }  // own inverse
__host__ __device__ constexpr int row_of(int k) { return gray(k & 3); }  // DPP row of horizon step k

template <int N>
struct Cfg {
  static constexpr int n = ND * N, m = CD * N, R = (N + 3) / 4, NH = n * (n + 1) / 2;
  static constexpr int REC = MPCQP_REC_SIZE(N);
};

template <int N>
struct WSmem {
  using C = Cfg<N>;
  double rec[C::REC];
  alignas(16) double Bw[N][3][ND];  // rows 6-8 of B_d(k) = I_w^-1 skew(foot) dt (rows 9-11: dt/m I)
  double lam[N][ND];                // gradient adjoint lambda_k (states 0..11)
  double vec[2][16];                // sequential 13-vectors (gradient forward sweep)
  union U {
    struct Hs {  // setup: |H| (fp32, packed upper triangle, column-major), S_k B_k, Ruiz vectors
      float H32[C::NH];
      float D32[C::n];
      alignas(16) double G[N][144];
      alignas(16) double V[2][144];
      double S[144], T[144];
      double D[C::n], Dt[C::n], q[C::n], cm[C::n], E[C::m];
      double ak[C::m][3];
    } h;
    struct Fs {  // solve: per-step factors + factorization scratch
      alignas(16) double Gi[N][144];
      alignas(16) double K[N][144];
      alignas(16) double Acl[N][144];
      alignas(16) double P[144], PB[144], PA[144], F[144], Gm[144];
      double Rt[N][ND][3];  // R'_k: row i, the three columns of its foot block
    } f;
  } u;
};

// ---- cross-lane primitives ---------------------------------------------------------------------
#define WV_FM(A, M, L) "v_fmac_f64_dpp " A ", %[x], " M " row_newbcast:" #L " row_mask:0xf bank_mask:0xf\n\t"
// y_i = sum_c M[i][c] x_c, x_c broadcast from lane 4(c/3)+c%3 of each DPP row, M row i in `c`.
// Two accumulators (even / odd c).  s_nop 1: a VALU write of x just before needs 2 wait states
// before a DPP read of it.
__device__ __forceinline__ double mv12(double x, const double (&c)[12]) {
  double a0 = 0.0, a1 = 0.0;
  asm("s_nop 1\n\t"
      WV_FM("%[a0]", "%[c0]", 0) WV_FM("%[a1]", "%[c1]", 1) WV_FM("%[a0]", "%[c2]", 2)
      WV_FM("%[a1]", "%[c3]", 4) WV_FM("%[a0]", "%[c4]", 5) WV_FM("%[a1]", "%[c5]", 6)
      WV_FM("%[a0]", "%[c6]", 8) WV_FM("%[a1]", "%[c7]", 9) WV_FM("%[a0]", "%[c8]", 10)
      WV_FM("%[a1]", "%[c9]", 12) WV_FM("%[a0]", "%[c10]", 13) WV_FM("%[a1]", "%[c11]", 14)
      : [a0] "+v"(a0), [a1] "+v"(a1)
      : [x] "v"(x), [c0] "v"(c[0]), [c1] "v"(c[1]), [c2] "v"(c[2]), [c3] "v"(c[3]), [c4] "v"(c[4]),
        [c5] "v"(c[5]), [c6] "v"(c[6]), [c7] "v"(c[7]), [c8] "v"(c[8]), [c9] "v"(c[9]), [c10] "v"(c[10]),
        [c11] "v"(c[11]));
  return a0 + a1;
}
// sum over states 6..11 (lanes 8, 9, 10, 12, 13, 14) of c[s-6] x_s
__device__ __forceinline__ double mv6(double x, const double (&c)[6]) {
  double a0 = 0.0, a1 = 0.0;
  asm("s_nop 1\n\t"
      WV_FM("%[a0]", "%[c0]", 8) WV_FM("%[a1]", "%[c1]", 9) WV_FM("%[a0]", "%[c2]", 10)
      WV_FM("%[a1]", "%[c3]", 12) WV_FM("%[a0]", "%[c4]", 13) WV_FM("%[a1]", "%[c5]", 14)
      : [a0] "+v"(a0), [a1] "+v"(a1)
      : [x] "v"(x), [c0] "v"(c[0]), [c1] "v"(c[1]), [c2] "v"(c[2]), [c3] "v"(c[3]), [c4] "v"(c[4]),
        [c5] "v"(c[5]));
  return a0 + a1;
}
#undef WV_FM

// quad_perm DPP of a double
constexpr int QP_PRIM = 0x50;  // [0,0,1,1]: row lane a reads variable a>>1 (fx: rows 0,1; fy: rows 2,3)
constexpr int QP_B0 = 0x00, QP_B1 = 0x55, QP_B2 = 0xAA, QP_B3 = 0xFF;  // quad broadcasts
constexpr int QP_02 = 0x08;  // [0,2,0,0]
constexpr int QP_13 = 0x5D;  // [1,3,1,1]
constexpr int QP_X1 = 0xB1, QP_X2 = 0x4E;

// Move a per-row vector from DPP row FROM to row TO (rows one bit apart).  permlane16_swap(v, v)
// returns {v with odd rows := even rows, v with even rows := odd rows}; permlane32_swap likewise
// for row pairs (0,2), (1,3).
template <int FROM, int TO>
__device__ __forceinline__ double rmove(double v) {
  static_assert((FROM ^ TO) == 1 || (FROM ^ TO) == 2, "rows must differ in one bit");
  const unsigned lo = (unsigned)__double2loint(v), hi = (unsigned)__double2hiint(v);
  if constexpr ((FROM ^ TO) == 1) {
    const auto l2 = __builtin_amdgcn_permlane16_swap(lo, lo, false, false);
    const auto h2 = __builtin_amdgcn_permlane16_swap(hi, hi, false, false);
    return FROM < TO ? __hiloint2double((int)h2[0], (int)l2[0]) : __hiloint2double((int)h2[1], (int)l2[1]);
  } else {
    const auto l2 = __builtin_amdgcn_permlane32_swap(lo, lo, false, false);
    const auto h2 = __builtin_amdgcn_permlane32_swap(hi, hi, false, false);
    return FROM < TO ? __hiloint2double((int)h2[0], (int)l2[0]) : __hiloint2double((int)h2[1], (int)l2[1]);
  }
}

template <int V>
struct IC {
  static constexpr int value = V;
};
template <int B, int E, class Fn>
__device__ __forceinline__ void sfor(Fn&& f) {
  if constexpr (B < E) {
    f(IC<B>{});
    sfor<B + 1, E>(f);
  }
}

__device__ __forceinline__ void ld12(double (&c)[12], const double* p) {  // 12 contiguous, 16-B aligned
  const double2* p2 = reinterpret_cast<const double2*>(p);
#pragma unroll
  for (int i = 0; i < 6; ++i) {
    const double2 v = p2[i];
    c[2 * i] = v.x;
    c[2 * i + 1] = v.y;
  }
}
__device__ __forceinline__ void ld12s(double (&c)[12], const double* p) {  // a column (stride 12)
#pragma unroll
  for (int i = 0; i < 12; ++i) c[i] = p[12 * i];
}

// The 12x12 discrete A = I + A_c dt (calculate_A_mat_c + state_space_discretization,
// ConvexMpc.cpp:110-156) restricted to states 0..11: off-diagonals (0,6)=cy dt, (0,7)=sy dt,
// (1,6)=-sy dt, (1,7)=cy dt, (2,8)=dt, (3..5, 9..11)=dt.
struct Adisc {
  double ad0, ad1, dt;
  __device__ __forceinline__ double atv(int i, const double* v) const {  // (A'v)_i
    double s = v[i];
    if (i == 6) s = (s + ad0 * v[0]) + (-ad1) * v[1];
    else if (i == 7) s = (s + ad1 * v[0]) + ad0 * v[1];
    else if (i == 8) s = s + dt * v[2];
    else if (i >= 9) s = s + dt * v[i - 6];
    return s;
  }
  __device__ __forceinline__ double ma(const double* M, int r, int j) const {  // (M A)_{rj}
    const double* mr = M + 12 * r;
    double s = mr[j];
    if (j == 6) s = (s + mr[0] * ad0) + mr[1] * (-ad1);
    else if (j == 7) s = (s + mr[0] * ad1) + mr[1] * ad0;
    else if (j == 8) s = s + mr[2] * dt;
    else if (j >= 9) s = s + mr[j - 6] * dt;
    return s;
  }
  __device__ __forceinline__ double atm(const double* M, int i, int j) const {  // (A'M)_{ij}
    double s = M[12 * i + j];
    if (i == 6) s = (s + ad0 * M[j]) + (-ad1) * M[12 + j];
    else if (i == 7) s = (s + ad1 * M[j]) + ad0 * M[12 + j];
    else if (i == 8) s = s + dt * M[24 + j];
    else if (i >= 9) s = s + dt * M[12 * (i - 6) + j];
    return s;
  }
  __device__ __forceinline__ double at(int u, int j) const {  // A[u][j]
    if (u == j) return 1.0;
    if (j == 6) return u == 0 ? ad0 : (u == 1 ? -ad1 : 0.0);
    if (j == 7) return u == 0 ? ad1 : (u == 1 ? ad0 : 0.0);
    if (j == 8) return u == 2 ? dt : 0.0;
    if (j >= 9) return u == j - 6 ? dt : 0.0;
    return 0.0;
  }
};

// (M B_k)_{rc} = sum_{s=6..11} M[r][s] B_k[s][c]
template <int N>
__device__ __forceinline__ double mb(const WSmem<N>& sm, const double* M, int k, int r, int c, double dtm) {
  const double* mr = M + 12 * r;
  return ((mr[6] * sm.Bw[k][0][c] + mr[7] * sm.Bw[k][1][c]) + mr[8] * sm.Bw[k][2][c]) + mr[9 + c % 3] * dtm;
}
// (B_k' M)_{ij} = sum_{s=6..11} B_k[s][i] M[s][j]
template <int N>
__device__ __forceinline__ double btm(const WSmem<N>& sm, const double* M, int k, int i, int j, double dtm) {
  return ((sm.Bw[k][0][i] * M[72 + j] + sm.Bw[k][1][i] * M[84 + j]) + sm.Bw[k][2][i] * M[96 + j]) +
         dtm * M[12 * (9 + i % 3) + j];
}

// I_w^-1, I_w = R I_b R' (calculate_B_mat_c, ConvexMpc.cpp:132-138; Eigen's cofactor inverse)
__device__ __forceinline__ void iw_inverse(const double* rec, double (&Iwinv)[9]) {
  const double* R = rec + MPCQP_REC_ROT;
  const double* Ib = rec + MPCQP_REC_INERTIA;
  double tmp[9], Iw[9];
#pragma unroll
  for (int i = 0; i < 3; ++i)
#pragma unroll
    for (int j = 0; j < 3; ++j) {
      double s = 0.0;
#pragma unroll
      for (int k = 0; k < 3; ++k) s += R[i * 3 + k] * Ib[k * 3 + j];
      tmp[i * 3 + j] = s;
    }
#pragma unroll
  for (int i = 0; i < 3; ++i)
#pragma unroll
    for (int j = 0; j < 3; ++j) {
      double s = 0.0;
#pragma unroll
      for (int k = 0; k < 3; ++k) s += tmp[i * 3 + k] * R[j * 3 + k];
      Iw[i * 3 + j] = s;
    }
  auto cof = [&](int i, int j) {
    const int i1 = (i + 1) % 3, i2 = (i + 2) % 3, j1 = (j + 1) % 3, j2 = (j + 2) % 3;
    return Iw[i1 * 3 + j1] * Iw[i2 * 3 + j2] - Iw[i1 * 3 + j2] * Iw[i2 * 3 + j1];
  };
  const double det = (cof(0, 0) * Iw[0] + cof(1, 0) * Iw[3]) + cof(2, 0) * Iw[6];
  const double invdet = 1.0 / det;
#pragma unroll
  for (int i = 0; i < 3; ++i)
#pragma unroll
    for (int j = 0; j < 3; ++j) Iwinv[j * 3 + i] = cof(i, j) * invdet;
}

__device__ __forceinline__ int hidx(int i, int j) { return j * (j + 1) / 2 + i; }  // packed upper, i <= j

// A~'v for the three variables of a leg, from the quad's rows (lane a: row a, v4: row 4).
// Lane a < 3 returns component a.  AK0: row a's coefficient on fx (a < 2) / fy (a >= 2);
// AK1: row a's coefficient on fz; AK4: row 4's coefficient on fz.
__device__ __forceinline__ double quad_at(double v, double v4, double AK0, double AK1, double AK4, int a) {
  const double p0 = AK0 * v, p1 = AK1 * v;
  const double s01 = dpp<QP_02>(p0) + dpp<QP_13>(p0);
  const double tt = p1 + dpp<QP_X1>(p1);
  const double s2 = (tt + dpp<QP_X2>(tt)) + AK4 * v4;
  return a < 2 ? s01 : s2;
}

// ---- factorization of c B'Q̄B + R' (LDS, one wave; R' in F.Rt) ------------------------------------
template <int N>
__device__ void factorize(WSmem<N>& sm, const mpcqp_params& p, const Adisc& A, double c, double dtm) {
  auto& F = sm.u.f;
  const int t = threadIdx.x;
  for (int e = t; e < 144; e += NT) {
    const int i = e / 12, j = e % 12;
    F.P[e] = (i == j) ? c * (2.0 * p.q_weights[i]) : 0.0;
    F.K[0][e] = 0.0;
    F.Acl[0][e] = 0.0;
    F.Acl[N - 1][e] = 0.0;
  }
  wave_sync();
  for (int k = N - 1; k >= 0; --k) {
    for (int e = t; e < 144; e += NT) {  // PB = P B_k, PA = P A
      const int r = e / 12, j = e % 12;
      F.PB[e] = mb(sm, F.P, k, r, j, dtm);
      if (k >= 1) F.PA[e] = A.ma(F.P, r, j);
    }
    wave_sync();
    for (int e = t; e < 144; e += NT) {  // G = R'_k + B_k' PB, F = B_k' PA
      const int i = e / 12, j = e % 12;
      const double rt = (i / 3 == j / 3) ? F.Rt[k][i][j % 3] : 0.0;
      F.Gm[e] = rt + btm(sm, F.PB, k, i, j, dtm);
      if (k >= 1) F.F[e] = btm(sm, F.PA, k, i, j, dtm);
    }
    wave_sync();
    {  // G^-1 by Gauss-Jordan (SPD, no pivoting); entries t, t+64, t+128 (< 144)
      double* G = F.Gm;
      for (int piv = 0; piv < 12; ++piv) {
        const double dinv = 1.0 / G[piv * 12 + piv];
        auto gj = [&](int e) __attribute__((always_inline)) {
          const int i = e / 12, j = e % 12;
          if (i == piv && j == piv) return dinv;
          if (i == piv) return G[piv * 12 + j] * dinv;
          if (j == piv) return -G[i * 12 + piv] * dinv;
          return G[i * 12 + j] - G[i * 12 + piv] * (G[piv * 12 + j] * dinv);
        };
        const double u0 = gj(t), u1 = gj(t + 64);
        const double u2 = t + 128 < 144 ? gj(t + 128) : 0.0;
        wave_sync();
        G[t] = u0;
        G[t + 64] = u1;
        if (t + 128 < 144) G[t + 128] = u2;
        wave_sync();
      }
      for (int e = t; e < 144; e += NT) F.Gi[k][e] = G[e];
    }
    wave_sync();
    if (k >= 1) {
      for (int e = t; e < 144; e += NT) {  // K_k = G^-1 F
        const int i = e / 12, j = e % 12;
        double s = 0.0;
        for (int q = 0; q < 12; ++q) s += F.Gi[k][i * 12 + q] * F.F[q * 12 + j];
        F.K[k][e] = s;
      }
      wave_sync();
      for (int e = t; e < 144; e += NT) {  // Acl_k = A - B_k K_k, P_k = cQ + A'PA - F'K_k
        const int i = e / 12, j = e % 12;
        double bk = 0.0;
        if (i >= 6 && i < 9) {
          for (int q = 0; q < 12; ++q) bk += sm.Bw[k][i - 6][q] * F.K[k][q * 12 + j];
        } else if (i >= 9) {
          const int a = i - 9;
          bk = dtm * (((F.K[k][a * 12 + j] + F.K[k][(3 + a) * 12 + j]) + F.K[k][(6 + a) * 12 + j]) +
                      F.K[k][(9 + a) * 12 + j]);
        }
        if (k <= N - 2) F.Acl[k][e] = A.at(i, j) - bk;
        double fk = 0.0;
        for (int q = 0; q < 12; ++q) fk += F.F[q * 12 + i] * F.K[k][q * 12 + j];
        F.P[e] = (((i == j) ? c * (2.0 * p.q_weights[i]) : 0.0) + A.atm(F.PA, i, j)) - fk;
      }
      wave_sync();
    }
  }
}

// Phase timing (debug builds with -DMPCQP_PHASE_TIMING): lane 0 of each traced robot appends
// {phase id, s_memtime, s_memrealtime (100 MHz), 0} to the trace buffer instead of check records.
#ifdef MPCQP_PHASE_TIMING
#define WV_MARK(id)                                                                     \
  do {                                                                                  \
    if (trace && threadIdx.x == 0 && inst < trace_cap && nmark < MPCQP_TRACE_LEN) {     \
      double* tm_ = trace + ((size_t)inst * MPCQP_TRACE_LEN + nmark) * 4;                \
      tm_[0] = (id);                                                                    \
      tm_[1] = (double)__builtin_readcyclecounter();                                    \
      tm_[2] = (double)__builtin_amdgcn_s_memrealtime();                                \
      ++nmark;                                                                          \
    }                                                                                   \
  } while (0)
#else
#define WV_MARK(id) \
  do {              \
  } while (0)
#endif

template <int N>
__global__ __launch_bounds__(NT, 2) void wave_kernel(const double* __restrict__ recs, int batch,
                                                     mpcqp_result* __restrict__ results,
                                                     double* __restrict__ solution, double* __restrict__ trace,
                                                     int trace_cap, mpcqp_params p) {
  using C = Cfg<N>;
  constexpr int n = C::n, m = C::m, R = C::R;
  __shared__ WSmem<N> sm;
  const int inst = blockIdx.x;
  if (inst >= batch) return;
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
  {
    const double* rg = recs + (size_t)inst * C::REC;
    bool bad = false;
    for (int e = t; e < C::REC; e += NT) {
      const double v = rg[e];
      sm.rec[e] = v;
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
      return;
    }
  }
  wave_sync();
  WV_MARK(1);
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
    // forward: a_i = A_d^{i+1} x0 (13 states), e_i = 2q (a_i - x_ref_i) (ConvexMpc.cpp:215-217)
    if (t < SD) sm.vec[0][t] = rec[MPCQP_REC_X0 + t];
    wave_sync();
    for (int i = 0; i < N; ++i) {
      if (t < SD) {
        const double* pv = sm.vec[i & 1];
        double s;
        if (t == 0) s = (pv[0] + A.ad0 * pv[6]) + A.ad1 * pv[7];
        else if (t == 1) s = (pv[1] + (-A.ad1) * pv[6]) + A.ad0 * pv[7];
        else if (t == 2) s = pv[2] + dt * pv[8];
        else if (t <= 5) s = pv[t] + dt * pv[t + 6];
        else if (t == 11) s = pv[11] + dt * pv[12];
        else s = pv[t];
        sm.vec[(i + 1) & 1][t] = s;
        if (t < ND) sm.lam[i][t] = 2 * p.q_weights[t] * (s - rec[MPCQP_REC_XREF + SD * i + t]);
      }
      wave_sync();
    }
    // backward: lambda_j = e_j + A' lambda_{j+1}
    for (int j = N - 2; j >= 0; --j) {
      if (t < ND) sm.lam[j][t] = sm.lam[j][t] + A.atv(t, sm.lam[j + 1]);
      wave_sync();
    }
  }

  WV_MARK(2);
  // ---- 2. |H| (fp32, packed) from H_jk = B_j' (A')^{k-j} S_k B_k (+ R on the diagonal) -------------
  auto& HS = sm.u.h;
  for (int e = t; e < 144; e += NT) {
    const int i = e / 12, j = e % 12;
    HS.S[e] = (i == j) ? 2 * p.q_weights[i] : 0.0;
  }
  wave_sync();
  for (int k = N - 1; k >= 0; --k) {
    for (int e = t; e < 144; e += NT) HS.G[k][e] = mb(sm, HS.S, k, e / 12, e % 12, dtm);  // G_k = S_k B_k
    if (k >= 1) {
      for (int e = t; e < 144; e += NT) HS.T[e] = A.ma(HS.S, e / 12, e % 12);
      wave_sync();
      for (int e = t; e < 144; e += NT) {
        const int i = e / 12, j = e % 12;
        HS.S[e] = ((i == j) ? 2 * p.q_weights[i] : 0.0) + A.atm(HS.T, i, j);
      }
    }
    wave_sync();
  }
  for (int k = 0; k < N; ++k) {
    const double* V = HS.G[k];  // V_{j,k} = (A')^{k-j} G_k, double-buffered
    int wb = 0;
    for (int j = k; j >= 0; --j) {
      for (int e = t; e < 144; e += NT) {
        const int b = e / 12, aa = e % 12;
        double h = btm(sm, V, j, b, aa, dtm);
        if (j == k && b == aa) h += 2 * p.r_weights[b];
        const int row = ND * j + b, col = ND * k + aa;
        if (row <= col) HS.H32[hidx(row, col)] = (float)dabs(h);
        if (j > 0) HS.V[wb][e] = A.atm(V, b, aa);
      }
      wave_sync();
      V = HS.V[wb];
      wb ^= 1;
    }
  }

  WV_MARK(3);
  // ---- 3. OSQP scale_data (scaling.c) with the scaling deferred: P~ = c D H D is never formed -------
  // Column inf-norms of P~ are (c D_j) max_i D_i |H_ij| (H symmetric), from the fp32 |H|.
  for (int j = t; j < n; j += NT) {
    const int k = j / ND, ii = j % ND;
    const double* lm = sm.lam[k];
    HS.q[j] = ((sm.Bw[k][0][ii] * lm[6] + sm.Bw[k][1][ii] * lm[7]) + sm.Bw[k][2][ii] * lm[8]) + dtm * lm[9 + ii % 3];
    HS.D[j] = 1.0;
    HS.D32[j] = 1.0f;
  }
  for (int r = t; r < m; r += NT) {  // unscaled A rows (ConvexMpc.cpp:46-58)
    const int k5 = r % 5;
    const double az = k5 == 4 ? 0.0 : ((k5 & 1) ? -mu : mu);
    HS.ak[r][0] = k5 < 2 ? 1.0 : 0.0;
    HS.ak[r][1] = (k5 == 2 || k5 == 3) ? 1.0 : 0.0;
    HS.ak[r][2] = k5 < 4 ? az : 1.0;
    HS.E[r] = 1.0;
  }
  wave_sync();
  auto colmax = [&]() __attribute__((always_inline)) {
    for (int j = t; j < n; j += NT) {
      float mx = 0.0f;
      for (int i = 0; i < n; ++i) {
        const float h = HS.H32[i <= j ? hidx(i, j) : hidx(j, i)];
        mx = fmaxf(mx, HS.D32[i] * h);
      }
      HS.cm[j] = (double)mx;
    }
  };
  double c_s = 1.0;
  if (p.scaling > 0) {
    colmax();
    wave_sync();
  }
  for (int pass = 0; pass < p.scaling; ++pass) {
    for (int j = t; j < n; j += NT) {
      const int f = j / 3, aa = j % 3;
      double ca = 0.0;
      for (int k = 0; k < 5; ++k) ca = fmax(ca, dabs(HS.ak[5 * f + k][aa]));
      const double pc = (c_s * HS.D[j]) * HS.cm[j];
      HS.Dt[j] = 1.0 / sqrt(limit_scaling(fmax(pc, ca)));
    }
    wave_sync();
    for (int r = t; r < m; r += NT) {  // A <- E A D
      const int f = r / 5;
      const double et =
          1.0 / sqrt(limit_scaling(fmax(fmax(dabs(HS.ak[r][0]), dabs(HS.ak[r][1])), dabs(HS.ak[r][2]))));
      HS.ak[r][0] = (HS.ak[r][0] * et) * HS.Dt[3 * f];
      HS.ak[r][1] = (HS.ak[r][1] * et) * HS.Dt[3 * f + 1];
      HS.ak[r][2] = (HS.ak[r][2] * et) * HS.Dt[3 * f + 2];
      HS.E[r] *= et;
    }
    for (int j = t; j < n; j += NT) {
      HS.q[j] = HS.Dt[j] * HS.q[j];
      HS.D[j] = HS.D[j] * HS.Dt[j];
      HS.D32[j] = (float)HS.D[j];
    }
    wave_sync();
    colmax();  // column norms of the D-scaled P (cost normalization)
    double sv = 0.0, qv = 0.0;
    for (int j = t; j < n; j += NT) {
      sv += (c_s * HS.D[j]) * HS.cm[j];
      qv = fmax(qv, dabs(HS.q[j]));
    }
    sv = wave_sum(sv);
    qv = wave_max(qv);
    double c_temp = sv / n;
    const double inf_norm_q = limit_scaling(qv);
    c_temp = dmax(c_temp, inf_norm_q);
    c_temp = limit_scaling(c_temp);
    c_temp = 1. / c_temp;
    for (int j = t; j < n; j += NT) HS.q[j] *= c_temp;
    c_s *= c_temp;
    wave_sync();
  }
  const double cost_c = c_s, cinv = 1. / c_s;
  WV_MARK(4);

  // ---- 4. lane registers: variables (D, q~) and rows (E, A~, bounds, rho) — set_rho_vec -----------
  const double rho0 = dmin(dmax(p.rho, RHO_MIN), RHO_MAX);
  double X[R], Qv[R], Dv[R], DI[R], PX[R], PXO[R], DX[R], RHS[R];
  double Z[R], Y[R], DY[R], Ev[R], AK0[R], AK1[R];
  double Z4[R], Y4[R], DY4[R], E4[R], L4[R], U4[R], AK4[R], RHO4[R];
  bool kvr[R], vvr[R];
  const double cont = rec[MPCQP_REC_CONTACTS + leg] != 0.0 ? 1.0 : 0.0;
#pragma unroll
  for (int r = 0; r < R; ++r) {
    const int k = 4 * r + ig;
    const bool kv = k < N, vv = kv && av;
    kvr[r] = kv;
    vvr[r] = vv;
    const int kc = kv ? k : 0;
    const int ci = ND * kc + idx, ri = CD * kc + 5 * leg + a, r4 = CD * kc + 5 * leg + 4;
    Dv[r] = vv ? HS.D[ci] : 1.0;
    DI[r] = 1. / Dv[r];
    Qv[r] = vv ? HS.q[ci] : 0.0;
    Ev[r] = kv ? HS.E[ri] : 1.0;
    E4[r] = kv ? HS.E[r4] : 1.0;
    AK0[r] = kv ? HS.ak[ri][a >> 1] : 0.0;
    AK1[r] = kv ? HS.ak[ri][2] : 0.0;
    AK4[r] = kv ? HS.ak[r4][2] : 0.0;
    // bounds (ConvexMpc.cpp:223-245), clipped to +-OSQP_INFTY, scaled by E
    double l4 = rec[MPCQP_REC_FZMIN] * cont, u4 = rec[MPCQP_REC_FZMAX] * cont;
    l4 = dmin(dmax(l4, -OSQP_INF), OSQP_INF);
    u4 = dmin(dmax(u4, -OSQP_INF), OSQP_INF);
    L4[r] = E4[r] * l4;
    U4[r] = E4[r] * u4;
    X[r] = 0.0; PX[r] = 0.0; PXO[r] = 0.0; DX[r] = 0.0;
    Z[r] = 0.0; Y[r] = 0.0; DY[r] = 0.0; Z4[r] = 0.0; Y4[r] = 0.0; DY4[r] = 0.0;
    RHS[r] = vv ? sigma * 0.0 - Qv[r] : 0.0;  // cold start: compute_rhs with x = z = y = 0
  }
  auto rho4_of = [&](int r, double rho) __attribute__((always_inline)) {
    const bool loose = L4[r] < -OSQP_INF * MIN_SCALING && U4[r] > OSQP_INF * MIN_SCALING;
    const bool eq = U4[r] - L4[r] < RHO_TOL;
    return loose ? RHO_MIN : (eq ? RHO_EQ_OVER_RHO_INEQ * rho : rho);
  };
#pragma unroll
  for (int r = 0; r < R; ++r) RHO4[r] = rho4_of(r, rho0);
  // rows 0-3: l = 0 / u = +inf (rows 0, 2) or l = -inf / u = 0 (rows 1, 3): always inequalities
  auto lo03 = [&](int r) __attribute__((always_inline)) { return (a & 1) ? Ev[r] * -OSQP_INF : Ev[r] * 0.0; };
  auto hi03 = [&](int r) __attribute__((always_inline)) { return (a & 1) ? Ev[r] * 0.0 : Ev[r] * OSQP_INF; };
  wave_sync();  // every LDS read of the setup image precedes its reuse by the factorization

  // ---- 5. ADMM (osqp_solve) ------------------------------------------------------------------------
  auto& F = sm.u.f;
  double rho = rho0, pri_res = 0.0, dua_res = 0.0;
  int status = MPCQP_STATUS_UNSOLVED, iters = 0, rho_updates = 0, ntrace = 0;
  bool need_factor = true;
  int to_check = p.check_termination, to_adapt = p.adaptive_rho_interval;
  for (int iter = 1; iter <= p.max_iter; ++iter) {
    if (need_factor) {
      WV_MARK(10);
      // R'_k foot blocks: c 2r + D^-1 (sigma I + A~' diag(rho) A~) D^-1
#pragma unroll
      for (int r = 0; r < R; ++r) {
        const double k00 = dpp<QP_B0>(AK0[r]), k01 = dpp<QP_B1>(AK0[r]), k02 = dpp<QP_B2>(AK0[r]),
                     k03 = dpp<QP_B3>(AK0[r]);
        const double k10 = dpp<QP_B0>(AK1[r]), k11 = dpp<QP_B1>(AK1[r]), k12 = dpp<QP_B2>(AK1[r]),
                     k13 = dpp<QP_B3>(AK1[r]);
        const double d0 = dpp<QP_B0>(Dv[r]), d1 = dpp<QP_B1>(Dv[r]), d2 = dpp<QP_B2>(Dv[r]);
        const double ak4 = AK4[r], r4 = RHO4[r];
        // rows of the foot: r0 [k00,0,k10] r1 [k01,0,k11] r2 [0,k02,k12] r3 [0,k03,k13] r4 [0,0,ak4]
        auto coef = [&](int row, int col) __attribute__((always_inline)) {
          if (row == 4) return col == 2 ? ak4 : 0.0;
          const double kp = row == 0 ? k00 : row == 1 ? k01 : row == 2 ? k02 : k03;
          const double kz = row == 0 ? k10 : row == 1 ? k11 : row == 2 ? k12 : k13;
          if (col == 2) return kz;
          return (col == (row >> 1)) ? kp : 0.0;
        };
        const int k = 4 * r + ig;
        const double da = a == 0 ? d0 : (a == 1 ? d1 : d2);
#pragma unroll
        for (int b = 0; b < 3; ++b) {
          double s = 0.0;
#pragma unroll
          for (int row = 0; row < 5; ++row) s += (coef(row, av ? a : 2) * (row == 4 ? r4 : rho)) * coef(row, b);
          const double db = b == 0 ? d0 : (b == 1 ? d1 : d2);
          const double rt = (av && a == b ? cost_c * (2.0 * p.r_weights[idx]) : 0.0) +
                            ((1.0 / da) * ((av && a == b ? sigma : 0.0) + s)) * (1.0 / db);
          if (kvr[r] && av) F.Rt[k][idx][b] = rt;
        }
      }
      wave_sync();
      factorize<N>(sm, p, A, cost_c, dtm);
      wave_sync();
      need_factor = false;
      WV_MARK(12);
    }

    // ---- KKT solve: u = (c B'Q̄B + R')^-1 D^-1 rhs, x~ = D^-1 u ----
    double U[R];
    const bool tm_it = iter == 60;
    if (tm_it) WV_MARK(40);
    {
      double W[R], AKw[R], BKw[R], SMv[R], G[R], Hh[R], XS[R];
#pragma unroll
      for (int r = 0; r < R; ++r) {
        W[r] = DI[r] * RHS[r];
        SMv[r] = 0.0;
        XS[r] = 0.0;
      }
#pragma unroll
      for (int r = 0; r < R; ++r) {  // a_k = K_k' w_k, b_k = G_k^-1 w_k
        const int kc = min(4 * r + ig, N - 1);
        double c[12];
        ld12s(c, &F.K[kc][idx]);
        AKw[r] = mv12(W[r], c);
        ld12(c, &F.Gi[kc][12 * idx]);
        BKw[r] = mv12(W[r], c);
      }
      if (tm_it) WV_MARK(41);
      {  // backward chain: s_{N-1} = -a_{N-1}; s_k = Acl_k' s_{k+1} - a_k; SMv (row of k) = s_{k+1}
        double cur = -AKw[(N - 1) >> 2];
        sfor<0, N - 1>([&](auto J) {
          constexpr int k = N - 2 - decltype(J)::value;
          const double mvv = rmove<row_of(k + 1), row_of(k)>(cur);
          SMv[k >> 2] = (q == row_of(k)) ? mvv : SMv[k >> 2];
          if constexpr (k >= 1) {
            double c[12];
            ld12s(c, &F.Acl[k][idx]);
            cur = mv12(mvv, c) - AKw[k >> 2];
          }
        });
      }
      if (tm_it) WV_MARK(42);
#pragma unroll
      for (int r = 0; r < R; ++r) {  // g_k = b_k + G_k^-1 B_k' s_{k+1}; h_k = B_k g_k
        const int kc = min(4 * r + ig, N - 1);
        const double c6[6] = {sm.Bw[kc][0][idx], sm.Bw[kc][1][idx], sm.Bw[kc][2][idx],
                              a == 0 ? dtm : 0.0, a == 1 ? dtm : 0.0, a == 2 ? dtm : 0.0};
        const double tt = mv6(SMv[r], c6);
        double c[12];
        ld12(c, &F.Gi[kc][12 * idx]);
        G[r] = BKw[r] + mv12(tt, c);
        ld12(c, &sm.Bw[kc][av ? a : 2][0]);
#pragma unroll
        for (int cc = 0; cc < 12; ++cc)
          c[cc] = (leg == 2 && av) ? c[cc] : ((leg == 3 && av && cc % 3 == a) ? dtm : 0.0);
        Hh[r] = mv12(G[r], c);
      }
      if (tm_it) WV_MARK(43);
      {  // forward chain: x_1 = h_0; x_{k+1} = Acl_k x_k + h_k; XS (row of k) = x_k
        double cur = Hh[0];
        sfor<1, N>([&](auto K) {
          constexpr int k = decltype(K)::value;
          const double mvv = rmove<row_of(k - 1), row_of(k)>(cur);
          XS[k >> 2] = (q == row_of(k)) ? mvv : XS[k >> 2];
          if constexpr (k <= N - 2) {
            double c[12];
            ld12(c, &F.Acl[k][12 * idx]);
            cur = mv12(mvv, c) + Hh[k >> 2];
          }
        });
      }
      if (tm_it) WV_MARK(44);
#pragma unroll
      for (int r = 0; r < R; ++r) {  // u_k = g_k - K_k x_k
        const int kc = min(4 * r + ig, N - 1);
        double c[12];
        ld12(c, &F.K[kc][12 * idx]);
        U[r] = G[r] - mv12(XS[r], c);
      }
    }
    if (tm_it) WV_MARK(45);

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
    const double rinv = 1. / rho;
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const double xt = DI[r] * U[r];
      const double xp = dpp<QP_PRIM>(xt), xz = dpp<QP_B2>(xt);
      const double zt = AK0[r] * xp + AK1[r] * xz;
      const double zt4 = AK4[r] * xz;
      {
        const double zr = alpha * zt + (1.0 - alpha) * Z[r];
        const double zn = dmin(dmax(zr + rinv * Y[r], lo03(r)), hi03(r));
        const double dyv = rho * (zr - zn);
        Z[r] = zn;
        Y[r] = Y[r] + dyv;
        DY[r] = dyv;
      }
      {
        const double r4 = RHO4[r];
        const double zr = alpha * zt4 + (1.0 - alpha) * Z4[r];
        const double zn = dmin(dmax(zr + (1. / r4) * Y4[r], L4[r]), U4[r]);
        const double dyv = r4 * (zr - zn);
        Z4[r] = zn;
        Y4[r] = Y4[r] + dyv;
        DY4[r] = dyv;
      }
      const double kd = quad_at(rho * zt, RHO4[r] * zt4, AK0[r], AK1[r], AK4[r], a);
      if (vvr[r]) {
        const double xo = X[r];
        const double xn = alpha * xt + (1.0 - alpha) * xo;
        DX[r] = xn - xo;
        X[r] = xn;
        const double pxt = (RHS[r] - sigma * xt) - kd;
        PXO[r] = PX[r];
        PX[r] = alpha * pxt + (1.0 - alpha) * PX[r];
      }
    }

    if (tm_it) WV_MARK(46);
    if (need_info) {
      // ---- update_info / check_termination / adapt_rho (osqp.c, auxil.c) ----
      double mx[14];
#pragma unroll
      for (int k = 0; k < 14; ++k) mx[k] = 0.0;
#pragma unroll
      for (int r = 0; r < R; ++r) {
        const double xp = dpp<QP_PRIM>(X[r]), xz = dpp<QP_B2>(X[r]);
        const double ax = AK0[r] * xp + AK1[r] * xz, ax4 = AK4[r] * xz;
        const double aty = quad_at(Y[r], Y4[r], AK0[r], AK1[r], AK4[r], a);
        if (kvr[r]) {
          const double ei = 1.0 / Ev[r], ei4 = 1.0 / E4[r];
          const double pr = ax + (-1.0) * Z[r], pr4 = ax4 + (-1.0) * Z4[r];
          mx[0] = dmax(mx[0], dmax(dabs(ei * pr), dabs(ei4 * pr4)));
          mx[1] = dmax(mx[1], dmax(dabs(pr), dabs(pr4)));
          mx[2] = dmax(mx[2], dmax(dabs(ei * Z[r]), dabs(ei4 * Z4[r])));
          mx[3] = dmax(mx[3], dmax(dabs(Z[r]), dabs(Z4[r])));
          mx[4] = dmax(mx[4], dmax(dabs(ei * ax), dabs(ei4 * ax4)));
          mx[5] = dmax(mx[5], dmax(dabs(ax), dabs(ax4)));
        }
        if (vvr[r]) {
          const double d = (Qv[r] + 1.0 * PX[r]) + 1.0 * aty;
          mx[6] = dmax(mx[6], dabs(DI[r] * d));
          mx[7] = dmax(mx[7], dabs(d));
          mx[8] = dmax(mx[8], dabs(DI[r] * Qv[r]));
          mx[9] = dmax(mx[9], dabs(Qv[r]));
          mx[10] = dmax(mx[10], dabs(DI[r] * aty));
          mx[11] = dmax(mx[11], dabs(aty));
          mx[12] = dmax(mx[12], dabs(DI[r] * PX[r]));
          mx[13] = dmax(mx[13], dabs(PX[r]));
        }
      }
#pragma unroll
      for (int k = 0; k < 14; ++k) mx[k] = wave_max(mx[k]);
      pri_res = mx[0];
      dua_res = cinv * mx[6];
      iters = iter;
      auto check = [&](bool approx) __attribute__((always_inline)) -> int {
        double eps_abs = p.eps_abs, eps_rel = p.eps_rel, eps_pinf = p.eps_prim_inf, eps_dinf = p.eps_dual_inf;
        if (pri_res > OSQP_INF || dua_res > OSQP_INF) return MPCQP_STATUS_NON_CVX;
        if (approx) { eps_abs *= 10; eps_rel *= 10; eps_pinf *= 10; eps_dinf *= 10; }
        const double eps_prim = eps_abs + eps_rel * dmax(mx[2], mx[4]);
        const bool prim_ok = pri_res < eps_prim;
        bool prim_inf = false, dual_inf = false;
        if (!prim_ok) {
          // is_primal_infeasible: delta_y projected onto the polar of the recession cone
          double nd = 0.0, lh = 0.0, dyp[R], dyp4[R];
#pragma unroll
          for (int r = 0; r < R; ++r) {
            auto proj = [&](double d, double lo, double hi) __attribute__((always_inline)) {
              if (hi > OSQP_INF * MIN_SCALING) {
                if (lo < -OSQP_INF * MIN_SCALING) d = 0.0;
                else d = dmin(d, 0.0);
              } else if (lo < -OSQP_INF * MIN_SCALING) {
                d = dmax(d, 0.0);
              }
              return d;
            };
            const double lo = lo03(r), hi = hi03(r);
            const double d = proj(DY[r], lo, hi), d4 = proj(DY4[r], L4[r], U4[r]);
            dyp[r] = d;
            dyp4[r] = d4;
            if (kvr[r]) {
              nd = dmax(nd, dmax(dabs(Ev[r] * d), dabs(E4[r] * d4)));
              lh += hi * dmax(d, 0.0) + lo * dmin(d, 0.0);
              if (a == 0) lh += U4[r] * dmax(d4, 0.0) + L4[r] * dmin(d4, 0.0);
            }
          }
          const double ndy = wave_max(nd);
          if (ndy > DIV_TOL) {
            lh = wave_sum(lh);
            if (lh < eps_pinf * ndy) {
              double an = 0.0;
#pragma unroll
              for (int r = 0; r < R; ++r) {
                const double atd = quad_at(dyp[r], dyp4[r], AK0[r], AK1[r], AK4[r], a);
                if (vvr[r]) an = dmax(an, dabs(DI[r] * atd));
              }
              an = wave_max(an);
              prim_inf = an < eps_pinf * ndy;
            }
          }
        }
        const double eps_dual = eps_abs + eps_rel * (cinv * dmax(dmax(mx[8], mx[10]), mx[12]));
        const bool dual_ok = dua_res < eps_dual;
        if (!dual_ok) {
          // is_dual_infeasible (P~ delta_x = P~x_new - P~x_old)
          double nx = 0.0, qd = 0.0;
#pragma unroll
          for (int r = 0; r < R; ++r)
            if (vvr[r]) {
              nx = dmax(nx, dabs(Dv[r] * DX[r]));
              qd += Qv[r] * DX[r];
            }
          const double ndx = wave_max(nx);
          if (ndx > DIV_TOL) {
            qd = wave_sum(qd);
            if (qd < cost_c * eps_dinf * ndx) {
              double pd = 0.0;
#pragma unroll
              for (int r = 0; r < R; ++r)
                if (vvr[r]) pd = dmax(pd, dabs(DI[r] * (PX[r] - PXO[r])));
              pd = wave_max(pd);
              if (pd < cost_c * eps_dinf * ndx) {
                double viol = 0.0;
#pragma unroll
                for (int r = 0; r < R; ++r) {
                  const double dp = dpp<QP_PRIM>(DX[r]), dz = dpp<QP_B2>(DX[r]);
                  const double v = (1.0 / Ev[r]) * (AK0[r] * dp + AK1[r] * dz);
                  const double v4 = (1.0 / E4[r]) * (AK4[r] * dz);
                  const double lo = lo03(r), hi = hi03(r);
                  if (kvr[r]) {
                    if ((hi < OSQP_INF * MIN_SCALING && v > eps_dinf * ndx) ||
                        (lo > -OSQP_INF * MIN_SCALING && v < -eps_dinf * ndx))
                      viol = 1.0;
                    if ((U4[r] < OSQP_INF * MIN_SCALING && v4 > eps_dinf * ndx) ||
                        (L4[r] > -OSQP_INF * MIN_SCALING && v4 < -eps_dinf * ndx))
                      viol = 1.0;
                  }
                }
                viol = wave_max(viol);
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
#ifndef MPCQP_PHASE_TIMING
      if (trace && t == 0 && inst < trace_cap && ntrace < MPCQP_TRACE_LEN && is_check) {
        double* tp = trace + ((size_t)inst * MPCQP_TRACE_LEN + ntrace) * 4;
        tp[0] = iter; tp[1] = pri_res; tp[2] = dua_res; tp[3] = rho;
      }
#endif
      ntrace += is_check ? 1 : 0;
      if (done) break;
      if (refactor) {
#pragma unroll
        for (int r = 0; r < R; ++r) RHO4[r] = rho4_of(r, rho);
        need_factor = true;
      }
    }
    // ---- next right-hand side: sigma x - q~ + A~'(rho z - y) ----
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const double at = quad_at(rho * Z[r] - Y[r], RHO4[r] * Z4[r] - Y4[r], AK0[r], AK1[r], AK4[r], a);
      RHS[r] = vvr[r] ? (sigma * X[r] - Qv[r]) + at : 0.0;
    }
    if (tm_it) WV_MARK(47);
  }

  WV_MARK(20);
  // ---- 6. store_solution + unscale + compute_grf extraction (A1RobotControl.cpp:555-561) --------
  const bool has_sol = status != MPCQP_STATUS_PRIMAL_INFEASIBLE &&
                       status != MPCQP_STATUS_PRIMAL_INFEASIBLE_INACCURATE &&
                       status != MPCQP_STATUS_DUAL_INFEASIBLE &&
                       status != MPCQP_STATUS_DUAL_INFEASIBLE_INACCURATE && status != MPCQP_STATUS_NON_CVX;
  double ob = 0.0;
#pragma unroll
  for (int r = 0; r < R; ++r)
    if (vvr[r]) ob += 0.5 * X[r] * PX[r] + Qv[r] * X[r];
  ob = wave_sum(ob);
  double xs0 = 0.0;
#pragma unroll
  for (int r = 0; r < R; ++r) {
    const double xs = has_sol ? Dv[r] * X[r] : NAN;
    if (r == 0) xs0 = xs;
    if (solution && vvr[r]) solution[(size_t)inst * n + ND * (4 * r + ig) + idx] = xs;
  }
  // u0 = step 0 = round 0, DPP row 0 (lanes 0..15); f_i = R^T u0[3i:3i+3], NaN legs skipped
  mpcqp_result* res = results + inst;
  const double u00 = dpp<QP_B0>(xs0), u01 = dpp<QP_B1>(xs0), u02 = dpp<QP_B2>(xs0);
  const double nrm = sqrt(u00 * u00 + u01 * u01 + u02 * u02);
  const bool nanleg = isnan(nrm);
  const unsigned long long nanmask = __ballot(q == 0 && a == 0 && nanleg);
  if (q == 0 && av) {
    const double* Rm = rec + MPCQP_REC_ROT;
    double s = 0.0;
    s += Rm[0 * 3 + a] * u00;
    s += Rm[1 * 3 + a] * u01;
    s += Rm[2 * 3 + a] * u02;
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

template <int N>
static hipError_t launch_wave(const LaunchArgs& a) {
  hipLaunchKernelGGL((wv::wave_kernel<N>), dim3(a.batch), dim3(wv::NT), 0, (hipStream_t)a.stream, a.recs, a.batch,
                     a.results, a.solution, a.trace, a.trace_cap, a.p);
  return hipGetLastError();
}
template <int N>
static hipError_t occupancy_wave(int* blocks) {
  return hipOccupancyMaxActiveBlocksPerMultiprocessor(blocks, wv::wave_kernel<N>, wv::NT, 0);
}

#define MPCQP_WAVE_FOR_EACH_N(X) X(1) X(2) X(3) X(4) X(5) X(6) X(7) X(8) X(9) X(10)

hipError_t launch_wave_any(const LaunchArgs& a) {
  switch (a.p.horizon) {
#define CASE(K) \
  case K: return launch_wave<K>(a);
    MPCQP_WAVE_FOR_EACH_N(CASE)
#undef CASE
    default: return hipErrorInvalidValue;
  }
}
hipError_t occupancy_wave_any(int horizon, int* blocks) {
  switch (horizon) {
#define CASE(K) \
  case K: return occupancy_wave<K>(blocks);
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
