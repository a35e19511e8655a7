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

// Warm-start slot of one robot (binary64, caller-owned device memory): everything the reference's
// persistent OsqpEigen solver carries from one tick to the next.  Scaled quantities are stored as
// the kernel used them; the zero pattern of H's upper triangle (one bit per entry, MW words per
// column) and the friction coefficient mu the constraint matrix was built with decide between
// osqp_update_P and OsqpEigen's re-init on the next tick.
template <int N>
struct WarmLayout {
  static constexpr int n = ND * N, m = CD * N, MW = (n + 63) / 64;
  static constexpr int FLAG = 0, RHO = 1, C = 2, MU = 3, D = 4, E = D + n, QT = E + m, AK = QT + n, X = AK + 2 * m,
                       Z = X + n, Y = Z + m, MASK = Y + m, SIZE = MASK + MW * n;
  static_assert(SIZE == warm_state_doubles(N), "warm-start slot layout");
};

template <int N>
struct WSmem {
  using C = Cfg<N>;
  static constexpr int NK = N > 1 ? N - 1 : 1;  // K_k stored for k = 1..N-1
  static constexpr int NA = N > 2 ? N - 2 : 1;  // Acl_k stored for k = 1..N-2
  alignas(16) double Bw[N][3][ND];  // rows 6-8 of B_d(k) = I_w^-1 skew(foot) dt (rows 9-11: dt/m I)
  union U {
    struct Hs {  // setup: record, Ruiz vectors
      double rec[C::REC];
      double D[C::n], Dt[C::n], q[C::n], E[C::m];
      double lam[N][ND];  // gradient adjoint lambda_k (states 0..11)
      double vec[2][16];  // sequential 13-vectors (gradient forward sweep)
      double Ap[2][C::m];  // unscaled A entries per row: [0] on fx / fy (rows 0-3), [1] on fz
      double qn[C::n];     // this tick's gradient (warm start: q of the Ruiz passes is the old one)
    } h;
    struct Fs {  // solve: per-step factors (the factorization itself runs in registers)
      alignas(16) double Gi[N][144];
      alignas(16) double K[NK][144];
      alignas(16) double Acl[NA][144];
      double Rt[N][4][6];             // R'_k foot blocks, upper triangle (00 01 02 11 12 22)
    } f;
  } u;
};

// ---- cross-lane primitives ---------------------------------------------------------------------
#define WV_FM(A, M, L) "v_fmac_f64_dpp " A ", %[x], " M " row_newbcast:" #L " row_mask:0xf bank_mask:0xf\n\t"
// y_i = sum_c M[i][c] x_c, x_c broadcast from lane 4(c/3)+c%3 of each DPP row, M row i in `c`.
// Hazards (the compiler cannot see into the asm): a DPP instruction needs 2 wait states after a
// VALU write of ANY of its VGPR operands and 5 after an EXEC write.  Hence the leading s_nop 4 and
// three accumulators in rotation (each is re-read 3 instructions after it was written).
__device__ __forceinline__ double mv12(double x, const double (&c)[12]) {
  double a0 = 0.0, a1 = 0.0, a2 = 0.0;
  asm("s_nop 4\n\t"
      WV_FM("%[a0]", "%[c0]", 0) WV_FM("%[a1]", "%[c1]", 1) WV_FM("%[a2]", "%[c2]", 2)
      WV_FM("%[a0]", "%[c3]", 4) WV_FM("%[a1]", "%[c4]", 5) WV_FM("%[a2]", "%[c5]", 6)
      WV_FM("%[a0]", "%[c6]", 8) WV_FM("%[a1]", "%[c7]", 9) WV_FM("%[a2]", "%[c8]", 10)
      WV_FM("%[a0]", "%[c9]", 12) WV_FM("%[a1]", "%[c10]", 13) WV_FM("%[a2]", "%[c11]", 14)
      : [a0] "+v"(a0), [a1] "+v"(a1), [a2] "+v"(a2)
      : [x] "v"(x), [c0] "v"(c[0]), [c1] "v"(c[1]), [c2] "v"(c[2]), [c3] "v"(c[3]), [c4] "v"(c[4]),
        [c5] "v"(c[5]), [c6] "v"(c[6]), [c7] "v"(c[7]), [c8] "v"(c[8]), [c9] "v"(c[9]), [c10] "v"(c[10]),
        [c11] "v"(c[11]));
  return (a0 + a1) + a2;
}
// sum over states 6..11 (lanes 8, 9, 10, 12, 13, 14) of c[s-6] x_s
__device__ __forceinline__ double mv6(double x, const double (&c)[6]) {
  double a0 = 0.0, a1 = 0.0, a2 = 0.0;
  asm("s_nop 4\n\t"
      WV_FM("%[a0]", "%[c0]", 8) WV_FM("%[a1]", "%[c1]", 9) WV_FM("%[a2]", "%[c2]", 10)
      WV_FM("%[a0]", "%[c3]", 12) WV_FM("%[a1]", "%[c4]", 13) WV_FM("%[a2]", "%[c5]", 14)
      : [a0] "+v"(a0), [a1] "+v"(a1), [a2] "+v"(a2)
      : [x] "v"(x), [c0] "v"(c[0]), [c1] "v"(c[1]), [c2] "v"(c[2]), [c3] "v"(c[3]), [c4] "v"(c[4]),
        [c5] "v"(c[5]));
  return (a0 + a1) + a2;
}
// Two / three independent mat-vecs interleaved in one block (each has its own x and rows); every
// accumulator is re-read 4 (x2) or 6 (x3) instructions after its last write.
#define WV_T2(L, I, J) WV_FX("%[a" #J "]", "%[x0]", "%[p" #I "]", L) WV_FX("%[b" #J "]", "%[x1]", "%[q" #I "]", L)
#define WV_T3(L, I, J) WV_T2(L, I, J) WV_FX("%[d" #J "]", "%[x2]", "%[r" #I "]", L)
#define WV_FX(A, X, M, L) "v_fmac_f64_dpp " A ", " X ", " M " row_newbcast:" #L " row_mask:0xf bank_mask:0xf\n\t"
#define WV_OPS12(P, C) [P##0] "v"(C[0]), [P##1] "v"(C[1]), [P##2] "v"(C[2]), [P##3] "v"(C[3]), [P##4] "v"(C[4]), \
    [P##5] "v"(C[5]), [P##6] "v"(C[6]), [P##7] "v"(C[7]), [P##8] "v"(C[8]), [P##9] "v"(C[9]),                \
    [P##10] "v"(C[10]), [P##11] "v"(C[11])
__device__ __forceinline__ void mv12x2(double x0, double x1, const double (&c0)[12], const double (&c1)[12],
                                       double& y0, double& y1) {
  double a0 = 0.0, a1 = 0.0, b0 = 0.0, b1 = 0.0;
  asm("s_nop 4\n\t"
      WV_T2(0, 0, 0) WV_T2(1, 1, 1) WV_T2(2, 2, 0) WV_T2(4, 3, 1) WV_T2(5, 4, 0) WV_T2(6, 5, 1)
      WV_T2(8, 6, 0) WV_T2(9, 7, 1) WV_T2(10, 8, 0) WV_T2(12, 9, 1) WV_T2(13, 10, 0) WV_T2(14, 11, 1)
      : [a0] "+v"(a0), [a1] "+v"(a1), [b0] "+v"(b0), [b1] "+v"(b1)
      : [x0] "v"(x0), [x1] "v"(x1), WV_OPS12(p, c0), WV_OPS12(q, c1));
  y0 = a0 + a1;
  y1 = b0 + b1;
}
__device__ __forceinline__ void mv12x3(double x0, double x1, double x2, const double (&c0)[12],
                                       const double (&c1)[12], const double (&c2)[12], double& y0, double& y1,
                                       double& y2) {
  double a0 = 0.0, a1 = 0.0, b0 = 0.0, b1 = 0.0, d0 = 0.0, d1 = 0.0;
  asm("s_nop 4\n\t"
      WV_T3(0, 0, 0) WV_T3(1, 1, 1) WV_T3(2, 2, 0) WV_T3(4, 3, 1) WV_T3(5, 4, 0) WV_T3(6, 5, 1)
      WV_T3(8, 6, 0) WV_T3(9, 7, 1) WV_T3(10, 8, 0) WV_T3(12, 9, 1) WV_T3(13, 10, 0) WV_T3(14, 11, 1)
      : [a0] "+v"(a0), [a1] "+v"(a1), [b0] "+v"(b0), [b1] "+v"(b1), [d0] "+v"(d0), [d1] "+v"(d1)
      : [x0] "v"(x0), [x1] "v"(x1), [x2] "v"(x2), WV_OPS12(p, c0), WV_OPS12(q, c1), WV_OPS12(r, c2));
  y0 = a0 + a1;
  y1 = b0 + b1;
  y2 = d0 + d1;
}
#undef WV_T2
#undef WV_T3
#undef WV_FX
#undef WV_OPS12
// y[r] = M_r x[r] for the R register rounds of a parallel phase, interleaved.
template <int R>
__device__ __forceinline__ void mv_rounds(const double (&x)[R], const double (&c)[R][12], double (&y)[R]) {
  if constexpr (R == 1) {
    y[0] = mv12(x[0], c[0]);
  } else if constexpr (R == 2) {
    mv12x2(x[0], x[1], c[0], c[1], y[0], y[1]);
  } else if constexpr (R == 3) {
    mv12x3(x[0], x[1], x[2], c[0], c[1], c[2], y[0], y[1], y[2]);
  } else {
#pragma unroll
    for (int r = 0; r < R; ++r) y[r] = mv12(x[r], c[r]);
  }
}
// init + sum_c M[c] x_c: the chains' "- a_k" / "+ h_k" folded into the first accumulator
__device__ __forceinline__ double mv12a(double x, const double (&c)[12], double init) {
  double a0 = init, a1 = 0.0, a2 = 0.0;
  asm("s_nop 4\n\t"
      WV_FM("%[a1]", "%[c1]", 1) WV_FM("%[a2]", "%[c2]", 2) WV_FM("%[a0]", "%[c0]", 0)
      WV_FM("%[a1]", "%[c4]", 5) WV_FM("%[a2]", "%[c5]", 6) WV_FM("%[a0]", "%[c3]", 4)
      WV_FM("%[a1]", "%[c7]", 9) WV_FM("%[a2]", "%[c8]", 10) WV_FM("%[a0]", "%[c6]", 8)
      WV_FM("%[a1]", "%[c10]", 13) WV_FM("%[a2]", "%[c11]", 14) WV_FM("%[a0]", "%[c9]", 12)
      : [a0] "+v"(a0), [a1] "+v"(a1), [a2] "+v"(a2)
      : [x] "v"(x), [c0] "v"(c[0]), [c1] "v"(c[1]), [c2] "v"(c[2]), [c3] "v"(c[3]), [c4] "v"(c[4]),
        [c5] "v"(c[5]), [c6] "v"(c[6]), [c7] "v"(c[7]), [c8] "v"(c[8]), [c9] "v"(c[9]), [c10] "v"(c[10]),
        [c11] "v"(c[11]));
  return (a1 + a2) + a0;
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

// rmove without register copies: one permlane swap per dword (the source's other rows are
// clobbered, the result's other rows are undefined).
template <int FROM, int TO>
__device__ __forceinline__ double rmove2(double v) {
  static_assert((FROM ^ TO) == 1 || (FROM ^ TO) == 2, "rows must differ in one bit");
  unsigned lo = (unsigned)__double2loint(v), hi = (unsigned)__double2hiint(v), ol, oh;
  if constexpr ((FROM ^ TO) == 1) {
    if constexpr (FROM < TO)  // vdst.odd <- src.even
      asm volatile("s_nop 1\n\tv_permlane16_swap_b32 %0, %2\n\tv_permlane16_swap_b32 %1, %3"
                   : "=&v"(ol), "=&v"(oh), "+v"(lo), "+v"(hi));
    else  // src.even <- vdst.odd
      asm volatile("s_nop 1\n\tv_permlane16_swap_b32 %2, %0\n\tv_permlane16_swap_b32 %3, %1"
                   : "=&v"(ol), "=&v"(oh), "+v"(lo), "+v"(hi));
  } else {
    if constexpr (FROM < TO)  // vdst rows 2-3 <- src rows 0-1
      asm volatile("s_nop 1\n\tv_permlane32_swap_b32 %0, %2\n\tv_permlane32_swap_b32 %1, %3"
                   : "=&v"(ol), "=&v"(oh), "+v"(lo), "+v"(hi));
    else  // src rows 0-1 <- vdst rows 2-3
      asm volatile("s_nop 1\n\tv_permlane32_swap_b32 %2, %0\n\tv_permlane32_swap_b32 %3, %1"
                   : "=&v"(ol), "=&v"(oh), "+v"(lo), "+v"(hi));
  }
  return __hiloint2double((int)oh, (int)ol);
}
// sum of a lane's value over the four quads of its DPP row (component a of every leg)
__device__ __forceinline__ double legsum(double v) {
  v = v + dpp<0x128>(v);  // row_ror:8
  return v + dpp<0x124>(v);  // row_ror:4
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

// index of (r, c) in a symmetric 3x3 stored as its upper triangle 00 01 02 11 12 22
__device__ __forceinline__ int sym6(int r, int c) {
  const int lo = r < c ? r : c, hi = r < c ? c : r;
  return lo == 0 ? hi : (lo == 1 ? 2 + hi : 5);
}

// ---- factorization on the matrix cores -------------------------------------------------------------
// Every 12x12 product of the Riccati step runs as 16x16 (zero-padded) v_mfma_f64_16x16x4f64 (IEEE
// binary64 FMAs).  Matrices live in the MFMA result ("D") layout: lane j + 16 g, register v holds
// row 4v + g, column j.  In that layout register kb of a matrix X is exactly the B operand of K-block
// kb (X[4kb + kk][j] at lane j + 16 kk) and the A operand of K-block kb of X' (X'[i][4kb + kk] at
// lane i + 16 kk), so products chain without any data movement: C = A X takes A' and X in D layout.
typedef double mf4 __attribute__((ext_vector_type(4)));

struct Dm {  // a 16x16 matrix in D layout
  mf4 r;
};
// C (+)= (Aᵀ given as `at`)ᵀ X over K-blocks KB0..KB1-1
template <int KB0, int KB1>
__device__ __forceinline__ mf4 mfma_chain(const mf4& at, const mf4& x, mf4 c) {
#pragma unroll
  for (int kb = KB0; kb < KB1; ++kb) c = __builtin_amdgcn_mfma_f64_16x16x4f64(at[kb], x[kb], c, 0, 0, 0);
  return c;
}
// value of lane group GP (same lane within the group) in every group
template <int GP>
__device__ __forceinline__ double bcast_group(double x) {
  const int g = threadIdx.x >> 4;
  const double y = xor16(x);  // group g ^ 1
  const double z = ((g & 1) == (GP & 1)) ? x : y;
  const double w = xor32(z);  // group g ^ 2
  return ((g & 2) == (GP & 2)) ? z : w;
}
// lane L of the lane's DPP row (exact: 0 + 1 * x; a -0 becomes +0).  Used only in straight-line
// code without EXEC writes, so the DPP source hazard needs 2 wait states, not 5.
template <int L>
__device__ __forceinline__ double rbcast(double x, double one) {
  double acc = 0.0;
  asm("s_nop 1\n\tv_fmac_f64_dpp %0, %1, %2 row_newbcast:%3 row_mask:0xf bank_mask:0xf"
      : "+v"(acc)
      : "v"(x), "v"(one), "i"(L));
  return acc;
}
// 1 / d: hardware reciprocal + two Newton steps (correct to the last bit or one ulp; the pivots of
// an SPD matrix are positive and normal)
__device__ __forceinline__ double recip(double d) {
  double r = __builtin_amdgcn_rcp(d);
  double e = __builtin_fma(-d, r, 1.0);
  r = __builtin_fma(r, e, r);
  e = __builtin_fma(-d, r, 1.0);
  return __builtin_fma(r, e, r);
}
// In-place Gauss-Jordan inverse of the symmetric positive definite leading 12x12 block (scalar
// pivots, no pivoting: stable for SPD).  Pad rows / columns 12-15 must hold the identity.
__device__ __forceinline__ void gj_inverse12(mf4& g) {
  const int j = threadIdx.x & 15, grp = threadIdx.x >> 4;
  const double one = 1.0;
  sfor<0, 12>([&](auto P) __attribute__((always_inline)) {
    constexpr int p = decltype(P)::value, vp = p / 4, gp = p % 4;
    const double rowp = bcast_group<gp>(g[vp]);  // G[p][j]
    const double piv = rbcast<p>(rowp, one);     // G[p][p]
    const double pinv = recip(piv);
    const double rs = rowp * pinv;
    const bool jp = j == p;
#pragma unroll
    for (int v = 0; v < 4; ++v) {
      const double col = rbcast<p>(g[v], one);  // G[4v + grp][p]
      const double upd = jp ? -col * pinv : g[v] - col * rs;
      if (v == vp) g[v] = (grp == gp) ? (jp ? pinv : rs) : upd;  // row p
      else g[v] = upd;
    }
  });
}

// The Riccati recursion of c B'Q̄B + R' (R'_k foot blocks in F.Rt) -> G_k^-1, K_k, Acl_k in LDS.
template <int N>
__device__ void factorize_mfma(WSmem<N>& sm, const mpcqp_params& p, const Adisc& A, double c, double dtm) {
  auto& F = sm.u.f;
  const int j = threadIdx.x & 15, grp = threadIdx.x >> 4;
  mf4 Ad, At, cQ, P;
#pragma unroll
  for (int v = 0; v < 4; ++v) {
    const int u = 4 * v + grp;
    const bool in = u < 12 && j < 12;
    Ad[v] = in ? A.at(u, j) : 0.0;
    At[v] = in ? A.at(j, u) : 0.0;
    cQ[v] = (in && u == j) ? c * (2.0 * p.q_weights[u]) : 0.0;
    P[v] = cQ[v];
  }
  for (int k = N - 1; k >= 0; --k) {
    // B_k (rows 6-8: B_w, rows 9-11: dt/m on the matching force component) and B_k', D layout
    mf4 Bk, Bt, G;
#pragma unroll
    for (int v = 0; v < 4; ++v) {
      const int u = 4 * v + grp;
      auto bsc = [&](int s, int cc) __attribute__((always_inline)) {  // B_k[s][cc]
        if (cc >= 12) return 0.0;
        if (s >= 6 && s < 9) return sm.Bw[k][s - 6][cc];
        if (s >= 9 && s < 12) return (cc % 3 == s - 9) ? dtm : 0.0;
        return 0.0;
      };
      Bk[v] = bsc(u, j);
      Bt[v] = bsc(j, u);
      // R'_k: 3x3 foot blocks (upper triangle stored); identity on the pad
      double rv = 0.0;
      if (u < 12 && j < 12 && u / 3 == j / 3) rv = F.Rt[k][u / 3][sym6(u % 3, j % 3)];
      if (u >= 12 && u == j) rv = 1.0;
      G[v] = rv;
    }
    const mf4 zero = {0.0, 0.0, 0.0, 0.0};
    // G = R' + B'(P B): P B needs only B's rows 6-11 (K-blocks 1, 2); B' P B likewise
    const mf4 PB = mfma_chain<1, 3>(P, Bk, zero);
    G = mfma_chain<1, 3>(Bk, PB, G);
    gj_inverse12(G);
    if (j < 12)
#pragma unroll
      for (int v = 0; v < 3; ++v) F.Gi[k][12 * (4 * v + grp) + j] = G[v];
    if (k >= 1) {
      const mf4 PA = mfma_chain<0, 3>(P, Ad, zero);         // P A
      const mf4 Fm = mfma_chain<1, 3>(Bk, PA, zero);        // F = B' P A
      const mf4 K = mfma_chain<0, 3>(G, Fm, zero);          // K = G^-1 F
      if (j < 12)
#pragma unroll
        for (int v = 0; v < 3; ++v) F.K[k - 1][12 * (4 * v + grp) + j] = K[v];
      if (k <= N - 2) {
        mf4 nBt;
#pragma unroll
        for (int v = 0; v < 4; ++v) nBt[v] = -Bt[v];
        const mf4 Acl = mfma_chain<0, 3>(nBt, K, Ad);       // A - B K
        if (j < 12)
#pragma unroll
          for (int v = 0; v < 3; ++v) F.Acl[k - 1][12 * (4 * v + grp) + j] = Acl[v];
      }
      mf4 nF;
#pragma unroll
      for (int v = 0; v < 4; ++v) nF[v] = -Fm[v];
      P = mfma_chain<0, 3>(nF, K, mfma_chain<0, 3>(Ad, PA, cQ));  // cQ + A'PA - F'K
    }
  }
  wave_sync();
}

// ---- OSQP scale_data (scaling.c) as a kernel of its own -------------------------------------------
// Ruiz equilibration is embarrassingly parallel over the columns of P~ = c D H D, so it runs before
// wave_kernel with one thread per column (NTS threads per robot) and, for n <= 128, the column of H
// generated once into registers instead of once per pass.  It writes a per-robot image (ScaleImg:
// D, E, the scaled gradient q~, the raw gradient, the A entries the passes used, c, the warm-start
// branch) that wave_kernel reads in place of its own setup.  H's columns come from the same closed
// form as before (see gen_col), so every norm is binary64; only the order of the cost-scaling sum
// over columns differs from the single-wave version (a different but equally exact summation).
template <int N>
struct ScaleImg {
  static constexpr int n = ND * N, m = CD * N;
  static constexpr int D = 0, E = D + n, Q = E + m, QN = Q + n, AP = QN + n, CS = AP + 2 * m, MODE = CS + 1,
                       SIZE = MODE + 1;
  static_assert(SIZE == scale_image_doubles(N), "scale image layout");
};

template <int N>
struct ScaleCfg {
  static constexpr int n = ND * N, m = CD * N;
#ifndef MPCQP_SCALE_TPC
#define MPCQP_SCALE_TPC 2
#endif
  static constexpr bool HREG = N <= 10;              // the thread's entries cached in registers
  static constexpr int TPC = HREG ? MPCQP_SCALE_TPC : 1;  // threads per column (adjacent lanes)
  static constexpr int BPT = (N + TPC - 1) / TPC;    // horizon blocks of the column per thread
  static constexpr int NTS = ((TPC * n + 63) / 64) * 64;
  static constexpr int NWS = NTS / 64;
  static constexpr int WPE = NWS >= 2 ? NWS / 2 : 1;  // waves per SIMD for two robots per CU
  static constexpr int RPT = (m + NTS - 1) / NTS;   // constraint rows per thread
};

template <int N>
struct ScaleSmem {
  using C = Cfg<N>;
  alignas(16) double Bw[N][3][ND];
  double rec[C::REC];
  double D[C::n], q[C::n], qn[C::n], E[C::m];
  double lam[N][ND];
  double vec[2][16];
  double Ap[2][C::m];
  double red[2][16];
};

// block-wide sum of sv and max of qv in one barrier (wave partials summed in wave order)
template <int NW>
__device__ __forceinline__ void block_sum_max(double& sv, double& qv, double (*red)[16]) {
  sv = wave_sum(sv);
  qv = wave_max(qv);
  if constexpr (NW > 1) {
    if ((threadIdx.x & 63) == 0) {
      red[0][threadIdx.x >> 6] = sv;
      red[1][threadIdx.x >> 6] = qv;
    }
    __syncthreads();
    double s = red[0][0], q = red[1][0];
#pragma unroll
    for (int i = 1; i < NW; ++i) {
      s += red[0][i];
      q = fmax(q, red[1][i]);
    }
    sv = s;
    qv = q;
  }
}

// Column c of H = B'Q̄B + R in closed form (A_c is nilpotent on the 12 moving states, A_c^2 = 0,
// so A^m = I + m Ac with Ac := dt A_c, and
//   S_j = sum_{m=0}^{M_j} (A^m)' Q A^m = (M_j+1) Q + T1_j (Q Ac + Ac'Q) + T2_j Ac'Q Ac,
//   M_j = N-1-j, T1 = M(M+1)/2, T2 = M(M+1)(2M+1)/6.  With y = B_k e_a (column c = 12k + a):
//   block j <= k:  H_jk e_a = B_j' (A')^{k-j} S_k y = B_j' (g + (k-j) Ac'g),   g = S_k y
//   block j >  k:  H_jk e_a = B_j' S_j A^{j-k} y   = B_j' S_j (y + (j-k) Ac y)
// where only rows 6-11 of the 12-vector inside B_j' matter).  Blocks jb .. jb+NB-1 (< N) only;
// sink(jj, b, ri, hv) receives entry ri = 12 j + b of block j = jb + jj, jj and b compile-time.
template <int N, int NB, bool UNROLL, class Sink>
__device__ __forceinline__ void gen_col(const ScaleSmem<N>& sm, const mpcqp_params& p, const Adisc& A, double dtm,
                                        int c, int jb, Sink&& sink) {
  const double dt = A.dt;
  const int k = c / ND, a2 = c % ND;
  double y[12], w[12];
#pragma unroll
  for (int s2 = 0; s2 < 12; ++s2) y[s2] = 0.0;
  y[6] = sm.Bw[k][0][a2];
  y[7] = sm.Bw[k][1][a2];
  y[8] = sm.Bw[k][2][a2];
  y[9 + a2 % 3] = dtm;
  w[0] = A.ad0 * y[6] + A.ad1 * y[7];
  w[1] = (-A.ad1) * y[6] + A.ad0 * y[7];
  w[2] = dt * y[8];
  w[3] = dt * y[9];
  w[4] = dt * y[10];
  w[5] = dt * y[11];
#pragma unroll
  for (int s2 = 6; s2 < 12; ++s2) w[s2] = 0.0;
  double qy[12], qw[12];
#pragma unroll
  for (int s2 = 0; s2 < 12; ++s2) {
    qy[s2] = 2 * p.q_weights[s2] * y[s2];
    qw[s2] = 2 * p.q_weights[s2] * w[s2];
  }
  auto actv = [&](const double (&v)[12], double (&o)[6]) __attribute__((always_inline)) {
    o[0] = A.ad0 * v[0] + (-A.ad1) * v[1];
    o[1] = A.ad1 * v[0] + A.ad0 * v[1];
    o[2] = dt * v[2];
    o[3] = dt * v[3];
    o[4] = dt * v[4];
    o[5] = dt * v[5];
  };
  double u1[6], u2[6];
  actv(qy, u1);
  actv(qw, u2);
  const double Mk = (double)(N - 1 - k);
  const double T1k = Mk * (Mk + 1) / 2, T2k = Mk * (Mk + 1) * (2 * Mk + 1) / 6;
  double g[12];
#pragma unroll
  for (int s2 = 0; s2 < 12; ++s2) {
    const double ac = s2 >= 6 ? u1[s2 - 6] : 0.0, ac2 = s2 >= 6 ? u2[s2 - 6] : 0.0;
    g[s2] = ((Mk + 1) * qy[s2] + T1k * (qw[s2] + ac)) + T2k * ac2;
  }
  double h[6];
  actv(g, h);
  auto block = [&](int jj) __attribute__((always_inline)) {
    const int j = jb + jj;
    if (j >= N) return;
    const bool up = j <= k;
    const double d = (double)(j - k);
    const double Mj = (double)(N - 1 - j);
    const double T1j = Mj * (Mj + 1) / 2, T2j = Mj * (Mj + 1) * (2 * Mj + 1) / 6;
    const double cg = up ? 1.0 : 0.0, ch = up ? -d : 0.0;
    const double cqy = up ? 0.0 : Mj + 1, cqw = up ? 0.0 : (Mj + 1) * d + T1j;
    const double cu1 = up ? 0.0 : T1j, cu2 = up ? 0.0 : T1j * d + T2j;
    double v[6];
#pragma unroll
    for (int s2 = 0; s2 < 6; ++s2)
      v[s2] = ((((cg * g[6 + s2] + ch * h[s2]) + cqy * qy[6 + s2]) + cqw * qw[6 + s2]) + cu1 * u1[s2]) + cu2 * u2[s2];
    const double* bw0 = sm.Bw[j][0];
    const double* bw1 = sm.Bw[j][1];
    const double* bw2 = sm.Bw[j][2];
#pragma unroll
    for (int b = 0; b < 12; ++b) {
      double hv = ((bw0[b] * v[0] + bw1[b] * v[1]) + bw2[b] * v[2]) + dtm * v[3 + b % 3];
      if (j == k && b == a2) hv += 2 * p.r_weights[b];
      sink(jj, b, ND * j + b, hv);
    }
  };
  if constexpr (UNROLL) {
    sfor<0, NB>([&](auto JJ) __attribute__((always_inline)) { block(decltype(JJ)::value); });
  } else {
#pragma unroll 1
    for (int jj = 0; jj < NB; ++jj) block(jj);
  }
}

template <int N>
__global__ __launch_bounds__(ScaleCfg<N>::NTS, ScaleCfg<N>::WPE) void scale_kernel(const double* __restrict__ recs, int batch,
                                                                 double* __restrict__ wstate,
                                                                 double* __restrict__ img, mpcqp_params p) {
  using C = Cfg<N>;
  using SC = ScaleCfg<N>;
  using WL = WarmLayout<N>;
  using SI = ScaleImg<N>;
  constexpr int n = C::n, m = C::m, NTS = SC::NTS;
  __shared__ ScaleSmem<N> sm;
  const int inst = blockIdx.x;
  if (inst >= batch) return;
  const int t = threadIdx.x;
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
  {
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
      for (int j = N - 2; j >= 0; --j) {
        if (t < ND) sm.lam[j][t] = sm.lam[j][t] + A.atv(t, sm.lam[j + 1]);
        wave_sync();
      }
    }
    __syncthreads();
  }
  // thread t: column j0 = t / 4, blocks jb .. jb+BPT-1 of it (the column's four threads are a quad)
  constexpr int BPT = SC::BPT;
  const int j0 = t / SC::TPC, jb = (t % SC::TPC) * BPT;
  const bool lead = (t % SC::TPC) == 0;  // the lane that owns the column's per-column values
  if (lead && j0 < n) {
    const int k = j0 / ND, ii = j0 % ND;
    const double* lm = sm.lam[k];
    const double g = ((sm.Bw[k][0][ii] * lm[6] + sm.Bw[k][1][ii] * lm[7]) + sm.Bw[k][2][ii] * lm[8]) + dtm * lm[9 + ii % 3];
    sm.q[j0] = g;
    sm.qn[j0] = g;
    sm.D[j0] = 1.0;
  }
  for (int r = t; r < m; r += NTS) {
    sm.E[r] = 1.0;
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
#pragma unroll
        for (int jj = 0; jj < BPT; ++jj) {
          const int j = jb + jj;
          if (j < N) {
            const double* dj = sm.D + ND * j;
#pragma unroll
            for (int b = 0; b < 12; ++b) {
              if (b & 1) mx1 = fmax(mx1, dj[b] * dabs(hc[12 * jj + b]));
              else mx0 = fmax(mx0, dj[b] * dabs(hc[12 * jj + b]));
            }
          }
        }
      } else {
        gen_col<N, BPT, false>(sm, p, A, dtm, j0, jb, [&](int, int b, int ri, double hv) __attribute__((always_inline)) {
          if (b & 1) mx1 = fmax(mx1, sm.D[ri] * dabs(hv));
          else mx0 = fmax(mx0, sm.D[ri] * dabs(hv));
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
  auto acol = [&](int j) __attribute__((always_inline)) {
    const int f = j / 3, aa = j % 3;
    const double* e = sm.E + 5 * f;
    const double* a0 = sm.Ap[0] + 5 * f;
    const double* a1 = sm.Ap[1] + 5 * f;
    double mx;
    if (aa == 0) mx = dmax(e[0] * dabs(a0[0]), e[1] * dabs(a0[1]));
    else if (aa == 1) mx = dmax(e[2] * dabs(a0[2]), e[3] * dabs(a0[3]));
    else
      mx = dmax(dmax(dmax(dmax(dabs(a1[0]) * e[0], dabs(a1[1]) * e[1]), dabs(a1[2]) * e[2]), dabs(a1[3]) * e[3]),
                e[4] * dabs(a1[4]));
    return mx * sm.D[j];
  };
  auto arow = [&](int r) __attribute__((always_inline)) {
    const int f = r / 5, k5 = r % 5;
    const double e = sm.E[r];
    const double* d = sm.D + 3 * f;
    if (k5 == 4) return (e * dabs(sm.Ap[1][r])) * d[2];
    return dmax((e * dabs(sm.Ap[0][r])) * d[k5 >> 1], (dabs(sm.Ap[1][r]) * e) * d[2]);
  };
  double c_s = 1.0, cm = 0.0;
  // First column pass (D = 1): the raw norms, and H's zero pattern (warm start only): same pattern
  // -> osqp_update_P (unscale with the old scaling, rescale with the previous A and q, keep iterates
  // and rho); a changed pattern or mu -> re-init (fresh scaling and rho, the previous unscaled x, y)
  bool pattern_changed = false;
  if (p.scaling > 0 || ws) {
    cm = colmax(true);
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
  for (int pass = 0; pass < p.scaling; ++pass) {
    // new scaling factors from the current D, E (every thread reads before anyone writes)
    double dtv = 1.0;
    if (lead && j0 < n) {
      const double pc = (c_s * sm.D[j0]) * cm;
      dtv = 1.0 / sqrt(limit_scaling(fmax(pc, acol(j0))));
    }
    double et[SC::RPT];
#pragma unroll
    for (int rr = 0; rr < SC::RPT; ++rr) {
      const int r = t + NTS * rr;
      et[rr] = r < m ? 1.0 / sqrt(limit_scaling(arow(r))) : 1.0;
    }
    __syncthreads();
#pragma unroll
    for (int rr = 0; rr < SC::RPT; ++rr) {
      const int r = t + NTS * rr;
      if (r < m) sm.E[r] *= et[rr];
    }
    if (lead && j0 < n) {
      sm.q[j0] = dtv * sm.q[j0];
      sm.D[j0] = sm.D[j0] * dtv;
    }
    __syncthreads();
    cm = colmax(false);  // column norms of the D-scaled P (cost normalization)
    double sv = 0.0, qv = 0.0;
    if (lead && j0 < n) {
      sv = (c_s * sm.D[j0]) * cm;
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
  double* out = img + (size_t)inst * SI::SIZE;
  if (lead && j0 < n) {
    out[SI::D + j0] = sm.D[j0];
    out[SI::Q + j0] = sm.q[j0];
    out[SI::QN + j0] = sm.qn[j0];
  }
  for (int r = t; r < m; r += NTS) {
    out[SI::E + r] = sm.E[r];
    out[SI::AP + r] = sm.Ap[0][r];
    out[SI::AP + m + r] = sm.Ap[1][r];
  }
  if (t == 0) {
    out[SI::CS] = c_s;
    out[SI::MODE] = (double)mode;
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
__global__ __launch_bounds__(NT, 1) void wave_kernel(const double* __restrict__ recs, int batch,
                                                     mpcqp_result* __restrict__ results,
                                                     double* __restrict__ solution, double* __restrict__ trace,
                                                     int trace_cap, double* __restrict__ wstate,
                                                     const double* __restrict__ img, mpcqp_params p) {
  using C = Cfg<N>;
  using WL = WarmLayout<N>;
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
      return;
    }
  }
  wave_sync();
  WV_MARK(1);
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
  // what the solve needs from the record after the setup image is recycled
  double Rot[9];
#pragma unroll
  for (int e = 0; e < 9; ++e) Rot[e] = rec[MPCQP_REC_ROT + e];
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

  // ---- 3. OSQP scale_data: the image scale_kernel wrote (D, E, q~, raw q, A entries, c, branch) ----
  using SI = ScaleImg<N>;
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
  // Warm start (A1RobotControl.h:67 member solver, :522-538): the slot of the previous tick.
  double* const ws = wstate ? wstate + (size_t)inst * WL::SIZE : nullptr;
  wave_sync();
  const double cost_c = c_s, cinv = 1. / c_s;
  WV_MARK(4);

  // ---- 4. lane registers: variables (D, q~) and rows (E, A~, bounds, rho) — set_rho_vec -----------
  // update_P keeps the adapted rho (settings->rho); setup and re-init start from the settings'
  const double rho0 = mode == 1 ? ws[WL::RHO] : dmin(dmax(p.rho, RHO_MIN), RHO_MAX);
  double X[R], Qv[R], Dv[R], DI[R], PX[R], PXO[R], DX[R], RHS[R];
  double Z[R], Y[R], DY[R], Ev[R], AK0[R], AK1[R];
  double Z4[R], Y4[R], DY4[R], E4[R], L4[R], U4[R], AK4[R], RHO4[R];
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
    // update_P then osqp_update_lin_cost: q~ = c (D q) of this tick's gradient
    Qv[r] = vv ? (mode == 1 ? (HS.qn[ci] * Dv[r]) * c_s : HS.q[ci]) : 0.0;
    Ev[r] = kv ? HS.E[ri] : 1.0;
    E4[r] = kv ? HS.E[r4] : 1.0;
    // A~ = E A D: row a < 4 has A on fx (a < 2) / fy (a >= 2) and on fz; row 4 on fz
    AK0[r] = kv ? (HS.Ap[0][ri] * Ev[r]) * HS.D[cf + (a >> 1)] : 0.0;
    AK1[r] = kv ? (HS.Ap[1][ri] * Ev[r]) * HS.D[cf + 2] : 0.0;
    AK4[r] = kv ? (HS.Ap[1][r4] * E4[r]) * HS.D[cf + 2] : 0.0;
    // bounds (ConvexMpc.cpp:223-245), clipped to +-OSQP_INFTY, scaled by E
    double l4 = fzmin * cont, u4 = fzmax * cont;
    l4 = dmin(dmax(l4, -OSQP_INF), OSQP_INF);
    u4 = dmin(dmax(u4, -OSQP_INF), OSQP_INF);
    L4[r] = E4[r] * l4;
    U4[r] = E4[r] * u4;
    X[r] = 0.0; PX[r] = 0.0; PXO[r] = 0.0; DX[r] = 0.0;
    Z[r] = 0.0; Y[r] = 0.0; DY[r] = 0.0; Z4[r] = 0.0; Y4[r] = 0.0; DY4[r] = 0.0;
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
  auto rho4_of = [&](int r, double rho) __attribute__((always_inline)) {
    const bool loose = L4[r] < -OSQP_INF * MIN_SCALING && U4[r] > OSQP_INF * MIN_SCALING;
    const bool eq = U4[r] - L4[r] < RHO_TOL;
    return loose ? RHO_MIN : (eq ? RHO_EQ_OVER_RHO_INEQ * rho : rho);
  };
  double RI4[R];  // 1 / rho of row 4 (OSQP rho_inv_vec), refreshed with rho
#pragma unroll
  for (int r = 0; r < R; ++r) {
    RHO4[r] = rho4_of(r, rho0);
    RI4[r] = 1. / RHO4[r];
  }
  if (mode != 0) {
    // P~x of the warm iterate (the loop carries P~x through the KKT identity from here):
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
        HS.lam[i][t] = 2 * p.q_weights[t] * xn;
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
                         dtm * lm[9 + idx % 3]) + (2 * p.r_weights[idx]) * HS.Dt[ND * k + idx];
      PX[r] = vvr[r] ? (c_s * Dv[r]) * hv : 0.0;
      // compute_rhs from the warm x, z, y: sigma x - q~ + A~'(rho z - y)
      const double at = quad_at(rho0 * Z[r] - Y[r], RHO4[r] * Z4[r] - Y4[r], AK0[r], AK1[r], AK4[r], a);
      RHS[r] = vvr[r] ? (sigma * X[r] - Qv[r]) + at : 0.0;
    }
  }
  // rows 0-3: l = 0 / u = +inf (rows 0, 2) or l = -inf / u = 0 (rows 1, 3): always inequalities
  auto lo03 = [&](int r) __attribute__((always_inline)) { return (a & 1) ? Ev[r] * -OSQP_INF : Ev[r] * 0.0; };
  // the projection onto those bounds needs no E: [0, +inf) for rows 0, 2, (-inf, 0] for rows 1, 3
  // (equal to clamping at E * -+OSQP_INF for every operand below 1e30 E in magnitude)
  const double LO03 = (a & 1) ? -INFINITY : 0.0, HI03 = (a & 1) ? 0.0 : INFINITY;
  auto hi03 = [&](int r) __attribute__((always_inline)) { return (a & 1) ? Ev[r] * 0.0 : Ev[r] * OSQP_INF; };
  wave_sync();  // every LDS read of the setup image precedes its reuse by the factorization

  // ---- 5. ADMM (osqp_solve) ------------------------------------------------------------------------
  auto& F = sm.u.f;
  double rho = rho0, rinv = 1. / rho0, pri_res = 0.0, dua_res = 0.0;
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
          if (kvr[r] && av && b >= a) F.Rt[k][leg][sym6(a, b)] = rt;
        }
      }
      wave_sync();
      factorize_mfma<N>(sm, p, A, cost_c, dtm);
      wave_sync();
      need_factor = false;
      WV_MARK(12);
    }

    // ---- KKT solve: u = (c B'Q̄B + R')^-1 D^-1 rhs, x~ = D^-1 u ----
    double U[R];
    const bool tm_it = iter == 60;
    if (tm_it) WV_MARK(40);
    {
      // LDS operands are loaded one phase ahead of their use; sched_barrier keeps the scheduler from
      // sinking a prefetch back down to its consumer (counted lgkmcnt waits then cover only it).
      double W[R], AKw[R], SMv[R], G[R], Hh[R], XS[R], tt[R];
      double cA[R][12], cB[R][12], cw[R][3];
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
#pragma unroll
      for (int r = 0; r < R; ++r) ld12s(cA[r], &F.K[kk[r]][idx]);
      if constexpr (N >= 3) ld12s(cn, &F.Acl[N - 3][idx]);
      __builtin_amdgcn_sched_barrier(0);
      // a_k = K_k' w_k (k >= 1)
      mv_rounds<R>(W, cA, AKw);
#pragma unroll
      for (int r = 0; r < R; ++r) {  // for g_k: G_k^-1 rows and B_k' columns
        ld12(cB[r], &F.Gi[kc[r]][12 * idx]);
        cw[r][0] = sm.Bw[kc[r]][0][idx];
        cw[r][1] = sm.Bw[kc[r]][1][idx];
        cw[r][2] = sm.Bw[kc[r]][2][idx];
      }
      __builtin_amdgcn_sched_barrier(0);
      if (tm_it) WV_MARK(41);
      {  // backward chain: s_{N-1} = -a_{N-1}; s_k = Acl_k' s_{k+1} - a_k; SMv (row of k) = s_{k+1}
        double cur = -AKw[(N - 1) >> 2];
        sfor<0, N - 1>([&](auto J) {
          constexpr int k = N - 2 - decltype(J)::value;
          const double mvv = rmove2<row_of(k + 1), row_of(k)>(cur);
          SMv[k >> 2] = (q == row_of(k)) ? mvv : SMv[k >> 2];
          if constexpr (k >= 1) {
            double cc[12];
#pragma unroll
            for (int e = 0; e < 12; ++e) cc[e] = cn[e];
            if constexpr (k >= 2) ld12s(cn, &F.Acl[k - 2][idx]);  // the next step's column
            __builtin_amdgcn_sched_barrier(0);
            cur = mv12a(mvv, cc, -AKw[k >> 2]);
          }
        });
      }
      if (tm_it) WV_MARK(42);
      // g_k = G_k^-1 (w_k + B_k' s_{k+1})
#pragma unroll
      for (int r = 0; r < R; ++r) {
        const double c6[6] = {cw[r][0], cw[r][1], cw[r][2], a == 0 ? dtm : 0.0, a == 1 ? dtm : 0.0,
                              a == 2 ? dtm : 0.0};
        tt[r] = W[r] + mv6(SMv[r], c6);
      }
#pragma unroll
      for (int r = 0; r < R; ++r) ld12(cA[r], &sm.Bw[kc[r]][av ? a : 2][0]);  // for h_k
      __builtin_amdgcn_sched_barrier(0);
      mv_rounds<R>(tt, cB, G);
      // h_k = B_k g_k: rows 6-8 (leg-2 lanes) B_w g, rows 9-11 (leg-3 lanes) dt/m times the sum of
      // the legs' matching force component, rows 0-5 zero
      if constexpr (N >= 3) ld12(cn, &F.Acl[0][12 * idx]);
#pragma unroll
      for (int r = 0; r < R; ++r) ld12(cB[r], &F.K[kk[r]][12 * idx]);  // for u_k
      __builtin_amdgcn_sched_barrier(0);
      {
        double hb[R];
        mv_rounds<R>(G, cA, hb);
#pragma unroll
        for (int r = 0; r < R; ++r) {
          const double ls = dtm * legsum(G[r]);
          Hh[r] = leg == 2 ? hb[r] : (leg == 3 ? ls : 0.0);
        }
      }
      if (tm_it) WV_MARK(43);
      {  // forward chain: x_1 = h_0; x_{k+1} = Acl_k x_k + h_k; XS (row of k) = x_k
        double cur = Hh[0];
        sfor<1, N>([&](auto K) {
          constexpr int k = decltype(K)::value;
          const double mvv = rmove2<row_of(k - 1), row_of(k)>(cur);
          XS[k >> 2] = (q == row_of(k)) ? mvv : XS[k >> 2];
          if constexpr (k <= N - 2) {
            double cc[12];
#pragma unroll
            for (int e = 0; e < 12; ++e) cc[e] = cn[e];
            if constexpr (k + 1 <= N - 2) ld12(cn, &F.Acl[k][12 * idx]);  // the next step's row
            __builtin_amdgcn_sched_barrier(0);
            cur = mv12a(mvv, cc, Hh[k >> 2]);
          }
        });
      }
      if (tm_it) WV_MARK(44);
      // u_k = g_k - K_k x_k (x_0 = 0)
      {
        double kx[R];
        mv_rounds<R>(XS, cB, kx);
#pragma unroll
        for (int r = 0; r < R; ++r) U[r] = G[r] - kx[r];
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
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const double xt = DI[r] * U[r];
      const double xp = dpp<QP_PRIM>(xt), xz = dpp<QP_B2>(xt);
      const double zt = AK0[r] * xp + AK1[r] * xz;
      const double zt4 = AK4[r] * xz;
      {  // (fmin/fmax = the reference's c_min/c_max on these non-NaN operands)
        const double zr = alpha * zt + (1.0 - alpha) * Z[r];
        const double zn = fmin(fmax(zr + rinv * Y[r], LO03), HI03);
        const double dyv = rho * (zr - zn);
        Z[r] = zn;
        Y[r] = Y[r] + dyv;
        DY[r] = dyv;
      }
      {
        const double r4 = RHO4[r];
        const double zr = alpha * zt4 + (1.0 - alpha) * Z4[r];
        const double zn = fmin(fmax(zr + RI4[r] * Y4[r], L4[r]), U4[r]);
        const double dyv = r4 * (zr - zn);
        Z4[r] = zn;
        Y4[r] = Y4[r] + dyv;
        DY4[r] = dyv;
      }
      const double kd = quad_at(rho * zt, RHO4[r] * zt4, AK0[r], AK1[r], AK4[r], a);
      // every lane updates (values of padding lanes / steps past N are never read unmasked)
      const double xo = X[r];
      const double xn = alpha * xt + (1.0 - alpha) * xo;
      DX[r] = xn - xo;
      X[r] = xn;
      const double pxt = (RHS[r] - sigma * xt) - kd;
      PXO[r] = PX[r];
      PX[r] = alpha * pxt + (1.0 - alpha) * PX[r];
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
        for (int r = 0; r < R; ++r) {
          RHO4[r] = rho4_of(r, rho);
          RI4[r] = 1. / RHO4[r];
        }
        rinv = 1. / rho;
        need_factor = true;
      }
    }
    // ---- next right-hand side: sigma x - q~ + A~'(rho z - y) ----
#pragma unroll
    for (int r = 0; r < R; ++r) {
      // (padding lanes and steps past N compute values nothing reads unmasked)
      const double at = quad_at(rho * Z[r] - Y[r], RHO4[r] * Z4[r] - Y4[r], AK0[r], AK1[r], AK4[r], a);
      RHS[r] = (sigma * X[r] - Qv[r]) + at;
    }
    if (tm_it) WV_MARK(47);
  }

  WV_MARK(20);
  if (ws) {  // the solver persists: scaling, scaled data, iterates and rho for the next tick
    if (t == 0) {
      ws[WL::FLAG] = 1.0;
      ws[WL::RHO] = rho;
      ws[WL::C] = cost_c;
      ws[WL::MU] = mu;
    }
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const int k = 4 * r + ig;
      if (vvr[r]) {
        const int ci = ND * k + idx;
        ws[WL::D + ci] = Dv[r];
        ws[WL::QT + ci] = Qv[r];
        ws[WL::X + ci] = X[r];
      }
      if (kvr[r]) {
        const int ri = CD * k + 5 * leg + a, r4 = CD * k + 5 * leg + 4;
        ws[WL::E + ri] = Ev[r];
        ws[WL::AK + ri] = AK0[r];
        ws[WL::AK + m + ri] = AK1[r];
        ws[WL::Z + ri] = Z[r];
        ws[WL::Y + ri] = Y[r];
        if (a == 0) {
          ws[WL::E + r4] = E4[r];
          ws[WL::AK + r4] = 0.0;
          ws[WL::AK + m + r4] = AK4[r];
          ws[WL::Z + r4] = Z4[r];
          ws[WL::Y + r4] = Y4[r];
        }
      }
    }
  }
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
  hipLaunchKernelGGL((wv::scale_kernel<N>), dim3(a.batch), dim3(wv::ScaleCfg<N>::NTS), 0, (hipStream_t)a.stream,
                     a.recs, a.batch, a.wstate, a.work, a.p);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL((wv::wave_kernel<N>), dim3(a.batch), dim3(wv::NT), 0, (hipStream_t)a.stream, a.recs, a.batch,
                     a.results, a.solution, a.trace, a.trace_cap, a.wstate, a.work, a.p);
  return hipGetLastError();
}
template <int N>
static hipError_t occupancy_wave(int* blocks) {
  return hipOccupancyMaxActiveBlocksPerMultiprocessor(blocks, wv::wave_kernel<N>, wv::NT, 0);
}

#define MPCQP_WAVE_FOR_EACH_N(X) \
  X(1) X(2) X(3) X(4) X(5) X(6) X(7) X(8) X(9) X(10) X(11) X(12) X(13) X(14) X(15) X(16) X(17) X(18) X(19) X(20)

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
