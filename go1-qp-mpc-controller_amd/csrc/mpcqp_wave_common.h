// mpcqp_wave_common.h — device pieces shared by the one-wave (mpcqp_wave.hip) and the
// wave-per-round (mpcqp_wave_mw.hip) solve kernels: lane layout, cross-lane mat-vecs, the
// discrete dynamics, the MFMA Riccati factorization, and the scale_kernel image layout.
// Not installed.
#pragma once
#include <type_traits>

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

// Stored 12x12 factors (G_k^-1, K_k, Acl_k): row r starts at double mo(r) = 12 r + 2 [r >= 4] (a
// 16-B gap after row 3) and matrices are MS = 146 doubles apart.  The DPP rows of a wave read 12
// distinct rows of one matrix (chains) or rows {0-2, 9-11} of one matrix with rows {3-8} of the
// next (parallel phases); with this layout both land on 12 distinct 16-B bank slots of every
// ds_read_b128 lane group (row-major 12 x 12 at stride 144 put rows r and r + 8 on one slot:
// 2-way conflicts, 449 extra LDS cycles per iteration measured with SQ_LDS_BANK_CONFLICT).
constexpr int MS = 146;
__host__ __device__ constexpr int mo(int r) { return 12 * r + (r >= 4 ? 2 : 0); }

template <int N>
struct SchurLds;
// Riccati factors (KS = 0; the factorization itself runs in registers).  With SACL the closed-loop
// matrices Acl_k = A - B_k K_k are stored for the chains; without (long horizons: the three factor
// families would leave room for only two robots per CU) the chains apply A and B_k K_k separately,
// and the R'_k foot blocks share G_k^-1's slot (read by factorization step k before it writes G_k^-1).
#ifndef MPCQP_ACL_MAXN
#define MPCQP_ACL_MAXN 12
#endif
template <int N, bool SACL>
struct RicFactors;
template <int N>
struct RicFactors<N, true> {
  static constexpr bool HAS_ACL = true;
  static constexpr int NK = N > 1 ? N - 1 : 1;  // K_k stored for k = 1..N-1
  static constexpr int NA = N > 2 ? N - 2 : 1;  // Acl_k stored for k = 1..N-2
  alignas(16) double Gi[N][MS];
  alignas(16) double K[NK][MS];
  alignas(16) double Acl[NA][MS];
  double Rt[N][4][6];  // R'_k foot blocks, upper triangle (00 01 02 11 12 22)
  __device__ double* rt(int k) { return &Rt[k][0][0]; }
};
// Without Acl, G_k^-1 (symmetric) is kept as its upper triangle, rows packed (row r at poff(r)),
// GPS doubles per step and 4R steps (whole register rounds, so that every lane's row can be read
// at a compile-time offset from a per-lane base): the three families then need 40.7 KB at N = 20,
// four robots per CU.
__host__ __device__ constexpr int poff(int r) { return 12 * r - r * (r - 1) / 2; }
constexpr int GPS = 80;
static_assert(poff(11) + 1 <= GPS, "packed 12 x 12 upper triangle");
template <int N>
struct RicFactors<N, false> {
  static constexpr bool HAS_ACL = false;
  static constexpr int NK = N > 1 ? N - 1 : 1;
  alignas(16) double Gp[4 * ((N + 3) / 4)][GPS];
  alignas(16) double K[NK][MS];
  __device__ double* rt(int k) { return &Gp[k][0]; }
};
template <int N, int KS>
struct WSmem {
  using C = Cfg<N>;
  static constexpr bool SACL = N <= MPCQP_ACL_MAXN;
  static constexpr int NK = N > 1 ? N - 1 : 1;  // K_k stored for k = 1..N-1
  static constexpr int NA = N > 2 ? N - 2 : 1;  // Acl_k stored for k = 1..N-2 (SACL)
  alignas(16) double Bw[N][3][ND];  // rows 6-8 of B_d(k) = I_w^-1 skew(foot) dt (rows 9-11: dt/m I)
  union U {
    struct Hs {  // setup: record, Ruiz vectors
      double rec[C::REC];
      double D[C::n], Dt[C::n], q[C::n], E[C::m];
      double lam[N][ND];  // gradient adjoint lambda_k (states 0..11)
      double vec[2][16];  // sequential 13-vectors (gradient forward sweep)
      double qn[C::n];     // this tick's gradient (warm start: q of the Ruiz passes is the old one)
      // OSQP scale_data inside the Schur-form wave (scale_wave, KS = 1 only): the Ruiz passes' second
      // D / E buffers, the unscaled A entries and the raw column norms (inside the union: no LDS added)
      static constexpr int FX = KS == 1 ? 1 : 0;
      double Dx[FX ? C::n : 1], Ex[FX ? C::m : 1], Ap[2][FX ? C::m : 1], cm0[FX ? C::n : 1];
    } h;
    // KS = 0: the Riccati factors; KS = 1: the impulse-space Schur form (mpcqp_schur.h)
    typename std::conditional<KS == 0, RicFactors<N, SACL>, SchurLds<N>>::type f;
  } u;
};

// ---- DPP wait states in the inline-asm blocks -------------------------------------------------
// A DPP instruction reads its src0 at least 2 wait states after a VALU write of it, and at least 5
// after a VALU write of EXEC (v_cmpx, which these kernels never emit; tools/isa_hazards.py checks
// both in the compiled code).  An s_nop is not free for a lone wave: s_nop 1 costs 8.4 cycles on
// MI355X, as much as two f64 FMAs (tools/mb/mb_valu).  The compiler cannot see into an asm block, so
// each block that may follow the VALU write of its src0 starts with a wait: WV_NOP_HEAD (2 states).
// A block whose src0 an earlier block of the same sequence already read (the sources of a sequence are
// materialized together before its first block) waits for nothing (WV_NOP_INNER).  tools/isa_hazards.py
// verifies the placement on the compiled product kernels (tests/test_isa_hazards.py); the round-4
// placement (s_nop 4 / s_nop 1 at every block) remains as MPCQP_NOP_SAFE: C2 1.737 -> 1.677 ms,
// C4 6.75 -> 6.20 ms, bitwise equal results (profiles/r05/nop_lean).
#ifndef MPCQP_NOP_SAFE
#define WV_NOP_HEAD "s_nop 1\n\t"
#define WV_NOP_INNER ""
#define WV_NOP_HEAD1 "s_nop 1\n\t"
#define WV_NOP_INNER1 ""
#define WV_NOP_PERM "s_nop 0\n\t"
#else
#define WV_NOP_HEAD "s_nop 4\n\t"
#define WV_NOP_INNER "s_nop 4\n\t"
#define WV_NOP_HEAD1 "s_nop 1\n\t"
#define WV_NOP_INNER1 "s_nop 1\n\t"
#define WV_NOP_PERM "s_nop 1\n\t"
#endif

// ---- cross-lane primitives ---------------------------------------------------------------------
#define WV_FM(A, M, L) "v_fmac_f64_dpp " A ", %[x], " M " row_newbcast:" #L " row_mask:0xf bank_mask:0xf\n\t"
#ifndef MPCQP_MV_MULTI_ACC
// y_i = sum_c M[i][c] x_c, x_c broadcast from lane 4(c/3)+c%3 of each DPP row, M row i in `c`.
// One accumulator per mat-vec, the terms in column order: a dependent v_fmac_f64_dpp chain issues as
// fast as independent ones for a lone wave (4.4 against 5.35 cycles, tools/mb/mb_valu), so rotating
// accumulators only cost the zeroing moves and the closing adds (the round-4 form: MPCQP_MV_MULTI_ACC).
// Each FMA reads the accumulator its predecessor just wrote.  The DPP wait-state requirement (VALU
// write, then a DPP read of that VGPR: 2 states) concerns the operand read through the lane permute,
// src0 (here x, written before the block's head wait); the accumulator is an ordinary dependent VALU
// operand.  LLVM's hazard recognizer applies the rule to every operand of a DPP instruction, so this
// reading is not the compiler's: tools/mb/mb_valu checks the chain numerically on MI355X (bitwise the
// host's fma chain) beside the src0 case it does not cover.
#define WV_OPS12(P, C) [P##0] "v"(C[0]), [P##1] "v"(C[1]), [P##2] "v"(C[2]), [P##3] "v"(C[3]), [P##4] "v"(C[4]), \
    [P##5] "v"(C[5]), [P##6] "v"(C[6]), [P##7] "v"(C[7]), [P##8] "v"(C[8]), [P##9] "v"(C[9]),                \
    [P##10] "v"(C[10]), [P##11] "v"(C[11])
#define WV_OPS6(P, C) [P##0] "v"(C[0]), [P##1] "v"(C[1]), [P##2] "v"(C[2]), [P##3] "v"(C[3]), [P##4] "v"(C[4]), \
    [P##5] "v"(C[5])
#define WV_M12(A) WV_FM(A, "%[c0]", 0) WV_FM(A, "%[c1]", 1) WV_FM(A, "%[c2]", 2) WV_FM(A, "%[c3]", 4)  \
    WV_FM(A, "%[c4]", 5) WV_FM(A, "%[c5]", 6) WV_FM(A, "%[c6]", 8) WV_FM(A, "%[c7]", 9)                 \
    WV_FM(A, "%[c8]", 10) WV_FM(A, "%[c9]", 12) WV_FM(A, "%[c10]", 13) WV_FM(A, "%[c11]", 14)
#define WV_M6HI(A) WV_FM(A, "%[c0]", 8) WV_FM(A, "%[c1]", 9) WV_FM(A, "%[c2]", 10) WV_FM(A, "%[c3]", 12) \
    WV_FM(A, "%[c4]", 13) WV_FM(A, "%[c5]", 14)
#define WV_M6LO(A) WV_FM(A, "%[c0]", 0) WV_FM(A, "%[c1]", 1) WV_FM(A, "%[c2]", 2) WV_FM(A, "%[c3]", 4)  \
    WV_FM(A, "%[c4]", 5) WV_FM(A, "%[c5]", 6)
__device__ __forceinline__ double mv12(double x, const double (&c)[12]) {
  double a = 0.0;
  asm(WV_NOP_HEAD WV_M12("%[a]") : [a] "+&v"(a) : [x] "v"(x), WV_OPS12(c, c));
  return a;
}
// sum over states 6..11 (lanes 8, 9, 10, 12, 13, 14) of c[s-6] x_s
__device__ __forceinline__ double mv6(double x, const double (&c)[6]) {
  double a = 0.0;
  asm(WV_NOP_HEAD WV_M6HI("%[a]") : [a] "+&v"(a) : [x] "v"(x), WV_OPS6(c, c));
  return a;
}
// Two / three independent mat-vecs interleaved in one block (each has its own x and rows)
#define WV_FX(A, X, M, L) "v_fmac_f64_dpp " A ", " X ", " M " row_newbcast:" #L " row_mask:0xf bank_mask:0xf\n\t"
#define WV_T2(L, I) WV_FX("%[a]", "%[x0]", "%[p" #I "]", L) WV_FX("%[b]", "%[x1]", "%[q" #I "]", L)
#define WV_T3(L, I) WV_T2(L, I) WV_FX("%[d]", "%[x2]", "%[r" #I "]", L)
__device__ __forceinline__ void mv12x2(double x0, double x1, const double (&c0)[12], const double (&c1)[12],
                                       double& y0, double& y1) {
  double a = 0.0, b = 0.0;
  asm(WV_NOP_HEAD
      WV_T2(0, 0) WV_T2(1, 1) WV_T2(2, 2) WV_T2(4, 3) WV_T2(5, 4) WV_T2(6, 5)
      WV_T2(8, 6) WV_T2(9, 7) WV_T2(10, 8) WV_T2(12, 9) WV_T2(13, 10) WV_T2(14, 11)
      : [a] "+&v"(a), [b] "+&v"(b)
      : [x0] "v"(x0), [x1] "v"(x1), WV_OPS12(p, c0), WV_OPS12(q, c1));
  y0 = a;
  y1 = b;
}
__device__ __forceinline__ void mv12x3(double x0, double x1, double x2, const double (&c0)[12],
                                       const double (&c1)[12], const double (&c2)[12], double& y0, double& y1,
                                       double& y2) {
  double a = 0.0, b = 0.0, d = 0.0;
  asm(WV_NOP_HEAD
      WV_T3(0, 0) WV_T3(1, 1) WV_T3(2, 2) WV_T3(4, 3) WV_T3(5, 4) WV_T3(6, 5)
      WV_T3(8, 6) WV_T3(9, 7) WV_T3(10, 8) WV_T3(12, 9) WV_T3(13, 10) WV_T3(14, 11)
      : [a] "+&v"(a), [b] "+&v"(b), [d] "+&v"(d)
      : [x0] "v"(x0), [x1] "v"(x1), [x2] "v"(x2), WV_OPS12(p, c0), WV_OPS12(q, c1), WV_OPS12(r, c2));
  y0 = a;
  y1 = b;
  y2 = d;
}
#undef WV_T2
#undef WV_T3
#undef WV_FX
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
// init + sum_c M[c] x_c: the chains' "- a_k" / "+ h_k" as the accumulator's start
__device__ __forceinline__ double mv12a(double x, const double (&c)[12], double init) {
  double a = init;
  asm(WV_NOP_HEAD WV_M12("%[a]") : [a] "+&v"(a) : [x] "v"(x), WV_OPS12(c, c));
  return a;
}
// init + sum over states 6..11 (lanes 8, 9, 10, 12, 13, 14) of c[s-6] x_s
__device__ __forceinline__ double mv6a(double x, const double (&c)[6], double init) {
  double a = init;
  asm(WV_NOP_HEAD WV_M6HI("%[a]") : [a] "+&v"(a) : [x] "v"(x), WV_OPS6(c, c));
  return a;
}
// init + sum over states 0..5 (lanes 0, 1, 2, 4, 5, 6) of c[s] x_s
__device__ __forceinline__ double mv6lo_a(double x, const double (&c)[6], double init) {
  double a = init;
  asm(WV_NOP_HEAD WV_M6LO("%[a]") : [a] "+&v"(a) : [x] "v"(x), WV_OPS6(c, c));
  return a;
}
// One middle step of each chain of the Acl-free Riccati form (N > 12) in one block, so that the
// step's wait states come from its own independent FMAs instead of s_nop (8.4 cycles for 2 states):
// only m, the row-moved chain value, is a fresh VALU result at the block's start.  Every accumulator
// takes the same FMAs in the same order as the separate helpers (bitwise the same results).
//   backward: tk = w + sum_hi bcast(m) bc (mv6a);  s = m + sum_lo bcast(m) cat (mv6lo_a), then
//             s += sum bcast(tk) kc (mv12a(tk, kc, s)): s is the chain's next value
//   forward:  nu = -g + sum bcast(m) kc (mv12a);  ax = m + sum_hi bcast(m) cax (mv6a);
//             hb = sum bcast(nu) bc (mv12)
#define WV_FY(A, X, M, L) "v_fmac_f64_dpp %[" A "], %[" X "], %[" M "] row_newbcast:" #L " row_mask:0xf bank_mask:0xf\n\t"
__device__ __forceinline__ void chain_bwd(double m, const double (&bc)[6], const double (&cat)[6],
                                          const double (&kc)[12], double& tk, double& s) {
  asm(WV_NOP_HEAD
      WV_FY("t", "m", "b0", 8) WV_FY("s", "m", "a0", 0) WV_FY("t", "m", "b1", 9) WV_FY("s", "m", "a1", 1)
      WV_FY("t", "m", "b2", 10) WV_FY("s", "m", "a2", 2) WV_FY("t", "m", "b3", 12) WV_FY("s", "m", "a3", 4)
      WV_FY("t", "m", "b4", 13) WV_FY("t", "m", "b5", 14) WV_FY("s", "m", "a4", 5) WV_FY("s", "m", "a5", 6)
      // (tk's last write is two instructions back)
      WV_FY("s", "t", "k0", 0) WV_FY("s", "t", "k1", 1) WV_FY("s", "t", "k2", 2) WV_FY("s", "t", "k3", 4)
      WV_FY("s", "t", "k4", 5) WV_FY("s", "t", "k5", 6) WV_FY("s", "t", "k6", 8) WV_FY("s", "t", "k7", 9)
      WV_FY("s", "t", "k8", 10) WV_FY("s", "t", "k9", 12) WV_FY("s", "t", "k10", 13) WV_FY("s", "t", "k11", 14)
      : [t] "+&v"(tk), [s] "+&v"(s)
      : [m] "v"(m), WV_OPS6(b, bc), WV_OPS6(a, cat), WV_OPS12(k, kc));
}
__device__ __forceinline__ void chain_fwd(double m, const double (&kc)[12], const double (&cax)[6],
                                          const double (&bc)[12], double& nu, double& ax, double& hb) {
  asm(WV_NOP_HEAD
      WV_FY("n", "m", "k0", 0) WV_FY("x", "m", "c0", 8) WV_FY("n", "m", "k1", 1) WV_FY("x", "m", "c1", 9)
      WV_FY("n", "m", "k2", 2) WV_FY("x", "m", "c2", 10) WV_FY("n", "m", "k3", 4) WV_FY("x", "m", "c3", 12)
      WV_FY("n", "m", "k4", 5) WV_FY("n", "m", "k5", 6) WV_FY("n", "m", "k6", 8) WV_FY("n", "m", "k7", 9)
      WV_FY("n", "m", "k8", 10) WV_FY("n", "m", "k9", 12) WV_FY("n", "m", "k10", 13) WV_FY("n", "m", "k11", 14)
      WV_FY("x", "m", "c4", 13) WV_FY("x", "m", "c5", 14)
      // (nu's last write is two instructions back)
      WV_FY("h", "n", "d0", 0) WV_FY("h", "n", "d1", 1) WV_FY("h", "n", "d2", 2) WV_FY("h", "n", "d3", 4)
      WV_FY("h", "n", "d4", 5) WV_FY("h", "n", "d5", 6) WV_FY("h", "n", "d6", 8) WV_FY("h", "n", "d7", 9)
      WV_FY("h", "n", "d8", 10) WV_FY("h", "n", "d9", 12) WV_FY("h", "n", "d10", 13) WV_FY("h", "n", "d11", 14)
      : [n] "+&v"(nu), [x] "+&v"(ax), [h] "+&v"(hb)
      : [m] "v"(m), WV_OPS12(k, kc), WV_OPS6(c, cax), WV_OPS12(d, bc));
}
#undef WV_FY
#undef WV_OPS12
#undef WV_OPS6
#undef WV_M12
#undef WV_M6HI
#undef WV_M6LO
#else
// y_i = sum_c M[i][c] x_c, x_c broadcast from lane 4(c/3)+c%3 of each DPP row, M row i in `c`.
// Hazards (the compiler cannot see into the asm): a DPP instruction needs 2 wait states after a
// VALU write of ANY of its VGPR operands and 5 after an EXEC write.  Hence the leading s_nop 4 and
// three accumulators in rotation (each is re-read 3 instructions after it was written).
__device__ __forceinline__ double mv12(double x, const double (&c)[12]) {
  double a0 = 0.0, a1 = 0.0, a2 = 0.0;
  asm(WV_NOP_HEAD
      WV_FM("%[a0]", "%[c0]", 0) WV_FM("%[a1]", "%[c1]", 1) WV_FM("%[a2]", "%[c2]", 2)
      WV_FM("%[a0]", "%[c3]", 4) WV_FM("%[a1]", "%[c4]", 5) WV_FM("%[a2]", "%[c5]", 6)
      WV_FM("%[a0]", "%[c6]", 8) WV_FM("%[a1]", "%[c7]", 9) WV_FM("%[a2]", "%[c8]", 10)
      WV_FM("%[a0]", "%[c9]", 12) WV_FM("%[a1]", "%[c10]", 13) WV_FM("%[a2]", "%[c11]", 14)
      : [a0] "+&v"(a0), [a1] "+&v"(a1), [a2] "+&v"(a2)
      : [x] "v"(x), [c0] "v"(c[0]), [c1] "v"(c[1]), [c2] "v"(c[2]), [c3] "v"(c[3]), [c4] "v"(c[4]),
        [c5] "v"(c[5]), [c6] "v"(c[6]), [c7] "v"(c[7]), [c8] "v"(c[8]), [c9] "v"(c[9]), [c10] "v"(c[10]),
        [c11] "v"(c[11]));
  return (a0 + a1) + a2;
}
// sum over states 6..11 (lanes 8, 9, 10, 12, 13, 14) of c[s-6] x_s
__device__ __forceinline__ double mv6(double x, const double (&c)[6]) {
  double a0 = 0.0, a1 = 0.0, a2 = 0.0;
  asm(WV_NOP_HEAD
      WV_FM("%[a0]", "%[c0]", 8) WV_FM("%[a1]", "%[c1]", 9) WV_FM("%[a2]", "%[c2]", 10)
      WV_FM("%[a0]", "%[c3]", 12) WV_FM("%[a1]", "%[c4]", 13) WV_FM("%[a2]", "%[c5]", 14)
      : [a0] "+&v"(a0), [a1] "+&v"(a1), [a2] "+&v"(a2)
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
  asm(WV_NOP_HEAD
      WV_T2(0, 0, 0) WV_T2(1, 1, 1) WV_T2(2, 2, 0) WV_T2(4, 3, 1) WV_T2(5, 4, 0) WV_T2(6, 5, 1)
      WV_T2(8, 6, 0) WV_T2(9, 7, 1) WV_T2(10, 8, 0) WV_T2(12, 9, 1) WV_T2(13, 10, 0) WV_T2(14, 11, 1)
      : [a0] "+&v"(a0), [a1] "+&v"(a1), [b0] "+&v"(b0), [b1] "+&v"(b1)
      : [x0] "v"(x0), [x1] "v"(x1), WV_OPS12(p, c0), WV_OPS12(q, c1));
  y0 = a0 + a1;
  y1 = b0 + b1;
}
__device__ __forceinline__ void mv12x3(double x0, double x1, double x2, const double (&c0)[12],
                                       const double (&c1)[12], const double (&c2)[12], double& y0, double& y1,
                                       double& y2) {
  double a0 = 0.0, a1 = 0.0, b0 = 0.0, b1 = 0.0, d0 = 0.0, d1 = 0.0;
  asm(WV_NOP_HEAD
      WV_T3(0, 0, 0) WV_T3(1, 1, 1) WV_T3(2, 2, 0) WV_T3(4, 3, 1) WV_T3(5, 4, 0) WV_T3(6, 5, 1)
      WV_T3(8, 6, 0) WV_T3(9, 7, 1) WV_T3(10, 8, 0) WV_T3(12, 9, 1) WV_T3(13, 10, 0) WV_T3(14, 11, 1)
      : [a0] "+&v"(a0), [a1] "+&v"(a1), [b0] "+&v"(b0), [b1] "+&v"(b1), [d0] "+&v"(d0), [d1] "+&v"(d1)
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
  asm(WV_NOP_HEAD
      WV_FM("%[a1]", "%[c1]", 1) WV_FM("%[a2]", "%[c2]", 2) WV_FM("%[a0]", "%[c0]", 0)
      WV_FM("%[a1]", "%[c4]", 5) WV_FM("%[a2]", "%[c5]", 6) WV_FM("%[a0]", "%[c3]", 4)
      WV_FM("%[a1]", "%[c7]", 9) WV_FM("%[a2]", "%[c8]", 10) WV_FM("%[a0]", "%[c6]", 8)
      WV_FM("%[a1]", "%[c10]", 13) WV_FM("%[a2]", "%[c11]", 14) WV_FM("%[a0]", "%[c9]", 12)
      : [a0] "+&v"(a0), [a1] "+&v"(a1), [a2] "+&v"(a2)
      : [x] "v"(x), [c0] "v"(c[0]), [c1] "v"(c[1]), [c2] "v"(c[2]), [c3] "v"(c[3]), [c4] "v"(c[4]),
        [c5] "v"(c[5]), [c6] "v"(c[6]), [c7] "v"(c[7]), [c8] "v"(c[8]), [c9] "v"(c[9]), [c10] "v"(c[10]),
        [c11] "v"(c[11]));
  return (a1 + a2) + a0;
}

// init + sum over states 6..11 (lanes 8, 9, 10, 12, 13, 14) of c[s-6] x_s
__device__ __forceinline__ double mv6a(double x, const double (&c)[6], double init) {
  double a0 = init, a1 = 0.0, a2 = 0.0;
  asm(WV_NOP_HEAD
      WV_FM("%[a1]", "%[c0]", 8) WV_FM("%[a2]", "%[c1]", 9) WV_FM("%[a0]", "%[c2]", 10)
      WV_FM("%[a1]", "%[c3]", 12) WV_FM("%[a2]", "%[c4]", 13) WV_FM("%[a0]", "%[c5]", 14)
      : [a0] "+&v"(a0), [a1] "+&v"(a1), [a2] "+&v"(a2)
      : [x] "v"(x), [c0] "v"(c[0]), [c1] "v"(c[1]), [c2] "v"(c[2]), [c3] "v"(c[3]), [c4] "v"(c[4]),
        [c5] "v"(c[5]));
  return (a1 + a2) + a0;
}
// init + sum over states 0..5 (lanes 0, 1, 2, 4, 5, 6) of c[s] x_s
__device__ __forceinline__ double mv6lo_a(double x, const double (&c)[6], double init) {
  double a0 = init, a1 = 0.0, a2 = 0.0;
  asm(WV_NOP_HEAD
      WV_FM("%[a1]", "%[c0]", 0) WV_FM("%[a2]", "%[c1]", 1) WV_FM("%[a0]", "%[c2]", 2)
      WV_FM("%[a1]", "%[c3]", 4) WV_FM("%[a2]", "%[c4]", 5) WV_FM("%[a0]", "%[c5]", 6)
      : [a0] "+&v"(a0), [a1] "+&v"(a1), [a2] "+&v"(a2)
      : [x] "v"(x), [c0] "v"(c[0]), [c1] "v"(c[1]), [c2] "v"(c[2]), [c3] "v"(c[3]), [c4] "v"(c[4]),
        [c5] "v"(c[5]));
  return (a1 + a2) + a0;
}

#endif  // MPCQP_MV_MULTI_ACC
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
      asm volatile(WV_NOP_PERM "v_permlane16_swap_b32 %0, %2\n\tv_permlane16_swap_b32 %1, %3"
                   : "=&v"(ol), "=&v"(oh), "+&v"(lo), "+&v"(hi));
    else  // src.even <- vdst.odd
      asm volatile(WV_NOP_PERM "v_permlane16_swap_b32 %2, %0\n\tv_permlane16_swap_b32 %3, %1"
                   : "=&v"(ol), "=&v"(oh), "+&v"(lo), "+&v"(hi));
  } else {
    if constexpr (FROM < TO)  // vdst rows 2-3 <- src rows 0-1
      asm volatile(WV_NOP_PERM "v_permlane32_swap_b32 %0, %2\n\tv_permlane32_swap_b32 %1, %3"
                   : "=&v"(ol), "=&v"(oh), "+&v"(lo), "+&v"(hi));
    else  // src rows 0-1 <- vdst rows 2-3
      asm volatile(WV_NOP_PERM "v_permlane32_swap_b32 %2, %0\n\tv_permlane32_swap_b32 %3, %1"
                   : "=&v"(ol), "=&v"(oh), "+&v"(lo), "+&v"(hi));
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
__device__ __forceinline__ void ld12s(double (&c)[12], const double* p) {  // a column of a stored factor
#pragma unroll
  for (int i = 0; i < 12; ++i) c[i] = p[mo(i)];
}
// The same column as 12 separate ds_read_b64, issued without waiting: the compiler pairs ld12s's
// loads into ds_read2_b64, which moves 16 B per lane in 8 LDS-array cycles against 2 x 2 for two
// ds_read_b64.  The compiler does not track these loads: the values are valid only after
// lds_wait<n>(c), n = the number of LDS instructions issued after them that may stay in flight
// (LDS returns in order; lgkmcnt holds at most 15).
__device__ __forceinline__ unsigned lds_off(const double* p) {
  return (unsigned)(uintptr_t)(const __attribute__((address_space(3))) double*)p;
}
__device__ __forceinline__ void ldcol(double (&c)[12], const double* p) {
  static_assert(mo(11) * 8 == 1072 && mo(4) * 8 == 400, "column offsets below");
  const unsigned ad = lds_off(p);
  asm volatile(
      "ds_read_b64 %0, %12\n\t"
      "ds_read_b64 %1, %12 offset:96\n\t"
      "ds_read_b64 %2, %12 offset:192\n\t"
      "ds_read_b64 %3, %12 offset:288\n\t"
      "ds_read_b64 %4, %12 offset:400\n\t"
      "ds_read_b64 %5, %12 offset:496\n\t"
      "ds_read_b64 %6, %12 offset:592\n\t"
      "ds_read_b64 %7, %12 offset:688\n\t"
      "ds_read_b64 %8, %12 offset:784\n\t"
      "ds_read_b64 %9, %12 offset:880\n\t"
      "ds_read_b64 %10, %12 offset:976\n\t"
      "ds_read_b64 %11, %12 offset:1072"
      : "=&v"(c[0]), "=&v"(c[1]), "=&v"(c[2]), "=&v"(c[3]), "=&v"(c[4]), "=&v"(c[5]), "=&v"(c[6]),
        "=&v"(c[7]), "=&v"(c[8]), "=&v"(c[9]), "=&v"(c[10]), "=&v"(c[11])
      : "v"(ad));
}
template <int CNT>
__device__ __forceinline__ void lds_wait(double (&c)[12]) {
  static_assert(CNT >= 0 && CNT <= 15, "lgkmcnt range");
  asm volatile("s_waitcnt lgkmcnt(%12)"
               : "+&v"(c[0]), "+&v"(c[1]), "+&v"(c[2]), "+&v"(c[3]), "+&v"(c[4]), "+&v"(c[5]), "+&v"(c[6]),
                 "+&v"(c[7]), "+&v"(c[8]), "+&v"(c[9]), "+&v"(c[10]), "+&v"(c[11])
               : "n"(CNT));
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
#ifdef MPCQP_RBCAST_FMA
  double acc = 0.0;
  asm("s_nop 1\n\tv_fmac_f64_dpp %0, %1, %2 row_newbcast:%3 row_mask:0xf bank_mask:0xf"
      : "+&v"(acc)
      : "v"(x), "v"(one), "i"(L));
  return acc;
#else
  (void)one;  // one v_mov_b64_dpp; the compiler sees it and inserts the DPP wait states itself
  return __builtin_amdgcn_update_dpp(0.0, x, 0x150 + L, 0xF, 0xF, false);
#endif
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
    // register 3 holds the pad rows 12-15: identity, zero in every pivot column, never changes
#pragma unroll
    for (int v = 0; v < 3; ++v) {
      const double col = rbcast<p>(g[v], one);  // G[4v + grp][p]
      const double upd = jp ? -col * pinv : g[v] - col * rs;
      if (v == vp) g[v] = (grp == gp) ? (jp ? pinv : rs) : upd;  // row p
      else g[v] = upd;
    }
  });
}

// The Riccati recursion of c B'Q̄B + R' (R'_k foot blocks in F.Rt) -> G_k^-1, K_k, Acl_k in LDS.
template <int N, class SM>
// q2j: 2 q_j of the lane's column j = lane & 15 (j < 12), loaded once by the caller (a per-lane index
// into the parameters is a memory round trip)
__device__ void factorize_mfma(SM& sm, const mpcqp_params& p, const Adisc& A, double c, double dtm, double q2j) {
  auto& F = sm.u.f;
  const int j = threadIdx.x & 15, grp = threadIdx.x >> 4;
  mf4 Ad, At, cQ, P;
#pragma unroll
  for (int v = 0; v < 4; ++v) {
    const int u = 4 * v + grp;
    const bool in = u < 12 && j < 12;
    Ad[v] = in ? A.at(u, j) : 0.0;
    At[v] = in ? A.at(j, u) : 0.0;
    cQ[v] = (in && u == j) ? c * q2j : 0.0;
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
      if (u < 12 && j < 12 && u / 3 == j / 3) rv = F.rt(k)[6 * (u / 3) + sym6(u % 3, j % 3)];
      if (u >= 12 && u == j) rv = 1.0;
      G[v] = rv;
    }
    const mf4 zero = {0.0, 0.0, 0.0, 0.0};
    // G = R' + B'(P B): P B needs only B's rows 6-11 (K-blocks 1, 2); B' P B likewise
    const mf4 PB = mfma_chain<1, 3>(P, Bk, zero);
    G = mfma_chain<1, 3>(Bk, PB, G);
    // the products that do not need G^-1 go to the matrix cores before the (VALU) inverse, so
    // they run under it (step 0 computes them for nothing)
    const mf4 PA = mfma_chain<0, 3>(P, Ad, zero);   // P A
    const mf4 Fm = mfma_chain<1, 3>(Bk, PA, zero);  // F = B' P A
    const mf4 Pq = mfma_chain<0, 3>(Ad, PA, cQ);    // cQ + A'P A
    gj_inverse12(G);
    if constexpr (std::remove_reference_t<decltype(F)>::HAS_ACL) {
      if (j < 12)
#pragma unroll
        for (int v = 0; v < 3; ++v) F.Gi[k][mo(4 * v + grp) + j] = G[v];
    } else {
#pragma unroll
      for (int v = 0; v < 3; ++v) {  // upper triangle (row <= column), rows packed
        const int row = 4 * v + grp;
        if (j < 12 && row <= j) F.Gp[k][poff(row) + j - row] = G[v];
      }
    }
    if (k >= 1) {
      const mf4 K = mfma_chain<0, 3>(G, Fm, zero);          // K = G^-1 F
      if (j < 12)
#pragma unroll
        for (int v = 0; v < 3; ++v) F.K[k - 1][mo(4 * v + grp) + j] = K[v];
      if constexpr (std::remove_reference_t<decltype(F)>::HAS_ACL) {
        if (k <= N - 2) {
          mf4 nBt;
#pragma unroll
          for (int v = 0; v < 4; ++v) nBt[v] = -Bt[v];
          const mf4 Acl = mfma_chain<0, 3>(nBt, K, Ad);       // A - B K
          if (j < 12)
#pragma unroll
            for (int v = 0; v < 3; ++v) F.Acl[k - 1][mo(4 * v + grp) + j] = Acl[v];
        }
      }
      mf4 nF;
#pragma unroll
      for (int v = 0; v < 4; ++v) nF[v] = -Fm[v];
      P = mfma_chain<0, 3>(nF, K, Pq);  // cQ + A'PA - F'K
    }
  }
  wave_sync();
}

// ---- OSQP scale_data (scaling.c) as a kernel of its own -------------------------------------------
// Ruiz equilibration is embarrassingly parallel over the columns of P~ = c D H D, so it runs before
// wave_kernel with one thread per column (NTS threads per robot) and, for n <= 128, the column of H
// generated once into registers instead of once per pass.  It writes a per-robot image (ScaleImg:
// D, E, the scaled gradient q~, c, the warm-start branch, and for warm slots the raw gradient) that
// wave_kernel reads in place of its own setup.  H's columns come from the same closed
// form as before (see gen_col), so every norm is binary64; only the order of the cost-scaling sum
// over columns differs from the single-wave version (a different but equally exact summation).
// B6_k Gram pivot ratio below which a robot is handed to the Riccati form (scale_kernel's screen)
#ifndef MPCQP_SCHUR_GRAM_TOL
#define MPCQP_SCHUR_GRAM_TOL 1e-6
#endif
constexpr double SCHUR_GRAM_TOL = MPCQP_SCHUR_GRAM_TOL;
// The Schur form's hand-off to the Riccati form (mpcqp_schur.h), decided at every update_info
// iteration from the latest factorization's max_i S_ii (a lower bound on the condition of S) and that
// iteration's observed cancellation of the push-through identity, schur_solve's
// amp = max|R'^-1 w| / max|u|: one KKT solve then loses about eps * S_max * amp of relative accuracy.
// A robot leaves when S_max * amp > SCHUR_AMP or S_max > SCHUR_SMAX (a hard cap).
// History: round 4 handed over on S_max > 1e4 (four feet in contact, state weights x 5 / x 100: u0 off
// the oracle by 4e-4 / 1e-3 without a hand-off, 9e-7 with it); round 5 lowered that to 3e3 after a
// loop change moved FMA contraction and the mixed-gait golden set from 1.0e-9 to 1.3e-7.  Round 6
// (profiles/r06/cancel: 7,254 robots — stance / mixed at weights x 1, 5, 100, the golden sets, C2 and
// C5 samples — solved to the end by the Schur form in builds with -ffp-contract=fast and =on): the
// worst u0 error of the robots a bound keeps, S_max <= 3e3: 8.3e-9 (fast) / 6.8e-9 (on), 52 handed
// over; S_max * amp <= 5e4: 2.4e-9 / 2.0e-9, 69 handed over (C2: 0 of 2048, C5: 14 of 2048);
// <= 3e4: 1.1e-9 / 8.1e-10 but C5 hands over 101 of 8192 robots and takes 3.15 ms instead of 2.91
// (profiles/r06/cancel/ab.txt: a few late hand-offs re-solved from the start end the batch).
#ifndef MPCQP_SCHUR_SMAX
#define MPCQP_SCHUR_SMAX 1e4
#endif
constexpr double SCHUR_SMAX = MPCQP_SCHUR_SMAX;
#ifndef MPCQP_SCHUR_AMP
#define MPCQP_SCHUR_AMP 5e4
#endif
constexpr double SCHUR_AMP = MPCQP_SCHUR_AMP;
template <int N>
struct ScaleImg {
  static constexpr int n = ND * N, m = CD * N;
  static constexpr int D = 0, E = D + n, Q = E + m, QN = Q + n, CS = QN + n, MODE = CS + 1, DEGEN = MODE + 1,
                       SIZE = DEGEN + 1;
  static_assert(SIZE == scale_image_doubles(N), "scale image layout");
};

template <int N>
struct ScaleCfg {
  static constexpr int n = ND * N, m = CD * N;
  // Columns of H cached in registers across the passes (off: since the bound-decided passes, H is
  // generated once per robot, and without the cache four robots fit a CU at N = 10)
#ifndef MPCQP_SCALE_HREG_MAXN
#define MPCQP_SCALE_HREG_MAXN 0
#endif
  static constexpr bool HREG = N <= MPCQP_SCALE_HREG_MAXN;
#ifndef MPCQP_SCALE_TPC
#define MPCQP_SCALE_TPC 2
#endif
#ifndef MPCQP_SCALE_TPC_LONG
#define MPCQP_SCALE_TPC_LONG 1
#endif
  static constexpr int TPC = HREG ? MPCQP_SCALE_TPC : MPCQP_SCALE_TPC_LONG;  // threads per column (adjacent lanes)
  static constexpr int BPT = (N + TPC - 1) / TPC;    // horizon blocks of the column per thread
  // at least two waves: wave 1 runs the degenerate-feet screen (one lane per horizon step) while
  // wave 0 runs the gradient sweep, so N <= 5 (n <= 60) still launches threads 64 .. 64 + N - 1
  static constexpr int NTS = ((TPC * n + 63) / 64) * 64 > 64 + N ? ((TPC * n + 63) / 64) * 64 : ((64 + N + 63) / 64) * 64;
  static constexpr int NWS = NTS / 64;
  // waves per SIMD the register allocation must allow (launch bounds): two, i.e. 256 VGPRs and no
  // spills.  N = 10: two waves per robot, four robots per CU; N = 20: four waves per robot, two per
  // CU (three per CU spilled 43 VGPRs: the same step time, 21 MB more HBM traffic per C4 solve,
  // profiles/r05/w20; three waves at N = 10 is slower, profiles/r05/sweep_reg)
#ifdef MPCQP_SCALE_WPE
  static constexpr int WPE = MPCQP_SCALE_WPE;
#else
  static constexpr int WPE = 2;
#endif
  static constexpr int RPT = (m + NTS - 1) / NTS;   // constraint rows per thread
};

template <int N>
struct ScaleSmem {
  using C = Cfg<N>;
  alignas(16) double Bw[N][3][ND];
  double rec[C::REC];
  double D[2][C::n], q[C::n], qn[C::n], E[2][C::m];  // D, E double-buffered over the Ruiz passes
  double lam[N][ND];
  double vec[2][16];
  double Ap[2][C::m];
  double red[2][16];
  double cm0[C::n];      // raw column norms of H (the first pass, D = 1)
  double red4[2][5 * 16];  // bound passes: per-wave partials, double-buffered by pass parity
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
// SM: any LDS image with the B_w rows (Bw[N][3][ND]).
template <int N, int NB, bool UNROLL, class SM, class Sink>
__device__ __forceinline__ void gen_col(const SM& sm, const mpcqp_params& p, const Adisc& A, double dtm,
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

}  // namespace wv
}  // namespace mpcqp
