// mpcqp_schur.h — the KKT solve of wave_kernel for horizons N <= 10 through the problem's
// velocity-impulse structure (a Woodbury / Schur-complement form with a dense 6N x 6N core),
// replacing the Riccati chains: every ADMM iteration becomes one dense 6N x 6N mat-vec spread over
// the 64 lanes plus per-leg 3x3 and per-step 6x12 products, with no sequential horizon recursion.
// Not installed.
//
// Structure (ConvexMpc.cpp:110-211; A_c is nilpotent on the 12 moving states, Ac^2 = 0).  An input
// u_j enters the state only through its impulse v_j = B_j^(6) u_j on the angular / linear
// velocities (rows 6-11 of B_d(j): I_w^-1 [r_l]x dt and dt/m I), and
//   x_{i+1}[6:12] = sum_{j<=i} v_j,   x_{i+1}[0:6] = Ac6 sum_{j<=i} (i - j) v_j,
// so B'Q̄B = B6' M B6 with B6 = blockdiag(B_j^(6)) (6N x 12N) and the 6N x 6N matrix
//   M_jl = beta_jl Qv + alpha_jl Ac6' Qp Ac6,  beta_jl = N - max(j,l),
//   alpha_jl = sum_{i=max(j,l)}^{N-1} (i - j)(i - l),  Qv = diag 2q[6:12], Qp = diag 2q[0:6].
// OSQP's reduced KKT matrix (scaled) is K = D (c B6'M B6 + R') D with R' = c R + D^-1 (sigma I +
// A~' diag(rho) A~) D^-1, 3x3 block-diagonal per foot (mpcqp_wave.hip header).  With C = c M,
// G = B6 R'^-1 B6' = L L' (6x6 blocks per step, Cholesky), Li = L^-1, S = I + L' C L (SPD, all
// eigenvalues >= 1, condition ~1e0-1e3 on the Go1 workload):
//   (c B6'M B6 + R')^-1 w = R'^-1 w - B' (I - S^-1) B w,   B := Li B6 R'^-1  (6N x 12N, per step 6x12)
// (push-through identity; exact in real arithmetic).  Per factorization (rho change): R'^-1 per
// foot, B (per step), S (6N x 6N) and Q = I - S^-1 by a blocked Gauss-Jordan sweep (schur_gj_mfma).  Per ADMM
// iteration:  z = B w (6x12 per step),  q = Q z (dense, one lane per row of Q),  u = R'^-1 w - B' q.
//
// Lane roles inside the one wave of a robot: the ADMM layout of wave_kernel (variable lanes: step
// 4r + gray(q) of round r in DPP row q, lane 4 leg + a) and, for the dense part, one lane per impulse
// unknown i = 6 k + c (step k, component c: omega_x,y,z, v_x,y,z), i < 6N <= 60.  The two meet
// through LDS (w out, q back), in order within the wave.
#pragma once
#include "mpcqp_wave_common.h"

// 1 (default): Q = I - S^-1 by the blocked Gauss-Jordan sweep on the matrix cores (schur_gj_mfma);
// 0: the in-register scalar sweep (schur_gj_valu).  Same box, 3 repetitions
// (profiles/r06/gj_mfma/ab_final.txt): C2 1.549 -> 1.537 ms, C5 2.925 -> 2.901 ms; the sweep alone
// 30.6k -> 27.1k cycles (tools/mb/mb_gjsweep).  Built with -mllvm -amdgpu-mfma-vgpr-form (Makefile):
// MFMA results in VGPRs, without which the tiles spill.
#ifndef MPCQP_GJ_MFMA
#define MPCQP_GJ_MFMA 1
#endif

namespace mpcqp {
namespace wv {

template <int N>
struct SchurCfg {
  static_assert(N >= 1 && N <= 10, "one lane per impulse unknown: 6N <= 64");
  static constexpr int NI = 6 * N;  // impulse unknowns
  // LDS row stride of Q (doubles).  A row is read as 64 columns, but 62 doubles apart the rows of
  // lanes i .. i+7 of a ds_read_b128 sit on eight distinct 16-B bank groups (a 512-B stride would
  // put all of them on one), and the two columns a row reads past its end (62, 63: the next row's
  // first two, or a zero tail) only ever multiply pad unknowns, whose z is 0.
  static constexpr int QS = 62;
  static constexpr int BS = 14;  // row stride of B in LDS: 112 B, conflict-free b128 rows
};

// Factorization scratch: lives in the rows of Q (which every factorization rewrites at its end).
template <int N>
struct SchurScratch {
  static constexpr int NI = SchurCfg<N>::NI;
  alignas(16) double Rt[N][4][6];   // R'_k foot blocks, upper triangle (00 01 02 11 12 22)
  alignas(16) double Ri[N][4][9];   // R'^-1 foot blocks, row-major
  alignas(16) double B6R[NI][12];   // rows of B6 R'^-1 (step k = i / 6)
  alignas(16) double G[N][36];      // G_k = B_k R'_k^-1 B_k' (row c written by lane 6k + c)
};

template <int N>
struct SchurLds {
  static constexpr int NI = SchurCfg<N>::NI, QS = SchurCfg<N>::QS, BS = SchurCfg<N>::BS;
  union {
    // I - S^-1: row i at Q + QS i in absolute column order, columns NI .. QS-1 zero, plus a zero
    // tail for the last row's columns 62, 63
    alignas(16) double Q[NI * QS + 2];
    SchurScratch<N> s;
  };
  alignas(16) double Bm[NI][BS];      // B = Li B6 R'^-1: row i = 6 k + c (12 used)
  alignas(16) double wv[12 * N + 4];  // w = D^-1 rhs by variable index 12 k + 3 leg + a
  alignas(16) double qv[64];          // q = Q z by impulse index
};
static_assert(sizeof(SchurScratch<10>) <= sizeof(double) * (60 * 62 + 2), "scratch must fit in Q");

// ---- cross-lane pieces ---------------------------------------------------------------------------
// acc[l % 4] += bcast_l(x) * c[l] for the 16 lanes l of x's DPP row (four accumulators in rotation:
// each is re-read four instructions after its last write).  Hazard: x and c may have been written
// by VALU just before (2 wait states) or EXEC by a branch (5): the leading s_nop 4.
#define SC_F(A, C, L) "v_fmac_f64_dpp %[" A "], %[x], %[" C "] row_newbcast:" #L " row_mask:0xf bank_mask:0xf\n\t"
#define SC_MV16_BODY                                                                              \
  SC_F("a0", "c0", 0) SC_F("a1", "c1", 1) SC_F("a2", "c2", 2) SC_F("a3", "c3", 3)                 \
  SC_F("a0", "c4", 4) SC_F("a1", "c5", 5) SC_F("a2", "c6", 6) SC_F("a3", "c7", 7)                 \
  SC_F("a0", "c8", 8) SC_F("a1", "c9", 9) SC_F("a2", "c10", 10) SC_F("a3", "c11", 11)             \
  SC_F("a0", "c12", 12) SC_F("a1", "c13", 13) SC_F("a2", "c14", 14) SC_F("a3", "c15", 15)
#define SC_MV16_OPS                                                                               \
  : [a0] "+&v"(a0), [a1] "+&v"(a1), [a2] "+&v"(a2), [a3] "+&v"(a3)                                    \
  : [x] "v"(x), [c0] "v"(c[0]), [c1] "v"(c[1]), [c2] "v"(c[2]), [c3] "v"(c[3]), [c4] "v"(c[4]),   \
    [c5] "v"(c[5]), [c6] "v"(c[6]), [c7] "v"(c[7]), [c8] "v"(c[8]), [c9] "v"(c[9]), [c10] "v"(c[10]), \
    [c11] "v"(c[11]), [c12] "v"(c[12]), [c13] "v"(c[13]), [c14] "v"(c[14]), [c15] "v"(c[15])
// HEAD: x may have just been written (the first block of a sequence); otherwise x was read by an
// earlier block of the sequence (WV_NOP_INNER)
template <bool HEAD>
__device__ __forceinline__ void mv16(double x, const double* c, double& a0, double& a1, double& a2, double& a3) {
  if constexpr (HEAD)
    asm(WV_NOP_HEAD SC_MV16_BODY SC_MV16_OPS);
  else
    asm(WV_NOP_INNER SC_MV16_BODY SC_MV16_OPS);
}
#undef SC_MV16_BODY
#undef SC_MV16_OPS
#undef SC_F
// s[l] += bcast_l(x) * g for the 16 lanes l of x's DPP row (a rank-1 row update; independent
// destinations, so no accumulator latency).
#define SC_U(L) "v_fmac_f64_dpp %[s" #L "], %[x], %[g] row_newbcast:" #L " row_mask:0xf bank_mask:0xf\n\t"
__device__ __forceinline__ void upd16(double x, double g, double* s) {
  asm("s_nop 4\n\t"
      SC_U(0) SC_U(1) SC_U(2) SC_U(3) SC_U(4) SC_U(5) SC_U(6) SC_U(7)
      SC_U(8) SC_U(9) SC_U(10) SC_U(11) SC_U(12) SC_U(13) SC_U(14) SC_U(15)
      : [s0] "+&v"(s[0]), [s1] "+&v"(s[1]), [s2] "+&v"(s[2]), [s3] "+&v"(s[3]), [s4] "+&v"(s[4]), [s5] "+&v"(s[5]),
        [s6] "+&v"(s[6]), [s7] "+&v"(s[7]), [s8] "+&v"(s[8]), [s9] "+&v"(s[9]), [s10] "+&v"(s[10]),
        [s11] "+&v"(s[11]), [s12] "+&v"(s[12]), [s13] "+&v"(s[13]), [s14] "+&v"(s[14]), [s15] "+&v"(s[15])
      : [x] "v"(x), [g] "v"(g));
}
#undef SC_U
// s[e] += bcast_(O+e)(x) * g for e < 4: a quarter of upd16, so that other work can be scheduled
// between the quarters (s_nop 1: x may have been written by VALU just before)
#define SC_U4(A, L) "v_fmac_f64_dpp %[" A "], %[x], %[g] row_newbcast:" #L " row_mask:0xf bank_mask:0xf\n\t"
// FIRST: the first quarter of a chunk's update (x may have just been written); the others follow a
// block that read the same x (WV_NOP_INNER1)
#define SC_DEF_UPD4(O, L0, L1, L2, L3)                                                               \
  template <bool FIRST>                                                                              \
  __device__ __forceinline__ void upd4_##O(double x, double g, double* s) {                          \
    if constexpr (FIRST)                                                                             \
      asm(WV_NOP_HEAD1 SC_U4("s0", L0) SC_U4("s1", L1) SC_U4("s2", L2) SC_U4("s3", L3)               \
          : [s0] "+&v"(s[0]), [s1] "+&v"(s[1]), [s2] "+&v"(s[2]), [s3] "+&v"(s[3])                      \
          : [x] "v"(x), [g] "v"(g));                                                                 \
    else                                                                                             \
      asm(WV_NOP_INNER1 SC_U4("s0", L0) SC_U4("s1", L1) SC_U4("s2", L2) SC_U4("s3", L3)              \
          : [s0] "+&v"(s[0]), [s1] "+&v"(s[1]), [s2] "+&v"(s[2]), [s3] "+&v"(s[3])                      \
          : [x] "v"(x), [g] "v"(g));                                                                 \
  }
SC_DEF_UPD4(0, 0, 1, 2, 3)
SC_DEF_UPD4(4, 4, 5, 6, 7)
SC_DEF_UPD4(8, 8, 9, 10, 11)
SC_DEF_UPD4(12, 12, 13, 14, 15)
#undef SC_DEF_UPD4
#undef SC_U4
// columns 16 C .. 16 C + 15 of the lane's row s (those below NI: pad columns stay 0)
template <int C, int NI, bool HEAD = true>
__device__ __forceinline__ void upd_chunk(double x, double g, double* s) {
  if constexpr (16 * C + 0 < NI) upd4_0<HEAD>(x, g, s + 16 * C + 0);
  if constexpr (16 * C + 4 < NI) upd4_4<false>(x, g, s + 16 * C + 4);
  if constexpr (16 * C + 8 < NI) upd4_8<false>(x, g, s + 16 * C + 8);
  if constexpr (16 * C + 12 < NI) upd4_12<false>(x, g, s + 16 * C + 12);
}

// a_j = sum_e bcast_(Lj)(x[e]) * v[e] for four lanes Lj of x's DPP row, each an fma chain in e
// order starting from 0 (so lanes i and m form the dot product of their vectors bitwise alike); the
// four chains interleave, each accumulator re-read four instructions after its last write.
#define SC_D(A, X, V, L) "v_fmac_f64_dpp %[" A "], %[" X "], %[" V "] row_newbcast:%[" L "] row_mask:0xf bank_mask:0xf\n\t"
#define SC_D4(X, V) SC_D("a0", X, V, "l0") SC_D("a1", X, V, "l1") SC_D("a2", X, V, "l2") SC_D("a3", X, V, "l3")
#define SC_DOT_BODY SC_D4("x0", "v0") SC_D4("x1", "v1") SC_D4("x2", "v2") SC_D4("x3", "v3") SC_D4("x4", "v4") SC_D4("x5", "v5")
#define SC_DOT_OPS                                                                                \
  : [a0] "+&v"(a0), [a1] "+&v"(a1), [a2] "+&v"(a2), [a3] "+&v"(a3)                                    \
  : [x0] "v"(x[0]), [x1] "v"(x[1]), [x2] "v"(x[2]), [x3] "v"(x[3]), [x4] "v"(x[4]), [x5] "v"(x[5]), \
    [v0] "v"(v[0]), [v1] "v"(v[1]), [v2] "v"(v[2]), [v3] "v"(v[3]), [v4] "v"(v[4]), [v5] "v"(v[5]), \
    [l0] "n"(L0), [l1] "n"(L1), [l2] "n"(L2), [l3] "n"(L3)
// HEAD: the first block after x's row copies were made
template <bool HEAD, int L0, int L1, int L2, int L3>
__device__ __forceinline__ void dot6x4(const double (&x)[6], const double (&v)[6], double& a0, double& a1, double& a2,
                                       double& a3) {
  if constexpr (HEAD)
    asm(WV_NOP_HEAD1 SC_DOT_BODY SC_DOT_OPS);
  else
    asm(WV_NOP_INNER1 SC_DOT_BODY SC_DOT_OPS);
}
#undef SC_DOT_BODY
#undef SC_DOT_OPS
#undef SC_D4
#undef SC_D

// Row broadcasts: c_s = the value DPP row s holds, in every DPP row (lane l of each row gets lane
// l of row s).  permlane16_swap(v, v) gives [r0 r0 r2 r2] / [r1 r1 r3 r3] (rows 0..3), and a
// permlane32_swap of each of those with itself gives [r0 x4] / [r2 x4] and [r1 x4] / [r3 x4].
__device__ __forceinline__ void rowbcast4(double v, double& c0, double& c1, double& c2, double& c3) {
  const unsigned lo = (unsigned)__double2loint(v), hi = (unsigned)__double2hiint(v);
  const auto l16 = __builtin_amdgcn_permlane16_swap(lo, lo, false, false);
  const auto h16 = __builtin_amdgcn_permlane16_swap(hi, hi, false, false);
  const auto la = __builtin_amdgcn_permlane32_swap(l16[0], l16[0], false, false);
  const auto ha = __builtin_amdgcn_permlane32_swap(h16[0], h16[0], false, false);
  const auto lb = __builtin_amdgcn_permlane32_swap(l16[1], l16[1], false, false);
  const auto hb = __builtin_amdgcn_permlane32_swap(h16[1], h16[1], false, false);
  c0 = __hiloint2double((int)ha[0], (int)la[0]);
  c2 = __hiloint2double((int)ha[1], (int)la[1]);
  c1 = __hiloint2double((int)hb[0], (int)lb[0]);
  c3 = __hiloint2double((int)hb[1], (int)lb[1]);
}

#if MPCQP_GJ_MFMA
// ---- blocked Gauss-Jordan on the matrix cores (MPCQP_GJ_MFMA) ------------------------------------
// S as 16x16 tiles in the MFMA result layout of mpcqp_wave_common.h (tile X[I][J]: lane j + 16 g,
// register v holds S[16 I + 4 v + g][16 J + j]), in which register kb of a tile is the B operand of
// K-block kb and, of the transposed tile, the A operand: C += A X takes A' and X as they are.

// x: odd DPP rows <-> y: even rows (permlane16_swap); x: rows 2, 3 <-> y: rows 0, 1 (permlane32_swap)
__device__ __forceinline__ void swap16d(double& x, double& y) {
  const auto l = __builtin_amdgcn_permlane16_swap((unsigned)__double2loint(x), (unsigned)__double2loint(y), false, false);
  const auto h = __builtin_amdgcn_permlane16_swap((unsigned)__double2hiint(x), (unsigned)__double2hiint(y), false, false);
  x = __hiloint2double((int)h[0], (int)l[0]);
  y = __hiloint2double((int)h[1], (int)l[1]);
}
__device__ __forceinline__ void swap32d(double& x, double& y) {
  const auto l = __builtin_amdgcn_permlane32_swap((unsigned)__double2loint(x), (unsigned)__double2loint(y), false, false);
  const auto h = __builtin_amdgcn_permlane32_swap((unsigned)__double2hiint(x), (unsigned)__double2hiint(y), false, false);
  x = __hiloint2double((int)h[0], (int)l[0]);
  y = __hiloint2double((int)h[1], (int)l[1]);
}
// 4x4 (DPP row, register) transpose: afterwards y[r] in row g = y[g] in row r before
// (tools/mb/mfma_f64_layout.hip checks it)
__device__ __forceinline__ void transpose_rows(double (&y)[4]) {
  swap16d(y[0], y[1]);
  swap16d(y[2], y[3]);
  swap32d(y[0], y[2]);
  swap32d(y[1], y[3]);
}

// a += (lane L's a) * g, one register (GJ_FMA1) or four (GJ_FMA4) per asm block; HEAD: the block
// may follow the VALU write of a source (2 wait states).  Volatile, so the blocks keep their order:
// a pivot's first block follows the previous pivot's last one by the next pivot's head block, and the
// previous pivot's new column (a plain select, which the compiler may sink to its first use) is in
// the head block.  tools/isa_hazards.py checks the placement.
#define GJ_F(I) "v_fmac_f64_dpp %[a" #I "], %[a" #I "], %[g] row_newbcast:%[l] row_mask:0xf bank_mask:0xf\n\t"
template <int L, bool HEAD>
__device__ __forceinline__ void gj_fma1(double& a0, double g) {
  if constexpr (HEAD)
    asm volatile("s_nop 1\n\t" GJ_F(0) : [a0] "+v"(a0) : [g] "v"(g), [l] "n"(L));
  else
    asm volatile(GJ_F(0) : [a0] "+v"(a0) : [g] "v"(g), [l] "n"(L));
}
template <int L, bool HEAD>
__device__ __forceinline__ void gj_fma4(double& a0, double& a1, double& a2, double& a3, double g) {
  if constexpr (HEAD)
    asm volatile("s_nop 1\n\t" GJ_F(0) GJ_F(1) GJ_F(2) GJ_F(3)
        : [a0] "+v"(a0), [a1] "+v"(a1), [a2] "+v"(a2), [a3] "+v"(a3) : [g] "v"(g), [l] "n"(L));
  else
    asm volatile(GJ_F(0) GJ_F(1) GJ_F(2) GJ_F(3)
        : [a0] "+v"(a0), [a1] "+v"(a1), [a2] "+v"(a2), [a3] "+v"(a3) : [g] "v"(g), [l] "n"(L));
}
#undef GJ_F
// columns of pivot p's row update other than p (overwritten) and p + 1 (updated first), column p - 1
// first: the previous pivot's last write (its new column) may sit just before the update, so it goes
// into the block with the wait states
template <int PV>
struct GjCols {
  static constexpr int count(int p) { return PV - 1 - (p + 1 < PV ? 1 : 0); }
  static constexpr int at(int p, int n) {
    if (p > 0 && n == 0) return p - 1;
    int c = 0;
    for (int k = p > 0 ? 1 : 0;; ++c) {
      if (c == p || c == p + 1 || c == p - 1) continue;
      if (k == n) return c;
      ++k;
    }
  }
};
// In-place Gauss-Jordan inverse of a symmetric positive definite 16x16 tile in the row layout (lane t
// of every DPP row holds row t in R[0..15]) whose first PV rows / columns are the matrix and whose pad
// holds the identity; scalar pivots, no pivoting.  Row p reaches every lane by row_newbcast, so a
// pivot is one prelude (pivot, reciprocal, the lane's factor) and PV - 1 DPP FMAs.  Software
// pipelined: column p + 1 is updated first, then the next prelude's dependent chain is issued among
// the other columns' FMAs.  issue(IC<p>) runs at pivot p (the caller's matrix-core work).
template <int PV, class Issue>
__device__ __forceinline__ void gj_rows(double (&R)[16], int li, Issue&& issue) {
  const double one = 1.0;
  struct Pv {
    double g, newc;
  };
  auto prelude = [&](auto P) __attribute__((always_inline)) {
    constexpr int p = decltype(P)::value;
    Pv o;
    const double pinv = recip(rbcast<p>(R[p], one));
    const double cp = R[p] * pinv;
    o.g = li == p ? pinv - 1.0 : -cp;
    o.newc = li == p ? pinv : -cp;
    return o;
  };
  Pv cur = prelude(IC<0>{});
  sfor<0, PV>([&](auto P) __attribute__((always_inline)) {
    constexpr int p = decltype(P)::value;
    using C = GjCols<PV>;
    constexpr int n = C::count(p), n4 = n / 4;
    // the other columns' blocks: chunk q < n4 four columns, then the single columns
    auto chunk = [&](auto Q) __attribute__((always_inline)) {
      constexpr int q = decltype(Q)::value;
      if constexpr (q < n4) {
        constexpr int c0 = C::at(p, 4 * q), c1 = C::at(p, 4 * q + 1), c2 = C::at(p, 4 * q + 2), c3 = C::at(p, 4 * q + 3);
        gj_fma4<p, q == 0>(R[c0], R[c1], R[c2], R[c3], cur.g);
      }
    };
    auto singles = [&]() __attribute__((always_inline)) {
      sfor<4 * n4, n>([&](auto Q) __attribute__((always_inline)) {
        constexpr int q = decltype(Q)::value;
        constexpr int c0 = C::at(p, q);
        gj_fma1<p, q == 0>(R[c0], cur.g);
      });
    };
    Pv nxt;
    if constexpr (p + 1 < PV) {
      gj_fma1<p, true>(R[p + 1], cur.g);
      nxt = prelude(IC<p + 1>{});
    }
    issue(P);
    sfor<0, n4>(chunk);
    singles();
    R[p] = cur.newc;
    if constexpr (p + 1 < PV) cur = nxt;
  });
}

// Q = I - S^-1 by a blocked Gauss-Jordan sweep over 16x16 tiles (NB = ceil(6N / 16) block rows).
// Step k: P = X_kk^-1 (VALU, gj_rows), X_kj <- P X_kj, X_ij <- X_ij - X_ik X_kj, X_kk <- P (i, j != k;
// the column panel X_ik <- -X_ik P is implied, below).  The sweep keeps X sign-symmetric,
// X_ba = s X_ab' with s = -1 when exactly one of blocks a, b has been swept, so one tile per pair
// {a, b} is kept, in the orientation the sweep needs next: (a, b), a < b, until step b needs row b,
// which transposes it through LDS (X_ba = -X_ab') and keeps (b, a) from then on.  X_ik enters only as
// an A operand, i.e. as X_ik' = s X_ki: a step is the row panel X_kj of every j != k and the update
// of every kept pair (9 chains of NB K-blocks at NB = 4).  The panel and update that produce the next
// pivot tile go first; the step's other MFMAs are issued among the next tile's pivots (GjPlanSym).
// Pad K-blocks of a short last block are skipped.
template <int NB, int k>
struct GjPlanSym {
  static constexpr int kn = k + 1 < NB ? k + 1 : -1;  // the next pivot block (its panel went first)
  // a chain: kind 0 the row panel X_kb -> RP[b], kind 2 the update of kept tile X_ab
  static constexpr int code(int kind, int a, int b) { return 100 * kind + 10 * a + b; }
  // the kept orientation of pair {i, j}, i < j, both != k, during step k
  static constexpr int orient(int i, int j) { return j < k ? code(2, j, i) : code(2, i, j); }
  // group 1: row panels and the updates whose B operand is the next pivot block's (lookahead) panel;
  // group 2: the updates that need a group-1 row panel
  static constexpr int list(int grp, int n) {
    int m = 0;
    if (grp == 1)
      for (int jj = 0; jj < NB; ++jj)
        if (jj != k && jj != kn) {
          if (m == n) return code(0, k, jj);
          ++m;
        }
    for (int i = 0; i < NB; ++i)
      for (int jj = i; jj < NB; ++jj) {
        if (i == k || jj == k || (i == kn && jj == kn)) continue;
        const int cd = i == jj ? code(2, i, i) : orient(i, jj);
        if (((cd % 10) == kn) == (grp == 1)) {
          if (m == n) return cd;
          ++m;
        }
      }
    return -1 - m;
  }
  static constexpr int count(int grp) { return -1 - list(grp, 1000); }
};

// S - I in the lane's row (lane t = row t, S[m] = column m; rows and columns NI..63 zero) -> Q in F.Q.
// pre(): run after the sweep, before the first store to Q (the factorization scratch lives there);
// mark(id): internal phase marks 60-64 (the caller records them after the sweep).
template <int N, class Pre, class Mark>
__device__ __forceinline__ void schur_gj_mfma(const double (&S)[64], SchurLds<N>& F, int t, Pre&& pre, Mark&& mark) {
  constexpr int NI = SchurCfg<N>::NI, QS = SchurCfg<N>::QS, NB = (NI + 15) / 16;
  const int j = t & 15, grp = t >> 4;
  mf4 X[NB][NB];
  // the upper tiles: X[I][J][v] in row g = S[16 I + 4 v + g] of lane 16 J + j, plus the identity
#pragma unroll
  for (int I = 0; I < NB; ++I)
#pragma unroll
    for (int v = 0; v < 4; ++v) {
      double y[4] = {S[16 * I + 4 * v], S[16 * I + 4 * v + 1], S[16 * I + 4 * v + 2], S[16 * I + 4 * v + 3]};
#ifndef MPCQP_GJ_DBG_NOCONV  // (microbenchmark builds only: timing without the tile transposes)
      transpose_rows(y);
#endif
#pragma unroll
      for (int J = I; J < NB; ++J) X[I][J][v] = y[J] + ((I == J && j == 4 * v + grp) ? 1.0 : 0.0);
    }
  mark(60);  // tiles made
  const mf4 zero = {0.0, 0.0, 0.0, 0.0};
  // LDS staging above the live scratch (R'^-1): the pivot tile, then one buffer per transposed tile
  double* stage = F.Q + 64 * N;
  static_assert(64 * N + 256 * NB <= NI * QS + 2, "staging inside Q");
  auto to_rows = [&](const mf4& d, double (&R)[16]) __attribute__((always_inline)) {
#pragma unroll
    for (int v = 0; v < 4; ++v) stage[16 * (4 * v + grp) + j] = d[v];
    wave_sync();
    const double2* r2 = reinterpret_cast<const double2*>(stage + 16 * j);
#pragma unroll
    for (int c = 0; c < 8; ++c) {
      const double2 w = r2[c];
      R[2 * c] = w.x;
      R[2 * c + 1] = w.y;
    }
    wave_sync();
  };
  auto from_rows = [&](const double (&R)[16]) __attribute__((always_inline)) {
    mf4 d;
    const bool b0 = (grp & 1) != 0, b1 = (grp & 2) != 0;
#pragma unroll
    for (int v = 0; v < 4; ++v) {
      const double lo = b0 ? R[4 * v + 1] : R[4 * v], hi = b0 ? R[4 * v + 3] : R[4 * v + 2];
      d[v] = b1 ? hi : lo;
    }
    return d;
  };
  constexpr int PV0 = NI < 16 ? NI : 16;
  mf4 P;
  {
    double R[16];
    to_rows(X[0][0], R);
    gj_rows<PV0>(R, j, [](auto) {});
    P = from_rows(R);
  }
  mark(61);  // first pivot tile swept
  sfor<0, NB>([&](auto K) __attribute__((always_inline)) {
    constexpr int k = decltype(K)::value;
    constexpr int PV = NI - 16 * k < 16 ? NI - 16 * k : 16;
    constexpr int KB = (PV + 3) / 4;
    using Plan = GjPlanSym<NB, k>;
    constexpr int kn = Plan::kn, n1 = Plan::count(1), n2 = Plan::count(2), NT = (n1 + n2) * KB;
    // row k before the step: X_kj (j > k, kept as is) and X_kj = -X_jk' (j < k, transposed here)
    mf4 T[NB];
#pragma unroll
    for (int jj = 0; jj < k; ++jj) {
      double* buf = stage + 256 * (1 + jj);
#pragma unroll
      for (int v = 0; v < 4; ++v) buf[16 * (4 * v + grp) + j] = X[jj][k][v];
      wave_sync();
#pragma unroll
      for (int v = 0; v < 4; ++v) T[jj][v] = -buf[16 * j + 4 * v + grp];
    }
#pragma unroll
    for (int jj = k + 1; jj < NB; ++jj) T[jj] = X[k][jj];
    mf4 NA[NB];  // (-X_ak)' = -s X_ka for a != k
#pragma unroll
    for (int a = 0; a < NB; ++a)
      if (a != k) NA[a] = a < k ? T[a] : -T[a];
    mark(62);  // row k transposed
    mf4 RP[NB];
    auto issue = [&](auto TT) __attribute__((always_inline)) {
      constexpr int tt = decltype(TT)::value;
      constexpr bool g1 = tt < n1 * KB;
      constexpr int kb = g1 ? tt / n1 : (tt - n1 * KB) / n2;
      constexpr int cd = g1 ? Plan::list(1, tt % n1) : Plan::list(2, (tt - n1 * KB) % n2);
      constexpr int kind = cd / 100, a = (cd / 10) % 10, b = cd % 10;
#ifdef MPCQP_GJ_DBG_NOTASK  // (microbenchmark builds only: timing without the MFMA tasks)
      if constexpr (true) {
      } else
#endif
      if constexpr (kind == 0)
        RP[b] = __builtin_amdgcn_mfma_f64_16x16x4f64(P[kb], T[b][kb], kb == 0 ? zero : RP[b], 0, 0, 0);
      else if constexpr (b == kn)
        X[a][b] = __builtin_amdgcn_mfma_f64_16x16x4f64(NA[a][kb], X[k][kn][kb], X[a][b], 0, 0, 0);
      else
        X[a][b] = __builtin_amdgcn_mfma_f64_16x16x4f64(NA[a][kb], RP[b][kb], X[a][b], 0, 0, 0);
    };
    if constexpr (kn >= 0) {
      // the next pivot tile's panel and update (a chain of 2 KB dependent MFMAs)
      X[k][kn] = mfma_chain<0, KB>(P, T[kn], zero);
      X[kn][kn] = mfma_chain<0, KB>(NA[kn], X[k][kn], X[kn][kn]);
      constexpr int PVn = NI - 16 * kn < 16 ? NI - 16 * kn : 16;
      double R[16];
      to_rows(X[kn][kn], R);
      mark(63);  // lookahead done, next pivot tile in rows
#ifdef MPCQP_GJ_DBG_NOROWS  // (microbenchmark builds only: timing without the pivot sweeps)
      sfor<0, NT>(issue);
      if constexpr (false)
#endif
      gj_rows<PVn>(R, j, [&](auto Pp) __attribute__((always_inline)) {
        constexpr int p = decltype(Pp)::value;
        sfor<p * NT / PVn, (p + 1) * NT / PVn>(issue);
      });
#pragma unroll
      for (int jj = 0; jj < NB; ++jj)
        if (jj != k && jj != kn) X[k][jj] = RP[jj];
      X[k][k] = P;
      P = from_rows(R);
    } else {
      sfor<0, NT>(issue);
#pragma unroll
      for (int jj = 0; jj < NB; ++jj)
        if (jj != k) X[k][jj] = RP[jj];
      X[k][k] = P;
    }
    mark(64);  // step done
  });
  pre();
  wave_sync();
#ifndef MPCQP_GJ_DBG_NOSTORE  // (microbenchmark builds only: timing without the stores to Q)
  // Q = I - X from the kept tiles (diagonal, and (b, a) with b > a: X_ab = X_ba', S^-1 symmetric);
  // columns 16 NB .. QS-1 of a short horizon: zero
  if constexpr (16 * NB < QS) {
    if (t < NI)
#pragma unroll
      for (int m = 16 * NB; m < QS; m += 2) *reinterpret_cast<double2*>(&F.Q[QS * t + m]) = make_double2(0.0, 0.0);
  }
#ifdef MPCQP_GJ_STORE_SEL
  // branch-free stores: an entry outside Q (pad rows / columns) goes to the lane's own slot of qv,
  // which the KKT solve and P~x write before they read it.  0.9k cycles less per factorization in
  // tools/mb/mb_gjsweep, but C2 / C5 unchanged within noise in the product (profiles/r06/gj_mfma/
  // store_ab.txt): off
  double* const dummy = &F.qv[t];
#endif
#pragma unroll
  for (int I = 0; I < NB; ++I)
#pragma unroll
    for (int J = 0; J <= I; ++J)
#pragma unroll
      for (int v = 0; v < 4; ++v) {
        const int r = 16 * I + 4 * v + grp, c = 16 * J + j;
        const double x = ((I == J && j == 4 * v + grp) ? 1.0 : 0.0) - X[I][J][v];
#ifdef MPCQP_GJ_STORE_SEL
        *(r < NI && c < QS ? &F.Q[QS * r + c] : dummy) = x;
        if (I != J) *(c < NI && r < QS ? &F.Q[QS * c + r] : dummy) = x;
#else
        if (r < NI && c < QS) F.Q[QS * r + c] = x;
        if (I != J && c < NI && r < QS) F.Q[QS * c + r] = x;
#endif
      }
#else
  {  // keep the sweep's results live
    double ck = 0.0;
#pragma unroll
    for (int I = 0; I < NB; ++I)
#pragma unroll
      for (int J = 0; J <= I; ++J)
#pragma unroll
        for (int v = 0; v < 4; ++v) ck += X[I][J][v];
    F.qv[t] = ck;
  }
#endif
  if (t == 0) *reinterpret_cast<double2*>(&F.Q[QS * NI]) = make_double2(0.0, 0.0);
}
#endif

// alpha_jl of M (integer valued, exact in binary64): sum_{i=max(j,l)}^{N-1} (i - j)(i - l)
__device__ __forceinline__ double alpha_jl(int N, int j, int l) {
  const int M = j > l ? j : l, K = N - 1, cnt = K - M + 1;
  const int s1 = (M + K) * cnt / 2;
  const int s2 = K * (K + 1) * (2 * K + 1) / 6 - (M - 1) * M * (2 * M - 1) / 6;
  return (double)(s2 - (j + l) * s1 + j * l * cnt);
}

// The in-register scalar sweep (MPCQP_GJ_MFMA == 0): S - I in the lane's row (lane t = row t) ->
// Q = I - S^-1 in F.Q.  pre(): run after the sweep, before the first store to Q.
template <int N, class Pre>
__device__ __forceinline__ void schur_gj_valu(double (&S)[64], SchurLds<N>& F, int t, Pre&& pre) {
  constexpr int NI = SchurCfg<N>::NI, QS = SchurCfg<N>::QS;
  const int i = t < NI ? t : NI - 1;
  const bool iv = t < NI;
  // In-place Gauss-Jordan inverse of S (SPD: no pivoting).  With pivots 0..p-1 done, the current
  // matrix X has X[p][j] = X[j][p] for j >= p and X[p][j] = -X[j][p] for j < p, so row p is lane
  // j's own column p with a sign: each pivot makes four 16-lane row copies of it with the
  // row-swap permutes and every lane applies X[t][j] += X[p][j] g_t with row_newbcast FMAs.
  // Software-pipelined: the chunk holding the next pivot's column is updated first, then the next
  // pivot's row broadcast and reciprocal (a long dependent chain) are issued among the other chunks'
  // independent FMAs.  Pad columns (>= NI) are skipped: their row entries are all zero.
  struct Piv {
    double x[4], g, newc;
  };
  auto prelude = [&](auto P) __attribute__((always_inline)) {
    constexpr int pv = decltype(P)::value;
    Piv o;
    const double col = S[pv] + (t == pv ? 1.0 : 0.0);
    const double rj = t < pv ? -col : col;
    // row p of the current matrix in every DPP row, absolute column order (copy s' = columns
    // 16 s' .. 16 s' + 15); the pivot X[p][p] is lane p & 15 of copy p >> 4
    rowbcast4(rj, o.x[0], o.x[1], o.x[2], o.x[3]);
    asm("" : "+&v"(o.x[0]), "+&v"(o.x[1]), "+&v"(o.x[2]), "+&v"(o.x[3]));  // all four made here
    const double a0 = __builtin_amdgcn_update_dpp(0.0, o.x[pv >> 4], 0x150 + (pv & 15), 0xF, 0xF, false);
    const double pinv = recip(a0);
    const double cp = col * pinv;
    o.g = t == pv ? pinv - 1.0 : -cp;
    o.newc = t == pv ? pinv : -cp;
    return o;
  };
  Piv cur = prelude(IC<0>{});
  sfor<0, NI>([&](auto P) __attribute__((always_inline)) {
    constexpr int pv = decltype(P)::value;
    constexpr int cs = (pv + 1 < NI ? pv + 1 : pv) >> 4;
    upd_chunk<cs, NI>(cur.x[cs], cur.g, S);
    Piv nxt;
    if constexpr (pv + 1 < NI) nxt = prelude(IC<pv + 1>{});
    // (the other chunks' row copies were made with the first one's, before its update: no wait)
    if constexpr (cs != 0) upd_chunk<0, NI, false>(cur.x[0], cur.g, S);
    if constexpr (cs != 1) upd_chunk<1, NI, false>(cur.x[1], cur.g, S);
    if constexpr (cs != 2) upd_chunk<2, NI, false>(cur.x[2], cur.g, S);
    if constexpr (cs != 3) upd_chunk<3, NI, false>(cur.x[3], cur.g, S);
    S[pv] = cur.newc;
    if constexpr (pv + 1 < NI) cur = nxt;
  });
  pre();
  wave_sync();
  // Q = I - S^-1 (columns NI .. QS-1: 0; the last row's tail: 0): -S^-1, then each row's diagonal
  if (iv) {
#pragma unroll
    for (int m = 0; m < QS; m += 2) {
      const double q0 = m < NI ? -S[m] : 0.0;
      const double q1 = m + 1 < NI ? -S[m + 1] : 0.0;
      *reinterpret_cast<double2*>(&F.Q[QS * i + m]) = make_double2(q0, q1);
    }
    F.Q[QS * i + i] += 1.0;
  }
  if (t == 0) *reinterpret_cast<double2*>(&F.Q[QS * NI]) = make_double2(0.0, 0.0);
  wave_sync();
}

// ---- factorization (once per rho) ----------------------------------------------------------------
// Inputs: sc.Rt (R'_k foot blocks, written by the caller's variable lanes), sm.Bw.  Outputs: Q and
// B in LDS and, per lane, RI[r][3] (row a of R'^-1 of its foot, variable role).
// (G_k is positive definite for the robots that reach it: scale_kernel screens out rank-deficient
// B6_k, whose robots the Riccati form solves)
// smax: max_i S_ii (>= 1; a lower bound on the condition of S, whose eigenvalues are >= 1), from the
// lanes' own V, W rows: S_ii = 1 + beta_kk |v_i|^2 + alpha_kk |w_i|^2 (the hand-off at the checks
// weighs it with the KKT solve's observed cancellation, schur_solve's amp).
template <int N, int R, class SM, class Mark>
__device__ __forceinline__ void schur_factor(SM& sm, SchurLds<N>& F, const mpcqp_params& p, const Adisc& A, double cost_c,
                             double dtm, double (&RI)[R][3], Mark&& mark, double& smax) {
  constexpr int QS = SchurCfg<N>::QS;
  constexpr int NI = SchurCfg<N>::NI;
  auto& sc = F.s;
  // the lane id through an opaque copy: the per-lane masks derived from it (t == pivot, ...) are
  // then computed here, not hoisted out of the ADMM loop into spilled registers
  int t = threadIdx.x;
  asm volatile("" : "+&v"(t));
  const int q = t >> 4, li = t & 15, leg = li >> 2, a = li & 3;
  const bool av = a < 3;
  const int ig = gray(q);
  // impulse role: lane i = 6 k + c
  const int i = t < NI ? t : NI - 1;
  const bool iv = t < NI;
  const int k = i / 6, c = i % 6;
  mark(25);  // entry (the R' blocks are in LDS)
#ifdef MPCQP_REPEAT_PROLOGUE  // cost measurement builds: the (idempotent) prologue runs twice
  double vw[12];
  for (int rep = 0; rep < 2; ++rep) {
#endif
  // R'^-1 per foot (cofactor inverse of the symmetric 3x3): the variable lane's row a
#pragma unroll
  for (int r = 0; r < R; ++r) {
    const int k = 4 * r + ig;
    const int kc = k < N ? k : N - 1;
    const double* m = sc.Rt[kc][leg];
    const double m00 = m[0], m01 = m[1], m02 = m[2], m11 = m[3], m12 = m[4], m22 = m[5];
    const double c00 = m11 * m22 - m12 * m12, c01 = m02 * m12 - m01 * m22, c02 = m01 * m12 - m02 * m11;
    const double c11 = m00 * m22 - m02 * m02, c12 = m01 * m02 - m00 * m12, c22 = m00 * m11 - m01 * m01;
    const double inv = recip((m00 * c00 + m01 * c01) + m02 * c02);
    const double i0 = sel3(a, c00, c01, c02) * inv, i1 = sel3(a, c01, c11, c12) * inv,
                 i2 = sel3(a, c02, c12, c22) * inv;
    if (k < N && av) {
      sc.Ri[k][leg][3 * a + 0] = i0;
      sc.Ri[k][leg][3 * a + 1] = i1;
      sc.Ri[k][leg][3 * a + 2] = i2;
    }
  }
  wave_sync();
  mark(21);  // R'^-1 per foot done
  // row c of B6 R'^-1: rows 0-2 of B6 are B_w (3 x 12), rows 3-5 dt/m on the matching component
  double br[12];
#pragma unroll
  for (int l = 0; l < 4; ++l)
#pragma unroll
    for (int b = 0; b < 3; ++b) {
      const double* ri = sc.Ri[k][l];
      double s;
      if (c < 3) {
        const double* bw = sm.Bw[k][c < 3 ? c : 0] + 3 * l;
        s = (bw[0] * ri[b] + bw[1] * ri[3 + b]) + bw[2] * ri[6 + b];
      } else {
        s = dtm * ri[3 * (c - 3) + b];
      }
      br[3 * l + b] = s;
    }
  if (iv)
#pragma unroll
    for (int j = 0; j < 12; ++j) sc.B6R[i][j] = br[j];
  // row c of G_k = (B6 R'^-1)_k B6_k'; the Cholesky below reads only its lower triangle, each entry
  // written by exactly one lane
#pragma unroll
  for (int d = 0; d < 6; ++d) {
    double s;
    if (d < 3) {
      const double* bw = sm.Bw[k][d];
      s = 0.0;
#pragma unroll
      for (int j = 0; j < 12; ++j) s += br[j] * bw[j];
    } else {
      s = dtm * (((br[d - 3] + br[d]) + br[d + 3]) + br[d + 6]);
    }
    if (iv && d <= c) sc.G[k][6 * c + d] = s;
  }
  wave_sync();
  mark(22);  // B6 R'^-1 rows and G rows done
  // Cholesky G_k = L L' and Li = L^-1 (every lane of the step, redundantly)
  double L[6][6], Li[6][6], Ldi[6];
#pragma unroll
  for (int r2 = 0; r2 < 6; ++r2)
#pragma unroll
    for (int c2 = 0; c2 < 6; ++c2) L[r2][c2] = 0.0;
#pragma unroll
  for (int cc = 0; cc < 6; ++cc) {
    double s = sc.G[k][6 * cc + cc];
#pragma unroll
    for (int e = 0; e < cc; ++e) s -= L[cc][e] * L[cc][e];
    const double dg = sqrt(s), dinv = recip(dg);
    L[cc][cc] = dg;
    Ldi[cc] = dinv;
#pragma unroll
    for (int r2 = cc + 1; r2 < 6; ++r2) {
      double v = sc.G[k][6 * r2 + cc];
#pragma unroll
      for (int e = 0; e < cc; ++e) v -= L[r2][e] * L[cc][e];
      L[r2][cc] = v * dinv;
    }
  }
#pragma unroll
  for (int cc = 0; cc < 6; ++cc) {  // forward substitution, column cc of L^-1
#pragma unroll
    for (int r2 = 0; r2 < 6; ++r2) {
      if (r2 < cc) {
        Li[r2][cc] = 0.0;
        continue;
      }
      double v = r2 == cc ? 1.0 : 0.0;
#pragma unroll
      for (int e = cc; e < r2; ++e) v -= L[r2][e] * Li[e][cc];
      Li[r2][cc] = v * Ldi[r2];
    }
  }
  mark(23);  // Cholesky of G_k and L^-1 done
  // the lane's column c of L and row c of Li (c is per lane: selects, not register indexing)
  double Lc[6], lic[6];
#pragma unroll
  for (int e = 0; e < 6; ++e) {
    double v = L[e][0], w = Li[0][e];
#pragma unroll
    for (int cc = 1; cc < 6; ++cc) {
      v = c == cc ? L[e][cc] : v;
      w = c == cc ? Li[cc][e] : w;
    }
    Lc[e] = v;
    lic[e] = w;
  }
  // row c of B = Li (B6 R'^-1)
  double bl[12];
#pragma unroll
  for (int j = 0; j < 12; ++j) {
    double s = 0.0;
#pragma unroll
    for (int e = 0; e < 6; ++e) s += lic[e] * sc.B6R[6 * k + e][j];
    bl[j] = s;
  }
  // columns of sqrt(c) Qv^1/2 L_k and sqrt(c) Qp^1/2 Ac6 L_k (Ac6 = A[0:6, 6:12])
#ifndef MPCQP_REPEAT_PROLOGUE
  double vw[12];
#endif
#pragma unroll
  for (int e = 0; e < 6; ++e) vw[e] = sqrt(cost_c * (2.0 * p.q_weights[6 + e])) * Lc[e];
#pragma unroll
  for (int e = 0; e < 6; ++e) {
    double s = 0.0;
#pragma unroll
    for (int f = 0; f < 6; ++f) s += A.at(e, 6 + f) * Lc[f];
    vw[6 + e] = sqrt(cost_c * (2.0 * p.q_weights[e])) * s;
  }
  mark(24);  // B rows and the S factors V, W done
  // sc.B6R is read above by every lane before any lane writes B (in-order LDS of one wave)
  if (iv)
#pragma unroll
    for (int j = 0; j < 12; ++j) F.Bm[i][j] = bl[j];
  // pad lanes: zero columns (their rows of S stay 0; nothing reads their broadcasts)
#pragma unroll
  for (int e = 0; e < 12; ++e) vw[e] = iv ? vw[e] : 0.0;
#ifdef MPCQP_REPEAT_PROLOGUE
  wave_sync();
  }
#endif
  {
    double sv = 0.0, sw = 0.0;
#pragma unroll
    for (int e = 0; e < 6; ++e) {
      sv += vw[e] * vw[e];
      sw += vw[6 + e] * vw[6 + e];
    }
    const double sii = (1.0 + (double)(N - k) * sv) + alpha_jl(N, k, k) * sw;
    smax = wave_max(iv ? sii : 0.0);
  }
  mark(13);
  // S - I = L'CL = beta o (V V') + alpha o (W W') (V, W: the 6-column halves of vw; beta, alpha per
  // step pair), row i in absolute column order, by row_newbcast dot products against four row
  // copies of each column: no LDS.  Entry (i, m) is the same fma chains by lanes i and m and the
  // same symmetric coefficients, so S is exactly symmetric.
  double S[64];
#pragma unroll
  for (int m = 0; m < 64; ++m) S[m] = 0.0;
  sfor<0, 2>([&](auto PART) __attribute__((always_inline)) {
    constexpr int part = decltype(PART)::value;
    double xc[4][6], v6[6];
#pragma unroll
    for (int e = 0; e < 6; ++e) {
      v6[e] = vw[6 * part + e];
      rowbcast4(v6[e], xc[0][e], xc[1][e], xc[2][e], xc[3][e]);
    }
    sfor<0, (NI + 3) / 4>([&](auto B) __attribute__((always_inline)) {
      constexpr int m0 = 4 * decltype(B)::value, sr = m0 >> 4, l0 = m0 & 15;
      double acc[4] = {0.0, 0.0, 0.0, 0.0};
      dot6x4<(m0 & 15) == 0, l0, l0 + 1, l0 + 2, l0 + 3>(xc[sr], v6, acc[0], acc[1], acc[2], acc[3]);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int m = m0 + j;
        if (m < NI) {
          const int l = m / 6;
          if constexpr (part == 0) S[m] = (double)(N - (k > l ? k : l)) * acc[j];
          else S[m] = fma(alpha_jl(N, k, l), acc[j], S[m]);
        }
      }
    });
  });
  // S holds L'CL so far: the sweep adds the identity (schur_gj_valu: to each diagonal entry when its
  // pivot comes, entry (j, j) being read first by pivot j; the MFMA forms: to the tiles) and pad rows
  // stay 0.
  mark(14);
#if MPCQP_GJ_MFMA
  // internal marks: cycle counts kept in registers, recorded after the sweep (no branch inside it)
  long long gts[12];
  int gid[12], ng = 0;
  auto stamp = [&](int id) __attribute__((always_inline)) {
#ifdef MPCQP_PHASE_TIMING
    gid[ng] = id;
    gts[ng] = (long long)__builtin_readcyclecounter();
    ++ng;
#endif
    (void)id;
  };
  schur_gj_mfma<N>(
      S, F, t,
      [&]() __attribute__((always_inline)) {
        // the lane's rows of R'^-1, read back from the scratch (before Q overwrites it)
#pragma unroll
        for (int r = 0; r < R; ++r) {
          const int kk = 4 * r + ig;
          const int kc = kk < N ? kk : N - 1;
          const double* ri = sc.Ri[kc][leg] + 3 * (av ? a : 2);
          RI[r][0] = ri[0];
          RI[r][1] = ri[1];
          RI[r][2] = ri[2];
        }
      },
      stamp);
  wave_sync();
  mark(15);  // (after the stores to Q: f_gj covers them)
  for (int e = 0; e < ng; ++e) mark(gid[e], gts[e]);
#else
  schur_gj_valu<N>(S, F, t, [&]() __attribute__((always_inline)) {
    mark(15);
    // the lane's rows of R'^-1, read back from the scratch (before Q overwrites it)
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const int kk = 4 * r + ig;
      const int kc = kk < N ? kk : N - 1;
      const double* ri = sc.Ri[kc][leg] + 3 * (av ? a : 2);
      RI[r][0] = ri[0];
      RI[r][1] = ri[1];
      RI[r][2] = ri[2];
    }
  });
#endif
}

// ---- KKT solve (every ADMM iteration) ------------------------------------------------------------
// W[r]: w = D^-1 rhs in the variable layout; returns U[r] = (c B6'M B6 + R')^-1 w.
// AMP (update_info iterations): amp = max|R'^-1 w| / max|u| over the robot's variables, the
// cancellation of the push-through identity u = R'^-1 w - B'(I - S^-1)B w in this solve: the rounding
// errors of both terms (and of S^-1) reach u amplified by it.
template <int N, int R, bool AMP = false>
__device__ __forceinline__ void schur_solve(SchurLds<N>& F, const double (&W)[R], const double (&RI)[R][3],
                                            const bool (&vvr)[R], double (&U)[R], double& amp) {
  constexpr int NI = SchurCfg<N>::NI, QS = SchurCfg<N>::QS, BS = SchurCfg<N>::BS;
  const int t = threadIdx.x, q = t >> 4, li = t & 15, leg = li >> 2, a = li & 3;
  const bool av = a < 3;
  const int ig = gray(q);
  const int idx = 3 * leg + (av ? a : 2);
  const int i = t < NI ? t : NI - 1;
  const int k = i / 6;
  // Q is constant between factorizations: its first two 16-column chunks are loaded before
  // anything else (sched_barrier keeps the scheduler from sinking them to their use)
  const double2* qr2 = reinterpret_cast<const double2*>(F.Q + QS * i);
  double c0[16], c1[16];
  auto load = [&](double (&c)[16], int s) __attribute__((always_inline)) {
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const double2 v = qr2[8 * s + e];
      c[2 * e] = v.x;
      c[2 * e + 1] = v.y;
    }
  };
  load(c0, 0);
  load(c1, 1);
  __builtin_amdgcn_sched_barrier(0);
#pragma unroll
  for (int r = 0; r < R; ++r)
    if (vvr[r]) F.wv[12 * (4 * r + ig) + idx] = W[r];
  wave_sync();
  // impulse role: z = B w of the lane's step (its row of B from LDS)
  double z;
  {
    // (the twelve loads as arrays first: measured 1.8 % faster than loading inside the fma loop;
    // pinning them with a sched_barrier, or storing the padding lanes' w branch-free into qv, was
    // slower)
    const double2* w2 = reinterpret_cast<const double2*>(&F.wv[12 * k]);
    const double2* b2 = reinterpret_cast<const double2*>(F.Bm[i]);
    double2 v[6], bb[6];
#pragma unroll
    for (int j = 0; j < 6; ++j) {
      v[j] = w2[j];
      bb[j] = b2[j];
    }
    double za = 0.0, zb = 0.0;
#pragma unroll
    for (int j = 0; j < 6; ++j) {
      za = fma(bb[j].x, v[j].x, za);
      zb = fma(bb[j].y, v[j].y, zb);
    }
    z = t < NI ? za + zb : 0.0;
  }
  // variable role: R'^-1 w of the lane's foot (independent of the dense product below)
  double r1[R];
#pragma unroll
  for (int r = 0; r < R; ++r) {
    const int kk = 4 * r + ig;
    const int kc = kk < N ? kk : N - 1;
    const double* wf = &F.wv[12 * kc + 3 * leg];
    r1[r] = (RI[r][0] * wf[0] + RI[r][1] * wf[1]) + RI[r][2] * wf[2];
  }
  // q = Q z: z in every DPP row (absolute order), 64 row_newbcast FMAs
  double z0, z1, z2, z3;
  rowbcast4(z, z0, z1, z2, z3);
  // all four row copies exist before the first block (which waits for them): the later blocks then
  // need no wait (the compiler would otherwise sink a copy's permlane to just before its block)
  asm("" : "+&v"(z0), "+&v"(z1), "+&v"(z2), "+&v"(z3));
  double a0 = 0.0, a1 = 0.0, a2 = 0.0, a3 = 0.0;
  mv16<true>(z0, c0, a0, a1, a2, a3);
  load(c0, 2);
  mv16<false>(z1, c1, a0, a1, a2, a3);
  load(c1, 3);
  mv16<false>(z2, c0, a0, a1, a2, a3);
  mv16<false>(z3, c1, a0, a1, a2, a3);
  const double qi = (a0 + a1) + (a2 + a3);
  if (t < NI) F.qv[t] = qi;
  wave_sync();
  // variable role: u = R'^-1 w - B' q (column idx of B_k from LDS)
#pragma unroll
  for (int r = 0; r < R; ++r) {
    const int kk = 4 * r + ig;
    const int kc = kk < N ? kk : N - 1;
    const double2* q2 = reinterpret_cast<const double2*>(&F.qv[6 * kc]);
    const double2 qa = q2[0], qb = q2[1], qc = q2[2];
    const double* bc = &F.Bm[6 * kc][idx];
    const double y = ((((bc[0] * qa.x + bc[BS] * qa.y) + bc[2 * BS] * qb.x) + bc[3 * BS] * qb.y) + bc[4 * BS] * qc.x) +
                     bc[5 * BS] * qc.y;
    U[r] = r1[r] - y;
  }
  if constexpr (AMP) {
    double mr = 0.0, mu = 0.0;
#pragma unroll
    for (int r = 0; r < R; ++r) {
      mr = vvr[r] ? fmax(mr, dabs(r1[r])) : mr;
      mu = vvr[r] ? fmax(mu, dabs(U[r])) : mu;
    }
    mr = wave_max(mr);
    mu = wave_max(mu);
    amp = mu > 0.0 ? mr / mu : (mr > 0.0 ? INFINITY : 1.0);
  }
}

// ---- P~v (termination checks, dual-infeasibility test, objective) --------------------------------
// out = c D H (D v) with H = B6' M B6 + R (2 R on the diagonal), computed directly like OSQP's
// update_info mat_vec (osqp auxil.c; oracle/mpc_oracle.c:760) instead of being carried through the
// iterations: z = B6 (D v) on the impulse lanes, M z, then B6' (M z) + R D v on the variable lanes.
// DVv[r] = D v and Dd[r] = D in the variable layout.  Uses wv / qv (not Q or B).
// M z without an LDS round trip: z's four row copies (rowbcast4) feed row_newbcast FMAs, so lane
// (k, c) accumulates, step l ascending, s2[f] += alpha_kl z_(l,f) and s1[f] += beta_kl z_(l,f) for
// all six components f and keeps s1[c]: the same fma chains as summing z_(l,c) read from LDS.
// alpha_kl and beta_kl are exact integers formed in binary64 (no integer division).
#define PX_F(A, C, L) "v_fmac_f64_dpp %[" A "], %[x], %[" C "] row_newbcast:%[" L "] row_mask:0xf bank_mask:0xf\n\t"
// s2[f] += bcast_(L0+f)(x) * al, s1[f] += bcast_(L0+f)(x) * be, f < 6 (lanes L0 .. L0+5 of x's row)
#define PX_STEP_BODY                                                                             \
  PX_F("b0", "al", "l0") PX_F("b1", "al", "l1") PX_F("b2", "al", "l2") PX_F("b3", "al", "l3")          \
  PX_F("b4", "al", "l4") PX_F("b5", "al", "l5")                                                      \
  PX_F("a0", "be", "l0") PX_F("a1", "be", "l1") PX_F("a2", "be", "l2") PX_F("a3", "be", "l3")          \
  PX_F("a4", "be", "l4") PX_F("a5", "be", "l5")
#define PX_STEP_OPS                                                                               \
  : [a0] "+&v"(s1[0]), [a1] "+&v"(s1[1]), [a2] "+&v"(s1[2]), [a3] "+&v"(s1[3]), [a4] "+&v"(s1[4]), [a5] "+&v"(s1[5]), \
    [b0] "+&v"(s2[0]), [b1] "+&v"(s2[1]), [b2] "+&v"(s2[2]), [b3] "+&v"(s2[3]), [b4] "+&v"(s2[4]), [b5] "+&v"(s2[5]) \
  : [x] "v"(x), [al] "v"(al), [be] "v"(be), [l0] "n"(L0), [l1] "n"(L0 + 1), [l2] "n"(L0 + 2),       \
    [l3] "n"(L0 + 3), [l4] "n"(L0 + 4), [l5] "n"(L0 + 5)
// HEAD: the first block after x's row copies were made (al and be are not DPP sources)
template <bool HEAD, int L0>
__device__ __forceinline__ void px_step(double x, double al, double be, double (&s1)[6], double (&s2)[6]) {
  static_assert(L0 + 5 <= 15, "a step's six unknowns inside one DPP row");
  if constexpr (HEAD)
    asm(WV_NOP_HEAD PX_STEP_BODY PX_STEP_OPS);
  else
    asm(WV_NOP_INNER PX_STEP_BODY PX_STEP_OPS);
}
#undef PX_STEP_BODY
#undef PX_STEP_OPS
#undef PX_F
// one component of a step whose unknowns straddle two DPP rows
#define PX_ONE_BODY                                                                                \
  "v_fmac_f64_dpp %[b], %[x], %[al] row_newbcast:%[l] row_mask:0xf bank_mask:0xf\n\t"                \
  "v_fmac_f64_dpp %[a], %[x], %[be] row_newbcast:%[l] row_mask:0xf bank_mask:0xf\n\t"
#define PX_ONE_OPS : [a] "+&v"(s1), [b] "+&v"(s2) : [x] "v"(x), [al] "v"(al), [be] "v"(be), [l] "n"(L)
template <bool HEAD, int L>
__device__ __forceinline__ void px_one(double x, double al, double be, double& s1, double& s2) {
  if constexpr (HEAD)
    asm(WV_NOP_HEAD PX_ONE_BODY PX_ONE_OPS);
  else
    asm(WV_NOP_INNER PX_ONE_BODY PX_ONE_OPS);
}
#undef PX_ONE_BODY
#undef PX_ONE_OPS
// q2c = 2 q_(6+c) of the lane's impulse component c, r2i = 2 r_idx of its variable component (per-lane
// constants the kernel loads once: a per-lane index into the parameters is a memory round trip)
template <int N, int R, class SM>
__device__ __forceinline__ void schur_px(const SM& sm, SchurLds<N>& F, const mpcqp_params& p, const Adisc& A,
                                         double dtm, double cost_c, double q2c, double r2i, const double (&DVv)[R],
                                         const double (&Dd)[R], const bool (&vvr)[R], double (&out)[R]) {
  constexpr int NI = SchurCfg<N>::NI;
  const int t = threadIdx.x, q = t >> 4, li = t & 15, leg = li >> 2, a = li & 3;
  const bool av = a < 3;
  const int ig = gray(q);
  const int idx = 3 * leg + (av ? a : 2);
#pragma unroll
  for (int r = 0; r < R; ++r)
    if (vvr[r]) F.wv[12 * (4 * r + ig) + idx] = DVv[r];
  wave_sync();
  // impulse role, lane i = 6 k + c: z = B6_k (D v)_k (rows 0-2: B_w, rows 3-5: dt/m leg sums)
  const int i = t < NI ? t : NI - 1, k = i / 6, c = i % 6;
  double z;
  {
    const double* w = &F.wv[12 * k];
    const double* bw = sm.Bw[k][c < 3 ? c : 0];
    double zw = 0.0;
#pragma unroll
    for (int j = 0; j < 12; ++j) zw += bw[j] * w[j];
    const int cc = c < 3 ? 0 : c - 3;
    const double zv = dtm * (((w[cc] + w[3 + cc]) + w[6 + cc]) + w[9 + cc]);
    z = t < NI ? (c < 3 ? zw : zv) : 0.0;
  }
  // (M z)_(k,c) = Qv_c sum_l beta_kl z_(l,c) + (Ac6' Qp Ac6 sum_l alpha_kl z_l)_c
  double mz;
  {
    double zc[4];
    rowbcast4(z, zc[0], zc[1], zc[2], zc[3]);
    // all four row copies exist before the first block (which waits for them): otherwise the compiler
    // may sink a copy's permlane to just before the first block that reads it, which has no wait
    // (tools/isa_hazards.py --all found that at N = 7 and 8: a px_one block reading zc[1] / zc[2])
    asm("" : "+&v"(zc[0]), "+&v"(zc[1]), "+&v"(zc[2]), "+&v"(zc[3]));
    double s1[6] = {0.0, 0.0, 0.0, 0.0, 0.0, 0.0}, s2[6] = {0.0, 0.0, 0.0, 0.0, 0.0, 0.0};
    // alpha_kl = sum_{i >= max(k,l)} (i-k)(i-l): l >= k: (l-k) T1(N-1-l) + T2(N-1-l); l < k:
    // (k-l) T1(N-1-k) + T2(N-1-k), T1(m) = m(m+1)/2, T2(m) = m(m+1)(2m+1)/6 (all exact integers)
    const double mk = (double)(N - 1 - k);
    const double t1k = mk * (mk + 1.0) * 0.5;
    const double t2k = (mk * (mk + 1.0) * (2.0 * mk + 1.0)) / 6.0;
    sfor<0, N>([&](auto LL) __attribute__((always_inline)) {
      constexpr int l = decltype(LL)::value, L0 = 6 * l;
      constexpr int ml = N - 1 - l;
      constexpr double t1l = ml * (ml + 1) / 2, t2l = ml * (ml + 1) * (2 * ml + 1) / 6;
      const double al = k <= l ? fma((double)(l - k), t1l, t2l) : fma((double)(k - l), t1k, t2k);
      const double be = (double)(N - (k > l ? k : l));
      if constexpr ((L0 >> 4) == ((L0 + 5) >> 4)) {
        px_step<l == 0, L0 & 15>(zc[L0 >> 4], al, be, s1, s2);
      } else {
        sfor<0, 6>([&](auto FF) __attribute__((always_inline)) {
          constexpr int f = decltype(FF)::value, Lf = L0 + f;
          px_one<l == 0 && f == 0, Lf & 15>(zc[Lf >> 4], al, be, s1[f], s2[f]);
        });
      }
    });
    // w_e = 2 q_e (Ac6 s2)_e; Ac6 = A[0:6, 6:12]
    const double w0 = (2.0 * p.q_weights[0]) * (A.ad0 * s2[0] + A.ad1 * s2[1]);
    const double w1 = (2.0 * p.q_weights[1]) * ((-A.ad1) * s2[0] + A.ad0 * s2[1]);
    double wc = 0.0, s1c = s1[0];
#pragma unroll
    for (int e = 2; e < 6; ++e) wc = c == e ? (2.0 * p.q_weights[e]) * (A.dt * s2[e]) : wc;
#pragma unroll
    for (int e = 1; e < 6; ++e) s1c = c == e ? s1[e] : s1c;
    // (Ac6' w)_c: c = 0, 1 mix the yaw rotation; c = 2: dt w_2; c >= 3: dt w_c
    const double ac = c == 0 ? A.ad0 * w0 + (-A.ad1) * w1 : (c == 1 ? A.ad1 * w0 + A.ad0 * w1 : A.dt * wc);
    mz = q2c * s1c + ac;
  }
  if (t < NI) F.qv[t] = mz;
  wave_sync();
  // variable role: (B6' M z)_j + 2 r_j (D v)_j, times c D
#pragma unroll
  for (int r = 0; r < R; ++r) {
    const int kk = 4 * r + ig;
    const int kc = kk < N ? kk : N - 1;
    const double* mk = &F.qv[6 * kc];
    const double hv = ((((sm.Bw[kc][0][idx] * mk[0] + sm.Bw[kc][1][idx] * mk[1]) + sm.Bw[kc][2][idx] * mk[2]) +
                        dtm * mk[3 + (av ? a : 2)]) +
                       r2i * DVv[r]);
    out[r] = vvr[r] ? (cost_c * Dd[r]) * hv : 0.0;
  }
  wave_sync();
}

}  // namespace wv
}  // namespace mpcqp
