// mpcqp_dx.hip — the OSQP 0.6 solve of ConvexMpc's QP with an EXPLICIT inverse of the reduced
// KKT matrix held in registers across one workgroup per robot (horizons 1-10, path 5).
//
// Reference path: A1RobotControl::compute_grf (src/a1_cpp/src/A1RobotControl.cpp:446-562) ->
// ConvexMpc (src/a1_cpp/src/ConvexMpc.cpp:7-245) -> OsqpEigen 0.6.3 / OSQP 0.6 (restated in
// oracle/mpc_oracle.c: set_rho_vec, update_xz_tilde, update_x/z/y, update_info,
// check_termination, adapt_rho, store_solution).  scale_kernel (mpcqp_wave.hip) runs OSQP's
// scale_data first and hands over the same image as for wave_kernel.
//
// Why an explicit inverse.  OSQP's linear system changes only when rho changes (about three
// times per solve) while the ADMM loop solves it ~135 times.  The reduced KKT matrix
//   K = P~ + sigma I + A~' diag(rho) A~      (n x n, n = 12 N, SPD)
// is inverted once per rho (in-register Gauss-Jordan), after which every iteration is ONE dense
// mat-vec x~ = K^-1 rhs: n^2 independent FMAs spread over the workgroup, no dependency chain.
// (The Riccati path, wave_kernel, needs two sequential 12x12 mat-vec chains per iteration.)
//
// Lane layout (RW = 30 matrix rows per wave, NWV = ceil(n / 30) waves).  Lane l of wave w:
//   half h = l >> 5, DPP row within the half q2 = (l >> 4) & 1, lane in the row lr = l & 15;
//   lr < 15 holds variable / matrix row i = 30 w + 15 q2 + lr (lr = 15 is padding);
//   register R[c] = K^-1[i][HS h + c], HS = n / 2 (both halves of the wave hold the same rows).
// A foot (its fx, fy, fz variables i = 3f + a) is three consecutive lanes of one DPP row, and
// its five constraint rows sit on its six lanes: rows 2a + h (a < 2) and row 4 on (a = 2, h = 0).
// Per-foot operations (A~x, A~'y) are row_shl / row_shr DPP moves plus one permlane32 swap.
//
// Mat-vec y = K^-1 v: v goes to LDS (one double per variable), every lane loads the KD values of
// its half it broadcasts (column 16 k + lr), and y_i is KD blocks of 16 `v_fmac_f64_dpp
// row_newbcast` (column c's value broadcast from lane c % 16 of the lane's own DPP row) over the
// HS registers, plus one permlane32 swap to add the two halves.
//
// Gauss-Jordan (in place, no pivoting: stable for SPD; n steps).  Step p needs the pivot row in
// every lane.  K stays symmetric up to the sign of the already-pivoted columns
// (a_pj = -a_jp when exactly one of p, j has been pivoted), so lane j contributes s_j a_jp from
// its own register and the row is assembled in LDS with one ds_write per lane; the update is
// then 16-lane DPP broadcasts again.  The next step's pivot column is updated first and
// published before the rest of the step (one barrier per step, double-buffered).
// Arithmetic is binary64 throughout.
//
// Status: experimental (debug path 5), parity-green against the oracle, SLOWER than the default
// Riccati wave path at the bench batch: the Gauss-Jordan inverse costs n^3 FMAs
// (2x the Riccati factorization's work) behind a barrier per pivot, and the iteration, although
// free of the Riccati chains, is latency-bound behind its per-iteration barrier and the
// permlane / DPP hand-offs at one or two waves per SIMD (K's row takes 120 of the 256 VGPRs).
// Debug build: -DDXE_DUMP writes K, K^-1, D, E, c, rho of the first factorization into
// `solution` (tools/dx_dump.py); -DMPCQP_DX_WPE=2 sizes the registers for two waves per SIMD.
#include "mpcqp_wave_common.h"

namespace mpcqp {
namespace dx {

using wv::Adisc;
using wv::ScaleImg;
using wv::WarmLayout;
using wv::gen_col;
using wv::iw_inverse;
using wv::recip;
using wv::sfor;

template <int N>
struct DCfg {
  static constexpr int n = ND * N, m = CD * N, HS = n / 2;
  static constexpr int HSP = (HS + 3) / 4 * 4;  // registers per lane (blocks of 4, 8, 12, 16 FMAs)
  static constexpr int KD = (HSP + 15) / 16;    // broadcast registers per lane
  static constexpr int SEG = 16 * KD;           // LDS segment of one half (zero padded)
  static constexpr int RW = 30;                 // matrix rows per wave (10 feet)
  static constexpr int NWV = (n + RW - 1) / RW;
  static constexpr int NTH = 64 * NWV;
  static constexpr int REC = MPCQP_REC_SIZE(N);
};

template <int N>
struct DSmem {
  using C = DCfg<N>;
  alignas(16) double Bw[N][3][ND];  // rows 6-8 of B_d(k) (gen_col, setup)
  alignas(16) double pb[2][2 * C::SEG];  // pivot rows (factorization), double-buffered
  alignas(16) double wb[2][2 * C::SEG];  // mat-vec operands (iterations), double-buffered
  double rec[C::REC];
  double D[C::n];
  double red[2][C::NWV][16];
  double st[5][C::NTH];  // the iterates, parked through a factorization
  double xs[ND];
};

// ---- DPP broadcast blocks ---------------------------------------------------------------------
// Hazards (the compiler cannot see into the asm): a DPP instruction needs 2 wait states after a
// VALU write of any of its VGPR operands and 5 after an EXEC write: every block starts with
// s_nop 4; inside a block no operand is written before it is read (accumulators rotate over 4).
#define DXG(I) "v_fmac_f64_dpp %[r" #I "], %[x], %[f] row_newbcast:" #I " row_mask:0xf bank_mask:0xf\n\t"
#define DXM(I, A) "v_fmac_f64_dpp %[a" #A "], %[x], %[r" #I "] row_newbcast:" #I " row_mask:0xf bank_mask:0xf\n\t"
#define DXG4(a, b, c, d) DXG(a) DXG(b) DXG(c) DXG(d)
#define DXM4(a, b, c, d) DXM(a, 0) DXM(b, 1) DXM(c, 2) DXM(d, 3)
#define DXRO(I) [r##I] "+&v"(R[C0 + I])  // early-clobber: no input may share its register
#define DXRI(I) [r##I] "v"(R[C0 + I])
#define DXRO4(a, b, c, d) DXRO(a), DXRO(b), DXRO(c), DXRO(d)
#define DXRI4(a, b, c, d) DXRI(a), DXRI(b), DXRI(c), DXRI(d)

// R[16 KB + L] += x(lane L of the DPP row) * f   (Gauss-Jordan update of one broadcast block)
template <int KB, int HSP>
__device__ __forceinline__ void gj_blk(double (&R)[HSP], double x, double f) {
  constexpr int C0 = 16 * KB, CNT = HSP - C0 < 16 ? HSP - C0 : 16;
  if constexpr (CNT == 16) {
    asm("s_nop 4\n\t" DXG4(0, 1, 2, 3) DXG4(4, 5, 6, 7) DXG4(8, 9, 10, 11) DXG4(12, 13, 14, 15)
        : DXRO4(0, 1, 2, 3), DXRO4(4, 5, 6, 7), DXRO4(8, 9, 10, 11), DXRO4(12, 13, 14, 15)
        : [x] "v"(x), [f] "v"(f));
  } else if constexpr (CNT == 12) {
    asm("s_nop 4\n\t" DXG4(0, 1, 2, 3) DXG4(4, 5, 6, 7) DXG4(8, 9, 10, 11)
        : DXRO4(0, 1, 2, 3), DXRO4(4, 5, 6, 7), DXRO4(8, 9, 10, 11)
        : [x] "v"(x), [f] "v"(f));
  } else if constexpr (CNT == 8) {
    asm("s_nop 4\n\t" DXG4(0, 1, 2, 3) DXG4(4, 5, 6, 7) : DXRO4(0, 1, 2, 3), DXRO4(4, 5, 6, 7) : [x] "v"(x), [f] "v"(f));
  } else {
    static_assert(CNT == 4, "block sizes are multiples of 4");
    asm("s_nop 4\n\t" DXG4(0, 1, 2, 3) : DXRO4(0, 1, 2, 3) : [x] "v"(x), [f] "v"(f));
  }
}
// acc[0..3] += sum_L x(lane L) * R[16 KB + L]   (mat-vec over one broadcast block)
template <int KB, int HSP>
__device__ __forceinline__ void mv_blk(const double (&R)[HSP], double x, double (&acc)[4]) {
  constexpr int C0 = 16 * KB, CNT = HSP - C0 < 16 ? HSP - C0 : 16;
  if constexpr (CNT == 16) {
    asm("s_nop 4\n\t" DXM4(0, 1, 2, 3) DXM4(4, 5, 6, 7) DXM4(8, 9, 10, 11) DXM4(12, 13, 14, 15)
        : [a0] "+&v"(acc[0]), [a1] "+&v"(acc[1]), [a2] "+&v"(acc[2]), [a3] "+&v"(acc[3])
        : [x] "v"(x), DXRI4(0, 1, 2, 3), DXRI4(4, 5, 6, 7), DXRI4(8, 9, 10, 11), DXRI4(12, 13, 14, 15));
  } else if constexpr (CNT == 12) {
    asm("s_nop 4\n\t" DXM4(0, 1, 2, 3) DXM4(4, 5, 6, 7) DXM4(8, 9, 10, 11)
        : [a0] "+&v"(acc[0]), [a1] "+&v"(acc[1]), [a2] "+&v"(acc[2]), [a3] "+&v"(acc[3])
        : [x] "v"(x), DXRI4(0, 1, 2, 3), DXRI4(4, 5, 6, 7), DXRI4(8, 9, 10, 11));
  } else if constexpr (CNT == 8) {
    asm("s_nop 4\n\t" DXM4(0, 1, 2, 3) DXM4(4, 5, 6, 7)
        : [a0] "+&v"(acc[0]), [a1] "+&v"(acc[1]), [a2] "+&v"(acc[2]), [a3] "+&v"(acc[3])
        : [x] "v"(x), DXRI4(0, 1, 2, 3), DXRI4(4, 5, 6, 7));
  } else {
    static_assert(CNT == 4, "block sizes are multiples of 4");
    asm("s_nop 4\n\t" DXM4(0, 1, 2, 3)
        : [a0] "+&v"(acc[0]), [a1] "+&v"(acc[1]), [a2] "+&v"(acc[2]), [a3] "+&v"(acc[3])
        : [x] "v"(x), DXRI4(0, 1, 2, 3));
  }
}
#undef DXG
#undef DXM
#undef DXG4
#undef DXM4
#undef DXRO
#undef DXRI
#undef DXRO4
#undef DXRI4

// A cross-lane operation must run with every lane active: never as an operand of ?: (C++
// evaluates only the chosen operand, so the compiler branches round it and the source lanes are
// inactive: v_permlane32_swap then never delivers the partner's value).  pin() also keeps a
// computed cross-lane result from being sunk into a branch that only one select arm needs.
__device__ __forceinline__ double pin(double v) {
  asm volatile("" : "+v"(v));
  return v;
}
// DPP shifts inside a 16-lane row: row_shl:S (lane l reads lane l + S), row_shr:S (l - S)
template <int S>
__device__ __forceinline__ double shl(double v) { return pin(dpp<0x100 + S>(v)); }
template <int S>
__device__ __forceinline__ double shr(double v) { return pin(dpp<0x110 + S>(v)); }

// block-wide max / sum of K values per lane (wave reduction, then the NWV wave partials in wave
// order: every lane ends with the bitwise-same result); rp alternates the two LDS buffers so one
// barrier per reduction suffices.
template <int NWV, int K, bool SUM>
__device__ __forceinline__ void block_red(double (&v)[K], double (*red)[NWV][16], int& rp) {
#pragma unroll
  for (int k = 0; k < K; ++k) v[k] = SUM ? wave_sum(v[k]) : wave_max(v[k]);
  if constexpr (NWV > 1) {
    const int w = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0)
#pragma unroll
      for (int k = 0; k < K; ++k) red[rp][w][k] = v[k];
    __syncthreads();
#pragma unroll
    for (int k = 0; k < K; ++k) {
      double s = red[rp][0][k];
#pragma unroll
      for (int ww = 1; ww < NWV; ++ww) s = SUM ? s + red[rp][ww][k] : dmax(s, red[rp][ww][k]);
      v[k] = s;
    }
    rp ^= 1;
  }
}

template <int N>
#ifndef MPCQP_DX_WPE
// waves per SIMD the register budget is sized for: at 2 (256 VGPRs) the compiler spills ~170
// VGPRs to scratch and the N = 6 build failed parity (N = 1-5, 7-10 passed); at 1 (VGPRs + AGPRs
// up to 512) nothing spills, all horizons pass, and the per-iteration cost is the same
// (11.8 vs 12.0 us per 4096-robot batch, tools/dx_timing.py)
#define MPCQP_DX_WPE 1
#endif
__global__ __launch_bounds__(DCfg<N>::NTH, MPCQP_DX_WPE) void dx_kernel(const double* __restrict__ recs, int batch,
                                                              mpcqp_result* __restrict__ results,
                                                              double* __restrict__ solution, double* __restrict__ trace,
                                                              int trace_cap, double* __restrict__ wstate,
                                                              const double* __restrict__ img, mpcqp_params p) {
  using DC = DCfg<N>;
  using WL = WarmLayout<N>;
  using SI = ScaleImg<N>;
  constexpr int n = DC::n, m = DC::m, HS = DC::HS, HSP = DC::HSP, KD = DC::KD, SEG = DC::SEG, NWV = DC::NWV,
                NTH = DC::NTH;
  __shared__ DSmem<N> sm;
  const int inst = blockIdx.x;
  if (inst >= batch) return;
  const int t = threadIdx.x, w = t >> 6, l = t & 63, h = l >> 5, lr = l & 15;
  const int i = DC::RW * w + 15 * ((l >> 4) & 1) + lr;
  const bool vv = lr < 15 && i < n;        // lane holds a variable / matrix row
  const int ic = vv ? i : 0;
  const int ii = vv ? i : -1;              // for comparisons with a pivot / step index
  const int f = ic / 3, a = ic % 3;        // foot-step f (= 4 k + leg), component a
  const int leg = f & 3;
  const bool hasrow = vv && (a < 2 || h == 0);
  const int ri = 5 * f + (a < 2 ? 2 * a + h : 4);  // this lane's constraint row
  const double alpha = p.alpha, sigma = p.sigma;
  int rp = 0;  // reduction buffer parity

  // ---- 0. record -> LDS, non-finite guard, zeroed broadcast buffers ------------------------------
  {
    const double* rg = recs + (size_t)inst * DC::REC;
    int bad = 0;
    for (int e = t; e < DC::REC; e += NTH) {
      const double v = rg[e];
      sm.rec[e] = v;
      bad |= !isfinite(v);
    }
    for (int e = t; e < 2 * 2 * SEG; e += NTH) {
      (&sm.pb[0][0])[e] = 0.0;
      (&sm.wb[0][0])[e] = 0.0;
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
        for (int e = t; e < n; e += NTH) solution[(size_t)inst * n + e] = NAN;
      return;
    }
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
  // B_d(k) rows 6-8 (calculate_B_mat_c, Utils.cpp:35-41)
  {
    double Iwinv[9];
    iw_inverse(rec, Iwinv);
    for (int e = t; e < N * 36; e += NTH) {
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

  // ---- 1. the scale_kernel image (OSQP scale_data): D, E, q~, A~, c, warm-start branch -----------
  const double* im = img + (size_t)inst * SI::SIZE;
  for (int j = t; j < n; j += NTH) sm.D[j] = im[SI::D + j];
  const double c_s = im[SI::CS];
  const int mode = (int)im[SI::MODE];  // 0 cold, 1 osqp_update_P, 2 OsqpEigen re-init
  double* const ws = wstate ? wstate + (size_t)inst * WL::SIZE : nullptr;
  const double cost_c = c_s, cinv = 1. / c_s;
  const double rho0 = mode == 1 ? ws[WL::RHO] : dmin(dmax(p.rho, RHO_MIN), RHO_MAX);
  // Per-lane constants are re-derived from the image / record where they are needed (volatile
  // loads: the compiler may neither hoist nor merge them) instead of being held in registers
  // through the factorization, which needs all but a few of the 256 VGPRs for K's row.
  auto ldv = [&](const double* ptr) __attribute__((always_inline)) { return *(const volatile double*)ptr; };
  auto var_D = [&]() __attribute__((always_inline)) { return vv ? ldv(im + SI::D + ic) : 1.0; };
  auto row_E = [&]() __attribute__((always_inline)) { return hasrow ? ldv(im + SI::E + ri) : 1.0; };
  // update_P then osqp_update_lin_cost: q~ = c (D q) of this tick's gradient
  auto var_Q = [&]() __attribute__((always_inline)) {
    return vv ? (mode == 1 ? (ldv(im + SI::QN + ic) * var_D()) * c_s : ldv(im + SI::Q + ic)) : 0.0;
  };
  // A~ = E A D: rows 0-3 on the own variable (fx / fy) and fz, row 4 on fz
  auto row_A = [&](double& akp, double& akz) __attribute__((always_inline)) {
    akp = 0.0;
    akz = 0.0;
    if (hasrow) {
      const double Er = ldv(im + SI::E + ri), Dfz = ldv(im + SI::D + 3 * f + 2);
      if (a < 2) {
        akp = (ldv(im + SI::AP + ri) * Er) * ldv(im + SI::D + ic);
        akz = (ldv(im + SI::AP + m + ri) * Er) * Dfz;
      } else {
        akp = (ldv(im + SI::AP + m + ri) * Er) * Dfz;
      }
    }
  };
  // bounds (ConvexMpc.cpp:223-245), clipped to +-OSQP_INFTY, scaled by E: OSQP's scaled l, u
  auto row_LU = [&](double& lc, double& uc) __attribute__((always_inline)) {
    lc = 0.0;
    uc = 0.0;
    if (hasrow) {
      const double Er = ldv(im + SI::E + ri);
      if (a < 2) {
        lc = h ? Er * -OSQP_INF : Er * 0.0;
        uc = h ? Er * 0.0 : Er * OSQP_INF;
      } else {
        const volatile double* rv = rec;
        const double cont = rv[MPCQP_REC_CONTACTS + leg] != 0.0 ? 1.0 : 0.0;
        double l4 = rv[MPCQP_REC_FZMIN] * cont, u4 = rv[MPCQP_REC_FZMAX] * cont;
        l4 = dmin(dmax(l4, -OSQP_INF), OSQP_INF);
        u4 = dmin(dmax(u4, -OSQP_INF), OSQP_INF);
        lc = Er * l4;
        uc = Er * u4;
      }
    }
  };
  auto rho_of = [&](double rho, double lc, double uc) __attribute__((always_inline)) {  // set_rho_vec
    if (!hasrow) return rho;
    const bool loose = lc < -OSQP_INF * MIN_SCALING && uc > OSQP_INF * MIN_SCALING;
    const bool eq = uc - lc < RHO_TOL;
    return loose ? RHO_MIN : (eq ? RHO_EQ_OVER_RHO_INEQ * rho : rho);
  };
  // the loop's per-lane constants: q~, A~ row, projection box (rows 0-3 need no E: [0, +inf) for
  // rows 0, 2 and (-inf, 0] for rows 1, 3), rho vector
  double Qv, AKp, AKz, Lp, Up, RHOr, RIr;
  auto refresh = [&](double rho) __attribute__((always_inline)) {
    Qv = var_Q();
    row_A(AKp, AKz);
    double lc, uc;
    row_LU(lc, uc);
    Lp = (hasrow && a < 2) ? (h ? -INFINITY : 0.0) : lc;
    Up = (hasrow && a < 2) ? (h ? 0.0 : INFINITY) : uc;
    RHOr = rho_of(rho, lc, uc);
    RIr = 1. / RHOr;
  };
  refresh(rho0);

  // the foot's fz value for each lane of the foot
  auto fzv = [&](double v) __attribute__((always_inline)) {
    const double s1 = shl<1>(v), s2 = shl<2>(v);
    return a == 0 ? s2 : (a == 1 ? s1 : v);
  };
  // (A~' v)_i for a per-row value v (rowless lanes contribute 0); both halves get the same value
  auto at_op = [&](double v) __attribute__((always_inline)) {
    const double xo = AKp * v, zo = AKz * v;
    const double so = xo + xor32(xo);   // rows on the own variable, both halves
    const double zs = zo + xor32(zo);   // the fz coefficients of variable a's rows (a < 2)
    const double s1 = shr<1>(zs), s2 = shr<2>(zs);  // from a = 1 (l - 1) and a = 0 (l - 2)
    return a == 2 ? (so + s2) + s1 : so;
  };

  // initial iterates (cold: zero; update_P: the previous scaled iterates; re-init: unscaled with
  // the previous scaling, rescaled with the new one)
  double X = 0.0, Z = 0.0, Y = 0.0, PX = 0.0;
  if (mode == 1) {
    X = vv ? ws[WL::X + ic] : 0.0;
    Z = hasrow ? ws[WL::Z + ri] : 0.0;
    Y = hasrow ? ws[WL::Y + ri] : 0.0;
  } else if (mode == 2) {
    const double cinv_o = 1. / ws[WL::C];
    X = vv ? (1. / var_D()) * (ws[WL::D + ic] * ws[WL::X + ic]) : 0.0;
    Y = hasrow ? c_s * ((1. / row_E()) * ((ws[WL::E + ri] * ws[WL::Y + ri]) * cinv_o)) : 0.0;
  }
  if (mode == 2) Z = AKp * X + AKz * fzv(X);  // z = A~ x
  double RHS = vv ? sigma * 0.0 - Qv : 0.0;  // cold start: compute_rhs with x = z = y = 0
  if (mode != 0) {
    const double at = at_op(RHOr * Z - Y);
    RHS = vv ? (sigma * X - Qv) + at : 0.0;
  }
  __syncthreads();  // Bw, D in LDS

  // ---- K^-1 in registers ----------------------------------------------------------------------
  double R[HSP];
  int pbp = 0, wbp = 0;
  auto colpos = [&](int j) __attribute__((always_inline)) { return j < HS ? j : SEG + (j - HS); };
  // y_i = sum_j R_ij v_j for the v in LDS buffer vb (written by the h == 0 variable lanes)
  auto kmv = [&](const double* vb) __attribute__((always_inline)) {
    double wk[KD];
#pragma unroll
    for (int kk = 0; kk < KD; ++kk) wk[kk] = vb[SEG * h + 16 * kk + lr];
    double acc[4] = {0.0, 0.0, 0.0, 0.0};
    sfor<0, KD>([&](auto KB) __attribute__((always_inline)) {
      mv_blk<decltype(KB)::value>(R, wk[decltype(KB)::value], acc);
    });
    const double y = (acc[0] + acc[1]) + (acc[2] + acc[3]);
    return y + xor32(y);
  };
  // K = P~ + sigma I + A~' diag(rho) A~, row i, in R.  want_px: also P~x (warm start).
  auto form_K = [&](bool want_px) __attribute__((always_inline)) {
    // foot block of sigma I + A~' diag(rho) A~ on row i (columns 3f .. 3f+2), first: after it no
    // per-lane constant is live through H's generation and the inverse
    double m0, m1, m2;
    {
      const double pp = (AKp * RHOr) * AKp, pz = (AKp * RHOr) * AKz, zz = (AKz * RHOr) * AKz;
      const double PP = pp + xor32(pp), PZ = pz + xor32(pz), ZZ = zz + xor32(zz);
      const double pz1 = shr<1>(PZ), pz2 = shr<2>(PZ), zz1 = shr<1>(ZZ), zz2 = shr<2>(ZZ);
      m0 = a == 0 ? PP + sigma : (a == 1 ? 0.0 : pz2);
      m1 = a == 0 ? 0.0 : (a == 1 ? PP + sigma : pz1);
      m2 = a == 2 ? ((PP + zz2) + zz1) + sigma : PZ;
    }
    // H's row does not change between factorizations: without this fence the compiler hoists
    // all of it (and the D loads) out of the ADMM loop and keeps 120 doubles live in scratch
    asm volatile("" ::: "memory");
    const int icx = opaque(ic);
#pragma unroll
    for (int c = 0; c < HSP; ++c) R[c] = 0.0;
    // one horizon block at a time (the column constants are recomputed per block: cheaper than
    // holding them and every block's B_w rows live next to R)
    sfor<0, N>([&](auto JB) __attribute__((always_inline)) {
      constexpr int jb = decltype(JB)::value;
      __builtin_amdgcn_sched_barrier(0);
      gen_col<N, 1, true>(sm, p, A, dtm, icx, jb, [&](int, int b, int, double hv) __attribute__((always_inline)) {
        const int c0 = ND * jb + b;
        if (c0 < HS) {
          if (h == 0) R[c0] = hv;
        } else {
          if (h == 1) R[c0 - HS] = hv;
        }
      });
    });
    __builtin_amdgcn_sched_barrier(0);
    // P~ = c (D H D)  (scale_data: D P D, then the cost scale)
    const double Dv = sm.D[ic];
#pragma unroll
    for (int c = 0; c < HS; ++c) R[c] = cost_c * ((Dv * R[c]) * sm.D[HS * h + c]);
    if (want_px) {  // warm start: P~x of the parked iterate
      if (vv && h == 0) sm.wb[wbp][colpos(i)] = sm.st[0][t];
      __syncthreads();
      sm.st[3][t] = kmv(sm.wb[wbp]);
      wbp ^= 1;
    }
    const int fl = f - 2 * N * h;  // the foot's column triplet inside this half
#pragma unroll
    for (int c = 0; c < HS; ++c) {
      const double mv = (c % 3 == 0) ? m0 : ((c % 3 == 1) ? m1 : m2);
      R[c] += (c / 3 == fl) ? mv : 0.0;
    }
  };
  // In-place Gauss-Jordan inverse of K (row i in R).
  auto gj = [&]() __attribute__((always_inline)) {
    if (vv && h == 0) sm.pb[pbp][colpos(i)] = R[0];  // step 0: column 0 = row 0
#pragma unroll 1
    for (int hp = 0; hp < 2; ++hp) {
      const int irel = ii - HS * hp;  // row index relative to this half's first pivot
      sfor<0, HS>([&](auto CP) __attribute__((always_inline)) {
        constexpr int cp = decltype(CP)::value;
        constexpr int cn = (cp + 1) % HS, kbn = cn / 16;
        const int pv = HS * hp + cp;
#ifdef DXE_DUMP
        if (pv >= p.max_iter) return;  // debug: stop after max_iter steps
#endif
        __builtin_amdgcn_sched_barrier(0);
        __syncthreads();
        const double* pr = sm.pb[pbp];
        double rk[KD];
#pragma unroll
        for (int kk = 0; kk < KD; ++kk) rk[kk] = pr[SEG * h + 16 * kk + lr];
        const double app = pr[SEG * hp + cp];
        pbp ^= 1;
        const double piv = recip(app);
        const double own = R[cp];
        const double sw = pin(xor32(own));  // every lane swaps (a ternary would branch round it)
        const double fi = (h == hp) ? own : sw;  // K[i][p]
        const bool me = irel == cp;
        // row p: K[p][j] / K[p][p] = K[p][j] - (1 - 1/K[p][p]) K[p][j]; other rows: K[i][j] - K[i][p] r_j
        const double nf = me ? piv - 1.0 : -(fi * piv);
        const double newcol = me ? piv : -(fi * piv);
        // the next pivot column first, published for the next step: s_j K[j][p+1]
        gj_blk<kbn>(R, rk[kbn], nf);
        if (pv + 1 < n) {
          const int hn = (cp + 1 == HS) ? hp + 1 : hp;
          if (vv && h == hn) sm.pb[pbp][colpos(i)] = irel <= cp ? -R[cn] : R[cn];
        }
        sfor<0, KD>([&](auto KB) __attribute__((always_inline)) {
          if constexpr (decltype(KB)::value != kbn) gj_blk<decltype(KB)::value>(R, rk[decltype(KB)::value], nf);
        });
        R[cp] = (h == hp) ? newcol : R[cp];
      });
    }
  };

  // ---- 2. ADMM (osqp_solve) ----------------------------------------------------------------------
  double rho = rho0, pri_res = 0.0, dua_res = 0.0;
  int status = MPCQP_STATUS_UNSOLVED, iters = 0, rho_updates = 0, ntrace = 0;
  bool need_factor = true, first_factor = true;
  int to_check = p.check_termination, to_adapt = p.adaptive_rho_interval;
  for (int iter = 1; iter <= p.max_iter; ++iter) {
    if (need_factor) {
      sm.st[0][t] = X;
      sm.st[1][t] = Z;
      sm.st[2][t] = Y;
      sm.st[3][t] = PX;
      sm.st[4][t] = RHS;
      form_K(first_factor && mode != 0);
#ifdef DXE_DUMP  // debug: K, K^-1, D, E, c, rho of the first factorization into `solution`
      double* dump = solution + (size_t)inst * (2 * n * n + n + m + 2);
      if (vv)
        for (int c = 0; c < HS; ++c) dump[i * n + HS * h + c] = R[c];
      gj();
      if (vv)
        for (int c = 0; c < HS; ++c) dump[n * n + i * n + HS * h + c] = R[c];
      if (vv && h == 0) dump[2 * n * n + i] = var_D();
      if (hasrow) dump[2 * n * n + n + ri] = row_E();
      if (t == 0) {
        dump[2 * n * n + n + m] = cost_c;
        dump[2 * n * n + n + m + 1] = rho;
      }
      return;
#endif
      gj();
      asm volatile("" ::: "memory");
      refresh(rho);
      X = sm.st[0][t];
      Z = sm.st[1][t];
      Y = sm.st[2][t];
      PX = sm.st[3][t];
      RHS = sm.st[4][t];
      need_factor = false;
      first_factor = false;
    }
    // x~ = K^-1 rhs
    if (vv && h == 0) sm.wb[wbp][colpos(i)] = RHS;
    __syncthreads();
    const double xt = kmv(sm.wb[wbp]);
    wbp ^= 1;
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

    // update_x / update_z / update_y; P~x~ by the KKT identity P~x~ = rhs - sigma x~ - A~'rho A~x~
    // (DY, DX, P~x_old: for the infeasibility tests of a check iteration only)
    double DX = 0.0, DY = 0.0, PXO = 0.0;
    {
      const double zt = AKp * xt + AKz * fzv(xt);
      const double zr = alpha * zt + (1.0 - alpha) * Z;
      const double zn = fmin(fmax(zr + RIr * Y, Lp), Up);  // (the reference's c_min/c_max)
      const double dyv = RHOr * (zr - zn);
      Z = zn;
      Y = Y + dyv;
      DY = dyv;
      const double kd = at_op(RHOr * zt);
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
      const double Er = row_E(), Dv = var_D(), DI = 1. / Dv;
      double Lc, Uc;
      row_LU(Lc, Uc);
      double mx[14];
#pragma unroll
      for (int k = 0; k < 14; ++k) mx[k] = 0.0;
      const double ax = AKp * X + AKz * fzv(X);
      const double aty = at_op(Y);
      if (hasrow) {
        const double ei = 1.0 / Er;
        const double pr = ax + (-1.0) * Z;
        mx[0] = dabs(ei * pr);
        mx[1] = dabs(pr);
        mx[2] = dabs(ei * Z);
        mx[3] = dabs(Z);
        mx[4] = dabs(ei * ax);
        mx[5] = dabs(ax);
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
      block_red<NWV, 14, false>(mx, sm.red, rp);
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
          double d = DY;
          if (Uc > OSQP_INF * MIN_SCALING) {
            if (Lc < -OSQP_INF * MIN_SCALING) d = 0.0;
            else d = dmin(d, 0.0);
          } else if (Lc < -OSQP_INF * MIN_SCALING) {
            d = dmax(d, 0.0);
          }
          if (!hasrow) d = 0.0;
          double nd[1] = {hasrow ? dabs(Er * d) : 0.0};
          block_red<NWV, 1, false>(nd, sm.red, rp);
          const double ndy = nd[0];
          if (ndy > DIV_TOL) {
            double lh[1] = {hasrow ? Uc * dmax(d, 0.0) + Lc * dmin(d, 0.0) : 0.0};
            block_red<NWV, 1, true>(lh, sm.red, rp);
            if (lh[0] < eps_pinf * ndy) {
              const double atd = at_op(d);
              double an[1] = {vv ? dabs(DI * atd) : 0.0};
              block_red<NWV, 1, false>(an, sm.red, rp);
              prim_inf = an[0] < eps_pinf * ndy;
            }
          }
        }
        const double eps_dual = eps_abs + eps_rel * (cinv * dmax(dmax(mx[8], mx[10]), mx[12]));
        const bool dual_ok = dua_res < eps_dual;
        if (!dual_ok) {
          // is_dual_infeasible (P~ delta_x = P~x_new - P~x_old)
          double nx[1] = {vv ? dabs(Dv * DX) : 0.0};
          block_red<NWV, 1, false>(nx, sm.red, rp);
          const double ndx = nx[0];
          if (ndx > DIV_TOL) {
            double qd[1] = {(vv && h == 0) ? Qv * DX : 0.0};
            block_red<NWV, 1, true>(qd, sm.red, rp);
            if (qd[0] < cost_c * eps_dinf * ndx) {
              double pd[1] = {vv ? dabs(DI * (PX - PXO)) : 0.0};
              block_red<NWV, 1, false>(pd, sm.red, rp);
              if (pd[0] < cost_c * eps_dinf * ndx) {
                const double v = (1.0 / Er) * (AKp * DX + AKz * fzv(DX));
                double viol[1] = {0.0};
                if (hasrow && ((Uc < OSQP_INF * MIN_SCALING && v > eps_dinf * ndx) ||
                               (Lc > -OSQP_INF * MIN_SCALING && v < -eps_dinf * ndx)))
                  viol[0] = 1.0;
                block_red<NWV, 1, false>(viol, sm.red, rp);
                dual_inf = viol[0] == 0.0;
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
      if (trace && t == 0 && inst < trace_cap && ntrace < MPCQP_TRACE_LEN && is_check) {
        double* tp = trace + ((size_t)inst * MPCQP_TRACE_LEN + ntrace) * 4;
        tp[0] = iter; tp[1] = pri_res; tp[2] = dua_res; tp[3] = rho;
      }
      ntrace += is_check ? 1 : 0;
      if (done) break;
      if (refactor) {
        RHOr = rho_of(rho, Lc, Uc);
        RIr = 1. / RHOr;
        need_factor = true;
      }
    }
    // ---- next right-hand side: sigma x - q~ + A~'(rho z - y) ----
    RHS = (sigma * X - Qv) + at_op(RHOr * Z - Y);
  }

  if (ws) {  // the solver persists: scaling, scaled data, iterates and rho for the next tick
    if (t == 0) {
      ws[WL::FLAG] = 1.0;
      ws[WL::RHO] = rho;
      ws[WL::C] = cost_c;
      ws[WL::MU] = mu;
    }
    if (vv && h == 0) {
      ws[WL::D + i] = var_D();
      ws[WL::QT + i] = Qv;
      ws[WL::X + i] = X;
    }
    if (hasrow) {
      ws[WL::E + ri] = row_E();
      ws[WL::AK + ri] = a < 2 ? AKp : 0.0;
      ws[WL::AK + m + ri] = a < 2 ? AKz : AKp;
      ws[WL::Z + ri] = Z;
      ws[WL::Y + ri] = Y;
    }
  }
  // ---- 3. store_solution + unscale + compute_grf extraction (A1RobotControl.cpp:555-561) --------
  const bool has_sol = status != MPCQP_STATUS_PRIMAL_INFEASIBLE &&
                       status != MPCQP_STATUS_PRIMAL_INFEASIBLE_INACCURATE &&
                       status != MPCQP_STATUS_DUAL_INFEASIBLE &&
                       status != MPCQP_STATUS_DUAL_INFEASIBLE_INACCURATE && status != MPCQP_STATUS_NON_CVX;
  double ob[1] = {(vv && h == 0) ? 0.5 * X * PX + Qv * X : 0.0};
  block_red<NWV, 1, true>(ob, sm.red, rp);
  const double xs = has_sol ? var_D() * X : NAN;
  if (solution && vv && h == 0) solution[(size_t)inst * n + i] = xs;
  if (vv && h == 0 && i < ND) sm.xs[i] = xs;
  __syncthreads();
  mpcqp_result* res = results + inst;
  if (t < ND) {  // u0 = step 0; f_i = R^T u0[3i:3i+3], NaN legs skipped
    const int lg = t / 3, aa = t % 3;
    const double u00 = sm.xs[3 * lg], u01 = sm.xs[3 * lg + 1], u02 = sm.xs[3 * lg + 2];
    const double nrm = sqrt(u00 * u00 + u01 * u01 + u02 * u02);
    const double* Rot = rec + MPCQP_REC_ROT;
    double s = 0.0;
    s += sel3(aa, Rot[0], Rot[1], Rot[2]) * u00;
    s += sel3(aa, Rot[3], Rot[4], Rot[5]) * u01;
    s += sel3(aa, Rot[6], Rot[7], Rot[8]) * u02;
    res->u0[t] = sm.xs[t];
    res->f_body[t] = isnan(nrm) ? 0.0 : s;
  }
  if (t == 0) {
    int legs = 0;
    for (int lg = 0; lg < 4; ++lg) {
      const double u00 = sm.xs[3 * lg], u01 = sm.xs[3 * lg + 1], u02 = sm.xs[3 * lg + 2];
      if (isnan(sqrt(u00 * u00 + u01 * u01 + u02 * u02))) legs |= 1 << lg;
    }
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

// Self-test of the row shifts and the broadcast blocks: out[64 * k + lane]
__global__ void dx_selftest_kernel(double* out) {
  const int t = threadIdx.x;
  const double x = 100.0 * (t >> 4) + (t & 15);
  out[t] = shl<1>(x);
  out[64 + t] = shl<2>(x);
  out[128 + t] = shr<1>(x);
  out[192 + t] = shr<2>(x);
  double R[16];
  for (int c = 0; c < 16; ++c) R[c] = (double)c;
  gj_blk<0>(R, x, 1.0);  // R[c] = c + x(lane c of the row)
  double acc[4] = {0.0, 0.0, 0.0, 0.0};
  mv_blk<0>(R, 1.0, acc);  // sum_c R[c]
  out[256 + t] = R[5];
  out[320 + t] = (acc[0] + acc[1]) + (acc[2] + acc[3]);
}

}  // namespace dx

template <int N>
static hipError_t launch_dx(const LaunchArgs& a) {
  hipError_t e = launch_scale_any(a);  // scale_kernel<N> (mpcqp_wave.hip): the scaling image in a.work
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL((dx::dx_kernel<N>), dim3(a.batch), dim3(dx::DCfg<N>::NTH), 0, (hipStream_t)a.stream, a.recs,
                     a.batch, a.results, a.solution, a.trace, a.trace_cap, a.wstate, a.work, a.p);
  return hipGetLastError();
}
template <int N>
static hipError_t occupancy_dx(int* blocks) {
  return hipOccupancyMaxActiveBlocksPerMultiprocessor(blocks, dx::dx_kernel<N>, dx::DCfg<N>::NTH, 0);
}

#ifdef MPCQP_DX_ONE  // experiment builds: one horizon only
#define MPCQP_DX_FOR_EACH_N(X) X(MPCQP_DX_ONE)
#else
#define MPCQP_DX_FOR_EACH_N(X) X(1) X(2) X(3) X(4) X(5) X(6) X(7) X(8) X(9) X(10)
#endif

hipError_t launch_dx_any(const LaunchArgs& a) {
  switch (a.p.horizon) {
#define CASE(K) \
  case K: return launch_dx<K>(a);
    MPCQP_DX_FOR_EACH_N(CASE)
#undef CASE
    default: return hipErrorInvalidValue;
  }
}
hipError_t occupancy_dx_any(int horizon, int* blocks) {
  switch (horizon) {
#define CASE(K) \
  case K: return occupancy_dx<K>(blocks);
    MPCQP_DX_FOR_EACH_N(CASE)
#undef CASE
    default: return hipErrorInvalidValue;
  }
}
hipError_t dx_selftest(double* d_out, void* stream) {
  hipLaunchKernelGGL(dx::dx_selftest_kernel, dim3(1), dim3(64), 0, (hipStream_t)stream, d_out);
  return hipGetLastError();
}
}  // namespace mpcqp
