// Microbenchmark: issue cost of the binary64 VALU forms the solver is built from, for ONE wave per
// SIMD (the solver's occupancy): independent v_fmac_f64 (plain and DPP row_newbcast), dependent
// chains of each, v_permlane16/32_swap, v_mov_b64_dpp, s_nop, v_accvgpr moves.  Cycles per
// instruction from s_memtime around 64 x 16-instruction blocks, median over the workgroups.
// Numeric check (exit status 1 on a mismatch): the single-accumulator mat-vec chain of
// mpcqp_wave_common.h (mv12: twelve v_fmac_f64_dpp row_newbcast into one accumulator, each reading
// the accumulator its predecessor wrote with no wait state between them) against the host's fma
// chain, bitwise; and, for reference, the hazard the wait states guard: the DPP source written by the
// instruction just before.
//   hipcc -O3 --offload-arch=gfx950 tools/mb/mb_valu.hip -o tools/mb/mb_valu && tools/mb/mb_valu
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#include <algorithm>
#include <cmath>
#include <vector>

#define REP16(X) X X X X X X X X X X X X X X X X
#define KERNEL(NAME, BODY, NINS)                                                                   \
  __global__ __launch_bounds__(64) void NAME(double* out, long long* cyc, int iters) {              \
    double a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5,     \
           a6 = a0 + 6, a7 = a0 + 7, x = 1.0 / (1.0 + threadIdx.x), g = 0.5;                      \
    unsigned u0 = threadIdx.x, u1 = threadIdx.x * 3;                                              \
    long long c0 = 0;                                                                              \
    for (int it = 0; it < iters + 1; ++it) {                                                       \
      if (it == 1) c0 = __builtin_readcyclecounter();                                              \
      BODY                                                                                         \
    }                                                                                              \
    const long long c1 = __builtin_readcyclecounter();                                             \
    out[blockIdx.x * 64 + threadIdx.x] = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7 + u0 + u1;          \
    if (threadIdx.x == 0) cyc[blockIdx.x] = (c1 - c0);                                             \
  }

// 8 independent accumulators, plain FMA
#define B_FMA asm volatile(REP16("v_fmac_f64 %0, %8, %9\n\tv_fmac_f64 %1, %8, %9\n\t" \
  "v_fmac_f64 %2, %8, %9\n\tv_fmac_f64 %3, %8, %9\n\tv_fmac_f64 %4, %8, %9\n\tv_fmac_f64 %5, %8, %9\n\t" \
  "v_fmac_f64 %6, %8, %9\n\tv_fmac_f64 %7, %8, %9\n\t") \
  : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(x), "v"(g));
KERNEL(k_fma, B_FMA, 128)
// 8 independent accumulators, DPP row_newbcast FMA (the mat-vec / Gauss-Jordan form)
#define DF(A, L) "v_fmac_f64_dpp " A ", %8, %9 row_newbcast:" #L " row_mask:0xf bank_mask:0xf\n\t"
#define B_DPP asm volatile("s_nop 4\n\t" REP16(DF("%0", 0) DF("%1", 1) DF("%2", 2) DF("%3", 3) DF("%4", 4) \
  DF("%5", 5) DF("%6", 6) DF("%7", 7)) \
  : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(x), "v"(g));
KERNEL(k_dpp, B_DPP, 128)
// one dependent chain (latency): plain and DPP
#define B_CHAIN asm volatile(REP16("v_fmac_f64 %0, %1, %2\n\tv_fmac_f64 %0, %1, %2\n\t" \
  "v_fmac_f64 %0, %1, %2\n\tv_fmac_f64 %0, %1, %2\n\tv_fmac_f64 %0, %1, %2\n\tv_fmac_f64 %0, %1, %2\n\t" \
  "v_fmac_f64 %0, %1, %2\n\tv_fmac_f64 %0, %1, %2\n\t") : "+v"(a0) : "v"(x), "v"(g));
KERNEL(k_chain, B_CHAIN, 128)
#define DC(L) "v_fmac_f64_dpp %0, %1, %2 row_newbcast:" #L " row_mask:0xf bank_mask:0xf\n\t"
#define B_DCHAIN asm volatile("s_nop 4\n\t" REP16(DC(0) DC(1) DC(2) DC(3) DC(4) DC(5) DC(6) DC(7)) \
  : "+v"(a0) : "v"(x), "v"(g));
KERNEL(k_dchain, B_DCHAIN, 128)
// three accumulators in rotation (the solver's mv12 shape)
#define B_ROT3 asm volatile("s_nop 4\n\t" REP16(DF("%0", 0) DF("%1", 1) DF("%2", 2) DF("%0", 4) DF("%1", 5) \
  DF("%2", 6)) : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(x), "v"(g));
KERNEL(k_rot3, B_ROT3, 96)
// permlane swaps (32-bit), 8 independent per block
#define B_PERM asm volatile(REP16("v_permlane16_swap_b32 %0, %1\n\tv_permlane32_swap_b32 %0, %1\n\t" \
  "v_permlane16_swap_b32 %0, %1\n\tv_permlane32_swap_b32 %0, %1\n\t") : "+v"(u0), "+v"(u1));
KERNEL(k_perm, B_PERM, 64)
// accvgpr round trips
#define B_ACC asm volatile(REP16("v_accvgpr_write_b32 a0, %0\n\tv_accvgpr_write_b32 a1, %1\n\t" \
  "v_accvgpr_read_b32 %0, a2\n\tv_accvgpr_read_b32 %1, a3\n\t") : "+v"(u0), "+v"(u1) :: "a0", "a1", "a2", "a3");
KERNEL(k_acc, B_ACC, 64)
// s_nop 1 alone
#define B_NOP asm volatile(REP16("s_nop 1\n\ts_nop 1\n\ts_nop 1\n\ts_nop 1\n\t") ::);
KERNEL(k_nop, B_NOP, 64)
// v_max_f64 / v_add_f64 independent
#define B_MAX asm volatile(REP16("v_max_f64 %0, %0, %8\n\tv_max_f64 %1, %1, %8\n\tv_add_f64 %2, %2, %8\n\t" \
  "v_add_f64 %3, %3, %8\n\tv_max_f64 %4, %4, %8\n\tv_max_f64 %5, %5, %8\n\tv_add_f64 %6, %6, %8\n\tv_add_f64 %7, %7, %8\n\t") \
  : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(x));
KERNEL(k_max, B_MAX, 128)

// DPP FMA patterns: accumulator count 1 / 2 / 4 with a distinct multiplier per instruction (the
// mat-vec shape), and one accumulator with the same multiplier
#define B_D1C asm volatile("s_nop 4\n\t" REP16(DG("%0", "%1", 0) DG("%0", "%2", 1) DG("%0", "%3", 2) DG("%0", "%4", 3) \
  DG("%0", "%5", 4) DG("%0", "%6", 5) DG("%0", "%7", 6) DG("%0", "%9", 7)) \
  : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(x), "v"(g));
#define DG(A, C, L) "v_fmac_f64_dpp " A ", %8, " C " row_newbcast:" #L " row_mask:0xf bank_mask:0xf\n\t"
KERNEL(k_d1c, B_D1C, 128)
#define B_D2C asm volatile("s_nop 4\n\t" REP16(DG("%0", "%2", 0) DG("%1", "%3", 1) DG("%0", "%4", 2) DG("%1", "%5", 3) \
  DG("%0", "%6", 4) DG("%1", "%7", 5) DG("%0", "%9", 6) DG("%1", "%9", 7)) \
  : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(x), "v"(g));
KERNEL(k_d2c, B_D2C, 128)
#define B_D4C asm volatile("s_nop 4\n\t" REP16(DG("%0", "%4", 0) DG("%1", "%5", 1) DG("%2", "%6", 2) DG("%3", "%7", 3) \
  DG("%0", "%5", 4) DG("%1", "%6", 5) DG("%2", "%7", 6) DG("%3", "%9", 7)) \
  : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(x), "v"(g));
KERNEL(k_d4c, B_D4C, 128)
// plain FMA with a distinct multiplier per instruction, 4 accumulators
#define PG(A, C) "v_fmac_f64 " A ", %8, " C "\n\t"
#define B_P4C asm volatile(REP16(PG("%0", "%4") PG("%1", "%5") PG("%2", "%6") PG("%3", "%7") \
  PG("%0", "%5") PG("%1", "%6") PG("%2", "%7") PG("%3", "%9")) \
  : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(x), "v"(g));
KERNEL(k_p4c, B_P4C, 128)

// the mv12 chain: a += bcast_L(x) * c[n] over the twelve lanes L of WV_M12, one accumulator
#define CK(N, L) "v_fmac_f64_dpp %[a], %[x], %[c" #N "] row_newbcast:" #L " row_mask:0xf bank_mask:0xf\n\t"
#define CK12 CK(0, 0) CK(1, 1) CK(2, 2) CK(3, 4) CK(4, 5) CK(5, 6) CK(6, 8) CK(7, 9) CK(8, 10) CK(9, 12) CK(10, 13) CK(11, 14)
#define CK_OPS [c0] "v"(c[0]), [c1] "v"(c[1]), [c2] "v"(c[2]), [c3] "v"(c[3]), [c4] "v"(c[4]), [c5] "v"(c[5]), \
    [c6] "v"(c[6]), [c7] "v"(c[7]), [c8] "v"(c[8]), [c9] "v"(c[9]), [c10] "v"(c[10]), [c11] "v"(c[11])
__global__ __launch_bounds__(64) void k_check(const double* xin, const double* cin, double* out, int hazard) {
  const int t = threadIdx.x;
  double x = xin[t], c[12];
  for (int n = 0; n < 12; ++n) c[n] = cin[12 * t + n];
  double a = 0.0;
  if (hazard)  // x rewritten by the instruction just before the first DPP read of it
    asm volatile("s_nop 4\n\tv_add_f64 %[x], %[x], 1.0\n\t" CK12 : [a] "+v"(a), [x] "+v"(x) : CK_OPS);
  else
    asm volatile("s_nop 4\n\t" CK12 : [a] "+v"(a) : [x] "v"(x), CK_OPS);
  out[t] = a;
}
static int check_chain(bool hazard) {
  double hx[64], hc[64 * 12], ho[64], *dx, *dc, *dout;
  for (int t = 0; t < 64; ++t) {
    hx[t] = 1.0 / (3.0 + t) - 0.125 * (t & 7);
    for (int n = 0; n < 12; ++n) hc[12 * t + n] = 0.37 * n - 1.0 / (1.0 + t + n);
  }
  hipMalloc(&dx, sizeof(hx));
  hipMalloc(&dc, sizeof(hc));
  hipMalloc(&dout, sizeof(ho));
  hipMemcpy(dx, hx, sizeof(hx), hipMemcpyHostToDevice);
  hipMemcpy(dc, hc, sizeof(hc), hipMemcpyHostToDevice);
  hipLaunchKernelGGL(k_check, dim3(1), dim3(64), 0, 0, dx, dc, dout, hazard ? 1 : 0);
  hipMemcpy(ho, dout, sizeof(ho), hipMemcpyDeviceToHost);
  const int lanes[12] = {0, 1, 2, 4, 5, 6, 8, 9, 10, 12, 13, 14};
  int bad = 0;
  for (int t = 0; t < 64; ++t) {
    double a = 0.0;
    for (int n = 0; n < 12; ++n) {
      const double xb = hx[16 * (t / 16) + lanes[n]] + (hazard ? 1.0 : 0.0);
      a = std::fma(xb, hc[12 * t + n], a);
    }
    bad += a != ho[t];
  }
  hipFree(dx);
  hipFree(dc);
  hipFree(dout);
  return bad;
}

typedef void (*kfn)(double*, long long*, int);
int main() {
  const int blocks = 1024, iters = 200;  // one 64-thread wave per SIMD on 256 CUs
  double* d_out;
  long long* d_cyc;
  hipMalloc(&d_out, sizeof(double) * blocks * 64);
  hipMalloc(&d_cyc, sizeof(long long) * blocks);
  struct K {
    const char* name;
    kfn f;
    int ins;
  } ks[] = {{"v_fmac_f64 x8 indep", k_fma, 128},          {"v_fmac_f64_dpp x8 indep", k_dpp, 128},
            {"v_fmac_f64 dep chain", k_chain, 128},       {"v_fmac_f64_dpp dep chain", k_dchain, 128},
            {"v_fmac_f64_dpp 3 acc rot", k_rot3, 96},    {"v_permlane16/32_swap", k_perm, 64},
            {"v_accvgpr write/read", k_acc, 64},          {"s_nop 1", k_nop, 64},
            {"v_max/add_f64 x8 indep", k_max, 128},       {"dpp fma 1 acc, 8 mults", k_d1c, 128},
            {"dpp fma 2 acc, 8 mults", k_d2c, 128},       {"dpp fma 4 acc, 8 mults", k_d4c, 128},
            {"plain fma 4 acc, 8 mults", k_p4c, 128}};
  std::vector<long long> cyc(blocks);
  for (auto& k : ks) {
    hipLaunchKernelGGL(k.f, dim3(blocks), dim3(64), 0, 0, d_out, d_cyc, 2);
    hipLaunchKernelGGL(k.f, dim3(blocks), dim3(64), 0, 0, d_out, d_cyc, iters);
    hipDeviceSynchronize();
    hipMemcpy(cyc.data(), d_cyc, sizeof(long long) * blocks, hipMemcpyDeviceToHost);
    std::sort(cyc.begin(), cyc.end());
    const double med = (double)cyc[blocks / 2] / ((double)iters * k.ins);
    printf("%-28s %6.2f cycles/instruction (median over %d waves)\n", k.name, med, blocks);
  }
  const int bad = check_chain(false), bad_h = check_chain(true);
  printf("dependent DPP FMA chain, one accumulator (mv12 form): %d of 64 lanes differ from the host fma chain\n", bad);
  printf("(reference) DPP source written 0 wait states before: %d of 64 lanes differ\n", bad_h);
  return bad ? 1 : 0;
}
