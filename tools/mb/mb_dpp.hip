// Microbenchmark: what the 1.1-cycle premium of v_fmac_f64_dpp over v_fmac_f64 depends on (one wave
// per SIMD).  Explicit VGPR numbers, so the register banks (v[n]: bank n mod 4) of the DPP source,
// the multiplier and the accumulators are fixed.  Cycles per instruction, median over the waves.
//   hipcc -O3 --offload-arch=gfx950 tools/mb/mb_dpp.hip -o tools/mb/mb_dpp && tools/mb/mb_dpp
#include <hip/hip_runtime.h>
#include <stdio.h>

#include <algorithm>
#include <vector>

#define REP8(X) X X X X X X X X
#define CLOB "v0", "v1", "v2", "v3", "v4", "v5", "v6", "v7", "v8", "v9", "v10", "v11", "v12", "v13", "v14", \
  "v15", "v16", "v17", "v18", "v19", "v20", "v21", "v22", "v23", "v24", "v25", "v26", "v27", "v28", "v29", \
  "v30", "v31", "v32", "v33", "v34", "v35", "v36", "v37", "v38", "v39"
#define INIT asm volatile("v_cvt_f64_u32 v[0:1], %0\n\t" \
  "v_mov_b64 v[2:3], v[0:1]\n\tv_mov_b64 v[4:5], v[0:1]\n\tv_mov_b64 v[6:7], v[0:1]\n\t" \
  "v_mov_b64 v[8:9], v[0:1]\n\tv_mov_b64 v[10:11], v[0:1]\n\tv_mov_b64 v[12:13], v[0:1]\n\t" \
  "v_mov_b64 v[14:15], v[0:1]\n\tv_mov_b64 v[16:17], v[0:1]\n\tv_mov_b64 v[18:19], v[0:1]\n\t" \
  "v_mov_b64 v[20:21], v[0:1]\n\tv_mov_b64 v[22:23], v[0:1]\n\tv_mov_b64 v[24:25], v[0:1]\n\t" \
  "v_mov_b64 v[26:27], v[0:1]\n\tv_mov_b64 v[28:29], v[0:1]\n\tv_mov_b64 v[30:31], v[0:1]\n\t" \
  "v_mov_b64 v[32:33], v[0:1]\n\tv_mov_b64 v[34:35], v[0:1]\n\tv_mov_b64 v[36:37], v[0:1]\n\t" \
  "v_mov_b64 v[38:39], v[0:1]\n\ts_nop 4" :: "v"(threadIdx.x) : CLOB);
#define KERNEL(NAME, BODY, NINS)                                                                  \
  __global__ __launch_bounds__(64) void NAME(double* out, long long* cyc, int iters) {             \
    INIT                                                                                          \
    long long c0 = 0;                                                                             \
    for (int it = 0; it < iters + 1; ++it) {                                                      \
      if (it == 1) c0 = __builtin_readcyclecounter();                                             \
      asm volatile(BODY ::: CLOB);                                                                \
    }                                                                                             \
    const long long c1 = __builtin_readcyclecounter();                                            \
    double r;                                                                                     \
    asm volatile("v_add_f64 %0, v[8:9], v[10:11]\n\tv_add_f64 %0, %0, v[12:13]" : "=v"(r) :: CLOB); \
    out[blockIdx.x * 64 + threadIdx.x] = r;                                                       \
    if (threadIdx.x == 0) cyc[blockIdx.x] = (c1 - c0);                                            \
  }

// D(acc, src0, src1, lane): acc += bcast_lane(src0) * src1
#define D(A, X, G, L) "v_fmac_f64_dpp " A ", " X ", " G " row_newbcast:" #L " row_mask:0xf bank_mask:0xf\n\t"
#define P(A, X, G) "v_fmac_f64 " A ", " X ", " G "\n\t"
// x = v[0:1] (bank 0), g = v[2:3] (bank 2); accumulators in bank 0 (v8, v12, ...) or 2 (v10, v14, ...)
#define ACC_B0 D("v[8:9]", "v[0:1]", "v[2:3]", 0) D("v[12:13]", "v[0:1]", "v[2:3]", 1) D("v[16:17]", "v[0:1]", "v[2:3]", 2) \
  D("v[20:21]", "v[0:1]", "v[2:3]", 3) D("v[24:25]", "v[0:1]", "v[2:3]", 4) D("v[28:29]", "v[0:1]", "v[2:3]", 5)   \
  D("v[32:33]", "v[0:1]", "v[2:3]", 6) D("v[36:37]", "v[0:1]", "v[2:3]", 7)
#define ACC_B2 D("v[10:11]", "v[0:1]", "v[2:3]", 0) D("v[14:15]", "v[0:1]", "v[2:3]", 1) D("v[18:19]", "v[0:1]", "v[2:3]", 2) \
  D("v[22:23]", "v[0:1]", "v[2:3]", 3) D("v[26:27]", "v[0:1]", "v[2:3]", 4) D("v[30:31]", "v[0:1]", "v[2:3]", 5)   \
  D("v[34:35]", "v[0:1]", "v[2:3]", 6) D("v[38:39]", "v[0:1]", "v[2:3]", 7)
// x in bank 2 (v[4:5]), g in bank 0 (v[6:7]): accumulators bank 0 / bank 2
#define ACC_X2_B0 D("v[8:9]", "v[4:5]", "v[6:7]", 0) D("v[12:13]", "v[4:5]", "v[6:7]", 1) D("v[16:17]", "v[4:5]", "v[6:7]", 2) \
  D("v[20:21]", "v[4:5]", "v[6:7]", 3) D("v[24:25]", "v[4:5]", "v[6:7]", 4) D("v[28:29]", "v[4:5]", "v[6:7]", 5)   \
  D("v[32:33]", "v[4:5]", "v[6:7]", 6) D("v[36:37]", "v[4:5]", "v[6:7]", 7)
// same lane every instruction (row_newbcast:3) vs varying: is it the lane change?
#define ACC_SAMEL D("v[8:9]", "v[0:1]", "v[2:3]", 3) D("v[12:13]", "v[0:1]", "v[2:3]", 3) D("v[16:17]", "v[0:1]", "v[2:3]", 3) \
  D("v[20:21]", "v[0:1]", "v[2:3]", 3) D("v[24:25]", "v[0:1]", "v[2:3]", 3) D("v[28:29]", "v[0:1]", "v[2:3]", 3)   \
  D("v[32:33]", "v[0:1]", "v[2:3]", 3) D("v[36:37]", "v[0:1]", "v[2:3]", 3)
// two interleaved DPP sources (x0 = v[0:1], x1 = v[4:5])
#define ACC_2X D("v[8:9]", "v[0:1]", "v[2:3]", 0) D("v[12:13]", "v[4:5]", "v[2:3]", 1) D("v[16:17]", "v[0:1]", "v[2:3]", 2) \
  D("v[20:21]", "v[4:5]", "v[2:3]", 3) D("v[24:25]", "v[0:1]", "v[2:3]", 4) D("v[28:29]", "v[4:5]", "v[2:3]", 5)   \
  D("v[32:33]", "v[0:1]", "v[2:3]", 6) D("v[36:37]", "v[4:5]", "v[2:3]", 7)
// one accumulator chain, same operands (the known 4.38 case) and fresh multipliers
#define CHAIN_SAME D("v[8:9]", "v[0:1]", "v[2:3]", 0) D("v[8:9]", "v[0:1]", "v[2:3]", 1) D("v[8:9]", "v[0:1]", "v[2:3]", 2) \
  D("v[8:9]", "v[0:1]", "v[2:3]", 3) D("v[8:9]", "v[0:1]", "v[2:3]", 4) D("v[8:9]", "v[0:1]", "v[2:3]", 5)   \
  D("v[8:9]", "v[0:1]", "v[2:3]", 6) D("v[8:9]", "v[0:1]", "v[2:3]", 7)
#define CHAIN_FRESH D("v[8:9]", "v[0:1]", "v[10:11]", 0) D("v[8:9]", "v[0:1]", "v[14:15]", 1) D("v[8:9]", "v[0:1]", "v[18:19]", 2) \
  D("v[8:9]", "v[0:1]", "v[22:23]", 3) D("v[8:9]", "v[0:1]", "v[26:27]", 4) D("v[8:9]", "v[0:1]", "v[30:31]", 5)   \
  D("v[8:9]", "v[0:1]", "v[34:35]", 6) D("v[8:9]", "v[0:1]", "v[38:39]", 7)
// fresh multipliers in bank 0 with the chain in bank 0 and x in bank 0
#define CHAIN_FRESH_B0 D("v[8:9]", "v[0:1]", "v[12:13]", 0) D("v[8:9]", "v[0:1]", "v[16:17]", 1) D("v[8:9]", "v[0:1]", "v[20:21]", 2) \
  D("v[8:9]", "v[0:1]", "v[24:25]", 3) D("v[8:9]", "v[0:1]", "v[28:29]", 4) D("v[8:9]", "v[0:1]", "v[32:33]", 5)   \
  D("v[8:9]", "v[0:1]", "v[36:37]", 6) D("v[8:9]", "v[0:1]", "v[4:5]", 7)
// plain FMA, same register pattern as ACC_B0 / CHAIN_FRESH
#define PACC_B0 P("v[8:9]", "v[0:1]", "v[2:3]") P("v[12:13]", "v[0:1]", "v[2:3]") P("v[16:17]", "v[0:1]", "v[2:3]") \
  P("v[20:21]", "v[0:1]", "v[2:3]") P("v[24:25]", "v[0:1]", "v[2:3]") P("v[28:29]", "v[0:1]", "v[2:3]")             \
  P("v[32:33]", "v[0:1]", "v[2:3]") P("v[36:37]", "v[0:1]", "v[2:3]")
#define PCHAIN_FRESH P("v[8:9]", "v[0:1]", "v[10:11]") P("v[8:9]", "v[0:1]", "v[14:15]") P("v[8:9]", "v[0:1]", "v[18:19]") \
  P("v[8:9]", "v[0:1]", "v[22:23]") P("v[8:9]", "v[0:1]", "v[26:27]") P("v[8:9]", "v[0:1]", "v[30:31]")             \
  P("v[8:9]", "v[0:1]", "v[34:35]") P("v[8:9]", "v[0:1]", "v[38:39]")
// DPP only every other instruction (DPP FMA, plain FMA on other registers)
#define MIX D("v[8:9]", "v[0:1]", "v[2:3]", 0) P("v[10:11]", "v[4:5]", "v[6:7]") D("v[12:13]", "v[0:1]", "v[2:3]", 1) \
  P("v[14:15]", "v[4:5]", "v[6:7]") D("v[16:17]", "v[0:1]", "v[2:3]", 2) P("v[18:19]", "v[4:5]", "v[6:7]")           \
  D("v[20:21]", "v[0:1]", "v[2:3]", 3) P("v[22:23]", "v[4:5]", "v[6:7]")
// v_mov_b64 DPP broadcast + plain FMA (two instructions per term)
#define MOVF "v_mov_b64_dpp v[4:5], v[0:1] row_newbcast:1 row_mask:0xf bank_mask:0xf\n\t" P("v[8:9]", "v[4:5]", "v[2:3]") \
  "v_mov_b64_dpp v[6:7], v[0:1] row_newbcast:2 row_mask:0xf bank_mask:0xf\n\t" P("v[12:13]", "v[6:7]", "v[2:3]")             \
  "v_mov_b64_dpp v[10:11], v[0:1] row_newbcast:3 row_mask:0xf bank_mask:0xf\n\t" P("v[16:17]", "v[10:11]", "v[2:3]")         \
  "v_mov_b64_dpp v[14:15], v[0:1] row_newbcast:4 row_mask:0xf bank_mask:0xf\n\t" P("v[20:21]", "v[14:15]", "v[2:3]")

KERNEL(k_acc_b0, REP8(ACC_B0), 64)
KERNEL(k_acc_b2, REP8(ACC_B2), 64)
KERNEL(k_acc_x2_b0, REP8(ACC_X2_B0), 64)
KERNEL(k_acc_samel, REP8(ACC_SAMEL), 64)
KERNEL(k_acc_2x, REP8(ACC_2X), 64)
KERNEL(k_chain_same, REP8(CHAIN_SAME), 64)
KERNEL(k_chain_fresh, REP8(CHAIN_FRESH), 64)
KERNEL(k_chain_fresh_b0, REP8(CHAIN_FRESH_B0), 64)
KERNEL(k_pacc_b0, REP8(PACC_B0), 64)
KERNEL(k_pchain_fresh, REP8(PCHAIN_FRESH), 64)
KERNEL(k_mix, REP8(MIX), 64)
KERNEL(k_movf, REP8(MOVF), 64)

typedef void (*kfn)(double*, long long*, int);
int main() {
  const int blocks = 1024, iters = 200;
  double* d_out;
  long long* d_cyc;
  hipMalloc(&d_out, sizeof(double) * blocks * 64);
  hipMalloc(&d_cyc, sizeof(long long) * blocks);
  struct K {
    const char* name;
    kfn f;
    int ins;
  } ks[] = {{"dpp 8 acc bank0, x b0 g b2", k_acc_b0, 64},    {"dpp 8 acc bank2, x b0 g b2", k_acc_b2, 64},
            {"dpp 8 acc bank0, x b2 g b0", k_acc_x2_b0, 64}, {"dpp 8 acc, same bcast lane", k_acc_samel, 64},
            {"dpp 8 acc, two x alternating", k_acc_2x, 64},  {"dpp chain, same operands", k_chain_same, 64},
            {"dpp chain, fresh g bank2", k_chain_fresh, 64}, {"dpp chain, fresh g bank0", k_chain_fresh_b0, 64},
            {"plain 8 acc bank0", k_pacc_b0, 64},            {"plain chain, fresh g", k_pchain_fresh, 64},
            {"dpp / plain alternating", k_mix, 64},          {"mov_b64_dpp + plain fma", k_movf, 64}};
  std::vector<long long> cyc(blocks);
  for (auto& k : ks) {
    hipLaunchKernelGGL(k.f, dim3(blocks), dim3(64), 0, 0, d_out, d_cyc, 2);
    hipLaunchKernelGGL(k.f, dim3(blocks), dim3(64), 0, 0, d_out, d_cyc, iters);
    hipDeviceSynchronize();
    hipMemcpy(cyc.data(), d_cyc, sizeof(long long) * blocks, hipMemcpyDeviceToHost);
    std::sort(cyc.begin(), cyc.end());
    printf("%-32s %6.2f cycles/instruction\n", k.name, (double)cyc[blocks / 2] / ((double)iters * k.ins));
  }
  return 0;
}
