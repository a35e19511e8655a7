// Microbenchmark: how binary64 DPP mat-vec chains (the wave kernel's Riccati backward/forward
// passes) scale with waves per SIMD.  Each wave repeats a 9-step chain of 12x12 mat-vecs whose
// matrices sit in LDS (the wave kernel's pattern: ld12 + 12 v_fmac_f64_dpp row_newbcast + a
// permlane row hand-off).  Residency per CU is forced with dynamic LDS (160 KiB / W per block).
// Also: dependent / independent v_fma_f64 and v_fmac_f64_dpp latency and issue rates.
//   hipcc -O3 --offload-arch=gfx950 tools/mb/mb_chain.hip -o tools/mb/mb_chain && tools/mb/mb_chain
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#define CK(x)                                                              \
  do {                                                                     \
    hipError_t e_ = (x);                                                   \
    if (e_ != hipSuccess) {                                                \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                             \
    }                                                                      \
  } while (0)

#define FM(A, M, L) "v_fmac_f64_dpp " A ", %[x], " M " row_newbcast:" #L " row_mask:0xf bank_mask:0xf\n\t"
__device__ __forceinline__ double mv12(double x, const double (&c)[12]) {
  double a0 = 0.0, a1 = 0.0, a2 = 0.0;
  asm("s_nop 4\n\t"
      FM("%[a0]", "%[c0]", 0) FM("%[a1]", "%[c1]", 1) FM("%[a2]", "%[c2]", 2)
      FM("%[a0]", "%[c3]", 4) FM("%[a1]", "%[c4]", 5) FM("%[a2]", "%[c5]", 6)
      FM("%[a0]", "%[c6]", 8) FM("%[a1]", "%[c7]", 9) FM("%[a2]", "%[c8]", 10)
      FM("%[a0]", "%[c9]", 12) FM("%[a1]", "%[c10]", 13) FM("%[a2]", "%[c11]", 14)
      : [a0] "+v"(a0), [a1] "+v"(a1), [a2] "+v"(a2)
      : [x] "v"(x), [c0] "v"(c[0]), [c1] "v"(c[1]), [c2] "v"(c[2]), [c3] "v"(c[3]), [c4] "v"(c[4]),
        [c5] "v"(c[5]), [c6] "v"(c[6]), [c7] "v"(c[7]), [c8] "v"(c[8]), [c9] "v"(c[9]), [c10] "v"(c[10]),
        [c11] "v"(c[11]));
  return (a0 + a1) + a2;
}
__device__ __forceinline__ double swap16(double v) {
  const unsigned lo = (unsigned)__double2loint(v), hi = (unsigned)__double2hiint(v);
  const auto l2 = __builtin_amdgcn_permlane16_swap(lo, lo, false, false);
  const auto h2 = __builtin_amdgcn_permlane16_swap(hi, hi, false, false);
  return __hiloint2double((int)h2[0], (int)l2[0]);
}

// 9-step chain, matrices in LDS (dynamic shared, first 9*144 doubles), ITERS repetitions
__global__ __launch_bounds__(64) void chain_kernel(double* out, long long* cyc, int iters) {
  extern __shared__ double lds[];
  const int t = threadIdx.x, idx = t & 15;
  for (int e = t; e < 9 * 144; e += 64) lds[e] = 1e-3 * ((e * 37) % 101) - 0.05;
  __builtin_amdgcn_wave_barrier();
  double cur = 0.5 + 0.01 * t;
  const long long c0 = __builtin_readcyclecounter();
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int k = 0; k < 9; ++k) {
      double c[12];
      const double* p = lds + 144 * k + (idx % 12);
#pragma unroll
      for (int i = 0; i < 12; ++i) c[i] = p[12 * i];
      cur = mv12(swap16(cur), c) - 0.25 * cur;
    }
  }
  const long long c1 = __builtin_readcyclecounter();
  out[blockIdx.x * 64 + t] = cur;
  if (t == 0) cyc[blockIdx.x] = c1 - c0;
}


// same chain with the matrices in registers (compute floor of a chain step)
__global__ __launch_bounds__(64) void chain_reg_kernel(double* out, long long* cyc, int iters) {
  const int t = threadIdx.x;
  double m[9][12];
#pragma unroll
  for (int k = 0; k < 9; ++k)
#pragma unroll
    for (int i = 0; i < 12; ++i) m[k][i] = 1e-3 * (((k * 12 + i) * 37 + t) % 101) - 0.05;
  double cur = 0.5 + 0.01 * t;
  const long long c0 = __builtin_readcyclecounter();
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int k = 0; k < 9; ++k) cur = mv12(swap16(cur), m[k]) - 0.25 * cur;
  }
  const long long c1 = __builtin_readcyclecounter();
  out[blockIdx.x * 64 + t] = cur;
  if (t == 0) cyc[blockIdx.x] = c1 - c0;
}
// LDS chain with the next step's matrix prefetched
__global__ __launch_bounds__(64) void chain_pf_kernel(double* out, long long* cyc, int iters) {
  extern __shared__ double lds[];
  const int t = threadIdx.x, idx = t & 15;
  for (int e = t; e < 9 * 144; e += 64) lds[e] = 1e-3 * ((e * 37) % 101) - 0.05;
  __builtin_amdgcn_wave_barrier();
  double cur = 0.5 + 0.01 * t;
  const double* base = lds + (idx % 12);
  double cn[12];
#pragma unroll
  for (int i = 0; i < 12; ++i) cn[i] = base[12 * i];
  const long long c0 = __builtin_readcyclecounter();
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int k = 0; k < 9; ++k) {
      double c[12];
#pragma unroll
      for (int i = 0; i < 12; ++i) c[i] = cn[i];
      const double* p = base + 144 * ((k + 1) % 9);
#pragma unroll
      for (int i = 0; i < 12; ++i) cn[i] = p[12 * i];
      cur = mv12(swap16(cur), c) - 0.25 * cur;
    }
  }
  const long long c1 = __builtin_readcyclecounter();
  out[blockIdx.x * 64 + t] = cur;
  if (t == 0) cyc[blockIdx.x] = c1 - c0;
}


// y = sum_c M[c] x_c + a  (accumulator a0 starts at `init`: the chain's "- a_k" folded in)
__device__ __forceinline__ double mv12i(double x, const double (&c)[12], double init) {
  double a0 = init, a1 = 0.0, a2 = 0.0;
  asm("s_nop 4\n\t"
      FM("%[a1]", "%[c1]", 1) FM("%[a2]", "%[c2]", 2) FM("%[a0]", "%[c0]", 0)
      FM("%[a1]", "%[c4]", 5) FM("%[a2]", "%[c5]", 6) FM("%[a0]", "%[c3]", 4)
      FM("%[a1]", "%[c7]", 9) FM("%[a2]", "%[c8]", 10) FM("%[a0]", "%[c6]", 8)
      FM("%[a1]", "%[c10]", 13) FM("%[a2]", "%[c11]", 14) FM("%[a0]", "%[c9]", 12)
      : [a0] "+v"(a0), [a1] "+v"(a1), [a2] "+v"(a2)
      : [x] "v"(x), [c0] "v"(c[0]), [c1] "v"(c[1]), [c2] "v"(c[2]), [c3] "v"(c[3]), [c4] "v"(c[4]),
        [c5] "v"(c[5]), [c6] "v"(c[6]), [c7] "v"(c[7]), [c8] "v"(c[8]), [c9] "v"(c[9]), [c10] "v"(c[10]),
        [c11] "v"(c[11]));
  return (a1 + a2) + a0;
}
// odd rows := even rows (other rows undefined): one permlane16_swap per dword, no copies
__device__ __forceinline__ double to_odd(double v) {
  unsigned lo = (unsigned)__double2loint(v), hi = (unsigned)__double2hiint(v);
  unsigned rl, rh;
  asm volatile("s_nop 1\n\tv_permlane16_swap_b32 %0, %2\n\tv_permlane16_swap_b32 %1, %3"
               : "=&v"(rl), "=&v"(rh), "+v"(lo), "+v"(hi));
  return __hiloint2double((int)rh, (int)rl);
}
// LDS chain, prefetch pinned by sched_barrier, folded subtraction, copy-free hand-off
__global__ __launch_bounds__(64) void chain_pf2_kernel(double* out, long long* cyc, int iters) {
  extern __shared__ double lds[];
  const int t = threadIdx.x, idx = t & 15;
  for (int e = t; e < 9 * 144; e += 64) lds[e] = 1e-3 * ((e * 37) % 101) - 0.05;
  __builtin_amdgcn_wave_barrier();
  double cur = 0.5 + 0.01 * t;
  const double ak = 0.125 * t;
  const double* base = lds + (idx % 12);
  double cn[12];
#pragma unroll
  for (int i = 0; i < 12; ++i) cn[i] = base[12 * i];
  const long long c0 = __builtin_readcyclecounter();
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int k = 0; k < 9; ++k) {
      double c[12];
#pragma unroll
      for (int i = 0; i < 12; ++i) c[i] = cn[i];
      const double* p = base + 144 * ((k + 1) % 9);
#pragma unroll
      for (int i = 0; i < 12; ++i) cn[i] = p[12 * i];
      __builtin_amdgcn_sched_barrier(0);
      cur = mv12i(to_odd(cur), c, -ak);
    }
  }
  const long long c1 = __builtin_readcyclecounter();
  out[blockIdx.x * 64 + t] = cur;
  if (t == 0) cyc[blockIdx.x] = c1 - c0;
}
// register matrices, folded subtraction, copy-free hand-off (compute floor of the new step)
__global__ __launch_bounds__(64) void chain_reg2_kernel(double* out, long long* cyc, int iters) {
  const int t = threadIdx.x;
  double m[9][12];
#pragma unroll
  for (int k = 0; k < 9; ++k)
#pragma unroll
    for (int i = 0; i < 12; ++i) m[k][i] = 1e-3 * (((k * 12 + i) * 37 + t) % 101) - 0.05;
  double cur = 0.5 + 0.01 * t;
  const double ak = 0.125 * t;
  const long long c0 = __builtin_readcyclecounter();
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int k = 0; k < 9; ++k) cur = mv12i(to_odd(cur), m[k], -ak);
  }
  const long long c1 = __builtin_readcyclecounter();
  out[blockIdx.x * 64 + t] = cur;
  if (t == 0) cyc[blockIdx.x] = c1 - c0;
}


// as chain_pf2, the matrix stored transposed so the lane's 12 coefficients are contiguous (b128)
__global__ __launch_bounds__(64) void chain_pf3_kernel(double* out, long long* cyc, int iters) {
  extern __shared__ double lds[];
  const int t = threadIdx.x, idx = t & 15;
  for (int e = t; e < 9 * 144; e += 64) lds[e] = 1e-3 * ((e * 37) % 101) - 0.05;
  __builtin_amdgcn_wave_barrier();
  double cur = 0.5 + 0.01 * t;
  const double ak = 0.125 * t;
  const double* base = lds + 12 * (idx % 12);
  double cn[12];
#pragma unroll
  for (int i = 0; i < 12; ++i) cn[i] = base[i];
  const long long c0 = __builtin_readcyclecounter();
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int k = 0; k < 9; ++k) {
      double c[12];
#pragma unroll
      for (int i = 0; i < 12; ++i) c[i] = cn[i];
      const double2* p = reinterpret_cast<const double2*>(base + 144 * ((k + 1) % 9));
#pragma unroll
      for (int i = 0; i < 6; ++i) {
        const double2 v = p[i];
        cn[2 * i] = v.x;
        cn[2 * i + 1] = v.y;
      }
      __builtin_amdgcn_sched_barrier(0);
      cur = mv12i(to_odd(cur), c, -ak);
    }
  }
  const long long c1 = __builtin_readcyclecounter();
  out[blockIdx.x * 64 + t] = cur;
  if (t == 0) cyc[blockIdx.x] = c1 - c0;
}
// chain_reg2 / chain_pf3 with no row hand-off (every DPP row carries the chain vector)
__global__ __launch_bounds__(64) void chain_reg3_kernel(double* out, long long* cyc, int iters) {
  const int t = threadIdx.x;
  double m[9][12];
#pragma unroll
  for (int k = 0; k < 9; ++k)
#pragma unroll
    for (int i = 0; i < 12; ++i) m[k][i] = 1e-3 * (((k * 12 + i) * 37 + t) % 101) - 0.05;
  double cur = 0.5 + 0.01 * t;
  const double ak = 0.125 * t;
  const long long c0 = __builtin_readcyclecounter();
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int k = 0; k < 9; ++k) cur = mv12i(cur, m[k], -ak);
  }
  const long long c1 = __builtin_readcyclecounter();
  out[blockIdx.x * 64 + t] = cur;
  if (t == 0) cyc[blockIdx.x] = c1 - c0;
}
__global__ __launch_bounds__(64) void chain_pf4_kernel(double* out, long long* cyc, int iters) {
  extern __shared__ double lds[];
  const int t = threadIdx.x, idx = t & 15;
  for (int e = t; e < 9 * 144; e += 64) lds[e] = 1e-3 * ((e * 37) % 101) - 0.05;
  __builtin_amdgcn_wave_barrier();
  double cur = 0.5 + 0.01 * t;
  const double ak = 0.125 * t;
  const double* base = lds + 12 * (idx % 12);
  double cn[12];
#pragma unroll
  for (int i = 0; i < 12; ++i) cn[i] = base[i];
  const long long c0 = __builtin_readcyclecounter();
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int k = 0; k < 9; ++k) {
      double c[12];
#pragma unroll
      for (int i = 0; i < 12; ++i) c[i] = cn[i];
      const double2* p = reinterpret_cast<const double2*>(base + 144 * ((k + 1) % 9));
#pragma unroll
      for (int i = 0; i < 6; ++i) {
        const double2 v = p[i];
        cn[2 * i] = v.x;
        cn[2 * i + 1] = v.y;
      }
      __builtin_amdgcn_sched_barrier(0);
      cur = mv12i(cur, c, -ak);
    }
  }
  const long long c1 = __builtin_readcyclecounter();
  out[blockIdx.x * 64 + t] = cur;
  if (t == 0) cyc[blockIdx.x] = c1 - c0;
}
// LDS chain, matrices prefetched TWO steps ahead; H = 1: with the permlane row hand-off
template <int H>
__global__ __launch_bounds__(64) void chain_pf5_kernel(double* out, long long* cyc, int iters) {
  extern __shared__ double lds[];
  const int t = threadIdx.x, idx = t & 15;
  for (int e = t; e < 9 * 144; e += 64) lds[e] = 1e-3 * ((e * 37) % 101) - 0.05;
  __builtin_amdgcn_wave_barrier();
  double cur = 0.5 + 0.01 * t;
  const double ak = 0.125 * t;
  const double* base = lds + 12 * (idx % 12);
  double c1n[12], c2n[12];
#pragma unroll
  for (int i = 0; i < 12; ++i) {
    c1n[i] = base[i];
    c2n[i] = base[144 + i];
  }
  const long long c0 = __builtin_readcyclecounter();
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int k = 0; k < 9; ++k) {
      double c[12];
#pragma unroll
      for (int i = 0; i < 12; ++i) {
        c[i] = c1n[i];
        c1n[i] = c2n[i];
      }
      const double2* p = reinterpret_cast<const double2*>(base + 144 * ((k + 2) % 9));
#pragma unroll
      for (int i = 0; i < 6; ++i) {
        const double2 v = p[i];
        c2n[2 * i] = v.x;
        c2n[2 * i + 1] = v.y;
      }
      __builtin_amdgcn_sched_barrier(0);
      cur = mv12i(H ? to_odd(cur) : cur, c, -ak);
    }
  }
  const long long c1 = __builtin_readcyclecounter();
  out[blockIdx.x * 64 + t] = cur;
  if (t == 0) cyc[blockIdx.x] = c1 - c0;
}
// chain_pf4 with only DPP row 0 loading (the chain runs in row 0; other rows idle)
__global__ __launch_bounds__(64) void chain_row0_kernel(double* out, long long* cyc, int iters) {
  extern __shared__ double lds[];
  const int t = threadIdx.x, idx = t & 15;
  for (int e = t; e < 9 * 144; e += 64) lds[e] = 1e-3 * ((e * 37) % 101) - 0.05;
  __builtin_amdgcn_wave_barrier();
  double cur = 0.5 + 0.01 * t;
  const double ak = 0.125 * t;
  const double* base = lds + 12 * (idx % 12);
  double cn[12];
#pragma unroll
  for (int i = 0; i < 12; ++i) cn[i] = base[i];
  const long long c0 = __builtin_readcyclecounter();
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int k = 0; k < 9; ++k) {
      double c[12];
#pragma unroll
      for (int i = 0; i < 12; ++i) c[i] = cn[i];
      if (t < 16) {
        const double2* p = reinterpret_cast<const double2*>(base + 144 * ((k + 1) % 9));
#pragma unroll
        for (int i = 0; i < 6; ++i) {
          const double2 v = p[i];
          cn[2 * i] = v.x;
          cn[2 * i + 1] = v.y;
        }
      }
      __builtin_amdgcn_sched_barrier(0);
      cur = mv12i(cur, c, -ak);
    }
  }
  const long long c1 = __builtin_readcyclecounter();
  out[blockIdx.x * 64 + t] = cur;
  if (t == 0) cyc[blockIdx.x] = c1 - c0;
}
// rows split the 12-term dot product: x rotated per row, 3 DPP FMAs, cross-row all-reduce
__device__ __forceinline__ double rot_row(double x, int q) {  // row q lanes a <- lanes a + 4q
  const double r12 = __hiloint2double(__builtin_amdgcn_update_dpp(0, __double2hiint(x), 0x12C, 0xF, 0xF, false),
                                      __builtin_amdgcn_update_dpp(0, __double2loint(x), 0x12C, 0xF, 0xF, false));
  const double r8 = __hiloint2double(__builtin_amdgcn_update_dpp(0, __double2hiint(x), 0x128, 0xF, 0xF, false),
                                     __builtin_amdgcn_update_dpp(0, __double2loint(x), 0x128, 0xF, 0xF, false));
  const double r4 = __hiloint2double(__builtin_amdgcn_update_dpp(0, __double2hiint(x), 0x124, 0xF, 0xF, false),
                                     __builtin_amdgcn_update_dpp(0, __double2loint(x), 0x124, 0xF, 0xF, false));
  const double a = (q & 1) ? r12 : x;
  const double b = (q & 1) ? r4 : r8;
  return (q & 2) ? b : a;
}
__device__ __forceinline__ double rowsum(double p) {
  unsigned al = (unsigned)__double2loint(p), ah = (unsigned)__double2hiint(p);
  unsigned bl = al, bh = ah;
  asm volatile("s_nop 1\n\tv_permlane16_swap_b32 %0, %2\n\tv_permlane16_swap_b32 %1, %3"
               : "+v"(al), "+v"(ah), "+v"(bl), "+v"(bh));
  double s = __hiloint2double((int)ah, (int)al) + __hiloint2double((int)bh, (int)bl);
  al = (unsigned)__double2loint(s); ah = (unsigned)__double2hiint(s);
  bl = al; bh = ah;
  asm volatile("s_nop 1\n\tv_permlane32_swap_b32 %0, %2\n\tv_permlane32_swap_b32 %1, %3"
               : "+v"(al), "+v"(ah), "+v"(bl), "+v"(bh));
  return __hiloint2double((int)ah, (int)al) + __hiloint2double((int)bh, (int)bl);
}
__global__ __launch_bounds__(64) void chain_split_kernel(double* out, long long* cyc, int iters) {
  extern __shared__ double lds[];
  const int t = threadIdx.x, idx = t & 15, q = t >> 4;
  for (int e = t; e < 9 * 4 * 48; e += 64) lds[e] = 1e-3 * ((e * 37) % 101) - 0.05;
  __builtin_amdgcn_wave_barrier();
  double cur = 0.5 + 0.01 * t;
  const double ak = 0.125 * t;
  const double* base = lds + 48 * q + 4 * (idx % 12);  // [k][row q][lane][4]
  double cn[3];
#pragma unroll
  for (int i = 0; i < 3; ++i) cn[i] = base[i];
  const long long c0 = __builtin_readcyclecounter();
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int k = 0; k < 9; ++k) {
      const double c0_ = cn[0], c1_ = cn[1], c2_ = cn[2];
      const double* p = base + 192 * ((k + 1) % 9);
#pragma unroll
      for (int i = 0; i < 3; ++i) cn[i] = p[i];
      __builtin_amdgcn_sched_barrier(0);
      const double xr = rot_row(cur, q);
      double a0 = 0.0, a1 = 0.0, a2 = 0.0;
      asm("s_nop 4\n\t"
          "v_fmac_f64_dpp %[a0], %[x], %[c0] row_newbcast:0 row_mask:0xf bank_mask:0xf\n\t"
          "v_fmac_f64_dpp %[a1], %[x], %[c1] row_newbcast:1 row_mask:0xf bank_mask:0xf\n\t"
          "v_fmac_f64_dpp %[a2], %[x], %[c2] row_newbcast:2 row_mask:0xf bank_mask:0xf"
          : [a0] "+v"(a0), [a1] "+v"(a1), [a2] "+v"(a2)
          : [x] "v"(xr), [c0] "v"(c0_), [c1] "v"(c1_), [c2] "v"(c2_));
      cur = rowsum((a0 + a1) + a2) - ak;
    }
  }
  const long long c1 = __builtin_readcyclecounter();
  out[blockIdx.x * 64 + t] = cur;
  if (t == 0) cyc[blockIdx.x] = c1 - c0;
}

// rows split the 12-term dot product with no rotation: 12 DPP FMAs, each writing only the row that
// owns its column (row q: columns 3q..3q+2 = lanes 4q..4q+2), then the cross-row all-reduce.
// Each lane loads 3 coefficients instead of 12 (4x less LDS traffic).
#define FMR(A, M, L, RM) "v_fmac_f64_dpp " A ", %[x], " M " row_newbcast:" #L " row_mask:" #RM " bank_mask:0xf\n\t"
__device__ __forceinline__ double mvq(double x, double m0, double m1, double m2, double init) {
  double a0 = init, a1 = 0.0, a2 = 0.0;
  asm("s_nop 4\n\t"
      FMR("%[a1]", "%[c1]", 1, 0x1) FMR("%[a2]", "%[c2]", 2, 0x1) FMR("%[a0]", "%[c0]", 0, 0x1)
      FMR("%[a1]", "%[c1]", 5, 0x2) FMR("%[a2]", "%[c2]", 6, 0x2) FMR("%[a0]", "%[c0]", 4, 0x2)
      FMR("%[a1]", "%[c1]", 9, 0x4) FMR("%[a2]", "%[c2]", 10, 0x4) FMR("%[a0]", "%[c0]", 8, 0x4)
      FMR("%[a1]", "%[c1]", 13, 0x8) FMR("%[a2]", "%[c2]", 14, 0x8) FMR("%[a0]", "%[c0]", 12, 0x8)
      : [a0] "+v"(a0), [a1] "+v"(a1), [a2] "+v"(a2)
      : [x] "v"(x), [c0] "v"(m0), [c1] "v"(m1), [c2] "v"(m2));
  return (a1 + a2) + a0;
}
__global__ __launch_bounds__(64) void chain_mask_kernel(double* out, long long* cyc, int iters) {
  extern __shared__ double lds[];
  const int t = threadIdx.x, idx = t & 15, q = t >> 4;
  for (int e = t; e < 9 * 4 * 48; e += 64) lds[e] = 1e-3 * ((e * 37) % 101) - 0.05;
  __builtin_amdgcn_wave_barrier();
  double cur = 0.5 + 0.01 * t;
  const double ak = q == 0 ? 0.125 * t : 0.0;
  const double* base = lds + 48 * q + 4 * (idx % 12);  // [k][row q][lane][4]
  double cn[3];
#pragma unroll
  for (int i = 0; i < 3; ++i) cn[i] = base[i];
  const long long c0 = __builtin_readcyclecounter();
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int k = 0; k < 9; ++k) {
      const double c0_ = cn[0], c1_ = cn[1], c2_ = cn[2];
      const double* p = base + 192 * ((k + 1) % 9);
#pragma unroll
      for (int i = 0; i < 3; ++i) cn[i] = p[i];
      __builtin_amdgcn_sched_barrier(0);
      cur = rowsum(mvq(cur, c0_, c1_, c2_, -ak));
    }
  }
  const long long c1 = __builtin_readcyclecounter();
  out[blockIdx.x * 64 + t] = cur;
  if (t == 0) cyc[blockIdx.x] = c1 - c0;
}
// as chain_mask with the matrices in registers (compute floor)
__global__ __launch_bounds__(64) void chain_mask_reg_kernel(double* out, long long* cyc, int iters) {
  const int t = threadIdx.x, q = t >> 4;
  double m[9][3];
#pragma unroll
  for (int k = 0; k < 9; ++k)
#pragma unroll
    for (int i = 0; i < 3; ++i) m[k][i] = 1e-3 * (((k * 12 + i) * 37 + t) % 101) - 0.05;
  double cur = 0.5 + 0.01 * t;
  const double ak = q == 0 ? 0.125 * t : 0.0;
  const long long c0 = __builtin_readcyclecounter();
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int k = 0; k < 9; ++k) cur = rowsum(mvq(cur, m[k][0], m[k][1], m[k][2], -ak));
  }
  const long long c1 = __builtin_readcyclecounter();
  out[blockIdx.x * 64 + t] = cur;
  if (t == 0) cyc[blockIdx.x] = c1 - c0;
}

// dependent v_fma_f64 chain (ILP 1) or 8 independent chains (ILP 8)
template <int ILP>
__global__ __launch_bounds__(64) void fma_kernel(double* out, long long* cyc, int iters) {
  extern __shared__ double lds[];
  (void)lds;
  const int t = threadIdx.x;
  double a[ILP];
#pragma unroll
  for (int j = 0; j < ILP; ++j) a[j] = 1.0 + 1e-3 * (t + j);
  const double b = 0.999999, c = 1e-9;
  const long long c0 = __builtin_readcyclecounter();
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int u = 0; u < 16; ++u)
#pragma unroll
      for (int j = 0; j < ILP; ++j) a[j] = __builtin_fma(a[j], b, c);
  }
  const long long c1 = __builtin_readcyclecounter();
  double s = 0.0;
#pragma unroll
  for (int j = 0; j < ILP; ++j) s += a[j];
  out[blockIdx.x * 64 + t] = s;
  if (t == 0) cyc[blockIdx.x] = c1 - c0;
}

// dependent v_fmac_f64_dpp (row_newbcast) chain, ILP 1 or 4
template <int ILP>
__global__ __launch_bounds__(64) void dppfma_kernel(double* out, long long* cyc, int iters) {
  extern __shared__ double lds[];
  (void)lds;
  const int t = threadIdx.x;
  double a[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) a[j] = 1.0 + 1e-3 * (t + j);
  const double x = 1e-9 * t, m = 0.5;
  const long long c0 = __builtin_readcyclecounter();
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int u = 0; u < 16; ++u) {
      if constexpr (ILP == 1) {
        asm volatile("v_fmac_f64_dpp %0, %1, %2 row_newbcast:3 row_mask:0xf bank_mask:0xf" : "+v"(a[0]) : "v"(x), "v"(m));
      } else {
        asm volatile(
            "v_fmac_f64_dpp %0, %4, %5 row_newbcast:3 row_mask:0xf bank_mask:0xf\n\t"
            "v_fmac_f64_dpp %1, %4, %5 row_newbcast:3 row_mask:0xf bank_mask:0xf\n\t"
            "v_fmac_f64_dpp %2, %4, %5 row_newbcast:3 row_mask:0xf bank_mask:0xf\n\t"
            "v_fmac_f64_dpp %3, %4, %5 row_newbcast:3 row_mask:0xf bank_mask:0xf"
            : "+v"(a[0]), "+v"(a[1]), "+v"(a[2]), "+v"(a[3])
            : "v"(x), "v"(m));
      }
    }
  }
  const long long c1 = __builtin_readcyclecounter();
  out[blockIdx.x * 64 + t] = a[0] + a[1] + a[2] + a[3];
  if (t == 0) cyc[blockIdx.x] = c1 - c0;
}

typedef void (*KFn)(double*, long long*, int);

static void run(const char* name, KFn fn, int waves_per_cu, int iters, double ops_per_iter) {
  int cus = 0;
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  const int blocks = cus * waves_per_cu * 4;  // 4 generations of resident waves
  size_t lds = (160 * 1024) / waves_per_cu;
  lds = lds / 16 * 16;
  if (lds < 9 * 192 * 8) lds = 9 * 192 * 8;
  double* out;
  long long* cyc;
  CK(hipMalloc(&out, sizeof(double) * 64 * blocks));
  CK(hipMalloc(&cyc, sizeof(long long) * blocks));
  CK(hipFuncSetAttribute((const void*)fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  hipLaunchKernelGGL(fn, dim3(blocks), dim3(64), lds, 0, out, cyc, iters);
  CK(hipDeviceSynchronize());
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  CK(hipEventRecord(e0, 0));
  hipLaunchKernelGGL(fn, dim3(blocks), dim3(64), lds, 0, out, cyc, iters);
  CK(hipEventRecord(e1, 0));
  CK(hipDeviceSynchronize());
  float ms = 0;
  CK(hipEventElapsedTime(&ms, e0, e1));
  long long* h = (long long*)malloc(sizeof(long long) * blocks);
  CK(hipMemcpy(h, cyc, sizeof(long long) * blocks, hipMemcpyDeviceToHost));
  double avg = 0;
  for (int i = 0; i < blocks; ++i) avg += (double)h[i];
  avg /= blocks;
  const double wave_ops = (double)blocks * iters * ops_per_iter;
  printf("%-14s W/CU=%2d  kernel %.3f ms  per-wave cycles/op %.2f  chip ns/op/wave-slot %.4f  ops/s %.3e\n", name,
         waves_per_cu, ms, avg / (iters * ops_per_iter), ms * 1e6 / wave_ops, wave_ops / (ms * 1e-3));
  free(h);
  CK(hipFree(out));
  CK(hipFree(cyc));
}

int main() {
  const int W[] = {4, 8, 12, 16};
  if (getenv("MB_MASK_ONLY")) {
    for (int w : W) run("chain_pf3", chain_pf3_kernel, w, 200, 9);
    for (int w : W) run("chain_reg2", chain_reg2_kernel, w, 200, 9);
    for (int w : W) run("chain_reg3", chain_reg3_kernel, w, 200, 9);
    for (int w : W) run("chain_pf4", chain_pf4_kernel, w, 200, 9);
    for (int w : W) run("chain_pf5", chain_pf5_kernel<0>, w, 200, 9);
    for (int w : W) run("chain_row0", chain_row0_kernel, w, 200, 9);
    for (int w : W) run("chain_pf5_hand", chain_pf5_kernel<1>, w, 200, 9);
    return 0;
  }
  for (int w : W) run("chain(step)", chain_kernel, w, 200, 9);
  for (int w : W) run("chain_reg", chain_reg_kernel, w, 200, 9);
  for (int w : W) run("chain_pf", chain_pf_kernel, w, 200, 9);
  for (int w : W) run("chain_pf2", chain_pf2_kernel, w, 200, 9);
  for (int w : W) run("chain_reg2", chain_reg2_kernel, w, 200, 9);
  for (int w : W) run("chain_pf3", chain_pf3_kernel, w, 200, 9);
  for (int w : W) run("chain_split", chain_split_kernel, w, 200, 9);
  for (int w : W) run("fma dep", fma_kernel<1>, w, 2000, 16);
  for (int w : W) run("fma ilp8", fma_kernel<8>, w, 500, 128);
  for (int w : W) run("dppfma dep", dppfma_kernel<1>, w, 2000, 16);
  for (int w : W) run("dppfma ilp4", dppfma_kernel<4>, w, 500, 64);
  return 0;
}
