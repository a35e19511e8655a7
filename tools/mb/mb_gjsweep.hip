// Microbenchmark: cycles of one factorization's Q = I - S^-1 at N = 10 (60x60 SPD S), one wave per
// SIMD with the solver's LDS footprint, for the two forms in mpcqp_schur.h: the in-register scalar
// sweep (schur_gj_valu) and the blocked sweep on the matrix cores (schur_gj_mfma).  S - I = V V' with a seeded V (60 x 12, like L'CL's rank 12
// per step pair), scaled so that max S_ii ~ 1e3.  Prints median cycles per call and the largest
// difference of each form's Q from the scalar sweep's, and the MFMA form's internal marks (60: tiles
// made, 61: first pivot tile swept, then per step 62: row k transposed, 63: next pivot tile in rows,
// 64: step done).  -DMPCQP_GJ_DBG_NOTASK / -DMPCQP_GJ_DBG_NOROWS time it without the MFMA tasks /
// without the pivot sweeps after the first (results then wrong; timing only).
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 -fno-strict-aliasing -DMPCQP_GJ_MFMA=1 \
//     -mllvm -amdgpu-mfma-vgpr-form -I go1-qp-mpc-controller_amd/csrc tools/mb/mb_gjsweep.hip -o tools/mb/mb_gjsweep
#include <hip/hip_runtime.h>
#include <stdio.h>

#include <algorithm>
#include <vector>

#include "mpcqp_schur.h"
using namespace mpcqp;
using namespace mpcqp::wv;

constexpr int NH = 10, NI = 6 * NH, QS = SchurCfg<NH>::QS;

__device__ double vfun(int i, int e, unsigned seed) {  // in [-1, 1)
  unsigned h = (unsigned)(i * 131 + e * 7919) ^ seed;
  h ^= h >> 13;
  h *= 0x5bd1e995u;
  h ^= h >> 15;
  return (double)(h & 0xFFFFFF) / 8388608.0 - 1.0;
}

template <int MODE>
__global__ __launch_bounds__(64) void k(double* qout, long long* cyc, int iters, long long* marks) {
  extern __shared__ double lds[];
  auto& F = *reinterpret_cast<SchurLds<NH>*>(lds);
  int t = threadIdx.x;
  asm volatile("" : "+v"(t));
  const unsigned seed = 977u * blockIdx.x + 1u;
  double vt[12];
#pragma unroll
  for (int e = 0; e < 12; ++e) vt[e] = t < NI ? 9.0 * vfun(t, e, seed) : 0.0;
  long long tot = 0, st[12] = {0};
  int ns = 0;
  for (int it = 0; it < iters; ++it) {
    ns = 0;
    double S[64];
#pragma unroll
    for (int m = 0; m < 64; ++m) {
      double s = 0.0;
      if (m < NI)
#pragma unroll
        for (int e = 0; e < 12; ++e) s += vt[e] * 9.0 * vfun(m, e, seed);
      S[m] = t < NI ? s : 0.0;
    }
    wave_sync();
    __builtin_amdgcn_sched_barrier(0);
    const long long c0 = __builtin_readcyclecounter();
    __builtin_amdgcn_sched_barrier(0);
    if constexpr (MODE == 0) schur_gj_valu<NH>(S, F, t, [] {});
    if constexpr (MODE == 1)
      schur_gj_mfma<NH>(S, F, t, [] {}, [&](int) {
        if (ns < 12) st[ns] = __builtin_readcyclecounter() - c0;
        ++ns;
      });
    __builtin_amdgcn_sched_barrier(0);
    const long long c1 = __builtin_readcyclecounter();
    __builtin_amdgcn_sched_barrier(0);
    tot += c1 - c0;
  }
  wave_sync();
  for (int e = t; e < NI * QS; e += 64) qout[(size_t)blockIdx.x * NI * QS + e] = F.Q[e];
  if (t == 0) {
    cyc[blockIdx.x] = tot / iters;
    for (int e = 0; e < 12; ++e) marks[blockIdx.x * 12 + e] = e < ns ? st[e] : -1;
  }
}

int main() {
  const int blocks = 1024, iters = 4;
  const size_t qn = (size_t)blocks * NI * QS;
  double* d_q;
  long long* d_c;
  hipMalloc(&d_q, sizeof(double) * qn * 3);
  hipMalloc(&d_c, sizeof(long long) * blocks * 3);
  const size_t lb = sizeof(SchurLds<NH>) > 40880 ? sizeof(SchurLds<NH>) : 40880;  // the solver's footprint
  void (*ks[2])(double*, long long*, int, long long*) = {k<0>, k<1>};
  long long* d_m;
  hipMalloc(&d_m, sizeof(long long) * blocks * 12 * 3);
  const char* names[2] = {"scalar sweep (schur_gj_valu)", "matrix cores (schur_gj_mfma)"};
  std::vector<double> q(qn * 3);
  for (int m = 0; m < 2; ++m) {
    hipFuncSetAttribute((const void*)ks[m], hipFuncAttributeMaxDynamicSharedMemorySize, (int)lb);
    hipLaunchKernelGGL(ks[m], dim3(blocks), dim3(64), lb, 0, d_q + qn * m, d_c + blocks * m, 1, d_m + blocks * 12 * m);
    hipLaunchKernelGGL(ks[m], dim3(blocks), dim3(64), lb, 0, d_q + qn * m, d_c + blocks * m, iters, d_m + blocks * 12 * m);
  }
  if (hipDeviceSynchronize() != hipSuccess) {
    printf("kernel failed\n");
    return 1;
  }
  std::vector<long long> c(blocks * 3);
  hipMemcpy(c.data(), d_c, sizeof(long long) * blocks * 3, hipMemcpyDeviceToHost);
  hipMemcpy(q.data(), d_q, sizeof(double) * qn * 3, hipMemcpyDeviceToHost);
  for (int m = 0; m < 2; ++m) {
    std::vector<long long> v(c.begin() + blocks * m, c.begin() + blocks * (m + 1));
    std::sort(v.begin(), v.end());
    double dmax = 0.0, qmax = 0.0;
    for (size_t e = 0; e < qn; ++e) {
      dmax = std::max(dmax, std::abs(q[qn * m + e] - q[e]));
      qmax = std::max(qmax, std::abs(q[e]));
    }
    printf("%-44s median %7lld cycles per factorization (p10 %lld, p90 %lld); max |Q - Q_scalar| %.3e (max |Q| %.3e)\n",
           names[m], v[blocks / 2], v[blocks / 10], v[blocks * 9 / 10], dmax, qmax);
  }
  std::vector<long long> mk(blocks * 12);
  hipMemcpy(mk.data(), d_m + blocks * 12 * 1, sizeof(long long) * blocks * 12, hipMemcpyDeviceToHost);
  printf("MFMA form, cycles from the call to each internal mark (median; last iteration):");
  for (int e = 0; e < 12; ++e) {
    std::vector<long long> v;
    for (int b = 0; b < blocks; ++b)
      if (mk[b * 12 + e] >= 0) v.push_back(mk[b * 12 + e]);
    if (v.empty()) break;
    std::sort(v.begin(), v.end());
    printf(" %lld", v[v.size() / 2]);
  }
  printf("\n");
  return 0;
}
