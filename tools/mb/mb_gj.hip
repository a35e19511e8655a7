// Microbenchmark: cycles of the factorization's building blocks on one wave (gfx950):
// the in-register 12x12 Gauss-Jordan inverse (gj_inverse12) and a dependent chain of
// v_mfma_f64_16x16x4f64 (the Riccati products).  4 waves per CU (one per SIMD), like the solver.
//   hipcc -O3 --offload-arch=gfx950 -I go1-qp-mpc-controller_amd/csrc tools/mb/mb_gj.hip -o tools/mb/mb_gj
#include <hip/hip_runtime.h>
#include <stdio.h>
#include "mpcqp_wave_common.h"
using namespace mpcqp::wv;

__global__ __launch_bounds__(64) void gj_kernel(double* out, long long* cyc, int iters) {
  const int j = threadIdx.x & 15, grp = threadIdx.x >> 4;
  mf4 g;
  for (int v = 0; v < 4; ++v) {  // SPD: diagonally dominant symmetric
    const int u = 4 * v + grp;
    double x = (u == j) ? 20.0 + u : 1.0 / (1.0 + u + j);
    if (u >= 12 || j >= 12) x = (u == j) ? 1.0 : 0.0;
    g[v] = x;
  }
  const long long c0 = __builtin_readcyclecounter();
  for (int it = 0; it < iters; ++it) gj_inverse12(g);
  const long long c1 = __builtin_readcyclecounter();
  out[blockIdx.x * 64 + threadIdx.x] = g[0] + g[1] + g[2] + g[3];
  if (threadIdx.x == 0) cyc[blockIdx.x] = c1 - c0;
}
__global__ __launch_bounds__(64) void gj2_kernel(double* out, long long* cyc, int iters) {
  const int j = threadIdx.x & 15, grp = threadIdx.x >> 4;
  mf4 g;
  for (int v = 0; v < 4; ++v) {
    const int u = 4 * v + grp;
    double x = (u == j) ? 20.0 + u : 1.0 / (1.0 + u + j);
    if (u >= 12 || j >= 12) x = (u == j) ? 1.0 : 0.0;
    g[v] = x;
  }
  const long long c0 = __builtin_readcyclecounter();
  for (int it = 0; it < iters; ++it) gj_inverse12(g);
  const long long c1 = __builtin_readcyclecounter();
  out[blockIdx.x * 64 + threadIdx.x] = g[0] + g[1] + g[2] + g[3];
  if (threadIdx.x == 0) cyc[blockIdx.x] = c1 - c0;
}
// one inverse each way: out[0..255] scalar GJ, out[256..511] 2x2-block GJ (D layout, 4 regs)
__global__ void gj_check(double* out) {
  const int j = threadIdx.x & 15, grp = threadIdx.x >> 4;
  mf4 g, h;
  for (int v = 0; v < 4; ++v) {
    const int u = 4 * v + grp;
    double x = (u == j) ? 3.0 + 0.5 * u : 0.3 / (1.0 + u + j) + ((u + j) % 3 == 0 ? 0.2 : 0.0);
    if (u >= 12 || j >= 12) x = (u == j) ? 1.0 : 0.0;
    g[v] = x;
    h[v] = x;
  }
  gj_inverse12(g);
  gj_inverse12(h);
  for (int v = 0; v < 4; ++v) {
    out[64 * v + threadIdx.x] = g[v];
    out[256 + 64 * v + threadIdx.x] = h[v];
  }
}
__global__ __launch_bounds__(64) void mfma_kernel(double* out, long long* cyc, int iters) {
  mf4 a, x, c = {0.0, 0.0, 0.0, 0.0};
  for (int v = 0; v < 4; ++v) {
    a[v] = 1e-3 * (threadIdx.x + v);
    x[v] = 1e-3 * (threadIdx.x - v);
  }
  const long long c0 = __builtin_readcyclecounter();
  for (int it = 0; it < iters; ++it) c = mfma_chain<0, 4>(a, x, c);  // 4 dependent MFMAs
  const long long c1 = __builtin_readcyclecounter();
  out[blockIdx.x * 64 + threadIdx.x] = c[0] + c[1] + c[2] + c[3];
  if (threadIdx.x == 0) cyc[blockIdx.x] = c1 - c0;
}

static void run(const char* name, void (*fn)(double*, long long*, int), int iters, double per) {
  int cus = 0;
  hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
  const int blocks = cus * 4;
  double* out;
  long long* cyc;
  hipMalloc(&out, sizeof(double) * 64 * blocks);
  hipMalloc(&cyc, sizeof(long long) * blocks);
  hipLaunchKernelGGL(fn, dim3(blocks), dim3(64), 0, 0, out, cyc, iters);
  hipDeviceSynchronize();
  hipLaunchKernelGGL(fn, dim3(blocks), dim3(64), 0, 0, out, cyc, iters);
  hipDeviceSynchronize();
  long long h[4096];
  hipMemcpy(h, cyc, sizeof(long long) * blocks, hipMemcpyDeviceToHost);
  double avg = 0;
  for (int i = 0; i < blocks; ++i) avg += (double)h[i];
  avg /= blocks;
  printf("%-12s cycles per %s: %.1f\n", name, name[0] == 'g' ? "12x12 inverse" : "MFMA (dependent)", avg / (iters * per));
  hipFree(out);
  hipFree(cyc);
}
int main() {
  double* d;
  hipMalloc(&d, 512 * sizeof(double));
  hipLaunchKernelGGL(gj_check, dim3(1), dim3(64), 0, 0, d);
  double hb[512];
  hipMemcpy(hb, d, sizeof(hb), hipMemcpyDeviceToHost);
  double md = 0, mx = 0;
  for (int i = 0; i < 256; ++i) {
    md = fmax(md, fabs(hb[i] - hb[256 + i]));
    mx = fmax(mx, fabs(hb[i]));
  }
  printf("2x2-block vs scalar Gauss-Jordan: max |diff| %.3e (max |entry| %.3e)\n", md, mx);
  run("gj_inverse12", gj_kernel, 200, 1);
  run("mfma_chain", mfma_kernel, 200, 4);
  return 0;
}
