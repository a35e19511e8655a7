// Checks the operand / result lane layouts assumed for v_mfma_f64_16x16x4f64 and the 4x4
// (lane group, register) transpose built from v_permlane16_swap / v_permlane32_swap:
//   A[i][k]: lane i + 16 k;  B[k][j]: lane j + 16 k;  D[i][j]: lane j + 16 (i / 4), register i % 4.
//   hipcc -O3 --offload-arch=gfx950 tools/mb/mfma_f64_layout.hip -o tools/mb/mfma_f64_layout
#include <hip/hip_runtime.h>
#include <stdio.h>

typedef double d4 __attribute__((ext_vector_type(4)));

__device__ inline void swap16(double& x, double& y) {  // x.odd groups <-> y.even groups
  unsigned xl = __double2loint(x), xh = __double2hiint(x), yl = __double2loint(y), yh = __double2hiint(y);
  asm volatile("s_nop 1\n\tv_permlane16_swap_b32 %0, %2\n\tv_permlane16_swap_b32 %1, %3"
               : "+v"(xl), "+v"(xh), "+v"(yl), "+v"(yh));
  x = __hiloint2double(xh, xl);
  y = __hiloint2double(yh, yl);
}
__device__ inline void swap32(double& x, double& y) {  // x.groups 2,3 <-> y.groups 0,1
  unsigned xl = __double2loint(x), xh = __double2hiint(x), yl = __double2loint(y), yh = __double2hiint(y);
  asm volatile("s_nop 1\n\tv_permlane32_swap_b32 %0, %2\n\tv_permlane32_swap_b32 %1, %3"
               : "+v"(xl), "+v"(xh), "+v"(yl), "+v"(yh));
  x = __hiloint2double(xh, xl);
  y = __hiloint2double(yh, yl);
}

__global__ void k(double* out) {
  const int l = threadIdx.x;
  const int i = l & 15, kk = l >> 4;
  // A[i][k] = 100 i + k + 1 ; B = [I4 | 0] (B[k][j] = j == k) ; C = 0  ->  D[i][j] = A[i][j] (j < 4)
  const double a = 100.0 * i + kk + 1;
  const double b = (i == kk) ? 1.0 : 0.0;
  d4 c = {0.0, 0.0, 0.0, 0.0};
  d4 d = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, 0, 0, 0);
  for (int v = 0; v < 4; ++v) out[64 * v + l] = d[v];
  // transpose of (group, register): t[g'] at group g = d[g] at group g'
  double t0 = d[0], t1 = d[1], t2 = d[2], t3 = d[3];
  swap16(t0, t1);
  swap16(t2, t3);
  swap32(t0, t2);
  swap32(t1, t3);
  out[256 + l] = t0;
  out[320 + l] = t1;
  out[384 + l] = t2;
  out[448 + l] = t3;
}

int main() {
  double* d;
  hipMalloc(&d, 512 * sizeof(double));
  hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d);
  double h[512];
  hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
  int bad = 0;
  for (int l = 0; l < 64; ++l)
    for (int v = 0; v < 4; ++v) {
      const int j = l & 15, ii = 4 * (l >> 4) + v;
      const double want = j < 4 ? 100.0 * ii + j + 1 : 0.0;
      if (h[64 * v + l] != want) {
        if (bad < 8) printf("D mismatch lane %d reg %d: got %g want %g\n", l, v, h[64 * v + l], want);
        ++bad;
      }
    }
  printf("D layout: %s (%d mismatches)\n", bad ? "WRONG" : "ok", bad);
  int badt = 0;
  for (int l = 0; l < 64; ++l)
    for (int r = 0; r < 4; ++r) {
      const int g = l >> 4, j = l & 15;
      // t_r at group g should be d[g] at group r: element D[4 r + g][j]
      const double want = h[64 * g + (16 * r + j)];
      if (h[256 + 64 * r + l] != want) {
        if (badt < 8) printf("T mismatch lane %d reg %d: got %g want %g\n", l, r, h[256 + 64 * r + l], want);
        ++badt;
      }
    }
  printf("transpose: %s (%d mismatches)\n", badt ? "WRONG" : "ok", badt);
  return 0;
}
