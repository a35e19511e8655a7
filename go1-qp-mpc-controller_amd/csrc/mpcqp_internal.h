// mpcqp_internal.h — shared between the kernels and the C-ABI layer (not installed).
#pragma once
#include <hip/hip_runtime.h>

#include "../../include/mpcqp.h"

#define MPCQP_TRACE_LEN 64  // termination-check records kept per instance by the debug trace

namespace mpcqp {

// Register-tile geometry: the (padded) 128x128 KKT inverse is spread over a grid of threads,
// each owning a SOLVE_BR x BC tile; the 16 threads of a tile row are 16 consecutive lanes.
constexpr int NP = 128;  // padded problem size (12N <= 120 for N <= 10)
constexpr int BC = 8;    // columns per thread (16 x 8 = 128)
#ifndef SOLVE_BR
#define SOLVE_BR 4       // rows per thread: 4 -> 512 threads (8 waves) per instance
#endif

struct LaunchArgs {
  const double* recs;
  int batch;
  mpcqp_result* results;
  double* solution;
  double* work;
  double* trace;
  int trace_cap;
  int grid;
  void* stream;
  mpcqp_params p;
};

hipError_t launch_solve_any(const LaunchArgs& a);
hipError_t launch_build_any(const LaunchArgs& a, double* P, double* q, double* l, double* u);
hipError_t occupancy_any(int horizon, int* blocks);
int solve_threads();

}  // namespace mpcqp
