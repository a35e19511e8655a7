// mpcqp_capi.cpp — extern "C" boundary (include/mpcqp.h) over the HIP kernels.
//
// Replaces, per batch of robots, the OsqpEigen::Solver lifecycle of the reference
// (A1RobotControl.h:67, A1RobotControl.cpp:522-555) and ConvexMpc's construction
// (ConvexMpc.cpp:7-68).  No exception crosses this boundary.
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <new>

#include "../../include/mpcqp.h"
#include "../../include/mpcqp_debug.h"
#include "mpcqp_internal.h"

struct mpcqp_handle {
  mpcqp_params p;
  int device = 0;
  int slots = 0;             // resident workgroups per device (occupancy x CUs), informational
  int cus = 0;               // compute units of the device
  double* work = nullptr;    // per-robot 12N x 16*ceil(12N/16) binary64 workspace (scaled Hessian)
  size_t work_cap = 0;       // instances the workspace can hold
  size_t work_per = 0;       // doubles per instance the workspace was sized for
  int* fb = nullptr;         // wave path: Schur -> Riccati hand-off counters, [4] ints per batch part
  // The wave path splits a batch into parts solved concurrently on internal streams (forked from
  // and joined to the caller's stream by events): one part's scale_kernel runs beside another
  // part's wave_kernel and the parts' dispatch tails interleave (split_parts; tools/split_exp.py,
  // profiles/r05/split).  Results are bitwise those of one launch.
  static constexpr int KMAX = 8;
  int split = 0;             // parts per solve: 0 = auto (split_parts), else MPCQP_SPLIT / mpcqp_set_split
  int fb_parts = 1;          // parts of the last solve (hand-off counters to sum)
  int split_w[KMAX] = {};    // relative part sizes (MPCQP_SPLIT_W="w0,w1,..."); all 0 = equal parts
  // sub[i] / ev_join[i] serve part i >= 1 (part 0 runs on the caller's stream), created lazily: only
  // the parts - 1 streams a split of that size uses, the first time it runs or at mpcqp_reserve
  hipStream_t sub[KMAX] = {};
  hipEvent_t ev_fork = nullptr;
  hipEvent_t ev_join[KMAX] = {};
  int path = 0;              // 0 auto (= 3), 3 Riccati wave; debug library only: 1 dense K^-1, 2 Riccati workgroup
  // host wrapper: device buffers, a private stream and two pinned staging chunks
  hipStream_t hstream = nullptr;
  char* pin[2] = {nullptr, nullptr};
  hipEvent_t pin_ev[2] = {nullptr, nullptr};
  bool pin_busy[2] = {false, false};
  double* d_recs = nullptr;
  mpcqp_result* d_res = nullptr;
  double* d_sol = nullptr;
  size_t cap = 0;
  double* d_bal_recs = nullptr;  // balance host wrapper staging
  mpcqp_result* d_bal_res = nullptr;
  size_t bal_cap = 0;
  char err[256] = {0};
};

namespace {

// Makes the handle's device current for one entry point and restores the caller's current device
// on every return path (a multi-GPU caller such as torch keeps its own device selection).
struct DeviceGuard {
  int prev = -1;
  hipError_t err;
  explicit DeviceGuard(int device) {
    if (hipGetDevice(&prev) != hipSuccess) prev = -1;
    err = hipSetDevice(device);
  }
  ~DeviceGuard() {
    if (prev >= 0) (void)hipSetDevice(prev);
  }
  DeviceGuard(const DeviceGuard&) = delete;
  DeviceGuard& operator=(const DeviceGuard&) = delete;
};

int set_hip_error(mpcqp_handle* h, hipError_t e, const char* where) {
  if (h) snprintf(h->err, sizeof(h->err), "%s: %s", where, hipGetErrorString(e));
  return MPCQP_ERR_HIP;
}

bool params_valid(const mpcqp_params* p) {
  if (!p) return false;
  if (p->horizon < 1 || p->horizon > MPCQP_MAX_HORIZON) return false;
  if (p->max_iter < 1 || p->scaling < 0 || p->check_termination < 0) return false;
  if (p->adaptive_rho && p->adaptive_rho_interval <= 0) return false;  // wall-clock interval unsupported
  if (!(p->rho > 0) || !(p->sigma > 0) || !(p->alpha > 0 && p->alpha < 2)) return false;
  if (!(p->eps_abs >= 0) || !(p->eps_rel >= 0)) return false;
  if (p->scaled_termination != 0) return false;  // reference uses the default (0)
  for (int i = 0; i < MPCQP_STATE_DIM; ++i)
    if (!isfinite(p->q_weights[i])) return false;
  for (int i = 0; i < MPCQP_NUM_DOF; ++i)
    if (!isfinite(p->r_weights[i])) return false;
  return true;
}

// 3 = scale_kernel + wave_kernel (the product path); 1, 2 = cross-check solvers of the debug build
int effective_path(const mpcqp_handle* h) { return h->path != 0 ? h->path : 3; }
size_t work_per_instance(const mpcqp_handle* h) {
  switch (effective_path(h)) {
#ifdef MPCQP_DEBUG_PATHS
    case 1: return mpcqp::workspace_doubles(h->p.horizon);
    case 2: return mpcqp::riccati_workspace_doubles(h->p.horizon);
#endif
    default: return mpcqp::scale_image_doubles(h->p.horizon);  // scale_kernel -> wave_kernel hand-off
  }
}
hipError_t occupancy_for(const mpcqp_handle* h, int* per_cu) {
  switch (effective_path(h)) {
#ifdef MPCQP_DEBUG_PATHS
    case 1: return mpcqp::occupancy_any(h->p.horizon, per_cu);
    case 2: return mpcqp::occupancy_riccati_any(h->p.horizon, per_cu);
#endif
    default: return mpcqp::occupancy_wave_any(h->p, per_cu);
  }
}
// (Re)size the per-instance workspace for `batch` instances of the current path.
hipError_t ensure_workspace(mpcqp_handle* h, int32_t batch, void* stream) {
  const size_t per = work_per_instance(h);
  if (per == 0) return hipSuccess;
  if ((size_t)batch <= h->work_cap && per <= h->work_per) return hipSuccess;
  hipError_t e = hipStreamSynchronize((hipStream_t)stream);
  if (e == hipSuccess) e = hipFree(h->work);
  if (e == hipSuccess) e = hipFree(h->fb);
  h->work = nullptr;
  h->fb = nullptr;
  const size_t cap = (size_t)batch > h->work_cap ? (size_t)batch : h->work_cap;
  h->work_cap = 0;
  h->work_per = 0;
  if (e == hipSuccess) e = hipMalloc(&h->work, sizeof(double) * per * cap);
  if (e == hipSuccess) e = hipMalloc(&h->fb, sizeof(int) * 4 * mpcqp_handle::KMAX);
  if (e == hipSuccess) e = hipMemset(h->fb, 0, sizeof(int) * 4 * mpcqp_handle::KMAX);
  if (e == hipSuccess) {
    h->work_cap = cap;
    h->work_per = per;
  }
  return e;
}

// Parts a wave-path solve of `batch` robots is split into.  Auto: three from 3072 robots, two from
// 2048 (measured, tools/split_exp.py, profiles/r05/split: three parts C2 1.630 -> 1.582 ms, C5
// 3.186 -> 2.971 ms, C4 5.44 -> 5.26 ms, C3's 8192-robot shard and 65536 robots unchanged; four
// parts are slower everywhere: the caller's stream plus three internal ones already fill the
// process's four hardware queues, and a fifth stream shares one in order).
int split_parts(const mpcqp_handle* h, int32_t batch) {
  int k = h->split > 0 ? h->split : (batch >= 3072 ? 3 : batch >= 2048 ? 2 : 1);
  if (k > mpcqp_handle::KMAX) k = mpcqp_handle::KMAX;
  if (k > batch) k = batch;
  return k < 1 ? 1 : k;
}

// The internal streams and events of a split into `parts` parts: parts 1 .. parts-1 each get a stream
// and a join event the first time a split of that size runs (or at mpcqp_reserve, for callers that
// capture the solve into a graph).  Nothing is created for an unsplit solve, so a process's hardware
// queues (GPU_MAX_HW_QUEUES = 4) are not filled with streams it never uses: a C3 rank holds the
// caller's stream, RCCL's and the split's two.
hipError_t ensure_split_streams(mpcqp_handle* h, int parts) {
  hipError_t e = hipSuccess;
  if (parts < 2) return e;
  if (!h->ev_fork) e = hipEventCreateWithFlags(&h->ev_fork, hipEventDisableTiming);
  for (int i = 1; i < parts && i < mpcqp_handle::KMAX && e == hipSuccess; ++i) {
    if (!h->sub[i]) e = hipStreamCreateWithFlags(&h->sub[i], hipStreamNonBlocking);
    if (e == hipSuccess && !h->ev_join[i]) e = hipEventCreateWithFlags(&h->ev_join[i], hipEventDisableTiming);
  }
  return e;
}

constexpr size_t PIN_CHUNK = (size_t)2 << 20;  // bytes per pinned staging chunk

bool host_pinned(const void* p) {
  hipPointerAttribute_t at;
  if (hipPointerGetAttributes(&at, p) != hipSuccess) {
    (void)hipGetLastError();
    return false;
  }
  return at.type == hipMemoryTypeHost;
}

// The host wrappers' private stream and pinned staging, created on first use.  The stream is a
// BLOCKING one (hipStreamDefault): it is ordered after work the caller queued on the legacy null
// stream (e.g. hipMemset / torch zeroing of warm slots), as the null-stream wrappers were before.
hipError_t ensure_host_io(mpcqp_handle* h) {
  hipError_t e = hipSuccess;
  if (!h->hstream) e = hipStreamCreateWithFlags(&h->hstream, hipStreamDefault);
  for (int i = 0; i < 2 && e == hipSuccess; ++i) {
    if (!h->pin[i]) e = hipHostMalloc((void**)&h->pin[i], PIN_CHUNK, hipHostMallocDefault);
    if (e == hipSuccess && !h->pin_ev[i]) e = hipEventCreateWithFlags(&h->pin_ev[i], hipEventDisableTiming);
  }
  return e;
}

// Host -> device on the wrapper stream.  A pinned source goes by one DMA; a pageable one through
// the two staging chunks, the host copy of chunk c + 1 overlapping the DMA of chunk c.
hipError_t copy_h2d(mpcqp_handle* h, void* dst, const void* src, size_t bytes) {
  if (host_pinned(src)) return hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, h->hstream);
  hipError_t e = hipSuccess;
  for (size_t off = 0, c = 0; off < bytes && e == hipSuccess; off += PIN_CHUNK, ++c) {
    const int s = (int)(c & 1);
    const size_t len = bytes - off < PIN_CHUNK ? bytes - off : PIN_CHUNK;
    if (h->pin_busy[s]) e = hipEventSynchronize(h->pin_ev[s]);
    if (e != hipSuccess) break;
    memcpy(h->pin[s], (const char*)src + off, len);
    e = hipMemcpyAsync((char*)dst + off, h->pin[s], len, hipMemcpyHostToDevice, h->hstream);
    if (e == hipSuccess) e = hipEventRecord(h->pin_ev[s], h->hstream);
    h->pin_busy[s] = e == hipSuccess;
  }
  return e;
}

// Device -> host on the wrapper stream, synchronous on return (same staging scheme as copy_h2d).
hipError_t copy_d2h(mpcqp_handle* h, void* dst, const void* src, size_t bytes) {
  hipError_t e;
  if (host_pinned(dst)) {
    e = hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, h->hstream);
    return e == hipSuccess ? hipStreamSynchronize(h->hstream) : e;
  }
  // chunk c is copied into staging slot c & 1 while chunk c - 1 is copied out of the other slot
  e = hipSuccess;
  const size_t nch = (bytes + PIN_CHUNK - 1) / PIN_CHUNK;
  for (size_t c = 0; c <= nch && e == hipSuccess; ++c) {
    if (c < nch) {
      const size_t off = c * PIN_CHUNK, len = bytes - off < PIN_CHUNK ? bytes - off : PIN_CHUNK;
      e = hipMemcpyAsync(h->pin[c & 1], (const char*)src + off, len, hipMemcpyDeviceToHost, h->hstream);
      if (e == hipSuccess) e = hipEventRecord(h->pin_ev[c & 1], h->hstream);
    }
    if (e == hipSuccess && c > 0) {
      const size_t off = (c - 1) * PIN_CHUNK, len = bytes - off < PIN_CHUNK ? bytes - off : PIN_CHUNK;
      e = hipEventSynchronize(h->pin_ev[(c - 1) & 1]);
      if (e == hipSuccess) memcpy((char*)dst + off, h->pin[(c - 1) & 1], len);
    }
  }
  h->pin_busy[0] = h->pin_busy[1] = false;
  return e;
}

}  // namespace

extern "C" {

void mpcqp_default_params(mpcqp_params* p, int32_t horizon) {
  if (!p) return;
  memset(p, 0, sizeof(*p));
  p->horizon = horizon;
  p->max_iter = 4000;
  p->scaling = 10;
  p->check_termination = 25;
  p->adaptive_rho = 1;
  p->adaptive_rho_interval = 25;
  p->scaled_termination = 0;
  p->warm_start = 0;
  // Go1CtrlStates.hpp:203-249 defaults
  const double q[13] = {80.0, 80.0, 1.0, 0.0, 0.0, 270.0, 1.0, 1.0, 20.0, 20.0, 20.0, 20.0, 0.0};
  const double r[12] = {1e-5, 1e-5, 1e-6, 1e-5, 1e-5, 1e-6, 1e-5, 1e-5, 1e-6, 1e-5, 1e-5, 1e-6};
  memcpy(p->q_weights, q, sizeof(q));
  memcpy(p->r_weights, r, sizeof(r));
  p->rho = 0.1;
  p->sigma = 1e-6;
  p->alpha = 1.6;
  p->eps_abs = 1e-3;
  p->eps_rel = 1e-3;
  p->eps_prim_inf = 1e-4;
  p->eps_dual_inf = 1e-4;
  p->adaptive_rho_tolerance = 5.0;
}

int32_t mpcqp_record_size(int32_t horizon) {
  if (horizon < 1) return 0;
  return MPCQP_REC_SIZE(horizon);
}

int32_t mpcqp_create(const mpcqp_params* params, int32_t device, mpcqp_handle** out) {
  if (!out) return MPCQP_ERR_INVALID_ARG;
  *out = nullptr;
  if (!params_valid(params)) return MPCQP_ERR_INVALID_ARG;
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) return MPCQP_ERR_NO_DEVICE;
  if (device < 0 || device >= ndev) return MPCQP_ERR_INVALID_ARG;
  mpcqp_handle* h = new (std::nothrow) mpcqp_handle();
  if (!h) return MPCQP_ERR_ALLOC;
  h->p = *params;
  h->device = device;
  DeviceGuard dg(device);
  hipError_t e = dg.err;
  if (e != hipSuccess) { delete h; return MPCQP_ERR_HIP; }
  int cus = 0, per_cu = 0;
  e = hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device);
  if (e == hipSuccess) e = occupancy_for(h, &per_cu);
  if (e != hipSuccess || cus <= 0) { delete h; return MPCQP_ERR_HIP; }
  if (per_cu < 1) per_cu = 1;
  h->slots = cus * per_cu;
  h->cus = cus;
  if (const char* sp = getenv("MPCQP_SPLIT")) h->split = atoi(sp);
  if (const char* sw = getenv("MPCQP_SPLIT_W")) {
    for (int i = 0; i < mpcqp_handle::KMAX && *sw; ++i) {
      char* end = nullptr;
      const long v = strtol(sw, &end, 10);
      if (end == sw) break;
      h->split_w[i] = v > 0 && v < 1000 ? (int)v : 0;
      sw = *end == ',' ? end + 1 : end;
    }
  }
  *out = h;
  return MPCQP_OK;
}

int32_t mpcqp_destroy(mpcqp_handle* h) {
  if (!h) return MPCQP_ERR_INVALID_ARG;
  DeviceGuard dg(h->device);
  (void)hipFree(h->work);
  (void)hipFree(h->fb);
  (void)hipFree(h->d_recs);
  (void)hipFree(h->d_res);
  (void)hipFree(h->d_sol);
  (void)hipFree(h->d_bal_recs);
  (void)hipFree(h->d_bal_res);
  if (h->hstream) (void)hipStreamSynchronize(h->hstream);
  for (int i = 0; i < 2; ++i) {
    if (h->pin_ev[i]) (void)hipEventDestroy(h->pin_ev[i]);
    (void)hipHostFree(h->pin[i]);
  }
  if (h->hstream) (void)hipStreamDestroy(h->hstream);
  for (int i = 0; i < mpcqp_handle::KMAX; ++i) {
    if (h->sub[i]) (void)hipStreamSynchronize(h->sub[i]);
    if (h->sub[i]) (void)hipStreamDestroy(h->sub[i]);
    if (h->ev_join[i]) (void)hipEventDestroy(h->ev_join[i]);
  }
  if (h->ev_fork) (void)hipEventDestroy(h->ev_fork);
  delete h;
  return MPCQP_OK;
}

static int32_t solve_device_impl(mpcqp_handle* h, const double* d_records, int32_t batch,
                                 mpcqp_result* d_results, double* d_solution, double* d_trace,
                                 int32_t trace_cap, void* stream, double* d_state = nullptr) {
  if (!h || batch < 0 || (batch > 0 && (!d_records || !d_results))) return MPCQP_ERR_INVALID_ARG;
  if (d_state && effective_path(h) != 3) return MPCQP_ERR_INVALID_ARG;  // warm start: the wave path
  if (batch == 0) return MPCQP_OK;
  DeviceGuard dg(h->device);
  hipError_t e = dg.err;
  if (e != hipSuccess) return set_hip_error(h, e, "hipSetDevice");
  // grow-only; a capture-safe caller pre-sizes with mpcqp_reserve()
  e = ensure_workspace(h, batch, stream);
  if (e != hipSuccess) return set_hip_error(h, e, "workspace hipMalloc");
  mpcqp::LaunchArgs a;
  a.recs = d_records;
  a.batch = batch;
  a.results = d_results;
  a.solution = d_solution;
  a.work = h->work;
  a.trace = d_trace;
  a.trace_cap = d_trace ? trace_cap : 0;
  a.wstate = d_state;
  a.fallback = h->fb;
  a.grid = batch;
  a.stream = stream;
  a.p = h->p;
  switch (effective_path(h)) {
#ifdef MPCQP_DEBUG_PATHS
    case 1: e = mpcqp::launch_solve_any(a); break;
    case 2: e = mpcqp::launch_riccati_any(a); break;
#endif
    default: {
      const int parts = split_parts(h, batch);
      h->fb_parts = parts;
      if (parts == 1) {
        e = mpcqp::launch_wave_any(a);
        break;
      }
      // fork: part 0 runs on the caller's stream, every other part on an internal stream that waits
      // for the work queued on the caller's stream so far (parts - 1 streams more: a process has
      // few hardware queues, GPU_MAX_HW_QUEUES = 4, and streams beyond them share one in order)
      e = ensure_split_streams(h, parts);
      if (e == hipSuccess) e = hipEventRecord(h->ev_fork, (hipStream_t)stream);
      const size_t rs = (size_t)MPCQP_REC_SIZE(h->p.horizon), n = (size_t)MPCQP_NUM_DOF * h->p.horizon;
      const size_t ws = (size_t)mpcqp::warm_state_doubles(h->p.horizon);
      // part boundaries: equal parts, or relative sizes split_w when every part gets a robot
      int bnd[mpcqp_handle::KMAX + 1];
      int64_t wsum = 0;
      for (int i = 0; i < parts; ++i) wsum = h->split_w[i] > 0 && wsum >= 0 ? wsum + h->split_w[i] : -1;
      bool weighted = wsum > 0;
      for (int i = 0, wc = 0; i <= parts; ++i) {
        bnd[i] = (int)(weighted ? (int64_t)batch * wc / wsum : (int64_t)batch * i / parts);
        if (i < parts && weighted) wc += h->split_w[i];
      }
      for (int i = 0; i < parts && weighted; ++i) weighted = bnd[i + 1] > bnd[i];
      for (int i = 0; i <= parts && !weighted; ++i) bnd[i] = (int)((int64_t)batch * i / parts);
      for (int i = 0; i < parts && e == hipSuccess; ++i) {
        const int b0 = bnd[i], b1 = bnd[i + 1];
        mpcqp::LaunchArgs ai = a;
        ai.recs = d_records + rs * b0;
        ai.batch = b1 - b0;
        ai.grid = b1 - b0;
        ai.results = d_results + b0;
        ai.solution = d_solution ? d_solution + n * b0 : nullptr;
        ai.work = h->work + h->work_per * b0;
        ai.trace = d_trace ? d_trace + (size_t)b0 * MPCQP_TRACE_LEN * 4 : nullptr;
        ai.trace_cap = d_trace && trace_cap > b0 ? trace_cap - b0 : 0;
        ai.wstate = d_state ? d_state + ws * b0 : nullptr;
        ai.fallback = h->fb + 4 * i;
        if (i == 0) {
          ai.stream = stream;
          e = mpcqp::launch_wave_any(ai);
          continue;
        }
        ai.stream = h->sub[i];
        e = hipStreamWaitEvent(h->sub[i], h->ev_fork, 0);
        if (e == hipSuccess) e = mpcqp::launch_wave_any(ai);
        if (e == hipSuccess) e = hipEventRecord(h->ev_join[i], h->sub[i]);
      }
      // join: the caller's stream waits for every other part
      for (int i = 1; i < parts && e == hipSuccess; ++i) e = hipStreamWaitEvent((hipStream_t)stream, h->ev_join[i], 0);
      break;
    }
  }
  if (e != hipSuccess) return set_hip_error(h, e, "solve_kernel launch");
  return MPCQP_OK;
}

int32_t mpcqp_solve_batch_device(mpcqp_handle* h, const double* d_records, int32_t batch,
                                 mpcqp_result* d_results, double* d_solution, void* stream) {
  return solve_device_impl(h, d_records, batch, d_results, d_solution, nullptr, 0, stream);
}

int32_t mpcqp_debug_solve_trace_device(mpcqp_handle* h, const double* d_records, int32_t batch,
                                       mpcqp_result* d_results, double* d_solution,
                                       double* d_trace, int32_t trace_cap, void* stream) {
  return solve_device_impl(h, d_records, batch, d_results, d_solution, d_trace, trace_cap, stream);
}

int32_t mpcqp_warm_state_size(int32_t horizon) {
  if (horizon < 1 || horizon > mpcqp::WAVE_MAX_HORIZON) return 0;
  return mpcqp::warm_state_doubles(horizon);
}

int32_t mpcqp_solve_batch_warm_device(mpcqp_handle* h, const double* d_records, int32_t batch, double* d_state,
                                      mpcqp_result* d_results, double* d_solution, void* stream) {
  if (batch > 0 && !d_state) return MPCQP_ERR_INVALID_ARG;
  return solve_device_impl(h, d_records, batch, d_results, d_solution, nullptr, 0, stream, d_state);
}

static int32_t solve_host_impl(mpcqp_handle* h, const double* h_records, int32_t batch, double* d_state,
                               mpcqp_result* h_results, double* h_solution) {
  if (!h || batch < 0 || (batch > 0 && (!h_records || !h_results))) return MPCQP_ERR_INVALID_ARG;
  if (batch == 0) return MPCQP_OK;
  if (d_state && effective_path(h) != 3) return MPCQP_ERR_INVALID_ARG;  // warm start: the wave path
  DeviceGuard dg(h->device);
  hipError_t e = dg.err;
  if (e != hipSuccess) return set_hip_error(h, e, "hipSetDevice");
  e = ensure_host_io(h);
  if (e != hipSuccess) return set_hip_error(h, e, "host staging");
  const size_t rs = (size_t)MPCQP_REC_SIZE(h->p.horizon);
  const size_t n = (size_t)MPCQP_NUM_DOF * h->p.horizon;
  if ((size_t)batch > h->cap) {
    (void)hipStreamSynchronize(h->hstream);
    (void)hipFree(h->d_recs);
    (void)hipFree(h->d_res);
    (void)hipFree(h->d_sol);
    h->d_recs = nullptr; h->d_res = nullptr; h->d_sol = nullptr; h->cap = 0;
    e = hipMalloc(&h->d_recs, sizeof(double) * rs * batch);
    if (e == hipSuccess) e = hipMalloc(&h->d_res, sizeof(mpcqp_result) * batch);
    if (e == hipSuccess) e = hipMalloc(&h->d_sol, sizeof(double) * n * batch);
    if (e != hipSuccess) return set_hip_error(h, e, "hipMalloc");
    h->cap = batch;
  }
  e = copy_h2d(h, h->d_recs, h_records, sizeof(double) * rs * batch);
  if (e != hipSuccess) return set_hip_error(h, e, "records H2D");
  int32_t rc = solve_device_impl(h, h->d_recs, batch, h->d_res, h_solution ? h->d_sol : nullptr,
                                 nullptr, 0, h->hstream, d_state);
  if (rc != MPCQP_OK) return rc;
  e = copy_d2h(h, h_results, h->d_res, sizeof(mpcqp_result) * batch);
  if (e == hipSuccess && h_solution) e = copy_d2h(h, h_solution, h->d_sol, sizeof(double) * n * batch);
  if (e != hipSuccess) return set_hip_error(h, e, "results D2H");
  return MPCQP_OK;
}

int32_t mpcqp_solve_batch_host(mpcqp_handle* h, const double* h_records, int32_t batch,
                               mpcqp_result* h_results, double* h_solution) {
  return solve_host_impl(h, h_records, batch, nullptr, h_results, h_solution);
}

int32_t mpcqp_solve_batch_warm_host(mpcqp_handle* h, const double* h_records, int32_t batch, double* d_state,
                                    mpcqp_result* h_results, double* h_solution) {
  if (batch > 0 && !d_state) return MPCQP_ERR_INVALID_ARG;
  return solve_host_impl(h, h_records, batch, d_state, h_results, h_solution);
}

int32_t mpcqp_build_qp_device(mpcqp_handle* h, const double* d_records, int32_t batch, double* d_P,
                              double* d_q, double* d_l, double* d_u, void* stream) {
  if (!h || batch < 0 || (batch > 0 && (!d_records || !d_P || !d_q || !d_l || !d_u)))
    return MPCQP_ERR_INVALID_ARG;
  if (batch == 0) return MPCQP_OK;
  DeviceGuard dg(h->device);
  hipError_t e = dg.err;
  if (e != hipSuccess) return set_hip_error(h, e, "hipSetDevice");
  mpcqp::LaunchArgs a;
  memset(&a, 0, sizeof(a));
  a.recs = d_records;
  a.batch = batch;
  a.stream = stream;
  a.p = h->p;
  e = mpcqp::launch_build_any(a, d_P, d_q, d_l, d_u);
  if (e != hipSuccess) return set_hip_error(h, e, "build_qp_kernel launch");
  return MPCQP_OK;
}

int32_t mpcqp_assemble_records_device(int32_t horizon, const double* d_states, int32_t batch, double* d_records,
                                      void* stream) {
  if (horizon < 1 || horizon > MPCQP_MAX_HORIZON || batch < 0 || (batch > 0 && (!d_states || !d_records)))
    return MPCQP_ERR_INVALID_ARG;
  if (batch == 0) return MPCQP_OK;
  return mpcqp::launch_assemble(horizon, d_states, batch, d_records, stream) == hipSuccess ? MPCQP_OK : MPCQP_ERR_HIP;
}

int32_t mpcqp_copy_warm_slots_device(int32_t horizon, const double* d_src, const int32_t* d_src_idx, double* d_dst,
                                     const int32_t* d_dst_idx, int32_t count, void* stream) {
  if (horizon < 1 || horizon > MPCQP_MAX_HORIZON || count < 0 || (count > 0 && (!d_src || !d_dst)))
    return MPCQP_ERR_INVALID_ARG;
  if (count == 0) return MPCQP_OK;
  return mpcqp::launch_copy_slots(d_src, d_src_idx, d_dst, d_dst_idx, count, mpcqp_warm_state_size(horizon), stream) ==
                 hipSuccess
             ? MPCQP_OK
             : MPCQP_ERR_HIP;
}

void mpcqp_balance_default_params(mpcqp_balance_params* p) {
  if (!p) return;
  const double q[6] = {1.0, 1.0, 1.0, 400.0, 400.0, 100.0};  // A1RobotControl.cpp:11
  for (int i = 0; i < 6; ++i) p->q_diag[i] = q[i];
  p->r = 1e-3;  // :12
  p->mu = 0.7;  // :13
  p->f_min = 0.0;
  p->f_max = 180.0;  // :14-15
}

int32_t mpcqp_balance_solve_device(mpcqp_handle* h, const mpcqp_balance_params* bp, const double* d_records,
                                   int32_t batch, mpcqp_result* d_results, void* stream) {
  if (!h || !bp || batch < 0 || (batch > 0 && (!d_records || !d_results))) return MPCQP_ERR_INVALID_ARG;
  if (batch == 0) return MPCQP_OK;
  DeviceGuard dg(h->device);
  hipError_t e = dg.err;
  if (e != hipSuccess) return set_hip_error(h, e, "hipSetDevice");
  e = mpcqp::launch_balance(*bp, h->p, d_records, batch, d_results, stream);
  if (e != hipSuccess) return set_hip_error(h, e, "balance_kernel launch");
  return MPCQP_OK;
}

int32_t mpcqp_balance_solve_host(mpcqp_handle* h, const mpcqp_balance_params* bp, const double* h_records,
                                 int32_t batch, mpcqp_result* h_results) {
  if (!h || !bp || batch < 0 || (batch > 0 && (!h_records || !h_results))) return MPCQP_ERR_INVALID_ARG;
  if (batch == 0) return MPCQP_OK;
  DeviceGuard dg(h->device);
  hipError_t e = dg.err;
  if (e != hipSuccess) return set_hip_error(h, e, "hipSetDevice");
  e = ensure_host_io(h);
  if (e != hipSuccess) return set_hip_error(h, e, "host staging");
  if ((size_t)batch > h->bal_cap) {
    (void)hipStreamSynchronize(h->hstream);
    (void)hipFree(h->d_bal_recs);
    (void)hipFree(h->d_bal_res);
    h->d_bal_recs = nullptr; h->d_bal_res = nullptr; h->bal_cap = 0;
    e = hipMalloc(&h->d_bal_recs, sizeof(double) * MPCQP_BAL_SIZE * batch);
    if (e == hipSuccess) e = hipMalloc(&h->d_bal_res, sizeof(mpcqp_result) * batch);
    if (e != hipSuccess) return set_hip_error(h, e, "hipMalloc");
    h->bal_cap = batch;
  }
  e = copy_h2d(h, h->d_bal_recs, h_records, sizeof(double) * MPCQP_BAL_SIZE * batch);
  if (e != hipSuccess) return set_hip_error(h, e, "records H2D");
  int32_t rc = mpcqp_balance_solve_device(h, bp, h->d_bal_recs, batch, h->d_bal_res, h->hstream);
  if (rc != MPCQP_OK) return rc;
  e = copy_d2h(h, h_results, h->d_bal_res, sizeof(mpcqp_result) * batch);
  if (e != hipSuccess) return set_hip_error(h, e, "results D2H");
  return MPCQP_OK;
}

int32_t mpcqp_joint_torques_device(const double* d_tq_records, const mpcqp_result* d_grf, int32_t batch,
                                   int32_t* d_counter, double* d_joint_torques, void* stream) {
  if (batch < 0 || (batch > 0 && (!d_tq_records || !d_grf || !d_counter || !d_joint_torques)))
    return MPCQP_ERR_INVALID_ARG;
  if (batch == 0) return MPCQP_OK;
  return mpcqp::launch_torques(d_tq_records, d_grf, batch, d_counter, d_joint_torques, stream) == hipSuccess
             ? MPCQP_OK
             : MPCQP_ERR_HIP;
}

const char* mpcqp_status_str(int32_t s) {
  switch (s) {
    case MPCQP_STATUS_SOLVED: return "solved";
    case MPCQP_STATUS_SOLVED_INACCURATE: return "solved inaccurate";
    case MPCQP_STATUS_PRIMAL_INFEASIBLE_INACCURATE: return "primal infeasible inaccurate";
    case MPCQP_STATUS_DUAL_INFEASIBLE_INACCURATE: return "dual infeasible inaccurate";
    case MPCQP_STATUS_MAX_ITER_REACHED: return "maximum iterations reached";
    case MPCQP_STATUS_PRIMAL_INFEASIBLE: return "primal infeasible";
    case MPCQP_STATUS_DUAL_INFEASIBLE: return "dual infeasible";
    case MPCQP_STATUS_NON_CVX: return "problem non convex";
    case MPCQP_STATUS_NAN_INPUT: return "non-finite input";
    case MPCQP_STATUS_UNSOLVED: return "unsolved";
    default: return "unknown status";
  }
}

const char* mpcqp_error_str(int32_t err) {
  switch (err) {
    case MPCQP_OK: return "ok";
    case MPCQP_ERR_INVALID_ARG: return "invalid argument";
    case MPCQP_ERR_HIP: return "HIP runtime error";
    case MPCQP_ERR_NO_DEVICE: return "no HIP device";
    case MPCQP_ERR_ALLOC: return "device allocation failed";
    default: return "unknown error";
  }
}

const char* mpcqp_last_error(mpcqp_handle* h) { return h ? h->err : "null handle"; }

int32_t mpcqp_abi_sizes(int32_t* params_size, int32_t* result_size) {
  if (params_size) *params_size = (int32_t)sizeof(mpcqp_params);
  if (result_size) *result_size = (int32_t)sizeof(mpcqp_result);
  return MPCQP_OK;
}

int32_t mpcqp_handle_slots(mpcqp_handle* h) { return h ? h->slots : 0; }

int32_t mpcqp_handoff_counts(mpcqp_handle* h, int32_t counts[3]) {
  if (!h || !counts) return MPCQP_ERR_INVALID_ARG;
  counts[0] = counts[1] = counts[2] = 0;
  if (!h->fb) return MPCQP_OK;  // no wave solve yet
  DeviceGuard g(h->device);
  hipError_t e = g.err;
  if (e == hipSuccess) e = hipDeviceSynchronize();
  int32_t all[4 * mpcqp_handle::KMAX];
  if (e == hipSuccess) e = hipMemcpy(all, h->fb, sizeof(int32_t) * 4 * h->fb_parts, hipMemcpyDeviceToHost);
  for (int i = 0; i < h->fb_parts && e == hipSuccess; ++i)
    for (int j = 0; j < 3; ++j) counts[j] += all[4 * i + j];
  return e == hipSuccess ? MPCQP_OK : set_hip_error(h, e, "mpcqp_handoff_counts");
}

int32_t mpcqp_debug_set_split(mpcqp_handle* h, int32_t parts) {
  if (!h || parts < 0 || parts > mpcqp_handle::KMAX) return -MPCQP_ERR_INVALID_ARG;
  const int32_t old = h->split;
  h->split = parts;
  return old;
}

int32_t mpcqp_debug_split_parts(mpcqp_handle* h, int32_t batch) {
  if (!h || batch < 1) return 0;
  return effective_path(h) == 3 ? split_parts(h, batch) : 1;
}

int32_t mpcqp_reserve(mpcqp_handle* h, int32_t batch) {
  if (!h || batch < 0) return MPCQP_ERR_INVALID_ARG;
  DeviceGuard dg(h->device);
  hipError_t e = dg.err;
  if (e == hipSuccess && ((size_t)batch > h->work_cap || work_per_instance(h) > h->work_per))
    e = hipDeviceSynchronize();
  if (e == hipSuccess) e = ensure_workspace(h, batch, nullptr);
  if (e != hipSuccess) return set_hip_error(h, e, "workspace hipMalloc");
  if (effective_path(h) == 3) e = ensure_split_streams(h, split_parts(h, batch));
  if (e != hipSuccess) return set_hip_error(h, e, "split streams");
  return MPCQP_OK;
}
int32_t mpcqp_solve_threads(int32_t horizon) {
  if (horizon < 1 || horizon > MPCQP_MAX_HORIZON) return 0;
  return 64;  // one wavefront per robot
}

int32_t mpcqp_debug_set_solver(mpcqp_handle* h, int32_t path) {
  if (!h) return MPCQP_ERR_INVALID_ARG;
#ifdef MPCQP_DEBUG_PATHS
  if (path < 0 || path > 3) return MPCQP_ERR_INVALID_ARG;
  if (path == 1 && h->p.horizon > mpcqp::DENSE_MAX_HORIZON) return MPCQP_ERR_INVALID_ARG;
#else
  if (path != 0 && path != 3) return MPCQP_ERR_INVALID_ARG;  // cross-check paths: libmpcqp_debug.so
#endif
  DeviceGuard dg(h->device);
  hipError_t e = dg.err;
  if (e != hipSuccess) return set_hip_error(h, e, "hipSetDevice");
  const int old = h->path;
  h->path = path;
  int per_cu = 0;
  e = occupancy_for(h, &per_cu);
  if (e != hipSuccess) {
    h->path = old;
    return set_hip_error(h, e, "occupancy query");
  }
  h->slots = per_cu * h->cus;
  return MPCQP_OK;
}

int32_t mpcqp_debug_scale_image_doubles(int32_t horizon) {
  if (horizon < 1 || horizon > MPCQP_MAX_HORIZON) return 0;
  return mpcqp::scale_image_doubles(horizon);
}

int32_t mpcqp_debug_scale_image_device(mpcqp_handle* h, const double* d_records, int32_t batch, double* d_state,
                                       double* d_img, void* stream) {
#ifdef MPCQP_DEBUG_PATHS
  if (!h || batch < 0 || (batch > 0 && (!d_records || !d_img))) return MPCQP_ERR_INVALID_ARG;
  if (batch == 0) return MPCQP_OK;
  DeviceGuard dg(h->device);
  hipError_t e = dg.err;
  if (e != hipSuccess) return set_hip_error(h, e, "hipSetDevice");
  e = ensure_workspace(h, batch, stream);  // (the fallback list the kernel resets)
  if (e != hipSuccess) return set_hip_error(h, e, "workspace hipMalloc");
  mpcqp::LaunchArgs a;
  memset(&a, 0, sizeof(a));
  a.recs = d_records;
  a.batch = batch;
  a.work = d_img;
  a.wstate = d_state;
  a.fallback = h->fb;
  a.stream = stream;
  a.p = h->p;
  e = mpcqp::launch_scale_any(a);
  if (e != hipSuccess) return set_hip_error(h, e, "scale_kernel launch");
  return MPCQP_OK;
#else
  (void)h; (void)d_records; (void)batch; (void)d_state; (void)d_img; (void)stream;
  return MPCQP_ERR_INVALID_ARG;  // libmpcqp_debug.so only
#endif
}

int32_t mpcqp_debug_wave_selftest(double* d_out, void* stream) {
  if (!d_out) return MPCQP_ERR_INVALID_ARG;
  return mpcqp::wave_selftest(d_out, stream) == hipSuccess ? MPCQP_OK : MPCQP_ERR_HIP;
}

}  // extern "C"
