// mpcqp_fleet.hip -- device-resident closed loop for a fleet of vehicles.
//
// One mpcqp_fleet_step = for every RUNNING vehicle, one iteration of the loop body of
// TrajectoryTracker.track (src/pipeline/control_stage.py:100-150):
//   k_fleet_build(relax=0)  window gather + tail padding (:101-105) fused into K1; mask = RUNNING
//   K2 (nominal ws)         _solve_with_relaxation's first solve (:43-46)
//   k_fleet_build(relax=1)  vehicles whose nominal status is not solved/solved_inaccurate
//                           (mpc_controller.py:137-139) get the relaxed window (v * 0.6, :48-49)
//   K2 (relaxed ws)         the retry with widened du_bounds (:50-56), masked to those vehicles
//   k_fleet_advance         abort (:108-110), plant f_discrete (:127), u_prev (:129),
//                           path_idx advance (:141-145), goal test (:147-150), trace (:128)
// The window is never materialised: lane k of a vehicle's wave reads row
// min(path_idx + k, len - 1) of its reference, which is numpy's slice + np.repeat padding.
#include "mpcqp_build.h"

namespace {
using mpcqp::fail;
using mpcqp::Launch;

__global__ __launch_bounds__(kWave) void k_fleet_build(mpcqp_params p, mpcqp_fleet f, int relax,
                                                       double* __restrict__ model) {
  const int b = blockIdx.x;
  const int lane = threadIdx.x;
  const int V = f.vehicles;
  if (b >= V) return;
  bool go;
  if (relax) {
    const int st = f.status[b];
    go = f.mask[b] && !(st == MPCQP_SOLVED || st == MPCQP_SOLVED_INACCURATE);
  } else {
    go = f.phase[b] == MPCQP_FLEET_RUNNING;
    // device-side validation of the loop state a C-ABI caller hands over (check_fleet cannot see
    // device data): an unusable reference aborts the vehicle, a full trace ends its run -- before
    // any indexed access
    const int len0 = f.ref_len[b], pi0 = f.path_idx[b], st0 = f.steps[b];
    const bool bad_ref = len0 < 1 || len0 > f.ref_stride || pi0 < 0;
    const bool full = st0 < 0 || st0 >= f.max_steps;
    if (go && (bad_ref || full)) {
      if (lane == 0) f.phase[b] = bad_ref ? MPCQP_FLEET_ABORTED : MPCQP_FLEET_OUT_OF_STEPS;
      go = false;
    }
  }
  if (lane == 0) f.mask[(size_t)relax * V + b] = go ? 1 : 0;
  if (!go) return;
  const int N = p.horizon;
  const int len = f.ref_len[b];
  const int pidx = f.path_idx[b];
  const double x0l = lane < 4 ? f.state[(size_t)b * 4 + lane] : 0.0;
  const double upl = (lane >= 4 && lane < 6) ? f.u_prev[(size_t)b * 2 + lane - 4] : 0.0;
  // window row k = ref[min(path_idx + k, len - 1)] (tail padding, control_stage.py:101-105)
  auto fetch = [&](int k, double& rx, double& ry, double& ryaw, double& rv) {
    const double* r = f.ref_global + ((size_t)b * f.ref_stride + min(pidx + k, len - 1)) * 4;
    rx = r[0];
    ry = r[1];
    ryaw = r[2];
    rv = relax ? r[3] * 0.6 : r[3];  // relaxed_reference[:, 3] *= 0.6 (control_stage.py:48-49)
  };
  if (N + 1 > kWave) {  // long windows: chunks of 64 rows
    build_qp_long(p, lane, fetch, x0l, upl, model + (size_t)b * model_stride(N));
    return;
  }
  double rx = 0.0, ry = 0.0, ryaw = 0.0, rv = 0.0;
  if (lane <= N) fetch(lane, rx, ry, ryaw, rv);
  build_qp(p, lane, rx, ry, ryaw, rv, x0l, upl, model + (size_t)b * model_stride(N));
}

__global__ __launch_bounds__(kWave) void k_fleet_advance(double dt, double L, mpcqp_fleet f) {
#pragma clang fp contract(off)
  const int b = blockIdx.x * kWave + threadIdx.x;
  const int V = f.vehicles;
  if (b >= V || f.phase[b] != MPCQP_FLEET_RUNNING) return;
  int which = -1;
  const int s0 = f.status[b];
  if (s0 == MPCQP_SOLVED || s0 == MPCQP_SOLVED_INACCURATE) {
    which = 0;
  } else if (f.mask[(size_t)V + b]) {
    const int s1 = f.status[(size_t)V + b];
    if (s1 == MPCQP_SOLVED || s1 == MPCQP_SOLVED_INACCURATE) which = 1;
  }
  if (which < 0) {
    f.phase[b] = MPCQP_FLEET_ABORTED;  // control_stage.py:108-110
    return;
  }
  const double* u = f.u0 + ((size_t)which * V + b) * 2;
  const double a = u[0], delta = u[1];
  double x[4], xn[4];
  for (int i = 0; i < 4; ++i) x[i] = f.state[(size_t)b * 4 + i];
  plant(x, a, delta, dt, L, xn);
  const int k = f.steps[b];
  if (k < 0 || k >= f.max_steps) {  // k_fleet_build already ended such a run; never write past the trace
    f.phase[b] = MPCQP_FLEET_OUT_OF_STEPS;
    return;
  }
  for (int i = 0; i < 4; ++i) f.state[(size_t)b * 4 + i] = xn[i];
  if (f.trace)
    for (int i = 0; i < 4; ++i) f.trace[((size_t)b * f.max_steps + k) * 4 + i] = xn[i];
  if (f.u_trace) {
    f.u_trace[((size_t)b * f.max_steps + k) * 2 + 0] = a;
    f.u_trace[((size_t)b * f.max_steps + k) * 2 + 1] = delta;
  }
  f.u_prev[(size_t)b * 2 + 0] = a;
  f.u_prev[(size_t)b * 2 + 1] = delta;
  f.steps[b] = k + 1;
  const int len = f.ref_len[b];
  int pi = f.path_idx[b];
  if (pi < len - 2 && fleet_off_row(xn[0], xn[1], f.ref_global + ((size_t)b * f.ref_stride + pi) * 4))
    f.path_idx[b] = pi + 1;
  int ph = MPCQP_FLEET_RUNNING;
  if (fleet_at_goal(xn[0], xn[1], f.goal[(size_t)b * 2], f.goal[(size_t)b * 2 + 1]))
    ph = MPCQP_FLEET_GOAL;
  else if (k + 1 >= f.max_steps)
    ph = MPCQP_FLEET_OUT_OF_STEPS;
  f.phase[b] = ph;
}

// the parameter blocks of one mpcqp_fleet_loop call, stream-ordered before the loop kernel
__global__ __launch_bounds__(kWave) void k_store_params(mpcqp_params pn, mpcqp_params pr, mpcqp_params* __restrict__ P) {
  static_assert(sizeof(mpcqp_params) % 4 == 0, "params copied by words");
  constexpr int W = (int)(sizeof(mpcqp_params) / 4);
  for (int w = threadIdx.x; w < W; w += kWave) {
    reinterpret_cast<uint32_t*>(P)[w] = reinterpret_cast<const uint32_t*>(&pn)[w];
    reinterpret_cast<uint32_t*>(P + 1)[w] = reinterpret_cast<const uint32_t*>(&pr)[w];
  }
}

// The fused loop's dispatch order: the vehicles by reference length, longest first (a bucket sort
// on the length, 1024 buckets; the order inside a bucket is immaterial -- vehicles are independent).
// One 1024-thread workgroup.
constexpr int kOrderBuckets = 1024;
__global__ __launch_bounds__(kOrderBuckets) void k_fleet_order(mpcqp_fleet f, int32_t* __restrict__ order) {
  __shared__ int cnt[kOrderBuckets];
  const int t = threadIdx.x, V = f.vehicles;
  const int span = f.ref_stride + 1;
  auto bucket = [&](int v) {
    int len = f.ref_len[v];
    len = len < 0 ? 0 : (len > f.ref_stride ? f.ref_stride : len);
    return (int)(((long long)(f.ref_stride - len) * kOrderBuckets) / span);  // longest -> bucket 0
  };
  cnt[t] = 0;
  __syncthreads();
  for (int v = t; v < V; v += kOrderBuckets) atomicAdd(&cnt[bucket(v)], 1);
  __syncthreads();
  for (int d = 1; d < kOrderBuckets; d <<= 1) {  // inclusive scan (Hillis-Steele)
    const int add = t >= d ? cnt[t - d] : 0;
    __syncthreads();
    cnt[t] += add;
    __syncthreads();
  }
  const int excl = t ? cnt[t - 1] : 0;
  __syncthreads();
  cnt[t] = excl;
  __syncthreads();
  for (int v = t; v < V; v += kOrderBuckets) order[atomicAdd(&cnt[bucket(v)], 1)] = v;
}

int check_fleet(const mpcqp_ws* nom, const mpcqp_ws* rel, const mpcqp_fleet* f) {
  if (!nom || !rel || !f) return fail(MPCQP_E_ARG, "null argument");
  if (nom == rel) return fail(MPCQP_E_ARG, "nominal and relaxed workspaces must differ");
  if (nom->p.horizon != rel->p.horizon) return fail(MPCQP_E_HORIZON, "workspaces differ in horizon");
  if (nom->device != rel->device) return fail(MPCQP_E_ARG, "workspaces on different devices");
  if (f->vehicles < 0 || f->vehicles > nom->max_batch || f->vehicles > rel->max_batch)
    return fail(MPCQP_E_BATCH, "fleet exceeds workspace capacity");
  if (f->ref_stride < 1 || f->max_steps < 1) return fail(MPCQP_E_ARG, "ref_stride and max_steps must be >= 1");
  if (!f->ref_global || !f->ref_len || !f->goal || !f->state || !f->u_prev || !f->path_idx || !f->phase ||
      !f->steps || !f->mask || !f->status || !f->u0)
    return fail(MPCQP_E_ARG, "null fleet buffer");
  return MPCQP_OK;
}

// enqueue one step (no validation)
int enqueue_step(mpcqp_ws* nom, mpcqp_ws* rel, const mpcqp_fleet* f, hipStream_t s) {
  const int V = f->vehicles;
  const mpcqp::launcher_t solve = mpcqp::launcher(nom->p);
  if (mpcqp::launcher(rel->p) != solve) return fail(MPCQP_E_ARG, "nominal and relaxed workspaces differ in kernel");
  if (!solve) return fail(MPCQP_E_HORIZON, "horizon not compiled into this build");
  const int rc = mpcqp::fleet_buffers(nom, rel, s);
  if (rc) return rc;
  nom->built_B = -1;  // the fleet overwrites the models: a later mpcqp_solve needs its own build
  rel->built_B = -1;
  nom->in_x0 = nom->in_ref = nom->in_up = nullptr;
  rel->in_x0 = rel->in_ref = rel->in_up = nullptr;
  hipLaunchKernelGGL(k_fleet_build, dim3(V), dim3(kWave), 0, s, nom->p, *f, 0, nom->model);
  solve(s, Launch{&nom->p, V, nom->model, nom->state, f->u0, f->X, nullptr, f->status, nullptr, nullptr, f->mask});
  hipLaunchKernelGGL(k_fleet_build, dim3(V), dim3(kWave), 0, s, rel->p, *f, 1, rel->model);
  solve(s, Launch{&rel->p, V, rel->model, rel->state, f->u0 + (size_t)2 * V, f->X, nullptr, f->status + V, nullptr,
                  nullptr, f->mask + V});
  hipLaunchKernelGGL(k_fleet_advance, dim3((V + kWave - 1) / kWave), dim3(kWave), 0, s, nom->p.dt,
                     nom->p.wheelbase_px, *f);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return fail(MPCQP_E_HIP, std::string("fleet step launch: ") + hipGetErrorString(e));
  return MPCQP_OK;
}

#define HIP_OR_FAIL(call)                                                                    \
  do {                                                                                       \
    hipError_t e_ = (call);                                                                  \
    if (e_ != hipSuccess) return fail(MPCQP_E_HIP, std::string(#call ": ") + hipGetErrorString(e_)); \
  } while (0)

// One captured step, replayed `steps` times on a private stream ordered against the caller's.
int run_graph(mpcqp_ws* nom, mpcqp_ws* rel, const mpcqp_fleet* f, int steps, hipStream_t user) {
  hipStream_t s2 = nullptr;
  hipEvent_t ev = nullptr;
  hipGraph_t g = nullptr;
  hipGraphExec_t ex = nullptr;
  int rc = MPCQP_OK;
  auto cleanup = [&]() {
    if (ex) (void)hipGraphExecDestroy(ex);
    if (g) (void)hipGraphDestroy(g);
    if (ev) (void)hipEventDestroy(ev);
    if (s2) (void)hipStreamDestroy(s2);
  };
  hipError_t e = hipStreamCreateWithFlags(&s2, hipStreamNonBlocking);
  if (e == hipSuccess) e = hipEventCreateWithFlags(&ev, hipEventDisableTiming);
  if (e == hipSuccess) e = hipEventRecord(ev, user);
  if (e == hipSuccess) e = hipStreamWaitEvent(s2, ev, 0);
  if (e == hipSuccess && (rc = mpcqp::fleet_buffers(nom, rel, user)) != MPCQP_OK) {  // outside the capture
    cleanup();
    return rc;
  }
  if (e == hipSuccess) e = hipStreamBeginCapture(s2, hipStreamCaptureModeThreadLocal);
  if (e != hipSuccess) {
    cleanup();
    return fail(MPCQP_E_HIP, std::string("fleet graph setup: ") + hipGetErrorString(e));
  }
  rc = enqueue_step(nom, rel, f, s2);
  e = hipStreamEndCapture(s2, &g);
  if (rc == MPCQP_OK && e != hipSuccess) rc = fail(MPCQP_E_HIP, std::string("hipStreamEndCapture: ") + hipGetErrorString(e));
  if (rc == MPCQP_OK) {
    e = hipGraphInstantiate(&ex, g, nullptr, nullptr, 0);
    for (int i = 0; e == hipSuccess && i < steps; ++i) e = hipGraphLaunch(ex, s2);
    if (e == hipSuccess) e = hipEventRecord(ev, s2);
    if (e == hipSuccess) e = hipStreamWaitEvent(user, ev, 0);
    // the replays must finish before the graph and its stream are released
    if (e == hipSuccess) e = hipStreamSynchronize(s2);
    if (e != hipSuccess) rc = fail(MPCQP_E_HIP, std::string("fleet graph replay: ") + hipGetErrorString(e));
  }
  cleanup();
  return rc;
}

}  // namespace

extern "C" {

int mpcqp_fleet_step(mpcqp_ws* nominal, mpcqp_ws* relaxed, const mpcqp_fleet* f, void* stream) {
  int rc = check_fleet(nominal, relaxed, f);
  if (rc) return rc;
  if (f->vehicles == 0) return MPCQP_OK;
  return enqueue_step(nominal, relaxed, f, static_cast<hipStream_t>(stream));
}

}  // extern "C"

namespace mpcqp {
int fleet_buffers(mpcqp_ws* nominal, mpcqp_ws* relaxed, hipStream_t s) {
  int rc = ensure_buffers(nominal, true, needs_state(nominal->p), s);
  if (rc == MPCQP_OK) rc = ensure_buffers(relaxed, true, needs_state(relaxed->p), s);
  return rc;
}

// the fused loop with the swarm's trigger (tr.max_replans > 0, mpcqp_swarm_loop) or without; nullptr
// looper (mid / long horizons, reproducible or debug mode): *fused = false, nothing enqueued
int enqueue_fleet_loop(mpcqp_ws* nominal, mpcqp_ws* relaxed, const mpcqp_fleet* f, int steps, const LoopTrigger& tr,
                       hipStream_t s, bool* fused) {
  const mpcqp::fleet_loop_t loop = mpcqp::fleet_looper(nominal->p);
  *fused = loop && mpcqp::fleet_looper(relaxed->p) == loop;
  if (!*fused) return MPCQP_OK;
  nominal->built_B = -1;  // as mpcqp_fleet_step: a later mpcqp_solve needs its own build
  relaxed->built_B = -1;
  nominal->in_x0 = nominal->in_ref = nominal->in_up = nullptr;
  relaxed->in_x0 = relaxed->in_ref = relaxed->in_up = nullptr;
  hipLaunchKernelGGL(k_store_params, dim3(1), dim3(kWave), 0, s, nominal->p, relaxed->p, nominal->dparams);
  LoopTrigger tro = tr;
  // longest first only when the vehicles outnumber the wave slots (2 per SIMD): with every vehicle
  // resident at once the order only changes which vehicles share a SIMD (measured: no gain)
  if (nominal->cus > 0 && f->vehicles > 8 * nominal->cus) {
    hipLaunchKernelGGL(k_fleet_order, dim3(1), dim3(kOrderBuckets), 0, s, *f, nominal->dorder);
    tro.order = nominal->dorder;
  }
  tro.pair = mpcqp::use_pairs(nominal, f->vehicles);
  loop(s, nominal->dparams, *f, steps, tro);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return fail(MPCQP_E_HIP, std::string("k_fleet_loop launch: ") + hipGetErrorString(e));
  return MPCQP_OK;
}
}  // namespace mpcqp

extern "C" {

int mpcqp_fleet_loop(mpcqp_ws* nominal, mpcqp_ws* relaxed, const mpcqp_fleet* f, int steps, void* stream) {
  int rc = check_fleet(nominal, relaxed, f);
  if (rc) return rc;
  if (steps < 0) return fail(MPCQP_E_ARG, "steps must be >= 0");
  if (f->vehicles == 0 || steps == 0) return MPCQP_OK;
  hipStream_t s = static_cast<hipStream_t>(stream);
  bool fused = false;
  rc = mpcqp::enqueue_fleet_loop(nominal, relaxed, f, steps, mpcqp::LoopTrigger{0.0, 0, nullptr, nullptr}, s, &fused);
  if (rc || fused) return rc;
  return run_graph(nominal, relaxed, f, steps, s);  // mid / long horizons, reproducible or debug mode
}

int mpcqp_fleet_run(mpcqp_ws* nominal, mpcqp_ws* relaxed, const mpcqp_fleet* f, int steps, int use_graph,
                    void* stream) {
  int rc = check_fleet(nominal, relaxed, f);
  if (rc) return rc;
  if (steps < 0) return fail(MPCQP_E_ARG, "steps must be >= 0");
  if (f->vehicles == 0 || steps == 0) return MPCQP_OK;
  hipStream_t s = static_cast<hipStream_t>(stream);
  if (use_graph) return run_graph(nominal, relaxed, f, steps, s);
  for (int i = 0; i < steps; ++i) {
    rc = enqueue_step(nominal, relaxed, f, s);
    if (rc) return rc;
  }
  return MPCQP_OK;
}

}  // extern "C"
