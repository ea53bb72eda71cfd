// mpcqp_swarm.hip -- BASELINE config 5 on the device: the fleet closed loop with a per-step
// replan trigger and the replanning itself, no host round trip.
//
// One mpcqp_swarm_step = one closed-loop step of every vehicle, then replanning of the vehicles
// the step left off their reference:
//   fleet step          mpcqp_fleet.hip: window + nominal/relaxed MPC + plant + path_idx + goal
//                       (src/pipeline/control_stage.py:100-150)
//   k_swarm_trigger     the roadmap trigger of README.md:146-148: a RUNNING vehicle farther than
//                       replan_distance from ref[path_idx], or one the step ABORTED (QP unsolved
//                       after relaxation), with replans left -> MPCQP_FLEET_REPLAN_*, the RRT*
//                       problem {current position -> goal} and the PCG64 state of its next seed
//   k_swarm_plan        RRT* tree growth (rrt_star.py:201-248), flagged vehicles only
//   k_swarm_paths       path extraction + shortcut pruning (rrt_star.py:245-262, 376-389)
//   k_swarm_smooth      centripetal Catmull-Rom (rrt_star.py:104-159, 264-283)
//   k_swarm_refbuild    build_reference (ref_builder.py:10-22) into a staging buffer
//   k_swarm_commit      success -> the new reference, path_idx 0, RUNNING (pose, speed and u_prev
//                       carry over); failure -> the vehicle keeps its reference (RUNNING) or stays
//                       ABORTED; either way one replan is used
// Every replanning kernel exits at once for an unflagged vehicle, so a step without replans
// costs a handful of empty launches; mpcqp_swarm_run replays the whole step as a hipGraph.
// mpcqp_swarm_loop runs the same thing as max_replans + 1 launches of the fused fleet loop
// (k_fleet_loop with the trigger: each vehicle steps until it triggers or ends) with the replanning
// kernels in between -- no per-step launches.
#include "mpcqp_build.h"
#include "mpcqp_plan.h"
#include "mpcqp_refbuild.h"

namespace {
using mpcqp::fail;

constexpr int kCatmullCap = 4096;  // deduplicated points per path (LDS of k_swarm_smooth / k_catmull_rom)
constexpr int kRefCap = 6144;      // smoothed points per path that build_reference stages in LDS

__device__ __forceinline__ bool replanning(int ph) {
  return ph == MPCQP_FLEET_REPLAN_RUNNING || ph == MPCQP_FLEET_REPLAN_ABORTED;
}

__global__ __launch_bounds__(kWave) void k_swarm_trigger(mpcqp_fleet f, mpcqp_swarm s) {
#pragma clang fp contract(off)
  const int v = blockIdx.x * kWave + threadIdx.x;
  if (v >= f.vehicles) return;
  const int ph = f.phase[v];
  const int used = s.replans[v];
  if (used < 0 || used >= s.max_replans) return;
  bool go = ph == MPCQP_FLEET_ABORTED;
  if (ph == MPCQP_FLEET_RUNNING && s.replan_distance > 0.0) {
    const int len = f.ref_len[v], pi = f.path_idx[v];
    if (len >= 1 && len <= f.ref_stride && pi >= 0 && pi < len) {
      go = swarm_off_track(f.state[(size_t)v * 4], f.state[(size_t)v * 4 + 1],
                           f.ref_global + ((size_t)v * f.ref_stride + pi) * 4, s.replan_distance);
    }
  }
  if (!go) return;
  f.phase[v] = ph == MPCQP_FLEET_ABORTED ? MPCQP_FLEET_REPLAN_ABORTED : MPCQP_FLEET_REPLAN_RUNNING;
  double* sg = s.start_goal + 4 * (size_t)v;
  sg[0] = f.state[(size_t)v * 4];
  sg[1] = f.state[(size_t)v * 4 + 1];
  sg[2] = f.goal[(size_t)v * 2];
  sg[3] = f.goal[(size_t)v * 2 + 1];
}

__global__ __launch_bounds__(kPlanThreads) void k_swarm_plan(mpcqp_fleet f, mpcqp_swarm s) {
  extern __shared__ double lds[];
  __shared__ PlanSmem sm;
  const int v = blockIdx.x;
  if (v >= f.vehicles || !replanning(f.phase[v])) return;
  const int M = s.rrt.max_iterations + 2;
  const uint64_t* rs = s.rng_table + ((size_t)v * s.max_replans + s.replans[v]) * 4;
  rrt_grow_one(s.rrt, s.occupancy, s.start_goal + 4 * (size_t)v, nullptr, rs, s.nodes + (size_t)v * M * 4,
               s.count + v, s.meta + 2 * (size_t)v, lds, sm);
}

__global__ __launch_bounds__(kPlanThreads) void k_swarm_paths(mpcqp_fleet f, mpcqp_swarm s) {
  extern __shared__ double lds[];
  __shared__ PlanSmem sm;
  const int v = blockIdx.x;
  if (v >= f.vehicles || !replanning(f.phase[v])) return;
  const size_t M = (size_t)s.rrt.max_iterations + 2;
  rrt_extract_one(s.rrt, s.prune, s.occupancy, s.nodes + (size_t)v * M * 4, s.count + v, s.meta + 2 * (size_t)v,
                  s.raw + (size_t)v * M * 2, s.raw_len + v, s.pruned + (size_t)v * M * 2, s.pruned_len + v, lds, sm);
}

// the planner's final path (rrt_star.py:264-283): smoothed when spline_samples > 1 and the
// smoothing gives >= 2 points, else the pruned path; smooth_len -1 = over capacity
__device__ void final_path(const double* pruned, int plen, const mpcqp_swarm& s, double* out, int32_t* out_len,
                           double* lds) {
  const int lane = threadIdx.x;
  int k = -2;
  if (plen >= 2 && s.spline_samples > 1)
    k = catmull_rom_one(pruned, plen, s.spline_samples, s.spline_alpha, s.dedupe_tol, lds, kCatmullCap, out,
                        s.path_cap);
  if (k == -1) {
    if (lane == 0) *out_len = -1;
    return;
  }
  if (k < 2) {  // no (usable) smoothing: the pruned path itself
    if (plen > s.path_cap) {
      if (lane == 0) *out_len = -1;
      return;
    }
    for (int i = lane; i < 2 * plen; i += kWave) out[i] = pruned[i];
    k = plen;
  }
  if (lane == 0) *out_len = k;
}

__global__ __launch_bounds__(kWave) void k_swarm_smooth(mpcqp_fleet f, mpcqp_swarm s) {
  extern __shared__ double lds[];
  const int v = blockIdx.x;
  if (v >= f.vehicles || !replanning(f.phase[v])) return;
  const size_t M = (size_t)s.rrt.max_iterations + 2;
  final_path(s.pruned + (size_t)v * M * 2, s.pruned_len[v], s, s.smooth + (size_t)v * s.path_cap * 2,
             s.smooth_len + v, lds);
}

__global__ __launch_bounds__(kWave) void k_swarm_refbuild(mpcqp_fleet f, mpcqp_swarm s) {
  extern __shared__ double lds[];
  const int v = blockIdx.x;
  if (v >= f.vehicles || !replanning(f.phase[v])) return;
  const int P = s.smooth_len[v];
  if (P < 1) {  // no plan (or over capacity): nothing to build
    if (threadIdx.x == 0) s.new_len[v] = 0;
    return;
  }
  build_reference_one(s.smooth + (size_t)v * s.path_cap * 2, P, s.path_cap < kRefCap ? s.path_cap : kRefCap,
                      s.desired_speed, s.horizon, s.dt, f.ref_stride, s.new_ref + (size_t)v * f.ref_stride * 4,
                      s.new_len + v, lds);
}

__global__ __launch_bounds__(kWave) void k_swarm_commit(mpcqp_fleet f, mpcqp_swarm s) {
  const int v = blockIdx.x;
  if (v >= f.vehicles) return;
  const int ph = f.phase[v];
  if (!replanning(ph)) return;
  const int len = s.new_len[v];
  const bool ok = s.meta[2 * (size_t)v + 1] >= 0 && len >= 1 && len <= f.ref_stride;
  if (ok) {
    double* dst = const_cast<double*>(f.ref_global) + (size_t)v * f.ref_stride * 4;
    const double* src = s.new_ref + (size_t)v * f.ref_stride * 4;
    for (int i = threadIdx.x; i < 4 * len; i += kWave) dst[i] = src[i];
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    const int used = s.replans[v];
    if (s.replan_step) s.replan_step[(size_t)v * s.max_replans + used] = ok ? f.steps[v] : -f.steps[v] - 1;
    s.replans[v] = used + 1;
    if (ok) {
      const_cast<int32_t*>(f.ref_len)[v] = len;
      f.path_idx[v] = 0;
      f.phase[v] = MPCQP_FLEET_RUNNING;
    } else {
      f.phase[v] = ph == MPCQP_FLEET_REPLAN_ABORTED ? MPCQP_FLEET_ABORTED : MPCQP_FLEET_RUNNING;
    }
  }
}

// batched smoothing of V paths (mpcqp_catmull_rom): path v = in[v * in_stride .. + in_len[v]) points
__global__ __launch_bounds__(kWave) void k_catmull_rom(int V, const double* __restrict__ in, const int32_t* __restrict__ in_len,
                                                       int in_stride, int samples, double alpha, double tol,
                                                       double* __restrict__ out, int32_t* __restrict__ out_len,
                                                       int out_stride) {
  extern __shared__ double lds[];
  const int v = blockIdx.x;
  if (v >= V) return;
  const int k = catmull_rom_one(in + (size_t)v * in_stride * 2, in_len[v], samples, alpha, tol, lds, kCatmullCap,
                                out + (size_t)v * out_stride * 2, out_stride);
  if (threadIdx.x == 0) out_len[v] = k;
}

int check_swarm(const mpcqp_fleet* f, const mpcqp_swarm* s) {
  if (!s) return fail(MPCQP_E_ARG, "null swarm");
  if (s->max_replans < 0) return fail(MPCQP_E_ARG, "max_replans must be >= 0");
  if (s->rrt.max_iterations < 1 || s->rrt.max_iterations > kMaxPlanIterations)
    return fail(MPCQP_E_ARG, "max_iterations outside [1, " + std::to_string(kMaxPlanIterations) + "]");
  if (s->rrt.width < 2 || s->rrt.height < 2) return fail(MPCQP_E_ARG, "grid must be at least 2 x 2");
  if (s->path_cap < 2) return fail(MPCQP_E_ARG, "path_cap must be >= 2");
  if (s->horizon < 1 || s->horizon > MPCQP_MAX_HORIZON) return fail(MPCQP_E_HORIZON, "bad swarm horizon");
  if (!(s->dt > 0.0) || !(s->desired_speed > 0.0)) return fail(MPCQP_E_ARG, "dt and desired_speed must be > 0");
  if (s->max_replans > 0 &&
      (!s->occupancy || !s->rng_table || !s->replans || !s->start_goal || !s->nodes || !s->count || !s->meta ||
       !s->raw || !s->raw_len || !s->pruned || !s->pruned_len || !s->smooth || !s->smooth_len || !s->new_ref ||
       !s->new_len))
    return fail(MPCQP_E_ARG, "null swarm buffer");
  (void)f;
  return MPCQP_OK;
}

size_t plan_lds(const mpcqp_rrt_params& p) {
  return ((size_t)(p.max_iterations + 2) * (3 * sizeof(double) + sizeof(int)) + 7) / 8 * 8;
}

struct ReplanLds {
  size_t plan, paths, smooth, refbuild;
  explicit ReplanLds(const mpcqp_swarm* s)
      : plan(plan_lds(s->rrt)),
        paths((size_t)(s->rrt.max_iterations + 2) * 2 * sizeof(double)),
        smooth(sizeof(double) * 2 * kCatmullCap),
        refbuild(sizeof(double) * 3 * (size_t)(s->path_cap < kRefCap ? s->path_cap : kRefCap)) {}
};

// dynamic-LDS limits of the replanning kernels (outside any stream capture)
int set_replan_attrs(const mpcqp_swarm* s) {
  const ReplanLds l(s);
  auto big = [](const void* k, size_t bytes) {
    return bytes > 65536 ? hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes) : hipSuccess;
  };
  hipError_t e = big(reinterpret_cast<const void*>(&k_swarm_plan), l.plan);
  if (e == hipSuccess) e = big(reinterpret_cast<const void*>(&k_swarm_paths), l.paths);
  if (e == hipSuccess) e = big(reinterpret_cast<const void*>(&k_swarm_smooth), l.smooth);
  if (e == hipSuccess) e = big(reinterpret_cast<const void*>(&k_swarm_refbuild), l.refbuild);
  if (e != hipSuccess) return fail(MPCQP_E_HIP, std::string("hipFuncSetAttribute: ") + hipGetErrorString(e));
  return MPCQP_OK;
}

// trigger (unless the fused loop already flagged the vehicles) + the replanning kernels
int enqueue_replan(const mpcqp_fleet* f, const mpcqp_swarm* s, hipStream_t st, bool trigger = true) {
  const int V = f->vehicles;
  if (s->max_replans == 0 || V == 0) return MPCQP_OK;
  const mpcqp_fleet fv = *f;
  const mpcqp_swarm sv = *s;
  const ReplanLds l(s);
  const size_t lp = l.plan, lx = l.paths, lc = l.smooth, lr = l.refbuild;
  if (trigger) hipLaunchKernelGGL(k_swarm_trigger, dim3((V + kWave - 1) / kWave), dim3(kWave), 0, st, fv, sv);
  hipLaunchKernelGGL(k_swarm_plan, dim3(V), dim3(kPlanThreads), lp, st, fv, sv);
  hipLaunchKernelGGL(k_swarm_paths, dim3(V), dim3(kPlanThreads), lx, st, fv, sv);
  hipLaunchKernelGGL(k_swarm_smooth, dim3(V), dim3(kWave), lc, st, fv, sv);
  hipLaunchKernelGGL(k_swarm_refbuild, dim3(V), dim3(kWave), lr, st, fv, sv);
  hipLaunchKernelGGL(k_swarm_commit, dim3(V), dim3(kWave), 0, st, fv, sv);
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) return fail(MPCQP_E_HIP, std::string("swarm replan launch: ") + hipGetErrorString(e));
  return MPCQP_OK;
}

}  // namespace

extern "C" {

int mpcqp_catmull_rom(int V, const double* in, const int32_t* in_len, int in_stride, int samples, double alpha,
                      double dedupe_tol, double* out, int32_t* out_len, int out_stride, void* stream) {
  if (V < 0) return fail(MPCQP_E_ARG, "V must be >= 0");
  if (V == 0) return MPCQP_OK;
  if (!in || !in_len || !out || !out_len) return fail(MPCQP_E_ARG, "null argument");
  if (in_stride < 1 || out_stride < 1) return fail(MPCQP_E_ARG, "strides must be >= 1");
  const size_t lds = sizeof(double) * 2 * kCatmullCap;
  hipError_t e = hipSuccess;
  if (lds > 65536)
    e = hipFuncSetAttribute(reinterpret_cast<const void*>(&k_catmull_rom), hipFuncAttributeMaxDynamicSharedMemorySize,
                            (int)lds);
  if (e != hipSuccess) return fail(MPCQP_E_HIP, std::string("hipFuncSetAttribute: ") + hipGetErrorString(e));
  hipLaunchKernelGGL(k_catmull_rom, dim3(V), dim3(kWave), lds, static_cast<hipStream_t>(stream), V, in, in_len,
                     in_stride, samples, alpha, dedupe_tol, out, out_len, out_stride);
  e = hipGetLastError();
  if (e != hipSuccess) return fail(MPCQP_E_HIP, std::string("k_catmull_rom launch: ") + hipGetErrorString(e));
  return MPCQP_OK;
}

int mpcqp_swarm_step(mpcqp_ws* nominal, mpcqp_ws* relaxed, const mpcqp_fleet* f, const mpcqp_swarm* s, void* stream) {
  int rc = check_swarm(f, s);
  if (rc) return rc;
  rc = mpcqp_fleet_step(nominal, relaxed, f, stream);
  if (rc) return rc;
  hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
  hipStream_t st = static_cast<hipStream_t>(stream);
  if (hipStreamIsCapturing(st, &cs) == hipSuccess && cs == hipStreamCaptureStatusNone) {
    rc = set_replan_attrs(s);
    if (rc) return rc;
  }
  return enqueue_replan(f, s, st);
}

int mpcqp_swarm_loop(mpcqp_ws* nominal, mpcqp_ws* relaxed, const mpcqp_fleet* f, const mpcqp_swarm* s, void* stream) {
  int rc = check_swarm(f, s);
  if (rc) return rc;
  rc = mpcqp_fleet_loop(nominal, relaxed, f, 0, stream);  // the fleet's checks (no work at 0 steps)
  if (rc) return rc;
  if (f->vehicles == 0) return MPCQP_OK;
  hipStream_t st = static_cast<hipStream_t>(stream);
  if (s->max_replans > 0 && (rc = set_replan_attrs(s)) != MPCQP_OK) return rc;
  // max_replans + 1 rounds: every vehicle runs until it triggers or ends, the flagged ones are
  // replanned; a vehicle's r-th trigger comes in round r - 1, so the last round triggers none
  const mpcqp::LoopTrigger tr{s->replan_distance, s->max_replans, s->replans, s->start_goal};
  for (int r = 0; r <= s->max_replans; ++r) {
    bool fused = false;
    rc = mpcqp::enqueue_fleet_loop(nominal, relaxed, f, f->max_steps, tr, st, &fused);
    if (rc) return rc;
    if (!fused)  // mid / long horizons, reproducible or debug mode: the stepped swarm to the end
      return mpcqp_swarm_run(nominal, relaxed, f, s, f->max_steps, 1, stream);
    if (r < s->max_replans && (rc = enqueue_replan(f, s, st, false)) != MPCQP_OK) return rc;
  }
  return MPCQP_OK;
}

int mpcqp_swarm_run(mpcqp_ws* nominal, mpcqp_ws* relaxed, const mpcqp_fleet* f, const mpcqp_swarm* s, int steps,
                    int use_graph, void* stream) {
  int rc = check_swarm(f, s);
  if (rc) return rc;
  if (steps < 0) return fail(MPCQP_E_ARG, "steps must be >= 0");
  if (!f || f->vehicles == 0 || steps == 0) return mpcqp_fleet_run(nominal, relaxed, f, 0, 0, stream);
  hipStream_t user = static_cast<hipStream_t>(stream);
  if (!use_graph) {
    for (int i = 0; i < steps; ++i) {
      rc = mpcqp_swarm_step(nominal, relaxed, f, s, stream);
      if (rc) return rc;
    }
    return MPCQP_OK;
  }
  hipStream_t s2 = nullptr;
  hipEvent_t ev = nullptr;
  hipGraph_t g = nullptr;
  hipGraphExec_t ex = nullptr;
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
  if (e == hipSuccess && ((rc = set_replan_attrs(s)) != MPCQP_OK ||  // outside the capture
                          (rc = mpcqp::fleet_buffers(nominal, relaxed, user)) != MPCQP_OK)) {
    cleanup();
    return rc;
  }
  if (e == hipSuccess) e = hipStreamBeginCapture(s2, hipStreamCaptureModeThreadLocal);
  if (e != hipSuccess) {
    cleanup();
    return fail(MPCQP_E_HIP, std::string("swarm graph setup: ") + hipGetErrorString(e));
  }
  rc = mpcqp_swarm_step(nominal, relaxed, f, s, s2);
  e = hipStreamEndCapture(s2, &g);
  if (rc == MPCQP_OK && e != hipSuccess)
    rc = fail(MPCQP_E_HIP, std::string("hipStreamEndCapture: ") + hipGetErrorString(e));
  if (rc == MPCQP_OK) {
    e = hipGraphInstantiate(&ex, g, nullptr, nullptr, 0);
    for (int i = 0; e == hipSuccess && i < steps; ++i) e = hipGraphLaunch(ex, s2);
    if (e == hipSuccess) e = hipEventRecord(ev, s2);
    if (e == hipSuccess) e = hipStreamWaitEvent(user, ev, 0);
    if (e == hipSuccess) e = hipStreamSynchronize(s2);
    if (e != hipSuccess) rc = fail(MPCQP_E_HIP, std::string("swarm graph replay: ") + hipGetErrorString(e));
  }
  cleanup();
  return rc;
}

}  // extern "C"
