// mpcqp.hip -- MI355X (gfx950) batched bicycle-MPC QP solver: the C-ABI, K1 and the launcher table.
//
// Replaces the reference's per-step MPC solve (CagriCatik/RRT-MPC):
//   K1 k_build     window -> LTV model      (src/control/mpc_controller.py:59-70,108,
//                                            src/control/vehicle_model.py:24-45)
//   K2 k_solve<N>  ONE fused kernel per horizon (mpcqp_solve.h): setup (condensing + OSQP Ruiz
//                  scaling, mpc_controller.py:53-117), ADMM (OSQP's iteration with the settings
//                  of :119-132), polish + outputs/status (:133-141), with no kernel boundary in
//                  between.
// One 64-lane wavefront owns one QP (B QPs -> B single-wave workgroups).  Vectors are distributed
// one decision variable per lane; the banded constraint operators are DPP lane shifts; the KKT
// inverse lives one row per lane in registers and the scaled Hessian in LDS, so the scaled
// problem never leaves the CU (the per-QP state buffer is written only with debug_state).
// The algorithm is restated sequentially in oracle/mpcqp_cpu.c -- see DESIGN.md.
#include "mpcqp_build.h"

#include <chrono>
#include <cstdlib>
#include <mutex>
#ifdef MPCQP_ONLY_N
#include "mpcqp_solve.h"  // development builds: one horizon, one translation unit
#endif


namespace {
using mpcqp::Launch;

// ------------------------------------------------------------------ K1: build
// Per QP (one wave, lane k = horizon step k in [0, N]) on caller-provided windows; the body
// (unwrap + linearize) is build_qp in mpcqp_build.h.
__global__ __launch_bounds__(kWave) void k_build(mpcqp_params p, int B, const double* __restrict__ x0,
                                                 const double* __restrict__ ref,
                                                 const double* __restrict__ u_prev,
                                                 double* __restrict__ model) {
  const int b = blockIdx.x;
  const int lane = threadIdx.x;
  if (b >= B) return;
  const int N = p.horizon;
  const double* rb = ref + (size_t)b * (N + 1) * 4;
  const double x0l = lane < 4 ? x0[(size_t)b * 4 + lane] : 0.0;
  const double upl = (lane >= 4 && lane < 6 && u_prev) ? u_prev[(size_t)b * 2 + lane - 4] : 0.0;
  if (N + 1 > kWave) {  // long windows: chunks of 64 rows
    build_qp_long(
        p, lane,
        [&](int k, double& rx, double& ry, double& ryaw, double& rv) {
          rx = rb[4 * k + 0];
          ry = rb[4 * k + 1];
          ryaw = rb[4 * k + 2];
          rv = rb[4 * k + 3];
        },
        x0l, upl, model + (size_t)b * model_stride(N));
    return;
  }
  double rx = 0.0, ry = 0.0, ryaw = 0.0, rv = 0.0;
  if (lane <= N) {
    rx = rb[4 * lane + 0];
    ry = rb[4 * lane + 1];
    ryaw = rb[4 * lane + 2];
    rv = rb[4 * lane + 3];
  }
  build_qp(p, lane, rx, ry, ryaw, rv, x0l, upl, model + (size_t)b * model_stride(N));
}

// ------------------------------------------------------------------ test hook: wave primitives
// out[op][lane] for the 64-lane input `in` (tests/test_gpu_parity.py checks them with numpy).
__global__ __launch_bounds__(kWave) void k_wave_ops(const double* __restrict__ in, double* __restrict__ out) {
  const int lane = threadIdx.x;
  const double v = in[lane];
  const double a = fabs(v);
  out[0 * kWave + lane] = scan_add(v, lane);
  out[1 * kWave + lane] = rscan_add(v, lane);
  out[2 * kWave + lane] = scan_max(a, lane);
  out[3 * kWave + lane] = rscan_max(a, lane);
  out[4 * kWave + lane] = wave_sum(v);
  out[5 * kWave + lane] = wave_max(a);
  out[6 * kWave + lane] = shr2(v);
  out[7 * kWave + lane] = shl2(v);
  out[8 * kWave + lane] = dpp<kWaveShr1>(v);
  out[9 * kWave + lane] = readlane(v, 37);
}

#ifdef MPCQP_ONLY_N  // development builds: instantiate a single horizon
#define MPCQP_L(N) ((N) == MPCQP_ONLY_N ? &mpcqp::launch_solve<MPCQP_ONLY_N> : nullptr)
#else
#define MPCQP_L(N) &mpcqp::launch_solve<N>
#endif
const mpcqp::launcher_t kLaunchers[MPCQP_WIDE_MIN_HORIZON] = {
    nullptr,     MPCQP_L(1),  MPCQP_L(2),  MPCQP_L(3),  MPCQP_L(4),  MPCQP_L(5),  MPCQP_L(6),  MPCQP_L(7),
    MPCQP_L(8),  MPCQP_L(9),  MPCQP_L(10), MPCQP_L(11), MPCQP_L(12), MPCQP_L(13), MPCQP_L(14), MPCQP_L(15),
    MPCQP_L(16), MPCQP_L(17), MPCQP_L(18), MPCQP_L(19), MPCQP_L(20), MPCQP_L(21), MPCQP_L(22), MPCQP_L(23),
    MPCQP_L(24), MPCQP_L(25), MPCQP_L(26), MPCQP_L(27), MPCQP_L(28), MPCQP_L(29), MPCQP_L(30), MPCQP_L(31),
    MPCQP_L(32)};
#undef MPCQP_L
#ifdef MPCQP_ONLY_N
#define MPCQP_F(N) ((N) == MPCQP_ONLY_N ? &mpcqp::launch_fleet_loop<MPCQP_ONLY_N> : nullptr)
#else
#define MPCQP_F(N) &mpcqp::launch_fleet_loop<N>
#endif
const mpcqp::fleet_loop_t kFleetLoops[MPCQP_WIDE_MIN_HORIZON] = {
    nullptr,     MPCQP_F(1),  MPCQP_F(2),  MPCQP_F(3),  MPCQP_F(4),  MPCQP_F(5),  MPCQP_F(6),  MPCQP_F(7),
    MPCQP_F(8),  MPCQP_F(9),  MPCQP_F(10), MPCQP_F(11), MPCQP_F(12), MPCQP_F(13), MPCQP_F(14), MPCQP_F(15),
    MPCQP_F(16), MPCQP_F(17), MPCQP_F(18), MPCQP_F(19), MPCQP_F(20), MPCQP_F(21), MPCQP_F(22), MPCQP_F(23),
    MPCQP_F(24), MPCQP_F(25), MPCQP_F(26), MPCQP_F(27), MPCQP_F(28), MPCQP_F(29), MPCQP_F(30), MPCQP_F(31),
    MPCQP_F(32)};
#undef MPCQP_F
#ifdef MPCQP_ONLY_N
#define MPCQP_P(N) ((N) == MPCQP_ONLY_N ? &mpcqp::launch_solve_pair<MPCQP_ONLY_N> : nullptr)
#else
#define MPCQP_P(N) &mpcqp::launch_solve_pair<N>
#endif
constexpr int kPairMaxHorizon = 15;  // n = 2N <= 30: two QPs per wave
const mpcqp::pair_launcher_t kPairLaunchers[kPairMaxHorizon + 1] = {
    nullptr,    MPCQP_P(1),  MPCQP_P(2),  MPCQP_P(3),  MPCQP_P(4),  MPCQP_P(5),  MPCQP_P(6),  MPCQP_P(7),
    MPCQP_P(8), MPCQP_P(9),  MPCQP_P(10), MPCQP_P(11), MPCQP_P(12), MPCQP_P(13), MPCQP_P(14), MPCQP_P(15)};
#undef MPCQP_P
#ifdef MPCQP_ONLY_N
#define MPCQP_S(N) ((N) == MPCQP_ONLY_N ? &mpcqp::launch_serve<MPCQP_ONLY_N> : nullptr)
#else
#define MPCQP_S(N) &mpcqp::launch_serve<N>
#endif
const mpcqp::serve_t kServers[MPCQP_WIDE_MIN_HORIZON] = {
    nullptr,     MPCQP_S(1),  MPCQP_S(2),  MPCQP_S(3),  MPCQP_S(4),  MPCQP_S(5),  MPCQP_S(6),  MPCQP_S(7),
    MPCQP_S(8),  MPCQP_S(9),  MPCQP_S(10), MPCQP_S(11), MPCQP_S(12), MPCQP_S(13), MPCQP_S(14), MPCQP_S(15),
    MPCQP_S(16), MPCQP_S(17), MPCQP_S(18), MPCQP_S(19), MPCQP_S(20), MPCQP_S(21), MPCQP_S(22), MPCQP_S(23),
    MPCQP_S(24), MPCQP_S(25), MPCQP_S(26), MPCQP_S(27), MPCQP_S(28), MPCQP_S(29), MPCQP_S(30), MPCQP_S(31),
    MPCQP_S(32)};
#undef MPCQP_S

// per-QP doubles of the solver state buffer (debug state of the one-wave kernel, the workspace
// of the long-horizon kernel)
size_t ws_state_stride(int N, bool wide) {
  if (!wide) return (size_t)state_stride(N);
  const size_t w = mpcqp::wide_stride(N);
  const size_t m = N <= MPCQP_MID_MAX_HORIZON ? mpcqp::mid_stride(N) : 0;
  return w > m ? w : m;
}

void launch_mid(hipStream_t s, const Launch& L) {
  switch (mpcqp::mid_bucket(L.p->horizon)) {  // N >= 33: N = 32 runs the one-wave kernel
    case 40: mpcqp::launch_solve_mid<40>(s, L); break;
    case 48: mpcqp::launch_solve_mid<48>(s, L); break;
    case 56: mpcqp::launch_solve_mid<56>(s, L); break;
    default: mpcqp::launch_solve_mid<64>(s, L); break;
  }
}

thread_local std::string g_err;
using mpcqp::fail;

int check_params(const mpcqp_params* p) {
  if (!p) return fail(MPCQP_E_ARG, "null params");
  if (p->horizon < 1 || p->horizon > MPCQP_MAX_HORIZON)
    return fail(MPCQP_E_HORIZON, "horizon " + std::to_string(p->horizon) + " outside [1, " +
                                     std::to_string(MPCQP_MAX_HORIZON) + "]");
  if (!mpcqp::launcher(*p)) return fail(MPCQP_E_HORIZON, "horizon not compiled into this build");
  if (p->reproducible != 0 && p->reproducible != 1) return fail(MPCQP_E_ARG, "reproducible must be 0 or 1");
  if (!(p->dt > 0.0) || !(p->wheelbase_px > 0.0)) return fail(MPCQP_E_ARG, "dt and wheelbase_px must be > 0");
  if (p->method != MPCQP_METHOD_ADMM && p->method != MPCQP_METHOD_NEWTON) return fail(MPCQP_E_ARG, "bad method");
  if (p->max_iter < 1 || p->check_termination < 1 || p->adaptive_rho_interval < 1 || p->polish_max_iter < 0 ||
      p->scaling < 0)
    return fail(MPCQP_E_ARG, "bad iteration settings");
  if (!(p->rho > 0.0) || !(p->sigma >= 0.0) || !(p->alpha > 0.0 && p->alpha < 2.0))
    return fail(MPCQP_E_ARG, "bad rho/sigma/alpha");
  return MPCQP_OK;
}

}  // namespace

namespace mpcqp {
int fail(int code, const std::string& msg) {
  g_err = msg;
  return code;
}
bool wide_solve(const mpcqp_params& p) { return p.horizon >= MPCQP_WIDE_MIN_HORIZON || p.reproducible != 0; }
launcher_t launcher(const mpcqp_params& p) {
  const int horizon = p.horizon;
  if (horizon < 1 || horizon > MPCQP_MAX_HORIZON) return nullptr;
  // fast mode up to MPCQP_MID_MAX_HORIZON: the mid kernel; beyond it, and in reproducible mode, the
  // workgroup kernel that restates the C code operation for operation
  if (wide_solve(p)) return p.reproducible == 0 && horizon <= MPCQP_MID_MAX_HORIZON ? &launch_mid : &launch_solve_wide;
  return horizon < MPCQP_WIDE_MIN_HORIZON ? kLaunchers[horizon] : nullptr;
}
int ensure_buffers(mpcqp_ws* ws, bool model, bool state, hipStream_t s) {
  model = model && !ws->model;
  state = state && !ws->state;
  if (!model && !state) return MPCQP_OK;
  hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
  if (s && hipStreamIsCapturing(s, &cs) == hipSuccess && cs != hipStreamCaptureStatusNone)
    return fail(MPCQP_E_STATE, "the workspace's model/state buffers are allocated at their first use, which "
                               "cannot be inside a stream capture: run the call once uncaptured first");
  int cur = -1;
  hipError_t e = hipGetDevice(&cur);
  if (e == hipSuccess && cur != ws->device) e = hipSetDevice(ws->device);
  const int N = ws->p.horizon;
  if (e == hipSuccess && model) e = hipMalloc(&ws->model, sizeof(double) * (size_t)model_stride(N) * (size_t)ws->max_batch);
  if (e == hipSuccess && state)
    e = hipMalloc(&ws->state, sizeof(double) * ws_state_stride(N, wide_solve(ws->p)) * (size_t)ws->max_batch);
  if (cur >= 0 && cur != ws->device) (void)hipSetDevice(cur);
  if (e != hipSuccess) return fail(MPCQP_E_HIP, std::string("hipMalloc (workspace buffers): ") + hipGetErrorString(e));
  return MPCQP_OK;
}
serve_t server(const mpcqp_params& p) {
  if (wide_solve(p) || p.debug_state || p.horizon < 1 || p.horizon >= MPCQP_WIDE_MIN_HORIZON) return nullptr;
  return kServers[p.horizon];
}
bool use_pairs(const mpcqp_ws* ws, int count) {
  const mpcqp_params& p = ws->p;
  if (wide_solve(p) || p.debug_state || p.horizon < 1 || p.horizon > kPairMaxHorizon || !kPairLaunchers[p.horizon])
    return false;
  if (ws->pairing == MPCQP_PAIR_ON) return true;
  if (ws->pairing == MPCQP_PAIR_OFF) return false;
  // auto: once the QPs outnumber the wave slots (2 per SIMD): below that every QP has a wave of its
  // own, and pairing would only make each wave wait for the slower of its two QPs
  return ws->cus > 0 && count > 8 * ws->cus;
}
fleet_loop_t fleet_looper(const mpcqp_params& p) {
  if (wide_solve(p) || p.debug_state || p.horizon < 1 || p.horizon >= MPCQP_WIDE_MIN_HORIZON) return nullptr;
  return kFleetLoops[p.horizon];
}
}  // namespace mpcqp

extern "C" {

int mpcqp_version(void) { return MPCQP_ABI_VERSION; }

const char* mpcqp_last_error(void) { return g_err.c_str(); }

int mpcqp_num_rows(int horizon) { return 5 * horizon + 1; }

int mpcqp_model_stride(int horizon) { return model_stride(horizon); }

int mpcqp_create(const mpcqp_params* p, int max_batch, int device, mpcqp_ws** ws) {
  if (!ws) return fail(MPCQP_E_ARG, "null ws");
  *ws = nullptr;
  int rc = check_params(p);
  if (rc) return rc;
  if (max_batch < 1) return fail(MPCQP_E_ARG, "max_batch must be >= 1");
  hipError_t e = hipSetDevice(device);
  if (e != hipSuccess) return fail(MPCQP_E_HIP, std::string("hipSetDevice: ") + hipGetErrorString(e));
  mpcqp_ws* w = new (std::nothrow) mpcqp_ws();
  if (!w) return fail(MPCQP_E_ARG, "out of host memory");
  w->p = *p;
  w->max_batch = max_batch;
  w->device = device;
  w->built_B = -1;
  w->model = nullptr;
  w->state = nullptr;
  w->in_x0 = w->in_ref = w->in_up = nullptr;
  w->dparams = nullptr;
  w->dorder = nullptr;
  w->stage_in = w->stage_in_d = nullptr;
  w->stage_out = w->stage_out_d = nullptr;
  w->stage_stream = nullptr;
  w->serve_box = w->serve_box_d = nullptr;
  w->serve_seq = 0;
  w->serve_live = false;
  w->serve_broken = false;
  w->serve_fault = 0;
  w->pairing = MPCQP_PAIR_AUTO;
  if (hipDeviceGetAttribute(&w->cus, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess) w->cus = 0;
  e = hipMalloc(&w->dparams, 2 * sizeof(mpcqp_params));
  if (e == hipSuccess) e = hipMalloc(&w->dorder, sizeof(int32_t) * (size_t)max_batch);
  if (e != hipSuccess) {
    if (w->dparams) (void)hipFree(w->dparams);
    delete w;
    return fail(MPCQP_E_HIP, std::string("hipMalloc: ") + hipGetErrorString(e));
  }
  // the long-horizon kernels always read the model block and work in the state buffer
  if (mpcqp::wide_solve(*p) && (rc = mpcqp::ensure_buffers(w, true, true, nullptr)) != MPCQP_OK) {
    mpcqp_destroy(w);
    return rc;
  }
  *ws = w;
  g_err.clear();
  return MPCQP_OK;
}

static void serve_stop(mpcqp_ws* ws);

int mpcqp_set_params(mpcqp_ws* ws, const mpcqp_params* p) {
  if (!ws) return fail(MPCQP_E_ARG, "null ws");
  int rc = check_params(p);
  if (rc) return rc;
  serve_stop(ws);  // a running B = 1 server holds the old parameter block
  if (p->horizon != ws->p.horizon) return fail(MPCQP_E_HORIZON, "set_params cannot change the horizon");
  if (p->reproducible != ws->p.reproducible) return fail(MPCQP_E_ARG, "set_params cannot change reproducible");
  ws->p = *p;
  // A build belongs to the parameter block it was made with (the fused solve derives its LTV model
  // from the params in effect at solve time, the K1 kernel from those at build time): new params
  // invalidate it, and the next mpcqp_solve needs a new mpcqp_build.
  ws->built_B = -1;
  ws->in_x0 = ws->in_ref = ws->in_up = nullptr;
  return MPCQP_OK;
}

void mpcqp_destroy(mpcqp_ws* ws) {
  if (!ws) return;
  (void)hipSetDevice(ws->device);
  serve_stop(ws);  // first: the frees below synchronise the device, which waits for a resident wave
  if (ws->stage_stream) (void)hipStreamSynchronize(ws->stage_stream);
  (void)hipFree(ws->model);
  (void)hipFree(ws->state);
  (void)hipFree(ws->dparams);
  (void)hipFree(ws->dorder);
  if (ws->serve_box) (void)hipHostFree(ws->serve_box);
  if (ws->stage_in) (void)hipHostFree(ws->stage_in);
  if (ws->stage_out) (void)hipHostFree(ws->stage_out);
  if (ws->stage_stream) (void)hipStreamDestroy(ws->stage_stream);
  delete ws;
}

int mpcqp_set_pairing(mpcqp_ws* ws, int mode) {
  if (!ws) return fail(MPCQP_E_ARG, "null ws");
  if (mode != MPCQP_PAIR_OFF && mode != MPCQP_PAIR_ON && mode != MPCQP_PAIR_AUTO)
    return fail(MPCQP_E_ARG, "pairing mode must be MPCQP_PAIR_OFF, _ON or _AUTO");
  ws->pairing = mode;
  return MPCQP_OK;
}

int mpcqp_build(mpcqp_ws* ws, int B, const double* x0, const double* ref, const double* u_prev, void* stream) {
  if (!ws || !x0 || !ref) return fail(MPCQP_E_ARG, "null argument");
  if (B < 0 || B > ws->max_batch) return fail(MPCQP_E_BATCH, "batch exceeds workspace capacity");
  ws->built_B = B;
  ws->in_x0 = ws->in_ref = ws->in_up = nullptr;
  if (B == 0) return MPCQP_OK;
  // The one-wave solve builds the model itself (K1 fused into k_solve: the model block never
  // touches HBM); the K1 kernel runs only for the long-horizon solve and for inspection builds.
  if (!mpcqp::wide_solve(ws->p) && !ws->p.debug_state) {
    ws->in_x0 = x0;
    ws->in_ref = ref;
    ws->in_up = u_prev;
    return MPCQP_OK;
  }
  hipStream_t s = static_cast<hipStream_t>(stream);
  const int rc = mpcqp::ensure_buffers(ws, true, mpcqp::needs_state(ws->p), s);
  if (rc) {
    ws->built_B = -1;
    return rc;
  }
  hipLaunchKernelGGL(k_build, dim3(B), dim3(kWave), 0, s, ws->p, B, x0, ref, u_prev, ws->model);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return fail(MPCQP_E_HIP, std::string("k_build launch: ") + hipGetErrorString(e));
  return MPCQP_OK;
}

int mpcqp_solve(mpcqp_ws* ws, int B, double* u0, double* X, double* U, int32_t* status, int32_t* iters,
                uint8_t* active, void* stream) {
  if (!ws || !status) return fail(MPCQP_E_ARG, "null argument");
  if (B != ws->built_B) return fail(MPCQP_E_STATE, "mpcqp_solve B differs from the last mpcqp_build");
  if (B == 0) return MPCQP_OK;
  hipStream_t s = static_cast<hipStream_t>(stream);
  Launch L{&ws->p, B, ws->model, ws->state, u0, X, U, status, iters, active, nullptr};
  L.x0 = ws->in_x0;
  L.ref = ws->in_ref;
  L.u_prev = ws->in_up;
  if (!(L.ref && mpcqp::use_pairs(ws, B) && kPairLaunchers[ws->p.horizon](s, L))) mpcqp::launcher(ws->p)(s, L);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return fail(MPCQP_E_HIP, std::string("k_solve launch: ") + hipGetErrorString(e));
  return MPCQP_OK;
}

// ------------------------------------------------------------------ B = 1 path
// Output block layout of the staged path (include/mpcqp.h): u0 | X | U | status | iters | active.
static void stage_offsets(int N, int32_t off[7]) {
  off[0] = 0;                        // u0     2 f64
  off[1] = 16;                       // X      4 x (N+1) f64
  off[2] = off[1] + 32 * (N + 1);    // U      2 x N f64
  off[3] = off[2] + 16 * N;          // status i32
  off[4] = off[3] + 4;               // iters  4 x i32
  off[5] = off[4] + 16;              // active 5N+1 u8
  off[6] = off[5] + 5 * N + 1;       // total bytes
}

int mpcqp_stage(mpcqp_ws* ws, double** in, void** out, int32_t offsets[6]) {
  if (!ws) return fail(MPCQP_E_ARG, "null ws");
  const int N = ws->p.horizon;
  int32_t off[7];
  stage_offsets(N, off);
  if (!ws->stage_in) {
    int cur = -1;
    hipError_t e = hipGetDevice(&cur);
    if (e == hipSuccess && cur != ws->device) e = hipSetDevice(ws->device);
    const unsigned fl = hipHostMallocMapped | hipHostMallocCoherent;
    double* hin = nullptr;
    uint8_t* hout = nullptr;
    void* din = nullptr;
    void* dout = nullptr;
    hipStream_t st = nullptr;
    if (e == hipSuccess) e = hipHostMalloc((void**)&hin, sizeof(double) * (size_t)(4 * (N + 1) + 6), fl);
    if (e == hipSuccess) e = hipHostMalloc((void**)&hout, (size_t)off[6], fl);
    if (e == hipSuccess) e = hipHostGetDevicePointer(&din, hin, 0);
    if (e == hipSuccess) e = hipHostGetDevicePointer(&dout, hout, 0);
    // the highest stream priority: the runtime gives each priority its own hardware queues, so the
    // resident server wave of mpcqp_solve_served never sits in a queue that torch's (default-priority)
    // streams share -- a queued packet behind a resident kernel waits until it leaves
    // (MPCQP_SERVE_PRIORITY=default: the default priority instead -- diagnostics, tools/diag/serve_block.py)
    int least = 0, greatest = 0;
    if (e == hipSuccess) e = hipDeviceGetStreamPriorityRange(&least, &greatest);
    const char* pr = std::getenv("MPCQP_SERVE_PRIORITY");
    const bool dflt = pr && std::strcmp(pr, "default") == 0;
    if (e == hipSuccess) e = hipStreamCreateWithPriority(&st, hipStreamNonBlocking, dflt ? least : greatest);
    if (cur >= 0 && cur != ws->device) (void)hipSetDevice(cur);
    if (e != hipSuccess) {
      if (hin) (void)hipHostFree(hin);
      if (hout) (void)hipHostFree(hout);
      return fail(MPCQP_E_HIP, std::string("B=1 staging blocks: ") + hipGetErrorString(e));
    }
    std::memset(hin, 0, sizeof(double) * (size_t)(4 * (N + 1) + 6));
    std::memset(hout, 0, (size_t)off[6]);
    ws->stage_in = hin;
    ws->stage_in_d = static_cast<double*>(din);
    ws->stage_out = hout;
    ws->stage_out_d = static_cast<uint8_t*>(dout);
    ws->stage_stream = st;
  }
  if (in) *in = ws->stage_in;
  if (out) *out = ws->stage_out;
  if (offsets)
    for (int i = 0; i < 6; ++i) offsets[i] = off[i];
  return MPCQP_OK;
}

int mpcqp_solve_staged(mpcqp_ws* ws) {
  if (!ws) return fail(MPCQP_E_ARG, "null ws");
  if (!ws->stage_in) return fail(MPCQP_E_STATE, "mpcqp_solve_staged before mpcqp_stage");
  const int N = ws->p.horizon;
  int32_t off[7];
  stage_offsets(N, off);
  const double* d = ws->stage_in_d;
  uint8_t* o = ws->stage_out_d;
  hipStream_t s = ws->stage_stream;
  int rc = mpcqp_build(ws, 1, d, d + 4, d + 4 + 4 * (N + 1), s);
  if (rc) return rc;
  rc = mpcqp_solve(ws, 1, reinterpret_cast<double*>(o + off[0]), reinterpret_cast<double*>(o + off[1]),
                   reinterpret_cast<double*>(o + off[2]), reinterpret_cast<int32_t*>(o + off[3]),
                   reinterpret_cast<int32_t*>(o + off[4]), o + off[5], s);
  if (rc) return rc;
  const hipError_t e = hipStreamSynchronize(s);
  if (e != hipSuccess) return fail(MPCQP_E_DEVICE, std::string("hipStreamSynchronize: ") + hipGetErrorString(e));
  return MPCQP_OK;
}

// One resident server wave per device: a workspace that raises a request first stops another
// workspace's live server on its device (the drop-in alternates nominal, relaxed and scaling-10
// workspaces), so two resident waves never hold two hardware queues and a switch costs one stop and
// one launch.  g_server[d]: the workspace whose server may be live on device d.
static std::mutex g_serve_mu;
static mpcqp_ws* g_server[64] = {};

// The B = 1 server (k_serve): ends a live server wave (kServeStop) and waits for it.  The caller
// holds ws->serve_mu.
static void serve_stop_locked(mpcqp_ws* ws) {
  {
    std::lock_guard<std::mutex> lk(g_serve_mu);
    if (g_server[ws->device & 63] == ws) g_server[ws->device & 63] = nullptr;
  }
  if (!ws->serve_live) return;
  auto* box = static_cast<mpcqp::ServeBox*>(ws->serve_box);
  __atomic_store_n(&box->req, mpcqp::kServeStop, __ATOMIC_RELEASE);
  (void)hipStreamSynchronize(ws->stage_stream);
  // the next request continues the sequence after the last completed one
  __atomic_store_n(&box->req, __atomic_load_n(&box->done, __ATOMIC_ACQUIRE), __ATOMIC_RELEASE);
  ws->serve_seq = __atomic_load_n(&box->done, __ATOMIC_ACQUIRE);
  ws->serve_live = false;
}
static void serve_stop(mpcqp_ws* ws) {
  if (!ws) return;
  std::lock_guard<std::mutex> own(ws->serve_mu);
  serve_stop_locked(ws);
}

int mpcqp_solve_served(mpcqp_ws* ws) {
  if (!ws) return fail(MPCQP_E_ARG, "null ws");
  if (!ws->stage_in) return fail(MPCQP_E_STATE, "mpcqp_solve_served before mpcqp_stage");
  if (ws->serve_broken)
    return fail(MPCQP_E_DEVICE, "B=1 server: an earlier request went unanswered; this workspace is unusable");
  const mpcqp::serve_t launch = mpcqp::server(ws->p);
  if (!launch) return mpcqp_solve_staged(ws);  // long horizons, reproducible or debug builds
  // this workspace's server state is ours for the whole call; another workspace's wave on this device
  // is stopped only when its own lock is free (try-lock, taken under g_serve_mu so that workspace cannot
  // be destroyed in between): a workspace busy in its own served call on another thread keeps its wave,
  // which leaves 2 ms after its last request -- two resident waves for that while, never a stop
  // that overwrites a pending request
  std::unique_lock<std::mutex> own(ws->serve_mu);
  mpcqp_ws* other = nullptr;
  std::unique_lock<std::mutex> other_lk;
  {
    std::lock_guard<std::mutex> lk(g_serve_mu);
    other = g_server[ws->device & 63];
    if (other && other != ws) {
      other_lk = std::unique_lock<std::mutex>(other->serve_mu, std::try_to_lock);
      if (!other_lk.owns_lock()) other = nullptr;
    } else {
      other = nullptr;
    }
    g_server[ws->device & 63] = ws;
  }
  if (other) serve_stop_locked(other);
  if (other_lk.owns_lock()) other_lk.unlock();
  if (!ws->serve_box) {
    int cur = -1;
    hipError_t e = hipGetDevice(&cur);
    if (e == hipSuccess && cur != ws->device) e = hipSetDevice(ws->device);
    void* box = nullptr;
    void* dbox = nullptr;
    if (e == hipSuccess) e = hipHostMalloc(&box, sizeof(mpcqp::ServeBox), hipHostMallocMapped | hipHostMallocCoherent);
    if (e == hipSuccess) e = hipHostGetDevicePointer(&dbox, box, 0);
    if (cur >= 0 && cur != ws->device) (void)hipSetDevice(cur);
    if (e != hipSuccess) {
      if (box) (void)hipHostFree(box);
      return fail(MPCQP_E_HIP, std::string("B=1 server mailbox: ") + hipGetErrorString(e));
    }
    std::memset(box, 0, sizeof(mpcqp::ServeBox));
    ws->serve_box = box;
    ws->serve_box_d = dbox;
    ws->serve_seq = 0;
  }
  auto* box = static_cast<mpcqp::ServeBox*>(ws->serve_box);
  uint32_t seq = ws->serve_seq + 1;
  if (seq == mpcqp::kServeStop) seq = 1;
  ws->serve_seq = seq;
  __atomic_store_n(&box->req, seq, __ATOMIC_RELEASE);  // after the caller's input writes (x86: ordered)
  auto relaunch = [&]() -> int {
    int32_t off[7];
    stage_offsets(ws->p.horizon, off);
    mpcqp::ServeLaunch L{};
    L.box = static_cast<mpcqp::ServeBox*>(ws->serve_box_d);
    L.in = ws->stage_in_d;
    L.out = ws->stage_out_d;
    for (int i = 0; i < 6; ++i) L.off[i] = off[i];
    L.idle_ticks = 200000;  // 2 ms at 100 MHz
    if (ws->serve_fault == 1) {  // mpcqp_debug_serve_fault: this launch is refused
      ws->serve_fault = 0;
      return fail(MPCQP_E_HIP, "k_serve launch: refused (mpcqp_debug_serve_fault)");
    }
    launch(ws->stage_stream, ws->p, L);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return fail(MPCQP_E_HIP, std::string("k_serve launch: ") + hipGetErrorString(e));
    ws->serve_live = true;
    return MPCQP_OK;
  };
  // the wave leaves 2 ms after its last request: past 1.5 ms, look before trusting it is there
  const auto now = std::chrono::steady_clock::now();
  if (ws->serve_live && now - ws->serve_last > std::chrono::microseconds(1500) &&
      hipStreamQuery(ws->stage_stream) == hipSuccess)
    ws->serve_live = false;
  if (!ws->serve_live) {
    const int rc = relaunch();
    if (rc) return rc;
  }
  // wait for done == seq; every ~20 us of waiting, look whether the wave left (idle timeout racing
  // this request, or a fault) and relaunch it
  long spins = 0;
  const auto t_start = now;
  while (__atomic_load_n(&box->done, __ATOMIC_ACQUIRE) != seq) {
    __builtin_ia32_pause();
    if (++spins % 2048 == 0) {
      const hipError_t q = hipStreamQuery(ws->stage_stream);
      if (q == hipSuccess) {  // the wave has exited
        if (__atomic_load_n(&box->done, __ATOMIC_ACQUIRE) == seq) break;
        ws->serve_live = false;
        const int rc = relaunch();
        if (rc) return rc;
      } else if (q != hipErrorNotReady) {
        ws->serve_live = false;
        return fail(MPCQP_E_DEVICE, std::string("B=1 server: ") + hipGetErrorString(q));
      }
      if (std::chrono::steady_clock::now() - t_start > std::chrono::seconds(30)) {
        // a stuck or queued wave may still write the output block: tell it to leave, and refuse every
        // later request on this workspace rather than hand its blocks to a new one
        __atomic_store_n(&box->req, mpcqp::kServeStop, __ATOMIC_RELEASE);
        ws->serve_live = false;
        ws->serve_broken = true;
        {  // no other workspace's request stops (or counts on) this wave any more
          std::lock_guard<std::mutex> lk(g_serve_mu);
          if (g_server[ws->device & 63] == ws) g_server[ws->device & 63] = nullptr;
        }
        return fail(MPCQP_E_DEVICE, "B=1 server: no answer within 30 s");
      }
    }
  }
  ws->serve_last = std::chrono::steady_clock::now();
  return MPCQP_OK;
}

const double* mpcqp_model_buffer(const mpcqp_ws* ws) { return ws ? ws->model : nullptr; }

const double* mpcqp_state_buffer(const mpcqp_ws* ws) { return ws ? ws->state : nullptr; }

int mpcqp_state_stride(int horizon) { return (int)ws_state_stride(horizon, horizon >= MPCQP_WIDE_MIN_HORIZON); }

int mpcqp_ws_state_stride(const mpcqp_ws* ws) {
  if (!ws) return fail(MPCQP_E_ARG, "null ws");
  return (int)ws_state_stride(ws->p.horizon, mpcqp::wide_solve(ws->p));
}

int mpcqp_debug_serve_fault(mpcqp_ws* ws, int mode) {
  if (!ws) return fail(MPCQP_E_ARG, "null ws");
  if (mode == 1) {  // the next server launch is refused
    ws->serve_fault = 1;
    return MPCQP_OK;
  }
  if (mode == 2) {  // the live wave leaves now, behind the host's back (serve_live stays set)
    if (!ws->serve_live) return fail(MPCQP_E_STATE, "no live server");
    auto* box = static_cast<mpcqp::ServeBox*>(ws->serve_box);
    __atomic_store_n(&box->req, mpcqp::kServeStop, __ATOMIC_RELEASE);
    (void)hipStreamSynchronize(ws->stage_stream);
    __atomic_store_n(&box->req, __atomic_load_n(&box->done, __ATOMIC_ACQUIRE), __ATOMIC_RELEASE);
    return MPCQP_OK;
  }
  if (mode == 3) return ws->serve_live ? 1 : 0;  // query: a server is believed resident
  return fail(MPCQP_E_ARG, "mode must be 1, 2 or 3");
}

#ifdef MPCQP_STAMPS
typedef hipError_t (*StampsFn)(unsigned long long* out32, int reset);
static StampsFn g_stamp_parts[64];
static int g_n_stamp_parts = 0;
extern "C" void mpcqp_register_stamps(StampsFn f) {
  if (g_n_stamp_parts < 64) g_stamp_parts[g_n_stamp_parts++] = f;
}
#endif

int mpcqp_debug_stamps(unsigned long long* out32, int reset) {
#ifdef MPCQP_STAMPS
  hipError_t e = hipDeviceSynchronize();
  if (e == hipSuccess && out32) e = hipMemcpyFromSymbol(out32, HIP_SYMBOL(g_stamps), sizeof(unsigned long long) * 32);
  if (e == hipSuccess && reset) {
    unsigned long long z[32] = {0};
    e = hipMemcpyToSymbol(HIP_SYMBOL(g_stamps), z, sizeof(z));
  }
  for (int i = 0; i < g_n_stamp_parts && e == hipSuccess; ++i) e = g_stamp_parts[i](out32, reset);
  if (e != hipSuccess) return fail(MPCQP_E_HIP, std::string("stamps: ") + hipGetErrorString(e));
  return MPCQP_OK;
#else
  (void)out32;
  (void)reset;
  return fail(MPCQP_E_ARG, "not a -DMPCQP_STAMPS diagnostic build");
#endif
}

int mpcqp_debug_wave_ops(const double* in, double* out, void* stream) {
  if (!in || !out) return fail(MPCQP_E_ARG, "null argument");
  hipLaunchKernelGGL(k_wave_ops, dim3(1), dim3(kWave), 0, static_cast<hipStream_t>(stream), in, out);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return fail(MPCQP_E_HIP, std::string("k_wave_ops launch: ") + hipGetErrorString(e));
  return MPCQP_OK;
}

}  // extern "C"
