// mpcqp.hip -- MI355X (gfx950) batched bicycle-MPC QP solver: kernels + C-ABI.
//
// Replaces the reference's per-step MPC solve (CagriCatik/RRT-MPC):
//   K1  k_build  : window -> LTV model      (src/control/mpc_controller.py:59-70,108,
//                                            src/control/vehicle_model.py:24-45)
//   K2a k_setup  : condense + Ruiz scaling   (mpc_controller.py:53-117 -> OSQP setup)
//   K2b k_admm   : OSQP ADMM iterations      (mpc_controller.py:119-132, settings :121-131)
//   K2c k_finish : polish + outputs/status   (OSQP polish; mpc_controller.py:133-141)
// One 64-lane wavefront owns one QP (B QPs -> B single-wave workgroups).  Every
// vector of the iteration is distributed one decision variable per lane; the
// structured constraint operators are DPP wave scans; the KKT inverse lives one
// row per lane in registers.  The phases are separate kernels so that each gets
// its own register budget (occupancy); the per-QP solver state between them
// (scaled Hessian + scaling vectors, ~20 KB at N=20) stays L2/MALL resident.
// The algorithm is restated sequentially in oracle/mpcqp_cpu.c -- see DESIGN.md.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <new>
#include <string>
#include <type_traits>
#include <utility>

#include "../../include/mpcqp.h"

namespace {

constexpr int kWave = 64;
constexpr double kPi = 3.141592653589793;
constexpr double kTwoPi = 6.283185307179586;
constexpr double kMinScaling = 1e-4;
constexpr double kMaxScaling = 1e4;
constexpr double kRhoMin = 1e-6;
constexpr double kRhoMax = 1e6;
constexpr double kDivTol = 1e-30;

// ------------------------------------------------------------------ layouts
__host__ __device__ constexpr int model_stride(int N) { return ((11 * N + 10) + 7) / 8 * 8; }

// Solver state per QP (doubles):
//   [0, n*n)            Pbar, symmetric, row-major
//   lane fields         kF* x 64 doubles, lane-contiguous
//   scalars             cscale, admm_ok, admm_it, n_fact
enum LaneField {
  kFq = 0,
  kFD,
  kFx,
  kFE0,
  kFE1,
  kFE2,
  kFlo0,
  kFlo1,
  kFlo2,
  kFhi0,
  kFhi1,
  kFhi2,
  kFw0,
  kFw1,
  kFw2,
  kNumFields
};
__host__ __device__ constexpr int state_lane_off(int N) { return (4 * N * N + 7) / 8 * 8; }
__host__ __device__ constexpr int state_scal_off(int N) { return state_lane_off(N) + kNumFields * kWave; }
__host__ __device__ constexpr int state_stride(int N) { return state_scal_off(N) + 8; }

// ------------------------------------------------------------------ wave primitives (DPP)
template <int CTRL>
__device__ __forceinline__ double dpp(double v) {
  const int lo = __builtin_amdgcn_update_dpp(0, __double2loint(v), CTRL, 0xf, 0xf, true);
  const int hi = __builtin_amdgcn_update_dpp(0, __double2hiint(v), CTRL, 0xf, 0xf, true);
  return __hiloint2double(hi, lo);
}
__device__ __forceinline__ double readlane(double v, int l) {
  return __hiloint2double(__builtin_amdgcn_readlane(__double2hiint(v), l),
                          __builtin_amdgcn_readlane(__double2loint(v), l));
}
constexpr int kRowShr1 = 0x111, kRowShr2 = 0x112, kRowShr4 = 0x114, kRowShr8 = 0x118;
constexpr int kRowShl1 = 0x101, kRowShl2 = 0x102, kRowShl4 = 0x104, kRowShl8 = 0x108;
constexpr int kWaveShr1 = 0x138, kWaveShl1 = 0x130;

// inclusive prefix sum over lanes 0..lane (zero-filled row shifts + row totals)
__device__ __forceinline__ double scan_add(double v, int lane) {
  v += dpp<kRowShr1>(v);
  v += dpp<kRowShr2>(v);
  v += dpp<kRowShr4>(v);
  v += dpp<kRowShr8>(v);
  const double t0 = readlane(v, 15), t1 = readlane(v, 31), t2 = readlane(v, 47);
  const int row = lane >> 4;
  double off = row >= 1 ? t0 : 0.0;
  if (row >= 2) off += t1;
  if (row >= 3) off += t2;
  return v + off;
}
// inclusive suffix sum over lanes lane..63
__device__ __forceinline__ double rscan_add(double v, int lane) {
  v += dpp<kRowShl1>(v);
  v += dpp<kRowShl2>(v);
  v += dpp<kRowShl4>(v);
  v += dpp<kRowShl8>(v);
  const double t1 = readlane(v, 16), t2 = readlane(v, 32), t3 = readlane(v, 48);
  const int row = lane >> 4;
  double off = row <= 2 ? t3 : 0.0;
  if (row <= 1) off += t2;
  if (row <= 0) off += t1;
  return v + off;
}
// inclusive prefix / suffix max of non-negative values
__device__ __forceinline__ double scan_max(double v, int lane) {
  v = fmax(v, dpp<kRowShr1>(v));
  v = fmax(v, dpp<kRowShr2>(v));
  v = fmax(v, dpp<kRowShr4>(v));
  v = fmax(v, dpp<kRowShr8>(v));
  const double t0 = readlane(v, 15), t1 = readlane(v, 31), t2 = readlane(v, 47);
  const int row = lane >> 4;
  double off = row >= 1 ? t0 : 0.0;
  if (row >= 2) off = fmax(off, t1);
  if (row >= 3) off = fmax(off, t2);
  return fmax(v, off);
}
__device__ __forceinline__ double rscan_max(double v, int lane) {
  v = fmax(v, dpp<kRowShl1>(v));
  v = fmax(v, dpp<kRowShl2>(v));
  v = fmax(v, dpp<kRowShl4>(v));
  v = fmax(v, dpp<kRowShl8>(v));
  const double t1 = readlane(v, 16), t2 = readlane(v, 32), t3 = readlane(v, 48);
  const int row = lane >> 4;
  double off = row <= 2 ? t3 : 0.0;
  if (row <= 1) off = fmax(off, t2);
  if (row <= 0) off = fmax(off, t1);
  return fmax(v, off);
}
// wave-uniform sum / max (row scans + four row totals)
__device__ __forceinline__ double wave_sum(double v) {
  v += dpp<kRowShr1>(v);
  v += dpp<kRowShr2>(v);
  v += dpp<kRowShr4>(v);
  v += dpp<kRowShr8>(v);
  return (readlane(v, 15) + readlane(v, 31)) + (readlane(v, 47) + readlane(v, 63));
}
__device__ __forceinline__ double wave_max(double v) {  // v >= 0
  v = fmax(v, dpp<kRowShr1>(v));
  v = fmax(v, dpp<kRowShr2>(v));
  v = fmax(v, dpp<kRowShr4>(v));
  v = fmax(v, dpp<kRowShr8>(v));
  return fmax(fmax(readlane(v, 15), readlane(v, 31)), fmax(readlane(v, 47), readlane(v, 63)));
}
// lane i <- lane i-2 (0 for i < 2);  lane i <- lane i+2 (0 past the wave)
__device__ __forceinline__ double shr2(double v) { return dpp<kWaveShr1>(dpp<kWaveShr1>(v)); }
__device__ __forceinline__ double shl2(double v) { return dpp<kWaveShl1>(dpp<kWaveShl1>(v)); }
__device__ __forceinline__ bool wave_any(bool b) { return __ballot(b) != 0ull; }

// ---- register broadcasts for the dense row-per-lane products (no LDS)
// A dense product over a vector v distributed one element per lane needs every lane to see
// every v_j.  bcast() replicates each 16-lane row of v into all four rows with the gfx950
// permlane swaps (w[c] lane l = v[16c + (l & 15)]); v_fmac_f64 with DPP row_newbcast:L then
// reads lane L of each row's copy as its multiplicand, so a broadcast-FMA is ONE VALU
// instruction with no memory latency.  Must run with all 64 lanes active.
template <int NW>  // rows needed: ceil(n / 16)
__device__ __forceinline__ void bcast(double v, double w[4]) {
  const int lo = __double2loint(v), hi = __double2hiint(v);
  const auto l16 = __builtin_amdgcn_permlane16_swap(lo, lo, false, false);  // rows {0,0,2,2} / {1,1,3,3}
  const auto h16 = __builtin_amdgcn_permlane16_swap(hi, hi, false, false);
  const auto la = __builtin_amdgcn_permlane32_swap(l16[0], l16[0], false, false);  // row 0 x4 / row 2 x4
  const auto ha = __builtin_amdgcn_permlane32_swap(h16[0], h16[0], false, false);
  w[0] = __hiloint2double(ha[0], la[0]);
  if constexpr (NW > 1) {
    const auto lb = __builtin_amdgcn_permlane32_swap(l16[1], l16[1], false, false);  // row 1 x4 / row 3 x4
    const auto hb = __builtin_amdgcn_permlane32_swap(h16[1], h16[1], false, false);
    w[1] = __hiloint2double(hb[0], lb[0]);
    if constexpr (NW > 3) w[3] = __hiloint2double(hb[1], lb[1]);
  }
  if constexpr (NW > 2) w[2] = __hiloint2double(ha[1], la[1]);
  // DPP reads of a VGPR need two wait states after its VALU write; tie the pad to w
  if constexpr (NW == 1) asm volatile("s_nop 1" : "+v"(w[0]));
  if constexpr (NW == 2) asm volatile("s_nop 1" : "+v"(w[0]), "+v"(w[1]));
  if constexpr (NW == 3) asm volatile("s_nop 1" : "+v"(w[0]), "+v"(w[1]), "+v"(w[2]));
  if constexpr (NW == 4) asm volatile("s_nop 1" : "+v"(w[0]), "+v"(w[1]), "+v"(w[2]), "+v"(w[3]));
}
// acc += w[lane 16*row + L] * m   (one v_fmac_f64_dpp)
template <int L>
__device__ __forceinline__ void fmac_bc(double& acc, double w, double m) {
  asm("v_fmac_f64_dpp %0, %1, %2 row_newbcast:%3 row_mask:0xf bank_mask:0xf" : "+v"(acc) : "v"(w), "v"(m), "i"(L));
}
// compile-time loop: f(std::integral_constant<int, I>) for I in [B, E)
template <int B, int E>
struct Unroll {
  template <class F>
  __device__ __forceinline__ static void run(F&& f) {
    if constexpr (B < E) {
      f(std::integral_constant<int, B>{});
      Unroll<B + 1, E>::run(f);
    }
  }
};

// Every kernel runs one wavefront per workgroup, and the LDS operations of one wavefront
// execute in program order: a broadcast through LDS needs only a compiler-level ordering
// point (wavefront-scope fence), not an s_barrier with its lgkmcnt(0) drain.
__device__ __forceinline__ void lds_sync() { __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront"); }

// ------------------------------------------------------------------ diagnostic stamps
// Built only with -DMPCQP_STAMPS (never in the measured library): per-phase s_memtime
// cycle sums, flushed once per wave into g_stamps[] (read by mpcqp_debug_stamps).
#ifdef MPCQP_STAMPS
__device__ unsigned long long g_stamps[16];
struct Stamps {
  unsigned long long acc[6] = {0, 0, 0, 0, 0, 0};
  unsigned long long t = 0;
  __device__ __forceinline__ void begin() {
    __builtin_amdgcn_sched_barrier(0);
    t = __builtin_amdgcn_s_memtime();
    __builtin_amdgcn_sched_barrier(0);
  }
  __device__ __forceinline__ void end(int s) {
    __builtin_amdgcn_sched_barrier(0);
    acc[s] += __builtin_amdgcn_s_memtime() - t;
    __builtin_amdgcn_sched_barrier(0);
  }
  __device__ __forceinline__ void flush(int base) {
    if (threadIdx.x == 0)
      for (int s = 0; s < 6; ++s) atomicAdd(&g_stamps[base + s], acc[s]);
  }
};
#else
struct Stamps {
  __device__ __forceinline__ void begin() {}
  __device__ __forceinline__ void end(int) {}
  __device__ __forceinline__ void flush(int) {}
};
#endif

__device__ __forceinline__ double limit_scaling(double v) {
  return v < kMinScaling ? 1.0 : (v > kMaxScaling ? kMaxScaling : v);
}

// numpy float mod (npy_divmod) for b > 0
__device__ __forceinline__ double np_mod(double a, double b) {
  double m = fmod(a, b);
  if (m != 0.0) {
    if (m < 0.0) m += b;
  } else {
    m = 0.0;
  }
  return m;
}

// ------------------------------------------------------------------ K1: build
// Per QP (one wave, lane k = horizon step k in [0, N]):
//   unwrapped yaw (np.unwrap, mpc_controller.py:60), then linearize() at
//   ref[max(k-1,0)], u = 0 (mpc_controller.py:65-70,108; vehicle_model.py:24-45).
// Model layout per QP (doubles): alpha[N] beta[N] gamma[N] eta[N] sigma[N] c0[N]
// c1[N] ref[(N+1)*4] x0[4] u_prev[2], stride model_stride(N).
__global__ __launch_bounds__(kWave) void k_build(mpcqp_params p, int B, const double* __restrict__ x0,
                                                 const double* __restrict__ ref,
                                                 const double* __restrict__ u_prev,
                                                 double* __restrict__ model) {
  const int b = blockIdx.x;
  const int lane = threadIdx.x;
  if (b >= B) return;
  const int N = p.horizon;
  const int S = model_stride(N);
  const double* rb = ref + (size_t)b * (N + 1) * 4;
  double* mb = model + (size_t)b * S;
  double rx = 0.0, ry = 0.0, ryaw = 0.0, rv = 0.0;
  if (lane <= N) {
    rx = rb[4 * lane + 0];
    ry = rb[4 * lane + 1];
    ryaw = rb[4 * lane + 2];
    rv = rb[4 * lane + 3];
  }
  // np.unwrap: ddmod = mod(dd + pi, 2pi) - pi; boundary fix; zero when |dd| < pi
  const double prev = dpp<kWaveShr1>(ryaw);
  double pc = 0.0;
  if (lane >= 1 && lane <= N) {
    const double dd = ryaw - prev;
    double ddmod = np_mod(dd + kPi, kTwoPi) + (-kPi);
    if (ddmod == -kPi && dd > 0.0) ddmod = kPi;
    pc = ddmod - dd;
    if (fabs(dd) < kPi) pc = 0.0;
  }
  // cumsum in numpy's sequential order (bit-exact)
  double cs = 0.0, mine = 0.0;
  for (int j = 1; j <= N; ++j) {
    cs = cs + readlane(pc, j);
    if (lane == j) mine = cs;
  }
  const double uyaw = lane == 0 ? ryaw : ryaw + mine;
  if (lane <= N) {
    mb[7 * N + 4 * lane + 0] = rx;
    mb[7 * N + 4 * lane + 1] = ry;
    mb[7 * N + 4 * lane + 2] = uyaw;
    mb[7 * N + 4 * lane + 3] = rv;
  }
  // linearisation point of step k: ref[max(k-1, 0)]
  // (DPP must run with every lane active: an exec-masked source lane reads as 0)
  const double psi_m1 = dpp<kWaveShr1>(uyaw);
  const double v_m1 = dpp<kWaveShr1>(rv);
  const double psi = lane == 0 ? uyaw : psi_m1;
  const double v = lane == 0 ? rv : v_m1;
  if (lane < N) {
    const double dt = p.dt, L = p.wheelbase_px;
    const double sec2 = 1.0 / (1.0 * 1.0 + 1e-9);
    double s, c;
    sincos(psi, &s, &c);
    const double al = -dt * v * s;
    const double ga = dt * v * c;
    mb[lane] = al;
    mb[N + lane] = dt * c;
    mb[2 * N + lane] = ga;
    mb[3 * N + lane] = dt * s;
    mb[4 * N + lane] = dt * (v / L) * sec2;
    mb[5 * N + lane] = -al * psi;
    mb[6 * N + lane] = -ga * psi;
  }
  if (lane < 4) mb[11 * N + 4 + lane] = x0[(size_t)b * 4 + lane];
  if (lane >= 4 && lane < 6) mb[11 * N + 4 + lane] = u_prev ? u_prev[(size_t)b * 2 + lane - 4] : 0.0;
}

// ------------------------------------------------------------------ K2a: setup
// Condensing (states and slacks eliminated) + OSQP Ruiz/cost scaling.
// Row slots owned by lane p (p < n = 2N):
//   slot 0: v row (p even): v_{p/2+1} - v0 = dt * sum_{j<=p/2} a_j   (mpc_controller.py:81-82,115-116)
//   slot 1: input row        U_p                                      (:83-86)
//   slot 2: rate row         U_p - U_{p-2} (u_prev at k = 0)          (:89-106)
template <int N>
struct SetupSmem {
  static constexpr int n = 2 * N;
  static constexpr int LD = n + 1;  // odd: conflict-free row and column access
  double P[n * LD];
  double buf[kWave];
  double model[model_stride(N)];
  double pre[4][N + 1];  // prefix sums of alpha, beta, gamma, eta
  double err[N + 1][4];  // free-response tracking error e_m = sx_m - r_m
  double g[n];
};

template <int N>
__global__ __launch_bounds__(kWave) void k_setup(mpcqp_params p, int B, const double* __restrict__ model,
                                                 double* __restrict__ state) {
  constexpr int n = 2 * N;
  constexpr int LD = SetupSmem<N>::LD;
  constexpr int S = model_stride(N);
  __shared__ SetupSmem<N> sm;
  const int b = blockIdx.x;
  const int lane = threadIdx.x;
  if (b >= B) return;
  const bool act = lane < n;
  const bool even = act && ((lane & 1) == 0);
  const int cc = lane & 1;  // 0 = acceleration, 1 = steering
  const double dt = p.dt;

  {
    const double* mb = model + (size_t)b * S;
    for (int i = lane; i < S; i += kWave) sm.model[i] = mb[i];
  }
  __syncthreads();
  const double* al = sm.model;
  const double* be = sm.model + N;
  const double* ga = sm.model + 2 * N;
  const double* et = sm.model + 3 * N;
  const double* si = sm.model + 4 * N;
  const double* c0 = sm.model + 5 * N;
  const double* c1 = sm.model + 6 * N;
  const double* rr = sm.model + 7 * N;
  const double* x0 = sm.model + 11 * N + 4;
  const double* up = sm.model + 11 * N + 8;

  // prefix sums (lanes 0..3, one array each) and free response (lane 4)
  if (lane < 4) {
    const double* a = sm.model + lane * N;
    double acc = 0.0;
    sm.pre[lane][0] = 0.0;
    for (int k = 0; k < N; ++k) {
      acc += a[k];
      sm.pre[lane][k + 1] = acc;
    }
  } else if (lane == 4) {
    double px = x0[0], py = x0[1];
    const double psi = x0[2], v = x0[3];
    for (int m = 1; m <= N; ++m) {
      const int k = m - 1;
      px = px + al[k] * psi + be[k] * v + c0[k];
      py = py + ga[k] * psi + et[k] * v + c1[k];
      sm.err[m][0] = px - rr[4 * m + 0];
      sm.err[m][1] = py - rr[4 * m + 1];
      sm.err[m][2] = psi - rr[4 * m + 2];
      sm.err[m][3] = v - rr[4 * m + 3];
    }
  }
  __syncthreads();

  // ---- condense: column `lane` of H (lane n -> g) by the backward adjoint recursion ----
  // mu_m = W_m s_m + A_m' mu_{m+1};  H[(i,c'), col] = (B_i e_c')' mu_{i+1}
  if (lane <= n) {
    double Q[4][4], QN[4][4];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        Q[i][j] = 0.5 * (p.q[4 * i + j] + p.q[4 * j + i]);
        QN[i][j] = 0.5 * (p.q_terminal[4 * i + j] + p.q_terminal[4 * j + i]);
      }
    const int j = lane >> 1;
    const bool gcol = lane == n;
    const double sj = gcol ? 0.0 : si[j];
    const double pa0 = gcol ? 0.0 : sm.pre[0][j + 1], pb0 = gcol ? 0.0 : sm.pre[1][j + 1];
    const double pg0 = gcol ? 0.0 : sm.pre[2][j + 1], pe0 = gcol ? 0.0 : sm.pre[3][j + 1];
    double mu0 = 0.0, mu1 = 0.0, mu2 = 0.0, mu3 = 0.0;
    for (int m = N; m >= 1; --m) {
      double s0, s1, s2, s3;
      if (gcol) {
        s0 = sm.err[m][0];
        s1 = sm.err[m][1];
        s2 = sm.err[m][2];
        s3 = sm.err[m][3];
      } else if (m > j) {
        if (cc == 0) {
          s0 = dt * (sm.pre[1][m] - pb0);
          s1 = dt * (sm.pre[3][m] - pe0);
          s2 = 0.0;
          s3 = dt;
        } else {
          s0 = sj * (sm.pre[0][m] - pa0);
          s1 = sj * (sm.pre[2][m] - pg0);
          s2 = sj;
          s3 = 0.0;
        }
      } else {
        s0 = s1 = s2 = s3 = 0.0;
      }
      const bool term = m == N;
      auto W = [&](int i, int k) -> double { return term ? QN[i][k] : Q[i][k]; };
      const double w0 = W(0, 0) * s0 + W(0, 1) * s1 + W(0, 2) * s2 + W(0, 3) * s3;
      const double w1 = W(1, 0) * s0 + W(1, 1) * s1 + W(1, 2) * s2 + W(1, 3) * s3;
      const double w2 = W(2, 0) * s0 + W(2, 1) * s1 + W(2, 2) * s2 + W(2, 3) * s3;
      const double w3 = W(3, 0) * s0 + W(3, 1) * s1 + W(3, 2) * s2 + W(3, 3) * s3;
      if (m < N) {
        const double m0 = mu0, m1 = mu1;
        mu0 = w0 + m0;
        mu1 = w1 + m1;
        mu2 = w2 + (mu2 + al[m] * m0 + ga[m] * m1);
        mu3 = w3 + (mu3 + be[m] * m0 + et[m] * m1);
      } else {
        mu0 = w0;
        mu1 = w1;
        mu2 = w2;
        mu3 = w3;
      }
      const double ha = dt * mu3, hd = si[m - 1] * mu2;
      if (gcol) {
        sm.g[2 * (m - 1)] = ha;
        sm.g[2 * (m - 1) + 1] = hd;
      } else {
        sm.P[(2 * (m - 1)) * LD + lane] = ha;
        sm.P[(2 * (m - 1) + 1) * LD + lane] = hd;
      }
    }
    if (!gcol) {
      const double R0 = 0.5 * (p.r[0 * 2 + cc] + p.r[cc * 2 + 0]);
      const double R1 = 0.5 * (p.r[1 * 2 + cc] + p.r[cc * 2 + 1]);
      sm.P[(2 * j) * LD + lane] += R0;
      sm.P[(2 * j + 1) * LD + lane] += R1;
    }
  }
  __syncthreads();

  // ---- unscaled data: P = 2H (column `lane`), q = 2g, folded row bounds ----
  double qv = act ? 2.0 * sm.g[lane] : 0.0;
  double cmax = 0.0;  // running column max of |P|
  if (act) {
#pragma unroll 8
    for (int i = 0; i < n; ++i) {
      const double t = 2.0 * sm.P[i * LD + lane];
      sm.P[i * LD + lane] = t;
      cmax = fmax(cmax, fabs(t));
    }
  }
  double lo[3], hi[3], wt[3], E[3];
  {
    const double off = lane < 2 ? up[cc] : 0.0;
    lo[0] = even ? p.v_bounds[0] - x0[3] : 0.0;
    hi[0] = even ? p.v_bounds[1] - x0[3] : 0.0;
    wt[0] = even ? p.slack_velocity : 0.0;
    lo[1] = act ? p.u_bounds[2 * cc] : 0.0;
    hi[1] = act ? p.u_bounds[2 * cc + 1] : 0.0;
    wt[1] = act ? p.slack_input : 0.0;
    lo[2] = act ? p.du_bounds[2 * cc] + off : 0.0;
    hi[2] = act ? p.du_bounds[2 * cc + 1] + off : 0.0;
    wt[2] = act ? p.slack_rate : 0.0;
    E[0] = even ? 1.0 : 0.0;
    E[1] = act ? 1.0 : 0.0;
    E[2] = act ? 1.0 : 0.0;
  }
  double D = act ? 1.0 : 0.0;
  double cscale = 1.0;

  // ---- Ruiz equilibration + cost scaling (OSQP scale_data, `scaling` iterations) ----
  for (int it = 0; it < p.scaling; ++it) {
    // column norms of [P; A] (first n columns of the KKT matrix)
    const double sufE = rscan_max(E[0], lane);  // max E over v rows >= p/2 (odd lanes carry 0)
    const double e2n = shl2(E[2]);
    double ccol = fmax(E[1], E[2]);
    if (lane + 2 < n) ccol = fmax(ccol, e2n);
    if (even) ccol = fmax(ccol, dt * sufE);
    ccol *= D;
    const double dl = act ? 1.0 / sqrt(limit_scaling(fmax(cmax, ccol))) : 0.0;
    // row norms of A
    const double preD = scan_max(even ? D : 0.0, lane);
    const double Dm2 = shr2(D);
    const double el0 = even ? 1.0 / sqrt(limit_scaling(E[0] * dt * preD)) : 0.0;
    const double el1 = act ? 1.0 / sqrt(limit_scaling(E[1] * D)) : 0.0;
    const double el2 = act ? 1.0 / sqrt(limit_scaling(E[2] * (lane >= 2 ? fmax(D, Dm2) : D))) : 0.0;
    // apply: P <- dl P dl (column `lane`), q <- dl q
    __syncthreads();
    sm.buf[lane] = dl;
    __syncthreads();
    double cm2 = 0.0;
    if (act) {
#pragma unroll 8
      for (int i = 0; i < n; ++i) {
        const double t = sm.P[i * LD + lane] * (sm.buf[i] * dl);
        sm.P[i * LD + lane] = t;
        cm2 = fmax(cm2, fabs(t));
      }
    }
    D *= dl;
    qv *= dl;
    E[0] *= el0;
    E[1] *= el1;
    E[2] *= el2;
    // cost scaling
    const double cn = wave_sum(act ? cm2 : 0.0) / n;
    const double qn = limit_scaling(wave_max(fabs(qv)));
    const double ct = 1.0 / limit_scaling(fmax(cn, qn));
    if (act) {
#pragma unroll 8
      for (int i = 0; i < n; ++i) sm.P[i * LD + lane] *= ct;
    }
    qv *= ct;
    cmax = cm2 * ct;
    cscale *= ct;
  }
  __syncthreads();

  // ---- write the solver state ----
  double* st = state + (size_t)b * state_stride(N);
  bool finite = isfinite(qv) && isfinite(cscale);
  if (act) {
    // symmetric Pbar: the lower-triangle value (computed by column `min`) for both halves
    for (int i = 0; i < n; ++i) {
      const double v = i >= lane ? sm.P[i * LD + lane] : sm.P[lane * LD + i];
      finite = finite && isfinite(v);
      st[i * n + lane] = v;
    }
  }
  double* lf = st + state_lane_off(N);
  double wb[3];
#pragma unroll
  for (int r = 0; r < 3; ++r) {
    lo[r] *= E[r];
    hi[r] *= E[r];
    wb[r] = E[r] > 0.0 ? cscale * wt[r] / (E[r] * E[r]) : 0.0;
    finite = finite && isfinite(lo[r]) && isfinite(hi[r]);
  }
  // non-finite data (NaN/inf in x0, ref or u_prev) -> status MPCQP_NUMERICAL_ERROR
  const bool bad_input = wave_any(!finite);
  lf[kFq * kWave + lane] = qv;
  lf[kFD * kWave + lane] = D;
  lf[kFx * kWave + lane] = 0.0;
#pragma unroll
  for (int r = 0; r < 3; ++r) {
    lf[(kFE0 + r) * kWave + lane] = E[r];
    lf[(kFlo0 + r) * kWave + lane] = lo[r];
    lf[(kFhi0 + r) * kWave + lane] = hi[r];
    lf[(kFw0 + r) * kWave + lane] = wb[r];
  }
  if (lane == 0) {
    double* sc = st + state_scal_off(N);
    sc[0] = cscale;
    sc[1] = bad_input ? -1.0 : 0.0;  // ADMM flag: -1 numerical error, 0 not converged, 1 converged
    sc[2] = 0.0;                     // admm iterations
    sc[3] = 0.0;                     // factorizations
  }
}

// ------------------------------------------------------------------ shared solver context
// Per-lane view of one scaled QP plus the structured operators and the KKT inverse.
template <int N>
struct Ctx {
  static constexpr int n = 2 * N;
  int lane;
  bool act, even;
  double dt;
  double D, qv;
  double E[3], lo[3], hi[3], wb[3];
  double cscale;
  const double* __restrict__ P;  // Pbar (global, L2-resident)
  double* buf;                   // LDS broadcast buffer, >= 2*kWave doubles
  double* sv;                    // LDS, N+1 doubles
  double* Dl;                    // LDS copy of D (n doubles)
  static constexpr int kNW = (n + 15) / 16;  // 16-lane rows holding the n variables
  // KKT inverse, row `lane`: A^{-1}[lane][j] = -r[j] (symmetric sweep operator)
  double r[n];

  __device__ __forceinline__ void load(const double* st, int ln, double dt_, double* buf_, double* sv_, double* Dl_,
                                       double* Ps) {
    lane = ln;
    act = ln < n;
    even = act && ((ln & 1) == 0);
    dt = dt_;
    buf = buf_;
    sv = sv_;
    Dl = Dl_;
    // Pbar is re-read by every factorization and every P-product: stage it in LDS once
    for (int i = ln; i < n * n; i += kWave) Ps[i] = st[i];
    P = Ps;
    const double* lf = st + state_lane_off(N);
    qv = lf[kFq * kWave + ln];
    D = lf[kFD * kWave + ln];
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      E[k] = lf[(kFE0 + k) * kWave + ln];
      lo[k] = lf[(kFlo0 + k) * kWave + ln];
      hi[k] = lf[(kFhi0 + k) * kWave + ln];
      wb[k] = lf[(kFw0 + k) * kWave + ln];
    }
    cscale = st[state_scal_off(N)];
    if (act) Dl[ln] = D;
    __syncthreads();
  }

  // Make the per-lane problem data opaque to the optimizer at the top of a solver
  // iteration: otherwise LICM hoists dozens of derived values (reciprocals, products,
  // masks) out of the loops and the kernel drops to one wave per SIMD.
  __device__ __forceinline__ void opaque() {
    asm volatile("" : "+v"(D), "+v"(qv), "+v"(lane));
    asm volatile("" : "+v"(E[0]), "+v"(E[1]), "+v"(E[2]));
    asm volatile("" : "+v"(lo[0]), "+v"(lo[1]), "+v"(lo[2]));
    asm volatile("" : "+v"(hi[0]), "+v"(hi[1]), "+v"(hi[2]));
    asm volatile("" : "+v"(wb[0]), "+v"(wb[1]), "+v"(wb[2]));
  }

  // z = Cbar x
  __device__ __forceinline__ void Cmul(double x, double z[3]) const {
    const double t = D * x;
    const double pre = scan_add(even ? t : 0.0, lane);
    const double tm2 = shr2(t);
    z[0] = E[0] * dt * pre;
    z[1] = E[1] * t;
    z[2] = E[2] * (lane >= 2 ? t - tm2 : t);
  }
  // x = Cbar' y
  __device__ __forceinline__ double CTmul(const double y[3]) const {
    const double suf = rscan_add(E[0] * y[0], lane);
    const double ey2 = E[2] * y[2];
    const double n2 = shl2(ey2);
    double t = (even ? dt * suf : 0.0) + E[1] * y[1] + ey2;
    if (lane + 2 < n) t -= n2;
    return act ? D * t : 0.0;
  }
  // (Pbar v)_lane, Pbar symmetric: lane reads its row as a conflict-free column of the LDS copy
  __device__ __forceinline__ double Pmul(double v) const {
    double w[4];
    bcast<kNW>(act ? v : 0.0, w);
    const int col = act ? lane : 0;
    double a[4] = {0.0, 0.0, 0.0, 0.0};
    Unroll<0, n>::run([&](auto jc) {
      constexpr int j = decltype(jc)::value;
      fmac_bc<j % 16>(a[j % 4], w[j / 16], P[j * n + col]);
    });
    return act ? (a[0] + a[1]) + (a[2] + a[3]) : 0.0;
  }
  // KKT matrix A = Pbar + s I + Cbar' diag(rw) Cbar, row `lane` -> r[]
  __device__ __forceinline__ void form(double s, const double rw[3]) {
    // opaque lane copy: keeps per-column masks/addresses from being hoisted out of solver loops
    int ln = lane;
    asm volatile("" : "+v"(ln));
    const bool ev_ln = ln < n && (ln & 1) == 0;
    const double ev = E[0] * E[0] * rw[0];
    const double suf = rscan_add(even ? ev : 0.0, lane);  // sum over v rows >= lane/2
    const double du2 = E[2] * E[2] * rw[2];
    const double du2n = shl2(du2);
    lds_sync();
    if (even) sv[lane >> 1] = suf;
    lds_sync();
    double diag = E[1] * E[1] * rw[1] + du2;
    if (ln + 2 < n) diag += du2n;
    const int col = ln < n ? ln : 0;
    const double Dm = ln < n ? D : 0.0;
    double wD[4];
    bcast<kNW>(Dm, wD);  // D_j of every lane j
    Unroll<0, n>::run([&](auto jc) {
      constexpr int j = decltype(jc)::value;
      double t = 0.0;
      if ((j & 1) == 0 && ev_ln) {
        const int mx = (ln > j ? ln : j) >> 1;
        t = dt * dt * sv[mx];
      }
      if (j == ln) t += diag;
      if (j == ln + 2) t -= du2n;
      if (j + 2 == ln) t -= du2;
      double v = ln < n ? P[j * n + col] + (j == ln ? s : 0.0) : 0.0;
      fmac_bc<j % 16>(v, wD[j / 16], Dm * t);
      r[j] = v;
    });
  }
  // Symmetric sweep operator on the rows in r[]: afterwards A^{-1} = -r (row `lane`).
  // Step k: every lane needs its own A[i][k] (register r[k]) and the pivot row A[k][j] =
  // A[j][k] (symmetry) -- the column r[k] of all lanes, register-broadcast by bcast() and read
  // through DPP row_newbcast, so each update r[j] += coef * A[k][j] is one v_fmac_f64_dpp.
  // The pivot row itself is the same FMA with coef = 1/d - 1 (A[k][j] <- A[k][j] / d), so the
  // update is uniform over lanes.  The step loop is unrolled at compile time (static register
  // indices and DPP lane immediates).  false on a non-positive pivot.
  __device__ __forceinline__ bool sweep() {
    bool ok = true;
    Unroll<0, n>::run([&](auto kc) {
      constexpr int k = decltype(kc)::value;
      double w[4];
      bcast<kNW>(r[k], w);
      const double d = readlane(r[k], k);
      ok = ok && (d > 0.0) && isfinite(d);
      const double inv = 1.0 / d;
      const bool piv = lane == k;
      const double ck = r[k] * inv;
      const double coef = piv ? inv - 1.0 : -ck;
      // next pivot column first: the next step's broadcast depends only on it
      if constexpr (k + 1 < n) fmac_bc<(k + 1) % 16>(r[k + 1], w[(k + 1) / 16], coef);
      Unroll<0, n>::run([&](auto jc) {
        constexpr int j = decltype(jc)::value;
        if constexpr (j != k && j != k + 1) fmac_bc<j % 16>(r[j], w[j / 16], coef);
      });
      r[k] = piv ? -inv : ck;
    });
    return ok;
  }
  // (A^{-1} v)_lane
  __device__ __forceinline__ double inv_mul(double v) const {
    double w[4];
    bcast<kNW>(act ? v : 0.0, w);
    double a[4] = {0.0, 0.0, 0.0, 0.0};
    Unroll<0, n>::run([&](auto jc) {
      constexpr int j = decltype(jc)::value;
      fmac_bc<j % 16>(a[j % 4], w[j / 16], r[j]);
    });
    return act ? -((a[0] + a[1]) + (a[2] + a[3])) : 0.0;
  }
};

template <int N>
struct SolveSmem {
  double P[4 * N * N];  // Pbar, row-major n x n (column reads by lane are conflict-free)
  double buf[2 * kWave];
  double sv[N + 1];
  double Dl[2 * N];
};

// ------------------------------------------------------------------ K2b: ADMM
template <int N>
__global__ __launch_bounds__(kWave) void k_admm(mpcqp_params p, int B, double* __restrict__ state) {
  __shared__ SolveSmem<N> sm;
  const int b = blockIdx.x;
  if (b >= B) return;
  double* st = state + (size_t)b * state_stride(N);
  Ctx<N> C;
  C.load(st, threadIdx.x, p.dt, sm.buf, sm.sv, sm.Dl, sm.P);
  const bool act = C.act;
  double x = 0.0, z[3] = {0.0, 0.0, 0.0}, y[3] = {0.0, 0.0, 0.0};
  double rho = p.rho;
  const double sg = p.sigma, alpha = p.alpha;
  bool bad = st[state_scal_off(N) + 1] < 0.0;  // non-finite problem data (k_setup)
  bool ok = false;
  int it = 0, nfact = 0;
  Stamps T, T2;
  T2.begin();
  while (it < p.max_iter && !bad && !ok) {
    {
      const double rw[3] = {rho, rho, rho};
      T.begin();
      C.form(sg, rw);
      T.end(0);
      ++nfact;
      T.begin();
      const bool okf = C.sweep();
      T.end(1);
      if (wave_any(!okf)) {
        bad = true;
        break;
      }
    }
    bool refactor = false;
    double prox_a[3], prox_b[3];  // zn = (rho vv + 2 w bnd) / (rho + 2 w)
#pragma unroll
    for (int r = 0; r < 3; ++r) {
      prox_a[r] = rho / (rho + 2.0 * C.wb[r]);
      prox_b[r] = 2.0 * C.wb[r] / (rho + 2.0 * C.wb[r]);
    }
    const double ir = 1.0 / rho;
    while (!refactor && it < p.max_iter) {
      ++it;
      C.opaque();
      T.begin();
      double tmp[3];
#pragma unroll
      for (int r = 0; r < 3; ++r) tmp[r] = rho * z[r] - y[r];
      const double rhs = C.CTmul(tmp) + sg * x - C.qv;
      const double xt = C.inv_mul(rhs);
      double zt[3];
      C.Cmul(xt, zt);
      x = alpha * xt + (1.0 - alpha) * x;
#pragma unroll
      for (int r = 0; r < 3; ++r) {
        const double v = alpha * zt[r] + (1.0 - alpha) * z[r];
        const double vv = v + y[r] * ir;
        double zn = vv;
        if (vv > C.hi[r])
          zn = prox_a[r] * vv + prox_b[r] * C.hi[r];
        else if (vv < C.lo[r])
          zn = prox_a[r] * vv + prox_b[r] * C.lo[r];
        y[r] = y[r] + rho * (v - zn);
        z[r] = zn;
      }
      T.end(2);
      if (it % p.check_termination == 0 || it == p.max_iter) {
        T.begin();
        double Ax[3];
        C.Cmul(x, Ax);
        const double Px = C.Pmul(x);
        const double Aty = C.CTmul(y);
        double pr = 0, nAx = 0, nz = 0, spr = 0, snAx = 0, snz = 0;
#pragma unroll
        for (int r = 0; r < 3; ++r) {
          if (C.E[r] > 0.0) {
            const double ie = 1.0 / C.E[r];
            pr = fmax(pr, fabs((Ax[r] - z[r]) * ie));
            nAx = fmax(nAx, fabs(Ax[r] * ie));
            nz = fmax(nz, fabs(z[r] * ie));
            spr = fmax(spr, fabs(Ax[r] - z[r]));
            snAx = fmax(snAx, fabs(Ax[r]));
            snz = fmax(snz, fabs(z[r]));
          }
        }
        double du = 0, nPx = 0, nAty = 0, nq = 0, sdu = 0, snPx = 0, snAty = 0, snq = 0;
        if (act) {
          const double id = 1.0 / C.D;
          const double rd = Px + C.qv + Aty;
          du = fabs(rd * id);
          nPx = fabs(Px * id);
          nAty = fabs(Aty * id);
          nq = fabs(C.qv * id);
          sdu = fabs(rd);
          snPx = fabs(Px);
          snAty = fabs(Aty);
          snq = fabs(C.qv);
        }
        pr = wave_max(pr);
        nAx = wave_max(nAx);
        nz = wave_max(nz);
        du = wave_max(du);
        nPx = wave_max(nPx);
        nAty = wave_max(nAty);
        nq = wave_max(nq);
        const double ic = 1.0 / C.cscale;
        du *= ic;
        const double ep = p.eps_abs + p.eps_rel * fmax(nAx, nz);
        const double ed = p.eps_abs + p.eps_rel * fmax(fmax(nPx, nAty), nq) * ic;
        T.end(3);
        // fmax drops NaNs, so test the iterate itself
        if (wave_any(!isfinite(x) || !isfinite(z[0] + z[1] + z[2]) || !isfinite(y[0] + y[1] + y[2])) ||
            !isfinite(pr) || !isfinite(du)) {
          bad = true;
          break;
        }
        if (pr <= ep && du <= ed) {
          ok = true;
          break;
        }
        if (p.adaptive_rho && it % p.adaptive_rho_interval == 0) {
          spr = wave_max(spr);
          snAx = wave_max(snAx);
          snz = wave_max(snz);
          sdu = wave_max(sdu);
          snPx = wave_max(snPx);
          snAty = wave_max(snAty);
          snq = wave_max(snq);
          const double pn = spr / (fmax(snAx, snz) + kDivTol);
          const double dn = sdu / (fmax(fmax(snPx, snAty), snq) + kDivTol);
          double rn = rho * sqrt(pn / (dn + kDivTol));
          rn = fmin(fmax(rn, kRhoMin), kRhoMax);
          if (rn > rho * p.adaptive_rho_tolerance || rn < rho / p.adaptive_rho_tolerance) {
            rho = rn;
            refactor = true;
          }
        }
      }
    }
  }
  double* lf = st + state_lane_off(N);
  lf[kFx * kWave + threadIdx.x] = act ? x : 0.0;
  if (threadIdx.x == 0) {
    double* sc = st + state_scal_off(N);
    sc[1] = bad ? -1.0 : (ok ? 1.0 : 0.0);
    sc[2] = (double)it;
    sc[3] = (double)nfact;
  }
  T2.end(0);
  T.flush(0);   // g_stamps[0..3]: form, sweep, ADMM iteration body, termination checks
  T2.flush(4);  // g_stamps[4]: whole k_admm
}

// ------------------------------------------------------------------ K2c: polish + outputs
template <int N>
__global__ __launch_bounds__(kWave) void k_finish(mpcqp_params p, int B, const double* __restrict__ model,
                                                  const double* __restrict__ state, double* __restrict__ u0o,
                                                  double* __restrict__ Xo, double* __restrict__ Uo,
                                                  int32_t* __restrict__ statuso, int32_t* __restrict__ iterso,
                                                  uint8_t* __restrict__ activeo) {
  constexpr int n = 2 * N;
  __shared__ SolveSmem<N> sm;
  const int b = blockIdx.x;
  if (b >= B) return;
  const int lane = threadIdx.x;
  const double* st = state + (size_t)b * state_stride(N);
  Ctx<N> C;
  C.load(st, lane, p.dt, sm.buf, sm.sv, sm.Dl, sm.P);
  const bool act = C.act;
  const bool use_admm = p.method == MPCQP_METHOD_ADMM;
  const bool do_polish = !use_admm || p.polish != 0;
  const double* sc = st + state_scal_off(N);
  const double admm_flag = sc[1];  // -1: non-finite data (k_setup) or ADMM numerical error
  bool bad = admm_flag < 0.0;
  const bool admm_ok = admm_flag > 0.0;
  const int admm_it = use_admm ? (int)sc[2] : 0;
  int nfact = use_admm ? (int)sc[3] : 0;
  double x = use_admm ? st[state_lane_off(N) + kFx * kWave + lane] : 0.0;
  const double x_admm = x;
  bool pol_ok = false;
  int pol_it = 0, n_ls = 0;
  Stamps T, T2;
  T2.begin();

  if (do_polish && !bad) {
    double zc[3];
    int cd[3];
    C.Cmul(x, zc);
#pragma unroll
    for (int r = 0; r < 3; ++r) cd[r] = zc[r] > C.hi[r] ? 2 : (zc[r] < C.lo[r] ? 1 : 0);
    while (pol_it < p.polish_max_iter) {
      ++pol_it;
      C.opaque();
      double rw[3], tmp[3];
#pragma unroll
      for (int r = 0; r < 3; ++r) {
        rw[r] = cd[r] ? 2.0 * C.wb[r] : 0.0;
        tmp[r] = cd[r] == 2 ? rw[r] * C.hi[r] : (cd[r] == 1 ? rw[r] * C.lo[r] : 0.0);
      }
      T.begin();
      C.form(0.0, rw);
      T.end(0);
      ++nfact;
      T.begin();
      const bool okf = C.sweep();
      T.end(1);
      if (wave_any(!okf)) {
        bad = true;
        break;
      }
      T.begin();
      const double rhs = C.CTmul(tmp) - C.qv;
      double xn = C.inv_mul(rhs);
      {  // one step of iterative refinement: res = rhs - M xn
        double zz[3], t3[3];
        C.Cmul(xn, zz);
#pragma unroll
        for (int r = 0; r < 3; ++r) t3[r] = rw[r] * zz[r];
        const double Mx = C.Pmul(xn) + C.CTmul(t3);
        xn += C.inv_mul(rhs - Mx);
      }
      double zn[3];
      C.Cmul(xn, zn);
      bool diff = false;
#pragma unroll
      for (int r = 0; r < 3; ++r) {
        const int c2 = zn[r] > C.hi[r] ? 2 : (zn[r] < C.lo[r] ? 1 : 0);
        diff = diff || (c2 != cd[r]);
      }
      T.end(2);
      if (wave_any(!isfinite(xn))) {
        bad = true;
        break;
      }
      if (!wave_any(diff)) {
        x = xn;
        pol_ok = true;
        break;
      }
      // Armijo backtracking on the scaled objective along d = xn - x
      T.begin();
      const double dx = act ? xn - x : 0.0;
      const double Px = C.Pmul(x);
      const double Pd = C.Pmul(dx);
      double zd[3], gt[3];
#pragma unroll
      for (int r = 0; r < 3; ++r) {
        zd[r] = zn[r] - zc[r];
        const double res = zc[r] > C.hi[r] ? zc[r] - C.hi[r] : (zc[r] < C.lo[r] ? zc[r] - C.lo[r] : 0.0);
        gt[r] = 2.0 * C.wb[r] * res;
      }
      const double gr = C.CTmul(gt);
      const double slope = wave_sum(act ? (Px + C.qv + gr) * dx : 0.0);
      const double qd = wave_sum(act ? dx * Pd : 0.0);
      const double lin = wave_sum(act ? (Px + C.qv) * dx : 0.0);
      const double q0 = wave_sum(act ? x * (0.5 * Px + C.qv) : 0.0);
      auto pen = [&](double t) -> double {
        double s = 0.0;
#pragma unroll
        for (int r = 0; r < 3; ++r) {
          const double zt = zc[r] + t * zd[r];
          const double d = zt > C.hi[r] ? zt - C.hi[r] : (zt < C.lo[r] ? C.lo[r] - zt : 0.0);
          s += C.wb[r] * d * d;
        }
        return wave_sum(s);
      };
      const double f0 = q0 + pen(0.0);
      double t = 1.0;
      for (int ls = 0; ls < 60; ++ls) {
        ++n_ls;
        const double ft = q0 + t * lin + 0.5 * t * t * qd + pen(t);
        if (ft <= f0 + 1e-4 * t * slope) break;
        t *= 0.5;
      }
      x = x + t * dx;
      C.Cmul(x, zc);
#pragma unroll
      for (int r = 0; r < 3; ++r) cd[r] = zc[r] > C.hi[r] ? 2 : (zc[r] < C.lo[r] ? 1 : 0);
      T.end(3);
    }
  }
  T2.end(0);
  T.flush(8);   // g_stamps[8..11]: polish form, sweep, solve+check, line search
  T2.flush(12); // g_stamps[12]: polish phase of k_finish
  if (wave_any(!isfinite(x))) bad = true;
  int status;
  if (bad) {
    status = MPCQP_NUMERICAL_ERROR;
  } else if (pol_ok) {
    status = MPCQP_SOLVED;
  } else if (use_admm) {
    if (do_polish) x = x_admm;  // polish failed: return the ADMM iterate (OSQP behaviour)
    status = admm_ok ? (do_polish ? MPCQP_SOLVED_INACCURATE : MPCQP_SOLVED) : MPCQP_MAX_ITER_REACHED;
  } else {
    status = MPCQP_MAX_ITER_REACHED;
  }

  // ---- outputs (unscaled) ----
  const double* mb = model + (size_t)b * model_stride(N);
  const int cc = lane & 1;
  const double U = act ? C.D * x : 0.0;
  const double dt = p.dt;
  const double x00 = mb[11 * N + 4], x01 = mb[11 * N + 5], x02 = mb[11 * N + 6], x03 = mb[11 * N + 7];
  const double up0 = mb[11 * N + 8], up1 = mb[11 * N + 9];
  const double sj = act ? mb[4 * N + (lane >> 1)] : 0.0;
  // v_{j+1} on lane 2j, psi_{j+1} on lane 2j+1
  const double vacc = scan_add(C.even ? U : 0.0, lane);
  const double sacc = scan_add((act && cc == 1) ? sj * U : 0.0, lane);
  // lane k <- (psi_k, v_k)
  const int srcv = lane == 0 ? 0 : 2 * (lane - 1);
  const double vk_s = __shfl(vacc, srcv < kWave ? srcv : 0, kWave);
  const double pk_s = __shfl(sacc, (srcv + 1) < kWave ? srcv + 1 : 0, kWave);
  const double vk = lane == 0 ? x03 : x03 + dt * vk_s;
  const double pk = lane == 0 ? x02 : x02 + pk_s;
  double t0 = 0.0, t1 = 0.0;
  if (lane < N) {
    t0 = mb[lane] * pk + mb[N + lane] * vk + mb[5 * N + lane];
    t1 = mb[2 * N + lane] * pk + mb[3 * N + lane] * vk + mb[6 * N + lane];
  }
  const double in0 = scan_add(t0, lane), in1 = scan_add(t1, lane);
  const double ex0 = dpp<kWaveShr1>(in0), ex1 = dpp<kWaveShr1>(in1);  // exclusive prefix
  const double Xk0 = x00 + ex0, Xk1 = x01 + ex1;
  if (Xo && lane <= N) {
    double* Xb = Xo + (size_t)b * 4 * (N + 1);
    Xb[0 * (N + 1) + lane] = Xk0;
    Xb[1 * (N + 1) + lane] = Xk1;
    Xb[2 * (N + 1) + lane] = pk;
    Xb[3 * (N + 1) + lane] = vk;
  }
  if (Uo && act) Uo[(size_t)b * n + cc * N + (lane >> 1)] = U;
  if (u0o && lane < 2) u0o[(size_t)b * 2 + lane] = U;
  const double Um2 = shr2(U);
  if (activeo) {
    uint8_t* ab = activeo + (size_t)b * (5 * N + 1);
    if (lane <= N) ab[lane] = vk > p.v_bounds[1] ? 2 : (vk < p.v_bounds[0] ? 1 : 0);
    if (act) {
      ab[N + 1 + lane] = U > p.u_bounds[2 * cc + 1] ? 2 : (U < p.u_bounds[2 * cc] ? 1 : 0);
      const double d = U - (lane < 2 ? (cc ? up1 : up0) : Um2);
      ab[3 * N + 1 + lane] = d > p.du_bounds[2 * cc + 1] ? 2 : (d < p.du_bounds[2 * cc] ? 1 : 0);
    }
  }
  if (lane == 0) {
    statuso[b] = status;
    if (iterso) {
      iterso[4 * (size_t)b + 0] = admm_it;
      iterso[4 * (size_t)b + 1] = pol_it;
      iterso[4 * (size_t)b + 2] = nfact;
      iterso[4 * (size_t)b + 3] = n_ls;
    }
  }
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

// ------------------------------------------------------------------ dispatch
struct Launch {
  const mpcqp_params* p;
  int B;
  const double* model;
  double* state;
  double *u0, *X, *U;
  int32_t *st, *it;
  uint8_t* ac;
};

template <int N>
void launch_solve(hipStream_t s, const Launch& L) {
  hipLaunchKernelGGL(k_setup<N>, dim3(L.B), dim3(kWave), 0, s, *L.p, L.B, L.model, L.state);
  if (L.p->method == MPCQP_METHOD_ADMM) hipLaunchKernelGGL(k_admm<N>, dim3(L.B), dim3(kWave), 0, s, *L.p, L.B, L.state);
  hipLaunchKernelGGL(k_finish<N>, dim3(L.B), dim3(kWave), 0, s, *L.p, L.B, L.model, L.state, L.u0, L.X, L.U, L.st,
                     L.it, L.ac);
}

typedef void (*launcher_t)(hipStream_t, const Launch&);

#ifdef MPCQP_ONLY_N  // development builds: instantiate a single horizon
#define MPCQP_L(N) ((N) == MPCQP_ONLY_N ? &launch_solve<MPCQP_ONLY_N> : nullptr)
#else
#define MPCQP_L(N) &launch_solve<N>
#endif
const launcher_t kLaunchers[MPCQP_MAX_HORIZON + 1] = {
    nullptr,     MPCQP_L(1),  MPCQP_L(2),  MPCQP_L(3),  MPCQP_L(4),  MPCQP_L(5),  MPCQP_L(6),  MPCQP_L(7),
    MPCQP_L(8),  MPCQP_L(9),  MPCQP_L(10), MPCQP_L(11), MPCQP_L(12), MPCQP_L(13), MPCQP_L(14), MPCQP_L(15),
    MPCQP_L(16), MPCQP_L(17), MPCQP_L(18), MPCQP_L(19), MPCQP_L(20), MPCQP_L(21), MPCQP_L(22), MPCQP_L(23),
    MPCQP_L(24), MPCQP_L(25), MPCQP_L(26), MPCQP_L(27), MPCQP_L(28), MPCQP_L(29), MPCQP_L(30), MPCQP_L(31)};
#undef MPCQP_L

thread_local std::string g_err;

int fail(int code, const std::string& msg) {
  g_err = msg;
  return code;
}

int check_params(const mpcqp_params* p) {
  if (!p) return fail(MPCQP_E_ARG, "null params");
  if (p->horizon < 1 || p->horizon > MPCQP_MAX_HORIZON)
    return fail(MPCQP_E_HORIZON, "horizon " + std::to_string(p->horizon) + " outside [1, 31]");
  if (!kLaunchers[p->horizon]) return fail(MPCQP_E_HORIZON, "horizon not compiled into this build");
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

struct mpcqp_ws {
  mpcqp_params p;
  int max_batch;
  int device;
  int built_B;
  double* model;
  double* state;
};

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
  const size_t mbytes = sizeof(double) * (size_t)model_stride(p->horizon) * (size_t)max_batch;
  const size_t sbytes = sizeof(double) * (size_t)state_stride(p->horizon) * (size_t)max_batch;
  e = hipMalloc(&w->model, mbytes);
  if (e == hipSuccess) e = hipMalloc(&w->state, sbytes);
  if (e != hipSuccess) {
    if (w->model) (void)hipFree(w->model);
    delete w;
    return fail(MPCQP_E_HIP, std::string("hipMalloc: ") + hipGetErrorString(e));
  }
  *ws = w;
  g_err.clear();
  return MPCQP_OK;
}

int mpcqp_set_params(mpcqp_ws* ws, const mpcqp_params* p) {
  if (!ws) return fail(MPCQP_E_ARG, "null ws");
  int rc = check_params(p);
  if (rc) return rc;
  if (p->horizon != ws->p.horizon) return fail(MPCQP_E_HORIZON, "set_params cannot change the horizon");
  ws->p = *p;
  return MPCQP_OK;
}

void mpcqp_destroy(mpcqp_ws* ws) {
  if (!ws) return;
  (void)hipSetDevice(ws->device);
  (void)hipFree(ws->model);
  (void)hipFree(ws->state);
  delete ws;
}

int mpcqp_build(mpcqp_ws* ws, int B, const double* x0, const double* ref, const double* u_prev, void* stream) {
  if (!ws || !x0 || !ref) return fail(MPCQP_E_ARG, "null argument");
  if (B < 0 || B > ws->max_batch) return fail(MPCQP_E_BATCH, "batch exceeds workspace capacity");
  ws->built_B = B;
  if (B == 0) return MPCQP_OK;
  hipStream_t s = static_cast<hipStream_t>(stream);
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
  Launch L{&ws->p, B, ws->model, ws->state, u0, X, U, status, iters, active};
  kLaunchers[ws->p.horizon](s, L);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return fail(MPCQP_E_HIP, std::string("k_solve launch: ") + hipGetErrorString(e));
  return MPCQP_OK;
}

const double* mpcqp_model_buffer(const mpcqp_ws* ws) { return ws ? ws->model : nullptr; }

const double* mpcqp_state_buffer(const mpcqp_ws* ws) { return ws ? ws->state : nullptr; }

int mpcqp_state_stride(int horizon) { return state_stride(horizon); }

int mpcqp_debug_stamps(unsigned long long* out16, int reset) {
#ifdef MPCQP_STAMPS
  hipError_t e = hipDeviceSynchronize();
  if (e == hipSuccess && out16) e = hipMemcpyFromSymbol(out16, HIP_SYMBOL(g_stamps), sizeof(unsigned long long) * 16);
  if (e == hipSuccess && reset) {
    unsigned long long z[16] = {0};
    e = hipMemcpyToSymbol(HIP_SYMBOL(g_stamps), z, sizeof(z));
  }
  if (e != hipSuccess) return fail(MPCQP_E_HIP, std::string("stamps: ") + hipGetErrorString(e));
  return MPCQP_OK;
#else
  (void)out16;
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
