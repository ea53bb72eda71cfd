// mpcqp.hip -- MI355X (gfx950) batched bicycle-MPC QP solver: kernels + C-ABI.
//
// Replaces the reference's per-step MPC solve (CagriCatik/RRT-MPC):
//   K1 k_build  : window -> LTV model   (src/control/mpc_controller.py:59-70,108,
//                                        src/control/vehicle_model.py:24-45)
//   K2 k_solve  : condense + ADMM/OSQP + polish
//                                       (src/control/mpc_controller.py:53-141; OSQP
//                                        settings of :121-131)
// One 64-lane wavefront owns one QP (B QPs -> B single-wave workgroups).  The QP
// never leaves the CU: LDS holds the scaled Hessian, registers hold one row of the
// KKT inverse per lane, and every vector of the ADMM iteration is distributed one
// decision variable per lane.  The algorithm is restated sequentially, operation
// for operation, in oracle/mpcqp_cpu.c (CPU baseline) -- see DESIGN.md.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <new>
#include <string>

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

__host__ __device__ constexpr int model_stride(int N) { return ((11 * N + 10) + 7) / 8 * 8; }

// ------------------------------------------------------------------ wave primitives
__device__ __forceinline__ double wave_max(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmax(v, __shfl_xor(v, o, kWave));
  return v;
}
__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, kWave);
  return v;
}
// inclusive prefix sum / max over lanes 0..lane
__device__ __forceinline__ double scan_sum(double v, int lane) {
#pragma unroll
  for (int d = 1; d < kWave; d <<= 1) {
    double t = __shfl_up(v, d, kWave);
    if (lane >= d) v += t;
  }
  return v;
}
__device__ __forceinline__ double scan_max(double v, int lane) {
#pragma unroll
  for (int d = 1; d < kWave; d <<= 1) {
    double t = __shfl_up(v, d, kWave);
    if (lane >= d) v = fmax(v, t);
  }
  return v;
}
// inclusive suffix sum / max over lanes lane..63
__device__ __forceinline__ double rscan_sum(double v, int lane) {
#pragma unroll
  for (int d = 1; d < kWave; d <<= 1) {
    double t = __shfl_down(v, d, kWave);
    if (lane + d < kWave) v += t;
  }
  return v;
}
__device__ __forceinline__ double rscan_max(double v, int lane) {
#pragma unroll
  for (int d = 1; d < kWave; d <<= 1) {
    double t = __shfl_down(v, d, kWave);
    if (lane + d < kWave) v = fmax(v, t);
  }
  return v;
}
__device__ __forceinline__ bool wave_any(bool b) { return __ballot(b) != 0ull; }

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
  const double prev = __shfl_up(ryaw, 1, kWave);
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
    cs = cs + __shfl(pc, j, kWave);
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
  const int src = lane == 0 ? 0 : lane - 1;
  const double psi = __shfl(uyaw, src, kWave);
  const double v = __shfl(rv, src, kWave);
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

// ------------------------------------------------------------------ K2: solve
// Row slots owned by lane p (p < n = 2N):
//   slot 0: v row (p even): v_{p/2+1} - v0 = dt * sum_{j<=p/2} a_j   (mpc_controller.py:81-82,115-116)
//   slot 1: input row        U_p                                      (:83-86)
//   slot 2: rate row         U_p - U_{p-2} (u_prev at k = 0)          (:89-106)
// Everything below is in OSQP's scaled space: x = D^-1 U, rows E * (C U), cost c.
template <int N>
struct Solver {
  static constexpr int n = 2 * N;
  static constexpr int LD = n + 1;  // odd leading dimension: conflict-free row and column access
  static constexpr int S = model_stride(N);

  struct Smem {
    double P[n * LD];   // scaled P = 2 c D H D
    double buf[2 * kWave];  // broadcast vector (the sweep keeps a wrapped copy in [n, 2n))
    double model[S];
    double pre[4][N + 1];  // prefix sums of alpha, beta, gamma, eta
    double err[N + 1][4];  // free-response tracking error e_m = sx_m - r_m
    double sv[N + 1];      // suffix sums over v rows of E^2 * weight
    double D[n];
    double g[n];
  };
};

template <int N>
__global__ __launch_bounds__(kWave) void k_solve(mpcqp_params p, int B, const double* __restrict__ model,
                                                 double* __restrict__ u0o, double* __restrict__ Xo,
                                                 double* __restrict__ Uo, int32_t* __restrict__ statuso,
                                                 int32_t* __restrict__ iterso, uint8_t* __restrict__ activeo) {
  using Sv = Solver<N>;
  constexpr int n = Sv::n;
  constexpr int LD = Sv::LD;
  constexpr int S = Sv::S;
  __shared__ typename Sv::Smem sm;
  const int b = blockIdx.x;
  const int lane = threadIdx.x;
  if (b >= B) return;
  const bool act = lane < n;
  const bool even = act && ((lane & 1) == 0);
  const int cc = lane & 1;  // 0 = acceleration, 1 = steering
  const double dt = p.dt;

  // ---- stage the model in LDS (coalesced) ----
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

  // prefix sums (lane 0..3 one array each) and free response (lane 4)
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
    const double e2n = __shfl_down(E[2], 2, kWave);
    double ccol = fmax(E[1], E[2]);
    if (lane + 2 < n) ccol = fmax(ccol, e2n);
    if (even) ccol = fmax(ccol, dt * sufE);
    ccol *= D;
    const double dl = act ? 1.0 / sqrt(limit_scaling(fmax(cmax, ccol))) : 0.0;
    // row norms of A
    const double preD = scan_max(even ? D : 0.0, lane);
    const double Dm2 = __shfl_up(D, 2, kWave);
    double el0 = even ? 1.0 / sqrt(limit_scaling(E[0] * dt * preD)) : 0.0;
    double el1 = act ? 1.0 / sqrt(limit_scaling(E[1] * D)) : 0.0;
    double el2 = act ? 1.0 / sqrt(limit_scaling(E[2] * (lane >= 2 ? fmax(D, Dm2) : D))) : 0.0;
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
  double wb[3];
#pragma unroll
  for (int r = 0; r < 3; ++r) {
    lo[r] *= E[r];
    hi[r] *= E[r];
    wb[r] = E[r] > 0.0 ? cscale * wt[r] / (E[r] * E[r]) : 0.0;
  }
  __syncthreads();
  if (act) sm.D[lane] = D;
  __syncthreads();

  // ---- structured operators ----
  // z = Cbar x
  auto Cmul = [&](double x, double z[3]) {
    const double t = D * x;
    const double pre = scan_sum(even ? t : 0.0, lane);
    const double tm2 = __shfl_up(t, 2, kWave);
    z[0] = E[0] * dt * pre;
    z[1] = E[1] * t;
    z[2] = E[2] * (lane >= 2 ? t - tm2 : t);
  };
  // x = Cbar' y
  auto CTmul = [&](const double y[3]) -> double {
    const double suf = rscan_sum(E[0] * y[0], lane);
    const double ey2 = E[2] * y[2];
    const double n2 = __shfl_down(ey2, 2, kWave);
    double t = (even ? dt * suf : 0.0) + E[1] * y[1] + ey2;
    if (lane + 2 < n) t -= n2;
    return act ? D * t : 0.0;
  };
  // (Pbar v)_lane
  auto Pmul = [&](double v) -> double {
    __syncthreads();
    sm.buf[lane] = act ? v : 0.0;
    __syncthreads();
    double acc = 0.0;
    if (act) {
#pragma unroll 8
      for (int j = 0; j < n; ++j) acc += sm.P[lane * LD + j] * sm.buf[j];
    }
    return acc;
  };

  // ---- KKT matrix rows in registers: A = Pbar + sig I + Cbar' diag(rw) Cbar ----
  // Row `lane` lives in a[]; the sweep below rotates it left once per pivot so
  // that every register index is static while the pivot loop stays rolled.
  double a[n];
  auto form_rows = [&](double sig, const double rw[3]) {
    // Opaque copy of the lane id: keeps the per-column masks and LDS addresses
    // below from being hoisted out of the solver loop (they would pin ~100 VGPRs).
    int ln = lane;
    asm volatile("" : "+v"(ln));
    const bool ev_ln = ln < n && (ln & 1) == 0;
    __syncthreads();
    const double ev = E[0] * E[0] * rw[0];
    const double suf = rscan_sum(even ? ev : 0.0, lane);  // sum over v rows >= lane/2
    if (even) sm.sv[lane >> 1] = suf;
    const double du2 = E[2] * E[2] * rw[2];
    const double du2n = __shfl_down(du2, 2, kWave);
    __syncthreads();
    double diag = E[1] * E[1] * rw[1] + du2;
    if (ln + 2 < n) diag += du2n;
    const int lrow = ln < n ? ln : 0;
#pragma unroll
    for (int j = 0; j < n; ++j) {
      double t = 0.0;
      if ((j & 1) == 0 && ev_ln) {
        const int mx = (ln > j ? ln : j) >> 1;
        t = dt * dt * sm.sv[mx];
      }
      if (j == ln) t += diag;
      if (j == ln + 2) t -= du2n;
      if (j + 2 == ln) t -= du2;
      const double v = sm.P[lrow * LD + j] + D * sm.D[j] * t + (j == ln ? sig : 0.0);
      a[j] = ln < n ? v : 0.0;
    }
  };
  // symmetric sweep operator: a <- -A^{-1} (row `lane`).  false on a non-positive pivot.
  auto sweep = [&]() -> bool {
    bool ok = true;
    for (int k = 0; k < n; ++k) {
      __syncthreads();
      sm.buf[lane] = a[0];  // column k == row k (symmetry); slot 0 holds absolute column k
      if (lane < n) sm.buf[lane + n] = a[0];
      __syncthreads();
      const double d = sm.buf[k];
      ok = ok && (d > 0.0) && isfinite(d);
      const double inv = 1.0 / d;
      const bool piv = lane == k;
      double f = a[0] * inv;
      if (piv) {
#pragma unroll
        for (int j = 1; j < n; ++j) a[j] = 0.0;
        f = -inv;
      }
      const double* col = sm.buf + k;  // col[j] = A[k][(k + j) mod n]
#pragma unroll
      for (int j = 1; j < n; ++j) a[j - 1] = fma(-f, col[j], a[j]);
      a[n - 1] = piv ? -inv : f;
    }
    return ok;
  };
  // -(a . v) with v broadcast through LDS == (A^{-1} v)_lane
  auto inv_mul = [&](double v) -> double {
    __syncthreads();
    sm.buf[lane] = act ? v : 0.0;
    __syncthreads();
    double acc0 = 0.0, acc1 = 0.0;
#pragma unroll
    for (int j = 0; j < n; j += 2) {
      acc0 = fma(a[j], sm.buf[j], acc0);
      if (j + 1 < n) acc1 = fma(a[j + 1], sm.buf[j + 1], acc1);
    }
    return act ? -(acc0 + acc1) : 0.0;
  };

  // ---- solver state ----
  double x = 0.0;
  double z[3] = {0.0, 0.0, 0.0}, y[3] = {0.0, 0.0, 0.0};
  bool bad = false, admm_ok = false, pol_ok = false;
  int admm_it = 0, pol_it = 0, n_fact = 0, n_ls = 0;
  const bool use_admm = p.method == MPCQP_METHOD_ADMM;
  const bool do_polish = (p.method == MPCQP_METHOD_NEWTON) || (p.polish != 0);
  double rho = p.rho;
  const double sig = p.sigma, alpha = p.alpha;
  double x_admm = 0.0;
  // polish state
  double zc[3] = {0.0, 0.0, 0.0};
  int cd[3] = {0, 0, 0};
  // phase 0 = ADMM, 1 = polish, 2 = done
  int phase = use_admm ? 0 : (do_polish ? 1 : 2);
  auto enter_polish = [&]() {
    x_admm = x;
    Cmul(x, zc);
#pragma unroll
    for (int r = 0; r < 3; ++r) cd[r] = zc[r] > hi[r] ? 2 : (zc[r] < lo[r] ? 1 : 0);
  };
  if (phase == 1) enter_polish();
  int it = 0;
  while (phase < 2) {
    // ---- (re)factor: the single inlined instance of form_rows + sweep ----
    double rw[3], tmp[3];
    if (phase == 0) {
      rw[0] = rw[1] = rw[2] = rho;
    } else {
#pragma unroll
      for (int r = 0; r < 3; ++r) rw[r] = cd[r] ? 2.0 * wb[r] : 0.0;
    }
    form_rows(phase == 0 ? sig : 0.0, rw);
    ++n_fact;
    if (wave_any(!sweep())) {
      bad = true;
      break;
    }
    if (phase == 0) {
      // ---- ADMM iterations with the current KKT inverse ----
      bool refactor = false;
      while (!refactor && it < p.max_iter) {
        ++it;
#pragma unroll
        for (int r = 0; r < 3; ++r) tmp[r] = rho * z[r] - y[r];
        const double rhs = CTmul(tmp) + sig * x - qv;
        const double xt = inv_mul(rhs);
        double zt[3];
        Cmul(xt, zt);
        x = alpha * xt + (1.0 - alpha) * x;
        const double ir = 1.0 / rho;
#pragma unroll
        for (int r = 0; r < 3; ++r) {
          const double v = alpha * zt[r] + (1.0 - alpha) * z[r];
          const double vv = v + y[r] * ir;
          double zn = vv;
          if (vv > hi[r])
            zn = (rho * vv + 2.0 * wb[r] * hi[r]) / (rho + 2.0 * wb[r]);
          else if (vv < lo[r])
            zn = (rho * vv + 2.0 * wb[r] * lo[r]) / (rho + 2.0 * wb[r]);
          y[r] = y[r] + rho * (v - zn);
          z[r] = zn;
        }
        admm_it = it;
        if (it % p.check_termination == 0 || it == p.max_iter) {
          double Ax[3];
          Cmul(x, Ax);
          const double Px = Pmul(x);
          const double Aty = CTmul(y);
          double pr = 0, nAx = 0, nz = 0, spr = 0, snAx = 0, snz = 0;
#pragma unroll
          for (int r = 0; r < 3; ++r) {
            if (E[r] > 0.0) {
              const double ie = 1.0 / E[r];
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
            const double id = 1.0 / D;
            const double rd = Px + qv + Aty;
            du = fabs(rd * id);
            nPx = fabs(Px * id);
            nAty = fabs(Aty * id);
            nq = fabs(qv * id);
            sdu = fabs(rd);
            snPx = fabs(Px);
            snAty = fabs(Aty);
            snq = fabs(qv);
          }
          pr = wave_max(pr);
          nAx = wave_max(nAx);
          nz = wave_max(nz);
          du = wave_max(du);
          nPx = wave_max(nPx);
          nAty = wave_max(nAty);
          nq = wave_max(nq);
          const double ic = 1.0 / cscale;
          du *= ic;
          const double ep = p.eps_abs + p.eps_rel * fmax(nAx, nz);
          const double ed = p.eps_abs + p.eps_rel * fmax(fmax(nPx, nAty), nq) * ic;
          if (!isfinite(pr) || !isfinite(du)) {
            bad = true;
            break;
          }
          if (pr <= ep && du <= ed) {
            admm_ok = true;
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
      if (bad) break;
      if (!refactor) {  // converged or out of iterations
        if (do_polish) {
          enter_polish();
          phase = 1;
        } else {
          phase = 2;
        }
      }
      continue;
    }
    // ---- polish step with the inverse of M = Pbar + sum_act 2 w C_r C_r' ----
    ++pol_it;
#pragma unroll
    for (int r = 0; r < 3; ++r) tmp[r] = cd[r] == 2 ? rw[r] * hi[r] : (cd[r] == 1 ? rw[r] * lo[r] : 0.0);
    const double rhs = CTmul(tmp) - qv;
    double xn = inv_mul(rhs);
    {  // one step of iterative refinement: res = rhs - M xn
      double zz[3], t3[3];
      Cmul(xn, zz);
#pragma unroll
      for (int r = 0; r < 3; ++r) t3[r] = rw[r] * zz[r];
      const double Mx = Pmul(xn) + CTmul(t3);
      xn += inv_mul(rhs - Mx);
    }
    double zn[3];
    Cmul(xn, zn);
    bool diff = false;
#pragma unroll
    for (int r = 0; r < 3; ++r) {
      const int c2 = zn[r] > hi[r] ? 2 : (zn[r] < lo[r] ? 1 : 0);
      diff = diff || (c2 != cd[r]);
    }
    if (!wave_any(diff)) {
      x = xn;
      pol_ok = true;
      phase = 2;
      continue;
    }
    // Armijo backtracking on the scaled objective along d = xn - x
    const double dx = act ? xn - x : 0.0;
    const double Px = Pmul(x);
    const double Pd = Pmul(dx);
    double zd[3], gt[3];
#pragma unroll
    for (int r = 0; r < 3; ++r) {
      zd[r] = zn[r] - zc[r];
      const double res = zc[r] > hi[r] ? zc[r] - hi[r] : (zc[r] < lo[r] ? zc[r] - lo[r] : 0.0);
      gt[r] = 2.0 * wb[r] * res;
    }
    const double gr = CTmul(gt);
    const double slope = wave_sum(act ? (Px + qv + gr) * dx : 0.0);
    const double qd = wave_sum(act ? dx * Pd : 0.0);
    const double lin = wave_sum(act ? (Px + qv) * dx : 0.0);
    const double q0 = wave_sum(act ? x * (0.5 * Px + qv) : 0.0);
    auto pen = [&](double t) -> double {
      double s = 0.0;
#pragma unroll
      for (int r = 0; r < 3; ++r) {
        const double zt = zc[r] + t * zd[r];
        const double d = zt > hi[r] ? zt - hi[r] : (zt < lo[r] ? lo[r] - zt : 0.0);
        s += wb[r] * d * d;
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
    Cmul(x, zc);
#pragma unroll
    for (int r = 0; r < 3; ++r) cd[r] = zc[r] > hi[r] ? 2 : (zc[r] < lo[r] ? 1 : 0);
    if (pol_it >= p.polish_max_iter) phase = 2;
  }
  int st;
  if (bad) {
    st = MPCQP_NUMERICAL_ERROR;
  } else if (pol_ok) {
    st = MPCQP_SOLVED;
  } else if (use_admm) {
    if (do_polish) x = x_admm;  // polish failed: return the ADMM iterate (OSQP behaviour)
    st = admm_ok ? (do_polish ? MPCQP_SOLVED_INACCURATE : MPCQP_SOLVED) : MPCQP_MAX_ITER_REACHED;
  } else {
    st = MPCQP_MAX_ITER_REACHED;
  }

  // ---- outputs (unscaled) ----
  const double U = act ? D * x : 0.0;
  // v_{j+1} on lane 2j, psi_{j+1} on lane 2j+1
  const double vacc = scan_sum(even ? U : 0.0, lane);
  const double sacc = scan_sum((act && cc == 1) ? si[lane >> 1] * U : 0.0, lane);
  // lane k <- (psi_k, v_k)
  const int srcv = lane == 0 ? 0 : 2 * (lane - 1);
  const double vk_s = __shfl(vacc, srcv < kWave ? srcv : 0, kWave);
  const double pk_s = __shfl(sacc, (srcv + 1) < kWave ? srcv + 1 : 0, kWave);
  const double vk = lane == 0 ? x0[3] : x0[3] + dt * vk_s;
  const double pk = lane == 0 ? x0[2] : x0[2] + pk_s;
  double t0 = 0.0, t1 = 0.0;
  if (lane < N) {
    t0 = al[lane] * pk + be[lane] * vk + c0[lane];
    t1 = ga[lane] * pk + et[lane] * vk + c1[lane];
  }
  const double in0 = scan_sum(t0, lane), in1 = scan_sum(t1, lane);
  const double ex0 = __shfl_up(in0, 1, kWave), ex1 = __shfl_up(in1, 1, kWave);  // exclusive prefix
  const double sx0 = lane == 0 ? 0.0 : ex0;
  const double sx1 = lane == 0 ? 0.0 : ex1;
  const double Xk0 = x0[0] + sx0, Xk1 = x0[1] + sx1;
  if (Xo && lane <= N) {
    double* Xb = Xo + (size_t)b * 4 * (N + 1);
    Xb[0 * (N + 1) + lane] = Xk0;
    Xb[1 * (N + 1) + lane] = Xk1;
    Xb[2 * (N + 1) + lane] = pk;
    Xb[3 * (N + 1) + lane] = vk;
  }
  if (Uo && act) Uo[(size_t)b * n + cc * N + (lane >> 1)] = U;
  if (u0o && lane < 2) u0o[(size_t)b * 2 + lane] = U;
  if (activeo) {
    uint8_t* ab = activeo + (size_t)b * (5 * N + 1);
    if (lane <= N) ab[lane] = vk > p.v_bounds[1] ? 2 : (vk < p.v_bounds[0] ? 1 : 0);
    const double Um2 = __shfl_up(U, 2, kWave);
    if (act) {
      ab[N + 1 + lane] = U > p.u_bounds[2 * cc + 1] ? 2 : (U < p.u_bounds[2 * cc] ? 1 : 0);
      const double d = U - (lane < 2 ? up[cc] : Um2);
      ab[3 * N + 1 + lane] = d > p.du_bounds[2 * cc + 1] ? 2 : (d < p.du_bounds[2 * cc] ? 1 : 0);
    }
  }
  if (lane == 0) {
    statuso[b] = st;
    if (iterso) {
      iterso[4 * (size_t)b + 0] = admm_it;
      iterso[4 * (size_t)b + 1] = pol_it;
      iterso[4 * (size_t)b + 2] = n_fact;
      iterso[4 * (size_t)b + 3] = n_ls;
    }
  }
}

// ------------------------------------------------------------------ dispatch
using solve_fn = void (*)(mpcqp_params, int, const double*, double*, double*, double*, int32_t*, int32_t*,
                          uint8_t*);

template <int N>
void launch_solve(hipStream_t s, const mpcqp_params& p, int B, const double* model, double* u0, double* X,
                  double* U, int32_t* st, int32_t* it, uint8_t* ac) {
  hipLaunchKernelGGL(k_solve<N>, dim3(B), dim3(kWave), 0, s, p, B, model, u0, X, U, st, it, ac);
}

typedef void (*launcher_t)(hipStream_t, const mpcqp_params&, int, const double*, double*, double*, double*,
                           int32_t*, int32_t*, uint8_t*);

#ifdef MPCQP_ONLY_N  // development builds: instantiate a single horizon
#define MPCQP_L(N) ((N) == MPCQP_ONLY_N ? &launch_solve<((N) == MPCQP_ONLY_N ? (N) : MPCQP_ONLY_N)> : nullptr)
#else
#define MPCQP_L(N) &launch_solve<N>
#endif
const launcher_t kLaunchers[MPCQP_MAX_HORIZON + 1] = {
    nullptr,      MPCQP_L(1),  MPCQP_L(2),  MPCQP_L(3),  MPCQP_L(4),  MPCQP_L(5),  MPCQP_L(6),  MPCQP_L(7),
    MPCQP_L(8),   MPCQP_L(9),  MPCQP_L(10), MPCQP_L(11), MPCQP_L(12), MPCQP_L(13), MPCQP_L(14), MPCQP_L(15),
    MPCQP_L(16),  MPCQP_L(17), MPCQP_L(18), MPCQP_L(19), MPCQP_L(20), MPCQP_L(21), MPCQP_L(22), MPCQP_L(23),
    MPCQP_L(24),  MPCQP_L(25), MPCQP_L(26), MPCQP_L(27), MPCQP_L(28), MPCQP_L(29), MPCQP_L(30), MPCQP_L(31)};
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
  const size_t bytes = sizeof(double) * (size_t)model_stride(p->horizon) * (size_t)max_batch;
  e = hipMalloc(&w->model, bytes);
  if (e != hipSuccess) {
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
  kLaunchers[ws->p.horizon](s, ws->p, B, ws->model, u0, X, U, status, iters, active);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return fail(MPCQP_E_HIP, std::string("k_solve launch: ") + hipGetErrorString(e));
  return MPCQP_OK;
}

const double* mpcqp_model_buffer(const mpcqp_ws* ws) { return ws ? ws->model : nullptr; }

}  // extern "C"
