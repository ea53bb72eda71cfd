// mpcqp_build.h -- per-QP body of K1 (window -> LTV model), shared by k_build (caller-provided
// windows, mpcqp.hip) and k_fleet_build (windows gathered from each vehicle's reference,
// mpcqp_fleet.hip).
#pragma once
#include "mpcqp_common.h"

namespace {

// The LTV coefficients of lane k < N (step k) and the unwrapped yaw of lane k <= N.
struct LaneModel {
  double uyaw, al, be, ga, et, si, c0, c1;
};

// One wave per QP, lane k <= N holding window row k's yaw and speed: np.unwrap of the yaw
// (mpc_controller.py:59-60), then linearize() at ref[max(k-1,0)], u = 0 (mpc_controller.py:65-70,
// 108; vehicle_model.py:24-45).  Every lane of the wave must call this (DPP reads inactive lanes
// as zero).  Pair: the QP owns one 32-lane half (Lanes<true>, lane = the lane within it).
template <bool Pair = false>
__device__ __forceinline__ LaneModel build_lane(const mpcqp_params& p, int lane, double ryaw, double rv) {
  using LN = Lanes<Pair>;
  const int N = p.horizon;
  LaneModel m{};
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
  // cumsum in numpy's sequential order (bit-exact).  Every correction is +0.0 or nonzero (ddmod -
  // dd of equal finite values is +0.0), so a window without a wrap sums to +0.0 throughout.
  double cs = 0.0, mine = 0.0;
  if (LN::any(pc != 0.0))
    for (int j = 1; j <= N; ++j) {
      cs = cs + LN::readv(pc, j);
      if (lane == j) mine = cs;
    }
  m.uyaw = lane == 0 ? ryaw : ryaw + mine;
  // linearisation point of step k: ref[max(k-1, 0)]
  const double psi_m1 = dpp<kWaveShr1>(m.uyaw);
  const double v_m1 = dpp<kWaveShr1>(rv);
  const double psi = lane == 0 ? m.uyaw : psi_m1;
  const double v = lane == 0 ? rv : v_m1;
  if (lane < N) {
    const double dt = p.dt, L = p.wheelbase_px;
    const double sec2 = 1.0 / (1.0 * 1.0 + 1e-9);
    double sn, c;
    sincos(psi, &sn, &c);
    m.al = -dt * v * sn;
    m.be = dt * c;
    m.ga = dt * v * c;
    m.et = dt * sn;
    m.si = dt * (v / L) * sec2;
    m.c0 = -m.al * psi;
    m.c1 = -m.ga * psi;
  }
  return m;
}

// build_lane + the model block of one QP written to mb (global or LDS):
// alpha[N] beta[N] gamma[N] eta[N] sigma[N] c0[N] c1[N] ref[(N+1)*4] x0[4] u_prev[2],
// stride model_stride(N).  x0l = x0[lane] on lanes 0..3, upl = u_prev[lane-4] on lanes 4..5.
template <bool Pair = false>
__device__ __forceinline__ void build_qp(const mpcqp_params& p, int lane, double rx, double ry, double ryaw,
                                         double rv, double x0l, double upl, double* __restrict__ mb) {
  const int N = p.horizon;
  const LaneModel m = build_lane<Pair>(p, lane, ryaw, rv);
  if (lane <= N) {
    mb[7 * N + 4 * lane + 0] = rx;
    mb[7 * N + 4 * lane + 1] = ry;
    mb[7 * N + 4 * lane + 2] = m.uyaw;
    mb[7 * N + 4 * lane + 3] = rv;
  }
  if (lane < N) {
    mb[lane] = m.al;
    mb[N + lane] = m.be;
    mb[2 * N + lane] = m.ga;
    mb[3 * N + lane] = m.et;
    mb[4 * N + lane] = m.si;
    mb[5 * N + lane] = m.c0;
    mb[6 * N + lane] = m.c1;
  }
  if (lane < 6) mb[11 * N + 4 + lane] = lane < 4 ? x0l : upl;
}

// Windows longer than a wave (N + 1 > 64 rows, the long-horizon solve): build_lane + build_qp over
// chunks of 64 rows (lane = row - base), the previous chunk's last raw yaw, unwrapped yaw, speed
// and running unwrap sum carried in -- per row the same operations in the same order.
// fetch(row, rx, ry, ryaw, rv) loads window row `row` <= N.  Every lane of the wave must call this.
template <class Fetch>
__device__ __forceinline__ void build_qp_long(const mpcqp_params& p, int lane, Fetch&& fetch, double x0l,
                                              double upl, double* __restrict__ mb) {
  const int N = p.horizon;
  const double dt = p.dt, L = p.wheelbase_px;
  const double sec2 = 1.0 / (1.0 * 1.0 + 1e-9);
  double c_yaw = 0.0, c_uyaw = 0.0, c_rv = 0.0, cs = 0.0;  // carries from the previous chunk
  for (int base = 0; base <= N; base += kWave) {
    const int k = base + lane;
    double rx = 0.0, ry = 0.0, ryaw = 0.0, rv = 0.0;
    if (k <= N) fetch(k, rx, ry, ryaw, rv);
    double prev = dpp<kWaveShr1>(ryaw);
    if (lane == 0) prev = c_yaw;
    double pc = 0.0;
    if (k >= 1 && k <= N) {
      const double dd = ryaw - prev;
      double ddmod = np_mod(dd + kPi, kTwoPi) + (-kPi);
      if (ddmod == -kPi && dd > 0.0) ddmod = kPi;
      pc = ddmod - dd;
      if (fabs(dd) < kPi) pc = 0.0;
    }
    // running sum in numpy's order; a chunk without a wrap leaves it unchanged (adding +0.0 to a
    // sum that is never -0.0 keeps its bits)
    double mine = cs;
    if (wave_any(pc != 0.0))
      for (int j = 0; j < kWave && base + j <= N; ++j) {
        if (base + j >= 1) cs = cs + readlane(pc, j);
        if (lane == j) mine = cs;
      }
    const double uyaw = k == 0 ? ryaw : ryaw + mine;
    double psi = dpp<kWaveShr1>(uyaw), v = dpp<kWaveShr1>(rv);
    if (lane == 0) {
      psi = k == 0 ? uyaw : c_uyaw;
      v = k == 0 ? rv : c_rv;
    }
    if (k <= N) {
      mb[7 * N + 4 * k + 0] = rx;
      mb[7 * N + 4 * k + 1] = ry;
      mb[7 * N + 4 * k + 2] = uyaw;
      mb[7 * N + 4 * k + 3] = rv;
    }
    if (k < N) {
      double sn, c;
      sincos(psi, &sn, &c);
      const double al = -dt * v * sn, ga = dt * v * c;
      mb[k] = al;
      mb[N + k] = dt * c;
      mb[2 * N + k] = ga;
      mb[3 * N + k] = dt * sn;
      mb[4 * N + k] = dt * (v / L) * sec2;
      mb[5 * N + k] = -al * psi;
      mb[6 * N + k] = -ga * psi;
    }
    c_yaw = readlane(ryaw, kWave - 1);
    c_uyaw = readlane(uyaw, kWave - 1);
    c_rv = readlane(rv, kWave - 1);
  }
  if (lane < 6) mb[11 * N + 4 + lane] = lane < 4 ? x0l : upl;
}

// ---- the closed loop's per-step arithmetic, shared by k_fleet_advance (mpcqp_fleet.hip) and the
// fused loop k_fleet_loop (mpcqp_solve.h): numpy's operation order, no contraction.
// vehicle_model.py:11-21
__device__ __forceinline__ void plant(const double x[4], double a, double delta, double dt, double L, double out[4]) {
#pragma clang fp contract(off)
  out[0] = x[0] + dt * x[3] * cos(x[2]);
  out[1] = x[1] + dt * x[3] * sin(x[2]);
  out[2] = x[2] + dt * (x[3] / L) * tan(delta);
  out[3] = x[3] + dt * a;
}
// path_idx advance test (control_stage.py:141-145): farther than 5 px from ref row r
__device__ __forceinline__ bool fleet_off_row(double x, double y, const double* r) {
#pragma clang fp contract(off)
  const double dx = x - r[0];
  const double dy = y - r[1];
  return dx * dx + dy * dy > 25.0;
}
// the config-5 off-track trigger (README.md:146-148): farther than d from ref row r
__device__ __forceinline__ bool swarm_off_track(double x, double y, const double* r, double d) {
#pragma clang fp contract(off)
  return hypot(x - r[0], y - r[1]) > d;
}
// goal test (control_stage.py:147-150)
__device__ __forceinline__ bool fleet_at_goal(double x, double y, double gx, double gy) {
#pragma clang fp contract(off)
  return hypot(x - gx, y - gy) < 8.0;
}

}  // namespace
