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
// as zero).
__device__ __forceinline__ LaneModel build_lane(const mpcqp_params& p, int lane, double ryaw, double rv) {
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
  if (wave_any(pc != 0.0))
    for (int j = 1; j <= N; ++j) {
      cs = cs + readlane(pc, j);
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
__device__ __forceinline__ void build_qp(const mpcqp_params& p, int lane, double rx, double ry, double ryaw,
                                         double rv, double x0l, double upl, double* __restrict__ mb) {
  const int N = p.horizon;
  const LaneModel m = build_lane(p, lane, ryaw, rv);
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

}  // namespace
