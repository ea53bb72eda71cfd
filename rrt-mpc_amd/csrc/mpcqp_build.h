// mpcqp_build.h -- per-QP body of K1 (window -> LTV model), shared by k_build (caller-provided
// windows, mpcqp.hip) and k_fleet_build (windows gathered from each vehicle's reference,
// mpcqp_fleet.hip).
#pragma once
#include "mpcqp_common.h"

namespace {

// One wave per QP, lane k <= N holding window row k = (rx, ry, ryaw, rv):
//   unwrapped yaw (np.unwrap, mpc_controller.py:59-60), then linearize() at
//   ref[max(k-1,0)], u = 0 (mpc_controller.py:65-70,108; vehicle_model.py:24-45).
// x0l = x0[lane] on lanes 0..3, upl = u_prev[lane-4] on lanes 4..5.
// Model layout per QP (doubles): alpha[N] beta[N] gamma[N] eta[N] sigma[N] c0[N]
// c1[N] ref[(N+1)*4] x0[4] u_prev[2], stride model_stride(N).
// Every lane of the wave must call this (DPP reads inactive lanes as zero).
__device__ __forceinline__ void build_qp(const mpcqp_params& p, int lane, double rx, double ry, double ryaw,
                                         double rv, double x0l, double upl, double* __restrict__ mb) {
  const int N = p.horizon;
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
  if (lane < 6) mb[11 * N + 4 + lane] = lane < 4 ? x0l : upl;
}

}  // namespace
