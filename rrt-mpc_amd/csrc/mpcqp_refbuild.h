// mpcqp_refbuild.h -- build_reference on one wave (device body).
//
// One 64-lane wave per polyline restates src/control/ref_builder.py:10-22 with the helpers of
// src/common/geometry.py:9-45, in numpy's operation order:
//   step   = max(2, 0.8 * v * dt)
//   resample_polyline: s = [0, cumsum(hypot(diff))] (sequential), samples = i * step for
//          i < ceil(total / step) (numpy arange fill), total appended unless isclose(last, total);
//          np.interp on (s, x) and (s, y) (largest j with s[j] <= sample, slope form);
//          a path of < 2 points or total < 1e-9 is returned unchanged
//   heading_from_path: atan2 of the prepended differences, np.unwrap (sequential cumsum)
//   curvature_slowdown: v * (0.6 + 0.4 / (1 + 4 min(|dyaw|, pi - |dyaw|)))
//   tail padding to horizon + 1 rows with the last row
// Samples are processed 64 per pass with carries (previous point, raw heading, unwrap offset,
// yaw) between passes.  The polyline and its arc lengths are staged in LDS for the searches.
// Arithmetic is kept uncontracted; hypot and atan2 are the device's (within an ulp of glibc's).
#pragma once
#include "mpcqp_common.h"

namespace {

constexpr int kMaxPoints = 6144;  // LDS: 3 doubles per point (144 KB at the cap)

__device__ __forceinline__ double bcast_lane(double v, int l) { return readlane(v, l); }

// lane i <- lane i-1, lane 0 <- carry: wave_shr:1 with bound_ctrl off keeps `old` where the
// source lane is out of range.  One DPP per half, executed by every lane (no select that the
// compiler could turn into an exec-masked DPP whose source lane reads as zero).
__device__ __forceinline__ double shr1_carry(double v, double carry) {
  const int lo = __builtin_amdgcn_update_dpp(__double2loint(carry), __double2loint(v), kWaveShr1, 0xf, 0xf, false);
  const int hi = __builtin_amdgcn_update_dpp(__double2hiint(carry), __double2hiint(v), kWaveShr1, 0xf, 0xf, false);
  return __hiloint2double(hi, lo);
}

// One polyline pv[0..P) (x, y interleaved) -> ref (stride rows x 4) and *ref_len, on the calling
// wave; lds: 3 * cap doubles.
__device__ void build_reference_one(const double* __restrict__ pv, int P, int cap, double speed, int horizon, double dt,
                                    int stride, double* __restrict__ ref, int32_t* __restrict__ ref_len, double* lds) {
#pragma clang fp contract(off)
  const int lane = threadIdx.x;
  if (P < 0 || P > cap) {  // ragged offsets outside the staged capacity
    if (lane == 0) *ref_len = MPCQP_REF_BAD_PATH;
    return;
  }
  double* S = lds;
  double* X = lds + cap;
  double* Y = lds + 2 * cap;
  for (int i = lane; i < P; i += kWave) {
    X[i] = pv[2 * i];
    Y[i] = pv[2 * i + 1];
  }
  __syncthreads();
  // arc length: sequential cumsum of the segment lengths, 64 segments per pass
  double run = 0.0;
  if (lane == 0) S[0] = 0.0;
  for (int base = 0; base < P - 1; base += kWave) {
    const int i = base + lane;
    const double d = i < P - 1 ? hypot(X[i + 1] - X[i], Y[i + 1] - Y[i]) : 0.0;
    const int cnt = min(kWave, P - 1 - base);
    double mine = 0.0;
    for (int j = 0; j < cnt; ++j) {
      run = run + bcast_lane(d, j);
      if (lane == j) mine = run;
    }
    if (lane < cnt) S[i + 1] = mine;
  }
  __syncthreads();
  const double step = fmax(2.0, 0.8 * speed * dt);
  const double total = P > 0 ? S[P - 1] : 0.0;
  const bool raw = P < 2 || total < 1e-9;  // resample_polyline returns the points unchanged
  int K = 0, M = P;
  if (!raw) {
    K = (int)ceil(total / step);
    const double last = (double)(K - 1) * step;
    M = fabs(last - total) <= 1e-8 + 1e-5 * fabs(total) ? K : K + 1;
  }
  const int rows = M == 0 ? 0 : max(M, horizon + 1);
  if (lane == 0) *ref_len = rows <= stride ? rows : -rows;
  if (rows == 0 || rows > stride) return;
  double* out = ref;
  // carries between passes
  double px = 0.0, py = 0.0, praw = 0.0, cum = 0.0, pyaw = 0.0;
  double lx = 0.0, ly = 0.0, lyaw = 0.0, lv = 0.0;
  for (int base = 0; base < M; base += kWave) {
    const int i = base + lane;
    const bool in = i < M;
    double x = 0.0, y = 0.0;
    if (in) {
      if (raw) {
        x = X[i];
        y = Y[i];
      } else {
        const double xs = i < K ? (double)i * step : total;
        // np.interp: j = largest index with S[j] <= xs
        int j;
        if (xs > S[P - 1]) {
          j = P;
        } else {
          int lo = 0, hi = P;  // bisection as numpy's binary_search_with_guess
          while (lo < hi) {
            const int mid = lo + ((hi - lo) >> 1);
            if (xs >= S[mid]) lo = mid + 1;
            else hi = mid;
          }
          j = lo - 1;
        }
        if (j >= P - 1) {
          x = X[P - 1];
          y = Y[P - 1];
        } else if (S[j] == xs) {
          x = X[j];
          y = Y[j];
        } else {
          const double ds = S[j + 1] - S[j];
          const double sx = (X[j + 1] - X[j]) / ds;
          const double sy = (Y[j + 1] - Y[j]) / ds;
          x = sx * (xs - S[j]) + X[j];
          y = sy * (xs - S[j]) + Y[j];
          if (isnan(x)) {
            x = sx * (xs - S[j + 1]) + X[j + 1];
            if (isnan(x) && X[j] == X[j + 1]) x = X[j];
          }
          if (isnan(y)) {
            y = sy * (xs - S[j + 1]) + Y[j + 1];
            if (isnan(y) && Y[j] == Y[j + 1]) y = Y[j];
          }
        }
      }
    }
    // heading_from_path: differences with the first point prepended
    const double xm = shr1_carry(x, px);
    const double ym = shr1_carry(y, py);
    const double dxv = i == 0 ? 0.0 : x - xm;
    const double dyv = i == 0 ? 0.0 : y - ym;
    const double rw = atan2(dyv, dxv);
    // np.unwrap: corrections where |dd| >= pi, cumulated in index order
    const double rm = shr1_carry(rw, praw);
    double pc = 0.0;
    if (in && i >= 1) {
      const double dd = rw - rm;
      double ddmod = np_mod(dd + kPi, kTwoPi) + (-kPi);
      if (ddmod == -kPi && dd > 0.0) ddmod = kPi;
      pc = ddmod - dd;
      if (fabs(dd) < kPi) pc = 0.0;
    }
    double mine = cum;
    uint64_t nz = __ballot(pc != 0.0);
    while (nz) {
      const int l = __builtin_ctzll(nz);
      nz &= nz - 1;
      cum = cum + bcast_lane(pc, l);
      if (lane >= l) mine = cum;
    }
    const double yaw = i == 0 ? rw : rw + mine;
    // curvature_slowdown
    const double ym1 = shr1_carry(yaw, pyaw);
    double hd = i == 0 ? 0.0 : fabs(yaw - ym1);
    hd = fmin(hd, kPi - hd);
    const double slow = 1.0 / (1.0 + 4.0 * hd);
    const double vr = speed * (0.6 + 0.4 * slow);
    if (in) {
      double* o = out + (size_t)i * 4;
      o[0] = x;
      o[1] = y;
      o[2] = yaw;
      o[3] = vr;
    }
    const int lastl = min(kWave, M - base) - 1;
    px = bcast_lane(x, lastl);
    py = bcast_lane(y, lastl);
    praw = bcast_lane(rw, lastl);
    pyaw = bcast_lane(yaw, lastl);
    lx = px;
    ly = py;
    lyaw = pyaw;
    lv = bcast_lane(vr, lastl);
  }
  for (int i = M + lane; i < rows; i += kWave) {  // tail padding with the last row
    double* o = out + (size_t)i * 4;
    o[0] = lx;
    o[1] = ly;
    o[2] = lyaw;
    o[3] = lv;
  }
}

}  // namespace
