// mpcqp_refbuild.hip -- batched build_reference on the device.
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
#include "mpcqp_refbuild.h"

namespace {
using mpcqp::fail;

__global__ __launch_bounds__(kWave) void k_build_reference(int V, const double* __restrict__ pts,
                                                           const int32_t* __restrict__ off, int cap, double speed,
                                                           int horizon, double dt, int stride,
                                                           double* __restrict__ ref, int32_t* __restrict__ ref_len) {
  extern __shared__ double lds[];
  const int v = blockIdx.x;
  if (v >= V) return;
  const int p0 = off[v];
  build_reference_one(pts + (size_t)p0 * 2, off[v + 1] - p0, cap, speed, horizon, dt, stride,
                      ref + (size_t)v * stride * 4, ref_len + v, lds);
}

}  // namespace

extern "C" {

int mpcqp_build_reference(int V, const double* pts, const int32_t* path_off, int max_points, double desired_speed,
                          int horizon, double dt, int ref_stride, double* ref, int32_t* ref_len, void* stream) {
  if (V < 0) return fail(MPCQP_E_ARG, "V must be >= 0");
  if (V == 0) return MPCQP_OK;
  if (!pts || !path_off || !ref || !ref_len) return fail(MPCQP_E_ARG, "null argument");
  if (max_points < 0 || max_points > kMaxPoints)
    return fail(MPCQP_E_ARG, "max_points outside [0, " + std::to_string(kMaxPoints) + "]");
  if (horizon < 1 || horizon > MPCQP_MAX_HORIZON) return fail(MPCQP_E_HORIZON, "horizon outside [1, MPCQP_MAX_HORIZON]");
  if (ref_stride < 1) return fail(MPCQP_E_ARG, "ref_stride must be >= 1");
  if (!(dt > 0.0) || !(desired_speed > 0.0)) return fail(MPCQP_E_ARG, "dt and desired_speed must be > 0");
  const int cap = max_points > 0 ? max_points : 1;
  const size_t lds = sizeof(double) * 3 * (size_t)cap;
  if (lds > 65536) {  // past the default dynamic-LDS limit
    hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(&k_build_reference),
                                       hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e != hipSuccess) return fail(MPCQP_E_HIP, std::string("hipFuncSetAttribute: ") + hipGetErrorString(e));
  }
  hipLaunchKernelGGL(k_build_reference, dim3(V), dim3(kWave), lds, static_cast<hipStream_t>(stream), V, pts,
                     path_off, cap, desired_speed, horizon, dt, ref_stride, ref, ref_len);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return fail(MPCQP_E_HIP, std::string("k_build_reference launch: ") + hipGetErrorString(e));
  return MPCQP_OK;
}

}  // extern "C"
