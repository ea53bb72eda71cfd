// mpcqp_inflate.hip -- occupancy-grid inflation on the device.
//
// Restates src/maps/inflate.py:18-51 as the reference runs it here (OpenCV absent ->
// _fallback_dilation): every cell within the disk dx^2 + dy^2 <= r^2 of an obstacle cell (0)
// becomes an obstacle; r <= 0 copies the grid.  One thread per output cell, B grids of one
// size per launch; byte traffic is (2r+1)^2 L1/L2-served reads per cell, one HBM pass over the
// grid in and out.
#include "mpcqp_common.h"

namespace {
using mpcqp::fail;

__global__ __launch_bounds__(256) void k_inflate(int B, int H, int W, int r, const uint8_t* __restrict__ occ,
                                                 uint8_t* __restrict__ out) {
  const int x = blockIdx.x * 16 + (threadIdx.x & 15);
  const int y = blockIdx.y * 16 + (threadIdx.x >> 4);
  const int b = blockIdx.z;
  if (x >= W || y >= H || b >= B) return;
  const uint8_t* g = occ + (size_t)b * H * W;
  uint8_t v = g[(size_t)y * W + x];
  if (r > 0 && v != 0) {
    const int y0 = max(0, y - r), y1 = min(H - 1, y + r);
    for (int yy = y0; yy <= y1 && v != 0; ++yy) {
      const int dy = yy - y;
      const int x0 = max(0, x - r), x1 = min(W - 1, x + r);
      for (int xx = x0; xx <= x1; ++xx) {
        const int dx = xx - x;
        if (dx * dx + dy * dy <= r * r && g[(size_t)yy * W + xx] == 0) {
          v = 0;
          break;
        }
      }
    }
  }
  out[(size_t)b * H * W + (size_t)y * W + x] = v;
}

}  // namespace

extern "C" {

int mpcqp_inflate(int B, int height, int width, int radius_px, const uint8_t* occupancy, uint8_t* out, void* stream) {
  if (B < 0 || height < 0 || width < 0) return fail(MPCQP_E_ARG, "negative size");
  if (B == 0 || height == 0 || width == 0) return MPCQP_OK;
  if (!occupancy || !out) return fail(MPCQP_E_ARG, "null argument");
  if (occupancy == out) return fail(MPCQP_E_ARG, "in-place inflation is not supported");
  dim3 grid((width + 15) / 16, (height + 15) / 16, B);
  hipLaunchKernelGGL(k_inflate, grid, dim3(256), 0, static_cast<hipStream_t>(stream), B, height, width, radius_px,
                     occupancy, out);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return fail(MPCQP_E_HIP, std::string("k_inflate launch: ") + hipGetErrorString(e));
  return MPCQP_OK;
}

}  // extern "C"
