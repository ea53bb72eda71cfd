// mpcqp_rrt.hip -- batched RRT* tree growth on the device.
//
// One 256-thread workgroup grows one planning problem's tree, restating
// RRTStarPlanner.plan (src/planning/rrt_star.py:201-248) iteration by iteration:
//   nearest        argmin of hypot over the tree, lowest index on ties          (:329-331)
//   steer          atan2 / cos / sin step from the nearest node                 (:333-337)
//   bounds + segment check (_segment_is_free: np.linspace samples, round-half-even,
//                  clipped grid lookups)                                         (:339-355)
//   choose parent  min cost over nodes within rewire_radius with a free segment;
//                  the nearest node unless a strictly cheaper one, first index   (:360-372)
//   rewire         every older node (not the root) within the radius that gets cheaper
//                  through the new node and has a free segment from it          (:374-383)
//   goal           within goal_radius and a free segment -> goal node appended  (:234-243)
// The per-iteration scans over the tree run across the 256 threads; the tree (x, y, cost,
// parent) lives in LDS.  The random samples (:320-325) are drawn on the host with the
// reference's own numpy calls (mpcqp/planning/rrt_star.py) and passed in, so every problem
// replays its seed's stream exactly.  Arithmetic is uncontracted; hypot / atan2 / sin / cos
// are the device's (within an ulp of the host libm).
#include "mpcqp_common.h"

namespace {
using mpcqp::fail;

constexpr int kPlanThreads = 256;
constexpr int kPlanWaves = kPlanThreads / kWave;
constexpr int kMaxPlanIterations = 5000;

struct Grid {
  const uint8_t* __restrict__ occ;
  int W, H;
  double cstep;
};

// _segment_is_free((ax, ay), (bx, by)): points i of np.linspace(a, b, n + 1) = i * step + a
// (last = b), Python round (half to even), clipped to the grid; false on an occupied cell.
// Points [i0, n] with stride `stride` (a single thread: i0 = 0, stride = 1).
__device__ bool segment_free(const Grid& g, double ax, double ay, double bx, double by, int i0, int stride) {
#pragma clang fp contract(off)
  const double dx = bx - ax, dy = by - ay;
  const double dist = hypot(dx, dy);
  const double st = fmax(g.cstep, 1e-3);
  const int n = max(1, (int)ceil(dist / st));
  const double sx = dx / n, sy = dy / n;
  for (int i = i0; i <= n; i += stride) {
    const double x = i == n ? bx : (double)i * sx + ax;
    const double y = i == n ? by : (double)i * sy + ay;
    const int xi = (int)fmin(fmax(rint(x), 0.0), (double)(g.W - 1));
    const int yi = (int)fmin(fmax(rint(y), 0.0), (double)(g.H - 1));
    if (g.occ[(size_t)yi * g.W + xi] == 0) return false;
  }
  return true;
}

struct PlanSmem {
  double red_d[kPlanWaves];
  int red_i[kPlanWaves];
  int flag;
};

// block argmin of (v, i): smallest v, then smallest i
__device__ void block_argmin(double& v, int& i, PlanSmem& s) {
  for (int o = kWave / 2; o > 0; o >>= 1) {
    const double v2 = __shfl_xor(v, o, kWave);
    const int i2 = __shfl_xor(i, o, kWave);
    if (v2 < v || (v2 == v && i2 < i)) {
      v = v2;
      i = i2;
    }
  }
  const int w = threadIdx.x / kWave;
  __syncthreads();
  if ((threadIdx.x & (kWave - 1)) == 0) {
    s.red_d[w] = v;
    s.red_i[w] = i;
  }
  __syncthreads();
  v = s.red_d[0];
  i = s.red_i[0];
  for (int k = 1; k < kPlanWaves; ++k)
    if (s.red_d[k] < v || (s.red_d[k] == v && s.red_i[k] < i)) {
      v = s.red_d[k];
      i = s.red_i[k];
    }
}

// block AND of a per-thread predicate
__device__ bool block_all(bool ok, PlanSmem& s) {
  __syncthreads();
  if (threadIdx.x == 0) s.flag = 1;
  __syncthreads();
  if (!ok) s.flag = 0;
  __syncthreads();
  return s.flag != 0;
}

__global__ __launch_bounds__(kPlanThreads) void k_rrt_plan(mpcqp_rrt_params p, int V, const uint8_t* __restrict__ occ,
                                                            const double* __restrict__ start_goal,
                                                            const double* __restrict__ samples,
                                                            double* __restrict__ nodes_out, int32_t* __restrict__ count_out,
                                                            int32_t* __restrict__ meta_out) {
#pragma clang fp contract(off)
  extern __shared__ double lds[];
  __shared__ PlanSmem sm;
  const int v = blockIdx.x;
  if (v >= V) return;
  const int tid = threadIdx.x;
  const int M = p.max_iterations + 2;
  double* X = lds;
  double* Y = lds + M;
  double* C = lds + 2 * M;
  int* Par = reinterpret_cast<int*>(lds + 3 * M);
  const Grid g{occ, p.width, p.height, p.collision_step};
  const double sx0 = start_goal[4 * v], sy0 = start_goal[4 * v + 1];
  const double gx = start_goal[4 * v + 2], gy = start_goal[4 * v + 3];
  if (tid == 0) {
    X[0] = sx0;
    Y[0] = sy0;
    C[0] = 0.0;
    Par[0] = -1;
  }
  __syncthreads();
  int count = 1, goal_index = -1, iterations = 0;
  const double* smp = samples + (size_t)v * p.max_iterations * 2;
  for (int it = 1; it <= p.max_iterations; ++it) {
    iterations = it;
    const double qx = smp[2 * (it - 1)], qy = smp[2 * (it - 1) + 1];
    // nearest (np.argmin: first minimum)
    double bd = INFINITY;
    int bi = 0x7fffffff;
    for (int i = tid; i < count; i += kPlanThreads) {
      const double d = hypot(X[i] - qx, Y[i] - qy);
      if (d < bd) {
        bd = d;
        bi = i;
      }
    }
    block_argmin(bd, bi, sm);
    const int near = bi;
    const double fx = X[near], fy = Y[near];
    const double th = atan2(qy - fy, qx - fx);
    const double nx = fx + p.step * cos(th);
    const double ny = fy + p.step * sin(th);
    if (!(0.0 <= nx && nx < (double)p.width && 0.0 <= ny && ny < (double)p.height)) continue;
    if (!block_all(segment_free(g, fx, fy, nx, ny, tid, kPlanThreads), sm)) continue;
    // choose parent
    const double c0 = C[near] + hypot(fx - nx, fy - ny);
    double bc = INFINITY;
    int bp = 0x7fffffff;
    for (int i = tid; i < count; i += kPlanThreads) {
      const double d = hypot(X[i] - nx, Y[i] - ny);
      if (d > p.rewire_radius) continue;
      if (!segment_free(g, X[i], Y[i], nx, ny, 0, 1)) continue;
      const double c = C[i] + d;
      if (c < bc) {
        bc = c;
        bp = i;
      }
    }
    block_argmin(bc, bp, sm);
    const int parent = bc < c0 ? bp : near;
    const double cost = bc < c0 ? bc : c0;
    const int ni = count;
    __syncthreads();
    if (tid == 0) {
      X[ni] = nx;
      Y[ni] = ny;
      C[ni] = cost;
      Par[ni] = parent;
    }
    __syncthreads();
    count = ni + 1;
    // rewire (every node updated at most once, from its own pre-rewire values)
    for (int i = tid; i < ni; i += kPlanThreads) {
      const double d = hypot(X[i] - nx, Y[i] - ny);
      if (d > p.rewire_radius) continue;
      if (Par[i] < 0) continue;
      const double c = cost + d;
      if (c < C[i] && segment_free(g, nx, ny, X[i], Y[i], 0, 1)) {
        C[i] = c;
        Par[i] = ni;
      }
    }
    __syncthreads();
    // goal
    if (hypot(nx - gx, ny - gy) < p.goal_radius) {
      if (!block_all(segment_free(g, nx, ny, gx, gy, tid, kPlanThreads), sm)) continue;
      if (tid == 0) {
        X[count] = gx;
        Y[count] = gy;
        C[count] = cost + hypot(nx - gx, ny - gy);
        Par[count] = ni;
      }
      goal_index = count;
      count += 1;
      __syncthreads();
      break;
    }
  }
  double* out = nodes_out + (size_t)v * M * 4;
  for (int i = tid; i < count; i += kPlanThreads) {
    out[4 * i + 0] = X[i];
    out[4 * i + 1] = Y[i];
    out[4 * i + 2] = C[i];
    out[4 * i + 3] = (double)Par[i];
  }
  if (tid == 0) {
    count_out[v] = count;
    meta_out[2 * v] = iterations;
    meta_out[2 * v + 1] = goal_index;
  }
}

}  // namespace

extern "C" {

int mpcqp_rrt_plan(const mpcqp_rrt_params* p, int V, const uint8_t* occupancy, const double* start_goal,
                   const double* samples, double* nodes, int32_t* count, int32_t* meta, void* stream) {
  if (!p) return fail(MPCQP_E_ARG, "null params");
  if (V < 0) return fail(MPCQP_E_ARG, "V must be >= 0");
  if (V == 0) return MPCQP_OK;
  if (!occupancy || !start_goal || !samples || !nodes || !count || !meta) return fail(MPCQP_E_ARG, "null argument");
  if (p->max_iterations < 1 || p->max_iterations > kMaxPlanIterations)
    return fail(MPCQP_E_ARG, "max_iterations outside [1, " + std::to_string(kMaxPlanIterations) + "]");
  if (p->width < 1 || p->height < 1) return fail(MPCQP_E_ARG, "empty grid");
  if (!(p->step > 0.0) || !(p->rewire_radius >= 0.0) || !(p->goal_radius >= 0.0) || !(p->collision_step >= 0.0))
    return fail(MPCQP_E_ARG, "bad planner parameters");
  const size_t lds = (size_t)(p->max_iterations + 2) * (3 * sizeof(double) + sizeof(int));
  const size_t lds_r = (lds + 7) / 8 * 8;
  if (lds_r > 65536) {
    hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(&k_rrt_plan),
                                       hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds_r);
    if (e != hipSuccess) return fail(MPCQP_E_HIP, std::string("hipFuncSetAttribute: ") + hipGetErrorString(e));
  }
  hipLaunchKernelGGL(k_rrt_plan, dim3(V), dim3(kPlanThreads), lds_r, static_cast<hipStream_t>(stream), *p, V,
                     occupancy, start_goal, samples, nodes, count, meta);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return fail(MPCQP_E_HIP, std::string("k_rrt_plan launch: ") + hipGetErrorString(e));
  return MPCQP_OK;
}

}  // extern "C"
