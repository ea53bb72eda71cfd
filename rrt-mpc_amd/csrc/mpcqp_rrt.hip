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
// parent) lives in LDS.  The random samples (:320-325) replay numpy's stream exactly: either
// drawn on the host and passed in, or drawn here from each problem's PCG64 state (numpy's
// generator: 128-bit LCG step, XSL-RR output; random() = (next64 >> 11) * 2^-53;
// integers(0, n) = Lemire's bounded draw on next32, which hands out the two halves of one
// next64 in turn -- numpy's has_uint32 buffer).  Arithmetic is uncontracted; hypot / atan2 / sin / cos
// are the device's (within an ulp of the host libm).
#include "mpcqp_plan.h"

namespace {
using mpcqp::fail;

__global__ __launch_bounds__(kPlanThreads) void k_rrt_plan(mpcqp_rrt_params p, int V, const uint8_t* __restrict__ occ,
                                                            const double* __restrict__ start_goal,
                                                            const double* __restrict__ samples,
                                                            const uint64_t* __restrict__ rng_state,
                                                            double* __restrict__ nodes_out, int32_t* __restrict__ count_out,
                                                            int32_t* __restrict__ meta_out) {
  extern __shared__ double lds[];
  __shared__ PlanSmem sm;
  const int v = blockIdx.x;
  if (v >= V) return;
  const int M = p.max_iterations + 2;
  rrt_grow_one(p, occ, start_goal + 4 * (size_t)v, samples ? samples + (size_t)v * p.max_iterations * 2 : nullptr,
               samples ? nullptr : rng_state + 4 * (size_t)v, nodes_out + (size_t)v * M * 4, count_out + v,
               meta_out + 2 * (size_t)v, lds, sm);
}

// Path extraction + shortcut pruning (rrt_star.py:245-262, _shortcut_prune :376-389) for the
// trees k_rrt_plan grew, one workgroup per problem (rrt_extract_one, mpcqp_plan.h).
__global__ __launch_bounds__(kPlanThreads) void k_rrt_paths(mpcqp_rrt_params p, int V, int prune,
                                                             const uint8_t* __restrict__ occ,
                                                             const double* __restrict__ nodes,
                                                             const int32_t* __restrict__ count,
                                                             const int32_t* __restrict__ meta,
                                                             double* __restrict__ raw, int32_t* __restrict__ raw_len,
                                                             double* __restrict__ pruned,
                                                             int32_t* __restrict__ pruned_len) {
  extern __shared__ double lds[];
  __shared__ PlanSmem sm;
  const int v = blockIdx.x;
  if (v >= V) return;
  const size_t M = (size_t)p.max_iterations + 2;
  rrt_extract_one(p, prune, occ, nodes + (size_t)v * M * 4, count + v, meta + 2 * (size_t)v, raw + (size_t)v * M * 2,
                  raw_len + v, pruned + (size_t)v * M * 2, pruned_len + v, lds, sm);
}

// The planner's elementary functions over arrays (mpcqp_plan_math): the values the RRT* kernels use.
__global__ __launch_bounds__(256) void k_plan_math(int op, int n, const double* __restrict__ a,
                                                    const double* __restrict__ b, double* __restrict__ o0,
                                                    double* __restrict__ o1, double* __restrict__ o2) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  if (op == 0) {
    o0[i] = mpcqp_math::py_hypot(a[i], b[i]);
  } else {
    double th, c, s;
    mpcqp_math::cr_steer(a[i], b[i], th, c, s);
    o0[i] = th;
    o1[i] = c;
    o2[i] = s;
  }
}

}  // namespace

extern "C" {

int mpcqp_plan_math(int op, int n, const double* a, const double* b, double* out0, double* out1, double* out2,
                    void* stream) {
  if (op != 0 && op != 1) return fail(MPCQP_E_ARG, "op must be 0 (hypot) or 1 (steer)");
  if (n < 0) return fail(MPCQP_E_ARG, "n must be >= 0");
  if (n == 0) return MPCQP_OK;
  if (!a || !b || !out0 || (op == 1 && (!out1 || !out2))) return fail(MPCQP_E_ARG, "null argument");
  hipLaunchKernelGGL(k_plan_math, dim3((n + 255) / 256), dim3(256), 0, static_cast<hipStream_t>(stream), op, n, a, b,
                     out0, out1, out2);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return fail(MPCQP_E_HIP, std::string("k_plan_math launch: ") + hipGetErrorString(e));
  return MPCQP_OK;
}

int mpcqp_rrt_paths(const mpcqp_rrt_params* p, int V, int prune, const uint8_t* occupancy, const double* nodes,
                    const int32_t* count, const int32_t* meta, double* raw, int32_t* raw_len, double* pruned,
                    int32_t* pruned_len, void* stream) {
  if (!p) return fail(MPCQP_E_ARG, "null params");
  if (V < 0) return fail(MPCQP_E_ARG, "V must be >= 0");
  if (V == 0) return MPCQP_OK;
  if (!occupancy || !nodes || !count || !meta || !raw || !raw_len || !pruned || !pruned_len)
    return fail(MPCQP_E_ARG, "null argument");
  if (p->max_iterations < 1 || p->max_iterations > kMaxPlanIterations)
    return fail(MPCQP_E_ARG, "max_iterations outside [1, " + std::to_string(kMaxPlanIterations) + "]");
  if (p->width < 2 || p->height < 2) return fail(MPCQP_E_ARG, "grid must be at least 2 x 2");
  const size_t lds = (size_t)(p->max_iterations + 2) * 2 * sizeof(double);
  if (lds > 65536) {
    hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(&k_rrt_paths),
                                       hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e != hipSuccess) return fail(MPCQP_E_HIP, std::string("hipFuncSetAttribute: ") + hipGetErrorString(e));
  }
  hipLaunchKernelGGL(k_rrt_paths, dim3(V), dim3(kPlanThreads), lds, static_cast<hipStream_t>(stream), *p, V,
                     prune, occupancy, nodes, count, meta, raw, raw_len, pruned, pruned_len);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return fail(MPCQP_E_HIP, std::string("k_rrt_paths launch: ") + hipGetErrorString(e));
  return MPCQP_OK;
}

int mpcqp_rrt_plan(const mpcqp_rrt_params* p, int V, const uint8_t* occupancy, const double* start_goal,
                   const double* samples, const uint64_t* rng_state, double* nodes, int32_t* count, int32_t* meta,
                   void* stream) {
  if (!p) return fail(MPCQP_E_ARG, "null params");
  if (V < 0) return fail(MPCQP_E_ARG, "V must be >= 0");
  if (V == 0) return MPCQP_OK;
  if (!occupancy || !start_goal || !nodes || !count || !meta) return fail(MPCQP_E_ARG, "null argument");
  if (!samples && !rng_state) return fail(MPCQP_E_ARG, "need samples or rng_state");
  if (p->max_iterations < 1 || p->max_iterations > kMaxPlanIterations)
    return fail(MPCQP_E_ARG, "max_iterations outside [1, " + std::to_string(kMaxPlanIterations) + "]");
  if (p->width < 2 || p->height < 2) return fail(MPCQP_E_ARG, "grid must be at least 2 x 2");
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
                     occupancy, start_goal, samples, rng_state, nodes, count, meta);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return fail(MPCQP_E_HIP, std::string("k_rrt_plan launch: ") + hipGetErrorString(e));
  return MPCQP_OK;
}

}  // extern "C"
