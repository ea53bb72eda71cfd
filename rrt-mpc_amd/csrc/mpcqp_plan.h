// mpcqp_plan.h -- device bodies of the planner stages (RRT* growth, path extraction + shortcut
// pruning, centripetal Catmull-Rom smoothing), one planning problem per workgroup.  Shared by
// the public batched entry points (mpcqp_rrt.hip) and the masked per-step replanning of the
// swarm (mpcqp_swarm.hip).
#pragma once
#include "mpcqp_common.h"
#include "mpcqp_math.h"

namespace {

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
  const double dist = mpcqp_math::py_hypot(dx, dy);
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
  double qx, qy;  // this iteration's sample (device sampling)
};

// numpy's PCG64 (bit_generator.state: state, inc) and the Generator draws _sample makes
struct Pcg64 {
  unsigned __int128 s, inc;
  int has32;
  uint32_t u32;
  __device__ uint64_t next64() {
    const unsigned __int128 mult = ((unsigned __int128)0x2360ED051FC65DA4ull << 64) | 0x4385DF649FCCF645ull;
    s = s * mult + inc;
    const uint64_t hi = (uint64_t)(s >> 64), lo = (uint64_t)s;
    const uint64_t x = hi ^ lo;
    const unsigned r = (unsigned)(s >> 122);
    return (x >> r) | (x << ((64u - r) & 63u));
  }
  __device__ uint32_t next32() {
    if (has32) {
      has32 = 0;
      return u32;
    }
    const uint64_t v = next64();
    has32 = 1;
    u32 = (uint32_t)(v >> 32);
    return (uint32_t)v;
  }
  __device__ double random() { return (double)(next64() >> 11) * (1.0 / 9007199254740992.0); }
  __device__ uint32_t bounded(uint32_t n) {  // integers(0, n), n >= 2
    uint64_t m = (uint64_t)next32() * n;
    uint32_t left = (uint32_t)m;
    if (left < n) {
      const uint32_t thr = (uint32_t)(0u - n) % n;
      while (left < thr) {
        m = (uint64_t)next32() * n;
        left = (uint32_t)m;
      }
    }
    return (uint32_t)(m >> 32);
  }
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

// RRTStarPlanner.plan's tree growth for ONE problem on the calling 256-thread workgroup (see
// mpcqp_rrt.hip): sg = {start x, y, goal x, y}; samples (max_iterations x 2) or the PCG64 state
// (4 uint64); nodes_out (max_iterations + 2) x 4, *count_out, meta_out[2] = {iterations, goal}.
// lds: (max_iterations + 2) * (3 doubles + 1 int) of dynamic shared memory.
__device__ void rrt_grow_one(const mpcqp_rrt_params& p, const uint8_t* __restrict__ occ, const double* sg,
                             const double* __restrict__ samples, const uint64_t* __restrict__ rng_state,
                             double* __restrict__ nodes_out, int32_t* __restrict__ count_out,
                             int32_t* __restrict__ meta_out, double* lds, PlanSmem& sm) {
#pragma clang fp contract(off)
  const int tid = threadIdx.x;
  const int M = p.max_iterations + 2;
  double* X = lds;
  double* Y = lds + M;
  double* C = lds + 2 * M;
  int* Par = reinterpret_cast<int*>(lds + 3 * M);
  const Grid g{occ, p.width, p.height, p.collision_step};
  const double sx0 = sg[0], sy0 = sg[1];
  const double gx = sg[2], gy = sg[3];
  if (tid == 0) {
    X[0] = sx0;
    Y[0] = sy0;
    C[0] = 0.0;
    Par[0] = -1;
  }
  __syncthreads();
  int count = 1, goal_index = -1, iterations = 0;
  const double* smp = samples;
  Pcg64 rng{};
  if (!smp && tid == 0) {
    const uint64_t* r = rng_state;  // {state lo, state hi, inc lo, inc hi}
    rng.s = ((unsigned __int128)r[1] << 64) | r[0];
    rng.inc = ((unsigned __int128)r[3] << 64) | r[2];
    rng.has32 = 0;
    rng.u32 = 0;
  }
  for (int it = 1; it <= p.max_iterations; ++it) {
    iterations = it;
    double qx, qy;
    if (smp) {
      qx = smp[2 * (it - 1)];
      qy = smp[2 * (it - 1) + 1];
    } else {  // _sample (rrt_star.py:320-325): one draw sequence per iteration, kept or not
      if (tid == 0) {
        if (rng.random() < p.goal_sample_rate) {
          sm.qx = gx;
          sm.qy = gy;
        } else {
          const uint32_t yy = rng.bounded((uint32_t)p.height);
          const uint32_t xx = rng.bounded((uint32_t)p.width);
          sm.qx = (double)xx;
          sm.qy = (double)yy;
        }
      }
      __syncthreads();
      qx = sm.qx;
      qy = sm.qy;
    }
    // nearest (np.argmin: first minimum)
    double bd = INFINITY;
    int bi = 0x7fffffff;
    for (int i = tid; i < count; i += kPlanThreads) {
      const double d = mpcqp_math::py_hypot(X[i] - qx, Y[i] - qy);
      if (d < bd) {
        bd = d;
        bi = i;
      }
    }
    block_argmin(bd, bi, sm);
    const int near = bi;
    const double fx = X[near], fy = Y[near];
    // _steer (rrt_star.py:307-311): math.atan2 / cos / sin, correctly rounded (mpcqp_math.h)
    double th, cth, sth;
    mpcqp_math::cr_steer(qy - fy, qx - fx, th, cth, sth);
    const double nx = fx + p.step * cth;
    const double ny = fy + p.step * sth;
    if (!(0.0 <= nx && nx < (double)p.width && 0.0 <= ny && ny < (double)p.height)) continue;
    if (!block_all(segment_free(g, fx, fy, nx, ny, tid, kPlanThreads), sm)) continue;
    // choose parent
    const double c0 = C[near] + mpcqp_math::py_hypot(fx - nx, fy - ny);
    double bc = INFINITY;
    int bp = 0x7fffffff;
    for (int i = tid; i < count; i += kPlanThreads) {
      const double d = mpcqp_math::py_hypot(X[i] - nx, Y[i] - ny);
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
      const double d = mpcqp_math::py_hypot(X[i] - nx, Y[i] - ny);
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
    if (mpcqp_math::py_hypot(nx - gx, ny - gy) < p.goal_radius) {
      if (!block_all(segment_free(g, nx, ny, gx, gy, tid, kPlanThreads), sm)) continue;
      if (tid == 0) {
        X[count] = gx;
        Y[count] = gy;
        C[count] = cost + mpcqp_math::py_hypot(nx - gx, ny - gy);
        Par[count] = ni;
      }
      goal_index = count;
      count += 1;
      __syncthreads();
      break;
    }
  }
  double* out = nodes_out;
  for (int i = tid; i < count; i += kPlanThreads) {
    out[4 * i + 0] = X[i];
    out[4 * i + 1] = Y[i];
    out[4 * i + 2] = C[i];
    out[4 * i + 3] = (double)Par[i];
  }
  if (tid == 0) {
    *count_out = count;
    meta_out[0] = iterations;
    meta_out[1] = goal_index;
  }
}

// Path extraction + shortcut pruning (rrt_star.py:245-262, _shortcut_prune :376-389) for the
// trees k_rrt_plan grew, one workgroup per problem.  Thread 0 walks the parent chain from the
// goal node into LDS; each pruning step i -> j takes the farthest j (> i + 1) whose segment is
// free, else i + 1 -- the reference's "j from the end down to the first free segment" loop.
// The candidates j are spread over the threads (each thread scans its own j's from the far
// end, so its first free one is its largest) and a block max picks j.  Coordinates are copied,
// never recomputed: raw and pruned paths are the host restatement's values bit for bit.
__device__ void rrt_extract_one(const mpcqp_rrt_params& p, int prune, const uint8_t* __restrict__ occ,
                                const double* __restrict__ nodes, const int32_t* __restrict__ count,
                                const int32_t* __restrict__ meta, double* __restrict__ raw, int32_t* __restrict__ raw_len,
                                double* __restrict__ pruned, int32_t* __restrict__ pruned_len, double* lds,
                                PlanSmem& sm) {
  const int tid = threadIdx.x;
  const int M = p.max_iterations + 2;
  double* X = lds;
  double* Y = lds + M;
  const double* tree = nodes;
  const int goal = meta[1];
  const int cnt = min(*count, M);
  if (tid == 0) {
    int n = 0;
    if (goal >= 0 && goal < cnt) {
      // depth first (bounded by the node count: a parent chain never revisits a node)
      for (int idx = goal; idx >= 0 && n < cnt; idx = (int)tree[4 * idx + 3]) ++n;
      int idx = goal;
      for (int k = n - 1; k >= 0; --k) {
        X[k] = tree[4 * idx];
        Y[k] = tree[4 * idx + 1];
        idx = (int)tree[4 * idx + 3];
      }
    }
    sm.flag = n;
  }
  __syncthreads();
  const int n = sm.flag;
  __syncthreads();
  double* r = raw;
  for (int k = tid; k < n; k += kPlanThreads) {
    r[2 * k] = X[k];
    r[2 * k + 1] = Y[k];
  }
  double* q = pruned;
  if (!prune || n <= 2) {
    for (int k = tid; k < n; k += kPlanThreads) {
      q[2 * k] = X[k];
      q[2 * k + 1] = Y[k];
    }
    if (tid == 0) {
      *raw_len = n;
      *pruned_len = n;
    }
    return;
  }
  const Grid g{occ, p.width, p.height, p.collision_step};
  if (tid == 0) {
    q[0] = X[0];
    q[1] = Y[0];
  }
  int k = 1;
  for (int i = 0; i < n - 1;) {  // every thread runs the same i sequence (block-uniform)
    int best = i + 1;
    for (int j = n - 1 - tid; j > i + 1; j -= kPlanThreads)
      if (segment_free(g, X[i], Y[i], X[j], Y[j], 0, 1)) {
        best = j;
        break;
      }
    double key = -(double)best;
    block_argmin(key, best, sm);
    if (tid == 0) {
      q[2 * k] = X[best];
      q[2 * k + 1] = Y[best];
    }
    ++k;
    i = best;
  }
  if (tid == 0) {
    *raw_len = n;
    *pruned_len = k;
  }
}

// Centripetal Catmull-Rom smoothing of one path on the calling wave (src/planning/rrt_star.py:104-159
// with _dedupe_consecutive :93-101), numpy's operations in numpy's order, uncontracted:
//   dedupe: keep a point when ||p - last kept|| > tol (sqrt of dx^2 + dy^2)
//   n == 1: the point; n == 2: (1 - t) p0 + t p1 on np.linspace(0, 1, max(2, S + 1))
//   else, segment i of [p0, pts, p_last]: knots t_{j+1} = t_j + (|d|^alpha if |d| > eps else eps),
//   t on np.linspace(t1, t2, max(2, S + 1), endpoint=False) = k * ((t2 - t1) / num) + t1, then the
//   Barry-Goldman pyramid; the last point appended.
// pts: LDS scratch for 2 * cap doubles.  Returns the number of points written (<= out_cap), or
// -1 when the deduplicated path exceeds cap or the output exceeds out_cap.  |.|^alpha is the
// device's pow (sqrt for alpha = 0.5), within an ulp of the host libm's.
__device__ int catmull_rom_one(const double* __restrict__ in, int P, int samples, double alpha, double tol,
                               double* pts, int cap, double* __restrict__ out, int out_cap) {
#pragma clang fp contract(off)
  const int lane = threadIdx.x & (kWave - 1);
  constexpr double eps = 1e-9;
  int n = 0;
  if (lane == 0 && P > 0) {
    pts[0] = in[0];
    pts[1] = in[1];
    n = 1;
    for (int i = 1; i < P && n >= 0; ++i) {
      const double dx = in[2 * i] - pts[2 * (n - 1)], dy = in[2 * i + 1] - pts[2 * (n - 1) + 1];
      if (sqrt(dx * dx + dy * dy) > tol) {
        if (n == cap) {
          n = -1;
          break;
        }
        pts[2 * n] = in[2 * i];
        pts[2 * n + 1] = in[2 * i + 1];
        ++n;
      }
    }
  }
  n = __shfl(n, 0, kWave);
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
  __syncthreads();
  if (n < 0) return -1;
  if (n <= 1) {
    if (n == 1 && lane < 2) {
      if (out_cap < 1) return -1;
      out[lane] = pts[lane];
    }
    return n;
  }
  const int num = samples + 1 > 2 ? samples + 1 : 2;
  if (n == 2) {
    if (num > out_cap) return -1;
    const double step = 1.0 / (double)(num - 1);
    for (int k = lane; k < num; k += kWave) {
      const double t = k == num - 1 ? 1.0 : (double)k * step + 0.0;
      out[2 * k] = (1.0 - t) * pts[0] + t * pts[2];
      out[2 * k + 1] = (1.0 - t) * pts[1] + t * pts[3];
    }
    return num;
  }
  const int total = (n - 1) * num + 1;
  if (total > out_cap) return -1;
  auto knot = [&](double ti, int a, int b) {  // tj(ti, pts[a], pts[b])
    const double dx = pts[2 * b] - pts[2 * a], dy = pts[2 * b + 1] - pts[2 * a + 1];
    const double d = sqrt(dx * dx + dy * dy);
    const double inc = d > eps ? (alpha == 0.5 ? sqrt(d) : pow(d, alpha)) : eps;
    return ti + inc;
  };
  for (int i = 0; i < n - 1; ++i) {
    // extended points [pts[0], pts..., pts[n-1]]: ext[j] = pts[clamp(j - 1, 0, n - 1)]
    const int i0 = i - 1 < 0 ? 0 : i - 1, i1 = i, i2 = i + 1, i3 = i + 2 > n - 1 ? n - 1 : i + 2;
    const double t0 = 0.0;
    const double t1 = knot(t0, i0, i1);
    const double t2 = knot(t1, i1, i2);
    const double t3 = knot(t2, i2, i3);
    const double d01 = fmax(t1 - t0, eps), d12 = fmax(t2 - t1, eps), d23 = fmax(t3 - t2, eps);
    const double d02 = fmax(t2 - t0, eps), d13 = fmax(t3 - t1, eps);
    const double step = (t2 - t1) / (double)num;
    for (int k = lane; k < num; k += kWave) {
      const double t = (double)k * step + t1;
      double c[2];
      for (int d = 0; d < 2; ++d) {
        const double p0 = pts[2 * i0 + d], p1 = pts[2 * i1 + d], p2 = pts[2 * i2 + d], p3 = pts[2 * i3 + d];
        const double a1 = (t1 - t) / d01 * p0 + (t - t0) / d01 * p1;
        const double a2 = (t2 - t) / d12 * p1 + (t - t1) / d12 * p2;
        const double a3 = (t3 - t) / d23 * p2 + (t - t2) / d23 * p3;
        const double b1 = (t2 - t) / d02 * a1 + (t - t0) / d02 * a2;
        const double b2 = (t3 - t) / d13 * a2 + (t - t1) / d13 * a3;
        c[d] = (t2 - t) / d12 * b1 + (t - t1) / d12 * b2;
      }
      out[2 * (i * num + k)] = c[0];
      out[2 * (i * num + k) + 1] = c[1];
    }
  }
  if (lane < 2) out[2 * (total - 1) + lane] = pts[2 * (n - 1) + lane];
  return total;
}

}  // namespace
