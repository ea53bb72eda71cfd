// Development microbenchmark (not part of the library): the one-wave solver's KKT sweep (Ctx<N>::sweep,
// rrt-mpc_amd/csrc/mpcqp_solve.h) and inverse product (inv_mul) in isolation, one wave alone on its SIMD
// and two per SIMD; cycles per pivot / per product from s_memtime.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=on -Wno-unused-value -I rrt-mpc_amd/csrc \
//     -o tools/micro/sweep_bench tools/micro/sweep_bench.hip && tools/micro/sweep_bench
#include "mpcqp_solve.h"

#include <cstdio>
#include <vector>

#ifndef SB_N
#define SB_N 20
#endif
constexpr int NN = SB_N, nn = 2 * SB_N, REPS = 16;

// the sweep with the pivot column broadcast staged through LDS (one ds_write, kNW ds_reads per step)
// instead of the permlane swaps: the variant under test
template <class Cx>
__device__ __forceinline__ bool sweep_lds(Cx& C, double* __restrict__ buf) {
  constexpr int n = Cx::n, NW = Cx::kNW;
  bool ok = true;
  const int lane = C.lane;
  const int rl = lane & 15;
  // column 0 published
  buf[lane] = C.r[0];
  Unroll<0, n>::run([&](auto kc) {
    constexpr int k = decltype(kc)::value;
    double* bk = buf + (k & 1) * 64;
    lds_sync();
    double w[4];
    Unroll<0, NW>::run([&](auto cc) {
      constexpr int c = decltype(cc)::value;
      w[c] = bk[16 * c + rl];
    });
    const double d = bk[k];
    asm volatile("s_nop 1" : "+v"(w[0]));
    ok = ok && (d > 0.0) && isfinite(d);
    double inv = __builtin_amdgcn_rcp(d);
    inv = fma(inv, fma(-d, inv, 1.0), inv);
    inv = fma(inv, fma(-d, inv, 1.0), inv);
    const bool piv = lane == k;
    const double ck = C.r[k] * inv;
    const double coef = piv ? inv - 1.0 : -ck;
    if constexpr (k + 1 < n) {
      fmac_bc<(k + 1) % 16>(C.r[k + 1], w[(k + 1) / 16], coef);
      buf[((k + 1) & 1) * 64 + lane] = C.r[k + 1];  // the next pivot column, published early
    }
    Unroll<0, n>::run([&](auto jc) {
      constexpr int j = decltype(jc)::value;
      if constexpr (j != k && j != k + 1) fmac_bc<j % 16>(C.r[j], w[j / 16], coef);
    });
    C.r[k] = piv ? -inv : ck;
  });
  return ok;
}

// the inverse product with the operand broadcast staged through LDS
template <class Cx>
__device__ __forceinline__ double inv_mul_lds(const Cx& C, double v, double* __restrict__ buf) {
  constexpr int n = Cx::n, NW = Cx::kNW;
  const int rl = C.lane & 15;
  lds_sync();
  buf[C.lane] = C.act ? v : 0.0;
  lds_sync();
  double w[4];
  Unroll<0, NW>::run([&](auto cc) {
    constexpr int c = decltype(cc)::value;
    w[c] = buf[16 * c + rl];
  });
  asm volatile("s_nop 1" : "+v"(w[0]));
  double a[4] = {0.0, 0.0, 0.0, 0.0};
  Unroll<0, n>::run([&](auto jc) {
    constexpr int j = decltype(jc)::value;
    fmac_bc<j % 16>(a[j % 4], w[j / 16], C.r[j]);
  });
  return -((a[0] + a[1]) + (a[2] + a[3]));
}

template <int MODE>
__global__ __launch_bounds__(64, 2) void k_bench(const double* __restrict__ A, double* __restrict__ out,
                                                 unsigned long long* cyc) {
  __shared__ SolveLds<NN> sm;
  __shared__ double bbuf[128];
  Ctx<NN> C;
  const int lane = threadIdx.x;
  C.init(lane, 0.1, sm.solve);
#pragma unroll
  for (int j = 0; j < nn; ++j) C.r[j] = lane < nn ? A[j * 64 + lane] : 0.0;
  double v = lane < nn ? 1.0 + 0.001 * lane : 0.0;
  bool ok = true;
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int rep = 0; rep < REPS; ++rep) {
    if constexpr (MODE == 0) {
      ok = C.sweep() && ok;
    } else if constexpr (MODE == 2) {
      ok = sweep_lds(C, bbuf) && ok;
    } else if constexpr (MODE == 3) {
      v = inv_mul_lds(C, v, bbuf) * 0.5;
    } else {
      v = C.inv_mul(v) * 0.5;
    }
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  double s = v + (ok ? 0.0 : 1.0);
#pragma unroll
  for (int j = 0; j < nn; ++j) s += C.r[j];
  out[blockIdx.x * 64 + lane] = s;
  if (lane == 0) cyc[blockIdx.x] = t1 - t0;
}

static std::vector<double> ref(64, 0.0);  // the reference sweep's outputs (MODE 0)

template <int MODE>
void run(const char* name, int blocks, const double* dA) {
  double* out;
  unsigned long long* cyc;
  hipMalloc(&out, sizeof(double) * blocks * 64);
  hipMalloc(&cyc, sizeof(unsigned long long) * blocks);
  for (int rep = 0; rep < 3; ++rep) hipLaunchKernelGGL(k_bench<MODE>, dim3(blocks), dim3(64), 0, 0, dA, out, cyc);
  hipDeviceSynchronize();
  std::vector<unsigned long long> h(blocks);
  hipMemcpy(h.data(), cyc, sizeof(unsigned long long) * blocks, hipMemcpyDeviceToHost);
  std::vector<double> o(64);
  hipMemcpy(o.data(), out, sizeof(double) * 64, hipMemcpyDeviceToHost);
  if (MODE == 0 || MODE == 1) ref = o;
  bool same = true;
  if (MODE == 2 || MODE == 3)
    for (int i = 0; i < 64; ++i) same = same && o[i] == ref[i];
  double mean = 0;
  for (auto x : h) mean += (double)x;
  mean /= blocks;
  const double per = MODE == 0 || MODE == 2 ? mean / (REPS * nn) : mean / REPS;
  printf("{\"N\": %d, \"what\": \"%s\", \"waves\": %d, \"cycles_per_%s\": %.1f, \"same_as_sweep\": %s}\n", NN,
         name, blocks, MODE == 0 || MODE == 2 ? "pivot" : "product", per, same ? "true" : "false");
  hipFree(out);
  hipFree(cyc);
}

int main() {
  // a well-conditioned SPD matrix: sweeping it back and forth stays finite
  std::vector<double> A(nn * 64, 0.0);
  for (int i = 0; i < nn; ++i)
    for (int j = 0; j < nn; ++j) A[j * 64 + i] = (i == j ? 4.0 : 0.0) + 1.0 / (1.0 + i + j);
  double* dA;
  hipMalloc(&dA, sizeof(double) * A.size());
  hipMemcpy(dA, A.data(), sizeof(double) * A.size(), hipMemcpyHostToDevice);
  int cus = 0;
  hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
  for (int per : {1, 2}) {
    run<0>("sweep", cus * 4 * per, dA);
    run<2>("sweep_lds_bcast", cus * 4 * per, dA);
    run<1>("inv_mul", cus * 4 * per, dA);
    run<3>("inv_mul_lds_bcast", cus * 4 * per, dA);
  }
  return 0;
}
