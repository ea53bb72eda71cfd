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

template <int MODE>
__global__ __launch_bounds__(64, 2) void k_bench(const double* __restrict__ A, double* __restrict__ out,
                                                 unsigned long long* cyc) {
  __shared__ SolveLds<NN> sm;
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
  double mean = 0;
  for (auto x : h) mean += (double)x;
  mean /= blocks;
  const double per = MODE == 0 ? mean / (REPS * nn) : mean / REPS;
  printf("{\"N\": %d, \"what\": \"%s\", \"waves\": %d, \"cycles_per_%s\": %.1f}\n", NN, name, blocks,
         MODE == 0 ? "pivot" : "product", per);
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
    run<1>("inv_mul", cus * 4 * per, dA);
  }
  return 0;
}
