// Development microbenchmark (not part of the library): issue cost of the f64 instructions the
// solver's dense products and sweeps are made of, one wave alone on its SIMD and two waves per SIMD.
//   hipcc --offload-arch=gfx950 -O3 -o tools/micro/fma_rates tools/micro/fma_rates.hip && tools/micro/fma_rates
// Each kernel runs ITER x 32 instructions of one kind on 8 independent accumulators (throughput) or
// on one (latency) and reports s_memtime cycles per instruction per wave.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

constexpr int ITER = 256;

template <int KIND>
__global__ __launch_bounds__(64) void k(double* out, unsigned long long* cyc, double seed) {
  double a[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) a[i] = seed * (threadIdx.x + i);
  double w = seed + threadIdx.x, m = 1.0000001;
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < ITER; ++it) {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        if constexpr (KIND == 0) {  // v_fmac_f64_dpp row_newbcast, 8 independent accumulators
          asm volatile("v_fmac_f64_dpp %0, %1, %2 row_newbcast:3 row_mask:0xf bank_mask:0xf" : "+v"(a[i]) : "v"(w), "v"(m));
        } else if constexpr (KIND == 1) {  // v_fmac_f64 (VOP2), 8 independent
          asm volatile("v_fmac_f64 %0, %1, %2" : "+v"(a[i]) : "v"(w), "v"(m));
        } else if constexpr (KIND == 2) {  // v_fma_f64 (VOP3), 8 independent
          asm volatile("v_fma_f64 %0, %1, %2, %0" : "+v"(a[i]) : "v"(w), "v"(m));
        } else if constexpr (KIND == 3) {  // v_fmac_f64_dpp, one dependent chain
          asm volatile("v_fmac_f64_dpp %0, %1, %2 row_newbcast:3 row_mask:0xf bank_mask:0xf" : "+v"(a[0]) : "v"(w), "v"(m));
        } else if constexpr (KIND == 4) {  // v_fmac_f64, one dependent chain
          asm volatile("v_fmac_f64 %0, %1, %2" : "+v"(a[0]) : "v"(w), "v"(m));
        } else if constexpr (KIND == 5) {  // v_mov_b32 (32-bit VALU), 8 independent
          int x;
          asm volatile("v_mov_b32 %0, %1" : "=v"(x) : "v"(i));
          a[i] += 0.0 * x;
        } else if constexpr (KIND == 6) {  // v_fmac_f64_dpp with 4 accumulators (the products' pattern)
          asm volatile("v_fmac_f64_dpp %0, %1, %2 row_newbcast:3 row_mask:0xf bank_mask:0xf" : "+v"(a[i & 3]) : "v"(w), "v"(m));
        }
      }
    }
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  double s = 0.0;
#pragma unroll
  for (int i = 0; i < 8; ++i) s += a[i];
  out[blockIdx.x * 64 + threadIdx.x] = s;
  if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

template <int KIND>
void run(const char* name, int blocks) {
  double* out;
  unsigned long long* cyc;
  hipMalloc(&out, sizeof(double) * blocks * 64);
  hipMalloc(&cyc, sizeof(unsigned long long) * blocks);
  for (int rep = 0; rep < 2; ++rep) hipLaunchKernelGGL(k<KIND>, dim3(blocks), dim3(64), 0, 0, out, cyc, 1e-3);
  hipDeviceSynchronize();
  std::vector<unsigned long long> h(blocks);
  hipMemcpy(h.data(), cyc, sizeof(unsigned long long) * blocks, hipMemcpyDeviceToHost);
  double mean = 0;
  for (auto v : h) mean += (double)v;
  mean /= blocks;
  const double insts = (double)ITER * 32;
  printf("{\"kind\": \"%s\", \"waves\": %d, \"cycles_per_inst\": %.3f}\n", name, blocks, mean / insts);
  hipFree(out);
  hipFree(cyc);
}

int main() {
  int cus = 0;
  hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
  for (int per : {1, 2, 3}) {
    const int blocks = cus * 4 * per;
    run<0>("fmac_f64_dpp x8", blocks);
    run<1>("fmac_f64 x8", blocks);
    run<2>("fma_f64 vop3 x8", blocks);
    run<3>("fmac_f64_dpp chain", blocks);
    run<4>("fmac_f64 chain", blocks);
    run<5>("mov_b32 x8", blocks);
    run<6>("fmac_f64_dpp x4", blocks);
  }
  return 0;
}
