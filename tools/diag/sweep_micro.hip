// Development: cycles of the long-horizon sweep in isolation (one 256-thread workgroup per CU,
// K in LDS) -- hipcc -O3 --offload-arch=gfx950 -I include -I rrt-mpc_amd/csrc tools/diag/sweep_micro.hip
#define MPCQP_SWEEP_MICRO 1
#include "mpcqp_wide.hip"
#include <cstdio>
#include <vector>

__global__ __launch_bounds__(256) void k_micro(const double* Kin, double* out, unsigned long long* cyc, int n, int reps) {
  extern __shared__ double lds[];
  const int ks = n + 1;
  for (int e = threadIdx.x; e < n * ks; e += 256) lds[e] = Kin[e];
  __syncthreads();
  double* c0 = lds + n * ks;
  double* c1 = c0 + n + 64;
  unsigned long long t0 = __builtin_amdgcn_s_memtime(), t1 = 0;
  unsigned long long r0 = __builtin_amdgcn_s_memrealtime();
  bool ok = true;
  for (int r = 0; r < reps; ++r) {
    const int per = 256 / n, chunk = (n + per - 1) / per;
    if (chunk <= 16) ok = ok && sweep_regs<16, 3>(lds, c0, c1, n, ks, threadIdx.x);
    else if (chunk <= 32) ok = ok && sweep_regs<32, 3>(lds, c0, c1, n, ks, threadIdx.x);
    else ok = ok && sweep_regs<64, 3>(lds, c0, c1, n, ks, threadIdx.x);
  }
  t1 = __builtin_amdgcn_s_memtime();
  unsigned long long r1 = __builtin_amdgcn_s_memrealtime();
  if (threadIdx.x == 0) { cyc[2 * blockIdx.x] = t1 - t0; cyc[2 * blockIdx.x + 1] = r1 - r0; }
  for (int e = threadIdx.x; e < n * ks; e += 256) out[(size_t)blockIdx.x * n * ks + e] = lds[e];
  if (threadIdx.x == 0 && !ok) out[0] = -1.0;
}

__global__ __launch_bounds__(256) void k_barrier(double* out, unsigned long long* cyc, int n, int reps, int mode) {
  extern __shared__ double lds[];
  for (int e = threadIdx.x; e < 4096; e += 256) lds[e] = 1.0 + e;
  __syncthreads();
  double acc = 0.0;
  unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int r = 0; r < reps; ++r)
    for (int k = 0; k < n; ++k) {
      if (mode >= 1) __syncthreads();
      if (mode >= 2) acc += lds[k];
      if (mode == 3) acc = 1.0 / acc;
      if (mode == 4) {
        float a[8];
#pragma unroll
        for (int q = 0; q < 8; ++q) a[q] = (float)acc + q;
#pragma unroll
        for (int it = 0; it < 32; ++it)
#pragma unroll
          for (int q = 0; q < 8; ++q) a[q] = __builtin_fmaf(a[q], 1.0001f, 0.5f);
        float t = 0.f;
#pragma unroll
        for (int q = 0; q < 8; ++q) t += a[q];
        acc += t;
      }
    }
  unsigned long long t1 = __builtin_amdgcn_s_memtime();
  if (threadIdx.x == 0) cyc[2 * blockIdx.x] = t1 - t0;
  out[blockIdx.x * 256 + threadIdx.x] = acc;
}

int main(int argc, char** argv) {
  if (argc > 3) {
    const int n = atoi(argv[1]), reps = atoi(argv[2]), mode = atoi(argv[3]);
    double* dO; unsigned long long* dc;
    hipMalloc(&dO, 256 * 256 * 8); hipMalloc(&dc, 256 * 16);
    hipLaunchKernelGGL(k_barrier, dim3(256), dim3(256), 4096 * 8, 0, dO, dc, n, reps, mode);
    std::vector<unsigned long long> c(512);
    hipMemcpy(c.data(), dc, 256 * 16, hipMemcpyDeviceToHost);
    printf("mode %d: %.1f ticks per step (mode 4: 256 fp32 FMAs + 8 adds per step, 1 wave/SIMD)\n", mode, (double)c[0] / n / reps);
    return 0;
  }
  const int n = argc > 1 ? atoi(argv[1]) : 64, reps = argc > 2 ? atoi(argv[2]) : 10, B = 256;
  const int ks = n + 1;
  std::vector<double> K(n * ks, 0.0);
  for (int i = 0; i < n; ++i)
    for (int j = 0; j < n; ++j) K[i * ks + j] = (i == j ? n + 1.0 : 0.0) + 1.0 / (1.0 + i + j);
  double *dK, *dO; unsigned long long* dc;
  hipMalloc(&dK, K.size() * 8); hipMalloc(&dO, (size_t)B * K.size() * 8); hipMalloc(&dc, B * 16);
  hipMemcpy(dK, K.data(), K.size() * 8, hipMemcpyHostToDevice);
  const size_t lds = (n * ks + 2 * (n + 64)) * 8;
  (void)hipFuncSetAttribute(reinterpret_cast<const void*>(k_micro), hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  hipLaunchKernelGGL(k_micro, dim3(B), dim3(256), lds, 0, dK, dO, dc, n, 1);
  hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);
  hipEventRecord(a);
  hipLaunchKernelGGL(k_micro, dim3(B), dim3(256), lds, 0, dK, dO, dc, n, reps);
  hipEventRecord(b); hipEventSynchronize(b);
  float ms; hipEventElapsedTime(&ms, a, b);
  std::vector<unsigned long long> c(2 * B);
  hipMemcpy(c.data(), dc, B * 16, hipMemcpyDeviceToHost);
  double s = 0, rt = 0;
  for (int i = 0; i < B; ++i) { s += c[2 * i]; rt += c[2 * i + 1]; }
  printf("n=%d reps=%d: %.0f memtime ticks/sweep, %.1f us/sweep (realtime 100MHz), kernel %.3f ms -> %.1f us/sweep; ticks/us %.0f\n",
         n, reps, s / B / reps, rt / B / reps / 100.0, ms, ms * 1e3 / reps, (s / B) / (rt / B / 100.0));
  return 0;
}
