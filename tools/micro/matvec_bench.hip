// Development microbenchmark: one-wave dense row-per-lane matvec y = R v (n = 40), dependent
// chain of T products, four broadcast strategies.  Not part of the library.
//   hipcc --offload-arch=gfx950 -O3 -o build/matvec_bench tools/micro/matvec_bench.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

constexpr int n = 40, W = 64, T = 256;

__device__ __forceinline__ void lds_sync() { __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront"); }

template <int L>
__device__ __forceinline__ double nb(double w) {
  long v = __builtin_bit_cast(long, w);
  const long o = __builtin_amdgcn_update_dpp(0L, v, 0x150 + L, 0xf, 0xf, false);
  return __builtin_bit_cast(double, o);
}
template <int L>
__device__ __forceinline__ void fmac_nb(double& acc, double w, double r) {
  asm volatile("v_fmac_f64_dpp %0, %1, %2 row_newbcast:%3 row_mask:0xf bank_mask:0xf"
               : "+v"(acc) : "v"(w), "v"(r), "i"(L));
}
__device__ __forceinline__ double readlane(double v, int l) {
  return __hiloint2double(__builtin_amdgcn_readlane(__double2hiint(v), l),
                          __builtin_amdgcn_readlane(__double2loint(v), l));
}

template <int V>
__global__ __launch_bounds__(W) void k(const double* __restrict__ R, double* __restrict__ out,
                                       unsigned long long* cyc) {
  extern __shared__ double dyn[];
  __shared__ double buf[64];
  const int lane = threadIdx.x;
  double r[n];
#pragma unroll
  for (int j = 0; j < n; ++j) r[j] = lane < n ? R[((size_t)blockIdx.x * n + j) * W + lane] : 0.0;
  double v = lane < n ? 1.0 : 0.0;
  if (lane < 64) buf[lane] = 0.0;
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < T; ++it) {
    double a0 = 0.0, a1 = 0.0;
    if constexpr (V == 0) {  // LDS broadcast of every element
      lds_sync();
      buf[lane] = v;
      lds_sync();
#pragma unroll
      for (int j = 0; j < n; j += 2) {
        a0 = fma(r[j], buf[j], a0);
        a1 = fma(r[j + 1], buf[j + 1], a1);
      }
    } else if constexpr (V == 1 || V == 2) {  // LDS replicate 16-chunks, DPP row_newbcast
      lds_sync();
      buf[lane] = v;
      lds_sync();
      double w[3];
#pragma unroll
      for (int c = 0; c < 3; ++c) w[c] = buf[16 * c + (lane & 15)];
#pragma unroll
      for (int c = 0; c < 3; ++c) {
#define ST(L)                                                       \
  if (16 * c + L < n) {                                             \
    if constexpr (V == 1) {                                         \
      if (L & 1) a1 = fma(nb<L>(w[c]), r[16 * c + L], a1);          \
      else a0 = fma(nb<L>(w[c]), r[16 * c + L], a0);                \
    } else {                                                        \
      if (L & 1) fmac_nb<L>(a1, w[c], r[16 * c + L]);               \
      else fmac_nb<L>(a0, w[c], r[16 * c + L]);                     \
    }                                                               \
  }
        ST(0) ST(1) ST(2) ST(3) ST(4) ST(5) ST(6) ST(7) ST(8) ST(9) ST(10) ST(11) ST(12) ST(13) ST(14) ST(15)
#undef ST
      }
    } else {  // readlane into SGPRs
#pragma unroll
      for (int j = 0; j < n; j += 2) {
        a0 = fma(r[j], readlane(v, j), a0);
        a1 = fma(r[j + 1], readlane(v, j + 1), a1);
      }
    }
    v = lane < n ? (a0 + a1) : 0.0;
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  out[(size_t)blockIdx.x * W + lane] = v;
  if (lane == 0) atomicAdd(cyc, t1 - t0);
  if (lane == 0 && dyn[0] == 12345.0) out[0] = 0;  // keep dynamic LDS allocated
}

int main() {
  const int B = 4096;
  std::vector<double> hR((size_t)B * n * W);
  for (size_t i = 0; i < hR.size(); ++i) hR[i] = ((i * 2654435761u) % 1000) / 1000.0 / n;
  double *R, *out;
  unsigned long long* cyc;
  hipMalloc(&R, hR.size() * 8);
  hipMalloc(&out, (size_t)B * W * 8);
  hipMalloc(&cyc, 8);
  hipMemcpy(R, hR.data(), hR.size() * 8, hipMemcpyHostToDevice);
  std::vector<double> ref;
  const char* names[] = {"lds_bcast", "dpp_nb_builtin", "dpp_nb_asm", "readlane"};
  for (int occ : {1, 2, 4}) {
    const size_t dyn = occ == 4 ? 1024 : (160 * 1024 / (4 * occ)) - 2048;
    for (int V = 0; V < 4; ++V) {
      auto kern = V == 0 ? k<0> : V == 1 ? k<1> : V == 2 ? k<2> : k<3>;
      hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)dyn);
      hipEvent_t e0, e1;
      hipEventCreate(&e0);
      hipEventCreate(&e1);
      float best = 1e30f;
      unsigned long long hc = 0;
      for (int rep = 0; rep < 3; ++rep) {
        hipMemset(cyc, 0, 8);
        hipEventRecord(e0);
        hipLaunchKernelGGL(kern, dim3(B), dim3(W), dyn, 0, R, out, cyc);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms;
        hipEventElapsedTime(&ms, e0, e1);
        if (ms < best) best = ms;
        hipMemcpy(&hc, cyc, 8, hipMemcpyDeviceToHost);
      }
      std::vector<double> h((size_t)B * W);
      hipMemcpy(h.data(), out, h.size() * 8, hipMemcpyDeviceToHost);
      double err = 0;
      if (ref.empty()) ref = h;
      for (size_t i = 0; i < h.size(); ++i) err = fmax(err, fabs(h[i] - ref[i]) / (fabs(ref[i]) + 1e-300));
      printf("occ~%d %-15s %8.3f ms  %7.0f cyc/matvec/wave  relerr %.2e\n", occ, names[V], best,
             (double)hc / B / T, err);
    }
  }
  return 0;
}
