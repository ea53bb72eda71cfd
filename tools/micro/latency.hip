// Development microbenchmark: cycles per operation for one lone wave (s_memtime), for the
// primitives of the ADMM iteration.  Not part of the library.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I rrt-mpc_amd/csrc -o tools/diag/latency tools/micro/latency.hip
#include <cstdio>

#include "mpcqp_common.h"

constexpr int R = 512;

template <int V>
__global__ __launch_bounds__(64) void k(const double* __restrict__ in, double* __restrict__ out,
                                        unsigned long long* cyc, int waves) {
  __shared__ double buf[128];
  if (blockIdx.x >= waves) return;
  const int lane = threadIdx.x;
  double v = in[lane], u = in[64 + lane];
  double r[40];
#pragma unroll
  for (int j = 0; j < 40; ++j) r[j] = in[lane] * (j + 1);
  buf[lane] = v;
  buf[64 + lane] = u;
  __syncthreads();
  double a0 = 0, a1 = 0, a2 = 0, a3 = 0;
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < R; ++it) {
    if constexpr (V == 0) {  // dependent v_fma_f64 chain: latency
#pragma unroll
      for (int j = 0; j < 16; ++j) v = fma(v, u, 1e-3);
    } else if constexpr (V == 1) {  // 4 independent chains: issue rate
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        a0 = fma(a0, u, 1e-3);
        a1 = fma(a1, u, 2e-3);
        a2 = fma(a2, u, 3e-3);
        a3 = fma(a3, u, 4e-3);
      }
    } else if constexpr (V == 2) {  // bcast + 40 v_fmac_f64_dpp (inv_mul body)
      double w[4];
      bcast<3>(v, w);
      double a[4] = {0, 0, 0, 0};
      Unroll<0, 40>::run([&](auto jc) {
        constexpr int j = decltype(jc)::value;
        fmac_bc<j % 16>(a[j % 4], w[j / 16], r[j]);
      });
      v = ((a[0] + a[1]) + (a[2] + a[3])) * 1e-3;
    } else if constexpr (V == 3) {  // prefix scan (row shifts + row_bcast)
      v = scan_add(v, lane) * 1e-3;
    } else if constexpr (V == 4) {  // suffix scan (row shifts + readlanes)
      v = rscan_add(v, lane) * 1e-3;
    } else if constexpr (V == 5) {  // wave_max
      v = wave_max(fabs(v)) * 0.5 + v;
    } else if constexpr (V == 6) {  // 16 dependent v_add_f64 with a DPP row_shr:1 source
#pragma unroll
      for (int j = 0; j < 16; ++j) v += dpp<kRowShr1>(v);
    } else if constexpr (V == 7) {  // LDS write + read round trip (wave-ordered)
      lds_sync();
      buf[lane] = v;
      lds_sync();
      v = buf[(lane + 1) & 63] * 0.5;
    } else if constexpr (V == 9) {  // LDS broadcast (ds_read_b128 of uniform addresses) + 40 plain fma
      lds_sync();
      buf[lane] = v;
      lds_sync();
      const double2* b2 = reinterpret_cast<const double2*>(buf);
      double a[4] = {0, 0, 0, 0};
#pragma unroll
      for (int j = 0; j < 20; ++j) {
        const double2 w = b2[j];
        a[(2 * j) % 4] = fma(w.x, r[2 * j], a[(2 * j) % 4]);
        a[(2 * j + 1) % 4] = fma(w.y, r[2 * j + 1], a[(2 * j + 1) % 4]);
      }
      v = ((a[0] + a[1]) + (a[2] + a[3])) * 1e-3;
    } else if constexpr (V == 10) {  // 40 plain fma on register operands (no broadcast): floor
      double a[4] = {0, 0, 0, 0};
#pragma unroll
      for (int j = 0; j < 40; ++j) a[j % 4] = fma(v, r[j], a[j % 4]);
      v = ((a[0] + a[1]) + (a[2] + a[3])) * 1e-3;
    } else if constexpr (V == 11 || V == 12) {  // bcast + 40 fmac_dpp, 8 (11) or 2 (12) chains
      constexpr int K = V == 11 ? 8 : 2;
      double w[4];
      bcast<3>(v, w);
      double a[8] = {0, 0, 0, 0, 0, 0, 0, 0};
      Unroll<0, 40>::run([&](auto jc) {
        constexpr int j = decltype(jc)::value;
        fmac_bc<j % 16>(a[j % K], w[j / 16], r[j]);
      });
      v = (((a[0] + a[1]) + (a[2] + a[3])) + ((a[4] + a[5]) + (a[6] + a[7]))) * 1e-3;
    } else if constexpr (V == 13) {  // bcast alone
      double w[4];
      bcast<3>(v, w);
      v = (w[0] + w[1] + w[2]) * 1e-3;
    } else if constexpr (V == 14) {  // 16 dependent wave_shr:1 DPP moves (lo + hi)
#pragma unroll
      for (int j = 0; j < 16; ++j) v = dpp<kWaveShr1>(v);
    } else if constexpr (V == 15) {  // 16 dependent select + fma (prox-like)
#pragma unroll
      for (int j = 0; j < 16; ++j) v = (v > u ? fma(v, 0.5, u) : v * 1.25);
    } else if constexpr (V == 16) {  // 16 dependent permlane32 swaps
#pragma unroll
      for (int j = 0; j < 16; ++j) {
        int lo = __double2loint(v), hi = __double2hiint(v);
        const auto a = __builtin_amdgcn_permlane32_swap(lo, lo, false, false);
        const auto b = __builtin_amdgcn_permlane32_swap(hi, hi, false, false);
        v = __hiloint2double(b[0], a[0]);
      }
    } else if constexpr (V == 17) {  // 16 dependent readlane(63) -> v_add (SGPR round trip)
#pragma unroll
      for (int j = 0; j < 16; ++j) v = readlane(v, 63) + v;
    } else if constexpr (V == 8) {  // 16 dependent shr2 (4 DPP movs each)
#pragma unroll
      for (int j = 0; j < 16; ++j) v = shr2(v) + 1.0;
    }
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  out[blockIdx.x * 64 + lane] = v + a0 + a1 + a2 + a3;
  if (lane == 0) cyc[blockIdx.x] = t1 - t0;
}

__global__ void k_spin(unsigned long long ticks, unsigned long long* out) {
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  unsigned long long t = t0;
  while (t - t0 < ticks) t = __builtin_amdgcn_s_memtime();
  if (threadIdx.x == 0) out[0] = t - t0;
}

template <int V>
void run(const char* name, double per, const double* din, double* dout, unsigned long long* dc, int waves, int grid) {
  hipLaunchKernelGGL(k<V>, dim3(grid), dim3(64), 0, 0, din, dout, dc, waves);
  hipLaunchKernelGGL(k<V>, dim3(grid), dim3(64), 0, 0, din, dout, dc, waves);
  unsigned long long c[4096];
  hipMemcpy(c, dc, sizeof(unsigned long long) * waves, hipMemcpyDeviceToHost);
  double m = 0;
  for (int i = 0; i < waves; ++i) m += (double)c[i];
  m /= waves;
  printf("%-34s waves=%4d  %8.1f cycles/op\n", name, waves, m / R / per);
}

int main() {
  double h[128];
  for (int i = 0; i < 128; ++i) h[i] = 0.5 + 1e-3 * i;
  double *din, *dout;
  unsigned long long* dc;
  hipMalloc(&din, sizeof h);
  hipMalloc(&dout, sizeof(double) * 64 * 4096);
  hipMalloc(&dc, sizeof(unsigned long long) * 4096);
  hipMemcpy(din, h, sizeof h, hipMemcpyHostToDevice);
  {  // s_memtime tick rate: spin 2e7 ticks, time with events
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    hipLaunchKernelGGL(k_spin, dim3(1), dim3(64), 0, 0, 1000000ull, dc);
    hipEventRecord(e0);
    hipLaunchKernelGGL(k_spin, dim3(1), dim3(64), 0, 0, 20000000ull, dc);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    printf("s_memtime: 2e7 ticks in %.3f ms -> %.3f GHz\n", ms, 2e7 / (ms * 1e-3) / 1e9);
  }
  for (int waves : {1, 2048, 4096}) {
    run<0>("fma f64 dependent (per fma)", 16, din, dout, dc, waves, waves);
    run<1>("fma f64 4 chains (per fma)", 16, din, dout, dc, waves, waves);
    run<2>("bcast + 40 fmac_dpp (per matvec)", 1, din, dout, dc, waves, waves);
    run<3>("scan_add (per scan)", 1, din, dout, dc, waves, waves);
    run<4>("rscan_add (per scan)", 1, din, dout, dc, waves, waves);
    run<5>("wave_max (per reduction)", 1, din, dout, dc, waves, waves);
    run<6>("add f64 + dpp row_shr (per add)", 16, din, dout, dc, waves, waves);
    run<7>("lds write+read (per round trip)", 1, din, dout, dc, waves, waves);
    run<8>("shr2 + add (per op)", 16, din, dout, dc, waves, waves);
    run<9>("lds bcast b128 + 40 fma (per matvec)", 1, din, dout, dc, waves, waves);
    run<10>("40 fma, no broadcast (per matvec)", 1, din, dout, dc, waves, waves);
    run<11>("bcast + 40 fmac_dpp 8 chains", 1, din, dout, dc, waves, waves);
    run<12>("bcast + 40 fmac_dpp 2 chains", 1, din, dout, dc, waves, waves);
    run<13>("bcast alone (+2 adds)", 1, din, dout, dc, waves, waves);
    run<14>("wave_shr1 dpp move (per move)", 16, din, dout, dc, waves, waves);
    run<15>("select + fma (per step)", 16, din, dout, dc, waves, waves);
    run<16>("permlane32 swap (per swap)", 16, din, dout, dc, waves, waves);
    run<17>("readlane + add (per step)", 16, din, dout, dc, waves, waves);
  }
  return 0;
}
