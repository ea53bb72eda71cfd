// mpcqp_common.h -- shared device primitives, layouts and the launch record of the batched
// MPC QP solver (included by mpcqp.hip and by the per-horizon solver objects).
#pragma once
#include <hip/hip_runtime.h>

#include <chrono>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <mutex>
#include <new>
#include <string>
#include <type_traits>
#include <utility>

#include "../../include/mpcqp.h"

namespace {

constexpr int kWave = 64;
constexpr double kPi = 3.141592653589793;
constexpr double kTwoPi = 6.283185307179586;
constexpr double kMinScaling = 1e-4;
constexpr double kMaxScaling = 1e4;
constexpr double kRhoMin = 1e-6;
constexpr double kRhoMax = 1e6;
constexpr double kDivTol = 1e-30;
constexpr double kRank1Min = 1e-10;  // smallest 1 + delta c'A^{-1}c accepted by a rank-1 update

// ------------------------------------------------------------------ layouts
__host__ __device__ constexpr int model_stride(int N) { return ((11 * N + 10) + 7) / 8 * 8; }

// Solver state per QP (doubles):
//   [0, n*n)            Pbar, symmetric, row-major
//   lane fields         kF* x 64 doubles, lane-contiguous
//   scalars             cscale, admm_ok, admm_it, n_fact
enum LaneField {
  kFq = 0,
  kFD,
  kFx,
  kFE0,
  kFE1,
  kFE2,
  kFlo0,
  kFlo1,
  kFlo2,
  kFhi0,
  kFhi1,
  kFhi2,
  kFw0,
  kFw1,
  kFw2,
  kNumFields
};
__host__ __device__ constexpr int state_lane_off(int N) { return (4 * N * N + 7) / 8 * 8; }
__host__ __device__ constexpr int state_scal_off(int N) { return state_lane_off(N) + kNumFields * kWave; }
__host__ __device__ constexpr int state_stride(int N) { return state_scal_off(N) + 8; }

// ------------------------------------------------------------------ wave primitives (DPP)
template <int CTRL>
__device__ __forceinline__ double dpp(double v) {
  const int lo = __builtin_amdgcn_update_dpp(0, __double2loint(v), CTRL, 0xf, 0xf, true);
  const int hi = __builtin_amdgcn_update_dpp(0, __double2hiint(v), CTRL, 0xf, 0xf, true);
  return __hiloint2double(hi, lo);
}
__device__ __forceinline__ double readlane(double v, int l) {
  return __hiloint2double(__builtin_amdgcn_readlane(__double2hiint(v), l),
                          __builtin_amdgcn_readlane(__double2loint(v), l));
}
constexpr int kRowShr1 = 0x111, kRowShr2 = 0x112, kRowShr4 = 0x114, kRowShr8 = 0x118;
constexpr int kRowShl1 = 0x101, kRowShl2 = 0x102, kRowShl4 = 0x104, kRowShl8 = 0x108;
constexpr int kWaveShr1 = 0x138, kWaveShl1 = 0x130;

// DPP with a row mask: rows outside ROWMASK read 0
template <int CTRL, int ROWMASK>
__device__ __forceinline__ double dpp_rows(double v) {
  const int lo = __builtin_amdgcn_update_dpp(0, __double2loint(v), CTRL, ROWMASK, 0xf, false);
  const int hi = __builtin_amdgcn_update_dpp(0, __double2hiint(v), CTRL, ROWMASK, 0xf, false);
  return __hiloint2double(hi, lo);
}
constexpr int kRowBcast15 = 0x142, kRowBcast31 = 0x143;  // GFX9 wave-level row broadcasts

// inclusive prefix sum over lanes 0..lane: zero-filled row shifts, then the row totals carried
// across rows by row_bcast:15 (rows 1, 3) and row_bcast:31 (rows 2, 3) -- no SGPR round trip
__device__ __forceinline__ double scan_add(double v, int lane) {
  (void)lane;
  v += dpp<kRowShr1>(v);
  v += dpp<kRowShr2>(v);
  v += dpp<kRowShr4>(v);
  v += dpp<kRowShr8>(v);
  v += dpp_rows<kRowBcast15, 0xa>(v);
  v += dpp_rows<kRowBcast31, 0xc>(v);
  return v;
}
// inclusive suffix sum over lanes lane..63
__device__ __forceinline__ double rscan_add(double v, int lane) {
  v += dpp<kRowShl1>(v);
  v += dpp<kRowShl2>(v);
  v += dpp<kRowShl4>(v);
  v += dpp<kRowShl8>(v);
  const double t1 = readlane(v, 16), t2 = readlane(v, 32), t3 = readlane(v, 48);
  const int row = lane >> 4;
  double off = row <= 2 ? t3 : 0.0;
  if (row <= 1) off += t2;
  if (row <= 0) off += t1;
  return v + off;
}
// inclusive prefix / suffix max of non-negative values
__device__ __forceinline__ double scan_max(double v, int lane) {
  v = fmax(v, dpp<kRowShr1>(v));
  v = fmax(v, dpp<kRowShr2>(v));
  v = fmax(v, dpp<kRowShr4>(v));
  v = fmax(v, dpp<kRowShr8>(v));
  const double t0 = readlane(v, 15), t1 = readlane(v, 31), t2 = readlane(v, 47);
  const int row = lane >> 4;
  double off = row >= 1 ? t0 : 0.0;
  if (row >= 2) off = fmax(off, t1);
  if (row >= 3) off = fmax(off, t2);
  return fmax(v, off);
}
__device__ __forceinline__ double rscan_max(double v, int lane) {
  v = fmax(v, dpp<kRowShl1>(v));
  v = fmax(v, dpp<kRowShl2>(v));
  v = fmax(v, dpp<kRowShl4>(v));
  v = fmax(v, dpp<kRowShl8>(v));
  const double t1 = readlane(v, 16), t2 = readlane(v, 32), t3 = readlane(v, 48);
  const int row = lane >> 4;
  double off = row <= 2 ? t3 : 0.0;
  if (row <= 1) off = fmax(off, t2);
  if (row <= 0) off = fmax(off, t1);
  return fmax(v, off);
}
// max / min without LLVM's IEEE-mode operand canonicalization (it adds a v_max_f64 x, x, x for
// every operand not known to be canonical -- DPP results, values kept opaque across solver
// iterations).  No kernel here produces signalling NaNs, and on quiet operands the instruction
// is IEEE maxNum / minNum, i.e. fmax / fmin bit for bit.
__device__ __forceinline__ double max_nc(double a, double b) {
  double r;
  asm("v_max_f64 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
  return r;
}
__device__ __forceinline__ double min_nc(double a, double b) {
  double r;
  asm("v_min_f64 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
  return r;
}
// wave-uniform sum / max: the inclusive scan's last lane
__device__ __forceinline__ double wave_sum(double v) { return readlane(scan_add(v, 0), 63); }
__device__ __forceinline__ double wave_max(double v) {  // v >= 0
  v = max_nc(v, dpp<kRowShr1>(v));
  v = max_nc(v, dpp<kRowShr2>(v));
  v = max_nc(v, dpp<kRowShr4>(v));
  v = max_nc(v, dpp<kRowShr8>(v));
  v = max_nc(v, dpp_rows<kRowBcast15, 0xa>(v));
  v = max_nc(v, dpp_rows<kRowBcast31, 0xc>(v));
  return readlane(v, 63);
}
// lane i <- lane i-2 (0 for i < 2);  lane i <- lane i+2 (0 past the wave)
__device__ __forceinline__ double shr2(double v) { return dpp<kWaveShr1>(dpp<kWaveShr1>(v)); }
__device__ __forceinline__ double shl2(double v) { return dpp<kWaveShl1>(dpp<kWaveShl1>(v)); }
__device__ __forceinline__ double shr4(double v) { return shr2(shr2(v)); }
__device__ __forceinline__ double shl4(double v) { return shl2(shl2(v)); }
__device__ __forceinline__ bool wave_any(bool b) { return __ballot(b) != 0ull; }

// ---- register broadcasts for the dense row-per-lane products (no LDS)
// A dense product over a vector v distributed one element per lane needs every lane to see
// every v_j.  bcast() replicates each 16-lane row of v into all four rows with the gfx950
// permlane swaps (w[c] lane l = v[16c + (l & 15)]); v_fmac_f64 with DPP row_newbcast:L then
// reads lane L of each row's copy as its multiplicand, so a broadcast-FMA is ONE VALU
// instruction with no memory latency.  Must run with all 64 lanes active.
template <int NW>  // rows needed: ceil(n / 16)
__device__ __forceinline__ void bcast(double v, double w[4]) {
  const int lo = __double2loint(v), hi = __double2hiint(v);
  const auto l16 = __builtin_amdgcn_permlane16_swap(lo, lo, false, false);  // rows {0,0,2,2} / {1,1,3,3}
  const auto h16 = __builtin_amdgcn_permlane16_swap(hi, hi, false, false);
  const auto la = __builtin_amdgcn_permlane32_swap(l16[0], l16[0], false, false);  // row 0 x4 / row 2 x4
  const auto ha = __builtin_amdgcn_permlane32_swap(h16[0], h16[0], false, false);
  w[0] = __hiloint2double(ha[0], la[0]);
  if constexpr (NW > 1) {
    const auto lb = __builtin_amdgcn_permlane32_swap(l16[1], l16[1], false, false);  // row 1 x4 / row 3 x4
    const auto hb = __builtin_amdgcn_permlane32_swap(h16[1], h16[1], false, false);
    w[1] = __hiloint2double(hb[0], lb[0]);
    if constexpr (NW > 3) w[3] = __hiloint2double(hb[1], lb[1]);
  }
  if constexpr (NW > 2) w[2] = __hiloint2double(ha[1], la[1]);
  // DPP reads of a VGPR need two wait states after its VALU write; tie the pad to w
  if constexpr (NW == 1) asm volatile("s_nop 1" : "+v"(w[0]));
  if constexpr (NW == 2) asm volatile("s_nop 1" : "+v"(w[0]), "+v"(w[1]));
  if constexpr (NW == 3) asm volatile("s_nop 1" : "+v"(w[0]), "+v"(w[1]), "+v"(w[2]));
  if constexpr (NW == 4) asm volatile("s_nop 1" : "+v"(w[0]), "+v"(w[1]), "+v"(w[2]), "+v"(w[3]));
}
// The same for a vector that lives in the lanes of rows 0-1 of each half (n <= 32 in the whole-wave
// layout, n <= 30 in a half): one permlane16 swap per word puts row 0 / row 1 of each half into both
// of its rows (w[0] / w[1]); with n <= 16 (NW = 1) row 0 is already where its lanes read it, and no
// lane moves at all (whole-wave layout only).  The lanes of the other rows read their own rows'
// values there: padding, which the callers keep finite (exact zeros).
template <int NW>
__device__ __forceinline__ void bcast_rows01(double v, double w[4]) {
  static_assert(NW <= 2, "two 16-lane rows");
  if constexpr (NW == 1) {
    w[0] = v;
    asm volatile("s_nop 1" : "+v"(w[0]));
  } else {
    const int lo = __double2loint(v), hi = __double2hiint(v);
    const auto l16 = __builtin_amdgcn_permlane16_swap(lo, lo, false, false);  // rows {0,0,2,2} / {1,1,3,3}
    const auto h16 = __builtin_amdgcn_permlane16_swap(hi, hi, false, false);
    w[0] = __hiloint2double(h16[0], l16[0]);
    w[1] = __hiloint2double(h16[1], l16[1]);
    // DPP reads of a VGPR need two wait states after its VALU write; tie the pad to w
    asm volatile("s_nop 1" : "+v"(w[0]), "+v"(w[1]));
  }
}
// acc += w[lane 16*row + L] * m   (one v_fmac_f64_dpp)
template <int L>
__device__ __forceinline__ void fmac_bc(double& acc, double w, double m) {
  asm("v_fmac_f64_dpp %0, %1, %2 row_newbcast:%3 row_mask:0xf bank_mask:0xf" : "+v"(acc) : "v"(w), "v"(m), "i"(L));
}
// ---- lane policies of the one-wave solver: a QP owns the whole wave (Lanes<false>, the layout
// above) or one 32-lane half of it (Lanes<true>: two QPs per wave, lanes 0-31 and 32-63, for
// n = 2N <= 30, where a whole-wave QP leaves lanes 30..63 computing on padding).  Every cross-lane
// operation of a half stays inside it: 16-lane-row DPP, permlane16 swaps (rows 0<->1, 2<->3),
// row_bcast:15 into rows 1 / 3, ds_bpermute within 32 lanes -- so the two QPs of a wave may take
// different branches (the other half is masked off), and a half's sums and scans add the same
// values in the same order as the whole-wave ones (lanes past n hold zeros in both layouts).
template <bool Pair>
struct Lanes;

template <>
struct Lanes<false> {
  static constexpr int kLanes = kWave;
  template <int NW>
  __device__ __forceinline__ static void vbcast(double v, double w[4]) {
    if constexpr (NW <= 2)
      bcast_rows01<NW>(v, w);  // rows 2-3 are padding: no permlane32 stage
    else
      bcast<NW>(v, w);
  }
  template <int K>
  __device__ __forceinline__ static double read(double v) { return readlane(v, K); }
  __device__ __forceinline__ static double readv(double v, int l) { return readlane(v, l); }
  __device__ __forceinline__ static int uniform(int l) { return __builtin_amdgcn_readfirstlane(l); }
  __device__ __forceinline__ static double sum(double v) { return wave_sum(v); }
  __device__ __forceinline__ static double max(double v) { return wave_max(v); }
  __device__ __forceinline__ static bool any(bool b) { return wave_any(b); }
  __device__ __forceinline__ static uint64_t ballot(bool b) { return __ballot(b); }
  __device__ __forceinline__ static double shr2(double v) { return ::shr2(v); }
  __device__ __forceinline__ static double shl2(double v) { return ::shl2(v); }
  __device__ __forceinline__ static double shr4(double v) { return ::shr4(v); }
  __device__ __forceinline__ static double shl4(double v) { return ::shl4(v); }
  __device__ __forceinline__ static double shr1(double v) { return dpp<kWaveShr1>(v); }  // lane 0 <- 0
  __device__ __forceinline__ static double shl1(double v) { return dpp<kWaveShl1>(v); }  // lane 63 <- 0
  __device__ __forceinline__ static double scan(double v, int lane) { return scan_add(v, lane); }
  __device__ __forceinline__ static double shfl(double v, int src) { return __shfl(v, src, kWave); }
};

// lane L of each 16-lane row, to the whole row (one v_mov_b32_dpp row_newbcast per word)
template <int L>
__device__ __forceinline__ double row_bc(double v) {
  const int lo = __builtin_amdgcn_update_dpp(0, __double2loint(v), 0x150 + L, 0xf, 0xf, false);
  const int hi = __builtin_amdgcn_update_dpp(0, __double2hiint(v), 0x150 + L, 0xf, 0xf, false);
  return __hiloint2double(hi, lo);
}

// Every result that crosses lanes is pinned (an empty asm volatile) where it is computed: the
// compiler turns a lane-dependent select of a DPP result (the half-boundary cuts below) into a
// branch and sinks the DPP into it, where its source lanes are masked off and read as 0.
template <>
struct Lanes<true> {
  static constexpr int kLanes = 32;
  __device__ __forceinline__ static int hl() { return (int)threadIdx.x & 31; }  // lane within the half
  __device__ __forceinline__ static double pin(double v) {
    asm volatile("" : "+v"(v));
    return v;
  }
  // w[c] lane l = v[16c + (l & 15)] of l's own half (c = 0, 1): one permlane16 swap per word, also
  // at NW = 1 (the sweep reads its pivot from w in every lane of the half)
  template <int NW>
  __device__ __forceinline__ static void vbcast(double v, double w[4]) {
    static_assert(NW <= 2, "a half holds 32 lanes");
    bcast_rows01<2>(v, w);
  }
  template <int K>
  __device__ __forceinline__ static double read(double v) {
    double w[4];
    bcast_rows01<2>(v, w);
    return pin(row_bc<K % 16>(w[K / 16]));
  }
  __device__ __forceinline__ static double readv(double v, int l) { return pin(__shfl(v, l, 32)); }
  __device__ __forceinline__ static int uniform(int l) { return l; }
  // inclusive scan within the rows, then rows 1 / 3 take rows 0 / 2's total: lane 31 / 63 = the sum
  __device__ __forceinline__ static double scan(double v, int lane) {
    (void)lane;
    v += dpp<kRowShr1>(v);
    v += dpp<kRowShr2>(v);
    v += dpp<kRowShr4>(v);
    v += dpp<kRowShr8>(v);
    v += dpp_rows<kRowBcast15, 0xa>(v);
    return pin(v);
  }
  __device__ __forceinline__ static double sum(double v) { return read<31>(scan(v, 0)); }
  __device__ __forceinline__ static double max(double v) {  // v >= 0
    v = max_nc(v, dpp<kRowShr1>(v));
    v = max_nc(v, dpp<kRowShr2>(v));
    v = max_nc(v, dpp<kRowShr4>(v));
    v = max_nc(v, dpp<kRowShr8>(v));
    v = max_nc(v, dpp_rows<kRowBcast15, 0xa>(v));
    return read<31>(v);
  }
  __device__ __forceinline__ static uint64_t ballot(bool b) {
    const uint64_t m = __ballot(b);
    return (threadIdx.x & 32) ? (m >> 32) : (m & 0xffffffffull);
  }
  __device__ __forceinline__ static bool any(bool b) { return ballot(b) != 0ull; }
  // wave shifts, cut at the half boundary (what crosses it reads as 0, as past the wave's ends)
  __device__ __forceinline__ static double shr2(double v) {
    const double d = pin(::shr2(v));
    return hl() >= 2 ? d : 0.0;
  }
  __device__ __forceinline__ static double shl2(double v) {
    const double d = pin(::shl2(v));
    return hl() < 30 ? d : 0.0;
  }
  __device__ __forceinline__ static double shr4(double v) { return shr2(shr2(v)); }
  __device__ __forceinline__ static double shl4(double v) { return shl2(shl2(v)); }
  __device__ __forceinline__ static double shr1(double v) {
    const double d = pin(dpp<kWaveShr1>(v));
    return hl() >= 1 ? d : 0.0;
  }
  __device__ __forceinline__ static double shl1(double v) {
    const double d = pin(dpp<kWaveShl1>(v));
    return hl() < 31 ? d : 0.0;
  }
  __device__ __forceinline__ static double shfl(double v, int src) { return pin(__shfl(v, src, 32)); }
};

// compile-time loop: f(std::integral_constant<int, I>) for I in [B, E)
template <int B, int E>
struct Unroll {
  template <class F>
  __device__ __forceinline__ static void run(F&& f) {
    if constexpr (B < E) {
      f(std::integral_constant<int, B>{});
      Unroll<B + 1, E>::run(f);
    }
  }
};

// Every kernel runs one wavefront per workgroup, and the LDS operations of one wavefront
// execute in program order: a broadcast through LDS needs only a compiler-level ordering
// point (wavefront-scope fence), not an s_barrier with its lgkmcnt(0) drain.
__device__ __forceinline__ void lds_sync() { __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront"); }

// ------------------------------------------------------------------ phase marks
// Built only with -DMPCQP_PHASE_MARKS for static analysis of the device assembly (never in the measured
// library): an assembly comment where a solver phase begins, so tools/isa_breakdown.py can attribute
// every instruction of k_solve<N> to the phase it executes in and weight it by the phase's count.
#ifdef MPCQP_PHASE_MARKS
#define MPCQP_MARK(name) asm volatile(";@phase " name)
#else
#define MPCQP_MARK(name)
#endif

// ------------------------------------------------------------------ diagnostic stamps
// Built only with -DMPCQP_STAMPS (never in the measured library): per-phase s_memtime
// cycle sums, flushed once per wave into g_stamps[] (read by mpcqp_debug_stamps).
#ifdef MPCQP_STAMPS
__device__ unsigned long long g_stamps[32];
struct Stamps {
  unsigned long long acc[6] = {0, 0, 0, 0, 0, 0};
  unsigned long long t = 0;
  __device__ __forceinline__ void begin() {
    __builtin_amdgcn_sched_barrier(0);
    t = __builtin_amdgcn_s_memtime();
    __builtin_amdgcn_sched_barrier(0);
  }
  __device__ __forceinline__ void end(int s) {
    __builtin_amdgcn_sched_barrier(0);
    acc[s] += __builtin_amdgcn_s_memtime() - t;
    __builtin_amdgcn_sched_barrier(0);
  }
  __device__ __forceinline__ void flush(int base) {
    if (threadIdx.x == 0)
      for (int s = 0; s < 6; ++s) atomicAdd(&g_stamps[base + s], acc[s]);
  }
};
#else
struct Stamps {
  __device__ __forceinline__ void begin() {}
  __device__ __forceinline__ void end(int) {}
  __device__ __forceinline__ void flush(int) {}
};
#endif

__device__ __forceinline__ double limit_scaling(double v) {
  return v < kMinScaling ? 1.0 : (v > kMaxScaling ? kMaxScaling : v);
}

// numpy float mod (npy_divmod) for b > 0
__device__ __forceinline__ double np_mod(double a, double b) {
  double m = fmod(a, b);
  if (m != 0.0) {
    if (m < 0.0) m += b;
  } else {
    m = 0.0;
  }
  return m;
}

}  // namespace

namespace mpcqp {
// One solve launch (device pointers; outputs may be null).
struct Launch {
  const mpcqp_params* p;
  int B;
  const double* model;
  double* state;
  double *u0, *X, *U;
  int32_t *st, *it;
  uint8_t* ac;
  const uint8_t* mask;  // QP b is solved iff mask == nullptr or mask[b] != 0 (fleet steps)
  // K1 fused into the solve: with ref != nullptr the kernel builds each QP's LTV model from the
  // caller's inputs itself (one-wave kernel); otherwise it reads `model` (K1 / fleet output)
  const double* x0 = nullptr;
  const double* ref = nullptr;
  const double* u_prev = nullptr;
};

typedef void (*launcher_t)(hipStream_t, const Launch&);
// two QPs per wave (k_solve_pair, N <= 15, fused K1); returns false where not instantiated
typedef bool (*pair_launcher_t)(hipStream_t, const Launch&);
template <int N>
bool launch_solve_pair(hipStream_t s, const Launch& L);
// K2a -> K2b -> K2c for horizon N; defined in mpcqp_solve.h, instantiated per horizon in
// mpcqp_part.hip objects (parallel build) or in mpcqp.hip itself (MPCQP_ONLY_N dev builds).
template <int N>
void launch_solve(hipStream_t s, const Launch& L);
// the fused closed loop of a fleet (k_fleet_loop<N>, mpcqp_solve.h; N <= 32, fast mode): `steps`
// loop steps of every RUNNING vehicle in one launch
// The config-5 replan trigger inside the fused loop (mpcqp_swarm_loop): after each step a RUNNING
// vehicle farther than replan_distance from ref[path_idx], or an ABORTED one, with replans left leaves
// the loop as MPCQP_FLEET_REPLAN_* with its replanning problem in start_goal.  max_replans = 0: off.
struct LoopTrigger {
  double replan_distance;
  int max_replans;
  const int32_t* replans;
  double* start_goal;
  // workgroup -> vehicle (nullptr: identity).  The fused loops dispatch the vehicles longest
  // reference first: a vehicle's step count follows its reference length, and the slowest
  // vehicles started last would set the run's tail once the vehicles outnumber the wave slots.
  const int32_t* order = nullptr;
  bool pair = false;  // two vehicles per wave (N <= 15): k_fleet_loop<N, true>
};
template <int N>
void launch_fleet_loop(hipStream_t s, const mpcqp_params* P, const mpcqp_fleet& f, int steps, const LoopTrigger& tr);
// The B = 1 server (mpcqp_solve_served): one resident wave that solves the QP of the workspace's
// staging block each time the host raises `req`, then publishes `done`.  In pinned, mapped,
// coherent host memory; req and done on separate 64-byte lines.
struct ServeBox {
  uint32_t req;
  uint32_t pad0[15];
  uint32_t done;
  uint32_t pad1[15];
};
constexpr uint32_t kServeStop = 0xffffffffu;  // req value that ends the server
struct ServeLaunch {
  ServeBox* box;      // device address of the mailbox
  const double* in;   // device address of the staging input block (x0 | ref | u_prev)
  uint8_t* out;       // device address of the staging output block
  int32_t off[6];     // output block offsets (u0, X, U, status, iters, active)
  uint64_t idle_ticks;  // s_memrealtime ticks (100 MHz) without a request after which the wave exits
};
template <int N>
void launch_serve(hipStream_t s, const mpcqp_params& p, const ServeLaunch& L);
typedef void (*serve_t)(hipStream_t, const mpcqp_params&, const ServeLaunch&);
// nullptr when the parameter block does not run the one-wave kernel; defined in mpcqp.hip
serve_t server(const mpcqp_params& p);
typedef void (*fleet_loop_t)(hipStream_t, const mpcqp_params*, const mpcqp_fleet&, int, const LoopTrigger&);
// nullptr when the parameter block does not run the one-wave kernel; defined in mpcqp.hip
fleet_loop_t fleet_looper(const mpcqp_params& p);
// k_solve_pair / k_fleet_loop<N, true> for `count` QPs or vehicles of this workspace's launch?
bool use_pairs(const mpcqp_ws* ws, int count);
// the long-horizon solve (N >= MPCQP_WIDE_MIN_HORIZON; mpcqp_wide.hip): one 256-thread workgroup
// per QP, L.state = its workspace (wide_stride(N) doubles per QP)
void launch_solve_wide(hipStream_t s, const Launch& L);
size_t wide_stride(int horizon);
// the mid-horizon fast solve (MPCQP_WIDE_MIN_HORIZON <= N <= MPCQP_MID_MAX_HORIZON, mpcqp_mid.hip):
// one workgroup of 4 x (1 or 2) waves per QP, instantiated per padded horizon bucket NT; L.state = its
// workspace (mid_stride(N) doubles per QP: the scaled Hessian)
template <int NT>
void launch_solve_mid(hipStream_t s, const Launch& L);
inline int mid_bucket(int N) { return N <= 40 ? 40 : (N <= 48 ? 48 : (N <= 56 ? 56 : 64)); }  // N >= 33
inline size_t mid_stride(int N) { return (size_t)2 * mid_bucket(N) * 128; }
// the solve of this parameter block runs a workgroup-per-QP kernel (long horizon or reproducible)
bool wide_solve(const mpcqp_params& p);
// launcher of the parameter block's horizon / kernel (nullptr when not compiled in); defined in mpcqp.hip
launcher_t launcher(const mpcqp_params& p);
// records msg as mpcqp_last_error() of the calling thread and returns code; defined in mpcqp.hip
int fail(int code, const std::string& msg);
}  // namespace mpcqp

// Workspace of one device: parameter block + per-QP model (K1 output) and solver state.
struct mpcqp_ws {
  mpcqp_params p;
  int max_batch;
  int device;
  int built_B;
  // per-QP model (K1 output) and solver state, allocated by ensure_buffers at the first call that
  // needs them: the fused one-wave solve builds the model on chip and keeps the scaled problem
  // there, so a workspace that only runs it holds neither (22 KB per QP at N = 20)
  double* model;
  double* state;
  // the inputs of the last mpcqp_build when the model is built inside the solve (fused K1)
  const double* in_x0;
  const double* in_ref;
  const double* in_up;
  // device copies of the parameter blocks of the last mpcqp_fleet_loop (nominal, relaxed): the fused
  // loop selects its block per solve, which a kernel argument cannot be (the compiler copies a
  // run-time-selected argument block to scratch); written by a kernel on the launch stream
  mpcqp_params* dparams;
  // the fused loop's dispatch order (max_batch vehicles), written by k_fleet_order on the stream
  int32_t* dorder;
  // the B = 1 path (mpcqp_stage / mpcqp_solve_staged): mapped host blocks and a private stream
  double* stage_in;      // host address (x0 | ref | u_prev)
  double* stage_in_d;    // its device address
  uint8_t* stage_out;    // host address (u0 | X | U | status | iters | active)
  uint8_t* stage_out_d;  // its device address
  hipStream_t stage_stream;
  // the B = 1 server: mailbox (host / device address), sequence number, a server kernel enqueued
  void* serve_box;
  void* serve_box_d;
  uint32_t serve_seq;
  bool serve_live;
  bool serve_broken;  // a request went unanswered (30 s): the workspace refuses B = 1 requests
  int serve_fault;    // mpcqp_debug_serve_fault: 1 = refuse the next server launch
  std::chrono::steady_clock::time_point serve_last;  // the last completed request (host clock)
  // guards the server fields above: held by mpcqp_solve_served for its whole call, by set_params /
  // destroy around their stop, and try-locked by another workspace's served call that would stop this
  // workspace's wave (it skips the stop while this one is busy)
  std::mutex serve_mu;
  // two QPs per wave for N <= 15 (MPCQP_PAIR_*, mpcqp_set_pairing)
  int pairing;
  int cus;  // the device's compute units (queried once at mpcqp_create; 0 if unknown)
};

namespace mpcqp {
// the fused fleet loop (mpcqp_fleet.hip), with the swarm's trigger when tr.max_replans > 0; *fused =
// false (nothing enqueued) when the parameter blocks do not run the one-wave kernel
int enqueue_fleet_loop(mpcqp_ws* nominal, mpcqp_ws* relaxed, const mpcqp_fleet* f, int steps, const LoopTrigger& tr,
                       hipStream_t s, bool* fused);
// allocate ws->model / ws->state (max_batch QPs) if requested and not yet there; refuses to allocate
// on a capturing stream (the first use must run outside a capture); defined in mpcqp.hip
int ensure_buffers(mpcqp_ws* ws, bool model, bool state, hipStream_t s);
// the solver-state buffer is read or written: the long-horizon kernels' workspace, debug state
inline bool needs_state(const mpcqp_params& p) { return wide_solve(p) || p.debug_state != 0; }
// the stepped fleet's buffers (k_fleet_build writes the models; mpcqp_fleet.hip), before a capture
int fleet_buffers(mpcqp_ws* nominal, mpcqp_ws* relaxed, hipStream_t s);
}  // namespace mpcqp
