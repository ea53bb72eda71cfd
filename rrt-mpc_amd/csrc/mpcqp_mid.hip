// mpcqp_mid.hip -- the fast solve for mid horizons, MPCQP_WIDE_MIN_HORIZON <= N <= MPCQP_MID_MAX_HORIZON.
//
// The one-wave kernel (mpcqp_solve.h) keeps a QP's KKT inverse one row per lane, which caps it at
// 2N <= 62 variables.  Here a QP owns one workgroup of P x R waves (R = 1 or 2 "row waves"): row i
// of the KKT inverse (i = 64 wp + lane, padded to NP = 2 NT rows) is split into P = 2 or 4 column parts
// h of CW = NP / P doubles each, held in the registers of waves (h, wp).  The h = 0 waves also own
// the QP's per-variable data (one decision variable per row, as in the one-wave kernel: the speed
// form W = (v_1, delta_0, v_2, ...), the banded soft rows, OSQP's scaling).  Dense products read
// their operand from LDS (broadcast reads) and add the parts' partial sums through LDS; the
// sweep publishes one pivot column per step through LDS (one barrier per pivot); neighbour shifts
// of the banded operators and the wave reductions cross the row waves through LDS.  The scaled
// Hessian Pbar lives in the QP's workspace slot (L2 / MALL resident; read for a factorization and
// for P x), column-interleaved so every read is one coalesced row of lanes.
//
// The algorithm is the one-wave kernel's (setup: condensing + OSQP Ruiz / cost scaling; ADMM with
// OSQP's rho / sigma / alpha / adaptive rho / termination; early polish attempts; the active-set
// polish with rank-1 inverse updates and the exact line search; OSQP's statuses), in the same
// order of operations except where a sum spans the parts or the two row waves (tree order).
// Template NT: the padded horizon; runtime N <= NT (variables past 2N are exact zeros and their
// pivots are skipped).  K1 runs as its own kernel (k_build) into the workspace model block.
#include "mpcqp_build.h"

namespace {
using mpcqp::Launch;

constexpr int kMidLD = 128;  // row stride (doubles) of the workspace Pbar
// Diagnostic builds only (-DMPCQP_MID_STAMPS, never the measured library): per-phase s_memtime sums of
// each QP's thread 0, added into g_mid_stamps[] at the end (read by mpcqp_debug_mid_stamps_<NT>).
#ifdef MPCQP_MID_STAMPS
constexpr int kMidStampSlots = 24;
__device__ unsigned long long g_mid_stamps[kMidStampSlots];
struct MidStamps {
  // 0..7 the phases, 9..14 the setup's sub-phases and 16..20 the polish's (mark()); [8] counts the QPs
  unsigned long long acc[kMidStampSlots] = {};
  unsigned long long t = 0, t2 = 0;
  __device__ __forceinline__ void begin() { t = t2 = __builtin_amdgcn_s_memtime(); }
  __device__ __forceinline__ void end(int k) { acc[k] += __builtin_amdgcn_s_memtime() - t; }
  __device__ __forceinline__ void mbegin() { t2 = __builtin_amdgcn_s_memtime(); }
  __device__ __forceinline__ void mark(int k) {
    const unsigned long long now = __builtin_amdgcn_s_memtime();
    acc[k] += now - t2;
    t2 = now;
  }
  __device__ __forceinline__ void flush() {
    if (threadIdx.x == 0) {
      for (int k = 0; k < kMidStampSlots; ++k)
        if (k != 8) atomicAdd(&g_mid_stamps[k], acc[k]);
      atomicAdd(&g_mid_stamps[8], 1ull);
    }
  }
};
#else
struct MidStamps {
  __device__ __forceinline__ void begin() {}
  __device__ __forceinline__ void end(int) {}
  __device__ __forceinline__ void mbegin() {}
  __device__ __forceinline__ void mark(int) {}
  __device__ __forceinline__ void flush() {}
};
#endif
constexpr int kMidWaves = 2;  // waves per SIMD the register allocation targets

// The workgroup barrier of this kernel, LDS-only: every cross-wave exchange goes through LDS, and the
// workspace entries a thread reads (its row of Pbar) are its own, ordered by the hardware, so a barrier
// need not wait for the outstanding global stores (the Pbar store of the setup, the band's
// read-modify-write in form()) as __syncthreads() would.
__device__ __forceinline__ void mid_barrier() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
}

// f(c, ld(c)) for c in [0, NT), the loads issued one group of G ahead of their uses and no further
// (a scheduling barrier per group): the operand column never occupies more than 2 G registers next to
// the NT doubles of the row (hoisting every load ahead of the FMAs spills the row).
template <int NT, int G = 4, class Ld, class F>
__device__ __forceinline__ void piped(Ld&& ld, F&& f) {
  using T = decltype(ld(std::integral_constant<int, 0>{}));
  T cur[G], nxt[G];
  Unroll<0, G>::run([&](auto kc) {
    constexpr int k = decltype(kc)::value;
    if constexpr (k < NT) cur[k] = ld(std::integral_constant<int, k>{});
  });
  Unroll<0, (NT + G - 1) / G>::run([&](auto gc) {
    constexpr int g = decltype(gc)::value;
    if constexpr ((g + 1) * G < NT) {
      Unroll<0, G>::run([&](auto kc) {
        constexpr int c = (g + 1) * G + decltype(kc)::value;
        if constexpr (c < NT) nxt[decltype(kc)::value] = ld(std::integral_constant<int, c>{});
      });
    }
    __builtin_amdgcn_sched_barrier(0);
    Unroll<0, G>::run([&](auto kc) {
      constexpr int c = g * G + decltype(kc)::value;
      if constexpr (c < NT) f(std::integral_constant<int, c>{}, cur[decltype(kc)::value]);
    });
    Unroll<0, G>::run([&](auto kc) { cur[decltype(kc)::value] = nxt[decltype(kc)::value]; });
  });
}

struct Rq {  // one step's loads of the prefix / free-response recurrence (mid_setup)
  double a, c, r;
};

template <int NT>
struct MidShape {
  static constexpr int NP = 2 * NT;                          // padded decision variables
  static constexpr int kRW = (NP + kWave - 1) / kWave;       // row waves (1 or 2)
  static constexpr int kNX = kRW * kWave;                    // rows covered
  // column parts of a row: 2 up to NT = 48 (the row part fits the registers of 2 waves per SIMD next to
  // the rest, and a workgroup of 2 or 4 waves leaves room for two per CU), 4 beyond
  static constexpr int kParts = NT <= 48 ? 2 : 4;
  static constexpr int CW = NP / kParts;                     // columns per part (even)
  static constexpr int kWaves = kParts * kRW;
  static constexpr int kThreads = kWaves * kWave;
  static_assert(NP % (2 * kParts) == 0, "parts of an even width");
};

template <int NT>
struct MidLds {
  using S = MidShape<NT>;
  static constexpr int X = S::kNX;
  double vb[X];                 // dense product operand
  double pp[S::kParts - 1][X];  // dense product partial sums of the parts h >= 1
  double cbb[2][X][2];          // sweep: the pivot pair's two columns per row (double buffered; Mid::sweep)
  double ex[2][5][X + 8];       // neighbour exchange: row i at [i + 4]; 4 zeros either side
  double vec[X];                // per-row broadcast (Ruiz scalings, rank-1 vector; ADMM step: C' tmp's own terms)
  double abx[2][X + 4];         // ADMM step: the terms of C' tmp for the variables 2 / 4 back (4 zeros past X)
  double qq[X];                 // ADMM step: q per row
  double tr[S::kParts][3][X];   // rank-1 terms per part
  double band[5][X];            // form(): band entries (i, i - 4 .. i + 4) per row
  double cf[6][X];              // Cbar coefficients per variable (rank-1 rows)
  double dw[3][X];              // polish: soft-row weight changes since the last factorization
  double blo[3][X], bhi[3][X], bwb[3][X], bE[3][X];  // per variable: scaled soft-row bounds, weights,
                                                     // row scalings (LDS, not registers: see Mid)
  double red[2][8][8];          // cross-wave reductions (two slots, up to 8 values, 8 waves)
  unsigned long long msk[2][3][2];  // changed-row ballots of the row waves (two slots)
  double model[model_stride(NT)];
  double pre[4][NT + 1];
  double err[4][NT + 1];
  double g[S::kNX + 2];
  double W[S::kNX + 2];
};

template <int NT>
struct Mid {
  using S = MidShape<NT>;
  static constexpr int NP = S::NP;
  static constexpr int CW = S::CW;
  static constexpr int kP = S::kParts;
  static constexpr int kNW = S::kWaves;
  MidLds<NT>* sm;
  double* Pg;  // Pbar of this QP: Pg[j * kMidLD + i] = Pbar[i][j]
  int lane, w, h, i, N, n;
  bool V, act, even;
  int xs, rs;  // exchange / reduction slot toggles (uniform)
  double dt, D, qv, cscale;
  // the soft rows' bounds / weights / row scalings live in LDS (read per use through the opaque row
  // index, so they are not hoisted into registers): 24 VGPRs the register budget needs elsewhere
  __device__ __forceinline__ double LO(int k) const { return sm->blo[k][i]; }
  __device__ __forceinline__ double HI(int k) const { return sm->bhi[k][i]; }
  __device__ __forceinline__ double WB(int k) const { return sm->bwb[k][i]; }
  __device__ __forceinline__ double EE(int k) const { return sm->bE[k][i]; }
  double c0, c10, c11, c20, c21, c22;
  double r[CW];  // KKT (inverse) row i, columns [h CW, h CW + CW): A^{-1}[i][j] = -r
  int n_full, n_r1;
  MidStamps T;  // phases: 0 setup, 1 ADMM factorizations, 2 ADMM iterations, 3 termination checks,
                // 4 polish factorizations / rank-1 updates, 5 polish rest, 6 outputs, 7 whole QP

  __device__ __forceinline__ static void sync() { mid_barrier(); }

  // The CW values v[h CW + c] (c < CW) of an LDS vector, in every lane for the fmac_bc products: lane
  // l loads element h CW + l (one conflict-free per-lane read) and the permlane broadcast (bcast,
  // mpcqp_common.h) replicates each 16-lane row into all four, so a dense product reads its operand
  // through DPP row_newbcast.  A broadcast LDS read per column instead (the same address in every lane,
  // 512 B out of the LDS per read) kept the LDS output port busy: 8 waves per CU x CW reads per product
  // or pivot is ~1.3k cycles at N = 40, the measured cost of a sweep step and of an ADMM iteration's
  // product (round 5: 1.5k / 2.25k cycles).  Every lane of the wave must call this.
  static constexpr int kNWc = (CW + 15) / 16;
  __device__ __forceinline__ void lbcast(const double* v, double w[4]) const {
    const double x = lane < CW ? v[h * CW + lane] : 0.0;
    bcast<kNWc>(x, w);
  }

  // opaque per-lane data at the top of solver iterations (keeps LICM from hoisting derived values)
  __device__ __forceinline__ void opaque() {
    asm volatile("" : "+v"(i));
    asm volatile("" : "+v"(D), "+v"(qv));
    asm volatile("" : "+v"(c0), "+v"(c10), "+v"(c11), "+v"(c20), "+v"(c21), "+v"(c22));
  }

  // ---- cross-row-wave primitives (every thread of the workgroup calls them: they synchronize)
  // neighbours of Q per-row values v[q] (rows >= n must pass 0): v at rows i - 2, i - 4, i + 2, i + 4
  // (0 outside [0, NP)); h = 1 threads get zeros
  template <int Q>
  __device__ __forceinline__ void xchg(const double* v, double* m2, double* m4, double* p2, double* p4) {
    double(*e)[S::kNX + 8] = sm->ex[xs];
    xs = __builtin_amdgcn_readfirstlane(xs ^ 1);
    if (V)
#pragma unroll
      for (int q = 0; q < Q; ++q) e[q][i + 4] = v[q];
    sync();
#pragma unroll
    for (int q = 0; q < Q; ++q) {
      if (m2) m2[q] = V ? e[q][i + 2] : 0.0;
      if (m4) m4[q] = V ? e[q][i] : 0.0;
      if (p2) p2[q] = V ? e[q][i + 6] : 0.0;
      if (p4) p4[q] = V ? e[q][i + 8] : 0.0;
    }
  }
  // K values reduced over the whole workgroup (sum or max >= 0), identical bits in every thread:
  // per wave in DPP tree order, then the waves in index order
  template <int K, bool MAX>
  __device__ __forceinline__ void reduce(double* v) {
    double(*rd)[8] = sm->red[rs];
    rs = __builtin_amdgcn_readfirstlane(rs ^ 1);
#pragma unroll
    for (int k = 0; k < K; ++k) {
      const double t = MAX ? wave_max(v[k]) : wave_sum(v[k]);
      if (lane == 0) rd[k][w] = t;
    }
    sync();
#pragma unroll
    for (int k = 0; k < K; ++k) {
      double s = rd[k][0];
#pragma unroll
      for (int q = 1; q < kNW; ++q) s = MAX ? max_nc(s, rd[k][q]) : s + rd[k][q];
      v[k] = s;
    }
  }
  __device__ __forceinline__ double bsum(double v) {
    reduce<1, false>(&v);
    return v;
  }
  __device__ __forceinline__ double bmax(double v) {
    reduce<1, true>(&v);
    return v;
  }
  __device__ __forceinline__ bool bany(bool b) { return bmax(wave_any(b) ? 1.0 : 0.0) > 0.0; }

  // z = Cbar x (V threads; x = 0 on rows >= n)
  __device__ __forceinline__ void Cmul(double x, double z[3]) {
    double xm2, xm4;
    xchg<1>(&x, &xm2, &xm4, nullptr, nullptr);
    z[0] = c0 * x;
    z[1] = c10 * x + c11 * xm2;
    z[2] = (c20 * x + c21 * xm2) + c22 * xm4;
  }
  // ... and the soft rows' bounds, loaded ahead of the exchange's barrier (their round trip hides there)
  __device__ __forceinline__ void Cmul(double x, double z[3], double lo_[3], double hi_[3]) {
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      lo_[k] = V ? LO(k) : 0.0;
      hi_[k] = V ? HI(k) : 0.0;
    }
    Cmul(x, z);
  }
  // x = Cbar' y: own rows' terms, the terms for the variable 2 back (a) and 4 back (b) of rows 2 / 4
  // ahead -- t + (a[i + 2] + b[i + 4]), the one-wave kernel's shl2(a + shl2(b))
  __device__ __forceinline__ double CTmul(const double y[3]) {
    double ab[2] = {c11 * y[1] + c21 * y[2], c22 * y[2]};
    const double t = (c0 * y[0] + c10 * y[1]) + c20 * y[2];
    double p2[2], p4[2];
    xchg<2>(ab, nullptr, nullptr, p2, p4);
    return t + (p2[0] + p4[1]);
  }

  // s = sum_c r[c] vb[h CW + c] over the parts: (K-part) v on V threads
  __device__ __forceinline__ double kmul(double v) {
    if (V) sm->vb[i] = act ? v : 0.0;
    sync();
    double w[4];
    lbcast(sm->vb, w);
    double a[4] = {0.0, 0.0, 0.0, 0.0};
    Unroll<0, CW>::run([&](auto cc) {
      constexpr int c = decltype(cc)::value;
      fmac_bc<c % 16>(a[c % 4], w[c / 16], r[c]);  // fma(vb[h CW + c], r[c], a): the same bits as fma(r, vb, a)
    });
    return combine((a[0] + a[1]) + (a[2] + a[3]));
  }
  // the parts' partial sums of row i added on the V thread: s0 + s1, or (s0 + s1) + (s2 + s3)
  __device__ __forceinline__ double combine(double s) {
    if (!V) sm->pp[h - 1][i] = s;
    sync();
    if (V) {
      if constexpr (kP == 2)
        s = s + sm->pp[0][i];
      else
        s = (s + sm->pp[0][i]) + (sm->pp[1][i] + sm->pp[2][i]);
    }
    return V && act ? s : 0.0;
  }
  __device__ __forceinline__ double inv_mul(double v) { return -kmul(v); }

  // The linear part of an ADMM iteration with two barriers instead of four, bit for bit the operations
  // of rhs = CTmul(tmp) + sg x - qv, xa = alpha inv_mul(rhs), Cmul(xa) (which cross the parts and row
  // waves through an exchange, the operand and the partial sums: one barrier each):
  //   1. each row's own terms of C' tmp and its x go to LDS;
  //   2. lane l assembles rhs of its part's column h CW + l from them (the terms 2 and 4 rows ahead
  //      read directly), broadcasts it by DPP into the product, and every part's partial sum goes to LDS;
  //   3. the V threads add the parts' sums of their row AND of the rows 2 and 4 back (the same sums in
  //      the same order as the owners'), which is all Cbar xa needs.
  // xa and za (= Cbar xa) on V threads.
  // The soft rows' bounds are loaded just before the second barrier (for the projection after it): their LDS
  // round trip hides in the barrier's wait, where few registers are live.
  __device__ __forceinline__ void admm_linear(const double tmp[3], double sg, double x, double alpha, double& xa,
                                              double za[3], double lo_[3], double hi_[3]) {
    if (V) {
      sm->abx[0][i] = c11 * tmp[1] + c21 * tmp[2];  // to the variable 2 back
      sm->abx[1][i] = c22 * tmp[2];                 // to the variable 4 back
      sm->vec[i] = (c0 * tmp[0] + c10 * tmp[1]) + c20 * tmp[2];
      sm->vb[i] = x;
    }
    sync();
    double rj = 0.0;
    if (lane < CW) {
      const int j = h * CW + lane;
      const double ct = sm->vec[j] + (sm->abx[0][j + 2] + sm->abx[1][j + 4]);  // CTmul's t + (p2 + p4)
      const double v = ct + sg * sm->vb[j] - sm->qq[j];
      rj = j < n ? v : 0.0;
    }
    double w[4];
    bcast<kNWc>(rj, w);
    double a[4] = {0.0, 0.0, 0.0, 0.0};
    Unroll<0, CW>::run([&](auto cc) {
      constexpr int c = decltype(cc)::value;
      fmac_bc<c % 16>(a[c % 4], w[c / 16], r[c]);
    });
    sm->tr[h][0][i] = (a[0] + a[1]) + (a[2] + a[3]);
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      lo_[k] = V ? LO(k) : 0.0;
      hi_[k] = V ? HI(k) : 0.0;
    }
    sync();
    if (V) {
      auto xa_of = [&](int row) -> double {  // combine's sum, inv_mul's sign, alpha
        const double* q0 = &sm->tr[0][0][0];
        constexpr int st = 3 * S::kNX;  // stride between the parts' rows of tr
        double s;
        if constexpr (kP == 2)
          s = q0[row] + q0[st + row];
        else
          s = (q0[row] + q0[st + row]) + (q0[2 * st + row] + q0[3 * st + row]);
        return alpha * -(row < n ? s : 0.0);
      };
      xa = xa_of(i);
      const double xm2 = i >= 2 ? xa_of(i - 2) : 0.0;
      const double xm4 = i >= 4 ? xa_of(i - 4) : 0.0;
      za[0] = c0 * xa;
      za[1] = c10 * xa + c11 * xm2;
      za[2] = (c20 * xa + c21 * xm2) + c22 * xm4;
    } else {
      xa = 0.0;
      za[0] = za[1] = za[2] = 0.0;
    }
  }
  // (Pbar v)_i from the workspace copy (coalesced: lanes read consecutive rows of one column)
  __device__ __forceinline__ double Pmul(double v) {
    if (V) sm->vb[i] = act ? v : 0.0;
    sync();
    double w[4];
    lbcast(sm->vb, w);
    int ii = i;  // opaque: the column addresses are recomputed per call, not hoisted out of the solver loops
    asm volatile("" : "+v"(ii));
    const double* pc = Pg + (size_t)(h * CW) * kMidLD + ii;
    double a[4] = {0.0, 0.0, 0.0, 0.0};
    piped<CW>([&](auto c) { return pc[(size_t)c * kMidLD]; },
              [&](auto cc, double pv) {
                constexpr int c = decltype(cc)::value;
                fmac_bc<c % 16>(a[c % 4], w[c / 16], pv);
              });
    return combine((a[0] + a[1]) + (a[2] + a[3]));
  }

  // KKT matrix A = Pbar + s I + Cbar' diag(rw) Cbar, row i -> r[].  The band entries (i, i + 2d - 4)
  // of row i are added into the thread's own Pbar entries in the workspace (addresses only this
  // thread reads), the half row is loaded, and the originals are written back.
  __device__ __forceinline__ void form(double s, const double rw[3]) {
    if (V) {
      double q[5] = {0.0, 0.0, 0.0, 0.0, 0.0};
      const double a1 = rw[1] * c11, a2 = rw[2] * c21, b2 = rw[2] * c22;
      q[0] = a1 * c11 + a2 * c21;  // lane p's term of entry (p - 2, p - 2)   (needed at i + 2)
      q[1] = b2 * c22;             // (p - 4, p - 4)                          (at i + 4)
      q[2] = a1 * c10 + a2 * c20;  // (p - 2, p)                              (at i + 2; own for (i, i - 2))
      q[3] = b2 * c21;             // (p - 4, p - 2)                          (at i + 4 / i + 2)
      q[4] = b2 * c20;             // (p - 4, p)                              (at i + 4; own for (i, i - 4))
      if (!act)
#pragma unroll
        for (int k = 0; k < 5; ++k) q[k] = 0.0;
      double p2[5], p4[5];
      xchg<5>(q, nullptr, nullptr, p2, p4);
      const double dg = (c0 * c0 * rw[0] + rw[1] * c10 * c10) + rw[2] * c20 * c20;
      const double b0 = (dg + p2[0] + p4[1]) + s;
      const double bp2 = p2[2] + p4[3];
      const double bp4 = p4[4];
      const double bm2 = i >= 2 ? q[2] + p2[3] : 0.0;  // = bp2 of row i - 2, same operands
      const double bm4 = i >= 4 ? q[4] : 0.0;          // = bp4 of row i - 4
      sm->band[0][i] = act ? bm4 : 0.0;
      sm->band[1][i] = act ? bm2 : 0.0;
      sm->band[2][i] = act ? b0 : 0.0;
      sm->band[3][i] = act ? bp2 : 0.0;
      sm->band[4][i] = act ? bp4 : 0.0;
    } else {
      xchg<5>(nullptr, nullptr, nullptr, nullptr, nullptr);
    }
    sync();
    int ii = i;  // opaque: addresses and masks recomputed per call (not hoisted into live registers)
    asm volatile("" : "+v"(ii));
    double orig[5];
    bool own[5];
    int addr[5];
#pragma unroll
    for (int d = 0; d < 5; ++d) {
      const int j = ii + 2 * d - 4;
      own[d] = ii < n && j >= 0 && j < n && j >= h * CW && j < h * CW + CW;
      addr[d] = own[d] ? j * kMidLD + ii : 0;
      orig[d] = own[d] ? Pg[addr[d]] : 0.0;
    }
#pragma unroll
    for (int d = 0; d < 5; ++d)
      if (own[d]) Pg[addr[d]] = orig[d] + sm->band[d][ii];
    // (same-thread accesses to the same addresses: the hardware keeps them in order, no waits)
    const double* pc = Pg + (size_t)(h * CW) * kMidLD + ii;
    Unroll<0, CW>::run([&](auto cc) {
      constexpr int c = decltype(cc)::value;
      r[c] = pc[(size_t)c * kMidLD];
    });
#pragma unroll
    for (int d = 0; d < 5; ++d)
      if (own[d]) Pg[addr[d]] = orig[d];
  }

  // Symmetric sweep on the rows in r[], pivots in pairs K = {k, k + 1} (n is even): afterwards A^{-1} = -r.
  // Sweeping a pair at once is the composition of its two single sweeps: with G = -A_KK^{-1} (2 x 2),
  //   A[i][j] -> A[i][j] + g_i . A[K][j]   (j not in K),  g_i = A'[i][K] . G,
  //   A[i][K] -> -g_i - e_i                 (the pair's columns),
  // where A'[i][K] is A[i][K] minus the unit vector of i when row i is one of the pair (then g_i = -G[i] -
  // e_i: row i becomes A_KK^{-1} A[K][j], its K entries -A_KK^{-1}[i]).  The part holding the pair's
  // columns publishes A'[.][K] through LDS (double buffered, row-major pairs); every thread reads its own
  // A'[i][K], the 2 x 2 block (unit vectors added back), and the two pivot rows A[K][j] = A'[j][K] of its
  // part's columns by per-lane reads and the DPP broadcast (lbcast).  G comes from the 2 x 2 block's own
  // sweep in every thread; its pivots are the sequential sweep's (the same non-positive-pivot test).
  // One barrier per two pivots.  The rounding differs from the pivot-by-pivot sweep; the optimum,
  // statuses and active sets do not.
  static constexpr int kSB = 2;
  static_assert(CW % kSB == 0, "a pivot pair lies inside one column part");
  // publish A'[i][k0], A'[i][k0 + 1] of this thread's row from its registers c0, c0 + 1
  template <int C0>
  __device__ __forceinline__ void publish(double (*q)[kSB], int k0) {
    double* o = q[i];
#pragma unroll
    for (int t = 0; t < kSB; ++t) o[t] = i == k0 + t ? r[C0 + t] - 1.0 : r[C0 + t];
  }
  __device__ __forceinline__ bool sweep() {
    bool ok = true;
    if (h == 0) publish<0>(sm->cbb[0], 0);
    for (int hk = 0; hk < kP; ++hk) {
      Unroll<0, CW / kSB>::run([&](auto cbc) {
        constexpr int cb = decltype(cbc)::value;
        constexpr int c0 = cb * kSB;  // the pair's first column, local to part hk
        const int k0 = hk * CW + c0;  // ... and global
        if (k0 < n) {
          sync();
          const int gb = hk * (CW / kSB) + cb;
          double (*q)[kSB] = sm->cbb[gb & 1];
          // G = -A_KK^{-1} by the 2 x 2 block's sweep
          double g00 = q[k0][0] + 1.0, g01 = q[k0][1], g11 = q[k0 + 1][1] + 1.0;
          ok = ok && (g00 > 0.0) && isfinite(g00);
          double inv = __builtin_amdgcn_rcp(g00);
          inv = fma(inv, fma(-g00, inv, 1.0), inv);
          inv = fma(inv, fma(-g00, inv, 1.0), inv);
          const double c1 = g01 * inv;
          g11 = fma(-c1, g01, g11);
          g00 = -inv;
          g01 = c1;
          ok = ok && (g11 > 0.0) && isfinite(g11);
          double inv1 = __builtin_amdgcn_rcp(g11);
          inv1 = fma(inv1, fma(-g11, inv1, 1.0), inv1);
          inv1 = fma(inv1, fma(-g11, inv1, 1.0), inv1);
          const double c0v = g01 * inv1;
          g00 = fma(-c0v, g01, g00);
          g01 = c0v;
          g11 = -inv1;
          // g_i = A'[i][K] . G
          const double a0 = q[i][0], a1 = q[i][1];
          double gm[kSB];
          gm[0] = fma(a1, g01, a0 * g00);
          gm[1] = fma(a1, g11, a0 * g01);
          // the two pivot rows of this part's columns, by DPP broadcast
          double w0[4], w1[4];
          {
            const double* qp = &q[h * CW][0];
            const double x0 = lane < CW ? qp[kSB * lane] : 0.0;
            const double x1 = lane < CW ? qp[kSB * lane + 1] : 0.0;
            bcast<kNWc>(x0, w0);
            bcast<kNWc>(x1, w1);
          }
          __builtin_amdgcn_sched_barrier(0);
          // fmac_bc: fma(A[K][j], g, r)
          auto upd = [&](auto jcc, const double g[kSB]) {
            constexpr int jc = decltype(jcc)::value;
            fmac_bc<jc % 16>(r[jc], w0[jc / 16], g[0]);
            fmac_bc<jc % 16>(r[jc], w1[jc / 16], g[1]);
          };
          // the next pair's columns first (the part that holds them), published for the next step
          constexpr int nc0 = c0 + kSB < CW ? c0 + kSB : 0;  // their first register
          const bool early = (c0 + kSB < CW ? h == hk : h == hk + 1) && k0 + kSB < n;
          if (early) {
            upd(std::integral_constant<int, nc0>{}, gm);
            upd(std::integral_constant<int, nc0 + 1>{}, gm);
            publish<nc0>(sm->cbb[(gb + 1) & 1], k0 + kSB);
          }
          // every other column of this part; no per-column branches (they cost the row's registers:
          // scratch): the columns done above take a zero update, the pair's own columns are overwritten
          double gs[kSB];
#pragma unroll
          for (int t = 0; t < kSB; ++t) gs[t] = early ? 0.0 : gm[t];
          Unroll<0, CW>::run([&](auto jcc) {
            constexpr int jc = decltype(jcc)::value;
            if constexpr (jc >= nc0 && jc < nc0 + kSB)
              upd(jcc, gs);
            else
              upd(jcc, gm);
          });
          if (h == hk) {
#pragma unroll
            for (int t = 0; t < kSB; ++t) r[c0 + t] = -gm[t] - (i == k0 + t ? 1.0 : 0.0);
          }
        }
      });
    }
    sync();
    return ok;
  }

  // Rank-1 change A' = A + delta c c' with c the row (tau, l) of Cbar (Sherman-Morrison, as the
  // one-wave kernel): u = A^{-1} c from at most three columns of the inverse, r += (kappa u_i) u_j.
  __device__ __forceinline__ bool rank1(int tau, int lu, double delta) {
    const double k0 = tau == 0 ? sm->cf[0][lu] : (tau == 1 ? sm->cf[1][lu] : sm->cf[3][lu]);
    const double k1 = lu >= 2 ? (tau == 1 ? sm->cf[2][lu] : (tau == 2 ? sm->cf[4][lu] : 0.0)) : 0.0;
    const double k2 = lu >= 4 ? (tau == 2 ? sm->cf[5][lu] : 0.0) : 0.0;
    const double kk[3] = {k0, k1, k2};
    double(*T)[X_()] = sm->tr[h];
#pragma unroll
    for (int a = 0; a < 3; ++a) {
      const int ja = lu - 2 * a;
      const bool mine = ja >= 0 && ja >= h * CW && ja < h * CW + CW;
      double t = 0.0;
      if (mine) t = kk[a] * pick<0, CW>(ja - h * CW);
      T[a][i] = t;
    }
    sync();
    if (V) {  // each term comes from one part (the others hold exact zeros): the one-wave order
      double t[3];
#pragma unroll
      for (int a = 0; a < 3; ++a) {
        if constexpr (kP == 2)
          t[a] = sm->tr[0][a][i] + sm->tr[1][a][i];
        else
          t[a] = (sm->tr[0][a][i] + sm->tr[1][a][i]) + (sm->tr[2][a][i] + sm->tr[3][a][i]);
      }
      const double u = (t[0] + t[1]) + t[2];
      sm->vec[i] = act ? -u : 0.0;
    }
    sync();
    const double* U = sm->vec;
    const double ui = U[i];
    const double cu = (k0 * U[lu] + k1 * U[lu >= 2 ? lu - 2 : 0]) + k2 * U[lu >= 4 ? lu - 4 : 0];
    const double den = 1.0 + delta * cu;
    if (!(den > kRank1Min) || !isfinite(den)) return false;  // uniform
    const double m = (delta / den) * ui;
    double w[4];
    lbcast(U, w);
    Unroll<0, CW>::run([&](auto cc) {
      constexpr int c = decltype(cc)::value;
      fmac_bc<c % 16>(r[c], w[c / 16], m);
    });
    return true;
  }
  static constexpr int X_() { return S::kNX; }
  template <int LO, int HI>
  __device__ __forceinline__ double pick(int j) const {
    if constexpr (HI - LO <= 2) {
      double v = r[LO];
      if constexpr (HI - LO == 2) v = j == LO + 1 ? r[LO + 1] : v;
      asm volatile("" : "+v"(v));
      return v;
    } else {
      constexpr int M = (LO + HI) / 2;
      if (j < M) return pick<LO, M>(j);
      return pick<M, HI>(j);
    }
  }
};

// ------------------------------------------------------------------ setup
// The one-wave kernel's setup_qp: condensing (column i of H by the backward adjoint recursion, here
// computed by both halves' threads of row i, each keeping its half), OSQP Ruiz + cost scaling on the
// rows in registers (column maxima = row maxima: H symmetric), Pbar to the workspace, the per-variable
// data.  Returns true on non-finite data.
template <int NT>
__device__ __forceinline__ bool mid_setup(const mpcqp_params& p, Mid<NT>& C) {
  using S = MidShape<NT>;
  MidLds<NT>& sm = *C.sm;
  const int N = C.N, n = C.n, i = C.i;
  const bool V = C.V, act = C.act, even = C.even;
  const int cc = i & 1;
  const double dt = p.dt;
  const double* mdl = sm.model;
  const double* al = mdl;
  const double* be = mdl + N;
  const double* ga = mdl + 2 * N;
  const double* et = mdl + 3 * N;
  const double* si = mdl + 4 * N;
  const double* cz0 = mdl + 5 * N;
  const double* cz1 = mdl + 6 * N;
  const double* rr = mdl + 7 * N;
  const double* x0 = mdl + 11 * N + 4;
  const double* up = mdl + 11 * N + 8;
  const int tid = threadIdx.x;
  // prefix sums and free response: ONE sequential recurrence on lanes 0..3 of wave 0 (one instruction
  // stream, every load ahead of the chain; the one-wave kernel's setup): lanes 0 / 1 the prefix sums of
  // alpha / gamma (pre[0] / pre[2]), lanes 2 / 3 the free response's x / y at W = 0,
  // acc <- acc + A[k] h + B[k] v_k + C[k], with (h, v, C) = (1, 0, 0) on the prefix lanes (exactly
  // acc + A[k]) and (psi, v_0 at k = 0, c0 | c1) on the free-response lanes.  The heading and speed rows
  // of e_m are lane-parallel (wave 1).
  if (tid < 4) {
    const bool fr = tid >= 2;
    const int q = tid & 1;
    const double* __restrict__ A = mdl + (q ? 2 * N : 0);
    const double* __restrict__ Bv = mdl + (q ? 3 * N : N);
    const double* __restrict__ Cc = mdl + (q ? 6 * N : 5 * N);
    const double* __restrict__ R = rr + 4 + q;
    const double h = fr ? x0[2] : 1.0, v0 = fr ? x0[3] : 0.0, one = fr ? 1.0 : 0.0;
    double acc = fr ? x0[q] : 0.0;
    double* __restrict__ out = fr ? sm.err[q] : sm.pre[2 * q];
    if (!fr) out[0] = 0.0;
    const double b0 = Bv[0];
    // the loads issued a group ahead of the chain (piped): all of them up front is 3 NT registers
    piped<NT, 8>(
        [&](auto kc) {
          constexpr int k = decltype(kc)::value;
          const int kk = k < N ? k : N - 1;  // (steps past N: loaded in range, not used)
          return Rq{A[kk], Cc[kk], R[4 * kk]};
        },
        [&](auto kc, const Rq& v) {
          constexpr int k = decltype(kc)::value;
          // straight-line: the steps past N (only the top 8: N >= NT - 7) keep acc and write rows the
          // condensing reads only into discarded selects
          const double an = acc + v.a * h + (k == 0 ? b0 : 0.0) * (k == 0 ? v0 : 0.0) + one * v.c;
          if constexpr (k >= NT - 8)
            acc = k < N ? an : acc;
          else
            acc = an;
          out[k + 1] = acc - one * v.r;
        });
  } else if (tid >= kWave && tid < kWave + N) {
    const int m = tid - kWave + 1;
    sm.err[2][m] = x0[2] - rr[4 * m + 2];
    sm.err[3][m] = 0.0 - rr[4 * m + 3];
  }
  // the band table of the input cost: kinds 0 / 1 / 2 (speed, the last speed, steering), the entry for
  // column col of row i at [kind][kNX + col - i] (one LDS read per column below instead of a compare-and-
  // select per column and band entry).  It lives in the rank-1 buffer, unused until the polish.
  const double r00 = 0.5 * (p.r[0] + p.r[0]) / (dt * dt), r10 = 0.5 * (p.r[2] + p.r[1]) / dt;
  const double r11 = 0.5 * (p.r[3] + p.r[3]);
  double* bt = &sm.tr[0][0][0];
  static_assert(sizeof(sm.tr) >= sizeof(double) * 3 * 2 * S::kNX, "band table in the rank-1 buffer");
  for (int e = tid; e < 3 * 2 * S::kNX; e += S::kThreads) {
    const int kind = e / (2 * S::kNX), d = e % (2 * S::kNX) - S::kNX;
    double v = 0.0;
    if (kind < 2) {
      if (d == 0) v = kind == 0 ? 2.0 * r00 : r00;
      if (d == 2 || d == -2) v = -r00;
      if (d == 1) v = r10;
      if (d == 3) v = -r10;
    } else {
      if (d == 0) v = r11;
      if (d == -1) v = r10;
      if (d == -3) v = -r10;
    }
    bt[e] = v;
  }
  mid_barrier();
  C.T.mark(9);

  // ---- condense: column i of H by the backward adjoint recursion, the rows of this thread's part into
  // r[]; the gradient column (the free response) on a lane of its own, into sm.g.
  // mu_m = W_m s_m + A_m' mu_{m+1};  H[(k, c'), col] = (B_k e_c')' mu_{k+1}
  // Every lane runs the same instruction stream (the one-wave kernel's condensing): the gradient column and
  // the two kinds of variable column differ only in lane constants and in which LDS row a lane reads per
  // step.  Per step m the column's state sensitivity s = (s0, s1, s2, s3) is
  //   speed v_{j+1} (i = 2 j):        (be_{j+1}, et_{j+1}, 0, 0) from m = j + 2 on, (0, 0, 0, 1) at m = j + 1
  //   steering delta_j (i = 2 j + 1): si_j (P_a[m] - P_a[j+1], P_g[m] - P_g[j+1], 1, 0) from m = j + 1 on
  //   gradient column:                e_m
  // Part h keeps rows [h CW, h CW + CW), i.e. the steps m = h CW / 2 + 1 .. h CW / 2 + CW / 2, and runs
  // the recursion only down to its first one.  The gradient lane is row n of part 0 (a padding row),
  // or, when the rows fill the row waves (n = kNX), a second pass on the last part's first row wave.
  double Q[4][4], QN[4][4];
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int b = 0; b < 4; ++b) {
      Q[a][b] = 0.5 * (p.q[4 * a + b] + p.q[4 * b + a]);
      QN[a][b] = 0.5 * (p.q_terminal[4 * a + b] + p.q_terminal[4 * b + a]);
    }
  // the cost weights are diagonal in the default parameters (a uniform branch)
  bool diag = true;
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int b = 0; b < 4; ++b)
      if (a != b) diag = diag && p.q[4 * a + b] == 0.0 && p.q_terminal[4 * a + b] == 0.0;
  constexpr int CW = S::CW;
  constexpr int kHS = CW / 2;  // steps per part: part h holds the rows of the steps h kHS + 1 .. h kHS + kHS
  const int hu = __builtin_amdgcn_readfirstlane(C.h);
  const int wpu = __builtin_amdgcn_readfirstlane(C.w % S::kRW);
  // the gradient column: row n of every part (a padding row, its part's rows in r[] like a variable
  // column, stored to sm.g after the pass), or, when the rows fill the row waves (n = kNX), a second
  // wave-uniform pass on the last part's first row wave that stores sm.g per step
  const bool g_lane = n < S::kNX && i == n;
  const bool g_pass = n == S::kNX && hu == S::kParts - 1 && wpu == 0;  // uniform
  // Straight-line code per part block (one uniform branch per block), so the scheduler pipelines the
  // steps' LDS reads: the mid buckets hold N >= NT - 7, so only the top 8 steps can lie past N or be
  // the terminal one, and those select instead of branching.
  static_assert(kHS >= 8, "the top 8 steps lie in the last part's block");
  auto recursion = [&](auto is_diag, auto is_gpass, bool gcol, int col, int hlo) {
    constexpr bool kDiag = decltype(is_diag)::value;
    constexpr bool kGPass = decltype(is_gpass)::value;  // second pass: the gradient column, stored per step
    const int j = col >> 1;
    const int cc = col & 1;
    const double sj = gcol ? 1.0 : si[j];
    const double pa0 = gcol ? 0.0 : sm.pre[0][j + 1], pg0 = gcol ? 0.0 : sm.pre[2][j + 1];
    const double bj = (!gcol && j + 1 < N) ? be[j + 1] : 0.0, ej = (!gcol && j + 1 < N) ? et[j + 1] : 0.0;
    const bool st = gcol || cc == 1;  // s0 / s1 from the prefix sums (or e_m)
    const double k01 = st ? sj : 0.0, o0 = st ? pa0 : 0.0, o1 = st ? pg0 : 0.0;
    const double b0 = st ? 0.0 : bj, b1 = st ? 0.0 : ej;
    const double kg = gcol ? 1.0 : 0.0;
    const double c2v = (!gcol && cc == 1) ? sj : 0.0;
    // thresholds: s0 / s1 live for m > t01, s2 for m > t2, s3 == 1 at m == t3
    const int t01 = gcol ? 0 : (cc == 1 ? j : j + 1);
    const int t2 = gcol ? 0 : j;
    const int t3 = (!gcol && cc == 0) ? j + 1 : -1;
    const double* X0 = gcol ? sm.err[0] : sm.pre[0];
    const double* X1 = gcol ? sm.err[1] : sm.pre[2];
    const double* X2 = gcol ? sm.err[2] : sm.pre[0];  // kg = 0: read, not used
    const double* X3 = gcol ? sm.err[3] : sm.pre[0];
    double mu0 = 0.0, mu1 = 0.0, mu2 = 0.0;
    auto step = [&](auto mcst) {
      constexpr int m = decltype(mcst)::value;
      constexpr bool kTop = m > NT - 8;  // may be past N (skipped: selects keep the state) or terminal
      const bool on = !kTop || m <= N;
      const bool term = kTop && m == N;
      double s0 = fma(k01, X0[m] - o0, b0);
      double s1 = fma(k01, X1[m] - o1, b1);
      s0 = m > t01 ? s0 : 0.0;
      s1 = m > t01 ? s1 : 0.0;
      const double s2 = fma(kg, X2[m], m > t2 ? c2v : 0.0);
      const double s3 = fma(kg, X3[m], m == t3 ? 1.0 : 0.0);
      auto Wm = [&](int a, int k) -> double {
        if constexpr (kTop)
          return term ? QN[a][k] : Q[a][k];
        else
          return Q[a][k];
      };
      double w0, w1, w2, w3;
      if constexpr (kDiag) {
        w0 = Wm(0, 0) * s0;
        w1 = Wm(1, 1) * s1;
        w2 = Wm(2, 2) * s2;
        w3 = Wm(3, 3) * s3;
      } else {
        w0 = Wm(0, 0) * s0 + Wm(0, 1) * s1 + Wm(0, 2) * s2 + Wm(0, 3) * s3;
        w1 = Wm(1, 0) * s0 + Wm(1, 1) * s1 + Wm(1, 2) * s2 + Wm(1, 3) * s3;
        w2 = Wm(2, 0) * s0 + Wm(2, 1) * s1 + Wm(2, 2) * s2 + Wm(2, 3) * s3;
        w3 = Wm(3, 0) * s0 + Wm(3, 1) * s1 + Wm(3, 2) * s2 + Wm(3, 3) * s3;
      }
      const double m0 = mu0, m1 = mu1;
      double ha = w3 + (be[m] * m0 + et[m] * m1);
      double n0 = w0 + m0;
      double n1 = w1 + m1;
      double n2 = w2 + (mu2 + al[m] * m0 + ga[m] * m1);
      if constexpr (kTop) {  // the terminal step starts the recursion; steps past N leave it at zero
        ha = term ? w3 : ha;
        n0 = term ? w0 : n0;
        n1 = term ? w1 : n1;
        n2 = term ? w2 : n2;
        mu0 = on ? n0 : mu0;
        mu1 = on ? n1 : mu1;
        mu2 = on ? n2 : mu2;
      } else {
        mu0 = n0;
        mu1 = n1;
        mu2 = n2;
      }
      const double hd = si[m - 1] * mu2;
      constexpr int row0 = 2 * (m - 1);
      if constexpr (kGPass) {
        if (on) {
          sm.g[row0] = ha;
          sm.g[row0 + 1] = hd;
        }
      } else {
        // rows row0, row0 + 1 of the step's part (CW is even); this block runs only on that part's
        // waves and the ones below it, so the store is a uniform test of the part
        if (hu == row0 / CW) {
          C.r[row0 % CW] = on ? ha : C.r[row0 % CW];
          C.r[row0 % CW + 1] = on ? hd : C.r[row0 % CW + 1];
        }
      }
    };
    Unroll<0, S::kParts>::run([&](auto bc) {
      constexpr int blk = S::kParts - 1 - decltype(bc)::value;  // the part whose steps these are
      if (blk >= hlo) {
        Unroll<0, kHS>::run([&](auto tc) {
          step(std::integral_constant<int, blk * kHS + kHS - decltype(tc)::value>{});
        });
      }
    });
  };
  {
    // first pass: every lane; inactive rows take column 0's constants and are zeroed below.  The rows
    // of the steps past N (N < NT) are not written: zeros.
#pragma unroll
    for (int c = 0; c < CW; ++c) C.r[c] = 0.0;
    if (diag)
      recursion(std::true_type{}, std::false_type{}, g_lane, act ? i : 0, hu);
    else
      recursion(std::false_type{}, std::false_type{}, g_lane, act ? i : 0, hu);
    if (g_lane)
#pragma unroll
      for (int c = 0; c < CW; ++c) sm.g[hu * CW + c] = C.r[c];
    if (!act)
#pragma unroll
      for (int c = 0; c < CW; ++c) C.r[c] = 0.0;
    if constexpr (S::NP == S::kNX) {
      if (g_pass) {  // n = kNX: the gradient column as a second, wave-uniform pass
        if (diag)
          recursion(std::true_type{}, std::true_type{}, true, 0, 0);
        else
          recursion(std::false_type{}, std::true_type{}, true, 0, 0);
      }
    }
  }
  const bool gthread = (g_lane && hu == 0) || (g_pass && C.lane == 0);
  mid_barrier();
  C.T.mark(10);
  // input cost sum_k U_k' R U_k with a_k = (v_{k+1} - v_k)/dt: a band of column i, read from the band
  // table at offset col - i (above)
  if (gthread) {
    sm.g[0] += -x0[3] * r00;
    sm.g[1] += -x0[3] * r10;
  }
  if (act) {
    const int kind = cc == 1 ? 2 : (i + 2 < n ? 0 : 1);
    const double* tb = bt + kind * (2 * S::kNX) + S::kNX + hu * CW - i;
#pragma unroll
    for (int c = 0; c < CW; ++c) C.r[c] += tb[c];
  }
  mid_barrier();

  // ---- unscaled data: P = 2H, q = 2g, folded row bounds (V threads: one variable per row)
  double qv = V && act ? 2.0 * sm.g[i] : 0.0;
  double cmx[4] = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
  for (int c = 0; c < CW; ++c) {
    C.r[c] = 2.0 * C.r[c];
    cmx[c % 4] = fmax(cmx[c % 4], fabs(C.r[c]));
  }
  // column max of |P| = row max (the parts combined)
  auto rowmax = [&](const double* cm4) -> double {
    double v = fmax(fmax(cm4[0], cm4[1]), fmax(cm4[2], cm4[3]));
    if (!V) sm.pp[C.h - 1][i] = v;
    mid_barrier();
    if (V) {
      if constexpr (S::kParts == 2)
        v = fmax(v, sm.pp[0][i]);
      else
        v = fmax(fmax(v, sm.pp[0][i]), fmax(sm.pp[1][i], sm.pp[2][i]));
    }
    mid_barrier();
    return V && act ? v : 0.0;
  };
  double cmax = rowmax(cmx);
  C.T.mark(11);
  double lo[3], hi[3], wt[3], E[3];
  const double idt = 1.0 / dt, v0 = x0[3];
  double k1[2], k2[3];
  const bool va = V && act, ve = V && even;
  k1[0] = va ? (even ? idt : 1.0) : 0.0;
  k1[1] = (ve && i >= 2) ? -idt : 0.0;
  k2[0] = va ? (even ? idt : 1.0) : 0.0;
  k2[1] = va ? (even ? (i >= 2 ? -2.0 * idt : 0.0) : (i >= 3 ? -1.0 : 0.0)) : 0.0;
  k2[2] = (ve && i >= 4) ? idt : 0.0;
  {
    const double ofa = i == 0 ? v0 * idt : 0.0;
    const double ofr = i < 2 ? up[cc] + ofa : (i == 2 ? -v0 * idt : 0.0);
    lo[0] = ve ? p.v_bounds[0] : 0.0;
    hi[0] = ve ? p.v_bounds[1] : 0.0;
    wt[0] = ve ? p.slack_velocity : 0.0;
    lo[1] = va ? p.u_bounds[2 * cc] + ofa : 0.0;
    hi[1] = va ? p.u_bounds[2 * cc + 1] + ofa : 0.0;
    wt[1] = va ? p.slack_input : 0.0;
    lo[2] = va ? p.du_bounds[2 * cc] + ofr : 0.0;
    hi[2] = va ? p.du_bounds[2 * cc + 1] + ofr : 0.0;
    wt[2] = va ? p.slack_rate : 0.0;
    E[0] = ve ? 1.0 : 0.0;
    E[1] = va ? 1.0 : 0.0;
    E[2] = va ? 1.0 : 0.0;
  }
  double D = va ? 1.0 : 0.0;
  double cscale = 1.0;
  auto rsqrt = [](double v) {
    double y = __builtin_amdgcn_rsq(v);
    y = y * fma(-0.5 * v, y * y, 1.5);
    return y * fma(-0.5 * v, y * y, 1.5);
  };
  double cpend = 1.0;
  for (int it = 0; it < p.scaling; ++it) {
    // column norms of [P; A]: own rows and the banded rows 2 and 4 ahead; row norms of A
    double ahead[2] = {fmax(E[1] * fabs(k1[1]), E[2] * fabs(k2[1])), E[2] * fabs(k2[2])};
    double a2[2], a4[2];
    C.template xchg<2>(ahead, nullptr, nullptr, a2, a4);
    double ccol = fmax(fmax(E[0], E[1] * fabs(k1[0])), E[2] * fabs(k2[0]));
    ccol = fmax(ccol, a2[0]);
    ccol = fmax(ccol, a4[1]);
    ccol *= D;
    const double dl = va ? rsqrt(limit_scaling(fmax(cmax, ccol))) : 0.0;
    double Dm2, Dm4;
    C.template xchg<1>(&D, &Dm2, &Dm4, nullptr, nullptr);
    const double r1 = fmax(fabs(k1[0]) * D, fabs(k1[1]) * Dm2);
    const double r2 = fmax(fmax(fabs(k2[0]) * D, fabs(k2[1]) * Dm2), fabs(k2[2]) * Dm4);
    const double el0 = ve ? rsqrt(limit_scaling(E[0] * D)) : 0.0;
    const double el1 = va ? rsqrt(limit_scaling(E[1] * r1)) : 0.0;
    const double el2 = va ? rsqrt(limit_scaling(E[2] * r2)) : 0.0;
    // P <- ct_prev dl P dl: the row's factor and the half's column factors from LDS
    if (V) sm.vec[i] = dl;
    mid_barrier();
    const double dlc = sm.vec[i] * cpend;
    const double* dj = sm.vec + C.h * CW;
    double cmp[4] = {0.0, 0.0, 0.0, 0.0};
    piped<CW>([&](auto c) { return dj[c]; }, [&](auto c, double dv) {
      const double t = C.r[c] * (dv * dlc);
      C.r[c] = t;
      cmp[c % 4] = fmax(cmp[c % 4], fabs(t));
    });
    const double cm2 = rowmax(cmp);  // (its barriers also order the next pass's writes of vec)
    D *= dl;
    qv *= dl;
    E[0] *= el0;
    E[1] *= el1;
    E[2] *= el2;
    double red2[2] = {va ? cm2 : 0.0, 0.0};
    C.template reduce<1, false>(red2);
    const double cn = red2[0] / n;
    const double qn = limit_scaling(C.bmax(fabs(qv)));
    const double ct = 1.0 / limit_scaling(fmax(cn, qn));
    cpend = ct;
    qv *= ct;
    cmax = cm2 * ct;
    cscale *= ct;
  }
#pragma unroll
  for (int c = 0; c < CW; ++c) C.r[c] *= cpend;
  C.T.mark(12);
  // Pbar to the workspace (every row, padding zeros included)
  {
    double* pc = C.Pg + (size_t)(C.h * CW) * kMidLD + i;
    bool fin = true;
#pragma unroll
    for (int c = 0; c < CW; ++c) {
      pc[(size_t)c * kMidLD] = C.r[c];
      fin = fin && isfinite(C.r[c]);
    }
    C.T.mark(13);
    bool finite = fin && isfinite(qv) && isfinite(cscale);
    double wb[3];
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      lo[k] *= E[k];
      hi[k] *= E[k];
      wb[k] = E[k] > 0.0 ? cscale * wt[k] / (E[k] * E[k]) : 0.0;
      finite = finite && isfinite(lo[k]) && isfinite(hi[k]);
    }
    const bool bad = C.bany(!finite);
    C.qv = qv;
    C.D = D;
    C.cscale = cscale;
    double Dm2, Dm4;
    C.template xchg<1>(&D, &Dm2, &Dm4, nullptr, nullptr);
    C.c0 = E[0] * D;
    C.c10 = (E[1] * k1[0]) * D;
    C.c11 = (E[1] * k1[1]) * Dm2;
    C.c20 = (E[2] * k2[0]) * D;
    C.c21 = (E[2] * k2[1]) * Dm2;
    C.c22 = (E[2] * k2[2]) * Dm4;
    if (V)
#pragma unroll
      for (int k = 0; k < 3; ++k) {
        sm.bE[k][i] = E[k];
        sm.blo[k][i] = lo[k];
        sm.bhi[k][i] = hi[k];
        sm.bwb[k][i] = wb[k];
      }
    if (V) {
      sm.cf[0][i] = C.c0;
      sm.cf[1][i] = C.c10;
      sm.cf[2][i] = C.c11;
      sm.cf[3][i] = C.c20;
      sm.cf[4][i] = C.c21;
      sm.cf[5][i] = C.c22;
    }
    mid_barrier();
    C.T.mark(14);
    return bad;
  }
}

// ------------------------------------------------------------------ polish (one-wave polish_qp)
template <int NT>
__device__ __forceinline__ int mid_polish(Mid<NT>& C, double& x, const double zg[3], int max_it, int& pol_it,
                                          int& nfact, int& n_ls) {
  const bool act = C.V && C.act;
  int result = 0;
  double zc[3];
  int cd[3];
  {
    double lo_[3], hi_[3];
    C.Cmul(x, zc, lo_, hi_);
#pragma unroll
    for (int k = 0; k < 3; ++k) cd[k] = zg[k] > hi_[k] ? 2 : (zg[k] < lo_[k] ? 1 : 0);
  }
  double Px = C.Pmul(x);
  const int kMaxRank1 = C.n / 2;
  double rwf[3] = {0.0, 0.0, 0.0};
  bool have_fact = false;
  for (int pass = 0; pass < max_it; ++pass) {
    ++pol_it;
    C.opaque();
    double rw[3], tmp[3];
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      rw[k] = cd[k] ? 2.0 * C.WB(k) : 0.0;
      tmp[k] = cd[k] == 2 ? rw[k] * C.HI(k) : (cd[k] == 1 ? rw[k] * C.LO(k) : 0.0);
    }
    C.T.mbegin();
    bool refac = !have_fact;
    if (!refac) {
      // changed soft rows: each row wave's ballots, combined through LDS (uniform in every thread)
      unsigned long long(*mk)[2] = C.sm->msk[C.rs];
      C.rs = __builtin_amdgcn_readfirstlane(C.rs ^ 1);
#pragma unroll
      for (int k = 0; k < 3; ++k) {
        const unsigned long long b = __ballot(act && rw[k] != rwf[k]);
        if (C.V && C.lane == 0) mk[k][C.w] = b;
        if (C.V) C.sm->dw[k][C.i] = rw[k] - rwf[k];
      }
      mid_barrier();
      unsigned long long chg[3][2];
      int nchg = 0;
#pragma unroll
      for (int k = 0; k < 3; ++k)
#pragma unroll
        for (int q = 0; q < 2; ++q) {
          chg[k][q] = q < MidShape<NT>::kRW ? mk[k][q] : 0ull;
          nchg += __popcll(chg[k][q]);
        }
      refac = nchg > kMaxRank1;
#pragma unroll
      for (int k = 0; k < 3; ++k)
#pragma unroll
        for (int q = 0; q < 2; ++q) {
          unsigned long long m = chg[k][q];
          while (m && !refac) {
            const int l = 64 * q + __builtin_ctzll(m);
            m &= m - 1;
            refac = !C.rank1(k, l, C.sm->dw[k][l]);
            ++C.n_r1;
          }
        }
    }
    C.T.mark(16);
    if (refac) {
      C.T.begin();
      C.form(0.0, rw);
      const bool okf = C.sweep();
      C.T.end(4);
      ++C.n_full;
      if (C.bany(!okf)) {
        result = -1;
        break;
      }
      have_fact = true;
    }
    ++nfact;
    C.T.mbegin();
#pragma unroll
    for (int k = 0; k < 3; ++k) rwf[k] = rw[k];
    const double rhs = C.CTmul(tmp) - C.qv;
    double xn = C.inv_mul(rhs);
    double zn[3], lo_[3], hi_[3];
    C.Cmul(xn, zn, lo_, hi_);
    bool diff = false;
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      const int c2 = zn[k] > hi_[k] ? 2 : (zn[k] < lo_[k] ? 1 : 0);
      diff = diff || (c2 != cd[k]);
    }
    if (C.bany(!isfinite(xn))) {
      result = -1;
      break;
    }
    const bool anyd = C.bany(diff);
    C.T.mark(17);
    if (!anyd) {
      double t3[3];
#pragma unroll
      for (int k = 0; k < 3; ++k) t3[k] = rw[k] * zn[k];
      const double Mx = C.Pmul(xn) + C.CTmul(t3);
      xn += C.inv_mul(rhs - Mx);
      C.Cmul(xn, zn);
      diff = false;
#pragma unroll
      for (int k = 0; k < 3; ++k) {
        const int c2 = zn[k] > hi_[k] ? 2 : (zn[k] < lo_[k] ? 1 : 0);
        diff = diff || (c2 != cd[k]);
      }
      if (C.bany(!isfinite(xn))) {
        result = -1;
        break;
      }
      if (!C.bany(diff)) {
        x = xn;
        result = 1;
        break;
      }
    }
    C.T.mark(18);
    // exact line search along d = xn - x
    double tb[3];
#pragma unroll
    for (int k = 0; k < 3; ++k) tb[k] = rw[k] * (zn[k] - (cd[k] == 2 ? hi_[k] : (cd[k] == 1 ? lo_[k] : 0.0)));
    const double ctb = C.CTmul(tb);
    const double dx = act ? xn - x : 0.0;
    const double Pd = act ? (-ctb - C.qv) - Px : 0.0;
    double zd[3];
#pragma unroll
    for (int k = 0; k < 3; ++k) zd[k] = zn[k] - zc[k];
    double s2[2] = {act ? dx * Pd : 0.0, act ? (Px + C.qv) * dx : 0.0};
    C.template reduce<2, false>(s2);
    const double qd = s2[0], lin = s2[1];
    // the soft rows' bounds (above) and weights in registers for the trials (LDS round trips per use otherwise)
    double wb2[3];
#pragma unroll
    for (int k = 0; k < 3; ++k) wb2[k] = 2.0 * C.WB(k);
    double t = 1.0;
    for (int ls = 0; ls < 40; ++ls) {
      ++n_ls;
      double g12[2] = {0.0, 0.0};
#pragma unroll
      for (int k = 0; k < 3; ++k) {
        const double zt = zc[k] + t * zd[k];
        const double rr = zt > hi_[k] ? zt - hi_[k] : (zt < lo_[k] ? zt - lo_[k] : 0.0);
        g12[0] += wb2[k] * rr * zd[k];
        if (rr != 0.0) g12[1] += wb2[k] * zd[k] * zd[k];
      }
      if (!C.V) g12[0] = g12[1] = 0.0;
      C.template reduce<2, false>(g12);
      const double d1 = lin + t * qd + g12[0];
      const double d2 = qd + g12[1];
      if (d1 <= 0.0 || !(d2 > 0.0)) break;
      const double tn = fmax(0.0, t - d1 / d2);
      if (tn >= t) break;
      bool moved = false;
#pragma unroll
      for (int k = 0; k < 3; ++k) {
        const double za = zc[k] + t * zd[k], zb = zc[k] + tn * zd[k];
        const int ca = za > hi_[k] ? 2 : (za < lo_[k] ? 1 : 0);
        const int cb = zb > hi_[k] ? 2 : (zb < lo_[k] ? 1 : 0);
        moved = moved || ca != cb;
      }
      t = tn;
      if (!C.bany(C.V && moved)) break;
    }
    C.T.mark(19);
    x = x + t * dx;
    Px = Px + t * Pd;
    C.Cmul(x, zc);
    C.T.mark(20);
#pragma unroll
    for (int k = 0; k < 3; ++k) cd[k] = zc[k] > hi_[k] ? 2 : (zc[k] < lo_[k] ? 1 : 0);
  }
  return result;
}

// ------------------------------------------------------------------ ADMM (one-wave admm_run)
struct MidAdmm {
  double x, z[3], y[3], rho, rho_next;
  int it, nfact;
  bool need_fact, rho_change;
};
enum : int { kMidBad = -1, kMidMaxIter = 0, kMidConverged = 1, kMidApprox = 3, kMidAttempt = 4 };

template <int NT>
__device__ __forceinline__ int mid_admm(const mpcqp_params& p, Mid<NT>& C, MidAdmm& S) {
  const bool act = C.V && C.act;
  const double sg = p.sigma, alpha = p.alpha;
  const bool early = p.polish != 0 && p.polish_from > 0;
  int ev = kMidMaxIter;
  bool done = false;
  if (C.V) C.sm->qq[C.i] = C.qv;  // read after the first iteration's barrier
  while (S.it < p.max_iter && !done) {
    if (S.need_fact) {
      const double rw[3] = {S.rho, S.rho, S.rho};
      C.T.begin();
      C.form(sg, rw);
      ++S.nfact;
      const bool okf = C.sweep();
      C.T.end(1);
      if (C.bany(!okf)) {
        ev = kMidBad;
        break;
      }
      S.need_fact = false;
    }
    const double rho = S.rho;
    double pb[3], rpb[3];
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      pb[k] = 2.0 * C.WB(k) / (rho + 2.0 * C.WB(k));
      rpb[k] = rho * pb[k];
    }
    const double ir = 1.0 / rho, oma = 1.0 - alpha;
    while (!S.need_fact && S.it < p.max_iter) {
      const int it = ++S.it;
      C.opaque();
      C.T.begin();
      double tmp[3];
#pragma unroll
      for (int k = 0; k < 3; ++k) tmp[k] = rho * S.z[k] - S.y[k];
      double xa, za[3], lo_[3], hi_[3];
      C.admm_linear(tmp, sg, S.x, alpha, xa, za, lo_, hi_);
      S.x = xa + oma * S.x;
#pragma unroll
      for (int k = 0; k < 3; ++k) {
        const double v = za[k] + oma * S.z[k];
        const double vv = v + S.y[k] * ir;
        const double d = vv - min_nc(max_nc(vv, lo_[k]), hi_[k]);
        S.z[k] = vv - pb[k] * d;
        S.y[k] = rpb[k] * d;
      }
      C.T.end(2);
      if (it % p.check_termination == 0 || it == p.max_iter) {
        C.T.begin();
        const double x = S.x;
        double Ax[3];
        C.Cmul(x, Ax);
        double mx[8] = {0, 0, 0, 0, 0, 0, 0, 0};  // pr nprim spr snprim du ndual sdu sndual
#pragma unroll
        for (int k = 0; k < 3; ++k) {
          if (C.EE(k) > 0.0) {
            const double ie = 1.0 / C.EE(k);
            mx[0] = fmax(mx[0], fabs((Ax[k] - S.z[k]) * ie));
            mx[1] = fmax(mx[1], fmax(fabs(Ax[k] * ie), fabs(S.z[k] * ie)));
            mx[2] = fmax(mx[2], fabs(Ax[k] - S.z[k]));
            mx[3] = fmax(mx[3], fmax(fabs(Ax[k]), fabs(S.z[k])));
          }
        }
        const double Px = C.Pmul(x);
        const double Aty = C.CTmul(S.y);
        if (act) {
          const double id = 1.0 / C.D;
          const double rd = Px + C.qv + Aty;
          mx[4] = fabs(rd * id);
          mx[5] = fmax(fmax(fabs(Px * id), fabs(Aty * id)), fabs(C.qv * id));
          mx[6] = fabs(rd);
          mx[7] = fmax(fmax(fabs(Px), fabs(Aty)), fabs(C.qv));
        }
        if (!C.V)
#pragma unroll
          for (int k = 0; k < 8; ++k) mx[k] = 0.0;
        const bool nonfin = C.V && (!isfinite(x) || !isfinite(S.z[0] + S.z[1] + S.z[2]) ||
                                    !isfinite(S.y[0] + S.y[1] + S.y[2]));
        C.template reduce<8, true>(mx);
        const bool nf = C.bany(nonfin);
        double pr = mx[0], nprim = mx[1], spr = mx[2], snprim = mx[3];
        double du = mx[4], ndual = mx[5], sdu = mx[6], sndual = mx[7];
        const double ic = 1.0 / C.cscale;
        du *= ic;
        const double ep = p.eps_abs + p.eps_rel * nprim;
        const double ed = p.eps_abs + p.eps_rel * ndual * ic;
        C.T.end(3);
        if (nf || !isfinite(pr) || !isfinite(du)) {
          ev = kMidBad;
          done = true;
          break;
        }
        if (pr <= ep && du <= ed) {
          ev = kMidConverged;
          done = true;
          break;
        }
        if (it == p.max_iter && pr <= 10.0 * p.eps_abs + 10.0 * p.eps_rel * nprim &&
            du <= 10.0 * p.eps_abs + 10.0 * p.eps_rel * ndual * ic)
          ev = kMidApprox;
        bool rc = false;
        double rn = rho;
        if (p.adaptive_rho && it % p.adaptive_rho_interval == 0) {
          const double pn = spr / (snprim + kDivTol);
          const double dn = sdu / (sndual + kDivTol);
          rn = rho * sqrt(pn / (dn + kDivTol));
          rn = fmin(fmax(rn, kRhoMin), kRhoMax);
          rc = rn > rho * p.adaptive_rho_tolerance || rn < rho / p.adaptive_rho_tolerance;
        }
        const bool near = p.polish_near > 0.0 && it >= 2 * p.check_termination &&
                          fmax(pr / ep, du / ed) < p.polish_near;
        if (early && (it >= p.polish_from || near) && it < p.max_iter) {
          S.rho_change = rc;
          S.rho_next = rn;
          ev = kMidAttempt;
          done = true;
          break;
        }
        if (rc) {
          S.rho = rn;
          S.need_fact = true;
        }
      }
    }
  }
  return ev;
}

// ------------------------------------------------------------------ status + outputs
template <int NT>
__device__ __forceinline__ void mid_finish(const mpcqp_params& p, int b, Mid<NT>& C, double x, double x_admm,
                                           int admm_flag, bool do_polish, bool pol_ok, bool bad, int admm_it,
                                           int nfact, int pol_it, int n_ls, double* __restrict__ u0o,
                                           double* __restrict__ Xo, double* __restrict__ Uo,
                                           int32_t* __restrict__ statuso, int32_t* __restrict__ iterso,
                                           uint8_t* __restrict__ activeo) {
  MidLds<NT>& sm = *C.sm;
  const int N = C.N, n = C.n, i = C.i;
  const bool use_admm = p.method == MPCQP_METHOD_ADMM;
  const bool approx = admm_flag == kMidApprox;
  const bool admm_ok = admm_flag == kMidConverged;
  if (C.bany(C.V && C.act && !isfinite(x))) bad = true;
  int status;
  if (bad) {
    status = MPCQP_NUMERICAL_ERROR;
  } else if (pol_ok) {
    status = MPCQP_SOLVED;
  } else if (use_admm) {
    if (do_polish) x = x_admm;
    status = admm_ok ? (do_polish ? MPCQP_SOLVED_INACCURATE : MPCQP_SOLVED)
                     : (approx ? MPCQP_SOLVED_INACCURATE : MPCQP_MAX_ITER_REACHED);
  } else {
    status = MPCQP_MAX_ITER_REACHED;
  }
  // W (speeds / steering, unscaled) to LDS; U by the variable's own thread
  const double* mdl = sm.model;
  const double x03 = mdl[11 * N + 7];
  if (C.V) sm.W[i] = C.act ? C.D * x : 0.0;
  mid_barrier();
  const int cc = i & 1;
  if (C.V && C.act) {
    const double W = sm.W[i];
    const double U = cc == 1 ? W : (W - (i == 0 ? x03 : sm.W[i - 2])) / p.dt;
    if (Uo) Uo[(size_t)b * n + cc * N + (i >> 1)] = U;
    if (u0o && i < 2) u0o[(size_t)b * 2 + i] = U;
    if (activeo) {
      uint8_t* ab = activeo + (size_t)b * (5 * N + 1);
      ab[N + 1 + i] = U > p.u_bounds[2 * cc + 1] ? 2 : (U < p.u_bounds[2 * cc] ? 1 : 0);
      double Um2;
      if (i < 2) {
        Um2 = cc ? mdl[11 * N + 9] : mdl[11 * N + 8];
      } else {
        const double Wm = sm.W[i - 2];
        Um2 = cc == 1 ? Wm : (Wm - (i - 2 == 0 ? x03 : sm.W[i - 4])) / p.dt;
      }
      const double d = U - Um2;
      ab[3 * N + 1 + i] = d > p.du_bounds[2 * cc + 1] ? 2 : (d < p.du_bounds[2 * cc] ? 1 : 0);
    }
  }
  // states on wave 0 (lanes 0..min(N, 63)): lane k <- (psi_k, v_k), positions by the LTV recursion; at
  // N = 64 the last state row (k = 64) is written from lane 63's inclusive sums (below)
  if (threadIdx.x < kWave) {
    const int k = threadIdx.x;
    const double x00 = mdl[11 * N + 4], x01 = mdl[11 * N + 5], x02 = mdl[11 * N + 6];
    double m_al = 0.0, m_be = 0.0, m_ga = 0.0, m_et = 0.0, m_si = 0.0, m_c0 = 0.0, m_c1 = 0.0, dl = 0.0;
    if (k < N) {
      m_al = mdl[k];
      m_be = mdl[N + k];
      m_ga = mdl[2 * N + k];
      m_et = mdl[3 * N + k];
      m_si = mdl[4 * N + k];
      m_c0 = mdl[5 * N + k];
      m_c1 = mdl[6 * N + k];
      dl = sm.W[2 * k + 1];  // delta_k
    }
    // psi_{k+1} = x02 + sum_{j <= k} si_j delta_j (the one-wave kernel's scan over the steering lanes)
    const double sacc = scan_add(k < N ? m_si * dl : 0.0, k);
    // the shift with every lane active (pinned: sunk into the k != 0 branch, lane 0 would read as 0)
    double psh = dpp<kWaveShr1>(sacc);
    asm volatile("" : "+v"(psh));
    const double pk = k == 0 ? x02 : x02 + psh;
    const double vk = k == 0 ? x03 : (k <= N ? sm.W[2 * (k - 1)] : 0.0);
    double t0 = 0.0, t1 = 0.0;
    if (k < N) {
      t0 = m_al * pk + m_be * vk + m_c0;
      t1 = m_ga * pk + m_et * vk + m_c1;
    }
    const double in0 = scan_add(t0, k), in1 = scan_add(t1, k);
    const double ex0 = dpp<kWaveShr1>(in0), ex1 = dpp<kWaveShr1>(in1);
    const double Xk0 = x00 + ex0, Xk1 = x01 + ex1;
    if (Xo && k <= N) {
      double* Xb = Xo + (size_t)b * 4 * (N + 1);
      Xb[0 * (N + 1) + k] = Xk0;
      Xb[1 * (N + 1) + k] = Xk1;
      Xb[2 * (N + 1) + k] = pk;
      Xb[3 * (N + 1) + k] = vk;
    }
    if (activeo && k <= N)
      activeo[(size_t)b * (5 * N + 1) + k] = vk > p.v_bounds[1] ? 2 : (vk < p.v_bounds[0] ? 1 : 0);
    // N = 64: the window has N + 1 = 65 states, one past the wave; state 64 is lane 63's inclusive sums
    // (psi_64 = x02 + sum_{j < 64} si_j delta_j, X_64 = x0 + sum_{j < 64} t_j) with v_64 = W[126]
    if (N + 1 > kWave && k == kWave - 1) {
      const double p64 = x02 + sacc, v64 = sm.W[2 * (kWave - 1)];
      if (Xo) {
        double* Xb = Xo + (size_t)b * 4 * (N + 1);
        Xb[0 * (N + 1) + kWave] = x00 + in0;
        Xb[1 * (N + 1) + kWave] = x01 + in1;
        Xb[2 * (N + 1) + kWave] = p64;
        Xb[3 * (N + 1) + kWave] = v64;
      }
      if (activeo)
        activeo[(size_t)b * (5 * N + 1) + kWave] = v64 > p.v_bounds[1] ? 2 : (v64 < p.v_bounds[0] ? 1 : 0);
    }
    if (k == 0) {
      statuso[b] = status;
      if (iterso) {
        iterso[4 * (size_t)b + 0] = admm_it;
        iterso[4 * (size_t)b + 1] = pol_it;
        iterso[4 * (size_t)b + 2] = nfact;
        iterso[4 * (size_t)b + 3] = n_ls;
      }
    }
  }
}

// ------------------------------------------------------------------ the kernel
template <int NT>
__global__ __launch_bounds__(MidShape<NT>::kThreads, kMidWaves) void k_solve_mid(
    mpcqp_params p, int B, const uint8_t* __restrict__ mask, const double* __restrict__ model,
    double* __restrict__ work, double* __restrict__ u0o, double* __restrict__ Xo, double* __restrict__ Uo,
    int32_t* __restrict__ statuso, int32_t* __restrict__ iterso, uint8_t* __restrict__ activeo) {
  using S = MidShape<NT>;
  __shared__ MidLds<NT> sm;
  const int b = blockIdx.x;
  if (b >= B || (mask && !mask[b])) return;
  const int tid = threadIdx.x;
  Mid<NT> C;
  C.sm = &sm;
  C.Pg = work + (size_t)b * (S::NP * kMidLD);
  C.lane = tid & (kWave - 1);
  C.w = tid / kWave;
  C.h = C.w / S::kRW;
  C.i = (C.w % S::kRW) * kWave + C.lane;
  C.N = p.horizon;
  C.n = 2 * p.horizon;
  C.V = C.h == 0;
  C.act = C.i < C.n;
  C.even = C.act && ((C.i & 1) == 0);
  C.xs = 0;
  C.rs = 0;
  C.dt = p.dt;
  C.n_full = C.n_r1 = 0;
  // the exchange buffers' guard entries (rows -4..-1 and past the end) read as zeros
  for (int e = tid; e < 2 * 5 * 8; e += S::kThreads) {
    const int slot = e / 40, q = (e / 8) % 5, k = e % 8;
    sm.ex[slot][q][k < 4 ? k : S::kNX + k] = 0.0;
  }
  if (tid < 8) sm.abx[tid >> 2][S::kNX + (tid & 3)] = 0.0;  // read as the rows past the end
  const int N = p.horizon;
  const double* mb = model + (size_t)b * model_stride(N);
  for (int e = tid; e < model_stride(N); e += S::kThreads) sm.model[e] = mb[e];
  mid_barrier();
  MidStamps TQ;
  TQ.begin();
  C.T.begin();
  bool bad = mid_setup<NT>(p, C);
  C.T.end(0);
  const bool use_admm = p.method == MPCQP_METHOD_ADMM;
  MidAdmm A;
  A.x = 0.0;
#pragma unroll
  for (int k = 0; k < 3; ++k) A.z[k] = A.y[k] = 0.0;
  A.rho = A.rho_next = p.rho;
  A.it = 0;
  A.nfact = 0;
  A.need_fact = true;
  A.rho_change = false;
  int flag = bad ? kMidBad : kMidMaxIter, pol_it = 0, n_ls = 0;
  double x = 0.0, x_admm = 0.0;
  bool do_polish = false, pol_ok = false;
  while (!bad) {
    int kind = 0;
    double zg[3];
    if (use_admm) {
      const int ev = mid_admm<NT>(p, C, A);
      if (ev == kMidAttempt) {
        kind = 1;
      } else {
        flag = ev;
        x = x_admm = C.V && C.act ? A.x : 0.0;
        do_polish = p.polish != 0 && flag == kMidConverged;
        kind = do_polish ? 2 : 0;
        bad = flag == kMidBad;
      }
#pragma unroll
      for (int k = 0; k < 3; ++k) zg[k] = A.z[k];
    } else {
      do_polish = true;
      kind = 2;
      C.Cmul(x, zg);
    }
    if (kind == 0) break;
    double xp = kind == 1 ? A.x : x;
    MidStamps TP;
    TP.begin();
    const int r_ = mid_polish<NT>(C, xp, zg, kind == 1 ? p.polish_attempt_max_iter : p.polish_max_iter, pol_it,
                                  A.nfact, n_ls);
    TP.end(0);
#ifdef MPCQP_MID_STAMPS
    C.T.acc[5] += TP.acc[0];
#endif
    if (kind == 2) {
      x = xp;
      bad = r_ < 0;
      pol_ok = r_ > 0;
      break;
    }
    if (r_ != 0) {
      flag = r_ > 0 ? 2 : kMidBad;
      bad = r_ < 0;
      pol_ok = r_ > 0;
      x = x_admm = C.V && C.act ? (pol_ok ? xp : A.x) : 0.0;
      break;
    }
    A.need_fact = true;
    if (A.rho_change) A.rho = A.rho_next;
    A.rho_change = false;
  }
  C.T.begin();
  mid_finish<NT>(p, b, C, x, x_admm, flag, do_polish, pol_ok, bad, A.it, A.nfact, pol_it, n_ls, u0o, Xo, Uo,
                 statuso, iterso, activeo);
  C.T.end(6);
  TQ.end(0);
#ifdef MPCQP_MID_STAMPS
  C.T.acc[7] += TQ.acc[0];
#endif
  C.T.flush();
}

}  // namespace

namespace mpcqp {
template <int NT>
void launch_solve_mid(hipStream_t s, const Launch& L) {
  hipLaunchKernelGGL(k_solve_mid<NT>, dim3(L.B), dim3(MidShape<NT>::kThreads), 0, s, *L.p, L.B, L.mask, L.model,
                     L.state, L.u0, L.X, L.U, L.st, L.it, L.ac);
}
// one bucket per object (parallel build): -DMPCQP_MID_PART=NT
#ifndef MPCQP_MID_PART
#error "define MPCQP_MID_PART (the bucket NT of this object)"
#endif
template void launch_solve_mid<MPCQP_MID_PART>(hipStream_t, const Launch&);
}  // namespace mpcqp

#ifdef MPCQP_MID_STAMPS
#define MPCQP_CAT2(a, b) a##b
#define MPCQP_CAT(a, b) MPCQP_CAT2(a, b)
extern "C" int MPCQP_CAT(mpcqp_debug_mid_stamps_, MPCQP_MID_PART)(unsigned long long* out, int reset) {
  hipError_t e = hipDeviceSynchronize();
  if (e == hipSuccess && out) e = hipMemcpyFromSymbol(out, HIP_SYMBOL(g_mid_stamps), sizeof(unsigned long long) * kMidStampSlots);
  if (e == hipSuccess && reset) {
    unsigned long long z[kMidStampSlots] = {0};
    e = hipMemcpyToSymbol(HIP_SYMBOL(g_mid_stamps), z, sizeof(z));
  }
  return e == hipSuccess ? 0 : -4;
}
#endif
