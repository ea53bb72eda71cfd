// mpcqp_solve.h -- K2 solver kernel (setup -> ADMM -> polish), templated on the horizon N.
#pragma once
#include "mpcqp_build.h"

namespace {
using mpcqp::Launch;

// The model block stays in LDS for the outputs (finish_qp) while Pbar is live, where that costs no
// occupancy (8 workgroups of Pbar + model fit a CU's 160 KB of LDS: N <= 23); past that, the model shares
// the setup's union with Pbar and the outputs re-derive it (K1 fused) or re-read it (workspace).
// Pbar storage.  N <= 23: row-major n x (n + 1) (column n: zero padding), lane `col` reads column
// col (conflict-free).  N >= 24: the lower triangle packed (row a, column b <= a at a (a + 1) / 2 + b)
// for 64 rows, rows n..63 zero: 16.6 KB instead of 32 N^2 bytes, so eight workgroups fit a CU's LDS
// (the full matrix allowed 7 at N = 24, 5 from N = 28 on) and the kernel runs 2 waves per SIMD (Pbar is read only by form() and Pmul: a factorization or a
// residual check, not per ADMM iteration).
template <int N>
constexpr bool kPackedP = N >= 24;

template <int N, bool Packed = kPackedP<N>>
struct SolveSmem {
  static constexpr int n = 2 * N;
  static constexpr int kPS = n + 1;  // row stride: column n is a zero padding column
  double pad0[4];     // zeros: form()'s band writes of the first rows land here when out of range
  double P[n * kPS];  // Pbar, row-major (lane `col` reads column col: conflict-free; lanes >= n read the zeros of column n)
  double pad1[4];     // zeros: ... and those of the last rows
  double band[5][n];  // Pbar's entries at form()'s band addresses (lane p: (p, p + d - 2)), restored after each form
};
template <int N>
struct SolveSmem<N, true> {
  static constexpr int n = 2 * N;
  static constexpr int kPS = 0;  // unused
  double P[kWave * (kWave + 1) / 2];  // lower triangle, packed by rows; rows >= n zero
  double band[3][n];                  // Pbar's entries (p, p - 2), (p, p - 1), (p, p) (form() adds there)
};
// packed index of (i, j), i / j any order
__device__ __forceinline__ int tri_idx(int i, int j) { return i >= j ? (i * (i + 1)) / 2 + j : (j * (j + 1)) / 2 + i; }
// a variable lane's position in the reference-facing order W = (v_1, delta_0, v_2, delta_1, ...) (the
// solver keeps the speeds in lanes 0..N-1 and the steering angles in lanes N..2N-1; Ctx); lanes past
// the variables map to themselves
template <int N>
__device__ __forceinline__ int interleaved(int p) {
  return p < N ? 2 * p : (p < 2 * N ? 2 * (p - N) + 1 : p);
}

// the whole-wave kernels' pivot-column buffers of the sweep (Ctx::sweep): 1 KB per wave
constexpr int kColBytes = 2 * kWave * 8;
template <int N>
constexpr bool kModelKept =
    8 * ((int)sizeof(SolveSmem<N>) + kColBytes) + 64 * model_stride(N) <= 163840;

template <int N>
struct SetupSmem {
  static constexpr int n = 2 * N;
  double buf[kWave];
  double model[kModelKept<N> ? 1 : model_stride(N)];
  double pre[4][N + 1];  // prefix sums of alpha, beta, gamma, eta
  double err[4][N + 1];  // free-response tracking error e_m = sx_m - r_m, component-major
  double g[n];
  // the input-cost band of H by row offset d = i - col in [-(n - 1), n - 1] (index d + n - 1), for the
  // four kinds of column: speed, steering, the last speed (its a_k has no successor), none (zeros)
  static constexpr int kBT = 2 * n - 1;
  double bt[4][kBT];
};

template <int N, bool Pair = false>
struct SolveLds {
  union {
    SetupSmem<N> setup;
    SolveSmem<N> solve;  // setup_qp writes Pbar when its own LDS data is dead
  };
  double model[kModelKept<N> ? model_stride(N) : 1];  // the model block, live to the end (kModelKept)
  // the sweep's pivot columns, double buffered (Ctx::sweep; the pair layout keeps register
  // broadcasts and allocates none: its 16 QPs per CU need every KB of the LDS)
  double col[Pair ? 1 : 2 * kWave];
  __device__ double* model_ptr() { return kModelKept<N> ? model : setup.model; }
};

// ------------------------------------------------------------------ shared solver context
// Per-lane view of one scaled QP plus the structured operators and the KKT inverse.
// Variables W = (v_1, ..., v_N, delta_0, ..., delta_{N-1}) in two blocks: lane j < N holds the speed
// v_{j+1}, lane N + j the steering delta_j (interleaved<N>() gives a lane's position in the
// reference-facing order v_1, delta_0, v_2, delta_1, ...).  The rows owned by lane p (slot 0: v row,
// speed lanes; slot 1: input row; slot 2: rate row) are banded in those variables:
//   slot 0  c0 x_p                                      (v_{p+1}: identity)
//   slot 1  c10 x_p + c11 x_{p-1}                       (a_j = (v_{j+1} - v_j)/dt; delta_j)
//   slot 2  c20 x_p + c21 x_{p-1} + c22 x_{p-2}         (a_j - a_{j-1}; delta_j - delta_{j-1})
// with c = (row scaling E x row coefficient) x the column scaling D of the variable it multiplies:
// the scaled operator Cbar = E C D with D folded into the coefficients.  "The same input one step
// back" is one lane back, so the banded operators move values by one and two lanes (a 64-bit DPP
// move per lane step); the coefficients that would reach across the block boundary (c11, c21, c22
// of a block's first lanes) are exact zeros, so what a shift carries across it is multiplied away.
template <int N, bool Pair = false>
struct Ctx {
  using LN = Lanes<Pair>;
  static constexpr int n = 2 * N;
  int lane;
  bool act, even;
  double dt;
  double D, qv;
  double E[3], lo[3], hi[3], wb[3];
  double c0, c10, c11, c20, c21, c22;  // Cbar's coefficients (see above)
  double cscale;
  static constexpr int kPS = SolveSmem<N>::kPS;  // Pbar row stride
  double* __restrict__ P;  // Pbar (LDS, row-major n x n, row stride kPS)
  double* __restrict__ colb;  // SolveLds::col: the sweep's pivot-column broadcast buffers
  const double* __restrict__ band;  // SolveSmem::band
  static constexpr int kNW = (n + 15) / 16;  // 16-lane rows holding the n variables
  // KKT inverse, row `lane`: A^{-1}[lane][j] = -r[j] (symmetric sweep operator)
  double r[n];
  // work counters (written to the solver state with debug_state; tools/qp_cycles.py)
  int n_full, n_r1;

  // Bind the context to this lane and the solve LDS (Pbar); the problem data fields are
  // filled by setup_qp.
  __device__ __forceinline__ void init(int ln, double dt_, SolveSmem<N>& s) {
    lane = ln;
    band = &s.band[0][0];
    n_full = 0;
    n_r1 = 0;
    act = ln < n;
    even = ln < N;  // the speed block
    dt = dt_;
    P = s.P;
  }

  // Make the per-lane problem data opaque to the optimizer at the top of a solver
  // iteration: otherwise LICM hoists dozens of derived values (reciprocals, products,
  // masks) out of the loops and the kernel drops to one wave per SIMD.
  __device__ __forceinline__ void opaque() {
    asm volatile("" : "+v"(D), "+v"(qv), "+v"(lane));
    asm volatile("" : "+v"(E[0]), "+v"(E[1]), "+v"(E[2]));
    asm volatile("" : "+v"(c0), "+v"(c10), "+v"(c11), "+v"(c20), "+v"(c21), "+v"(c22));
    asm volatile("" : "+v"(lo[0]), "+v"(lo[1]), "+v"(lo[2]));
    asm volatile("" : "+v"(hi[0]), "+v"(hi[1]), "+v"(hi[2]));
    asm volatile("" : "+v"(wb[0]), "+v"(wb[1]), "+v"(wb[2]));
  }

  // Every lane's view of v (one element per lane): w[c] lane l = v[16 c + (l & 15)], read by the
  // fmac_bc products through DPP row_newbcast: bcast() (permlane16/32 swaps + copies, ~12 VALU
  // instructions, ~110 cycles).  Staging through LDS instead (one ds_write + kNW ds_reads, no VALU
  // work) measured slower (+3 % at B = 4096, +9 % at B = 512): its round trip is on every product's
  // critical path.
  __device__ __forceinline__ void vbcast(double v, double w[4]) const { LN::template vbcast<kNW>(v, w); }

  // z = Cbar x: shifts only (no scans)
  __device__ __forceinline__ void Cmul(double x, double z[3]) const {
    const double xm1 = LN::shr1(x);
    const double xm2 = LN::shr1(xm1);
    z[0] = c0 * x;
    z[1] = c10 * x + c11 * xm1;
    z[2] = (c20 * x + c21 * xm1) + c22 * xm2;
  }
  // x = Cbar' y: the terms for the variables 1 and 2 back shifted in one chain, shl1(a + shl1(b))
  __device__ __forceinline__ double CTmul(const double y[3]) const {
    const double a = c11 * y[1] + c21 * y[2];  // to the variable 1 back
    const double b = c22 * y[2];               // to the variable 2 back
    const double t = (c0 * y[0] + c10 * y[1]) + c20 * y[2];
    return t + LN::shl1(a + LN::shl1(b));
  }
  // (Pbar v)_lane, Pbar symmetric: lane reads its row as a conflict-free column of the LDS copy
  // The column loads go out in groups of kPG ahead of their FMAs (the inline-asm FMAs pin each
  // load's register otherwise: one load + lgkmcnt(0) wait per column).
  // Past N = 24 the 9 registers of the look-ahead would spill the inverse: plain loads there.
  static constexpr int kPG = 4;
  __device__ __forceinline__ double Pmul(double v) const {
    double w[4];
    vbcast(act ? v : 0.0, w);
    const int col = act ? lane : n;  // lanes >= n read the zero padding column
    double a[4] = {0.0, 0.0, 0.0, 0.0};
    if constexpr (kPackedP<N>) {  // lanes >= n read their zero rows
      int ln = lane;
      asm volatile("" : "+v"(ln));
      const int Ti = (ln * (ln + 1)) / 2;
      Unroll<0, n>::run([&](auto jc) {
        constexpr int j = decltype(jc)::value;
        fmac_bc<j % 16>(a[j % 4], w[j / 16], P[ln >= j ? Ti + j : (j * (j + 1)) / 2 + ln]);
      });
      return act ? (a[0] + a[1]) + (a[2] + a[3]) : 0.0;
    } else if constexpr (N > 24) {
      Unroll<0, n>::run([&](auto jc) {
        constexpr int j = decltype(jc)::value;
        fmac_bc<j % 16>(a[j % 4], w[j / 16], P[j * kPS + col]);
      });
      return act ? (a[0] + a[1]) + (a[2] + a[3]) : 0.0;
    }
    double cur[kPG], nxt[kPG];
    Unroll<0, kPG>::run([&](auto kc) {
      constexpr int k = decltype(kc)::value;
      cur[k] = k < n ? P[k * kPS + col] : 0.0;
    });
    Unroll<0, (n + kPG - 1) / kPG>::run([&](auto gc) {
      constexpr int g = decltype(gc)::value;
      if constexpr ((g + 1) * kPG < n) {
        Unroll<0, kPG>::run([&](auto kc) {
          constexpr int j = (g + 1) * kPG + decltype(kc)::value;
          nxt[decltype(kc)::value] = j < n ? P[j * kPS + col] : 0.0;
        });
      }
      __builtin_amdgcn_sched_barrier(0);  // the next group's loads stay ahead of this group's FMAs
      Unroll<0, kPG>::run([&](auto kc) {
        constexpr int j = g * kPG + decltype(kc)::value;
        if constexpr (j < n) fmac_bc<j % 16>(a[j % 4], w[j / 16], cur[decltype(kc)::value]);
      });
      Unroll<0, kPG>::run([&](auto kc) { cur[decltype(kc)::value] = nxt[decltype(kc)::value]; });
    });
    return act ? (a[0] + a[1]) + (a[2] + a[3]) : 0.0;
  }
  // KKT matrix A = Pbar + s I + Cbar' diag(rw) Cbar, row `lane` -> r[].  The row part is a
  // band (lanes p-2 .. p+2 of the same block): its five entries per lane come from shifts.
  // From n >= 8 on, each lane adds its five band entries into its own row of Pbar in LDS
  // (read-modify-write), every lane loads its row as a column of the sum, and the lanes write the
  // original entries back: ~10 VALU instructions instead of a compare-and-select per column (the
  // band position j = lane + d is lane dependent, so registers cannot be addressed by it).
  // Entries outside the matrix have band value +-0: their addresses land in the zero padding
  // column, in pad0 / pad1, or (n >= 8) on an entry of a neighbouring row that no lane's band
  // touches, which gets its own value back.
  __device__ __forceinline__ void form(double s, const double rw[3]) {
    // opaque lane copy: keeps per-column masks/addresses from being hoisted out of solver loops
    int ln = lane;
    asm volatile("" : "+v"(ln));
    // row r of lane q (weight rw) adds rw c_i c_j at (q - i, q - j): lane p's diagonal takes its
    // own rows' c_0 terms, lane p+1's c_1 terms and lane p+2's c_2 terms, and so on
    const double a1 = rw[1] * c11, a2 = rw[2] * c21, b2 = rw[2] * c22;
    const double dg = (c0 * c0 * rw[0] + rw[1] * c10 * c10) + rw[2] * c20 * c20;
    const double b0 = (dg + LN::shl1(a1 * c11 + a2 * c21) + LN::shl2(b2 * c22)) + s;
    const double bp1 = LN::shl1(a1 * c10 + a2 * c20) + LN::shl2(b2 * c21);  // entry (p, p+1)
    const double bp2 = LN::shl2(b2 * c20);                                   // entry (p, p+2)
    const double bm1 = LN::shr1(bp1), bm2 = LN::shr2(bp2);  // symmetric: (p, p-1) = lane p-1's (., +1)
    const bool live = ln < n;
    if constexpr (kPackedP<N>) {
      // lower band entries only: lane p adds into (p, p - 2), (p, p - 1), (p, p); the upper ones
      // (p, p + 1), (p, p + 2) are lanes p + 1 / p + 2's (p + 1, p), (p + 2, p) (the same words)
      const int Ti = (ln * (ln + 1)) / 2;
      double* rowp = P + Ti + ln;
      const double* bo = band + ln;
      lds_sync();
      if (live) {
        if (ln >= 2) rowp[-2] = bo[0 * n] + bm2;
        if (ln >= 1) rowp[-1] = bo[1 * n] + bm1;
        rowp[0] = bo[2 * n] + b0;
      }
      lds_sync();
      Unroll<0, n>::run([&](auto jc) {  // lanes >= n read their zero rows
        constexpr int j = decltype(jc)::value;
        r[j] = P[ln >= j ? Ti + j : (j * (j + 1)) / 2 + ln];
      });
      lds_sync();
      int l2 = lane;
      asm volatile("" : "+v"(l2));
      if (l2 < n) {
        double* rp = P + (l2 * (l2 + 1)) / 2 + l2;
        const double* bp = band + l2;
        if (l2 >= 2) rp[-2] = bp[0 * n];
        if (l2 >= 1) rp[-1] = bp[1 * n];
        rp[0] = bp[2 * n];
      }
      lds_sync();
    } else if constexpr (n >= 8) {
      // entry (ln, ln - 2) (positive immediate offsets) and the saved originals, saved by setup_qp
      double* rowp = P + ln * (kPS + 1) - 2;
      const double* bo = band + ln;
      lds_sync();
      if (live) {
        rowp[0] = bo[0 * n] + bm2;
        rowp[1] = bo[1 * n] + bm1;
        rowp[2] = bo[2 * n] + b0;
        rowp[3] = bo[3 * n] + bp1;
        rowp[4] = bo[4 * n] + bp2;
      }
      lds_sync();
      // lanes >= n: the zero padding column, so their rows are exactly zero (from the opaque lane
      // copy: the column addresses are recomputed per form, not hoisted into live registers)
      const int c = live ? ln : n;
      Unroll<0, n>::run([&](auto jc) {
        constexpr int j = decltype(jc)::value;
        r[j] = P[j * kPS + c];
      });
      lds_sync();
      // restore Pbar; the addresses are recomputed from an opaque lane copy, so nothing but r[]
      // stays live across the loads
      int l2 = lane;
      asm volatile("" : "+v"(l2));
      if (l2 < n) {
        double* rp = P + l2 * (kPS + 1) - 2;
        const double* bp = band + l2;
        rp[0] = bp[0 * n];
        rp[1] = bp[1 * n];
        rp[2] = bp[2 * n];
        rp[3] = bp[3 * n];
        rp[4] = bp[4 * n];
      }
      lds_sync();
    } else {
      const int c = live ? ln : 0;
      // every lane loads (lanes >= n read column 0 and discard it): no exec-masked load per column
      Unroll<0, n>::run([&](auto jc) {
        constexpr int j = decltype(jc)::value;
        double t = 0.0;
        if (j == ln) t = b0;
        if (j == ln + 1) t = bp1;
        if (j + 1 == ln) t = bm1;
        if (j == ln + 2) t = bp2;
        if (j + 2 == ln) t = bm2;
        const double pv = P[j * kPS + c];
        r[j] = live ? pv + t : 0.0;
      });
    }
  }
  // Symmetric sweep operator on the rows in r[]: afterwards A^{-1} = -r (row `lane`).
  // Step k: every lane needs its own A[i][k] (register r[k]) and the pivot row A[k][j] =
  // A[j][k] (symmetry) -- the column r[k] of all lanes, read by each 16-lane row from the QP's LDS
  // buffer (the lane's row copy w[c] lane l = A[16c + (l & 15)][k]) and consumed through DPP
  // row_newbcast, so each update r[j] += coef * A[k][j] is one v_fmac_f64_dpp.  The pivot row itself
  // is the same FMA with coef = 1/d - 1 (A[k][j] <- A[k][j] / d), so the update is uniform over
  // lanes.  The step loop is unrolled at compile time (static register indices and DPP lane
  // immediates).  false on a non-positive pivot.
  // The column goes through LDS (one ds_write as soon as the previous step has updated it, kNW reads
  // of the row's values and one uniform read of the pivot; double buffered, the QP's own buffer -- a
  // half's in the pair layout) rather than permlane swaps and readlanes: fourteen VALU instructions
  // per pivot move to the LDS pipe, with a whole step of FMAs to hide the round trip -- 503 -> 442
  // cycles per pivot at two waves per SIMD, 352 -> 345 for a lone wave, the same bits
  // (tools/micro/sweep_bench.hip, profiles/r05_sweep_bench.json).
  // At n <= 32 (kNW <= 2) the register broadcast is a single permlane16 stage (none at n <= 16), and
  // a lone wave (B = 1, the closed loops) would wait out the LDS round trip on every pivot: 5.6k
  // against ~3.6k cycles per N = 10 factorization (profiles/r05_n_stamps/, r05_o_ab_register_sweep_n_le_32.json).  Those sizes
  // and the pair layout keep the register broadcasts (sweep_reg).
  static constexpr bool kRegBcast = Pair || kNW <= 2;
  __device__ __forceinline__ bool sweep() {
    if constexpr (kRegBcast) return sweep_reg();
    bool ok = true;
    int ln = lane;
    asm volatile("" : "+v"(ln));
    const int rl = ln & 15;
    lds_sync();
    colb[ln] = r[0];
    Unroll<0, n>::run([&](auto kc) {
      constexpr int k = decltype(kc)::value;
      const double* bk = colb + (k & 1) * kWave;
      lds_sync();
      double w[4];
      Unroll<0, kNW>::run([&](auto cc) {
        constexpr int c = decltype(cc)::value;
        w[c] = bk[16 * c + rl];
      });
      // the pivot A[k][k]: a vector reciprocal (v_rcp_f64 + two Newton steps, within an ulp of
      // 1/d), no IEEE division sequence on the step's critical path
      const double d = bk[k];
      // DPP reads of a VGPR need two wait states after its write; tie the pad to w
      asm volatile("s_nop 1" : "+v"(w[0]));
      ok = ok && (d > 0.0) && isfinite(d);
      double inv = __builtin_amdgcn_rcp(d);
      inv = fma(inv, fma(-d, inv, 1.0), inv);
      inv = fma(inv, fma(-d, inv, 1.0), inv);
      const bool piv = lane == k;
      const double ck = r[k] * inv;
      const double coef = piv ? inv - 1.0 : -ck;
      // the next pivot column first, published for the next step
      if constexpr (k + 1 < n) {
        fmac_bc<(k + 1) % 16>(r[k + 1], w[(k + 1) / 16], coef);
        colb[((k + 1) & 1) * kWave + ln] = r[k + 1];
      }
      Unroll<0, n>::run([&](auto jc) {
        constexpr int j = decltype(jc)::value;
        if constexpr (j != k && j != k + 1) fmac_bc<j % 16>(r[j], w[j / 16], coef);
      });
      r[k] = piv ? -inv : ck;
    });
    lds_sync();
    return ok;
  }
  // The register-broadcast sweep (n <= 32 and the pair layout): the column by vbcast, the pivot by
  // readlane (whole wave; 1/d is computed while the broadcast is in flight) or from the half's DPP
  // row (pair layout).  Staging through LDS measured 8 % slower in the pair layout (43.8M -> 40.2M
  // QP/s at N = 15, B = 16384, profiles/r05_i_ab.json).
  __device__ __forceinline__ bool sweep_reg() {
    bool ok = true;
    Unroll<0, n>::run([&](auto kc) {
      constexpr int k = decltype(kc)::value;
      double d, w[4];
      if constexpr (Pair) {
        vbcast(r[k], w);
        d = LN::pin(row_bc<k % 16>(w[k / 16]));
      } else {
        d = readlane(r[k], k);
        vbcast(r[k], w);
      }
      ok = ok && (d > 0.0) && isfinite(d);
      double inv = __builtin_amdgcn_rcp(d);
      inv = fma(inv, fma(-d, inv, 1.0), inv);
      inv = fma(inv, fma(-d, inv, 1.0), inv);
      const bool piv = lane == k;
      const double ck = r[k] * inv;
      const double coef = piv ? inv - 1.0 : -ck;
      // next pivot column first: the next step's broadcast depends only on it
      if constexpr (k + 1 < n) fmac_bc<(k + 1) % 16>(r[k + 1], w[(k + 1) / 16], coef);
      Unroll<0, n>::run([&](auto jc) {
        constexpr int j = decltype(jc)::value;
        if constexpr (j != k && j != k + 1) fmac_bc<j % 16>(r[j], w[j / 16], coef);
      });
      r[k] = piv ? -inv : ck;
    });
    return ok;
  }
  // Rank-1 change of the factorized matrix, A' = A + delta c c' with c the row (tau, l) of
  // Cbar (Sherman-Morrison): A'^{-1} = A^{-1} - kappa u u', u = A^{-1} c,
  // kappa = delta / (1 + delta c'u).  Used by the polish when a few soft rows enter or leave
  // the active set.  false (inverse untouched) when 1 + delta c'u is not safely positive.
  __device__ __forceinline__ bool rank1(int tau, int l, double delta) {
    const int lu = LN::uniform(l);
    // the row's coefficients on the variables lu, lu-1, lu-2 (lane lu's c; zero where they would
    // reach into the other block)
    const double k0 = LN::readv(tau == 0 ? c0 : (tau == 1 ? c10 : c20), lu);
    const double k1 = lu >= 1 ? LN::readv(tau == 1 ? c11 : (tau == 2 ? c21 : 0.0), lu) : 0.0;
    const double k2 = lu >= 2 ? LN::readv(tau == 2 ? c22 : 0.0, lu) : 0.0;
    // u = A^{-1} c: c has at most three entries, so u is three columns of the inverse -- by
    // symmetry the lane's own registers r[lu], r[lu-1], r[lu-2] (A^{-1}[i][j] = -r_i[j])
    double u = k0 * pick<0, n>(lu);
    MPCQP_MARK("pol.rank1");
    if (lu >= 1) u += k1 * pick<0, n>(lu - 1);
    MPCQP_MARK("pol.rank1");
    if (lu >= 2) u += k2 * pick<0, n>(lu - 2);
    MPCQP_MARK("pol.rank1");
    u = act ? -u : 0.0;
    // u through LDS (the sweep's buffer), as the sweep broadcasts its pivot columns: the three entries
    // of c'u by uniform reads, the rows for the update by the lanes (the pair layout: lane reads and
    // its one-stage register broadcast, as its sweep)
    double w[4], cu;
    if constexpr (kRegBcast) {
      cu = (k0 * LN::readv(u, lu) + k1 * LN::readv(u, lu >= 1 ? lu - 1 : 0)) + k2 * LN::readv(u, lu >= 2 ? lu - 2 : 0);
    } else {
      int ln = lane;
      asm volatile("" : "+v"(ln));
      lds_sync();
      colb[ln] = u;
      lds_sync();
      cu = (k0 * colb[lu] + k1 * colb[lu >= 1 ? lu - 1 : 0]) + k2 * colb[lu >= 2 ? lu - 2 : 0];
      Unroll<0, kNW>::run([&](auto cc) {
        constexpr int c = decltype(cc)::value;
        w[c] = colb[16 * c + (ln & 15)];
      });
      asm volatile("s_nop 1" : "+v"(w[0]));
    }
    const double den = 1.0 + delta * cu;
    if (!(den > kRank1Min) || !isfinite(den)) return false;
    const double m = (delta / den) * u;
    if constexpr (kRegBcast) vbcast(u, w);
    Unroll<0, n>::run([&](auto jc) {
      constexpr int j = decltype(jc)::value;
      fmac_bc<j % 16>(r[j], w[j / 16], m);
    });
    return true;
  }
  // r[j] of this lane for a wave-uniform j: uniform branches down to pairs of registers, one
  // select in the pair.  The asm pins each pair's value: merged through a phi as one load of a
  // variable address, the inverse row would be demoted to scratch memory.
  template <int LO, int HI>
  __device__ __forceinline__ double pick(int j) const {
    if constexpr (HI - LO <= 2) {
      MPCQP_MARK("pol.pick_leaf");
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
  // (A^{-1} v)_lane
  // The products read lanes 0..n-1 only, and the rows of lanes >= n are exactly zero (form()
  // writes zeros there and every update of them multiplies by a zero), so those lanes return zero
  // by themselves as long as what they read is finite.
  __device__ __forceinline__ double inv_mul(double v) const {
    double w[4];
    // whole wave at n <= 32: rows 2-3 read their own lanes' v (bcast_rows01), zeroed here
    if constexpr (!Pair && kNW <= 2)
      vbcast(act ? v : 0.0, w);
    else
      vbcast(v, w);
    // three chains: a dependent f64 FMA's latency (~9 cycles) is under two issue slots (~5.5 each),
    // and a DPP FMA that reads an accumulator written two instructions earlier needs a wait state
    // (two chains: an s_nop per pair; three chains none): config 2 +1.9 %, the config-4 shard +1.0 %,
    // B=1 +1.1 % over two chains, config 3 level (profiles/r05_t_ab_three_chain_invmul.json)
    double a[3] = {0.0, 0.0, 0.0};
    Unroll<0, n>::run([&](auto jc) {
      constexpr int j = decltype(jc)::value;
      fmac_bc<j % 16>(a[j % 3], w[j / 16], r[j]);
    });
    return -((a[0] + a[1]) + a[2]);
  }
};

// ------------------------------------------------------------------ a QP's raw inputs
// Where the fused K1 (setup_qp) and the outputs (finish_qp) read a QP's window, x0 and u_prev:
// BatchWin = the caller's batch buffers (mpcqp_build / mpcqp_solve: the pointer arguments of
// setup_qp / finish_qp, in_ref == nullptr when K1 ran as its own kernel), FleetWin = one vehicle of
// the fused closed loop.
struct BatchWin {
  static constexpr bool kFleet = false;
  __device__ __forceinline__ int lane() const { return threadIdx.x; }
};
// FleetWin: one vehicle of the fused closed loop (k_fleet_loop): window row k = the vehicle's
// reference row min(path_idx + k, len - 1) (control_stage.py:101-105), speed x 0.6 in the relaxed
// retry (:48-49); x0 / u_prev are the loop state.  The same gather as k_fleet_build.
struct FleetWin {
  static constexpr bool kFleet = true;
  const double* __restrict__ rows;
  int ln;  // the lane index, opaque per solve (k_fleet_loop)
  int len, pidx;
  bool relax;
  double x[4], u[2];
  template <int N>
  __device__ __forceinline__ void row(int k, double& rx, double& ry, double& ryaw, double& rv) const {
    const double* r = rows + (size_t)min(pidx + k, len - 1) * 4;
    rx = r[0];
    ry = r[1];
    ryaw = r[2];
    rv = relax ? r[3] * 0.6 : r[3];
  }
  __device__ __forceinline__ double x0l(int lane) const {
    return lane == 0 ? x[0] : (lane == 1 ? x[1] : (lane == 2 ? x[2] : (lane == 3 ? x[3] : 0.0)));
  }
  __device__ __forceinline__ double upl(int lane) const { return lane == 4 ? u[0] : (lane == 5 ? u[1] : 0.0); }
  __device__ __forceinline__ int lane() const { return ln; }
  __device__ __forceinline__ double x0v(int i) const { return x[i]; }
  __device__ __forceinline__ double upv(int i) const { return u[i]; }
};

// ServeWin: the B = 1 server (k_serve): the caller's buffers like BatchWin, with the lane index made
// opaque per solve (otherwise LICM hoists every lane-derived value of the solver out of the serve loop
// and holds it across requests).
struct ServeWin {
  static constexpr bool kFleet = false;
  int ln;
  __device__ __forceinline__ int lane() const { return ln; }
};

// ------------------------------------------------------------------ K2 phase 1: setup
// Condensing (states and slacks eliminated) + OSQP Ruiz/cost scaling.  Leaves the scaled
// problem on chip for the later phases: Pbar (symmetric, row-major) in the solve LDS, the
// per-lane data in C.  Returns true on non-finite problem data.  dbg (debug_state builds of
// the parameter block only) receives the solver state for inspection.
// Variables W = (v_1, delta_0, v_2, delta_1, ...) (a_k = (v_{k+1} - v_k)/dt: a bijective affine
// change of the reference's U, same optimum).  Row slots owned by lane p (p < n = 2N):
//   slot 0: v row (speed lanes p < N): v_{p+1}                         (mpc_controller.py:81-82,115-116)
//   slot 1: input row        a_k or delta_k (k = p mod N)              (:83-86)
//   slot 2: rate row         U_k - U_{k-1} (u_prev at k = 0)           (:89-106)
// the constant parts (v_0 = x0[3], u_prev) moved into the bounds.
template <int N, class Win, bool Pair = false>
__device__ __forceinline__ bool setup_qp(const mpcqp_params& p, int b, const double* __restrict__ model,
                                         const double* __restrict__ in_x0, const double* __restrict__ in_ref,
                                         const double* __restrict__ in_up, const Win& win, Ctx<N, Pair>& C,
                                         SolveLds<N, Pair>& lds, double* __restrict__ scratch, double* __restrict__ dbg) {
  using LN = Lanes<Pair>;
  constexpr int n = 2 * N;
  SetupSmem<N>& sm = lds.setup;
  (void)scratch;
  constexpr int S = model_stride(N);
  const int lane = win.lane();
  const bool act = lane < n;
  const bool even = act && lane < N;  // the speed block
  const int cc = lane >= N ? 1 : 0;   // 0 = acceleration (speed variable), 1 = steering
  const int kv = lane - cc * N;       // the step k of the lane's variable (v_{k+1} or delta_k)
  const double dt = p.dt;
  Stamps T, T2;
  T2.begin();
  T.begin();
  MPCQP_MARK("setup.k1");

  if constexpr (Win::kFleet) {  // the fleet loop: the vehicle's window -> LTV model into LDS
    double rx = 0.0, ry = 0.0, ryaw = 0.0, rv = 0.0;
    if (lane <= N) win.template row<N>(lane, rx, ry, ryaw, rv);
    build_qp<Pair>(p, lane, rx, ry, ryaw, rv, win.x0l(lane), win.upl(lane), lds.model_ptr());
  } else if (in_ref) {  // K1 fused: the window -> LTV model straight into LDS (mpcqp_build.h)
    const double* rb = in_ref + (size_t)b * (N + 1) * 4;
    double rx = 0.0, ry = 0.0, ryaw = 0.0, rv = 0.0;
    if (lane <= N) {
      rx = rb[4 * lane + 0];
      ry = rb[4 * lane + 1];
      ryaw = rb[4 * lane + 2];
      rv = rb[4 * lane + 3];
    }
    const double x0l = lane < 4 ? in_x0[(size_t)b * 4 + lane] : 0.0;
    const double upl = (lane >= 4 && lane < 6 && in_up) ? in_up[(size_t)b * 2 + lane - 4] : 0.0;
    build_qp<Pair>(p, lane, rx, ry, ryaw, rv, x0l, upl, lds.model_ptr());
  } else {
    const double* mb = model + (size_t)b * S;
    double* md = lds.model_ptr();
    for (int i = lane; i < S; i += LN::kLanes) md[i] = mb[i];
  }
  __syncthreads();
  const double* mdl = lds.model_ptr();
  const double* al = mdl;
  const double* be = mdl + N;
  const double* ga = mdl + 2 * N;
  const double* et = mdl + 3 * N;
  const double* si = mdl + 4 * N;
  const double* c0 = mdl + 5 * N;
  const double* c1 = mdl + 6 * N;
  const double* rr = mdl + 7 * N;
  const double* x0 = mdl + 11 * N + 4;
  const double* up = mdl + 11 * N + 8;

  // the band table of the input cost (condensing below adds row i of its column's kind at offset
  // i - lane): the same values the reference's R term puts on H's band
  if constexpr (n < kWave) {
    constexpr int kBT = SetupSmem<N>::kBT;
    const double r00 = 0.5 * (p.r[0] + p.r[0]) / (dt * dt), r10 = 0.5 * (p.r[2] + p.r[1]) / dt;
    const double r11 = 0.5 * (p.r[3] + p.r[3]);
    for (int e = lane; e < 4 * kBT; e += LN::kLanes) {
      const int kind = e / kBT, d = e % kBT - (n - 1);
      double v = 0.0;
      // column v_{j+1} (lane j): rows v_j, v_{j+1}, v_{j+2} at d = -1, 0, 1, delta_j at N, delta_{j+1}
      // at N + 1; column delta_j (lane N + j): rows v_{j+1} at -N, v_j at -N - 1.  The last speed
      // (kind 2) has no a_{j+1}: no v_{j+2} row (d = 1 would be delta_0) and no delta_{j+1} row.
      if (kind == 0 || kind == 2) {  // speed column (kind 2: the last one)
        if (d == 0) v = kind == 0 ? 2.0 * r00 : r00;
        if (d == -1 || (d == 1 && kind == 0)) v = -r00;
        if (d == N) v = r10;
        if (d == N + 1 && kind == 0) v = -r10;
      } else if (kind == 1) {  // steering column
        if (d == 0) v = r11;
        if (d == -N) v = r10;
        if (d == -N - 1) v = -r10;
      }
      (&sm.bt[0][0])[e] = v;
    }
  }
  // prefix sums (lanes 0..3, one array each) and free response (lane 4)
  MPCQP_MARK("setup.prefix");
  // ONE sequential recurrence on four lanes (one instruction stream): lanes 0 / 1 the prefix sums of
  // alpha / gamma (pre[0] / pre[2]), lanes 2 / 3 the free response's x / y (W = 0: v_k = 0 for k >= 1,
  // constant heading), acc <- acc + A[k] h + B[k] v_k + C[k] with (A, h, B, v, C) = (alpha | gamma, 1,
  // -, 0, 0) on the prefix lanes -- exactly acc + A[k] (A * 1 and the zero terms are exact) -- and
  // (alpha | gamma, psi, beta | eta, v_k, c0 | c1) on the free-response lanes, the reference's own
  // expression.  The heading and speed rows of e_m are lane-parallel.
  if (lane < 4) {
    const bool fr = lane >= 2;
    const int q = lane & 1;
    // per-lane rows of the model block (immediate offsets k below); 1 / 0 multipliers select the terms
    const double* __restrict__ A = mdl + (q ? 2 * N : 0);
    const double* __restrict__ Bv = mdl + (q ? 3 * N : N);
    const double* __restrict__ Cc = mdl + (q ? 6 * N : 5 * N);
    const double* __restrict__ R = rr + 4 + q;
    const double h = fr ? x0[2] : 1.0, v0 = fr ? x0[3] : 0.0, one = fr ? 1.0 : 0.0;
    double acc = fr ? x0[q] : 0.0;
    double* __restrict__ out = fr ? sm.err[q] : sm.pre[2 * q];
    if (!fr) out[0] = 0.0;
    // every load first (the model rows are not written here), then the dependent chain
    double a[N], c[N], r[N];
#pragma unroll
    for (int k = 0; k < N; ++k) {
      a[k] = A[k];
      c[k] = Cc[k];
      r[k] = R[4 * k];
    }
    const double b0 = Bv[0];
#pragma unroll
    for (int k = 0; k < N; ++k) {
      acc = acc + a[k] * h + (k == 0 ? b0 : 0.0) * (k == 0 ? v0 : 0.0) + one * c[k];
      out[k + 1] = acc - one * r[k];
    }
  }
  if (lane >= 1 && lane <= N) {
    sm.err[2][lane] = x0[2] - rr[4 * lane + 2];
    sm.err[3][lane] = 0.0 - rr[4 * lane + 3];
  }
  __syncthreads();
  T.end(0);
  T.begin();

  // ---- condense: column `lane` of H (lane n -> g) by the backward adjoint recursion ----
  // mu_m = W_m s_m + A_m' mu_{m+1};  H[(i,c'), col] = (B_i e_c')' mu_{i+1}
  // The column stays in registers (Pc) through the scaling; static indices need the m loop
  // fully unrolled.
  // At n = 64 (N = 32) no lane is left over for g: the second branch.
  MPCQP_MARK("setup.condense");
  double Pc[n];
  if constexpr (n < kWave) {
#pragma unroll
    for (int i = 0; i < n; ++i) Pc[i] = 0.0;
    if (lane <= n) {
      // Every lane runs the same instruction stream: the free-response column (lane n, which yields g)
      // and the two kinds of decision-variable column differ only in lane constants and in which LDS
      // row a lane reads per step, so the recursion has no branch and its loads pipeline.  Per step m
      // the column's state sensitivity is s = (s0, s1, s2, s3):
      //   speed v_{j+1} (cc = 0):      (be_{j+1}, et_{j+1}, 0, 0) from m = j + 2 on, (0, 0, 0, 1) at m = j + 1
      //   steering delta_j (cc = 1):   si_j (P_a[m] - P_a[j+1], P_g[m] - P_g[j+1], 1, 0) from m = j + 1 on
      //   free response (lane n):      e_m
      // s0 = fma(k, X0[m] - o0, b0) (s1 alike), s2 = fma(kg, X2[m], c2), s3 = fma(kg, X3[m], c3), each
      // gated to 0 before the column's first step: the values of the case analysis, exactly.
      const bool gcol = lane == n;
      const int j = kv;
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
      // the cost weights: Q / Q_N symmetrised, diagonal in the default parameters (a uniform branch)
      bool diag = true;
#pragma unroll
      for (int a = 0; a < 4; ++a)
#pragma unroll
        for (int b = 0; b < 4; ++b)
          if (a != b) diag = diag && p.q[4 * a + b] == 0.0 && p.q_terminal[4 * a + b] == 0.0;
      double mu0 = 0.0, mu1 = 0.0, mu2 = 0.0;
      auto recursion = [&](auto is_diag) {
        constexpr bool kDiag = decltype(is_diag)::value;
        if constexpr (kDiag)
          MPCQP_MARK("setup.condense");
        else
          MPCQP_MARK("setup.condense_full_q");
        double Q[4][4], QN[4][4];
#pragma unroll
        for (int a = 0; a < 4; ++a)
#pragma unroll
          for (int b = 0; b < 4; ++b) {
            Q[a][b] = 0.5 * (p.q[4 * a + b] + p.q[4 * b + a]);
            QN[a][b] = 0.5 * (p.q_terminal[4 * a + b] + p.q_terminal[4 * b + a]);
          }
#pragma unroll
        for (int m = N; m >= 1; --m) {
          double s0 = fma(k01, X0[m] - o0, b0);
          double s1 = fma(k01, X1[m] - o1, b1);
          s0 = m > t01 ? s0 : 0.0;
          s1 = m > t01 ? s1 : 0.0;
          const double s2 = fma(kg, X2[m], m > t2 ? c2v : 0.0);
          const double s3 = fma(kg, X3[m], m == t3 ? 1.0 : 0.0);
          const bool term = m == N;
          auto W = [&](int i, int k) -> double { return term ? QN[i][k] : Q[i][k]; };
          double w0, w1, w2, w3;
          if constexpr (kDiag) {
            w0 = W(0, 0) * s0;
            w1 = W(1, 1) * s1;
            w2 = W(2, 2) * s2;
            w3 = W(3, 3) * s3;
          } else {
            w0 = W(0, 0) * s0 + W(0, 1) * s1 + W(0, 2) * s2 + W(0, 3) * s3;
            w1 = W(1, 0) * s0 + W(1, 1) * s1 + W(1, 2) * s2 + W(1, 3) * s3;
            w2 = W(2, 0) * s0 + W(2, 1) * s1 + W(2, 2) * s2 + W(2, 3) * s3;
            w3 = W(3, 0) * s0 + W(3, 1) * s1 + W(3, 2) * s2 + W(3, 3) * s3;
          }
          // row v_m: its own cost term + the positions after it; row delta_{m-1}: si * heading adjoint
          double ha;
          if (m < N) {
            const double m0 = mu0, m1 = mu1;
            ha = w3 + (be[m] * m0 + et[m] * m1);
            mu0 = w0 + m0;
            mu1 = w1 + m1;
            mu2 = w2 + (mu2 + al[m] * m0 + ga[m] * m1);
          } else {
            ha = w3;
            mu0 = w0;
            mu1 = w1;
            mu2 = w2;
          }
          Pc[m - 1] = ha;
          Pc[N + m - 1] = si[m - 1] * mu2;
        }
      };
      if (diag)
        recursion(std::true_type{});
      else
        recursion(std::false_type{});
      MPCQP_MARK("setup.gcol");
      if (gcol)  // the free-response column is g
#pragma unroll
        for (int i = 0; i < n; ++i) sm.g[i] = Pc[i];
      // input cost sum_k U_k' R U_k with a_k = (v_{k+1} - v_k)/dt: a band of column `lane`, read from
      // the band table at offset i - lane (one LDS read per row at an immediate offset; a compare-and-
      // select per row and band entry cost ~25 instructions a row)
      MPCQP_MARK("setup.band");
      if (gcol) {  // the v_0 = x0[3] end of a_0
        const double r00 = 0.5 * (p.r[0] + p.r[0]) / (dt * dt), r10 = 0.5 * (p.r[2] + p.r[1]) / dt;
        sm.g[0] += -x0[3] * r00;
        sm.g[N] += -x0[3] * r10;
      }
      // the g column (lane n) reads kind 3 (all zeros) from offset 0: n - 1 - n would be the last word
      // of bt[2], not a zero
      const int kind = gcol ? 3 : (cc == 1 ? 1 : (lane + 1 < N ? 0 : 2));
      const double* tb = &sm.bt[kind][gcol ? 0 : n - 1 - lane];
#pragma unroll
      for (int i = 0; i < n; ++i) Pc[i] += tb[i];
    }
    __syncthreads();
    if (!act)
#pragma unroll
      for (int i = 0; i < n; ++i) Pc[i] = 0.0;  // lane n carried g
  } else {
    // n = 64 (N = 32): every lane holds a column, so g takes a second pass of the same recursion,
    // wave-uniform (its inputs are the free-response errors alone), stored by lane 0.  Unrolled by
    // template (a #pragma unroll of this body stops at clang's threshold, and Pc would then be
    // indexed dynamically: scratch memory).  Each step's LDS reads and lane compares stay in their
    // step (hoisted, they spill the column's 128 registers), and the input-cost band is added to the
    // step's two rows right there (the same sum ha + band as the band loop above).
#pragma unroll
    for (int i = 0; i < n; ++i) Pc[i] = 0.0;
    double Q[4][4], QN[4][4];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        Q[i][j] = 0.5 * (p.q[4 * i + j] + p.q[4 * j + i]);
        QN[i][j] = 0.5 * (p.q_terminal[4 * i + j] + p.q_terminal[4 * j + i]);
      }
    const double r00 = 0.5 * (p.r[0] + p.r[0]) / (dt * dt), r10 = 0.5 * (p.r[2] + p.r[1]) / dt;
    const double r11 = 0.5 * (p.r[3] + p.r[3]);
#pragma nounroll
    for (int gpass = 0; gpass < 2; ++gpass) {
      const int j = kv;
      const bool gcol = gpass == 1;
      const double sj = gcol ? 0.0 : si[j];
      const double pa0 = gcol ? 0.0 : sm.pre[0][j + 1], pg0 = gcol ? 0.0 : sm.pre[2][j + 1];
      const double bj = (!gcol && j + 1 < N) ? be[j + 1] : 0.0, ej = (!gcol && j + 1 < N) ? et[j + 1] : 0.0;
      double mu0 = 0.0, mu1 = 0.0, mu2 = 0.0;
      Unroll<0, N>::run([&](auto mc) __attribute__((always_inline)) {
        constexpr int m = N - decltype(mc)::value;
        double s0, s1, s2, s3;
        if (gcol) {
          s0 = sm.err[0][m];
          s1 = sm.err[1][m];
          s2 = sm.err[2][m];
          s3 = sm.err[3][m];
        } else if (m > j) {
          if (cc == 0) {
            s0 = m >= j + 2 ? bj : 0.0;
            s1 = m >= j + 2 ? ej : 0.0;
            s2 = 0.0;
            s3 = m == j + 1 ? 1.0 : 0.0;
          } else {
            s0 = sj * (sm.pre[0][m] - pa0);
            s1 = sj * (sm.pre[2][m] - pg0);
            s2 = sj;
            s3 = 0.0;
          }
        } else {
          s0 = s1 = s2 = s3 = 0.0;
        }
        const bool term = m == N;
        auto W = [&](int i, int k) -> double { return term ? QN[i][k] : Q[i][k]; };
        const double w0 = W(0, 0) * s0 + W(0, 1) * s1 + W(0, 2) * s2 + W(0, 3) * s3;
        const double w1 = W(1, 0) * s0 + W(1, 1) * s1 + W(1, 2) * s2 + W(1, 3) * s3;
        const double w2 = W(2, 0) * s0 + W(2, 1) * s1 + W(2, 2) * s2 + W(2, 3) * s3;
        const double w3 = W(3, 0) * s0 + W(3, 1) * s1 + W(3, 2) * s2 + W(3, 3) * s3;
        double ha;
        if (m < N) {
          const double m0 = mu0, m1 = mu1;
          ha = w3 + (be[m] * m0 + et[m] * m1);
          mu0 = w0 + m0;
          mu1 = w1 + m1;
          mu2 = w2 + (mu2 + al[m] * m0 + ga[m] * m1);
        } else {
          ha = w3;
          mu0 = w0;
          mu1 = w1;
          mu2 = w2;
        }
        const double hd = si[m - 1] * mu2;
        // two conditions, not an if/else: merged into one store through a select of the two
        // addresses, the column would be addressed through a generic pointer (scratch memory)
        if (gcol && lane == 0) {
          sm.g[m - 1] = ha;
          sm.g[N + m - 1] = hd;
        }
        if (!gcol) {
          int ln = lane;  // opaque per step: the band's compares are not hoisted out of the pass loop
          asm volatile("" : "+v"(ln));
          auto band = [&](int i) -> double {  // the band entry of row i in column ln
            const int d = i - ln;
            double add = 0.0;
            if (cc == 0) {  // the band table's values (above)
              const bool last = ln + 1 >= N;
              if (d == 0) add = last ? r00 : 2.0 * r00;
              if (d == -1 || (d == 1 && !last)) add = -r00;
              if (d == N) add = r10;
              if (d == N + 1 && !last) add = -r10;
            } else {
              if (d == 0) add = r11;
              if (d == -N) add = r10;
              if (d == -N - 1) add = -r10;
            }
            return add;
          };
          Pc[m - 1] = ha + band(m - 1);
          Pc[N + m - 1] = hd + band(N + m - 1);
        }
        __builtin_amdgcn_sched_barrier(0);
      });
      if (gcol && lane == 0) {  // the v_0 = x0[3] end of a_0
        sm.g[0] += -x0[3] * r00;
        sm.g[N] += -x0[3] * r10;
      }
    }
    __syncthreads();
  }
  T.end(1);
  T.begin();

  // ---- unscaled data: P = 2H (column `lane`), q = 2g, folded row bounds ----
  MPCQP_MARK("setup.unscaled");
  double qv = act ? 2.0 * sm.g[lane] : 0.0;
  double cmx[4] = {0.0, 0.0, 0.0, 0.0};  // column max of |P| (partial maxima)
#pragma unroll
  for (int i = 0; i < n; ++i) {
    Pc[i] = 2.0 * Pc[i];
    cmx[i % 4] = fmax(cmx[i % 4], fabs(Pc[i]));
  }
  double cmax = fmax(fmax(cmx[0], cmx[1]), fmax(cmx[2], cmx[3]));
  double lo[3], hi[3], wt[3], E[3];
  // unscaled row coefficients (slot 1: own, 1 back; slot 2: own, 1 back, 2 back): exact zeros where
  // the variable back is a constant (v_0, u_prev) or would lie in the other block
  const double idt = 1.0 / dt, v0 = x0[3];
  double k1[2], k2[3];
  k1[0] = act ? (even ? idt : 1.0) : 0.0;
  k1[1] = (even && kv >= 1) ? -idt : 0.0;
  k2[0] = act ? (even ? idt : 1.0) : 0.0;
  k2[1] = act ? (even ? (kv >= 1 ? -2.0 * idt : 0.0) : (kv >= 1 ? -1.0 : 0.0)) : 0.0;
  k2[2] = (even && kv >= 2) ? idt : 0.0;
  {
    // the rows' constant parts moved into the bounds: a_0 = (v_1 - v_0)/dt, a_1 - a_0 carries +v_0/dt
    const double ofa = lane == 0 ? v0 * idt : 0.0;
    const double ofr = (act && kv == 0) ? up[cc] + ofa : ((even && kv == 1) ? -v0 * idt : 0.0);
    lo[0] = even ? p.v_bounds[0] : 0.0;
    hi[0] = even ? p.v_bounds[1] : 0.0;
    wt[0] = even ? p.slack_velocity : 0.0;
    lo[1] = act ? p.u_bounds[2 * cc] + ofa : 0.0;
    hi[1] = act ? p.u_bounds[2 * cc + 1] + ofa : 0.0;
    wt[1] = act ? p.slack_input : 0.0;
    lo[2] = act ? p.du_bounds[2 * cc] + ofr : 0.0;
    hi[2] = act ? p.du_bounds[2 * cc + 1] + ofr : 0.0;
    wt[2] = act ? p.slack_rate : 0.0;
    E[0] = even ? 1.0 : 0.0;
    E[1] = act ? 1.0 : 0.0;
    E[2] = act ? 1.0 : 0.0;
  }
  double D = act ? 1.0 : 0.0;
  double cscale = 1.0;
  T.end(2);
  T.begin();

  // ---- Ruiz equilibration + cost scaling (OSQP scale_data, `scaling` iterations) ----
  // 1/sqrt by v_rsq_f64 + two Newton steps (within an ulp; any positive scaling is a valid
  // equilibration), the cost factor of each pass folded into the next pass's column scaling
  auto rsqrt = [](double v) {
    double y = __builtin_amdgcn_rsq(v);
    y = y * fma(-0.5 * v, y * y, 1.5);
    return y * fma(-0.5 * v, y * y, 1.5);
  };
  double cpend = 1.0;  // cost factor not yet applied to Pc
  MPCQP_MARK("setup.ruiz");
  for (int it = 0; it < p.scaling; ++it) {
    // column norms of [P; A] (first n columns of the KKT matrix): the lane's own rows and
    // the banded rows 1 and 2 ahead
    double ccol = fmax(fmax(E[0], E[1] * fabs(k1[0])), E[2] * fabs(k2[0]));
    ccol = fmax(ccol, LN::shl1(fmax(E[1] * fabs(k1[1]), E[2] * fabs(k2[1]))));
    ccol = fmax(ccol, LN::shl2(E[2] * fabs(k2[2])));
    ccol *= D;
    const double dl = act ? rsqrt(limit_scaling(fmax(cmax, ccol))) : 0.0;
    // row norms of A
    const double Dm1 = LN::shr1(D), Dm2 = LN::shr1(Dm1);
    const double r1 = fmax(fabs(k1[0]) * D, fabs(k1[1]) * Dm1);
    const double r2 = fmax(fmax(fabs(k2[0]) * D, fabs(k2[1]) * Dm1), fabs(k2[2]) * Dm2);
    const double el0 = even ? rsqrt(limit_scaling(E[0] * D)) : 0.0;
    const double el1 = act ? rsqrt(limit_scaling(E[1] * r1)) : 0.0;
    const double el2 = act ? rsqrt(limit_scaling(E[2] * r2)) : 0.0;
    // apply: P <- ct_prev dl P dl (column `lane`, the row factors read back from LDS), q <- dl q
    lds_sync();
    sm.buf[lane] = dl;
    lds_sync();
    const double dlc = dl * cpend;
    double cmp[4] = {0.0, 0.0, 0.0, 0.0};  // four partial maxima: no serial fmax chain (max is exact)
#pragma unroll
    for (int i = 0; i < n; ++i) {
      const double t = Pc[i] * (sm.buf[i] * dlc);
      Pc[i] = t;
      cmp[i % 4] = fmax(cmp[i % 4], fabs(t));
    }
    const double cm2 = fmax(fmax(cmp[0], cmp[1]), fmax(cmp[2], cmp[3]));
    D *= dl;
    qv *= dl;
    E[0] *= el0;
    E[1] *= el1;
    E[2] *= el2;
    // cost scaling
    const double cn = LN::sum(act ? cm2 : 0.0) / n;
    const double qn = limit_scaling(LN::max(fabs(qv)));
    const double ct = 1.0 / limit_scaling(fmax(cn, qn));
    cpend = ct;
    qv *= ct;
    cmax = cm2 * ct;
    cscale *= ct;
  }
#pragma unroll
  for (int i = 0; i < n; ++i) Pc[i] *= cpend;
  __syncthreads();
  T.end(3);
  T.begin();

  // ---- Pbar: symmetric (the lower-triangle value, computed by column min, for both halves),
  //      moved from the column-per-lane setup layout to the row-major solve layout ----
  // symmetric Pbar = the lower triangle (row i >= column lane, computed by column `lane`)
  bool finite = isfinite(qv) && isfinite(cscale);
  // the model block itself (LTV coefficients, window, x0, u_prev): a non-finite input flags the QP
  // even where the diagonal-cost condensing multiplies no zero weight into it (a position error at
  // N = 1 has no decision variable to reach)
#pragma unroll 4
  for (int i = lane; i < 11 * N + 10; i += LN::kLanes) finite = finite && isfinite(mdl[i]);
  MPCQP_MARK("setup.write");
  lds_sync();  // setup's LDS data is dead: Pbar overwrites it
  if constexpr (kPackedP<N>) {
    double* Pb = lds.solve.P;
    if (act) {
#pragma unroll
      for (int i = 0; i < n; ++i)
        if (i >= lane) {  // entry (i, lane)
          Pb[(i * (i + 1)) / 2 + lane] = Pc[i];
          finite = finite && isfinite(Pc[i]);
        }
    }
    for (int e = (n * (n + 1)) / 2 + lane; e < kWave * (kWave + 1) / 2; e += kWave) Pb[e] = 0.0;  // rows n..63
    lds_sync();
    if (act) {  // form()'s band addresses: save what they hold
      const double* rowp = Pb + (lane * (lane + 1)) / 2 + lane;
      lds.solve.band[0][lane] = lane >= 2 ? rowp[-2] : 0.0;
      lds.solve.band[1][lane] = lane >= 1 ? rowp[-1] : 0.0;
      lds.solve.band[2][lane] = rowp[0];
    }
  } else {
    constexpr int kPS = SolveSmem<N>::kPS;
    double* Pb = lds.solve.P;
    if (act) {
#pragma unroll
      for (int i = 0; i < n; ++i)
        if (i >= lane) {  // entry (i, lane) and its mirror (lane, i)
          Pb[i * kPS + lane] = Pc[i];
          Pb[lane * kPS + i] = Pc[i];
          finite = finite && isfinite(Pc[i]);
        }
    } else if (lane == n) {  // the zero padding column
#pragma unroll
      for (int i = 0; i < n; ++i) Pb[i * kPS + n] = 0.0;
    }
    if (lane < 4) lds.solve.pad0[lane] = 0.0;
    else if (lane < 8) lds.solve.pad1[lane - 4] = 0.0;
    if constexpr (n >= 8) {  // form()'s band addresses: save what they hold
      lds_sync();
      if (act) {
        const double* rowp = Pb + lane * (kPS + 1);
#pragma unroll
        for (int d = 0; d < 5; ++d) lds.solve.band[d][lane] = rowp[d - 2];
      }
    }
  }
  double wb[3];
#pragma unroll
  for (int r = 0; r < 3; ++r) {
    lo[r] *= E[r];
    hi[r] *= E[r];
    wb[r] = E[r] > 0.0 ? cscale * wt[r] / (E[r] * E[r]) : 0.0;
    finite = finite && isfinite(lo[r]) && isfinite(hi[r]);
  }
  // non-finite data (NaN/inf in x0, ref or u_prev) -> status MPCQP_NUMERICAL_ERROR
  const bool bad_input = LN::any(!finite);
  C.init(lane, dt, lds.solve);
  C.colb = lds.col;
  C.qv = qv;
  C.D = D;
  C.cscale = cscale;
  {  // Cbar's coefficients: row scaling x row coefficient x the column scaling of the variable
    const double Dm1 = LN::shr1(D), Dm2 = LN::shr1(Dm1);
    C.c0 = E[0] * D;
    C.c10 = (E[1] * k1[0]) * D;
    C.c11 = (E[1] * k1[1]) * Dm1;
    C.c20 = (E[2] * k2[0]) * D;
    C.c21 = (E[2] * k2[1]) * Dm1;
    C.c22 = (E[2] * k2[2]) * Dm2;
  }
#pragma unroll
  for (int r = 0; r < 3; ++r) {
    C.E[r] = E[r];
    C.lo[r] = lo[r];
    C.hi[r] = hi[r];
    C.wb[r] = wb[r];
  }
  __syncthreads();
  if (dbg) {  // in the reference-facing variable order (interleaved<N>)
    const int il = interleaved<N>(lane);
    if (act)
      for (int i = 0; i < n; ++i)
        dbg[interleaved<N>(i) * n + il] =
            kPackedP<N> ? lds.solve.P[tri_idx(i, lane)] : lds.solve.P[i * SolveSmem<N>::kPS + lane];
    double* lf = dbg + state_lane_off(N);
    lf[kFq * kWave + il] = qv;
    lf[kFD * kWave + il] = D;
    lf[kFx * kWave + il] = 0.0;
#pragma unroll
    for (int r = 0; r < 3; ++r) {
      lf[(kFE0 + r) * kWave + il] = E[r];
      lf[(kFlo0 + r) * kWave + il] = lo[r];
      lf[(kFhi0 + r) * kWave + il] = hi[r];
      lf[(kFw0 + r) * kWave + il] = wb[r];
    }
    if (lane == 0) {
      double* sc = dbg + state_scal_off(N);
      sc[0] = cscale;
      sc[1] = bad_input ? -1.0 : 0.0;  // ADMM flag: -1 numerical error, 0 not converged, 1 converged
      sc[2] = 0.0;                     // admm iterations
      sc[3] = 0.0;                     // factorizations
    }
  }
  T.end(4);
  T2.end(0);
  MPCQP_MARK("ctl");
  T.flush(16);   // g_stamps[16..20]: model/prefixes, condensing, unscaled data, Ruiz, Pbar + context
  T2.flush(21);  // g_stamps[21]: whole setup
  return bad_input;
}

// ------------------------------------------------------------------ K2c: polish
// Semismooth Newton / active-set iteration on the scaled problem from x (in/out): the first
// active-set guess classifies zg, later ones C x.  Each pass factorizes the Newton matrix of
// the current set (from scratch, or by rank-1 updates of the previous pass's inverse when few
// soft rows changed), solves with one step of iterative refinement, and stops when the set
// reproduces itself (the exact optimum: returns 1, x = that optimum); otherwise an exact line
// search along the Newton step.  0: not found within max_it passes, -1: numerical failure.
// Uses the KKT inverse registers (an ADMM phase that continues must refactor).
template <int N, bool Pair = false>
__device__ __forceinline__ int polish_qp(Ctx<N, Pair>& C, double& x, const double zg[3], int max_it, int& pol_it,
                                         int& nfact, int& n_ls) {
  using LN = Lanes<Pair>;
  constexpr int n = 2 * N;
  const bool act = C.act;
  int result = 0;
  Stamps T;
  double zc[3];
  int cd[3];
  C.Cmul(x, zc);
  double Px = C.Pmul(x);  // P x, carried along the passes
#pragma unroll
  for (int r = 0; r < 3; ++r) cd[r] = zg[r] > C.hi[r] ? 2 : (zg[r] < C.lo[r] ? 1 : 0);
  constexpr int kMaxRank1 = n / 2;  // more changed rows than this: refactor (form + sweep)
  double rwf[3] = {0.0, 0.0, 0.0};  // soft-row weights of the current factorization
  bool have_fact = false;
  for (int pass = 0; pass < max_it; ++pass) {
    MPCQP_MARK("pol.ctl");
    ++pol_it;
    C.opaque();
    double rw[3], tmp[3];
#pragma unroll
    for (int r = 0; r < 3; ++r) {
      rw[r] = cd[r] ? 2.0 * C.wb[r] : 0.0;
      tmp[r] = cd[r] == 2 ? rw[r] * C.hi[r] : (cd[r] == 1 ? rw[r] * C.lo[r] : 0.0);
    }
    // Factorize the Newton matrix of this active set: from scratch on the first pass, by
    // rank-1 updates of the previous inverse when only a few soft rows changed.
    bool refac = !have_fact;
    if (!refac) {
      uint64_t chg[3];
      int nchg = 0;
#pragma unroll
      for (int r = 0; r < 3; ++r) {
        chg[r] = LN::ballot(act && rw[r] != rwf[r]);
        nchg += __popcll(chg[r]);
      }
      refac = nchg > kMaxRank1;
      T.begin();
#pragma unroll
      for (int r = 0; r < 3; ++r) {
        uint64_t m = chg[r];
        while (m && !refac) {
          MPCQP_MARK("pol.rank1");
          const int l = __builtin_ctzll(m);
          m &= m - 1;
          refac = !C.rank1(r, l, LN::readv(rw[r] - rwf[r], l));
          ++C.n_r1;
        }
      }
      T.end(1);
    }
    MPCQP_MARK("pol.ctl");
    if (refac) {
      T.begin();
      MPCQP_MARK("pol.form");
      C.form(0.0, rw);
      T.end(0);
      T.begin();
      MPCQP_MARK("pol.sweep");
      const bool okf = C.sweep();
      T.end(1);
      MPCQP_MARK("pol.ctl");
      ++C.n_full;
      if (LN::any(!okf)) {
        result = -1;
        break;
      }
      have_fact = true;
    }
    ++nfact;
#pragma unroll
    for (int r = 0; r < 3; ++r) rwf[r] = rw[r];
    T.begin();
    MPCQP_MARK("pol.solve");
    const double rhs = C.CTmul(tmp) - C.qv;
    double xn = C.inv_mul(rhs);
    double zn[3];
    C.Cmul(xn, zn);
    bool diff = false;
#pragma unroll
    for (int r = 0; r < 3; ++r) {
      const int c2 = zn[r] > C.hi[r] ? 2 : (zn[r] < C.lo[r] ? 1 : 0);
      diff = diff || (c2 != cd[r]);
    }
    if (LN::any(!isfinite(xn))) {
      T.end(2);
      result = -1;
      break;
    }
    if (!LN::any(diff)) {
      // the set reproduces itself: one step of iterative refinement (res = rhs - M xn), then
      // accept if it still does
      MPCQP_MARK("pol.refine");
      double t3[3];
#pragma unroll
      for (int r = 0; r < 3; ++r) t3[r] = rw[r] * zn[r];
      const double Mx = C.Pmul(xn) + C.CTmul(t3);
      xn += C.inv_mul(rhs - Mx);
      C.Cmul(xn, zn);
      diff = false;
#pragma unroll
      for (int r = 0; r < 3; ++r) {
        const int c2 = zn[r] > C.hi[r] ? 2 : (zn[r] < C.lo[r] ? 1 : 0);
        diff = diff || (c2 != cd[r]);
      }
      if (LN::any(!isfinite(xn))) {
        T.end(2);
        result = -1;
        break;
      }
      if (!LN::any(diff)) {
        T.end(2);
        x = xn;
        result = 1;
        break;
      }
    }
    T.end(2);
    // exact line search along d = xn - x: phi(t) = f(x + t d) is convex piecewise quadratic,
    // phi' piecewise linear and nondecreasing; semismooth Newton on phi' from t = 1 downwards
    // lands on the minimizer in [0, 1] after a few pieces (two independent reductions a step).
    // P xn from the Newton system (P xn + q = -C' rw (C xn - bound)): no product with P.
    T.begin();
    MPCQP_MARK("pol.ls");
    double tb[3];
#pragma unroll
    for (int r = 0; r < 3; ++r)
      tb[r] = rw[r] * (zn[r] - (cd[r] == 2 ? C.hi[r] : (cd[r] == 1 ? C.lo[r] : 0.0)));
    const double dx = act ? xn - x : 0.0;
    const double Pd = act ? (-C.CTmul(tb) - C.qv) - Px : 0.0;
    double zd[3];
#pragma unroll
    for (int r = 0; r < 3; ++r) zd[r] = zn[r] - zc[r];
    const double qd = LN::sum(act ? dx * Pd : 0.0);
    const double lin = LN::sum(act ? (Px + C.qv) * dx : 0.0);
    double t = 1.0;
    for (int ls = 0; ls < 40; ++ls) {
      MPCQP_MARK("pol.lstrial");
      ++n_ls;
      double g1 = 0.0, g2 = 0.0;
#pragma unroll
      for (int r = 0; r < 3; ++r) {
        // zt - clamp(zt, lo, hi): zt - hi above, zt - lo below, exactly 0 inside (the same values
        // as the compare-and-select form, without its branches: zc, zd are finite here)
        const double zt = zc[r] + t * zd[r];
        const double rr = zt - min_nc(max_nc(zt, C.lo[r]), C.hi[r]);
        g1 += 2.0 * C.wb[r] * rr * zd[r];
        if (rr != 0.0) g2 += 2.0 * C.wb[r] * zd[r] * zd[r];
      }
      const double d1 = lin + t * qd + LN::sum(g1);
      const double d2 = qd + LN::sum(g2);
      if (d1 <= 0.0 || !(d2 > 0.0)) break;
      const double tn = fmax(0.0, t - d1 / d2);
      if (tn >= t) break;
      // same linear piece of phi' at tn as at t: tn is that piece's root, the minimizer
      bool moved = false;
#pragma unroll
      for (int r = 0; r < 3; ++r) {
        // the piece (above / inside / below) changed: lo <= hi, so the two compares decide it
        const double za = zc[r] + t * zd[r], zb = zc[r] + tn * zd[r];
        moved = moved || ((za > C.hi[r]) != (zb > C.hi[r])) || ((za < C.lo[r]) != (zb < C.lo[r]));
      }
      t = tn;
      if (!LN::any(moved)) break;
    }
    MPCQP_MARK("pol.lsend");
    x = x + t * dx;
    Px = Px + t * Pd;
    C.Cmul(x, zc);
#pragma unroll
    for (int r = 0; r < 3; ++r) cd[r] = zc[r] > C.hi[r] ? 2 : (zc[r] < C.lo[r] ? 1 : 0);
    T.end(3);
  }
  MPCQP_MARK("ctl");
  T.flush(8);  // g_stamps[8..11]: polish form, sweep/rank-1, solve+check, line search
  return result;
}

// ------------------------------------------------------------------ K2b: ADMM
// OSQP's iteration on the scaled problem (rho / sigma / alpha / adaptive rho / termination as
// the reference settings).  From iteration polish_from on, a termination check that fails also
// attempts the polish: an exact optimum found there satisfies the termination test itself.
// The loop state lives in the caller (AdmmState): admm_run stops at such an attempt and the
// caller resumes it after a failed one, so the kernel holds ONE inlined copy of the polish (the
// early attempts, the final polish and method newton share the call site in k_solve) -- the
// polish is a third of k_solve's code, which is larger than the 64 KB instruction cache.
struct AdmmState {
  double x, z[3], y[3], rho;
  double rho_next;  // the adaptive-rho update of the check that stopped for an attempt
  int it, nfact;
  bool need_fact;   // form + sweep at the next entry (start, rho change, after a failed attempt)
  bool rho_change;  // rho_next is pending (applied after a failed attempt)
};
enum : int { kAdmmBad = -1, kAdmmMaxIter = 0, kAdmmConverged = 1, kAdmmApprox = 3, kAdmmAttempt = 4 };

// Runs ADMM until an event: kAdmmBad (numerical error), kAdmmConverged (eps_abs/eps_rel met),
// kAdmmAttempt (a check asks for an early polish; rho_change/rho_next hold that check's
// adaptive-rho decision), kAdmmApprox / kAdmmMaxIter (max_iter reached within / outside 10x the
// tolerances: OSQP's solved_inaccurate / max_iter_reached).
template <int N, bool Pair = false>
__device__ __forceinline__ int admm_run(const mpcqp_params& p, Ctx<N, Pair>& C, AdmmState& S) {
  using LN = Lanes<Pair>;
  const bool act = C.act;
  const double sg = p.sigma, alpha = p.alpha;
  const bool early = p.polish != 0 && p.polish_from > 0;
  int ev = kAdmmMaxIter;
  bool done = false;
  Stamps T;
  while (S.it < p.max_iter && !done) {
    if (S.need_fact) {
      const double rw[3] = {S.rho, S.rho, S.rho};
      T.begin();
      MPCQP_MARK("admm.form");
#ifdef MPCQP_DIAG_FACT_TWICE  // diagnostic builds only: the marginal cost of an ADMM factorization
      C.form(sg, rw);
      (void)C.sweep();
#pragma unroll
      for (int j = 0; j < 2 * N; ++j) asm volatile("" : "+v"(C.r[j]));  // the first inverse is computed
#endif
      C.form(sg, rw);
      T.end(0);
      ++S.nfact;
      T.begin();
      MPCQP_MARK("admm.sweep");
      const bool okf = C.sweep();
      T.end(1);
      MPCQP_MARK("admm.fctl");
      if (LN::any(!okf)) {
        ev = kAdmmBad;
        break;
      }
      S.need_fact = false;
    }
    // The z-update is the prox of the eliminated slack's penalty w dist(z, [lo, hi])^2:
    //   zn = vv - pb (vv - clamp(vv, lo, hi)),  pb = 2w / (rho + 2w)
    // (= (rho vv + 2 w bnd) / (rho + 2 w) outside the bounds, vv inside), and the dual update
    // y + rho (v - zn) with vv = v + y / rho is exactly rho pb (vv - clamp): no selects, and no
    // cancellation of y against rho (v - zn).
    const double rho = S.rho;
    double pb[3], rpb[3];
#pragma unroll
    for (int r = 0; r < 3; ++r) {
      pb[r] = 2.0 * C.wb[r] / (rho + 2.0 * C.wb[r]);
      rpb[r] = rho * pb[r];
    }
    const double ir = 1.0 / rho, oma = 1.0 - alpha;
    // the next termination check's iteration (a multiple of check_termination): a compare per
    // iteration instead of an integer modulo (a dozen scalar instructions)
    int next_check = (S.it / p.check_termination + 1) * p.check_termination;
    while (!S.need_fact && S.it < p.max_iter) {
      MPCQP_MARK("admm.iter");
      const int it = ++S.it;
      C.opaque();
      T.begin();
      double tmp[3];
#pragma unroll
      for (int r = 0; r < 3; ++r) tmp[r] = rho * S.z[r] - S.y[r];
      const double rhs = C.CTmul(tmp) + sg * S.x - C.qv;
      // relaxation folded into the step: xa = alpha xt, Cbar xa = alpha Cbar xt
      const double xa = alpha * C.inv_mul(rhs);
      double za[3];
      C.Cmul(xa, za);
      S.x = xa + oma * S.x;
#pragma unroll
      for (int r = 0; r < 3; ++r) {
        const double v = za[r] + oma * S.z[r];
        const double vv = v + S.y[r] * ir;
        const double d = vv - min_nc(max_nc(vv, C.lo[r]), C.hi[r]);
        S.z[r] = vv - pb[r] * d;
        S.y[r] = rpb[r] * d;
      }
      T.end(2);
      if (it == next_check || it == p.max_iter) {
        MPCQP_MARK("admm.check");
        if (it == next_check) next_check += p.check_termination;
        T.begin();
        // Residual norms (OSQP: unscaled for termination, scaled for the rho update).  The
        // lane maxima are combined before the wave reductions (max distributes), which keeps
        // the check's live set small.
        const double x = S.x;
        double Ax[3];
        C.Cmul(x, Ax);
        double pr = 0, nprim = 0, spr = 0, snprim = 0;
#pragma unroll
        for (int r = 0; r < 3; ++r) {
          if (C.E[r] > 0.0) {
            const double ie = 1.0 / C.E[r];
            pr = fmax(pr, fabs((Ax[r] - S.z[r]) * ie));
            nprim = fmax(nprim, fmax(fabs(Ax[r] * ie), fabs(S.z[r] * ie)));
            spr = fmax(spr, fabs(Ax[r] - S.z[r]));
            snprim = fmax(snprim, fmax(fabs(Ax[r]), fabs(S.z[r])));
          }
        }
        pr = LN::max(pr);
        nprim = LN::max(nprim);
        spr = LN::max(spr);
        snprim = LN::max(snprim);
        const double Px = C.Pmul(x);
        const double Aty = C.CTmul(S.y);
        double du = 0, ndual = 0, sdu = 0, sndual = 0;
        if (act) {
          const double id = 1.0 / C.D;
          const double rd = Px + C.qv + Aty;
          du = fabs(rd * id);
          ndual = fmax(fmax(fabs(Px * id), fabs(Aty * id)), fabs(C.qv * id));
          sdu = fabs(rd);
          sndual = fmax(fmax(fabs(Px), fabs(Aty)), fabs(C.qv));
        }
        du = LN::max(du);
        ndual = LN::max(ndual);
        sdu = LN::max(sdu);
        sndual = LN::max(sndual);
        const double ic = 1.0 / C.cscale;
        du *= ic;
        const double ep = p.eps_abs + p.eps_rel * nprim;
        const double ed = p.eps_abs + p.eps_rel * ndual * ic;
        T.end(3);
        // fmax drops NaNs, so test the iterate itself
        if (LN::any(!isfinite(x) || !isfinite(S.z[0] + S.z[1] + S.z[2]) || !isfinite(S.y[0] + S.y[1] + S.y[2])) ||
            !isfinite(pr) || !isfinite(du)) {
          ev = kAdmmBad;
          done = true;
          break;
        }
        if (pr <= ep && du <= ed) {
          ev = kAdmmConverged;
          done = true;
          break;
        }
        // OSQP at max_iter: the same test with eps_abs and eps_rel x10 passes -> solved_inaccurate
        // (no polish); otherwise max_iter_reached (the loop ends by itself after this check)
        if (it == p.max_iter && pr <= 10.0 * p.eps_abs + 10.0 * p.eps_rel * nprim &&
            du <= 10.0 * p.eps_abs + 10.0 * p.eps_rel * ndual * ic)
          ev = kAdmmApprox;
        // this check's adaptive-rho decision (a function of its residuals alone)
        bool rc = false;
        double rn = rho;
        if (p.adaptive_rho && it % p.adaptive_rho_interval == 0) {
          const double pn = spr / (snprim + kDivTol);
          const double dn = sdu / (sndual + kDivTol);
          rn = rho * sqrt(pn / (dn + kDivTol));
          rn = fmin(fmax(rn, kRhoMin), kRhoMax);
          rc = rn > rho * p.adaptive_rho_tolerance || rn < rho / p.adaptive_rho_tolerance;
        }
        // early polish from polish_from on, or earlier once both residuals are near their
        // tolerances: the caller polishes, then resumes with this rho decision if it failed
        const bool near = p.polish_near > 0.0 && it >= 2 * p.check_termination &&
                          fmax(pr / ep, du / ed) < p.polish_near;
        if (early && (it >= p.polish_from || near) && it < p.max_iter) {
          S.rho_change = rc;
          S.rho_next = rn;
          ev = kAdmmAttempt;
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
  MPCQP_MARK("ctl");
  T.flush(0);  // g_stamps[0..3]: form, sweep, ADMM iteration body, termination checks
  return ev;
}

// The ADMM phase's solver state for debug_state (x, flag, iterations, factorizations).
template <int N>
__device__ __forceinline__ void admm_debug_state(double* __restrict__ dbg, bool act, double x, int flag, int it,
                                                 int nfact) {
  if (!dbg) return;
  dbg[state_lane_off(N) + kFx * kWave + interleaved<N>(threadIdx.x)] = act ? x : 0.0;
  if (threadIdx.x == 0) {
    double* sc = dbg + state_scal_off(N);
    sc[1] = flag < 0 ? -1.0 : (flag > 0 ? 1.0 : 0.0);
    sc[2] = (double)it;
    sc[3] = (double)nfact;
  }
}

// ------------------------------------------------------------------ K2c: status + outputs
// x: the returned iterate (the polish's last iterate when the final polish ran), x_admm: the
// ADMM iterate (returned when that polish did not converge, as OSQP does).
template <int N, class Win, bool Pair = false>
__device__ __forceinline__ int finish_qp(const mpcqp_params& p, int b, const double* __restrict__ model,
                                         const double* __restrict__ in_x0, const double* __restrict__ in_ref,
                                         const double* __restrict__ in_up, const Win& win, const double* kept_model,
                                         Ctx<N, Pair>& C,
                                          double x, double x_admm, int admm_flag, bool do_polish, bool pol_ok,
                                          bool bad, int admm_it, int nfact, int pol_it, int n_ls,
                                          double* __restrict__ u0o, double* __restrict__ Xo, double* __restrict__ Uo,
                                          int32_t* __restrict__ statuso, int32_t* __restrict__ iterso,
                                          uint8_t* __restrict__ activeo, double& Uout) {
  using LN = Lanes<Pair>;
  constexpr int n = 2 * N;
  const int lane = win.lane();
  const bool act = C.act;
  const bool use_admm = p.method == MPCQP_METHOD_ADMM;
  const bool approx = admm_flag == kAdmmApprox;  // OSQP's solved_inaccurate at max_iter: not polished
  const bool admm_ok = admm_flag == kAdmmConverged;
  Stamps T3;
  T3.begin();
  MPCQP_MARK("outputs");
  if (LN::any(!isfinite(x))) bad = true;
  int status;
  if (bad) {
    status = MPCQP_NUMERICAL_ERROR;
  } else if (pol_ok) {
    status = MPCQP_SOLVED;
  } else if (use_admm) {
    if (do_polish) x = x_admm;  // polish failed: return the ADMM iterate (OSQP behaviour)
    status = admm_ok ? (do_polish ? MPCQP_SOLVED_INACCURATE : MPCQP_SOLVED)
                     : (approx ? MPCQP_SOLVED_INACCURATE : MPCQP_MAX_ITER_REACHED);
  } else {
    status = MPCQP_MAX_ITER_REACHED;
  }

  // ---- outputs (unscaled): speeds W -> accelerations; states by the LTV recursion ----
  // the model's lane values: re-derived from the inputs when K1 is fused (the LDS copy is gone)
  double m_al = 0.0, m_be = 0.0, m_ga = 0.0, m_et = 0.0, m_si = 0.0, m_c0 = 0.0, m_c1 = 0.0;
  double x00, x01, x02, x03, up0, up1;
  if constexpr (kModelKept<N>) {  // the model block is still in LDS
    const double* mb = kept_model;
    if (lane < N) {
      m_al = mb[lane];
      m_be = mb[N + lane];
      m_ga = mb[2 * N + lane];
      m_et = mb[3 * N + lane];
      m_si = mb[4 * N + lane];
      m_c0 = mb[5 * N + lane];
      m_c1 = mb[6 * N + lane];
    }
    x00 = mb[11 * N + 4];
    x01 = mb[11 * N + 5];
    x02 = mb[11 * N + 6];
    x03 = mb[11 * N + 7];
    up0 = mb[11 * N + 8];
    up1 = mb[11 * N + 9];
  } else if constexpr (Win::kFleet) {
    double rx = 0.0, ry = 0.0, ryaw = 0.0, rv = 0.0;
    if (lane <= N) win.template row<N>(lane, rx, ry, ryaw, rv);
    const LaneModel m = build_lane<Pair>(p, lane, ryaw, rv);
    m_al = m.al;
    m_be = m.be;
    m_ga = m.ga;
    m_et = m.et;
    m_si = m.si;
    m_c0 = m.c0;
    m_c1 = m.c1;
    x00 = win.x0v(0);
    x01 = win.x0v(1);
    x02 = win.x0v(2);
    x03 = win.x0v(3);
    up0 = win.upv(0);
    up1 = win.upv(1);
  } else if (in_ref) {
    const double* rb = in_ref + (size_t)b * (N + 1) * 4;
    const double ryaw = lane <= N ? rb[4 * lane + 2] : 0.0, rv = lane <= N ? rb[4 * lane + 3] : 0.0;
    const LaneModel m = build_lane<Pair>(p, lane, ryaw, rv);
    m_al = m.al;
    m_be = m.be;
    m_ga = m.ga;
    m_et = m.et;
    m_si = m.si;
    m_c0 = m.c0;
    m_c1 = m.c1;
    x00 = in_x0[(size_t)b * 4 + 0];
    x01 = in_x0[(size_t)b * 4 + 1];
    x02 = in_x0[(size_t)b * 4 + 2];
    x03 = in_x0[(size_t)b * 4 + 3];
    up0 = in_up ? in_up[(size_t)b * 2 + 0] : 0.0;
    up1 = in_up ? in_up[(size_t)b * 2 + 1] : 0.0;
  } else {
    const double* mb = model + (size_t)b * model_stride(N);
    if (lane < N) {
      m_al = mb[lane];
      m_be = mb[N + lane];
      m_ga = mb[2 * N + lane];
      m_et = mb[3 * N + lane];
      m_si = mb[4 * N + lane];
      m_c0 = mb[5 * N + lane];
      m_c1 = mb[6 * N + lane];
    }
    x00 = mb[11 * N + 4];
    x01 = mb[11 * N + 5];
    x02 = mb[11 * N + 6];
    x03 = mb[11 * N + 7];
    up0 = mb[11 * N + 8];
    up1 = mb[11 * N + 9];
  }
  const int cc = lane >= N ? 1 : 0;
  const int kv = lane - cc * N;
  const double W = act ? C.D * x : 0.0;  // v_{j+1} on lane j, delta_j on lane N + j
  const double dt = p.dt;
  const double Wm1 = LN::shr1(W);       // lane k <- v_k (k = 1..N)
  const double U = !act ? 0.0 : (cc == 1 ? W : (W - (lane == 0 ? x03 : Wm1)) / dt);
  const double sj_all = LN::shfl(m_si, cc ? kv : 0);
  const double sj = act ? sj_all : 0.0;
  // psi_{j+1} - psi_0 on lane N + j
  const double sacc = LN::scan((act && cc == 1) ? sj * U : 0.0, lane);
  // lane k <- (psi_k, v_k)
  const int srcp = lane == 0 ? 0 : N + lane - 1;
  const double pk_s = LN::shfl(sacc, srcp < LN::kLanes ? srcp : 0);
  const double vk = lane == 0 ? x03 : Wm1;
  const double pk = lane == 0 ? x02 : x02 + pk_s;
  double t0 = 0.0, t1 = 0.0;
  if (lane < N) {
    t0 = m_al * pk + m_be * vk + m_c0;
    t1 = m_ga * pk + m_et * vk + m_c1;
  }
  const double in0 = LN::scan(t0, lane), in1 = LN::scan(t1, lane);
  const double ex0 = LN::shr1(in0), ex1 = LN::shr1(in1);  // exclusive prefix
  const double Xk0 = x00 + ex0, Xk1 = x01 + ex1;
  if (Xo && lane <= N) {
    double* Xb = Xo + (size_t)b * 4 * (N + 1);
    Xb[0 * (N + 1) + lane] = Xk0;
    Xb[1 * (N + 1) + lane] = Xk1;
    Xb[2 * (N + 1) + lane] = pk;
    Xb[3 * (N + 1) + lane] = vk;
  }
  Uout = U;
  if (Uo && act) Uo[(size_t)b * n + lane] = U;  // U[c][k] at c * N + k: the lane itself
  if (u0o && act && kv == 0) u0o[(size_t)b * 2 + cc] = U;
  const double Um1 = LN::shr1(U);
  if (activeo) {
    uint8_t* ab = activeo + (size_t)b * (5 * N + 1);
    if (lane <= N) ab[lane] = vk > p.v_bounds[1] ? 2 : (vk < p.v_bounds[0] ? 1 : 0);
    if (act) {  // input and rate rows in the reference-facing order (a_0, delta_0, a_1, ...)
      const int il = interleaved<N>(lane);
      ab[N + 1 + il] = U > p.u_bounds[2 * cc + 1] ? 2 : (U < p.u_bounds[2 * cc] ? 1 : 0);
      const double d = U - (kv == 0 ? (cc ? up1 : up0) : Um1);
      ab[3 * N + 1 + il] = d > p.du_bounds[2 * cc + 1] ? 2 : (d < p.du_bounds[2 * cc] ? 1 : 0);
    }
  }
  T3.end(0);
  T3.flush(13);  // g_stamps[13]: status + outputs
  if (lane == 0) {
    statuso[b] = status;
    if (iterso) {
      iterso[4 * (size_t)b + 0] = admm_it;
      iterso[4 * (size_t)b + 1] = pol_it;
      iterso[4 * (size_t)b + 2] = nfact;
      iterso[4 * (size_t)b + 3] = n_ls;
    }
  }
  return status;
}

// One QP through setup -> ADMM (+ early polish attempts) -> final polish -> outputs on the calling
// wave, for the fused fleet loop (k_fleet_loop; no debug state): returns the status, Ulane = the
// lane's U entry (lanes 0 and N: u0).  k_solve runs the same driver inline (below).
template <int N, class Win, bool Pair = false>
__device__ __forceinline__ int solve_one(const mpcqp_params& p, int b, const double* __restrict__ model,
                                         const double* __restrict__ in_x0, const double* __restrict__ in_ref,
                                         const double* __restrict__ in_up, const Win& win, SolveLds<N, Pair>& sm,
                                         double* __restrict__ u0o, double* __restrict__ Xo, double* __restrict__ Uo,
                                         int32_t* __restrict__ statuso, int32_t* __restrict__ iterso,
                                         uint8_t* __restrict__ activeo, double& Ulane) {
  double* const dbg = nullptr;
  const uint64_t t_start = __builtin_amdgcn_s_memtime();
  Stamps TK;
  TK.begin();
  Ctx<N, Pair> C;
  bool bad = setup_qp<N, Win, Pair>(p, b, model, in_x0, in_ref, in_up, win, C, sm, nullptr, dbg);
  const bool use_admm = p.method == MPCQP_METHOD_ADMM;
  AdmmState S;
  S.x = 0.0;
#pragma unroll
  for (int r = 0; r < 3; ++r) S.z[r] = S.y[r] = 0.0;
  S.rho = S.rho_next = p.rho;
  S.it = 0;
  S.nfact = 0;
  S.need_fact = true;
  S.rho_change = false;
  int flag = bad ? kAdmmBad : kAdmmMaxIter, pol_it = 0, n_ls = 0;
  double x = 0.0, x_admm = 0.0;
  bool do_polish = false, pol_ok = false;
  if (use_admm && bad) admm_debug_state<N>(dbg, C.act, 0.0, flag, 0, 0);
  // ADMM with its early polish attempts, then the final polish: ONE polish call site
  while (!bad) {
    // kind 1: early attempt (ADMM resumes if it fails), 2: final polish (OSQP polishes only a
    // solved ADMM run; method newton is the polish alone, from x = 0)
    int kind = 0;
    double zg[3];
    if (use_admm) {
      const int ev = admm_run<N, Pair>(p, C, S);
      if (ev == kAdmmAttempt) {
        kind = 1;
      } else {
        flag = ev;
        x = x_admm = C.act ? S.x : 0.0;
        admm_debug_state<N>(dbg, C.act, x, flag, S.it, S.nfact);
        do_polish = p.polish != 0 && flag == kAdmmConverged;
        kind = do_polish ? 2 : 0;
        bad = flag == kAdmmBad;
      }
#pragma unroll
      for (int r = 0; r < 3; ++r) zg[r] = S.z[r];  // first active-set guess: the ADMM z iterate
    } else {
      do_polish = true;
      kind = 2;
      C.Cmul(x, zg);
    }
    if (kind == 0) break;
    double xp = kind == 1 ? S.x : x;
    Stamps T2;
    T2.begin();
    const int r_ = polish_qp<N, Pair>(C, xp, zg, kind == 1 ? p.polish_attempt_max_iter : p.polish_max_iter, pol_it,
                                S.nfact, n_ls);
    T2.end(0);
    T2.flush(12);  // g_stamps[12]: polish
    if (kind == 2) {  // final polish: its iterate is returned when it converged
      x = xp;
      bad = r_ < 0;
      pol_ok = r_ > 0;
      break;
    }
    if (r_ != 0) {  // the attempt reached the exact optimum (ADMM flag 2) or failed numerically
      flag = r_ > 0 ? 2 : kAdmmBad;
      bad = r_ < 0;
      pol_ok = r_ > 0;
      x = x_admm = C.act ? (pol_ok ? xp : S.x) : 0.0;
      admm_debug_state<N>(dbg, C.act, x, flag, S.it, S.nfact);
      break;
    }
    // a failed attempt resumes ADMM: refactor (the attempt used the inverse's registers) with
    // the rho of that check's adaptive update
    S.need_fact = true;
    if (S.rho_change) S.rho = S.rho_next;
    S.rho_change = false;
  }
  const int status = finish_qp<N, Win, Pair>(p, b, model, in_x0, in_ref, in_up, win, sm.model, C, x, x_admm, flag, do_polish, pol_ok, bad, S.it,
                                  S.nfact, pol_it, n_ls, u0o, Xo, Uo, statuso, iterso, activeo, Ulane);
  TK.end(0);
  TK.flush(22);  // g_stamps[22]: the whole QP
  if (dbg && threadIdx.x == 0) {  // this wave's cycles, start to finish, and its work (tools/qp_cycles.py)
    dbg[state_scal_off(N) + 4] = (double)(__builtin_amdgcn_s_memtime() - t_start);
    dbg[state_scal_off(N) + 5] = (double)C.n_full;  // polish factorizations from scratch
    dbg[state_scal_off(N) + 6] = (double)C.n_r1;    // polish rank-1 updates
    dbg[state_scal_off(N) + 7] = (double)t_start;
  }
  return status;
}

// ------------------------------------------------------------------ K2: fused solve
// One wave runs its QP through setup -> ADMM -> polish/outputs without kernel boundaries, so
// the batch drains once (the slowest QP's whole chain) instead of once per phase.  The scaled
// problem never leaves the CU: Pbar stays in LDS, the per-lane data and the KKT inverse in
// registers (the state buffer is written only when debug_state is set).
// Occupancy: ~225 VGPRs (the KKT inverse is 2n of them) give 2 waves per SIMD; the launch
// bound's 2 keeps the compiler from trading that for AGPR spills (a branch-free condensing
// variant did, and ran at 1 wave per SIMD, +35 % at B = 4096).  Capping the
// registers for a third wave (168, fits the ~13 KB of LDS at N = 20) measured no faster at
// B = 4096: the four QPs per SIMD then run in 1.33 rounds instead of 2, but each wave shares
// its SIMD's FP64 issue with two others.
// From N = 29 on the KKT inverse (2N doubles per lane) fills the 256 registers of 2 waves per SIMD
// (a handful of cold values spill, <= 64 bytes of scratch); Pbar packed (N >= 24) keeps the LDS at
// eight workgroups per CU.  (Before: 1 wave per SIMD from N = 29, the LDS capping a CU at 5.)
template <int N>
constexpr int kSolveWavesPerEU = 2;

template <int N>
__global__ __launch_bounds__(kWave, kSolveWavesPerEU<N>) void k_solve(mpcqp_params p, int B, const uint8_t* __restrict__ mask,
                                                 const double* __restrict__ model, const double* __restrict__ in_x0,
                                                 const double* __restrict__ in_ref, const double* __restrict__ in_up,
                                                 double* __restrict__ state,
                                                 double* __restrict__ u0o, double* __restrict__ Xo,
                                                 double* __restrict__ Uo, int32_t* __restrict__ statuso,
                                                 int32_t* __restrict__ iterso, uint8_t* __restrict__ activeo) {
  __shared__ SolveLds<N> sm;
  const int b = blockIdx.x;
  if (b >= B || (mask && !mask[b])) return;
  // solve_one's driver, kept inline here with the debug state: the headline kernel's code
  // generation stays independent of the fleet loop's instantiation
  double* dbg = p.debug_state ? state + (size_t)b * state_stride(N) : nullptr;
  const uint64_t t_start = __builtin_amdgcn_s_memtime();
  Stamps TK;
  TK.begin();
  Ctx<N> C;
#ifdef MPCQP_DIAG_SETUP_TWICE  // diagnostic builds only: the marginal cost of the setup (tools/ab.py)
  (void)setup_qp<N>(p, b, model, in_x0, in_ref, in_up, BatchWin{}, C, sm, state + (size_t)b * state_stride(N), dbg);
#endif
  bool bad = setup_qp<N>(p, b, model, in_x0, in_ref, in_up, BatchWin{}, C, sm, state + (size_t)b * state_stride(N), dbg);
  const bool use_admm = p.method == MPCQP_METHOD_ADMM;
  AdmmState S;
  S.x = 0.0;
#pragma unroll
  for (int r = 0; r < 3; ++r) S.z[r] = S.y[r] = 0.0;
  S.rho = S.rho_next = p.rho;
  S.it = 0;
  S.nfact = 0;
  S.need_fact = true;
  S.rho_change = false;
  int flag = bad ? kAdmmBad : kAdmmMaxIter, pol_it = 0, n_ls = 0;
  double x = 0.0, x_admm = 0.0;
  bool do_polish = false, pol_ok = false;
  if (use_admm && bad) admm_debug_state<N>(dbg, C.act, 0.0, flag, 0, 0);
  // ADMM with its early polish attempts, then the final polish: ONE polish call site
  while (!bad) {
    // kind 1: early attempt (ADMM resumes if it fails), 2: final polish (OSQP polishes only a
    // solved ADMM run; method newton is the polish alone, from x = 0)
    int kind = 0;
    double zg[3];
    if (use_admm) {
      Stamps TA;
      TA.begin();
      const int ev = admm_run<N>(p, C, S);
      TA.end(0);
      TA.flush(4);  // g_stamps[4]: every admm_run call (slots 5..9 get zeros)
      if (ev == kAdmmAttempt) {
        kind = 1;
      } else {
        flag = ev;
        x = x_admm = C.act ? S.x : 0.0;
        admm_debug_state<N>(dbg, C.act, x, flag, S.it, S.nfact);
        do_polish = p.polish != 0 && flag == kAdmmConverged;
        kind = do_polish ? 2 : 0;
        bad = flag == kAdmmBad;
      }
#pragma unroll
      for (int r = 0; r < 3; ++r) zg[r] = S.z[r];  // first active-set guess: the ADMM z iterate
    } else {
      do_polish = true;
      kind = 2;
      C.Cmul(x, zg);
    }
    if (kind == 0) break;
    double xp = kind == 1 ? S.x : x;
    Stamps T2;
    T2.begin();
    const int r_ = polish_qp<N>(C, xp, zg, kind == 1 ? p.polish_attempt_max_iter : p.polish_max_iter, pol_it,
                                S.nfact, n_ls);
    T2.end(0);
    T2.flush(12);  // g_stamps[12]: polish
    if (kind == 2) {  // final polish: its iterate is returned when it converged
      x = xp;
      bad = r_ < 0;
      pol_ok = r_ > 0;
      break;
    }
    if (r_ != 0) {  // the attempt reached the exact optimum (ADMM flag 2) or failed numerically
      flag = r_ > 0 ? 2 : kAdmmBad;
      bad = r_ < 0;
      pol_ok = r_ > 0;
      x = x_admm = C.act ? (pol_ok ? xp : S.x) : 0.0;
      admm_debug_state<N>(dbg, C.act, x, flag, S.it, S.nfact);
      break;
    }
    // a failed attempt resumes ADMM: refactor (the attempt used the inverse's registers) with
    // the rho of that check's adaptive update
    S.need_fact = true;
    if (S.rho_change) S.rho = S.rho_next;
    S.rho_change = false;
  }
  double U;
#ifdef MPCQP_DIAG_OUTPUT_TWICE  // diagnostic builds only: the marginal cost of the outputs
  finish_qp<N>(p, b, model, in_x0, in_ref, in_up, BatchWin{}, sm.model, C, x, x_admm, flag, do_polish, pol_ok, bad, S.it,
               S.nfact, pol_it, n_ls, u0o, Xo, Uo, statuso, iterso, activeo, U);
#endif
  finish_qp<N>(p, b, model, in_x0, in_ref, in_up, BatchWin{}, sm.model, C, x, x_admm, flag, do_polish, pol_ok, bad, S.it,
               S.nfact, pol_it, n_ls, u0o, Xo, Uo, statuso, iterso, activeo, U);
  TK.end(0);
  TK.flush(22);  // g_stamps[22]: the whole QP
  if (dbg && threadIdx.x == 0) {  // this wave's cycles, start to finish, and its work (tools/qp_cycles.py)
    dbg[state_scal_off(N) + 4] = (double)(__builtin_amdgcn_s_memtime() - t_start);
    dbg[state_scal_off(N) + 5] = (double)C.n_full;  // polish factorizations from scratch
    dbg[state_scal_off(N) + 6] = (double)C.n_r1;    // polish rank-1 updates
    dbg[state_scal_off(N) + 7] = (double)t_start;
  }
}

// ------------------------------------------------------------------ K2, two QPs per wave
// N <= 15 (n <= 30 live lanes): lanes 0-31 solve QP 2w, lanes 32-63 QP 2w + 1 of workgroup w, each
// half through solve_one's driver with the half-wave lane policy (Lanes<true>) and its own LDS
// block; every operation of a QP is the one-wave kernel's, on the same values, so the results are
// the same bit for bit.  The two QPs of a wave run in lockstep while both iterate and mask each other
// off where they part (one polishes, one still iterates): the wave costs about the slower of its
// QPs, and a batch needs half the waves.  Fused K1 only (no workspace model, no debug state).
template <int N>
__global__ __launch_bounds__(kWave, kSolveWavesPerEU<N>) void k_solve_pair(mpcqp_params p, int B,
                                                      const uint8_t* __restrict__ mask,
                                                      const double* __restrict__ in_x0,
                                                      const double* __restrict__ in_ref,
                                                      const double* __restrict__ in_up,
                                                      double* __restrict__ u0o, double* __restrict__ Xo,
                                                      double* __restrict__ Uo, int32_t* __restrict__ statuso,
                                                      int32_t* __restrict__ iterso, uint8_t* __restrict__ activeo) {
  static_assert(2 * N <= 30, "two QPs per wave need n = 2N <= 30 (a padding lane or two per half)");
  __shared__ SolveLds<N, true> sm[2];
  const int h = threadIdx.x >> 5;
  const int b = 2 * blockIdx.x + h;
  if (b >= B || (mask && !mask[b])) return;  // that half only: the other QP runs on
  int ln = threadIdx.x & 31;
  asm volatile("" : "+v"(ln));
  double U;
  solve_one<N, ServeWin, true>(p, b, nullptr, in_x0, in_ref, in_up, ServeWin{ln}, sm[h], u0o, Xo, Uo, statuso,
                               iterso, activeo, U);
}

// ------------------------------------------------------------------ fused closed loop
// Every vehicle of a fleet runs `steps` iterations of the loop body of TrajectoryTracker.track
// (control_stage.py:100-150) on its own wave, with no kernel boundary between steps: the window
// gather fused into K1 (:101-105), the nominal solve and the relaxed retry (:33-56), abort
// (:108-110), the plant (:127), u_prev (:129), the path_idx advance (:141-145) and the goal test
// (:147-150) -- the operations of k_fleet_build / k_solve / k_fleet_advance (mpcqp_fleet.hip) in the
// same order, so the traces equal mpcqp_fleet_run's bit for bit.  The loop state (x, u_prev) stays
// in LDS across steps (no registers held through the solve); it is written back at the end.
// Pair: two vehicles per wave (N <= 15; lanes 0-31 / 32-63, as k_solve_pair), each half its own
// loop state, LDS block and control flow.
template <int N, bool Pair = false>
__global__ __launch_bounds__(kWave, kSolveWavesPerEU<N>) void k_fleet_loop(const mpcqp_params* __restrict__ P,
                                                                         mpcqp_fleet f, int steps,
                                                                         mpcqp::LoopTrigger tr) {
  using LN = Lanes<Pair>;
  __shared__ SolveLds<N, Pair> smv[Pair ? 2 : 1];
  __shared__ double lsv[Pair ? 12 : 6];  // loop state: x[4], u_prev[2] (per half)
  const int h = Pair ? (int)(threadIdx.x >> 5) : 0;
  SolveLds<N, Pair>& sm = smv[h];
  double* const ls = lsv + 6 * h;
  const int slot = 2 * (int)blockIdx.x + h;  // pair: may be V (odd V)
  const int b = Pair ? ((tr.order && slot < f.vehicles) ? tr.order[slot] : slot)
                     : (tr.order ? tr.order[blockIdx.x] : (int)blockIdx.x);
  const int lane = Pair ? (int)(threadIdx.x & 31) : (int)threadIdx.x;
  const int V = f.vehicles;
  if (b >= V) return;
  int phase = f.phase[b];
  // the swarm's trigger (mpcqp_swarm_loop): replans left for this vehicle
  const bool can_replan = tr.max_replans > 0 && tr.replans[b] >= 0 && tr.replans[b] < tr.max_replans;
  auto to_replan = [&](int ph, double x, double y) {  // k_swarm_trigger's transition and problem
    if (lane == 0) {
      f.phase[b] = ph == MPCQP_FLEET_ABORTED ? MPCQP_FLEET_REPLAN_ABORTED : MPCQP_FLEET_REPLAN_RUNNING;
      double* sg = tr.start_goal + 4 * (size_t)b;
      sg[0] = x;
      sg[1] = y;
      sg[2] = f.goal[(size_t)b * 2];
      sg[3] = f.goal[(size_t)b * 2 + 1];
    }
  };
  if (phase != MPCQP_FLEET_RUNNING) {
    // an ABORTED vehicle with replans left is replanned before it steps again (the stepped swarm's
    // trigger fires for it in every step)
    if (phase == MPCQP_FLEET_ABORTED && can_replan) to_replan(phase, f.state[(size_t)b * 4], f.state[(size_t)b * 4 + 1]);
    return;
  }
  const int len = f.ref_len[b];
  int pidx = f.path_idx[b];
  int k = f.steps[b];
  const double* rows = f.ref_global + (size_t)b * f.ref_stride * 4;
  if (lane < 4) ls[lane] = f.state[(size_t)b * 4 + lane];
  else if (lane < 6) ls[lane] = f.u_prev[(size_t)b * 2 + lane - 4];
  __syncthreads();
  for (int s = 0; s < steps; ++s) {
    // k_fleet_build's validation of the loop state, before any indexed access
    const bool bad_ref = len < 1 || len > f.ref_stride || pidx < 0;
    const bool full = k < 0 || k >= f.max_steps;
    if (bad_ref || full) {
      phase = bad_ref ? MPCQP_FLEET_ABORTED : MPCQP_FLEET_OUT_OF_STEPS;
      if (lane == 0) f.mask[b] = 0;
      break;
    }
    int which = -1;
    double U = 0.0;
#pragma nounroll
    for (int relax = 0; relax < 2; ++relax) {
      // the lane index and the parameter block opaque per solve: otherwise LICM hoists every
      // lane- and parameter-derived value of the solver out of the step loop and holds it through
      // the whole run (hundreds of registers of spills)
      int ln = lane;
      asm volatile("" : "+v"(ln));
      const mpcqp_params& p = P[relax];  // P = {nominal, relaxed} in global memory (ws->dparams)
      FleetWin win{rows, ln, len, pidx, relax != 0, {ls[0], ls[1], ls[2], ls[3]}, {ls[4], ls[5]}};
      double Ul;
      const int st = solve_one<N, FleetWin, Pair>(p, b, nullptr, nullptr, nullptr, nullptr, win, sm,
                                                  f.u0 + (size_t)relax * V * 2, f.X, nullptr,
                                                  f.status + (size_t)relax * V, nullptr, nullptr, Ul);
      __syncthreads();  // the next solve (or step) reuses the LDS
      if (lane == 0) f.mask[(size_t)relax * V + b] = 1;
      if (st == MPCQP_SOLVED || st == MPCQP_SOLVED_INACCURATE) {
        which = relax;
        U = Ul;
        break;
      }
    }
    if (which == 0 && lane == 0) f.mask[(size_t)V + b] = 0;
    if (which < 0) {
      phase = MPCQP_FLEET_ABORTED;  // control_stage.py:108-110
      break;
    }
    // k_fleet_advance (every lane computes the same values)
    const double a = LN::readv(U, 0), delta = LN::readv(U, N);  // u0: lanes 0 and N
    double x[4] = {ls[0], ls[1], ls[2], ls[3]}, xn[4];
    plant(x, a, delta, P[0].dt, P[0].wheelbase_px, xn);
    if (lane == 0) {
      if (f.trace)
        for (int i = 0; i < 4; ++i) f.trace[((size_t)b * f.max_steps + k) * 4 + i] = xn[i];
      if (f.u_trace) {
        f.u_trace[((size_t)b * f.max_steps + k) * 2 + 0] = a;
        f.u_trace[((size_t)b * f.max_steps + k) * 2 + 1] = delta;
      }
    }
    __syncthreads();
    if (lane < 4) ls[lane] = xn[lane];
    else if (lane == 4) ls[4] = a;
    else if (lane == 5) ls[5] = delta;
    __syncthreads();
    k = k + 1;
    if (pidx < len - 2 && fleet_off_row(xn[0], xn[1], rows + (size_t)pidx * 4)) pidx = pidx + 1;
    if (fleet_at_goal(xn[0], xn[1], f.goal[(size_t)b * 2], f.goal[(size_t)b * 2 + 1])) {
      phase = MPCQP_FLEET_GOAL;
      break;
    }
    if (k >= f.max_steps) {
      phase = MPCQP_FLEET_OUT_OF_STEPS;
      break;
    }
    // k_swarm_trigger after the step: off the reference (state and path_idx after the step)
    if (can_replan && tr.replan_distance > 0.0 && len >= 1 && len <= f.ref_stride && pidx >= 0 && pidx < len &&
        swarm_off_track(xn[0], xn[1], rows + (size_t)pidx * 4, tr.replan_distance)) {
      phase = MPCQP_FLEET_REPLAN_RUNNING;
      break;
    }
  }
  if (lane < 4) f.state[(size_t)b * 4 + lane] = ls[lane];
  else if (lane < 6) f.u_prev[(size_t)b * 2 + lane - 4] = ls[lane];
  if (lane == 0) {
    f.path_idx[b] = pidx;
    f.steps[b] = k;
    f.phase[b] = phase;
  }
  if ((phase == MPCQP_FLEET_ABORTED && can_replan) || phase == MPCQP_FLEET_REPLAN_RUNNING) {
    __syncthreads();
    to_replan(phase, ls[0], ls[1]);
  }
}

// ------------------------------------------------------------------ B = 1 server
// One resident wave serving the sequential closed loop of TrajectoryTracker.track: it waits for the
// host to raise box->req (system-scope loads of pinned host memory, s_sleep between polls), solves the
// one QP of the staging input block with solve_one (the k_solve driver), writes the outputs into the
// staging output block, releases them at system scope and publishes box->done = req.  No launch and no
// stream synchronisation per step.  Exit conditions every path reaches: req == kServeStop, or no new
// request within idle_ticks of s_memrealtime (the host relaunches the wave at its next request).
template <int N>
__global__ __launch_bounds__(kWave, 1) void k_serve(mpcqp_params p, mpcqp::ServeLaunch L) {  // one resident wave: the whole register file
  __shared__ SolveLds<N> sm;
  const int lane = threadIdx.x;
  uint32_t last = __builtin_amdgcn_readfirstlane(
      __hip_atomic_load(&L.box->done, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM));
  for (;;) {
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    uint32_t req = last;
    while (req == last) {
      req = __builtin_amdgcn_readfirstlane(
          __hip_atomic_load(&L.box->req, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM));
      if (req != last) break;
      if (__builtin_amdgcn_s_memrealtime() - t0 > L.idle_ticks) return;  // idle: leave, the host relaunches
      __builtin_amdgcn_s_sleep(1);
    }
    if (req == mpcqp::kServeStop) return;
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");  // system scope: the inputs the host wrote before req
    int ln = lane;  // opaque per solve (ServeWin)
    asm volatile("" : "+v"(ln));
    const double* in = L.in;
    uint8_t* o = L.out;
    double Ul;
    solve_one<N>(p, 0, nullptr, in, in + 4, in + 4 + 4 * (N + 1), ServeWin{ln}, sm,
                 reinterpret_cast<double*>(o + L.off[0]), reinterpret_cast<double*>(o + L.off[1]),
                 reinterpret_cast<double*>(o + L.off[2]), reinterpret_cast<int32_t*>(o + L.off[3]),
                 reinterpret_cast<int32_t*>(o + L.off[4]), o + L.off[5], Ul);
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");  // system scope: the outputs before done
    if (lane == 0) __hip_atomic_store(&L.box->done, req, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    last = req;
    __syncthreads();  // the next solve reuses the LDS
  }
}

}  // namespace

namespace mpcqp {
template <int N>
void launch_serve(hipStream_t s, const mpcqp_params& p, const ServeLaunch& L) {
  hipLaunchKernelGGL(k_serve<N>, dim3(1), dim3(kWave), 0, s, p, L);
}
template <int N>
void launch_solve(hipStream_t s, const Launch& L) {
  hipLaunchKernelGGL(k_solve<N>, dim3(L.B), dim3(kWave), 0, s, *L.p, L.B, L.mask, L.model, L.x0, L.ref, L.u_prev,
                     L.state, L.u0, L.X, L.U,
                     L.st, L.it, L.ac);
}
template <int N>
void launch_fleet_loop(hipStream_t s, const mpcqp_params* P, const mpcqp_fleet& f, int steps, const LoopTrigger& tr) {
  if constexpr (2 * N <= 30) {
    if (tr.pair) {
      hipLaunchKernelGGL((k_fleet_loop<N, true>), dim3((f.vehicles + 1) / 2), dim3(kWave), 0, s, P, f, steps, tr);
      return;
    }
  }
  hipLaunchKernelGGL(k_fleet_loop<N>, dim3(f.vehicles), dim3(kWave), 0, s, P, f, steps, tr);
}
// two QPs per wave (N <= 15, fused K1, no debug state); false: not available for this launch
template <int N>
bool launch_solve_pair(hipStream_t s, const Launch& L) {
  if constexpr (2 * N <= 30) {
    hipLaunchKernelGGL(k_solve_pair<N>, dim3((L.B + 1) / 2), dim3(kWave), 0, s, *L.p, L.B, L.mask, L.x0, L.ref,
                       L.u_prev, L.u0, L.X, L.U, L.st, L.it, L.ac);
    return true;
  } else {
    (void)s;
    (void)L;
    return false;
  }
}

}  // namespace mpcqp
